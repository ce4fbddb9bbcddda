"""IR -> output artifacts (reference ``internal/transformer/``).

* :class:`K8sTransformer` - Deployment/Service/Ingress/... YAMLs (or a Helm
  chart + optional operator), converted to the first version the target
  cluster supports; ``deploy.sh``/``NOTES.txt``/``Readme.md``.
* :class:`KnativeTransformer` - knative Services.
* :class:`ComposeTransformer` - a docker-compose v3.5 file.
* :class:`CICDTransformer` - Tekton pipeline/trigger objects under ``cicd/``.

``write_containers`` emits the new-image build scripts (reference
``transformer.go:48-151``); ``write_transformed_objects`` serialises one file
per object as ``<name>-<lowercase kind>.yaml`` through the typed-struct
marshaller + go-yaml emitter (``transformer.go:153-200``).
"""

import os
import shutil

from .. import assets
from ..apiresource.base import GOTYPE
from ..apiresourceset import K8sAPIResourceSet, KnativeAPIResourceSet, TektonAPIResourceSet
from ..k8s import convert, schema
from ..ops import native
from ..models import plan as plantypes
from ..utils import common, log, trace, yamlio
from ..utils.constants import (DEFAULT_DIRECTORY_PERMISSION, DEFAULT_EXECUTABLE_PERMISSION, DEFAULT_FILE_PERMISSION,
                               EXPOSE_SELECTOR, settings)

HELM_TEMPLATES_REL_PATH = "templates"
OPERATOR_SDK_TIMEOUT_S = 600  # the reference waits forever
CONTAINERS_DIR = "containers"
KNATIVE_GROUP = "serving.knative.dev"


def _mkdir(p):
    os.makedirs(p, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)


def write_containers(containers, outpath, root_dir, registry_url, registry_namespace):
    """Write new-container files and build/push scripts; True if any new image exists."""
    cpath = os.path.join(outpath, CONTAINERS_DIR)
    log.debug("containerspath %s", cpath)
    try:
        _mkdir(cpath)
    except OSError as e:
        log.error("Unable to create directory %s : %s", cpath, common.go_path_error(e, "mkdir"))
    log.debug("Total number of containers : %d", len(containers))
    buildscripts, dockerimages, manualimages = [], [], []
    batch = []
    made = set()
    for c in containers:
        log.debug("Container : %s", "true" if c.new else "false")
        if not c.new:
            continue
        if not c.new_files:
            manualimages.extend(c.image_names)
        log.debug("New Container : %s", c.image_names[0] if c.image_names else "")
        if c.new_files or not settings.fixed:
            # the reference also lists manual images in pushimages.sh although
            # buildimages.sh never builds them; "fixed" leaves them to Manualimages.md
            dockerimages.extend(c.image_names)
        for rel in sorted(c.new_files):
            wp = os.path.join(cpath, rel)
            d = os.path.dirname(wp)
            if d not in made:
                try:
                    _mkdir(d)
                except OSError as e:
                    log.error("Unable to create directory %s : %s", d, common.go_path_error(e, "mkdir"))
                    continue
                made.add(d)
            mode = DEFAULT_FILE_PERMISSION
            if common.go_ext(wp) == ".sh":
                mode = DEFAULT_EXECUTABLE_PERMISSION
                buildscripts.append(os.path.join(CONTAINERS_DIR, rel))
            log.debug("Writing at %s", wp)
            batch.append((wp, c.new_files[rel], mode))
    for (wp, _, _), err in zip(batch, native.write_files(batch)):
        if err is not None:
            log.warning("Error writing file at %s : %s", wp, common.go_path_error(err, "open"))
    if manualimages:
        wp = os.path.join(outpath, "Manualimages.md")
        if settings.fixed:
            _write_template("manualimages.md.tpl", {"Images": manualimages}, wp, DEFAULT_FILE_PERMISSION,
                            "Unable to create manual image : %s")
        else:
            # the reference hands the template a struct without the field it ranges over,
            # so template execution fails and no file is written
            log.warning("Unable to translate template %s to string using the data %s",
                        log.go_quote(assets.template("manualimages.md.tpl")), "{[" + " ".join(manualimages) + "]}")
            log.error("Unable to create manual image : template: manualimages:5:17: executing \"manualimages\" at "
                      "<.Images>: can't evaluate field Images in type struct { Scripts []string }")
    if buildscripts:
        script_map = {}
        for v in buildscripts:
            d, f = os.path.split(v)
            script_map[f] = d + "/" if d else ""
        if log.debug_enabled():
            log.debug("buildscripts %s", "[" + " ".join(buildscripts) + "]")
            log.debug("buildScriptMap %s", "map[" + " ".join("%s:%s" % (k, script_map[k]) for k in sorted(script_map)) + "]")
        _write_template("buildimages.sh.tpl", script_map, os.path.join(outpath, "buildimages.sh"),
                        DEFAULT_EXECUTABLE_PERMISSION, "Unable to create script to build images : %s")
        try:
            rel_root = common.go_rel(outpath, root_dir)
        except ValueError as e:
            log.error("Failed to make the root directory path %r relative to the output directory %r Error %r",
                      root_dir, outpath, str(e))
            rel_root = root_dir
        _write_template("copysources.sh.tpl", {"RelRootDir": rel_root, "Dst": CONTAINERS_DIR},
                        os.path.join(outpath, "copysources.sh"), DEFAULT_EXECUTABLE_PERMISSION,
                        "Unable to create script to build images : %s")
    if dockerimages:
        _write_template("pushimages.sh.tpl", {"Images": dockerimages, "RegistryURL": registry_url,
                                              "RegistryNamespace": registry_namespace},
                        os.path.join(outpath, "pushimages.sh"), DEFAULT_EXECUTABLE_PERMISSION,
                        "Unable to create script to push images : %s")
        return True
    return False


def _write_template(name, data, path, mode, error_fmt):
    """WriteTemplateToFile of a packaged template; a failure is logged with
    the caller's text and the run goes on, as in the reference."""
    from ..utils.gotemplate import TemplateError
    try:
        common.write_template_to_file(assets.template(name), data, path, mode)
    except TemplateError as e:
        log.error(error_fmt, e)
    except OSError as e:
        log.warning("Error writing file at %s : %s", path, common.go_path_error(e, "open"))
        log.error(error_fmt, common.go_path_error(e, "open"))


def serialize_object(obj):
    """One object -> YAML text exactly as the reference writes it."""
    clean = {k: v for k, v in obj.items() if k != GOTYPE}
    return yamlio.dumps_k8s(schema.marshal(clean))


def write_transformed_objects(path, objs):
    written = []
    try:
        _mkdir(path)
    except OSError as e:
        log.error("Unable to create directory %s : %s", path, common.go_path_error(e, "mkdir"))
        raise
    batch, kinds = [], []
    for obj in objs:
        try:
            data = serialize_object(obj)
        except Exception as e:  # noqa: BLE001
            log.error("Error while Encoding object : %s", e)
            continue
        name = (obj.get("metadata") or {}).get("name", "")
        batch.append((os.path.join(path, "%s-%s.yaml" % (name, obj.get("kind", "").lower())), data,
                      DEFAULT_FILE_PERMISSION))
        kinds.append(obj.get("kind"))
    # one batched, parallel write (ops/csrc/m2k_native.cpp:write_files)
    for (f, _, _), kind, err in zip(batch, kinds, native.write_files(batch)):
        if err is not None:
            log.error("Failed to write %r Error: %r", kind, common.go_path_error(err, "open"))
            continue
        written.append(f)
        log.debug("%r created", f)
    return written


class Transformer:
    def transform(self, ir):
        raise NotImplementedError

    def write_objects(self, outpath):
        raise NotImplementedError


def get_transformer(ir):
    if ir.kubernetes.artifact_type == plantypes.KNATIVE:
        return KnativeTransformer()
    return K8sTransformer()


def _parse_group_version(gv):
    """``schema.ParseGroupVersion(gv).String()``: "" and "/" are the empty
    version, no slash is a core version, one slash splits group and version;
    more is an error (None)."""
    if gv in ("", "/"):
        return ""
    n = gv.count("/")
    if n == 0:
        return gv
    if n == 1:
        group, ver = gv.split("/")
        return group + "/" + ver if group else ver
    return None


class K8sTransformer(Transformer):
    def __init__(self):
        self.root_dir = ""
        self.transformed_objects = []
        self.containers = []
        self.values = None
        self.target_cluster_spec = None
        self.helm = False
        self.name = ""
        self.ignore_unsupported_kinds = False  # never set by the reference's Transform
        self.exposed_service_paths = {}
        self.add_copy_sources_warning = False
        self.overlap_work = []  # callables run while operator-sdk runs (Helm only)
        self.before_operator = None  # called just before operator-sdk starts (Helm only)

    def transform(self, ir):
        log.debug("Starting Kubernetes transform")
        log.debug("Total services to be transformed : %d", len(ir.services))
        self.name = ir.name
        self.values = ir.values
        self.containers = ir.containers
        self.target_cluster_spec = ir.target_cluster_spec
        self.helm = ir.kubernetes.artifact_type == plantypes.HELM
        if settings.fixed:
            self.ignore_unsupported_kinds = ir.kubernetes.ignore_unsupported_kinds
        self.transformed_objects = K8sAPIResourceSet().create_api_resources(ir)
        self.root_dir = ir.root_dir
        self.add_copy_sources_warning = ir.add_copy_sources_warning
        for s in ir.sorted_services():
            if s.has_valid_annotation(EXPOSE_SELECTOR):
                self.exposed_service_paths[s.name] = s.service_rel_path
        log.debug("Total transformed objects : %d", len(self.transformed_objects))

    def convert_objects(self):
        """``convertToClusterSupportedKinds`` (k8stransformer.go:106-143): each
        object to the first version the cluster lists for its kind.  For a
        kind the cluster does not list, the reference keeps
        ``GroupVersionKind().String()`` (``apps/v1, Kind=Deployment``) as
        the version; ``ParseGroupVersion`` reads ``v1, Kind=Deployment`` as
        the version, so the conversion fails with "no kind ... is registered"
        and the object is written as it was.  A version with two slashes
        (malformed cluster metadata) drops the object."""
        objs = []
        for obj in self.transformed_objects:
            kind = obj.get("kind", "")
            versions = self.target_cluster_spec.get_supported_versions(kind)
            version = obj.get("apiVersion", "")
            if versions is None:
                if self.ignore_unsupported_kinds:
                    log.error("Kind %s unsupported in target cluster. Will ignore object. %s", kind,
                              "&TypeMeta{Kind:%s,APIVersion:%s,}" % (kind, version))   # %+v: TypeMeta's String()
                    continue
                if not settings.fixed:
                    group, _, ver = version.rpartition("/")
                    version = "%s/%s, Kind=%s" % (group, ver, kind)
            elif kind == "Service":
                for v in versions:
                    if not v.startswith(KNATIVE_GROUP):
                        version = v
            else:
                version = versions[0]
            gv = _parse_group_version(version)
            if gv is None:
                log.error("Unable to parse group version %s : unexpected GroupVersion string: %s", version, version)
                continue
            version = gv
            try:
                obj = (convert.convert_fixed if settings.fixed else convert.convert_to_version)(obj, version)
            except convert.ConversionError as e:
                log.error("Error while transforming version : %s. Writing in original version.", e)
            objs.append(obj)
        return objs

    def write_objects(self, outpath):
        """``Kubernetes.WriteObjects`` (k8stransformer.go:100-146).  For a Helm
        chart the operator-sdk run (seconds for the real tool) starts as soon
        as the chart is complete and overlaps the container build files, the
        readme and ``overlap_work`` (the caller's deferred writes), none of
        which it reads; it is waited for before returning."""
        if not self.helm:
            new_images = self._write_containers(outpath)
        artifacts = os.path.join(outpath, self.name)
        if self.helm:
            try:
                self.generate_helm_metadata(artifacts)
            except OSError as e:
                log.debug("Failed to generate helm metadata properly, continuing anyway. Error: %r", str(e))
            artifacts = os.path.join(artifacts, HELM_TEMPLATES_REL_PATH)
        log.debug("Total services to be serialized : %d", len(self.transformed_objects))
        try:
            write_transformed_objects(artifacts, self.convert_objects())
        except OSError as e:
            log.error("Error occurred while writing transformed objects %s", e)
        if self.helm:
            if self.before_operator is not None:
                self.before_operator()
            operator = self.start_operator(self.name, outpath)
            try:
                new_images = self._write_containers(outpath)
                self.write_readme(self.name, new_images, self.helm, self.add_copy_sources_warning, outpath)
                while self.overlap_work:  # shared with the caller: what is popped has run
                    self.overlap_work.pop(0)()
            finally:
                self.finish_operator(operator)
            return
        self.write_deploy_script(self.name, outpath)
        self.write_readme(self.name, new_images, self.helm, self.add_copy_sources_warning, outpath)

    def _write_containers(self, outpath):
        return write_containers(self.containers, outpath, self.root_dir, self.values.registry_url,
                                self.values.registry_namespace)

    def generate_helm_metadata(self, d):
        """``generateHelmMetadata`` (k8stransformer.go:156-217): each step
        that fails is logged and the rest still written."""
        from ..utils.gotemplate import TemplateError
        try:
            _mkdir(d)
        except OSError as e:
            log.error("Unable to create Helm Metadata directory %s : %s", d, common.go_path_error(e, "mkdir"))
            raise
        try:
            common.write_text(os.path.join(d, "README.md"), "This chart was created by Move2Kube\n")
        except OSError as e:
            log.error("Error while writing Readme : %s", common.go_path_error(e, "open"))
        base = common.go_base(d)
        try:
            common.write_template_to_file(assets.template("chart.yaml.tpl"), {"Name": base},
                                          os.path.join(d, "Chart.yaml"), DEFAULT_FILE_PERMISSION)
        except (OSError, TemplateError) as e:
            log.error("Error while writing Chart.yaml : %s",
                      common.go_path_error(e, "open") if isinstance(e, OSError) else e)
        try:
            _mkdir(os.path.join(d, HELM_TEMPLATES_REL_PATH))
        except OSError as e:
            log.error("Unable to create templates directory : %s", common.go_path_error(e, "mkdir"))
        notes = ""
        try:
            notes = common.get_string_from_template(assets.template("notes.txt.tpl"),
                                                    {"IsHelm": True, "ExposedServicePaths": self.exposed_service_paths})
        except TemplateError as e:
            paths = self.exposed_service_paths
            log.error("Failed to fill the NOTES.txt template %s with the service paths %s Error: %r",
                      assets.template("notes.txt.tpl"),
                      "map[" + " ".join("%s:%s" % (k, paths[k]) for k in sorted(paths)) + "]", str(e))
        try:
            common.write_text(os.path.join(d, HELM_TEMPLATES_REL_PATH, "NOTES.txt"),
                              assets.template("helmnotes.txt") + notes)
        except OSError as e:
            log.error("Error while writing Helm NOTES.txt : %s", common.go_path_error(e, "open"))
        values_path = os.path.join(d, "values.yaml")
        try:
            common.write_yaml(values_path, self.values)
        except OSError as e:
            # log.Warn("Error in writing Helm values", err): Sprint puts no space after a string operand
            log.warning("Error in writing Helm values%s", common.go_path_error(e, "open"))
        else:
            log.debug("Wrote Helm values to file: %s", values_path)
        common.write_template_to_file(assets.template("helminstall.sh.tpl"), {"Project": base},
                                      os.path.join(os.path.dirname(d), "helminstall.sh"), DEFAULT_EXECUTABLE_PERMISSION)

    @classmethod
    def create_operator(cls, project, basepath):
        """``createOperator`` (k8stransformer.go:226-247): ``operator-sdk init
        --plugins=helm`` over the chart in ``<out>/<project>-operator``."""
        return cls.finish_operator(cls.start_operator(project, basepath))

    @staticmethod
    def start_operator(project, basepath):
        """Launch operator-sdk without waiting; None if it cannot run."""
        sdk = shutil.which("operator-sdk")
        if sdk is None:
            log.warning("Unable to find operator-sdk. Skipping operator generation : exec: \"operator-sdk\": "
                        "executable file not found in $PATH")
            return None
        from ..utils import proc
        opath = os.path.join(basepath, project + "-operator")
        if os.path.exists(opath):
            shutil.rmtree(opath, ignore_errors=True)
        try:
            _mkdir(opath)
        except OSError as e:
            log.error("Unable to create Operator directory %s : %s", opath, common.go_path_error(e, "mkdir"))
            return None
        chart = os.path.abspath(os.path.join(basepath, project))
        span = trace.span("operator-sdk init (external tool)", "external")
        span.__enter__()
        out = common.unnamed_temp_file()  # not a pipe: nothing reads it until the tool exits
        try:
            child = proc.spawn([sdk, "init", "--plugins=helm", "--helm-chart=" + chart, "--domain=io",
                                "--group=" + project, "--version=v1alpha1"], cwd=opath, stdout=out,
                               stderr=proc.DEVNULL)
        except OSError as e:
            out.close()
            span.__exit__(None, None, None)
            # cmd.Output() that cannot start: "<err>, <no output>" (k8stransformer.go:243-246)
            err = "fork/exec %s: %s" % (sdk, common.go_errno_text(e.errno)) if e.errno else str(e)
            log.warning("Error during operator creation : %s, %s", err, "")
            return None
        return child, out, span

    @staticmethod
    def finish_operator(started):
        if started is None:
            return False
        child, out, span = started
        try:
            try:
                with trace.span("operator-sdk wait", "external"):  # the part no other work hid
                    r = child.wait(OPERATOR_SDK_TIMEOUT_S)  # killed when it overruns
            finally:
                span.__exit__(None, None, None)
            if r.timed_out:
                log.warning("Error during operator creation : timed out after %d seconds", OPERATOR_SDK_TIMEOUT_S)
                return False
            if r.returncode != 0:
                out.seek(0)
                log.warning("Error during operator creation : %s, %s", common.go_exit_status(r.returncode),
                            out.read().decode("utf-8", "replace"))
                return False
            return True
        finally:
            out.close()

    def write_deploy_script(self, proj, outpath):
        deploy = os.path.join(outpath, "deploy.sh")
        _write_or_log(assets.template("deploy.sh.tpl"), {"Project": proj}, deploy, DEFAULT_EXECUTABLE_PERMISSION,
                      "Failed to write the deploy script at path %r Error: %r", deploy)
        notes = os.path.join(outpath, "NOTES.txt")
        _write_or_log(assets.template("notes.txt.tpl"),
                      {"IsHelm": False, "IngressHost": self.target_cluster_spec.host,
                       "ExposedServicePaths": self.exposed_service_paths},
                      notes, DEFAULT_FILE_PERMISSION, "Failed to write the NOTES.txt file at path %r Error: %r", notes)

    @staticmethod
    def write_readme(project, new_images, helm, warn, outpath):
        _write_or_log(assets.template("k8sreadme.md.tpl"),
                      {"Project": project, "NewImages": new_images, "Helm": helm, "AddCopySourcesWarning": warn},
                      os.path.join(outpath, "Readme.md"), DEFAULT_FILE_PERMISSION, "Unable to write readme : %s")


def _write_or_log(tpl, data, path, mode, error_fmt, *prefix):
    """WriteTemplateToFile whose error the caller logs (``error_fmt`` with
    ``prefix`` arguments, then the error; %r arguments print Go-quoted)."""
    from ..utils.gotemplate import TemplateError
    try:
        common.write_template_to_file(tpl, data, path, mode)
    except (OSError, TemplateError) as e:
        if isinstance(e, OSError):
            text = common.go_path_error(e, "open")
            log.warning("Error writing file at %s : %s", path, text)
        else:
            text = str(e)
        log.error(error_fmt, *(prefix + (text,)))


class KnativeTransformer(Transformer):
    def __init__(self):
        self.transformed_objects = []
        self.name = ""

    def transform(self, ir):
        log.debug("Starting Knative transform")
        self.name = ir.name
        self.values = ir.values
        self.containers = ir.containers
        self.target_cluster_spec = ir.target_cluster_spec
        self.ignore_unsupported_kinds = ir.kubernetes.ignore_unsupported_kinds
        self.transformed_objects = KnativeAPIResourceSet().create_api_resources(ir)
        self.root_dir = ir.root_dir

    def write_objects(self, outpath):
        new_images = write_containers(self.containers, outpath, self.root_dir, self.values.registry_url,
                                      self.values.registry_namespace)
        try:
            write_transformed_objects(os.path.join(outpath, self.name), self.transformed_objects)
        except OSError as e:
            log.error("Error occurred while writing transformed objects %s", e)
        _write_or_log(assets.template("deploy.sh.tpl"), {"Project": self.name}, os.path.join(outpath, "deploy.sh"),
                      DEFAULT_EXECUTABLE_PERMISSION, "Unable to write deploy script : %s")
        _write_or_log(assets.template("knativereadme.md.tpl"), {"Project": self.name, "NewImages": new_images},
                      os.path.join(outpath, "Readme.md"), DEFAULT_FILE_PERMISSION, "Unable to write Readme : %s")


class ComposeTransformer(Transformer):
    """docker-compose v3.5 output: one entry per service (last container wins),
    published ports allocated from 8080 upwards."""

    def transform(self, ir):
        log.debug("Starting Compose transform")
        self.name = ir.name
        self.containers = ir.containers
        services = {}
        exposed = 8080
        for s in ir.sorted_services():
            for c in s.containers:
                ports = []
                for p in c.get("ports") or []:
                    pc = {}
                    if p.get("containerPort"):
                        pc["target"] = p["containerPort"]
                    pc["published"] = exposed
                    ports.append(pc)
                    exposed += 1
                env = {}
                envs = c.get("env") or []
                for e in envs:
                    env[e.get("name", "")] = e.get("value", "")
                if envs and not settings.fixed:
                    # `&e.Value` of the shared range variable: every entry ends up pointing
                    # at the last value (go<1.22 loop semantics)
                    last = envs[-1].get("value", "")
                    env = {k: last for k in env}
                svc = {}
                if c.get("name"):
                    svc["container_name"] = c["name"]
                if env:
                    svc["environment"] = yamlio.GoMap(env)
                if c.get("image"):
                    svc["image"] = c["image"]
                if ports:
                    svc["ports"] = ports
                services[s.name] = svc
        self.compose = {"version": "3.5", "services": yamlio.GoMap(services)} if services else {"version": "3.5"}

    def write_objects(self, outpath):
        try:
            _mkdir(outpath)
        except OSError as e:
            log.error("Unable to create output directory %s : %s", outpath, common.go_path_error(e, "mkdir"))
        path = os.path.join(outpath, "docker-compose.yaml")
        try:
            common.write_yaml(path, self.compose)
        except OSError as e:
            log.error("Unable to write docker compose file %s : %s", path, common.go_path_error(e, "open"))


class CICDTransformer(Transformer):
    def transform(self, ir):
        self.cached_objs = TektonAPIResourceSet().create_api_resources(ir)

    def write_objects(self, outpath):
        p = os.path.join(outpath, "cicd")
        try:
            _mkdir(p)
        except OSError as e:
            log.fatal("Failed to create the CI/CD directory at path %r. Error: %r", p, common.go_path_error(e, "mkdir"))
        try:
            write_transformed_objects(p, self.cached_objs)
        except OSError as e:
            log.error("Error occurred while writing transformed objects. Error: %r", common.go_path_error(e, "open"))
            raise
