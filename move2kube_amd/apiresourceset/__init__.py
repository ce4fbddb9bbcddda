"""API resource sets (reference ``internal/apiresourceset/``): the K8s set
(Deployment, Storage, Service, ImageStream, NetworkPolicy), the Knative set
and the Tekton CI/CD set; plus Kube2Kube/Knative2Kube discovery and
translation of existing manifests."""

from .. import apiresource as ar
from ..k8s import scheme
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..utils import common, log
from ..utils.constants import DEFAULT_STORAGE_CLASS_NAME, settings


def _intersection(a, b):
    ids = {id(x) for x in b}
    out = []
    for x in a:
        if id(x) in ids or any(x == y for y in b):
            out.append(x)
    return out


class K8sAPIResourceSet:
    scheme_name = "k8s"

    def get_api_resources(self, ir):
        spec = ir.target_cluster_spec
        return [ar.APIResource(ar.Deployment(spec)), ar.APIResource(ar.Storage(spec)), ar.APIResource(ar.Service(spec)),
                ar.APIResource(ar.ImageStream(spec)), ar.APIResource(ar.NetworkPolicy(spec))]

    def create_api_resources(self, ir):
        target = []
        ignored = list(ir.cached_objects)
        for res in self.get_api_resources(ir):
            res.set_cluster_context(ir.target_cluster_spec)
            res_ignored = res.load_resources(ir.cached_objects, ir)
            ignored = _intersection(ignored, res_ignored)
            target.extend(res.get_updated_resources(ir))
        target.extend(ignored)
        return target

    @staticmethod
    def _yaml_files(input_path):
        try:
            return common.get_files_by_ext(input_path, [".yml", ".yaml"])
        except (OSError, ValueError) as e:
            log.error("Unable to fetch yaml files at path %r Error: %r", input_path, str(e))
            raise

    @staticmethod
    def _read_and_decode(f, scheme_name):
        """ioutil.ReadFile + UniversalDeserializer().Decode of the planners,
        with their debug lines; None when either fails."""
        try:
            data = common.read_bytes(f)
        except OSError as e:
            log.debug("Failed to read the yaml file at path %r Error: %r", f, common.go_path_error(e, "open"))
            return None
        try:
            return scheme.decode(data, scheme_name)
        except scheme.DecodeError as e:
            log.debug("Failed to decode the file at path %r as a %s file. Error: %r", f, scheme_name, str(e))
            return None

    def get_service_options(self, input_path, plan):
        services = []
        for f in self._yaml_files(input_path):
            obj = self._read_and_decode(f, "k8s")
            if obj is None:
                continue
            try:
                name, _ = ar.Deployment.get_name_and_pod_spec(obj)
            except ValueError:
                continue
            s = new_k8s_service(name)
            s.source_artifacts[plantypes.K8S_FILE_ARTIFACT] = [f]
            services.append(s)
        return services

    def translate(self, services, plan):
        ir = irtypes.new_ir(plan)
        for service in services:
            files = service.source_artifacts.get(plantypes.K8S_FILE_ARTIFACT) or []
            if not files:
                log.warning("No k8s artifacts found in service %s", service.service_name)
                continue
            irs = irtypes.new_service_from_plan_service(service)
            try:
                data = common.read_bytes(files[0])
            except OSError as e:
                log.error("Unable to read the k8s file at path %r Error: %r", files[0], common.go_path_error(e, "open"))
                continue
            try:
                obj = scheme.decode(data, "k8s")
            except scheme.DecodeError as e:
                log.error("Failed to decode the k8s file at path %r Error: %r", files[0], str(e))
                continue
            try:
                _, ps = ar.Deployment.get_name_and_pod_spec(obj)
            except ValueError as e:
                log.error("Failed to get the pod specification for the k8s file at path %r Error: %r", files[0], str(e))
                continue
            irs.pod_spec = ps
            for c in ps.get("containers") or []:
                for p in c.get("ports") or []:
                    port = irtypes.Port(p.get("containerPort", 0), p.get("name", "") or "")
                    irs.add_port_forwarding(port, irtypes.Port(port.number, port.name))
            ir.services[service.service_name] = irs
        return ir


def new_k8s_service(name):
    s = plantypes.Service.new(name, plantypes.KUBE2KUBE)
    s.container_build_type = plantypes.REUSE
    s.add_source_type(plantypes.K8S_SOURCE)
    s.update_container_build_pipeline = False
    s.update_deploy_pipeline = True
    return s


class KnativeAPIResourceSet(K8sAPIResourceSet):
    scheme_name = "knative"

    def get_api_resources(self, ir):
        return [ar.APIResource(ar.KnativeService(ir.target_cluster_spec))]

    def get_service_options(self, input_path, plan):
        services = []
        for f in self._yaml_files(input_path):
            obj = self._read_and_decode(f, "knative")
            if obj is None:
                continue
            is_ksvc = obj.get("kind") == "Service" and obj.get("apiVersion") == "serving.knative.dev/v1"
            # The reference inverts this check: real Knative services are skipped and
            # any other Knative object dereferences nil.  The crash is always avoided; "fixed" compat
            # discovers the Knative services.
            if not (settings.fixed and is_ksvc):
                continue
            s = new_knative_service((obj.get("metadata") or {}).get("name", ""))
            s.source_artifacts[plantypes.KNATIVE_FILE_ARTIFACT] = [f]
            services.append(s)
        return services

    def translate(self, services, plan):
        ir = irtypes.new_ir(plan)
        for service in services:
            files = service.source_artifacts.get(plantypes.KNATIVE_FILE_ARTIFACT) or []
            if not files:
                log.warning("No knative artifacts found in service %s", service.service_name)
                continue
            irs = irtypes.new_service_from_plan_service(service)
            try:
                data = common.read_bytes(files[0])
            except OSError as e:
                log.error("Unable to read the knative file at path %r Error: %r", files[0], common.go_path_error(e, "open"))
                continue
            try:
                obj = scheme.decode(data, "knative")
            except scheme.DecodeError as e:
                log.error("Failed to decode the knative file at path %r Error: %r", files[0], str(e))
                continue
            if not (obj.get("kind") == "Service" and obj.get("apiVersion") == "serving.knative.dev/v1"):
                # %T of the decoded object: *<version package>.<Kind>
                actual = "*%s.%s" % (str(obj.get("apiVersion", "")).rsplit("/", 1)[-1], obj.get("kind", ""))
                log.error("The knative file at path %r does not contain the required type. Expected: %s Actual: %s",
                          files[0], "*v1.Service", actual)
                continue
            spec = ((obj.get("spec") or {}).get("template") or {}).get("spec") or {}
            ps = {k: v for k, v in spec.items() if k not in ("containerConcurrency", "timeoutSeconds")}
            irs.pod_spec = ps
            ir.services[service.service_name] = irs
        return ir


def new_knative_service(name):
    s = plantypes.Service.new(name, plantypes.KNATIVE2KUBE)
    s.container_build_type = plantypes.REUSE
    s.source_types = [plantypes.KNATIVE_SOURCE]
    s.update_container_build_pipeline = False
    s.update_deploy_pipeline = True
    return s


# ---------------------------------------------------------------------------
# Tekton
# ---------------------------------------------------------------------------

GIT_DOMAIN_PLACEHOLDER = "<TODO: insert git repo domain>"
KNOWN_HOSTS_PLACEHOLDER = "<TODO: insert the known host keys for your git repo>"
GIT_PRIVATE_KEY_PLACEHOLDER = "<TODO: insert the private ssh key for your git repo>"
REGISTRY_URL_PLACEHOLDER = "<TODO: insert the image registry URL>"
DOCKER_CONFIG_JSON_PLACEHOLDER = "<TODO: insert your docker config json>"


class TektonAPIResourceSet:
    def get_api_resources(self):
        return [ar.APIResource(ar.Service()), ar.APIResource(ar.ServiceAccount()), ar.APIResource(ar.RoleBinding()),
                ar.APIResource(ar.Role()), ar.APIResource(ar.Storage())]

    def get_tekton_api_resources(self):
        return [ar.EventListener(), ar.TriggerBinding(), ar.TriggerTemplate(), ar.Pipeline()]

    def create_api_resources(self, ir):
        ir = self.setup_ir(ir)
        out = []
        for a in self.get_api_resources():
            a.set_cluster_context(ir.target_cluster_spec)
            out.extend(a.get_updated_resources(ir))
        for h in self.get_tekton_api_resources():
            out.extend(h.create_new_resources(ir, []))
        return out

    @staticmethod
    def setup_ir(old):
        ir = irtypes.new_ir(plantypes.new_plan())
        ir.name = old.name
        ir.target_cluster_spec = old.target_cluster_spec
        ir.kubernetes = old.kubernetes
        ir.containers = [c for c in old.containers if c.new]
        proj = ir.name

        def p(n):
            return common.make_string_dns_subdomain_name_compliant("%s-%s" % (proj, n))
        pipeline = p("clone-build-push")
        git_secret_prefix = p("git-repo")
        clone_push_sa = p("clone-push")
        registry_secret = p("image-registry")
        listener = p("git-repo")
        binding = p("git-event")
        triggers_sa = p("tekton-triggers-admin")
        template = p("run-clone-build-push")
        workspace = p("shared-data")
        role = p("tekton-triggers-admin")
        role_binding = p("tekton-triggers-admin")
        ingress_name = p("git-repo")
        listener_svc = "el-" + listener
        tr = irtypes.TektonResources()
        tr.event_listeners = [{"name": listener, "service_account_name": triggers_sa,
                               "trigger_binding_name": binding, "trigger_template_name": template}]
        tr.trigger_bindings = [{"name": binding}]
        tr.trigger_templates = [{"name": template, "pipeline_name": pipeline, "pipeline_run_name": pipeline + "-$(uid)",
                                 "service_account_name": clone_push_sa, "workspace_name": workspace,
                                 "storage_class_name": DEFAULT_STORAGE_CLASS_NAME}]
        tr.pipelines = [{"name": pipeline, "workspace_name": workspace}]
        ir.tekton_resources = tr
        svc = irtypes.Service(ingress_name, "/" + listener_svc)
        svc.backend_service_name = listener_svc
        svc.only_ingress = True
        svc.pod_spec = {"containers": [{"ports": [{"containerPort": 8080}]}]}
        ir.services = {listener_svc: svc}
        ir.role_bindings.append(irtypes.RoleBinding(role_binding, role, triggers_sa))
        ir.roles.append(irtypes.Role(role, [
            irtypes.PolicyRule(["triggers.tekton.dev"], ["eventlisteners", "triggerbindings", "triggertemplates"], ["get"]),
            irtypes.PolicyRule(["tekton.dev"], ["pipelineruns"], ["create"]),
            irtypes.PolicyRule([""], ["configmaps"], ["get", "list", "watch"]),
        ]))
        registry_url = REGISTRY_URL_PLACEHOLDER
        if ir.kubernetes.registry_url:
            registry_url = ir.kubernetes.registry_url
            if registry_url == "docker.io":
                registry_url = "index.docker.io"
        secrets = [irtypes.Storage(name=registry_secret, storage_type=irtypes.SECRET_KIND,
                                   secret_type="kubernetes.io/dockerconfigjson",
                                   annotations={"tekton.dev/docker-0": registry_url},
                                   string_data={".dockerconfigjson": DOCKER_CONFIG_JSON_PLACEHOLDER})]
        from ..utils import git
        domains = []
        for c in ir.containers:
            host = git.url_hostname(c.repo_info.git_repo_url)
            if host:
                domains.append(host)
        domains = common.unique_strings(domains)
        if not domains:
            log.info("No remote git repos detected. You might want to configure the git repository links manually.")
        for d in domains:
            name = common.make_string_dns_subdomain_name_compliant("%s-%s" % (git_secret_prefix, d.replace(".", "-")))
            secrets.append(create_git_secret(name, d))
        ir.storages.extend(secrets)
        ir.service_accounts.append(irtypes.ServiceAccount(triggers_sa))
        ir.service_accounts.append(irtypes.ServiceAccount(clone_push_sa, [s.name for s in secrets]))
        return ir


def create_git_secret(name, domain):
    from ..qaengine import fetch_answer
    from ..models import qa
    from ..utils import knownhosts, sshkeys
    private_key = GIT_PRIVATE_KEY_PLACEHOLDER
    known = KNOWN_HOSTS_PLACEHOLDER
    if domain == "":
        domain = GIT_DOMAIN_PLACEHOLDER
    else:
        sshkeys.load_known_hosts_of_current_user()
        if domain in sshkeys.DOMAIN_TO_PUBLIC_KEYS:
            known = "\n".join(sshkeys.DOMAIN_TO_PUBLIC_KEYS[domain])
        else:
            line = knownhosts.get_known_hosts_line(domain)
            if line:
                known = line
            else:
                desc = ("Unable to find the public key for the domain %s from known_hosts, please enter it. If you are "
                        "not sure what this is press Enter and you will be able to edit it later: " % domain)
                example = sshkeys.DOMAIN_TO_PUBLIC_KEYS["github.com"][0]
                prob = qa.new_input_problem(desc, ["Ex : " + example], KNOWN_HOSTS_PLACEHOLDER)
                known = fetch_answer(prob).get_string_answer()
        key, ok = sshkeys.get_ssh_key(domain)
        if ok:
            private_key = key
    return irtypes.Storage(name=name, storage_type=irtypes.SECRET_KIND, secret_type="kubernetes.io/ssh-auth",
                           annotations={"tekton.dev/git-0": domain},
                           string_data={"ssh-privatekey": private_key, "known_hosts": known})

