"""CfManifest2Kube (reference ``internal/source/cfmanifest2kube.go``).

Planning: every CF manifest application becomes service options - a Reuse
service for docker-image apps, containerizer options for the app directory,
buildpack-matched options from ``CfContainerizers`` files, else Manual.  Apps
seen only in a collected running instance (``CfInstanceApps``) get the same
treatment.  Translation: env from the manifest plus the running instance,
``instances`` -> replicas, ports from the instance, else the container's
exposed ports, else 8080 (also exported as ``PORT``).
"""

import os

from .. import assets
from ..containerizer import Containerizers
from ..models import collection
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..utils import common, log
from ..utils.constants import DEFAULT_SERVICE_PORT, settings
from .cfmanifest import ManifestError, read_application_manifest
from .translator import Translator


def _get_cf_instance_app(file_apps, name):
    for path in sorted(file_apps):
        for app in file_apps[path]:
            if app.name == name:
                return path, app
    return "", collection.CfApplication()


def _get_cf_app_instance(path, appname):
    from ..models.base import read_document
    c = read_document(path, collection.CfInstanceApps.from_yaml, "CF_INSTANCE_APPS")
    for app in c.applications:
        if app.name == appname:
            return app
    raise ValueError("Failed to find the app %s in the cf apps file at path %s" % (appname, path))


class CfManifestTranslator(Translator):
    translation_type = plantypes.CFMANIFEST2KUBE

    def new_service(self, name):
        s = plantypes.Service.new(name, self.translation_type)
        s.add_source_type(plantypes.DIRECTORY_SOURCE)
        s.add_source_type(plantypes.CFMANIFEST_SOURCE)
        s.update_container_build_pipeline = True
        s.update_deploy_pipeline = True
        return s

    def _add_src(self, s, d):
        if not common.is_string_present(s.build_artifacts.get(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT), d):
            s.add_source_artifact(plantypes.SOURCE_DIRECTORY_ARTIFACT, d)
            s.add_build_artifact(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT, d)

    def get_service_options(self, input_path, plan):
        services = []
        cz = Containerizers().init_containerizers(input_path)
        try:
            files = common.get_files_by_ext(input_path, [".yml", ".yaml"])
        except OSError as e:
            log.warning("Unable to fetch yaml files and recognize cf manifest yamls at path %r Error: %r", input_path, str(e))
            raise
        # The built-in map (data.Cfbuildpacks_yaml) has its list at the top
        # level, not under spec, so the reference decodes it to an empty list
        # (kind "cfcontainerizers"); "fixed" compat uses it.
        containerizers = []
        if settings.fixed:
            containerizers = [collection.BuildpackContainerizer(b["buildpackName"], b["containerBuildType"], b["targetOptions"])
                              for b in assets.builtin_cf_buildpacks()]
        from ..models.base import decode_loaded
        docs = {}
        for f in files:   # every move2kube-group YAML counts: there is no kind check (cfmanifest2kube.go:67-76)
            try:
                docs[f] = text, data = common.read_move2kube_yaml_text(f)
                found = decode_loaded(f, text, data, collection.CfContainerizers.from_yaml, "CF_CONTAINERIZERS")
            except Exception as e:  # noqa: BLE001
                log.debug("Not a valid containerizer option file at path %r Error: %r", f, common.go_error_text(e))
                continue
            containerizers.extend(found.buildpack_containerizers)
        if log.debug_enabled():
            log.debug("Containerizers %s", "{TypeMeta:{APIVersion: Kind:cfcontainerizers} ObjectMeta:{Name:} "
                      "Spec:{BuildpackContainerizers:[%s]}}" % " ".join(b.go_plus_v() for b in containerizers))
        instance_apps = {}
        for f in files:
            try:
                text, data = docs.get(f) or common.read_move2kube_yaml_text(f)
                apps = decode_loaded(f, text, data, collection.CfInstanceApps.from_yaml, "CF_INSTANCE_APPS")
            except Exception as e:  # noqa: BLE001
                log.debug("Failed to read the yaml file at path %r Error: %r", f, common.go_error_text(e))
                continue
            if apps.kind != collection.CF_INSTANCE_APPS_KIND:
                log.debug("%s is not a valid apps file. Expected kind: %s Actual Kind: %s", log.go_quote(f),
                          collection.CF_INSTANCE_APPS_KIND, apps.kind)
                continue
            instance_apps.setdefault(f, []).extend(apps.applications)
        if log.debug_enabled():
            log.debug("Cf Instances %s", "map[" + " ".join(
                "%s:[%s]" % (k, " ".join(a.go_plus_v() for a in instance_apps[k])) for k in sorted(instance_apps)) + "]")
        # Every manifest app that is not a docker image has its build directory
        # probed by the containerizers (detect scripts, CNB builders); those
        # probes run as one batch, concurrently, instead of one app after
        # another as in the reference (only debug lines move).
        manifests = []
        probe = []
        for f in files:
            try:
                apps, _ = read_application_manifest(f, "", plantypes.YAMLS)
            except (ManifestError, OSError) as e:
                log.debug("Failed to parse the manifest file at path %r Error: %r", f, str(e))
                continue
            rows = []
            for app in apps:
                if app.path:
                    base = os.path.dirname(f) if settings.fixed else f
                    build_dir = common.go_join(base, app.path)
                else:
                    build_dir = os.path.dirname(f)
                app_name = app.name
                if app_name == "":
                    b = os.path.basename(f)
                    app_name = b[:len(b) - len(common.go_ext(b))]
                inst_path, inst = _get_cf_instance_app(instance_apps, app_name)
                rows.append((app, build_dir, app_name, inst_path, inst))
                if not (app.docker_image or inst.docker_image) and build_dir not in probe:
                    probe.append(build_dir)
            manifests.append((f, rows))
        probed = dict(zip(probe, cz.get_containerization_options_batch(plan, probe))) if probe else {}
        covered = []
        for f, rows in manifests:
            for app, build_dir, app_name, inst_path, inst in rows:
                if app.docker_image or inst.docker_image:
                    s = self.new_service(app_name)
                    s.container_build_type = plantypes.REUSE
                    s.image = app.docker_image or inst.docker_image
                    s.update_container_build_pipeline = False
                    services.append(s)
                    covered.append(app_name)
                    continue
                found = False
                for cop in probed[build_dir]:
                    s = self.new_service(app_name)
                    s.container_build_type = cop.containerization_type
                    s.target_options = list(cop.target_options)
                    s.add_source_artifact(plantypes.CFMANIFEST_ARTIFACT, f)
                    if inst.name:
                        s.add_source_artifact(plantypes.CF_RUNNING_MANIFEST_ARTIFACT, inst_path)
                    self._add_src(s, build_dir)
                    services.append(s)
                    covered.append(app_name)
                    found = True
                for c in containerizers:
                    matched = (app.buildpack.is_set and c.buildpack_name == app.buildpack.value) or \
                        c.buildpack_name in app.buildpacks
                    if not matched:
                        matched = (inst.buildpack and c.buildpack_name == inst.buildpack) or \
                            (inst.detected_buildpack and c.buildpack_name == inst.detected_buildpack)
                    if not matched:
                        continue
                    s = self.new_service(app_name)
                    s.container_build_type = c.container_build_type
                    s.target_options = list(c.target_options)
                    s.add_source_artifact(plantypes.CFMANIFEST_ARTIFACT, f)
                    if inst.name:
                        s.add_source_artifact(plantypes.CF_RUNNING_MANIFEST_ARTIFACT, inst_path)
                    self._add_src(s, build_dir)
                    services.append(s)
                    covered.append(app_name)
                    found = True
                if not found:
                    log.warning("No known containerization approach for %s even though it has a cf manifest %s; Defaulting to manual",
                                build_dir, os.path.basename(f))
                    s = self.new_service(app_name)
                    s.container_build_type = plantypes.MANUAL
                    s.add_source_artifact(plantypes.CFMANIFEST_ARTIFACT, f)
                    self._add_src(s, build_dir)
                    covered.append(app_name)
                    services.append(s)
            # apps only present in a running instance
            for app_file in sorted(instance_apps):
                for app in instance_apps[app_file]:
                    if common.is_string_present(covered, app.name) or app.name == "":
                        continue
                    build_dir = os.path.dirname(app_file)
                    if app.docker_image:
                        s = self.new_service(app.name)
                        s.container_build_type = plantypes.REUSE
                        s.image = app.docker_image
                        s.update_container_build_pipeline = False
                        services.append(s)
                        continue
                    found = False
                    for cop in cz.get_containerization_options(plan, build_dir):
                        s = self.new_service(app.name)
                        s.container_build_type = cop.containerization_type
                        s.target_options = list(cop.target_options)
                        s.add_source_artifact(plantypes.CF_RUNNING_MANIFEST_ARTIFACT, app_file)
                        self._add_src(s, build_dir)
                        services.append(s)
                        found = True
                    for c in containerizers:
                        if (app.buildpack and c.buildpack_name == app.buildpack) or \
                                (app.detected_buildpack and c.buildpack_name == app.detected_buildpack):
                            s = self.new_service(app.name)
                            s.container_build_type = c.container_build_type
                            s.target_options = list(c.target_options)
                            s.add_source_artifact(plantypes.CF_RUNNING_MANIFEST_ARTIFACT, app_file)
                            self._add_src(s, build_dir)
                            services.append(s)
                            found = True
                    if not found:
                        log.warning("No known containerization approach for %s even though it has a cf manifest %s; Defaulting to manual",
                                    build_dir, os.path.basename(f))
                        s = self.new_service(app.name)
                        s.container_build_type = plantypes.MANUAL
                        s.add_source_artifact(plantypes.CF_RUNNING_MANIFEST_ARTIFACT, app_file)
                        self._add_src(s, build_dir)
                        services.append(s)
        return services

    @staticmethod
    def _ports(sc, cont, inst, container):
        if inst.ports:
            for port in inst.ports:
                cont.setdefault("ports", []).append({"containerPort": port})
                sc.add_port_forwarding(irtypes.Port(port), irtypes.Port(port))
            cont.setdefault("env", []).append({"name": "PORT", "value": str(inst.ports[0])})
        elif container.exposed_ports:
            for port in container.exposed_ports:
                cont.setdefault("ports", []).append({"containerPort": port})
                sc.add_port_forwarding(irtypes.Port(port), irtypes.Port(port))
            cont.setdefault("env", []).append({"name": "PORT", "value": str(container.exposed_ports[0])})
        else:
            port = DEFAULT_SERVICE_PORT
            cont["ports"] = [{"containerPort": port}]
            sc.add_port_forwarding(irtypes.Port(port), irtypes.Port(port))
            cont.setdefault("env", []).append({"name": "PORT", "value": str(port)})

    def translate(self, services, plan):
        ir = irtypes.new_ir(plan)
        cz = Containerizers().init_containerizers(plan.root_dir)
        for service in services:
            if service.translation_type != self.translation_type:
                continue
            log.debug("Translating %s", service.service_name)
            inst = collection.CfApplication()
            running = service.source_artifacts.get(plantypes.CF_RUNNING_MANIFEST_ARTIFACT)
            if running:
                try:
                    inst = _get_cf_app_instance(running[0], service.service_name)
                except Exception as e:  # noqa: BLE001
                    log.debug("The file at path %s is not a valid cf apps file. Error: %r", running[0], str(e))
            paths = service.source_artifacts.get(plantypes.CFMANIFEST_ARTIFACT)
            if paths:
                path = paths[0]
                try:
                    apps, variables = read_application_manifest(path, service.service_name, plan.kubernetes.artifact_type)
                except (ManifestError, OSError) as e:
                    log.debug("Error while trying to parse manifest : %s", e)
                    continue
                log.debug("Using cf manifest file at path %s to translate service %s", path, service.service_name)
                try:
                    container = cz.get_container(plan, service)
                except Exception as e:  # noqa: BLE001
                    log.error("Failed to containerize service %s in cf manifest file at path %s Error: %r",
                              service.service_name, path, str(e))
                    continue
                ir.add_container(container)
                if not apps:
                    continue
                app = apps[0]
                sc = irtypes.new_service_from_plan_service(service)
                cont = {"name": service.service_name, "image": service.image}
                env = [{"name": k, "value": app.environment_variables[k]} for k in sorted(app.environment_variables)]
                for v in variables:
                    ir.values.global_variables[v] = v
                if app.instances.is_set:
                    sc.replicas = app.instances.value
                elif inst.instances != 0:
                    sc.replicas = inst.instances
                env += [{"name": k, "value": inst.env[k]} for k in sorted(inst.env)]
                if env:
                    cont["env"] = env
                self._ports(sc, cont, inst, container)
                sc.containers = [cont]
                ir.services[service.service_name] = sc
            else:
                log.debug("No cf manifest file found for service %s", service.service_name)
                try:
                    container = cz.get_container(plan, service)
                except Exception as e:  # noqa: BLE001
                    log.error("Failed to containerize service %s using cfmanifest translator. Error: %r",
                              service.service_name, str(e))
                    continue
                ir.add_container(container)
                sc = irtypes.new_service_from_plan_service(service)
                cont = {"name": service.service_name, "image": service.image}
                if inst.instances != 0:
                    sc.replicas = inst.instances
                env = [{"name": k, "value": inst.env[k]} for k in sorted(inst.env)]
                if env:
                    cont["env"] = env
                self._ports(sc, cont, inst, container)
                sc.containers = [cont]
                ir.services[service.service_name] = sc
        return ir
