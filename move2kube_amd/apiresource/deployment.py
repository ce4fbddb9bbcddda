"""Deployment-like workloads (reference ``internal/apiresource/deployment.go``).

Creates DaemonSet (``Daemon``), Job/Pod (restart Never/OnFailure), else the
first supported of DeploymentConfig -> Deployment -> ReplicationController ->
Pod, and converts between all of them (DeploymentConfigs get image-change
triggers).  Volume mounts without a volume are dropped and volumes are
converted to kinds the cluster supports.
"""

from ..utils import common, log
from ..utils.constants import settings
from .base import (GOTYPE, IAPIResource, get_annotations, get_pod_labels, get_service_labels, is_type,
                   object_meta_copy)
from .storage import convert_volume_by_supported_kind

POD = "Pod"
JOB = "Job"
DEPLOYMENT = "Deployment"
DEPLOYMENT_CONFIG = "DeploymentConfig"
REPLICATION_CONTROLLER = "ReplicationController"
DAEMONSET = "DaemonSet"


class Deployment(IAPIResource):
    def __init__(self, cluster_spec=None):
        self.cluster_spec = cluster_spec

    def get_supported_kinds(self):
        kinds = [POD, JOB, DEPLOYMENT, DEPLOYMENT_CONFIG, REPLICATION_CONTROLLER]
        if settings.fixed:
            kinds.append(DAEMONSET)
        return kinds

    # -- create ------------------------------------------------------------
    def create_new_resources(self, ir, supported):
        objs = []
        for service in ir.sorted_services():
            obj = None
            rp = service.restart_policy
            if service.daemon:
                if common.is_string_present(supported, DAEMONSET):
                    obj = self.create_daemonset(service)
                else:
                    log.error("Could not find a valid resource type in cluster to create a daemon set.")
            elif rp in ("Never", "OnFailure"):
                if common.is_string_present(supported, JOB):
                    obj = self.create_job(service)
                elif common.is_string_present(supported, POD):
                    obj = self.create_pod(service)
                    obj["spec"]["restartPolicy"] = "OnFailure"
                else:
                    log.error("Could not find a valid resource type in cluster to create a job/pod.")
            elif common.is_string_present(supported, DEPLOYMENT_CONFIG):
                obj = self.create_deployment_config(service)
            elif common.is_string_present(supported, DEPLOYMENT):
                obj = self.create_deployment(service)
            elif common.is_string_present(supported, REPLICATION_CONTROLLER):
                obj = self.create_replication_controller(service)
            elif common.is_string_present(supported, POD):
                obj = self.create_pod(service)
            else:
                log.error("Could not find a valid resource type in cluster to create a deployment")
            if obj is not None:
                objs.append(obj)
        return objs

    def _meta(self, service):
        m = {"name": service.name, "labels": get_pod_labels(service.name, service.networks)}
        ann = get_annotations(service)
        if ann:
            m["annotations"] = ann
        return m

    def _podspec(self, service, restart="Always"):
        ps = common.deep_copy(service.pod_spec)
        ps = self.convert_volumes_kinds_by_policy(ps)
        ps["restartPolicy"] = restart
        return ps

    def create_deployment(self, service):
        m, ps = self._meta(service), self._podspec(service)
        log.debug("Created deployment for %s", service.name)
        return self.to_deployment(m, ps, service.replicas)

    def create_deployment_config(self, service):
        m, ps = self._meta(service), self._podspec(service)
        log.debug("Created DeploymentConfig for %s", service.name)
        return self.to_deployment_config(m, ps, service.replicas)

    def create_replication_controller(self, service):
        m, ps = self._meta(service), self._podspec(service)
        log.debug("Created DeploymentConfig for %s", service.name)   # sic, deployment.go:230
        return self.to_replication_controller(m, ps, service.replicas)

    def create_pod(self, service):
        ps = self._podspec(service)
        return self.to_pod(self._meta(service), ps, ps["restartPolicy"])

    def create_daemonset(self, service):
        m = self._meta(service)
        ps = self._podspec(service)
        return {"kind": DAEMONSET, "apiVersion": "apps/v1", "metadata": m,
                "spec": {"selector": {"matchLabels": get_service_labels(m["name"])},
                         "template": {"metadata": object_meta_copy(m), "spec": ps}}}

    def create_job(self, service):
        m = self._meta(service)
        ps = self._podspec(service, "OnFailure")
        return {"kind": JOB, "apiVersion": "batch/v1", "metadata": m,
                "spec": {"template": {"metadata": object_meta_copy(m), "spec": ps}}}

    # -- conversions --------------------------------------------------------
    def to_deployment_config(self, m, ps, replicas):
        ps = self.convert_volumes_kinds_by_policy(ps)
        triggers = [{"type": "ConfigChange"}]
        for c in ps.get("containers") or []:
            _, tag = common.get_image_name_and_tag(c.get("image", ""))
            triggers.append({"type": "ImageChange", "imageChangeParams": {
                "automatic": True, "containerNames": [c.get("name", "")],
                "from": {"kind": "ImageStreamTag", "name": m.get("name", "") + ":" + tag}}})
        return {"kind": DEPLOYMENT_CONFIG, "apiVersion": "apps.openshift.io/v1", "metadata": m,
                "spec": {"replicas": int(replicas), "selector": get_service_labels(m.get("name", "")),
                         "template": {"metadata": object_meta_copy(m), "spec": ps}, "triggers": triggers}}

    def to_deployment(self, m, ps, replicas):
        ps = self.convert_volumes_kinds_by_policy(ps)
        return {"kind": DEPLOYMENT, "apiVersion": "apps/v1", "metadata": m,
                "spec": {"replicas": int(replicas), "selector": {"matchLabels": get_service_labels(m.get("name", ""))},
                         "template": {"metadata": object_meta_copy(m), "spec": ps}}}

    def to_replication_controller(self, m, ps, replicas):
        ps = self.convert_volumes_kinds_by_policy(ps)
        return {"kind": REPLICATION_CONTROLLER, "apiVersion": "v1", "metadata": m,
                "spec": {"replicas": int(replicas), "selector": get_service_labels(m.get("name", "")),
                         "template": {"metadata": object_meta_copy(m), "spec": ps}}}

    def pod_to_job(self, pod):
        ps = self.convert_volumes_kinds_by_policy(common.deep_copy(pod.get("spec") or {}))
        ps["restartPolicy"] = "OnFailure"
        m = pod.get("metadata") or {}
        return {"kind": JOB, "apiVersion": "batch/v1", "metadata": m,
                "spec": {"template": {"metadata": object_meta_copy(m), "spec": ps}}}

    def to_pod(self, m, ps, restart):
        ps = self.convert_volumes_kinds_by_policy(ps)
        ps["restartPolicy"] = restart
        return {"kind": POD, "apiVersion": "v1", "metadata": m, "spec": ps}

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        if is_type(obj, "apps/v1", DAEMONSET) or obj.get(GOTYPE) == "apps/v1.DaemonSet":
            if common.is_string_present(supported, DAEMONSET):
                return [obj], True
            return None, False
        spec = obj.get("spec") or {}
        tmpl_spec = (spec.get("template") or {}).get("spec") or {}
        replicas = spec.get("replicas")
        m = obj.get("metadata") or {}
        if is_type(obj, "v1", POD) and spec.get("restartPolicy") in ("OnFailure", "Never"):
            if common.is_string_present(supported, JOB):
                return [self.pod_to_job(obj)], True
            return [obj], True
        if is_type(obj, "batch/v1", JOB) and not common.is_string_present(supported, JOB):
            if common.is_string_present(supported, POD):
                return [self.to_pod(m, common.deep_copy(tmpl_spec), "OnFailure")], True
            log.warning("Both Job and Pod not supported. No other valid way to translate this object. : %s", m.get("name"))
            return [obj], True
        if common.is_string_present(supported, DEPLOYMENT_CONFIG):
            if is_type(obj, "apps/v1", DEPLOYMENT) or is_type(obj, "v1", REPLICATION_CONTROLLER):
                return [self.to_deployment_config(m, common.deep_copy(tmpl_spec), replicas or 0)], True
            if is_type(obj, "v1", POD):
                return [self.to_deployment_config(m, common.deep_copy(spec), 2)], True
            return [obj], True
        if common.is_string_present(supported, DEPLOYMENT):
            if is_type(obj, "apps.openshift.io/v1", DEPLOYMENT_CONFIG):
                return [self.to_deployment(m, common.deep_copy(tmpl_spec), replicas or 0)], True
            if is_type(obj, "v1", REPLICATION_CONTROLLER):
                return [self.to_deployment(m, common.deep_copy(tmpl_spec), replicas or 0)], True
            if is_type(obj, "v1", POD):
                return [self.to_deployment(m, common.deep_copy(spec), 2)], True
            return [obj], True
        if common.is_string_present(supported, REPLICATION_CONTROLLER):
            if is_type(obj, "apps.openshift.io/v1", DEPLOYMENT_CONFIG) or is_type(obj, "apps/v1", DEPLOYMENT):
                return [self.to_replication_controller(m, common.deep_copy(tmpl_spec), replicas or 0)], True
            if is_type(obj, "v1", POD):
                return [self.to_replication_controller(m, common.deep_copy(spec), 2)], True
            return [obj], True
        if common.is_string_present(supported, POD):
            if (is_type(obj, "apps.openshift.io/v1", DEPLOYMENT_CONFIG) or is_type(obj, "apps/v1", DEPLOYMENT)
                    or is_type(obj, "v1", REPLICATION_CONTROLLER)):
                return [self.to_pod(m, common.deep_copy(tmpl_spec), "Always")], True
            return [obj], True
        return None, False

    @staticmethod
    def get_name_and_pod_spec(obj):
        """(name, podspec) for a workload object (``GetNameAndPodSpec``)."""
        m = obj.get("metadata") or {}
        spec = obj.get("spec") or {}
        for gv, kind in (("apps.openshift.io/v1", DEPLOYMENT_CONFIG), ("apps/v1", DEPLOYMENT),
                         ("v1", REPLICATION_CONTROLLER), ("batch/v1", JOB), ("apps/v1", DAEMONSET)):
            if is_type(obj, gv, kind):
                return m.get("name", ""), common.deep_copy((spec.get("template") or {}).get("spec") or {})
        if is_type(obj, "v1", POD):
            return m.get("name", ""), common.deep_copy(spec)
        raise ValueError("Incompatible object type")

    def convert_volumes_kinds_by_policy(self, ps):
        vols = ps.get("volumes")
        if not vols:
            return ps
        names = {v.get("name") for v in vols}
        for c in ps.get("containers") or []:
            kept = []
            for vm in c.get("volumeMounts") or []:
                if vm.get("name") not in names:
                    log.warning("Couldn't find a corresponding volume for volume mount %s", vm.get("name"))
                    continue
                kept.append(vm)
            # the reference assigns the filtered list to a loop copy, so the mounts stay
            if settings.fixed and "volumeMounts" in c:
                c["volumeMounts"] = kept
        ps["volumes"] = [convert_volume_by_supported_kind(v, self.cluster_spec) for v in vols]
        return ps
