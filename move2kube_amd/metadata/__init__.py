"""Metadata loaders (reference ``internal/metadata/``): cluster metadata
(built-in profiles + collected ClusterMetadata), Kubernetes YAMLs to carry over
as cached objects, and QA caches found in the source tree."""


from .. import assets, qaengine
from ..k8s import scheme
from ..models import collection, qa
from ..models import plan as plantypes
from ..utils import common, log
from ..utils.constants import DEFAULT_CLUSTER_TYPE, DEFAULT_STORAGE_CLASS_NAME, settings


class Loader:
    def update_plan(self, input_path, plan):
        raise NotImplementedError

    def load_to_ir(self, plan, ir):
        raise NotImplementedError

    def __repr__(self):
        return "*metadata.%s" % type(self).__name__


def get_loaders():
    return [ClusterMDLoader(), K8sFilesLoader(), QACacheLoader()]


def _read_cluster_metadata(path):
    data = common.read_move2kube_yaml(path)
    cm = collection.ClusterMetadata.from_yaml(data)
    if cm.kind != collection.CLUSTER_METADATA_KIND:
        raise ValueError("The file at path %r is not a valid cluster metadata. Expected kind: %s Actual kind: %s"
                         % (path, collection.CLUSTER_METADATA_KIND, cm.kind))
    return cm


class ClusterMDLoader(Loader):
    def update_plan(self, input_path, plan):
        files = common.get_files_by_ext(input_path, [".yml", ".yaml"])
        for f in files:
            try:
                cm = _read_cluster_metadata(f)
            except Exception:  # noqa: BLE001
                continue
            plan.target_info_artifacts.setdefault(plantypes.K8S_CLUSTER_ARTIFACT, []).append(f)
            if plan.kubernetes.target_cluster_type == DEFAULT_CLUSTER_TYPE:
                plan.kubernetes.target_cluster_type = cm.name
            plan.kubernetes.ignore_unsupported_kinds = True

    def load_to_ir(self, plan, ir):
        clusters = self.get_clusters(plan)
        ttype = plan.kubernetes.target_cluster_type
        tpath = plan.kubernetes.target_cluster_path
        if ttype == "" and tpath == "":
            log.warning("Neither type nor path is specified for the target cluster. Going with the default cluster type: %s",
                        DEFAULT_CLUSTER_TYPE)
            ttype = DEFAULT_CLUSTER_TYPE
        if ttype and tpath:
            raise ValueError("Only one of type or path should be specified for the target cluster.")
        key = tpath if tpath else ttype
        cm = clusters.get(key)
        if cm is None and tpath and settings.fixed:
            # the reference keys clusters by name only, so a path target is never found;
            # "fixed" compat loads that file directly
            try:
                cm = _read_cluster_metadata(tpath)
            except Exception:  # noqa: BLE001
                cm = None
        if cm is None:
            raise ValueError("The requested target cluster %r was not found" % key)
        ir.target_cluster_spec = cm.spec.copy()

    @staticmethod
    def get_clusters(plan):
        clusters = {}
        for name, prof in assets.builtin_clusters().items():
            cm = collection.ClusterMetadata(name)
            # version lists are shared with the packaged profile: consumers only
            # read them, and load_to_ir takes a deep copy (cm.spec.copy())
            cm.spec = collection.ClusterMetadataSpec(prof["storageClasses"], prof["apiKindVersionMap"])
            if not cm.spec.storage_classes:
                cm.spec.storage_classes = [DEFAULT_STORAGE_CLASS_NAME]
            clusters[cm.name] = cm
        for p in plan.target_info_artifacts.get(plantypes.K8S_CLUSTER_ARTIFACT) or []:
            try:
                cm = _read_cluster_metadata(p)
            except Exception as e:  # noqa: BLE001
                log.error("Failed to load the cluster metadata at path %r Error: %r", p, str(e))
                continue
            if not cm.spec.storage_classes:
                cm.spec.storage_classes = [DEFAULT_STORAGE_CLASS_NAME]
            clusters[cm.name] = cm
        return clusters


class K8sFilesLoader(Loader):
    def update_plan(self, input_path, plan):
        for f in common.get_files_by_ext(input_path, [".yml", ".yaml"]):
            try:
                scheme.decode_file(f, "k8s")
            except (OSError, scheme.DecodeError) as e:
                log.debug("Failed to decode the file at path %r as a k8s file. Error: %r", f, str(e))
                continue
            plan.k8s_files.append(f)

    def load_to_ir(self, plan, ir):
        for f in plan.k8s_files:
            try:
                obj = scheme.decode_file(f, "k8s")
            except (OSError, scheme.DecodeError) as e:
                log.error("Failed to decode the file at path %r as a k8s file. Error: %r", f, str(e))
                continue
            ir.cached_objects.append(obj)


class QACacheLoader(Loader):
    def update_plan(self, input_path, plan):
        for f in common.get_files_by_ext(input_path, [".yml", ".yaml"]):
            try:
                data = common.read_move2kube_yaml(f)
            except Exception:  # noqa: BLE001
                continue
            if not isinstance(data, dict) or data.get("kind") != qa.QACACHE_KIND:
                continue
            plan.qa_caches.append(f)

    def load_to_ir(self, plan, ir):
        qaengine.add_caches(list(reversed(plan.qa_caches)))
