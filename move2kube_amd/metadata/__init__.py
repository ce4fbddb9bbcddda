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
    """``getClusterMetadata`` (clustermdloader.go:121-133)."""
    from ..models.base import read_document
    try:
        cm = read_document(path, collection.ClusterMetadata.from_yaml, "CLUSTER_METADATA")
    except Exception as e:  # noqa: BLE001
        log.debug("Failed to read the cluster metadata at path %r Error: %r", path, common.go_error_text(e))
        raise
    if cm.kind != collection.CLUSTER_METADATA_KIND:
        err = ValueError("The file at path %s is not a valid cluster metadata. Expected kind: %s Actual kind: %s"
                         % (log.go_quote(path), collection.CLUSTER_METADATA_KIND, cm.kind))
        log.debug(str(err))
        raise err
    return cm


class ClusterMDLoader(Loader):
    def update_plan(self, input_path, plan):
        try:
            files = common.get_files_by_ext(input_path, [".yml", ".yaml"])
        except (OSError, ValueError) as e:
            log.warning("Failed to fetch the cluster metadata yamls at path %r Error: %r", input_path, str(e))
            raise
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
        target = "{%s %s}" % (ttype, tpath)   # %v of the TargetCluster struct
        if ttype and tpath:
            raise ValueError("Only one of type or path should be specified for the target cluster. Target cluster: %s"
                             % target)
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
            raise ValueError("The requested target cluster %s was not found" % target)
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
                log.debug("No storage class in the cluster %s, adding [default] storage class", name)
            clusters[cm.name] = cm
        for p in plan.target_info_artifacts.get(plantypes.K8S_CLUSTER_ARTIFACT) or []:
            try:
                cm = _read_cluster_metadata(p)
            except Exception as e:  # noqa: BLE001
                log.error("Failed to load the cluster metadata at path %r Error: %r", p, str(e))
                continue
            if not cm.spec.storage_classes:
                cm.spec.storage_classes = [DEFAULT_STORAGE_CLASS_NAME]
                log.debug("No storage class in the cluster %s at path %r, adding [default] storage class", cm.name, p)
            clusters[cm.name] = cm
        return clusters


class K8sFilesLoader(Loader):
    def update_plan(self, input_path, plan):
        try:
            files = common.get_files_by_ext(input_path, [".yml", ".yaml"])
        except (OSError, ValueError) as e:
            log.error("Unable to fetch yaml files at path %r Error: %r", input_path, str(e))
            raise
        for f in files:
            try:
                data = common.read_bytes(f)
            except OSError as e:
                log.debug("Failed to read the yaml file at path %r Error: %r", f, common.go_path_error(e, "open"))
                continue
            try:
                scheme.decode(data, "k8s")
            except scheme.DecodeError as e:
                log.debug("Failed to decode the file at path %r as a k8s file. Error: %r", f, str(e))
                continue
            plan.k8s_files.append(f)

    def load_to_ir(self, plan, ir):
        for f in plan.k8s_files:
            try:
                data = common.read_bytes(f)
            except OSError as e:
                log.error("Failed to read the k8s file at path %r Error: %r", f, common.go_path_error(e, "open"))
                continue
            try:
                obj = scheme.decode(data, "k8s")
            except scheme.DecodeError as e:
                log.error("Failed to decode the file at path %r as a k8s file. Error: %r", f, str(e))
                continue
            ir.cached_objects.append(obj)


class QACacheLoader(Loader):
    def update_plan(self, input_path, plan):
        try:
            files = common.get_files_by_ext(input_path, [".yml", ".yaml"])
        except (OSError, ValueError) as e:
            log.error("Unable to fetch yaml files at path %r Error: %r", input_path, str(e))
            raise
        for f in files:
            try:
                data = common.read_move2kube_yaml(f)
            except Exception as e:  # noqa: BLE001
                log.debug("Failed to read the yaml file at path %r Error: %r", f, common.go_error_text(e))
                continue
            if not isinstance(data, dict) or data.get("kind") != qa.QACACHE_KIND:
                continue
            plan.qa_caches.append(f)

    def load_to_ir(self, plan, ir):
        qaengine.add_caches(list(reversed(plan.qa_caches)))
