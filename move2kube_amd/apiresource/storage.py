"""Storage objects: PVC, ConfigMap, Secret, pull secrets (reference
``internal/apiresource/storage.go``).  ConfigMaps and Secrets are converted
into each other when the cluster supports only one of them; PVC volumes fall
back to emptyDir when PVCs are unsupported."""

from ..models import ir as irtypes
from ..utils import common, log
from .base import IAPIResource, is_type

PVC_KIND = irtypes.PVC_KIND
CONFIGMAP_KIND = irtypes.CONFIGMAP_KIND
SECRET_KIND = irtypes.SECRET_KIND


class Storage(IAPIResource):
    def __init__(self, cluster=None):
        self.cluster = cluster

    def get_supported_kinds(self):
        return [PVC_KIND, CONFIGMAP_KIND, SECRET_KIND]

    def create_new_resources(self, ir, supported):
        objs = []
        for st in ir.storages:
            if st.storage_type == CONFIGMAP_KIND:
                if not common.is_string_present(supported, CONFIGMAP_KIND) and common.is_string_present(supported, SECRET_KIND):
                    objs.append(self.create_secret(st))
                else:
                    objs.append(self.create_configmap(st))
            if st.storage_type == SECRET_KIND:
                if not common.is_string_present(supported, SECRET_KIND) and common.is_string_present(supported, CONFIGMAP_KIND):
                    objs.append(self.create_configmap(st))
                else:
                    objs.append(self.create_secret(st))
            if st.storage_type == irtypes.PULL_SECRET_KIND:
                objs.append(self.create_secret(st))
            if st.storage_type == PVC_KIND:
                objs.append(self.create_pvc(st))
        return objs

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        if is_type(obj, "v1", CONFIGMAP_KIND):
            if not common.is_string_present(supported, CONFIGMAP_KIND) and common.is_string_present(supported, SECRET_KIND):
                return [convert_cfgmap_to_secret(obj)], True
            return [obj], True
        if is_type(obj, "v1", SECRET_KIND):
            if not common.is_string_present(supported, SECRET_KIND) and common.is_string_present(supported, CONFIGMAP_KIND):
                return [convert_secret_to_cfgmap(obj)], True
            return [obj], True
        if is_type(obj, "v1", PVC_KIND):
            if not common.is_string_present(supported, PVC_KIND):
                log.warning("PVC not supported in target cluster. [%s]", (obj.get("metadata") or {}).get("name"))
            return [obj], True
        return None, False

    @staticmethod
    def create_configmap(st):
        data = {k: (v.decode("utf-8", "surrogateescape") if isinstance(v, (bytes, bytearray)) else v)
                for k, v in (st.content or {}).items()}
        return {"kind": CONFIGMAP_KIND, "apiVersion": "v1",
                "metadata": {"name": common.make_file_name_compliant(st.name)}, "data": data}

    @staticmethod
    def create_secret(st):
        stype = "Opaque"
        if st.secret_type:
            stype = st.secret_type
        elif st.storage_type == irtypes.PULL_SECRET_KIND:
            stype = "kubernetes.io/dockerconfigjson"
        m = {"name": common.make_file_name_compliant(st.name)}
        if st.annotations:
            m["annotations"] = dict(st.annotations)
        obj = {"kind": SECRET_KIND, "apiVersion": "v1", "metadata": m, "type": stype}
        if st.string_data:
            obj["stringData"] = dict(st.string_data)
        if st.content:
            obj["data"] = dict(st.content)
        return obj

    @staticmethod
    def create_pvc(st):
        log.debug("%r", st.pvc_spec)
        return {"kind": PVC_KIND, "apiVersion": "v1", "metadata": {"name": st.name}, "spec": dict(st.pvc_spec or {})}


def convert_cfgmap_to_secret(cm):
    m = cm.get("metadata") or {}
    md = {"name": m.get("name", "")}
    if m.get("labels"):
        md["labels"] = dict(m["labels"])
    return {"kind": SECRET_KIND, "apiVersion": "v1", "metadata": md, "type": "Opaque",
            "data": {k: (common.go_bytes(v) if isinstance(v, str) else v) for k, v in (cm.get("data") or {}).items()}}


def convert_secret_to_cfgmap(s):
    import base64
    m = s.get("metadata") or {}
    md = {"name": m.get("name", "")}
    if m.get("labels"):
        md["labels"] = dict(m["labels"])
    data = {}
    for k, v in (s.get("data") or {}).items():
        if isinstance(v, (bytes, bytearray)):
            data[k] = v.decode("utf-8", "surrogateescape")
        else:
            try:
                data[k] = base64.b64decode(v).decode("utf-8", "surrogateescape")
            except ValueError:
                data[k] = str(v)
    return {"kind": CONFIGMAP_KIND, "apiVersion": "v1", "metadata": md, "data": data}


def convert_volume_by_supported_kind(volume, cluster):
    if not volume:
        return {}
    if cluster is None:
        return volume
    if volume.get("configMap") is not None:
        if cluster.get_supported_versions(CONFIGMAP_KIND) is None and cluster.get_supported_versions(SECRET_KIND) is not None:
            cm = volume["configMap"]
            sec = {"secretName": cm.get("name", "")}
            if cm.get("items"):
                sec["items"] = cm["items"]
            if cm.get("defaultMode") is not None:
                sec["defaultMode"] = cm["defaultMode"]
            return {"name": volume.get("name", ""), "secret": sec}
        return volume
    if volume.get("secret") is not None:
        if cluster.get_supported_versions(SECRET_KIND) is None and cluster.get_supported_versions(CONFIGMAP_KIND) is not None:
            sec = volume["secret"]
            cm = {"name": sec.get("secretName", "")}
            if sec.get("items"):
                cm["items"] = sec["items"]
            if sec.get("defaultMode") is not None:
                cm["defaultMode"] = sec["defaultMode"]
            return {"name": sec.get("secretName", ""), "configMap": cm}
        return volume
    if volume.get("persistentVolumeClaim") is not None:
        if cluster.get_supported_versions(PVC_KIND) is None:
            log.warning("PVC not supported in target cluster. Defaulting volume [%s] to emptyDir", volume.get("name"))
            return {"name": volume.get("name", ""), "emptyDir": {}}
        return volume
    if volume.get("hostPath") is not None or volume.get("emptyDir") is not None:
        return volume
    log.warning("Unsupported storage type (volume) detected")
    return {}
