"""Helm parameterizers (reference ``internal/parameterizer/``): image names ->
``{{ index .Values.services ... "imagetag" }}`` with the registry prefix for new
images, a shared storage class -> ``{{ .Values.storageclass }}``, ingress host ->
``{{ .Release.Name }}-{{ .Values.ingresshost }}``."""

from ..models import ir as irtypes
from ..models.output import CONTAINERS_TAG, IMAGE_TAG_TAG, PARAMETER_REGISTRY_PREFIX, SERVICES_TAG
from ..utils import common, log, trace
from ..utils.constants import settings


class ImageNameParameterizer:
    def parameterize(self, ir):
        newimages = []
        for c in ir.containers:
            if c.new:
                for img in c.image_names:
                    newimages.append("%s/%s/%s" % (ir.kubernetes.registry_url, ir.kubernetes.registry_namespace, img))
        ir.values.services = {}
        for s in ir.sorted_services():
            ir.values.services[s.name] = {}
            for c in s.containers:
                image = c.get("image", "")
                parts = image.split("/")
                n = ""
                if len(parts) == 3:
                    n += parts[0] + "/"
                if len(parts) > 1:
                    n += parts[1] + "/"
                if common.is_string_present(newimages, image):
                    n = PARAMETER_REGISTRY_PREFIX
                im, tag = common.get_image_name_and_tag(parts[-1])
                ir.values.services[s.name][c.get("name", "")] = tag
                new_tag = ('{{ index .Values.' + SERVICES_TAG + ' "' + s.name + '" "' + CONTAINERS_TAG + '" "'
                           + c.get("name", "") + '" "' + IMAGE_TAG_TAG + '"  }}')
                c["image"] = n + im + ":" + new_tag


class StorageClassParameterizer:
    def parameterize(self, ir):
        sc_map = {}
        for i, st in enumerate(ir.storages):
            if st.storage_type == irtypes.PVC_KIND:
                name = st.pvc_spec.get("storageClassName")
                if name is None:
                    if not settings.fixed:
                        # the reference dereferences a nil StorageClassName here and
                        # aborts the parameterizer; it is reported as a failed parameterizer instead.
                        raise ValueError("invalid memory address or nil pointer dereference (storageClassName)")
                    continue
                sc_map.setdefault(name, []).append(i)
        if len(sc_map) > 1:
            log.warning("Storage class not common across all PVC. Hence, parameterization is skipped.")
            return
        for name, idxs in sc_map.items():
            ir.values.storage_class = name
            for i in idxs:
                ir.storages[i].pvc_spec["storageClassName"] = "{{ .Values.storageclass }}"


class IngressParameterizer:
    def parameterize(self, ir):
        ir.values.ingress_host = ir.target_cluster_spec.host
        ir.target_cluster_spec.host = "{{ .Release.Name }}-{{ .Values.ingresshost }}"


def _go_type(x):
    """``%T`` of the reference's value: ``*parameterize.<type>``, the Go type name being
    the class name with its first letter lowered."""
    n = type(x).__name__
    return "*parameterize." + n[:1].lower() + n[1:]


def get_parameterizers():
    return [ImageNameParameterizer(), StorageClassParameterizer(), IngressParameterizer()]


def parameterize(ir):
    log.info("Begin Parameterization")
    for p in get_parameterizers():
        log.debug("[%s] Begin Parameterization", _go_type(p))
        try:
            with trace.span(type(p).__name__, "parameterizer"):
                p.parameterize(ir)
        except Exception as e:  # noqa: BLE001
            log.warning("[%s] Failed : %s", _go_type(p), e)
        else:
            log.debug("[%s] Done", _go_type(p))
    log.info("Parameterization done")
    return ir
