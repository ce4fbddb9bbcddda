"""GroupVersion conversion of generated objects (replaces the reference's
``scheme.ConvertToVersion`` call in ``internal/transformer/k8stransformer.go:134-140``).

Most kinds share one wire schema across the versions a cluster profile lists
(Deployment/DaemonSet in apps/v1, apps/v1beta2, extensions/v1beta1 ...), so
conversion re-labels ``apiVersion``.  Ingress changes shape between
``networking.k8s.io/v1`` and ``v1beta1``/``extensions/v1beta1``
(``backend.service{name,port}`` <-> ``serviceName``/``servicePort``,
``defaultBackend`` <-> ``backend``).  Unknown targets raise
:class:`ConversionError`; the caller then writes the object in its original
version, like the reference.
"""

import copy

from . import scheme


class ConversionError(ValueError):
    pass


_V1BETA1_INGRESS = ("networking.k8s.io/v1beta1", "extensions/v1beta1")


def _backend_to_v1beta1(b):
    if b is None:
        return None
    out = {}
    svc = b.get("service")
    if svc is not None:
        out["serviceName"] = svc.get("name", "")
        port = svc.get("port") or {}
        if port.get("name"):
            out["servicePort"] = port["name"]
        else:
            out["servicePort"] = port.get("number", 0)
    if b.get("resource") is not None:
        out["resource"] = b["resource"]
    return out


def _backend_to_v1(b):
    if b is None:
        return None
    out = {}
    if b.get("serviceName") or b.get("servicePort") not in (None, 0, ""):
        port = b.get("servicePort")
        p = {"name": port} if isinstance(port, str) else ({"number": port} if port else {})
        out["service"] = {"name": b.get("serviceName", ""), "port": p}
    if b.get("resource") is not None:
        out["resource"] = b["resource"]
    return out


def _convert_ingress(obj, target):
    src = obj.get("apiVersion", "")
    out = copy.deepcopy(obj)
    out["apiVersion"] = target
    spec = out.get("spec") or {}
    to_beta = target in _V1BETA1_INGRESS
    from_beta = src in _V1BETA1_INGRESS
    if to_beta and not from_beta:
        if "defaultBackend" in spec:
            spec["backend"] = _backend_to_v1beta1(spec.pop("defaultBackend"))
        for rule in spec.get("rules") or []:
            http = rule.get("http") or {}
            for path in http.get("paths") or []:
                if "backend" in path:
                    path["backend"] = _backend_to_v1beta1(path["backend"])
    elif from_beta and not to_beta:
        if "backend" in spec:
            spec["defaultBackend"] = _backend_to_v1(spec.pop("backend"))
        for rule in spec.get("rules") or []:
            http = rule.get("http") or {}
            for path in http.get("paths") or []:
                if "backend" in path:
                    path["backend"] = _backend_to_v1(path["backend"])
    if spec:
        out["spec"] = spec
    return out


def convert_to_version(obj, target_gv):
    kind = obj.get("kind", "")
    if not scheme.is_registered(target_gv, kind, scheme="all"):
        raise ConversionError('converting (%s) %s to %s: no kind "%s" is registered for version "%s"'
                              % (obj.get("apiVersion"), kind, target_gv, kind, target_gv))
    if kind == "Ingress":
        return _convert_ingress(obj, target_gv)
    out = dict(obj)
    out["apiVersion"] = target_gv
    return out
