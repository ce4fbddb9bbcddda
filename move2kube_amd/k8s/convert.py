"""GroupVersion conversion before writing (the reference's
``scheme.ConvertToVersion`` call in ``internal/transformer/k8stransformer.go:128-141``).

The reference converts with a ``runtime.Scheme`` that holds only *external*
types: OpenShift + kube + client-go + Tekton pipelines
(``internal/apiresourceset/k8sapiresourceset.go:45-52``), on apimachinery
v0.19.4 (``go.mod:40,51``).  ``Scheme.ConvertToVersion(obj, gv)`` then behaves
as follows, and so does :func:`convert_to_version`:

1. ``GroupVersion.KindForGroupVersionKinds`` only matches GVKs registered for
   the object's own Go type, i.e. its own group.  A target in another group
   (``extensions/v1beta1`` -> ``apps/v1``, ``rbac.authorization.k8s.io`` ->
   ``authorization.openshift.io``, ``networking.k8s.io`` ->
   ``extensions/v1beta1``) is a not-registered error.
2. The same group and version is a no-op (``copyAndSetTargetKind``).
3. The same group at another version needs ``s.New(target)`` (an unknown
   target version is a "no kind ... is registered" error) and then
   ``Converter.Convert``.  Since the 1.19 cycle the converter has no
   reflection fallback: it only calls registered or generated conversion
   functions, and none exists between two external API packages (those live
   with the internal types of k8s.io/kubernetes, which this scheme does not
   hold).  So every such pair is an "unknown conversion" error.

On an error the caller logs it and writes the original object, like the
reference; so no input object ever changes its apiVersion here.  With
``M2K_COMPAT=fixed`` (:func:`convert_fixed`) the transformer instead reshapes
an Ingress to the profile's preferred version and relabels ``extensions``/
``apps`` workloads, filling a missing ``selector`` from the pod template
labels so the result stays a valid object (DEVIATIONS.md §4).
"""


from ..utils import common, log
from . import scheme

# What NewNotRegisteredErrForTarget prints as the scheme name: the call site of
# runtime.NewScheme() in the reference.
_SCHEME_NAME = "github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46"


class ConversionError(ValueError):
    pass


def _split(gv):
    if "/" in gv:
        g, v = gv.split("/", 1)
        return g, v
    return "", gv


def _go_type(obj):
    """reflect.Type as printed by %v: ``<package>.<Kind>``; the k8s.io/api,
    OpenShift and Tekton packages are named after their version."""
    return "%s.%s" % (_split(obj.get("apiVersion", ""))[1], obj.get("kind", ""))


def _pkg_path(gv):
    """``reflect.Type.PkgPath()`` of the Go package that holds ``gv``'s types."""
    g, v = _split(gv)
    if g == "":
        return "k8s.io/api/core/" + v
    if g.endswith(".openshift.io"):
        return "github.com/openshift/api/%s/%s" % (g.split(".", 1)[0], v)
    if g == "tekton.dev":
        return "github.com/tektoncd/pipeline/pkg/apis/pipeline/" + v
    if g in ("apiextensions.k8s.io",):
        return "k8s.io/apiextensions-apiserver/pkg/apis/apiextensions/" + v
    if g in ("apiregistration.k8s.io",):
        return "k8s.io/kube-aggregator/pkg/apis/apiregistration/" + v
    return "k8s.io/api/%s/%s" % (g.split(".", 1)[0], v)


def convert_to_version(obj, target_gv):
    """``Scheme.ConvertToVersion(obj, target_gv)`` on the reference's scheme.
    Returns ``obj`` itself when it already has the target version, else raises
    :class:`ConversionError` (see the module docstring)."""
    src_gv = obj.get("apiVersion", "")
    kind = obj.get("kind", "")
    if not scheme.is_registered(src_gv, kind, scheme="k8s"):
        raise ConversionError("no kind is registered for the type %s in scheme %s"
                              % (_go_type(obj), log.go_quote(_SCHEME_NAME)))
    if src_gv == target_gv:
        return obj
    sg = _split(src_gv)[0]
    if sg != _split(target_gv)[0]:
        raise ConversionError("%s is not suitable for converting to %s in scheme %s"
                              % (_go_type(obj), log.go_quote(target_gv), log.go_quote(_SCHEME_NAME)))
    if not scheme.is_registered(target_gv, kind, scheme="k8s"):
        raise ConversionError("no kind %s is registered for version %s in scheme %s"
                              % (log.go_quote(kind), log.go_quote(target_gv), log.go_quote(_SCHEME_NAME)))
    raise ConversionError("converting (%s) %s to (%s) %s: unknown conversion"
                          % (_pkg_path(src_gv), kind, _pkg_path(target_gv), kind))


# -- M2K_COMPAT=fixed: reshape to the profile's version -------------------------

_V1BETA1_INGRESS = ("networking.k8s.io/v1beta1", "extensions/v1beta1")
_WORKLOADS = ("Deployment", "DaemonSet", "ReplicaSet", "StatefulSet")
_WORKLOAD_GROUPS = ("apps", "extensions")


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


def _reshape_ingress(obj, target):
    src = obj.get("apiVersion", "")
    out = common.deep_copy(obj)
    out["apiVersion"] = target
    spec = out.get("spec") or {}
    to_beta = target in _V1BETA1_INGRESS
    from_beta = src in _V1BETA1_INGRESS
    if to_beta and not from_beta:
        if "defaultBackend" in spec:
            spec["backend"] = _backend_to_v1beta1(spec.pop("defaultBackend"))
        conv = _backend_to_v1beta1
    elif from_beta and not to_beta:
        if "backend" in spec:
            spec["defaultBackend"] = _backend_to_v1(spec.pop("backend"))
        conv = _backend_to_v1
    else:
        conv = None
    if conv is not None:
        for rule in spec.get("rules") or []:
            for path in (rule.get("http") or {}).get("paths") or []:
                if "backend" in path:
                    path["backend"] = conv(path["backend"])
    if spec:
        out["spec"] = spec
    return out


def _relabel_workload(obj, target):
    out = common.deep_copy(obj)
    out["apiVersion"] = target
    spec = out.get("spec")
    if isinstance(spec, dict) and not spec.get("selector"):
        labels = ((spec.get("template") or {}).get("metadata") or {}).get("labels")
        if labels:
            spec["selector"] = {"matchLabels": dict(labels)}
    return out


def convert_fixed(obj, target_gv):
    """``M2K_COMPAT=fixed``: follow the profile's preferred version where the
    reference writes an object the target cluster may not serve.  Only Ingress
    and the apps/extensions workloads are reshaped; everything else (RBAC in
    particular, which OpenShift serves under both groups) follows
    :func:`convert_to_version`."""
    kind = obj.get("kind", "")
    src_gv = obj.get("apiVersion", "")
    if src_gv != target_gv and scheme.is_registered(target_gv, kind, scheme="k8s"):
        if kind == "Ingress":
            return _reshape_ingress(obj, target_gv)
        if kind in _WORKLOADS and _split(src_gv)[0] in _WORKLOAD_GROUPS and _split(target_gv)[0] in _WORKLOAD_GROUPS:
            return _relabel_workload(obj, target_gv)
    return convert_to_version(obj, target_gv)
