"""GroupVersion conversion before writing (the reference's
``scheme.ConvertToVersion`` call in ``internal/transformer/k8stransformer.go:128-141``).

The reference converts with a ``runtime.Scheme`` that holds only *external*
types: OpenShift + kube + client-go + Tekton pipelines
(``internal/apiresourceset/k8sapiresourceset.go:45-52``), on apimachinery
v0.19.4 (``go.mod:40``).  ``Scheme.ConvertToVersion(obj, gv)`` then behaves as
follows, and so does :func:`convert_to_version`:

1. ``GroupVersion.KindForGroupVersionKinds`` only matches GVKs registered for
   the object's own Go type, i.e. its own group.  A target in another group
   (``extensions/v1beta1`` -> ``apps/v1``, ``rbac.authorization.k8s.io`` ->
   ``authorization.openshift.io``, ``networking.k8s.io`` ->
   ``extensions/v1beta1``) is a not-registered error.
2. The same group and version is a no-op (``copyAndSetTargetKind``).
3. The same group at another version has no generated conversion function
   between two external packages, so the converter walks the destination
   struct and copies every field by name (``DestFromSource``): it fails as
   soon as a destination field has no source field of the same name and
   kind.  ``_SAME_GROUP`` records, per kind, which version pairs complete
   that walk (field sets compared across the k8s 1.19 API packages); e.g.
   Ingress ``networking.k8s.io/v1`` <-> ``v1beta1`` fails on
   ``defaultBackend``/``backend``, while ``apps/v1beta1`` -> ``apps/v1``
   Deployment succeeds (``rollbackTo`` has no destination and is dropped by
   the typed marshal of the target version, see ``schema.type_for``).

On an error the caller logs it and writes the original object, like the
reference.  With ``M2K_COMPAT=fixed`` (:func:`convert_fixed`) the transformer
instead reshapes an Ingress to the profile's preferred version and relabels
``extensions``/``apps`` workloads, filling a missing ``selector`` from the pod
template labels so the result stays a valid object (DEVIATIONS.md §4).
"""


from ..utils import common
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


def _has_subjects(obj):
    return bool(obj.get("subjects"))


# (group, kind) -> {(src version, dst version): verdict}; verdict True = the
# field walk completes, False = it fails, or a callable on the object that
# returns the same (for checks that depend on a slice being non-empty).
# Pairs not listed are identical field sets and convert.
_SAME_GROUP_FAIL = {
    ("networking.k8s.io", "Ingress"): {("v1", "v1beta1"): False, ("v1beta1", "v1"): False},
    ("apps", "Deployment"): {("v1", "v1beta1"): False, ("v1beta2", "v1beta1"): False},
    ("apps", "StatefulSet"): {("v1beta1", "v1"): False, ("v1beta1", "v1beta2"): False,
                              ("v1", "v1beta1"): False, ("v1beta2", "v1beta1"): False},
    ("autoscaling", "HorizontalPodAutoscaler"): {(a, b): False for a in ("v1", "v2beta1", "v2beta2")
                                                 for b in ("v1", "v2beta1", "v2beta2") if a != b},
    ("certificates.k8s.io", "CertificateSigningRequest"): {("v1", "v1beta1"): False, ("v1beta1", "v1"): False},
    ("apiextensions.k8s.io", "CustomResourceDefinition"): {("v1", "v1beta1"): False, ("v1beta1", "v1"): False},
    ("authorization.k8s.io", "SubjectAccessReview"): {("v1", "v1beta1"): False, ("v1beta1", "v1"): False},
    ("authorization.k8s.io", "LocalSubjectAccessReview"): {("v1", "v1beta1"): False, ("v1beta1", "v1"): False},
    ("node.k8s.io", "RuntimeClass"): {("v1alpha1", "v1beta1"): False, ("v1beta1", "v1alpha1"): False},
    ("tekton.dev", "*"): {("v1alpha1", "v1beta1"): False, ("v1beta1", "v1alpha1"): False},
}
for _k in ("RoleBinding", "ClusterRoleBinding"):
    # rbac v1alpha1 Subject has apiVersion where v1beta1/v1 have apiGroup
    _SAME_GROUP_FAIL[("rbac.authorization.k8s.io", _k)] = {
        (a, b): (lambda o: not _has_subjects(o))
        for a in ("v1alpha1", "v1beta1", "v1") for b in ("v1alpha1", "v1beta1", "v1")
        if a != b and "v1alpha1" in (a, b)}

# why the field walk stops, per (group, kind, destination version): the first
# destination field without a same-named, same-kinded source field
_MISSING_FIELD = {
    ("networking.k8s.io", "Ingress", "v1beta1"): "Spec.Backend not present in src",
    ("networking.k8s.io", "Ingress", "v1"): "Spec.DefaultBackend not present in src",
    ("apps", "Deployment", "v1beta1"): "Spec.RollbackTo not present in src",
    ("apps", "StatefulSet", "v1"): "Status.ObservedGeneration: *int64 and int64 differ",
    ("apps", "StatefulSet", "v1beta2"): "Status.ObservedGeneration: *int64 and int64 differ",
    ("apps", "StatefulSet", "v1beta1"): "Status.ObservedGeneration: int64 and *int64 differ",
    ("autoscaling", "HorizontalPodAutoscaler", "v1"): "Spec.TargetCPUUtilizationPercentage not present in src",
    ("autoscaling", "HorizontalPodAutoscaler", "v2beta1"): "Spec.Metrics: MetricSpec fields differ",
    ("autoscaling", "HorizontalPodAutoscaler", "v2beta2"): "Spec.Behavior not present in src",
    ("rbac.authorization.k8s.io", "RoleBinding", "v1"): "Subjects.APIGroup not present in src",
    ("rbac.authorization.k8s.io", "RoleBinding", "v1beta1"): "Subjects.APIGroup not present in src",
    ("rbac.authorization.k8s.io", "RoleBinding", "v1alpha1"): "Subjects.APIVersion not present in src",
}


def _same_group_ok(obj, group, kind, src_v, dst_v):
    table = _SAME_GROUP_FAIL.get((group, kind)) or _SAME_GROUP_FAIL.get((group, "*")) or {}
    verdict = table.get((src_v, dst_v), True)
    return verdict(obj) if callable(verdict) else verdict


def convert_to_version(obj, target_gv):
    """``Scheme.ConvertToVersion(obj, target_gv)`` on the reference's scheme.
    Returns the converted object (a shallow copy with the target apiVersion;
    the target version's typed marshal drops fields it does not have) or
    raises :class:`ConversionError`."""
    src_gv = obj.get("apiVersion", "")
    kind = obj.get("kind", "")
    if not scheme.is_registered(src_gv, kind, scheme="k8s"):
        raise ConversionError("%s is not registered in scheme %q" % (_go_type(obj), _SCHEME_NAME))
    if src_gv == target_gv:
        return obj
    sg, sv = _split(src_gv)
    tg, tv = _split(target_gv)
    if sg != tg:
        raise ConversionError('%s is not suitable for converting to "%s" in scheme "%s"'
                              % (_go_type(obj), target_gv, _SCHEME_NAME))
    if not scheme.is_registered(target_gv, kind, scheme="k8s") or not _same_group_ok(obj, sg, kind, sv, tv):
        why = _MISSING_FIELD.get((sg, kind.replace("ClusterRoleBinding", "RoleBinding"), tv),
                                 "fields differ between the versions")
        dst = dict(obj, apiVersion=target_gv)
        raise ConversionError("converting (%s) to (%s): %s" % (_go_type(obj), _go_type(dst), why))
    out = dict(obj)
    out["apiVersion"] = target_gv
    return out


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
