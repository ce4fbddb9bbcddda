"""The type registry ("scheme") used to recognise and decode Kubernetes YAMLs.

The reference decodes input YAMLs with a runtime.Scheme made of OpenShift +
kube + client-go + Tekton types (``internal/apiresourceset/k8sapiresourceset.go:45-58``)
and a separate Knative scheme (``knativeapiresourceset.go:38-43``).  A file is
a Kubernetes file iff its ``apiVersion``/``kind`` is registered.  The tables
below list the group/versions and kinds of those API packages (k8s 1.19,
OpenShift 4.6, Tekton pipelines 0.18 / triggers 0.10, Knative serving 0.19).
"""

from . import schema
from ..utils import yamlio

_CORE_V1 = ("Binding ComponentStatus ConfigMap Endpoints Event LimitRange Namespace Node PersistentVolume "
            "PersistentVolumeClaim Pod PodTemplate ReplicationController ResourceQuota Secret Service "
            "ServiceAccount EphemeralContainers")
_APPS = "ControllerRevision DaemonSet Deployment ReplicaSet StatefulSet"

K8S_GVKS = {
    "v1": _CORE_V1,
    "apps/v1": _APPS,
    "apps/v1beta1": "ControllerRevision Deployment StatefulSet",
    "apps/v1beta2": _APPS,
    "extensions/v1beta1": "DaemonSet Deployment Ingress NetworkPolicy PodSecurityPolicy ReplicaSet",
    "batch/v1": "Job",
    "batch/v1beta1": "CronJob",
    "batch/v2alpha1": "CronJob",
    "networking.k8s.io/v1": "Ingress IngressClass NetworkPolicy",
    "networking.k8s.io/v1beta1": "Ingress IngressClass",
    "rbac.authorization.k8s.io/v1": "ClusterRole ClusterRoleBinding Role RoleBinding",
    "rbac.authorization.k8s.io/v1beta1": "ClusterRole ClusterRoleBinding Role RoleBinding",
    "rbac.authorization.k8s.io/v1alpha1": "ClusterRole ClusterRoleBinding Role RoleBinding",
    "autoscaling/v1": "HorizontalPodAutoscaler",
    "autoscaling/v2beta1": "HorizontalPodAutoscaler",
    "autoscaling/v2beta2": "HorizontalPodAutoscaler",
    "policy/v1beta1": "PodDisruptionBudget PodSecurityPolicy Eviction",
    "storage.k8s.io/v1": "CSIDriver CSINode StorageClass VolumeAttachment",
    "storage.k8s.io/v1beta1": "CSIDriver CSINode StorageClass VolumeAttachment",
    "storage.k8s.io/v1alpha1": "VolumeAttachment",
    "scheduling.k8s.io/v1": "PriorityClass",
    "scheduling.k8s.io/v1beta1": "PriorityClass",
    "scheduling.k8s.io/v1alpha1": "PriorityClass",
    "coordination.k8s.io/v1": "Lease",
    "coordination.k8s.io/v1beta1": "Lease",
    "certificates.k8s.io/v1": "CertificateSigningRequest",
    "certificates.k8s.io/v1beta1": "CertificateSigningRequest",
    "admissionregistration.k8s.io/v1": "MutatingWebhookConfiguration ValidatingWebhookConfiguration",
    "admissionregistration.k8s.io/v1beta1": "MutatingWebhookConfiguration ValidatingWebhookConfiguration",
    "apiextensions.k8s.io/v1": "CustomResourceDefinition",
    "apiextensions.k8s.io/v1beta1": "CustomResourceDefinition",
    "apiregistration.k8s.io/v1": "APIService",
    "apiregistration.k8s.io/v1beta1": "APIService",
    "authentication.k8s.io/v1": "TokenReview",
    "authentication.k8s.io/v1beta1": "TokenReview",
    "authorization.k8s.io/v1": "LocalSubjectAccessReview SelfSubjectAccessReview SelfSubjectRulesReview SubjectAccessReview",
    "authorization.k8s.io/v1beta1": "LocalSubjectAccessReview SelfSubjectAccessReview SelfSubjectRulesReview SubjectAccessReview",
    "discovery.k8s.io/v1beta1": "EndpointSlice",
    "events.k8s.io/v1": "Event",
    "events.k8s.io/v1beta1": "Event",
    "node.k8s.io/v1beta1": "RuntimeClass",
    "node.k8s.io/v1alpha1": "RuntimeClass",
    "settings.k8s.io/v1alpha1": "PodPreset",
    "flowcontrol.apiserver.k8s.io/v1alpha1": "FlowSchema PriorityLevelConfiguration",
    # OpenShift 4.6
    "apps.openshift.io/v1": "DeploymentConfig DeploymentConfigRollback DeploymentLog DeploymentRequest",
    "route.openshift.io/v1": "Route",
    "image.openshift.io/v1": "Image ImageSignature ImageStream ImageStreamImage ImageStreamImport ImageStreamLayers "
                             "ImageStreamMapping ImageStreamTag ImageTag",
    "build.openshift.io/v1": "Build BuildConfig BuildLog BuildRequest BinaryBuildRequestOptions",
    "template.openshift.io/v1": "Template TemplateInstance BrokerTemplateInstance",
    "project.openshift.io/v1": "Project ProjectRequest",
    "authorization.openshift.io/v1": "ClusterRole ClusterRoleBinding Role RoleBinding RoleBindingRestriction "
                                     "LocalResourceAccessReview LocalSubjectAccessReview ResourceAccessReview "
                                     "SelfSubjectRulesReview SubjectAccessReview SubjectRulesReview",
    "security.openshift.io/v1": "SecurityContextConstraints PodSecurityPolicyReview PodSecurityPolicySelfSubjectReview "
                                "PodSecurityPolicySubjectReview RangeAllocation",
    "quota.openshift.io/v1": "AppliedClusterResourceQuota ClusterResourceQuota",
    "network.openshift.io/v1": "ClusterNetwork EgressNetworkPolicy HostSubnet NetNamespace",
    "oauth.openshift.io/v1": "OAuthAccessToken OAuthAuthorizeToken OAuthClient OAuthClientAuthorization",
    "user.openshift.io/v1": "Group Identity User UserIdentityMapping",
    "config.openshift.io/v1": "APIServer Authentication Build ClusterOperator ClusterVersion Console DNS FeatureGate "
                              "Image Infrastructure Ingress Network OAuth OperatorHub Project Proxy Scheduler",
    "operator.openshift.io/v1": "Authentication Console DNS Etcd IngressController KubeAPIServer Network OpenShiftAPIServer",
    "samples.operator.openshift.io/v1": "Config",
    # Tekton pipelines 0.18 (+ triggers registered through the same scheme helper)
    "tekton.dev/v1alpha1": "ClusterTask Condition Pipeline PipelineResource PipelineRun Run Task TaskRun",
    "tekton.dev/v1beta1": "ClusterTask Pipeline PipelineRun Task TaskRun",
}

KNATIVE_GVKS = {
    "serving.knative.dev/v1": "Configuration Revision Route Service",
    "serving.knative.dev/v1alpha1": "Configuration DomainMapping Revision Route Service",
    "serving.knative.dev/v1beta1": "Configuration Revision Route Service",
}

TRIGGERS_GVKS = {
    "triggers.tekton.dev/v1alpha1": "ClusterTriggerBinding EventListener TriggerBinding TriggerTemplate Trigger",
}


def _build(table):
    return {gv: set(kinds.split()) for gv, kinds in table.items()}


_K8S = _build(K8S_GVKS)
_KNATIVE = _build(KNATIVE_GVKS)
_ALL = dict(_K8S)
for _gv, _kinds in list(_KNATIVE.items()) + list(_build(TRIGGERS_GVKS).items()):
    _ALL.setdefault(_gv, set()).update(_kinds)


class DecodeError(ValueError):
    pass


def is_registered(gv, kind, scheme="k8s"):
    table = _K8S if scheme == "k8s" else _KNATIVE if scheme == "knative" else _ALL
    return kind in table.get(gv, ())


def decode(data, scheme="k8s"):
    """UniversalDeserializer().Decode: first YAML document -> object dict.

    Raises DecodeError when the document has no registered apiVersion/kind,
    or is nested too deeply for the recursive checks (this file only)."""
    try:
        return _decode(data, scheme)
    except RecursionError:
        raise DecodeError("document nested too deeply") from None


# runtime.NewScheme() names a scheme after its call site
# (naming.GetNameFromCallsite); the reference's schemes are created at these
# lines.  The path prefix depends on where the binary was built (parity unpinned).
_SCHEME_NAMES = {"k8s": "github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46",
                 "knative": "github.com/konveyor/move2kube/internal/apiresourceset/knativeapiresourceset.go:39"}
_FIND_KIND = ('struct { APIVersion string "json:\\"apiVersion,omitempty\\""; '
              'Kind string "json:\\"kind,omitempty\\"" }')


def _json_kind(v):
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    return "array" if isinstance(v, list) else "object"


def _interpret(obj):
    """``SimpleMetaFactory.Interpret``: apiVersion and kind through
    json.Unmarshal into a two-field struct (the first type error in document
    order), then ``schema.ParseGroupVersion``."""
    pre = "couldn't get version/kind; json parse error: "
    if obj is None:
        return "", ""
    if not isinstance(obj, dict):
        raise DecodeError(pre + "json: cannot unmarshal %s into Go value of type %s" % (_json_kind(obj), _FIND_KIND))
    for key in obj:
        if key in ("apiVersion", "kind"):
            v = obj[key]
            if v is not None and not isinstance(v, str):
                raise DecodeError(pre + "json: cannot unmarshal %s into Go struct field .%s of type string"
                                  % (_json_kind(v), key))
    gv = obj.get("apiVersion") or ""
    if gv.count("/") > 1:
        raise DecodeError("unexpected GroupVersion string: %s" % gv)
    return gv, obj.get("kind") or ""


def _decode(data, scheme):
    """The YAML serializer's ``Decode`` (apimachinery v0.19.4
    ``runtime/serializer/json``) for the reference's schemes, with its error
    texts: a YAML error, ``Interpret``, ``Object 'Kind' is missing in
    '<input>'``, ``Object 'apiVersion' is missing in '<input>'``, a kind the
    scheme does not register."""
    text = data.decode("utf-8", "surrogateescape") if isinstance(data, bytes) else data
    try:
        # sigs.k8s.io/yaml converts YAML to JSON with go-yaml v2 scalars
        docs = yamlio.load_all_v2(text)
    except (yamlio.YAMLError, ValueError) as e:
        raise DecodeError("error converting YAML to JSON: %s" % e)
    obj = docs[0] if docs else None
    gv, kind = _interpret(obj)
    if not kind:
        raise DecodeError("Object 'Kind' is missing in '%s'" % text)
    version = gv.rsplit("/", 1)[-1] if gv else ""
    if not version:
        raise DecodeError("Object 'apiVersion' is missing in '%s'" % text)
    if not is_registered(gv, kind, scheme):
        raise DecodeError('no kind "%s" is registered for version "%s" in scheme "%s"'
                          % (kind, gv, _SCHEME_NAMES.get(scheme, _SCHEME_NAMES["k8s"])))
    md = obj.get("metadata")
    if md is not None and not isinstance(md, dict):
        raise DecodeError("metadata must be an object")
    try:
        schema.check(obj)
    except ValueError as e:
        raise DecodeError(str(e))
    return obj


def decode_file(path, scheme="k8s"):
    from ..utils.common import read_bytes  # a FIFO in the tree is an error, not a hang
    return decode(read_bytes(path), scheme)


# version priority inside a group when it differs from the table order above
_PRIORITY_OVERRIDES = {"apps": ["v1", "v1beta2", "v1beta1"]}


def prioritized_versions_for_group(group):
    """``runtime.Scheme.PrioritizedVersionsForGroup`` for the k8s scheme: the
    registered group/versions of ``group``, most preferred first."""
    if group in _PRIORITY_OVERRIDES:
        return [(group + "/" + v) for v in _PRIORITY_OVERRIDES[group]]
    out = []
    for gv in K8S_GVKS:
        g = gv.split("/")[0] if "/" in gv else ""
        if g == group:
            out.append(gv)
    return out
