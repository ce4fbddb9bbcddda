"""Carried-over Kubernetes/OpenShift YAMLs converted to the kinds the target
cluster supports (reference ``internal/apiresource/deployment.go:105-168``,
``internal/apiresource/service.go`` and ``apiresource.go:58-153``):
DeploymentConfig / ReplicationController / Pod(Always) -> Deployment on
Kubernetes and -> DeploymentConfig on OpenShift, Pod(OnFailure) -> Job,
Ingress -> Route on OpenShift.  Re-created objects replace the loaded ones
wholesale (``merge`` = DeepCopyInto), so source replica counts do not
survive: the replica optimizer's 2 does."""

import os
import shutil

import pytest

from move2kube_amd import api
from move2kube_amd.utils import yamlio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "k8s_conversions")


def _run(tmp_path, monkeypatch, cluster):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = str(tmp_path / "src")
    shutil.copytree(FIXTURE, src)
    cache = tmp_path / "qa.yaml"
    cache.write_text(yamlio.dump({
        "apiVersion": "move2kube.konveyor.io/v1alpha1", "kind": "QACache",
        "spec": {"solutions": [{"description": "Choose the cluster type:",
                                "solution": {"type": "Select", "answer": [cluster]}, "resolved": True}]}}))
    out = os.path.join(api.translate(src, str(tmp_path / "out"), name="conv", qacaches=[str(cache)]), "conv")
    return {f: yamlio.load(open(os.path.join(out, f)).read()) for f in sorted(os.listdir(out))}


WORKLOADS = ("legacy-dc", "old-rc", "lone-pod", "plain-dep")


@pytest.mark.parametrize("cluster,kind,api_version", [("Kubernetes", "Deployment", "apps/v1"),
                                                     ("Openshift", "DeploymentConfig", "apps.openshift.io/v1")])
def test_workload_kinds(tmp_path, monkeypatch, cluster, kind, api_version):
    objs = _run(tmp_path, monkeypatch, cluster)
    for name in WORKLOADS:
        o = objs["%s-%s.yaml" % (name, kind.lower())]
        assert (o["apiVersion"], o["kind"]) == (api_version, kind)
        assert o["spec"]["replicas"] == 2
        assert o["spec"]["template"]["spec"]["restartPolicy"] == "Always"
        assert "%s-service.yaml" % name in objs
    job = objs["batch-pod-job.yaml"]
    assert (job["apiVersion"], job["kind"]) == ("batch/v1", "Job")
    assert job["spec"]["template"]["spec"]["restartPolicy"] == "OnFailure"


def test_ingress_and_openshift_extras(tmp_path, monkeypatch):
    k8s = _run(tmp_path / "k", monkeypatch, "Kubernetes")
    assert "web-ing-ingress.yaml" in k8s and "conv-ingress.yaml" in k8s
    assert not any(f.endswith("-route.yaml") or f.endswith("-imagestream.yaml") for f in k8s)
    ocp = _run(tmp_path / "o", monkeypatch, "Openshift")
    assert not any(f.endswith("-ingress.yaml") for f in ocp)
    route = ocp["web-ing-route.yaml"]
    assert route["spec"]["host"] == "web.example.com" and route["spec"]["to"]["name"] == "plain-dep"
    for name in WORKLOADS:
        assert "%s-imagestream.yaml" % name in ocp and "%s-route.yaml" % name in ocp


# -- typed decode (client-go UniversalDeserializer: sigs.k8s.io/yaml + encoding/json)

_DEPLOY = """apiVersion: apps/v1
kind: Deployment
metadata:
  name: d
  labels: {app: d}
spec:
  replicas: %s
  template:
    spec:
      containers:
      - name: c
        image: i
        ports:
        - containerPort: %s
"""


@pytest.mark.parametrize("replicas,port,ok", [
    ("2", "80", True),
    ("2.0", "80", True),          # JSON 2 after the YAML->JSON step
    ("2.5", "80", False),         # not an int32
    ('"2"', "80", False),         # string into *int32
    ("2", '"80"', False),         # string into int32 containerPort
    ("yes", "80", False),         # go-yaml v2: yes is a bool
])
def test_typed_decode_rejects_type_mismatches(replicas, port, ok):
    from move2kube_amd.k8s import scheme
    text = _DEPLOY % (replicas, port)
    if ok:
        assert scheme.decode(text)["spec"]["template"]["spec"]["containers"][0]["ports"][0]["containerPort"] == 80
    else:
        with pytest.raises(scheme.DecodeError, match="cannot unmarshal"):
            scheme.decode(text)


def test_typed_decode_string_maps_and_int_or_string():
    from move2kube_amd.k8s import scheme
    svc = "apiVersion: v1\nkind: Service\nmetadata: {name: s, labels: {version: %s}}\n" \
          "spec: {ports: [{port: 80, targetPort: %s}]}\n"
    assert scheme.decode(svc % ('"1"', "http"))["spec"]["ports"][0]["targetPort"] == "http"
    assert scheme.decode(svc % ('"1"', "8080"))["spec"]["ports"][0]["targetPort"] == 8080
    with pytest.raises(scheme.DecodeError, match="map\\[string\\]string|type string"):
        scheme.decode(svc % ("1", "http"))        # label value must be a string
    with pytest.raises(scheme.DecodeError):
        scheme.decode(svc % ('"1"', "1.5"))       # IntOrString takes no fractions


def test_emitted_objects_decode_back():
    """Every registered object in the expected output trees passes the typed decode."""
    from move2kube_amd.k8s import scheme, schema
    from move2kube_amd.utils import yamlio
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    n = 0
    for dp, _dn, fns in os.walk(golden):
        for fn in fns:
            if not fn.endswith((".yaml", ".yml")):
                continue
            with open(os.path.join(dp, fn)) as f:
                docs = yamlio.load_all_v2(f.read())
            for d in docs:
                if (isinstance(d, dict) and isinstance(d.get("kind"), str) and isinstance(d.get("apiVersion"), str)
                        and scheme.is_registered(d["apiVersion"], d["kind"], "all")):
                    schema.check(d)
                    n += 1
    assert n > 200


# -- GroupVersion conversion before writing (k8stransformer.go:128-141) --------

def _dep(gv, selector=True):
    d = {"apiVersion": gv, "kind": "Deployment", "metadata": {"name": "d"},
         "spec": {"template": {"metadata": {"labels": {"app": "d"}}, "spec": {"containers": []}}}}
    if selector:
        d["spec"]["selector"] = {"matchLabels": {"app": "d"}}
    return d


@pytest.mark.parametrize("obj,target,ok", [
    (_dep("apps/v1"), "apps/v1", True),                                  # no-op
    (_dep("apps/v1beta1"), "apps/v1", False),                            # same group: unknown conversion
    (_dep("apps/v1beta2"), "apps/v1", False),
    (_dep("apps/v1"), "apps/v1beta1", False),
    (_dep("apps/v1"), "apps/v9", False),                                 # no such version
    (_dep("extensions/v1beta1", selector=False), "apps/v1", False),      # other group
    ({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "r"}, "rules": []},
     "authorization.openshift.io/v1", False),
    ({"apiVersion": "rbac.authorization.k8s.io/v1beta1", "kind": "RoleBinding", "metadata": {"name": "r"},
      "subjects": [{"kind": "User", "name": "u"}], "roleRef": {"apiGroup": "", "kind": "Role", "name": "r"}},
     "rbac.authorization.k8s.io/v1", False),
    ({"apiVersion": "rbac.authorization.k8s.io/v1alpha1", "kind": "RoleBinding", "metadata": {"name": "r"},
      "subjects": [], "roleRef": {"apiGroup": "", "kind": "Role", "name": "r"}},
     "rbac.authorization.k8s.io/v1", False),
    ({"apiVersion": "batch/v2alpha1", "kind": "CronJob", "metadata": {"name": "c"}, "spec": {}},
     "batch/v1beta1", False),
    ({"apiVersion": "networking.k8s.io/v1", "kind": "Ingress", "metadata": {"name": "i"}, "spec": {}},
     "networking.k8s.io/v1beta1", False),
    ({"apiVersion": "networking.k8s.io/v1beta1", "kind": "Ingress", "metadata": {"name": "i"}, "spec": {}},
     "networking.k8s.io/v1", False),
    ({"apiVersion": "networking.k8s.io/v1", "kind": "Ingress", "metadata": {"name": "i"}, "spec": {}},
     "extensions/v1beta1", False),
])
def test_convert_to_version_follows_scheme_rules(obj, target, ok):
    from move2kube_amd.k8s import convert
    if ok:
        out = convert.convert_to_version(obj, target)
        assert out["apiVersion"] == target and out["kind"] == obj["kind"]
        assert obj["apiVersion"] != target or out is obj
    else:
        with pytest.raises(convert.ConversionError):
            convert.convert_to_version(obj, target)


def test_cross_group_error_text():
    from move2kube_amd.k8s import convert
    with pytest.raises(convert.ConversionError, match=r'^v1beta1\.Deployment is not suitable for converting '
                                                      r'to "apps/v1" in scheme '):
        convert.convert_to_version(_dep("extensions/v1beta1"), "apps/v1")


@pytest.mark.parametrize("obj,target,msg", [
    (_dep("apps/v1beta1"), "apps/v1",
     "converting (k8s.io/api/apps/v1beta1) Deployment to (k8s.io/api/apps/v1) Deployment: unknown conversion"),
    ({"apiVersion": "route.openshift.io/v1", "kind": "Route"}, "route.openshift.io/v2",
     'no kind "Route" is registered for version "route.openshift.io/v2" in scheme '
     '"github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46"'),
    ({"apiVersion": "example.com/v1", "kind": "Widget"}, "example.com/v2",
     'no kind is registered for the type v1.Widget in scheme '
     '"github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46"'),
])
def test_conversion_error_texts(obj, target, msg):
    """apimachinery v0.19.4: a registered same-group pair has no conversion
    function (no reflection fallback), an unknown target version or source
    type is a not-registered error.  The texts only reach the error log."""
    from move2kube_amd.k8s import convert
    with pytest.raises(convert.ConversionError) as e:
        convert.convert_to_version(obj, target)
    assert str(e.value) == msg


def test_unconverted_object_marshals_as_its_own_version():
    """apps/v1beta1 stays apps/v1beta1 and keeps ``rollbackTo``; an unconverted
    extensions/v1beta1 object keeps an absent selector absent."""
    from move2kube_amd.k8s import schema
    d = _dep("apps/v1beta1")
    d["spec"]["rollbackTo"] = {"revision": 1}
    out = schema.marshal(d)
    assert out["apiVersion"] == "apps/v1beta1" and out["spec"]["rollbackTo"] == {"revision": 1}
    legacy = schema.marshal(_dep("extensions/v1beta1", selector=False))
    assert "selector" not in legacy["spec"]
    assert schema.marshal(_dep("apps/v1", selector=False))["spec"]["selector"] is None


def test_fixed_mode_reshapes_and_fills_selector():
    from move2kube_amd.k8s import convert
    ing = {"apiVersion": "networking.k8s.io/v1", "kind": "Ingress", "metadata": {"name": "i"},
           "spec": {"rules": [{"http": {"paths": [{"path": "/", "backend": {
               "service": {"name": "s", "port": {"number": 80}}}}]}}]}}
    beta = convert.convert_fixed(ing, "networking.k8s.io/v1beta1")
    assert beta["spec"]["rules"][0]["http"]["paths"][0]["backend"] == {"serviceName": "s", "servicePort": 80}
    dep = convert.convert_fixed(_dep("extensions/v1beta1", selector=False), "apps/v1")
    assert dep["apiVersion"] == "apps/v1"
    assert dep["spec"]["selector"] == {"matchLabels": {"app": "d"}}
    role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "r"}, "rules": []}
    with pytest.raises(convert.ConversionError):
        convert.convert_fixed(role, "authorization.openshift.io/v1")


@pytest.mark.parametrize("text,msg", [
    ("version: 3\nservices: {}\n", "Object 'Kind' is missing in 'version: 3\nservices: {}\n'"),
    ("", "Object 'Kind' is missing in ''"),
    ("kind: Pod\n", "Object 'apiVersion' is missing in 'kind: Pod\n'"),
    ("- a\n", "couldn't get version/kind; json parse error: json: cannot unmarshal array into Go value of type "
              'struct { APIVersion string "json:\\"apiVersion,omitempty\\""; Kind string "json:\\"kind,omitempty\\"" }'),
    ("kind: 5\n", "couldn't get version/kind; json parse error: json: cannot unmarshal number into Go struct field "
                  ".kind of type string"),
    ("apiVersion: a/b/c\nkind: Pod\n", "unexpected GroupVersion string: a/b/c"),
    ("apiVersion: v1\nkind: Foo\n", 'no kind "Foo" is registered for version "v1" in scheme '
                                    '"github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46"'),
])
def test_decode_errors_read_like_the_universal_deserializer(text, msg):
    """The YAML serializer's Decode (apimachinery v0.19.4): what the planners
    log at debug level for every YAML file that is not a Kubernetes object."""
    from move2kube_amd.k8s import scheme
    with pytest.raises(scheme.DecodeError) as ei:
        scheme.decode(text)
    assert str(ei.value) == msg
