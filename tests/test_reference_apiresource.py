"""``internal/apiresource/networkpolicy_test.go``, one pytest per Go subtest,
comparing whole objects as the Go test does (``nil`` and an empty list are
different there, ``None`` and ``[]`` here)."""

import pytest

from conftest import ref_path
from goequal import assert_deep_equal
from move2kube_amd.apiresource.others import NetworkPolicy
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import yamlio


def _ir(nets=None):
    ir = irtypes.new_ir(plantypes.new_plan())
    for name, n in (nets or {}).items():
        s = irtypes.new_service_with_name(name)
        s.networks = list(n)
        ir.services[name] = s
    return ir


def _net_policy(name):
    """helperCreateNetworkPolicy"""
    return {"kind": "NetworkPolicy", "apiVersion": "networking.k8s.io/v1", "metadata": {"name": name},
            "spec": {"podSelector": {"matchLabels": {"foo": "bar"}}}}


def _secret(name, data):
    """helperCreateSecret (``Data`` is base64 in the object's JSON form)"""
    return {"kind": "Secret", "apiVersion": "v1", "metadata": {"name": name}, "type": "Opaque", "data": data}


def test_get_supported_kinds():
    assert NetworkPolicy().get_supported_kinds()


@pytest.mark.parametrize("services,kinds,want", [
    pytest.param(None, [], None, id="empty IR and empty supported kinds"),
    pytest.param(None, ["NetworkPolicy"], [], id="empty IR and some supported kinds"),
    pytest.param({"svc1": [], "svc2": []}, [], None, id="IR with some services and empty supported kinds"),
    pytest.param({"svc1": [], "svc2": []}, ["Pod", "Secret"], None,
                 id="IR with some services and but no acceptable supported kinds"),
    pytest.param({"svc1": [], "svc2": []}, ["NetworkPolicy"], [],
                 id="IR with some services and no networks and some supported kinds"),
])
def test_create_new_resources(services, kinds, want):
    assert_deep_equal(NetworkPolicy().create_new_resources(_ir(services), kinds), want)


def _go_yaml_network_policy(w):
    """A NetworkPolicy as common.ReadYaml fills it from the fixture (go-yaml
    keys are the lowercased Go field names), in the object's JSON form."""
    out = {"kind": w["typemeta"]["kind"], "apiVersion": w["typemeta"]["apiversion"],
           "metadata": {"name": w["objectmeta"]["name"]}, "spec": {}}
    spec = w["spec"]
    out["spec"]["podSelector"] = {"matchLabels": spec["podselector"]["matchlabels"]}
    out["spec"]["ingress"] = [{"from": [{"podSelector": {"matchLabels": f["podselector"]["matchlabels"]}}
                                        for f in rule["from"]]} for rule in spec["ingress"]]
    return out


@pytest.mark.reference
def test_create_new_resources_with_some_networks_and_some_supported_kinds():
    with open(ref_path("internal", "apiresource", "testdata", "networkpolicy", "create-new-resources.yaml")) as f:
        want = [_go_yaml_network_policy(w) for w in yamlio.load(f.read())]
    actual = NetworkPolicy().create_new_resources(_ir({"svc1": ["net1"], "svc2": ["net2"]}), ["NetworkPolicy"])
    assert len(actual) == len(want)
    for w in want:   # each expected policy exactly once, in any order (Go ranges over a map)
        assert sum(1 for a in actual if a == w) == 1, (w, actual)


@pytest.mark.parametrize("obj,kinds,want", [
    pytest.param({"kind": "NetworkPolicy"}, [], None, id="empty object and empty supported kinds"),
    pytest.param(_net_policy("net1"), [], None, id="some object and empty supported kinds"),
    pytest.param(_secret("sec1", {"key1": "dmFsMQ=="}), ["Pod", "NetworkPolicy", "Secret"], None,
                 id="invalid object and correct supported kinds"),
    pytest.param(_net_policy("net1"), ["Pod", "NetworkPolicy", "Secret"], [_net_policy("net1")],
                 id="some object and correct supported kinds"),
])
def test_convert_to_cluster_supported_kinds(obj, kinds, want):
    actual, ok = NetworkPolicy().convert_to_cluster_supported_kinds(obj, kinds, [], None)
    assert ok is (want is not None)
    if want is not None:
        assert_deep_equal(actual, want)
