"""API resource handlers (``internal/apiresource/networkpolicy_test.go`` + fixture)."""

import pytest

from conftest import ref_path
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


def test_no_supported_kinds():
    assert NetworkPolicy().create_new_resources(_ir(), []) == []
    assert NetworkPolicy().create_new_resources(_ir({"svc1": [], "svc2": []}), ["Pod", "Secret"]) == []


def test_no_networks():
    assert NetworkPolicy().create_new_resources(_ir({"svc1": [], "svc2": []}), ["NetworkPolicy"]) == []


@pytest.mark.reference
def test_networks_match_fixture():
    fixture = yamlio.load(open(ref_path("internal", "apiresource", "testdata", "networkpolicy",
                                        "create-new-resources.yaml")).read())
    want = []
    for w in fixture:
        sel = w["spec"]["podselector"]["matchlabels"]
        frm = w["spec"]["ingress"][0]["from"][0]["podselector"]["matchlabels"]
        want.append({"kind": w["typemeta"]["kind"], "apiVersion": w["typemeta"]["apiversion"],
                     "metadata": {"name": w["objectmeta"]["name"]},
                     "spec": {"podSelector": {"matchLabels": sel}, "ingress": [{"from": [{"podSelector": {"matchLabels": frm}}]}]}})
    got = NetworkPolicy().create_new_resources(_ir({"svc1": ["net1"], "svc2": ["net2"]}), ["NetworkPolicy"])
    key = lambda o: o["metadata"]["name"]  # noqa: E731
    assert sorted(got, key=key) == sorted(want, key=key)


def test_convert_to_cluster_supported_kinds():
    np_obj = {"kind": "NetworkPolicy", "apiVersion": "networking.k8s.io/v1", "metadata": {"name": "net1"},
              "spec": {"podSelector": {"matchLabels": {"foo": "bar"}}}}
    secret = {"kind": "Secret", "apiVersion": "v1", "metadata": {"name": "sec1"}, "type": "Opaque", "data": {"key1": "dmFsMQ=="}}
    h = NetworkPolicy()
    assert h.convert_to_cluster_supported_kinds({"kind": "NetworkPolicy"}, [], [], None)[1] is False
    assert h.convert_to_cluster_supported_kinds(np_obj, [], [], None)[1] is False
    assert h.convert_to_cluster_supported_kinds(secret, ["Pod", "NetworkPolicy", "Secret"], [], None)[1] is False
    objs, ok = h.convert_to_cluster_supported_kinds(np_obj, ["Pod", "NetworkPolicy", "Secret"], [], None)
    assert ok and objs == [np_obj]
