"""Storage objects on clusters that lack a kind (reference
``internal/apiresource/storage.go``): ConfigMaps and Secrets become each other
when the cluster has only one of them (``CreateNewResources`` :42-73,
``ConvertToClusterSupportedKinds`` :75-97, ``convertCfgMapToSecret`` /
``convertSecretToCfgMap`` :160-196), volumes follow (``convertVolumeBySupportedKind``
:243-277, including its quirk of naming a converted Secret volume after the
secret), and a PVC volume becomes an emptyDir where PVCs are missing."""

import base64

import pytest

import logparse
from move2kube_amd.apiresource import storage as st
from move2kube_amd.models import ir as irtypes
from move2kube_amd.utils import log

CM, SEC, PVC = st.CONFIGMAP_KIND, st.SECRET_KIND, st.PVC_KIND


def _kinds(objs):
    return [o["kind"] for o in objs]


@pytest.mark.parametrize("supported,want", [
    ([CM, SEC, PVC], [CM, SEC, SEC, PVC]),
    ([SEC, PVC], [SEC, SEC, SEC, PVC]),        # no ConfigMap: the ConfigMap storage becomes a Secret
    ([CM, PVC], [CM, CM, SEC, PVC]),           # no Secret: the Secret storage becomes a ConfigMap (pull secret stays)
    ([], [CM, SEC, SEC, PVC]),                 # neither: both kept as they are
])
def test_create_new_resources(supported, want):
    storages = [irtypes.Storage("cfg_a", CM, content={"k": b"v"}),
                irtypes.Storage("sec", SEC, content={"p": b"s"}),
                irtypes.Storage("pull", irtypes.PULL_SECRET_KIND, content={".dockerconfigjson": b"{}"}),
                irtypes.Storage("data", PVC, pvc_spec={"accessModes": ["ReadWriteOnce"]})]

    class _IR:
        pass
    ir = _IR()
    ir.storages = storages
    objs = st.Storage().create_new_resources(ir, supported)
    assert _kinds(objs) == want
    assert objs[0]["metadata"]["name"] == "cfg-a"          # MakeFileNameCompliant
    pull = objs[2]
    assert pull["type"] == "kubernetes.io/dockerconfigjson"
    assert objs[3] == {"kind": PVC, "apiVersion": "v1", "metadata": {"name": "data"},
                       "spec": {"accessModes": ["ReadWriteOnce"]}}


def test_create_secret_fields():
    s = st.Storage.create_secret(irtypes.Storage("git", SEC, content={"a": b"1"}, annotations={"x": "y"},
                                                 secret_type="kubernetes.io/ssh-auth", string_data={"k": "v"}))
    assert s == {"kind": SEC, "apiVersion": "v1", "metadata": {"name": "git", "annotations": {"x": "y"}},
                 "type": "kubernetes.io/ssh-auth", "stringData": {"k": "v"}, "data": {"a": b"1"}}
    assert st.Storage.create_secret(irtypes.Storage("o", SEC))["type"] == "Opaque"


def test_configmap_content_bytes_become_text():
    cm = st.Storage.create_configmap(irtypes.Storage("c", CM, content={"a": b"x\xff", "b": "y"}))
    assert cm["data"] == {"a": "x\udcff", "b": "y"}


@pytest.mark.parametrize("supported,kind_in,kind_out", [
    ([SEC], CM, SEC), ([CM, SEC], CM, CM), ([CM], SEC, CM), ([CM, SEC], SEC, SEC), ([], SEC, SEC),
])
def test_convert_to_cluster_supported_kinds(supported, kind_in, kind_out):
    labels = {"app": "a"}
    if kind_in == CM:
        obj = {"kind": CM, "apiVersion": "v1", "metadata": {"name": "c", "labels": labels}, "data": {"k": "v"}}
    else:
        obj = {"kind": SEC, "apiVersion": "v1", "metadata": {"name": "c", "labels": labels},
               "data": {"k": base64.b64encode(b"v").decode()}}
    objs, ok = st.Storage().convert_to_cluster_supported_kinds(obj, supported, [], None)
    assert ok and len(objs) == 1 and objs[0]["kind"] == kind_out
    assert objs[0]["metadata"] == {"name": "c", "labels": labels}
    if kind_in != kind_out:
        if kind_out == SEC:
            assert objs[0]["type"] == "Opaque" and objs[0]["data"] == {"k": b"v"}
        else:
            assert objs[0]["data"] == {"k": "v"}


def test_pvc_on_a_cluster_without_pvcs_is_kept_with_a_warning(capsys):
    log.set_verbose(False)
    obj = {"kind": PVC, "apiVersion": "v1", "metadata": {"name": "d"}}
    assert st.Storage().convert_to_cluster_supported_kinds(obj, [CM], [], None) == ([obj], True)
    assert logparse.logged(capsys.readouterr().err, "PVC not supported in target cluster. [d]", "warning")
    assert st.Storage().convert_to_cluster_supported_kinds({"kind": "Pod", "apiVersion": "v1"}, [], [], None) \
        == (None, False)


def test_secret_to_configmap_data_forms():
    s = {"metadata": {"name": "n"}, "data": {"raw": b"r\xff", "b64": base64.b64encode(b"text").decode(),
                                             "bad": "not base64!"}}
    cm = st.convert_secret_to_cfgmap(s)
    assert cm == {"kind": CM, "apiVersion": "v1", "metadata": {"name": "n"},
                  "data": {"raw": "r\udcff", "b64": "text", "bad": "not base64!"}}


class _Cluster:
    def __init__(self, kinds):
        self.kinds = kinds

    def get_supported_versions(self, kind):
        return ["v1"] if kind in self.kinds else None


@pytest.mark.parametrize("volume,kinds,want", [
    ({}, [CM], {}),
    ({"name": "v", "configMap": {"name": "c", "items": [{"key": "k", "path": "p"}], "defaultMode": 420}}, [SEC],
     {"name": "v", "secret": {"secretName": "c", "items": [{"key": "k", "path": "p"}], "defaultMode": 420}}),
    ({"name": "v", "configMap": {"name": "c"}}, [CM, SEC], {"name": "v", "configMap": {"name": "c"}}),
    # the converted volume is named after the secret (convertSecretVolumeToCfgMapVolume)
    ({"name": "v", "secret": {"secretName": "s", "items": [{"key": "k", "path": "p"}], "defaultMode": 256}}, [CM],
     {"name": "s", "configMap": {"name": "s", "items": [{"key": "k", "path": "p"}], "defaultMode": 256}}),
    ({"name": "v", "secret": {"secretName": "s"}}, [SEC], {"name": "v", "secret": {"secretName": "s"}}),
    ({"name": "v", "persistentVolumeClaim": {"claimName": "d"}}, [CM], {"name": "v", "emptyDir": {}}),
    ({"name": "v", "persistentVolumeClaim": {"claimName": "d"}}, [PVC],
     {"name": "v", "persistentVolumeClaim": {"claimName": "d"}}),
    ({"name": "v", "hostPath": {"path": "/x"}}, [], {"name": "v", "hostPath": {"path": "/x"}}),
    ({"name": "v", "emptyDir": {}}, [], {"name": "v", "emptyDir": {}}),
    ({"name": "v", "nfs": {"server": "s"}}, [], {}),
])
def test_convert_volume_by_supported_kind(volume, kinds, want, capsys):
    log.set_verbose(False)
    assert st.convert_volume_by_supported_kind(volume, _Cluster(kinds)) == want
    err = capsys.readouterr().err
    if "persistentVolumeClaim" in volume and PVC not in kinds:
        assert logparse.logged(err, "PVC not supported in target cluster. Defaulting volume [v] to emptyDir",
                               "warning")
    if "nfs" in volume:
        assert logparse.logged(err, "Unsupported storage type (volume) detected", "warning")


def test_volume_without_cluster_metadata_is_kept():
    v = {"name": "v", "nfs": {}}
    assert st.convert_volume_by_supported_kind(v, None) is v
