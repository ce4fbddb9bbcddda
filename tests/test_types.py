"""Model-type merge semantics, mirroring the reference's ``types/*_test.go``:

* ``types/collection/cluster_test.go`` - ClusterMetadata.Merge, GetSupportedVersions
* ``types/collection/{image,cfcontainerizers,cfinstanceapps}_test.go`` - the
  New* constructors set kind and apiVersion
* ``types/output/helmvaluesoutput_test.go`` - HelmValues.Merge
* ``types/info/versioninfo_test.go`` - VersionInfo.IsSameVersion
* ``types/plan/plan_test.go`` - KubernetesOutput.Merge, Service.Add*,
  Plan.AddServicesToPlan
"""

import pytest

from move2kube_amd.models import collection, info, output, plan


# -- collection ----------------------------------------------------------------

@pytest.mark.parametrize("cls,kind", [(collection.ImageInfo, "ImageMetadata"),
                                      (collection.CfContainerizers, "CfContainerizers"),
                                      (collection.CfInstanceApps, "CfInstanceApps")])
def test_new_collection_types(cls, kind):
    o = cls()
    assert o.kind == kind and o.api_version == "move2kube.konveyor.io/v1alpha1"


def _cmeta(name="", kind=None):
    c = collection.new_cluster_metadata(name)
    if kind is not None:
        c.kind = kind
    return c


def _cm_state(c):
    return (c.kind, c.api_version, c.name, list(c.spec.storage_classes),
            dict(c.spec.api_kind_version_map), c.spec.host)


def test_cluster_merge_two_empty():
    a, b, want = _cmeta(kind=""), _cmeta(kind=""), _cmeta(kind="")
    assert a.merge(b)
    assert _cm_state(a) == _cm_state(want)


def test_cluster_merge_non_empty_into_empty():
    a = _cmeta(kind="")
    b = _cmeta("ctxname1")
    want = _cmeta("")
    want.name = "ctxname1"
    want.spec.storage_classes = ["default"]
    assert a.merge(b)
    assert _cm_state(a) == _cm_state(want)


def test_cluster_merge_different_kinds():
    assert not _cmeta(kind="kind1").merge(_cmeta(kind="kind2"))


def test_cluster_merge_version_maps():
    val1 = ["1.0.0", "1.1.0", "1.1.1"]
    val2 = ["2.0.0", "2.2.0", "2.2.2"]
    a = _cmeta()
    a.spec.api_kind_version_map = {"key1": val1}
    b = _cmeta()
    b.spec.api_kind_version_map = {"key1": val2, "key2": val2}
    b.spec.host = "host"
    want = _cmeta()
    want.spec.storage_classes = ["default"]
    want.spec.api_kind_version_map = {"key1": val2}
    want.spec.host = "host"
    assert a.merge(b)
    assert _cm_state(a) == _cm_state(want)


def test_cluster_merge_storage_classes():
    a = _cmeta()
    a.spec.storage_classes = ["111", "222", "333"]
    b = _cmeta()
    b.spec.storage_classes = ["222", "333", "444"]
    assert a.merge(b)
    assert a.spec.storage_classes == ["222", "333"]


def test_get_supported_versions():
    c = _cmeta()
    assert c.spec.get_supported_versions("foobar_non_existent_key") is None
    c.spec.api_kind_version_map = {"key1": []}
    assert c.spec.get_supported_versions("key1") is None
    c.spec.api_kind_version_map = {"key1": ["0.1.0", "0.1.1", "1.2.3"]}
    assert c.spec.get_supported_versions("key1") == ["0.1.0", "0.1.1", "1.2.3"]


def test_new_cluster_metadata():
    c = _cmeta()
    assert c.kind == "ClusterMetadata"
    assert c.api_version == "move2kube.konveyor.io/v1alpha1"


# -- helm values ---------------------------------------------------------------

def _hv_state(h):
    return (h.registry_url, h.registry_namespace, h.storage_class, h.ingress_host,
            h.global_variables, h.services)


def test_helm_merge_empty():
    a, b = output.HelmValues(), output.HelmValues()
    a.merge(b)
    assert _hv_state(a) == _hv_state(output.HelmValues())


def test_helm_merge_scalars():
    a = output.HelmValues()
    a.registry_namespace, a.registry_url, a.storage_class = "namespace1", "url1", "storagecls1"
    b = output.HelmValues()
    b.registry_namespace, b.registry_url, b.storage_class = "namespace2", "url2", "storagecls2"
    a.merge(b)
    assert (a.registry_namespace, a.registry_url, a.storage_class) == ("namespace2", "url2", "storagecls2")


def test_helm_merge_global_variables():
    a, b = output.HelmValues(), output.HelmValues()
    a.global_variables["key1"] = "val1"
    b.global_variables["key1"] = "val2"
    a.merge(b)
    assert a.global_variables == {"key1": "val2"}


def test_helm_merge_image_tag_tree():
    a, b = output.HelmValues(), output.HelmValues()
    a.services["key1"] = {"name1": "tag1"}
    b.services["key1"] = {"name1": "tag2"}
    b.services["key2"] = {"name1": "tag1"}
    a.merge(b)
    assert a.services == {"key1": {"name1": "tag2"}, "key2": {"name1": "tag1"}}
    # merged sub-maps are copies, not aliases of the source
    b.services["key2"]["name1"] = "changed"
    assert a.services["key2"]["name1"] == "tag1"


# -- version info --------------------------------------------------------------

def test_version_info_same():
    assert info.get_version_info().is_same_version()


@pytest.mark.parametrize("ver", ["0.0.0", "100.0.0", "foobar"])
def test_version_info_different(ver):
    v = info.get_version_info()
    v.version = ver
    assert not v.is_same_version()


# -- plan ------------------------------------------------------------------------

def _k8s_out(url="", ns="", art="", cluster="", ignore=False):
    k = plan.KubernetesOutput()
    k.registry_url, k.registry_namespace, k.artifact_type = url, ns, art
    k.target_cluster_type, k.target_cluster_path = cluster, ""
    k.ignore_unsupported_kinds = ignore
    return k


def _ko_state(k):
    return vars(k).copy()


def test_k8s_output_merge_empty():
    a = _k8s_out()
    a.merge(_k8s_out())
    assert _ko_state(a) == _ko_state(_k8s_out())


@pytest.mark.parametrize("new_kw,want_kw", [
    ({}, {}),
    ({"url": "url1"}, {"url": "url1"}),
    ({"ns": "namespace1"}, {"ns": "namespace1"}),
    ({"cluster": "clus_type1"}, {"cluster": "clus_type1"}),
])
def test_k8s_output_merge_filled(new_kw, want_kw):
    base = dict(url="111", ns="222", art="333", cluster="444", ignore=False)
    a = _k8s_out(**base)
    a.merge(_k8s_out(art="type1", ignore=True, **new_kw))
    want = dict(base, art="type1", ignore=True, **want_kw)
    assert _ko_state(a) == _ko_state(_k8s_out(**want))


def test_add_source_and_build_artifacts():
    s = plan.Service.new("foo", "bar")
    s.add_source_artifact("key1", "val1")
    assert s.source_artifacts["key1"] == ["val1"]
    s.add_source_artifact("key1", "val2")
    assert s.source_artifacts["key1"] == ["val1", "val2"]
    s.add_build_artifact("key1", "val1")
    s.add_build_artifact("key1", "val2")
    assert s.build_artifacts["key1"] == ["val1", "val2"]


def test_add_source_type():
    s0 = plan.Service.new("foo", "bar")
    s0.add_source_type("src1")
    assert s0.source_types == ["src1"]
    s0.add_source_type("src1")
    assert s0.source_types == ["src1"]
    s2 = plan.Service.new("foo", "bar")
    s2.add_source_type("src2")
    s2.add_source_type("src1")
    assert s2.source_types == ["src2", "src1"]


def test_new_service():
    s = plan.Service.new("foo", "bar")
    assert (s.service_name, s.translation_type) == ("foo", "bar")
    assert s.source_types == [] and s.build_artifacts == {} and s.source_artifacts == {}


def _svc(name, tt):
    return plan.Service.new(name, tt)


def test_add_services_to_empty_plan():
    p = plan.Plan()
    svcs = [_svc("111", "111"), _svc("222", "222"), _svc("333", "333")]
    p.add_services_to_plan(svcs)
    for s in svcs:
        assert p.services[s.service_name] == [s]


def _filled():
    p = plan.Plan()
    p.services["111"] = [_svc("111", "111")]
    p.services["222"] = [_svc("222", "222")]
    p.services["333"] = [_svc("333", "333"), _svc("333", "444")]
    return p


def test_merge_all_services_into_filled_plan():
    p = _filled()
    p.add_services_to_plan([_svc("111", "111"), _svc("222", "222"), _svc("333", "333"), _svc("333", "444")])
    assert p == _filled()


def test_merge_some_and_add_some():
    p = _filled()
    s1 = _svc("444", "444")
    s1.build_artifacts[plan.SOURCE_DIRECTORY_BUILD_ARTIFACT] = ["src1"]
    s2 = _svc("444", "444")
    s2.build_artifacts[plan.SOURCE_DIRECTORY_BUILD_ARTIFACT] = ["src2"]
    p.add_services_to_plan([_svc("111", "111"), _svc("222", "222"), _svc("333", "333"), s1, s2])
    want = _filled()
    want.services["444"] = [s1, s2]
    assert p == want


@pytest.mark.parametrize("field,val", [
    ("target_options", ["opt1"]),
    ("source_types", ["type1"]),
])
def test_merge_is_idempotent(field, val):
    p = plan.Plan()
    p.services["111"] = [_svc("111", "111")]
    s = _svc("111", "111")
    setattr(s, field, list(val))
    p.add_services_to_plan([s])
    p.add_services_to_plan([s])
    want = plan.Plan()
    w = _svc("111", "111")
    setattr(w, field, list(val))
    want.services["111"] = [w]
    assert p == want
