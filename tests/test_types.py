"""The model types' own tests, one pytest per Go subtest (``types/*_test.go``),
each comparing whole values where Go compares whole values
(``reflect.DeepEqual`` / ``cmp.Equal`` / ``!=`` on structs; ``tests/goequal.py``):

* ``types/plan/plan_test.go`` - KubernetesOutput.Merge, Service.Add*,
  Plan.AddServicesToPlan, NewPlan, NewService
* ``types/collection/cluster_test.go`` - ClusterMetadata.Merge,
  GetSupportedVersions, NewClusterMetadata
* ``types/output/helmvaluesoutput_test.go`` - HelmValues.Merge
* ``types/info/versioninfo_test.go`` - GetVersionInfo, IsSameVersion

(``types/collection/{image,cfcontainerizers,cfinstanceapps}_test.go`` and
``types/qaengine/cache_test.go`` are in ``test_reference_common_io.py``.)"""

import pytest

from goequal import assert_deep_equal
from move2kube_amd.models import collection, info, output, plan
from move2kube_amd.utils import constants


# -- types/plan/plan_test.go: TestMerge ---------------------------------------------

def _k8s_out(url="", ns="", art="", cluster="", ignore=False):
    """``plan.KubernetesOutput{RegistryURL, RegistryNamespace, ArtifactType,
    TargetCluster{Type}, IgnoreUnsupportedKinds}``; ``{}`` is all zero."""
    k = plan.KubernetesOutput()
    k.registry_url, k.registry_namespace, k.artifact_type = url, ns, art
    k.target_cluster_type, k.target_cluster_path = cluster, ""
    k.ignore_unsupported_kinds = ignore
    return k


_FILLED = dict(url="111", ns="222", art="333", cluster="444", ignore=False)


def test_plan_merge_new_empty_k8s_output_into_empty_k8s_output():
    out1 = _k8s_out()
    out1.merge(_k8s_out())
    assert_deep_equal(out1, _k8s_out())


@pytest.mark.parametrize("new_kw,want_kw", [
    pytest.param({}, {}, id="merge artifact type and ignore supported kinds from new k8s output into filled k8s output"),
    pytest.param({"url": "url1"}, {"url": "url1"}, id="merge registry url from new k8s output into filled k8s output"),
    pytest.param({"ns": "namespace1"}, {"ns": "namespace1"},
                 id="merge registry namespace from new k8s output into filled k8s output"),
    pytest.param({}, {}, id="merge image pull secret from new k8s output into filled k8s output"),
    pytest.param({"cluster": "clus_type1"}, {"cluster": "clus_type1"},
                 id="merge cluster type from new k8s output into filled k8s output"),
])
def test_plan_merge_into_filled_k8s_output(new_kw, want_kw):
    out1 = _k8s_out(**_FILLED)
    out1.merge(_k8s_out(art="type1", ignore=True, **new_kw))
    assert_deep_equal(out1, _k8s_out(**dict(_FILLED, art="type1", ignore=True, **want_kw)))


# -- TestAddSourceArtifact / TestAddBuildArtifact ---------------------------------------

@pytest.mark.parametrize("kind", ["source", "build"])
def test_add_artifact_to_empty_service(kind):
    s = plan.Service.new("foo", "bar")
    getattr(s, "add_%s_artifact" % kind)("key1", "val1")
    assert_deep_equal(getattr(s, "%s_artifacts" % kind), {"key1": ["val1"]})


@pytest.mark.parametrize("kind", ["source", "build"])
def test_add_artifact_to_filled_service(kind):
    s = plan.Service.new("foo", "bar")
    add = getattr(s, "add_%s_artifact" % kind)
    add("key1", "val1")
    add("key1", "val2")
    assert_deep_equal(getattr(s, "%s_artifacts" % kind), {"key1": ["val1", "val2"]})


# -- TestAddSourceType ---------------------------------------------------------------------

def _svc_with(*sources):
    s = plan.Service.new("foo", "bar")
    for src in sources:
        s.add_source_type(src)
    return s


@pytest.mark.parametrize("before,want", [
    pytest.param((), ["src1"], id="add source to empty service"),
    pytest.param(("src1",), ["src1"], id="skip adding source to filled service"),
    pytest.param(("src2",), ["src2", "src1"], id="add source to filled service"),
])
def test_add_source_type(before, want):
    s = _svc_with(*before)
    s.add_source_type("src1")
    assert_deep_equal(s.source_types, want)


# -- TestAddServicesToPlan ----------------------------------------------------------------------

def _svc(name, tt):
    return plan.Service.new(name, tt)


def _filled():
    p = plan.new_plan()
    p.services["111"] = [_svc("111", "111")]
    p.services["222"] = [_svc("222", "222")]
    p.services["333"] = [_svc("333", "333"), _svc("333", "444")]
    return p


def test_add_all_services_to_empty_plan():
    p = plan.new_plan()
    services = [_svc("111", "111"), _svc("222", "222"), _svc("333", "333")]
    p.add_services_to_plan(services)
    for s in services:
        assert_deep_equal(p.services[s.service_name], [s])


def test_merge_all_services_to_filled_plan():
    p = _filled()
    p.add_services_to_plan([_svc("111", "111"), _svc("222", "222"), _svc("333", "333"), _svc("333", "444")])
    assert_deep_equal(p, _filled())


def test_merge_some_services_and_add_some_services_to_filled_plan():
    p = _filled()
    svc1 = _svc("444", "444")
    svc1.build_artifacts[plan.SOURCE_DIRECTORY_BUILD_ARTIFACT] = ["src1"]
    svc2 = _svc("444", "444")
    svc2.build_artifacts[plan.SOURCE_DIRECTORY_BUILD_ARTIFACT] = ["src2"]
    p.add_services_to_plan([_svc("111", "111"), _svc("222", "222"), _svc("333", "333"), svc1, svc2])
    want = _filled()
    want.services[svc1.service_name] = [svc1, svc2]
    assert_deep_equal(p, want)


def _merge_twice(setup):
    p = plan.new_plan()
    p.services["111"] = [_svc("111", "111")]
    svc1 = _svc("111", "111")
    setup(svc1)
    p.add_services_to_plan([svc1])
    p.add_services_to_plan([svc1])
    want = plan.new_plan()
    svc2 = _svc("111", "111")
    setup(svc2)
    want.services["111"] = [svc2]
    assert_deep_equal(p, want)


def test_merge_all_services_having_target_options_to_filled_plan():
    _merge_twice(lambda s: setattr(s, "target_options", ["opt1"]))


def test_merge_all_services_having_source_types_to_filled_plan():
    _merge_twice(lambda s: setattr(s, "source_types", ["type1"]))


def test_merge_all_services_having_build_artifacts_to_filled_plan():
    _merge_twice(lambda s: s.build_artifacts.__setitem__("111", ["art1"]))


def test_merge_all_services_having_source_artifacts_to_filled_plan():
    _merge_twice(lambda s: s.source_artifacts.__setitem__("111", ["art1"]))


# -- TestNewPlan / TestNewService ------------------------------------------------------------------

def test_new_plan():
    p = plan.new_plan()
    assert p.services is not None and p.target_info_artifacts is not None


def test_new_service():
    s = plan.Service.new("foo", "bar")
    assert (s.service_name, s.translation_type) == ("foo", "bar")
    assert s.source_types is not None and s.build_artifacts is not None and s.source_artifacts is not None


# -- types/collection/cluster_test.go ---------------------------------------------------------------

def _cmeta(name="", kind=None):
    c = collection.new_cluster_metadata(name)
    if kind is not None:
        c.kind = kind
    return c


def test_cluster_merging_2_empty_metadatas():
    cmeta1, cmeta2, want = _cmeta(kind=""), _cmeta(kind=""), _cmeta(kind="")
    assert cmeta1.merge(cmeta2)
    assert_deep_equal(cmeta1, want)


def test_cluster_merging_a_non_empty_metadata_into_an_empty_metadata():
    cmeta1 = _cmeta(kind="")
    want = _cmeta("")
    want.name = "ctxname1"
    want.spec.storage_classes = ["default"]
    assert cmeta1.merge(_cmeta("ctxname1"))
    assert_deep_equal(cmeta1, want)


def test_cluster_merging_metadata_with_different_kinds():
    assert not _cmeta(kind="kind1").merge(_cmeta(kind="kind2"))


def test_cluster_merging_version_maps_from_filled_metadata_into_filled_metadata():
    val1 = ["1.0.0", "1.1.0", "1.1.1"]
    val2 = ["2.0.0", "2.2.0", "2.2.2"]
    cmeta1 = _cmeta()
    cmeta1.spec.api_kind_version_map = {"key1": val1}
    cmeta2 = _cmeta()
    cmeta2.spec.api_kind_version_map = {"key1": val2, "key2": val2}
    cmeta2.spec.host = "host"
    want = _cmeta()
    want.spec.storage_classes = ["default"]
    want.spec.api_kind_version_map = {"key1": val2}
    want.spec.host = "host"
    assert cmeta1.merge(cmeta2)
    assert_deep_equal(cmeta1, want)


def test_cluster_merging_storage_classes_from_filled_metadata_into_filled_metadata():
    cmeta1 = _cmeta()
    cmeta1.spec.storage_classes = ["111", "222", "333"]
    cmeta2 = _cmeta()
    cmeta2.spec.storage_classes = ["222", "333", "444"]
    want = _cmeta()
    want.spec.storage_classes = ["222", "333"]
    assert cmeta1.merge(cmeta2)
    assert_deep_equal(cmeta1, want)


def test_get_nil_for_non_existent_key():
    assert _cmeta().spec.get_supported_versions("foobar_non_existent_key") is None


def test_get_nil_for_key_with_empty_list_of_supported_versions():
    c = _cmeta()
    c.spec.api_kind_version_map = {"key1": []}
    assert c.spec.get_supported_versions("key1") is None


def test_get_a_list_of_versions_for_a_valid_key():
    c = _cmeta()
    c.spec.api_kind_version_map = {"key1": ["0.1.0", "0.1.1", "1.2.3"]}
    assert_deep_equal(c.spec.get_supported_versions("key1"), ["0.1.0", "0.1.1", "1.2.3"])


def test_new_cluster_metadata():
    c = _cmeta()
    assert (c.kind, c.api_version) == (collection.CLUSTER_METADATA_KIND, constants.SCHEME_GROUP_VERSION)


# -- types/output/helmvaluesoutput_test.go ----------------------------------------------------------

def test_helm_merge_2_empty_helm_values():
    h1 = output.HelmValues()
    h1.merge(output.HelmValues())
    assert_deep_equal(h1, output.HelmValues())


def _helm(ns, url, sc):
    h = output.HelmValues()
    h.registry_namespace, h.registry_url, h.storage_class = ns, url, sc
    return h


def test_helm_merge_filled_helm_value_into_filled_helm_value():
    h1 = _helm("namespace1", "url1", "storagecls1")
    h1.merge(_helm("namespace2", "url2", "storagecls2"))
    assert_deep_equal(h1, _helm("namespace2", "url2", "storagecls2"))


def test_helm_merge_global_and_service_variables_into_filled_helm_value():
    h1, h2, want = output.HelmValues(), output.HelmValues(), output.HelmValues()
    h1.global_variables["key1"] = "val1"
    h2.global_variables["key1"] = "val2"
    want.global_variables["key1"] = "val2"
    h1.merge(h2)
    assert_deep_equal(h1, want)


def test_helm_merge_image_tag_tree_properly_into_filled_helm_value():
    h1, h2, want = output.HelmValues(), output.HelmValues(), output.HelmValues()
    h1.services["key1"] = {"name1": "tag1"}
    h2.services["key1"] = {"name1": "tag2"}
    h2.services["key2"] = {"name1": "tag1"}
    want.services["key1"] = {"name1": "tag2"}
    want.services["key2"] = {"name1": "tag1"}
    h1.merge(h2)
    assert_deep_equal(h1, want)
    # beyond Go: the merged sub-maps are copies, not aliases of the source
    h2.services["key2"]["name1"] = "changed"
    assert h1.services["key2"]["name1"] == "tag1"


# -- types/info/versioninfo_test.go -------------------------------------------------------------------

def test_get_version_info():
    assert info.get_version_info().is_same_version()


def test_is_same_version_same_version():
    assert info.get_version_info().is_same_version()


@pytest.mark.parametrize("ver", [pytest.param("0.0.0", id="older version"),
                                 pytest.param("100.0.0", id="newer version"),
                                 pytest.param("foobar", id="invalid version")])
def test_is_same_version_different(ver):
    v = info.get_version_info()
    v.version = ver
    assert not v.is_same_version()
