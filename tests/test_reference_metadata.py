"""``internal/metadata/{clustermdloader,k8sfiles,qacaches}_test.go``, one pytest
per Go subtest (testify suite methods included), comparing whole plans where
Go compares whole plans."""

import os
import shutil

import pytest

from conftest import ref_path
from goequal import assert_deep_equal
from move2kube_amd import metadata
from move2kube_amd.models import collection
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import common, constants

pytestmark = pytest.mark.reference

MD = ref_path("internal", "metadata")


@pytest.fixture
def md_cwd(tmp_path, monkeypatch):
    """cwd with a copy of the fixtures, so relative fixture paths match the reference's."""
    shutil.copytree(os.path.join(MD, "testdata"), str(tmp_path / "testdata"))
    monkeypatch.chdir(tmp_path)
    return tmp_path


def _plan_with(**fields):
    """plantypes.NewPlan() with some Spec fields set (the ``want`` plans)."""
    p = plantypes.new_plan()
    for k, v in fields.items():
        if k == "k8s_cluster_artifacts":
            p.target_info_artifacts[plantypes.K8S_CLUSTER_ARTIFACT] = v
        elif k == "target_cluster":
            p.kubernetes.target_cluster_type = v
        elif k == "ignore_unsupported_kinds":
            p.kubernetes.ignore_unsupported_kinds = v
        else:
            setattr(p, k, v)
    return p


# --- clustermdloader_test.go: TestUpdatePlan ------------------------------------------

def test_update_plan_when_there_are_no_files(tmp_path):
    p = plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan(str(tmp_path), p)
    assert_deep_equal(p, plantypes.new_plan())


def test_check_if_all_clusters_in_constant_were_loaded():
    cm_map = metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())
    names = []
    for f in common.get_files_by_ext(os.path.join(MD, "clusters"), [".yml", ".yaml"]):
        cm = collection.ClusterMetadata.from_yaml(common.read_move2kube_yaml(f))
        names.append(cm.name)
    assert sorted(names) == sorted(cm_map)   # both directions of the Go test


def test_builtin_profiles_match_reference_yamls():
    """Beyond the Go test: every built-in profile equals its reference yaml."""
    clusters = metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())
    for f in common.get_files_by_ext(os.path.join(MD, "clusters"), [".yml", ".yaml"]):
        cm = collection.ClusterMetadata.from_yaml(common.read_move2kube_yaml(f))
        got = clusters[cm.name]
        assert got.spec.storage_classes == (cm.spec.storage_classes or ["default"])
        assert got.spec.api_kind_version_map == cm.spec.api_kind_version_map, cm.name


@pytest.mark.parametrize("d", [pytest.param("emptyfiles", id="update plan with some empty files"),
                               pytest.param("invalidfiles", id="update plan with some invalid files")])
def test_update_plan_ignores_bad_files(md_cwd, d):
    p = plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan("testdata/" + d, p)
    assert_deep_equal(p, plantypes.new_plan())


def test_update_plan_with_some_valid_files(md_cwd):
    p = plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan("testdata/validfiles", p)
    want = _plan_with(k8s_cluster_artifacts=["testdata/validfiles/test1.yaml", "testdata/validfiles/test2.yml"],
                      target_cluster="name1", ignore_unsupported_kinds=True)
    assert_deep_equal(p, want)


# --- TestLoadToIR / TestGetClusters -------------------------------------------------------

def test_load_ir_with_an_empty_plan():
    p = plantypes.new_plan()
    ir = irtypes.new_ir(p)
    metadata.ClusterMDLoader().load_to_ir(p, ir)
    assert ir.target_cluster_spec.storage_classes


def test_check_default_cluster_type_is_valid():
    assert constants.DEFAULT_CLUSTER_TYPE in metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())


def _check_clusters(cm_map, file_keys=()):
    for k in ("IBM-IKS", "IBM-Openshift", "AWS-EKS"):
        assert k in cm_map
    for k, v in cm_map.items():
        assert v.kind == collection.CLUSTER_METADATA_KIND
        assert k == v.name or (k in file_keys and v.name == "name1")
        assert v.spec.storage_classes


def test_get_clusters_from_an_empty_plan():
    cm_map = metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())
    for k in (constants.DEFAULT_CLUSTER_TYPE, "Kubernetes", "Openshift"):
        assert k in cm_map
    _check_clusters(cm_map)


@pytest.mark.parametrize("d", [pytest.param("validfiles", id="get clusters from a filled plan"),
                               pytest.param("validfilesnostorageclasses", id="get clusters from a filled plan#01")])
def test_get_clusters_from_a_filled_plan(md_cwd, d):
    files = ["testdata/%s/test1.yaml" % d, "testdata/%s/test2.yml" % d]
    p = plantypes.new_plan()
    p.target_info_artifacts[plantypes.K8S_CLUSTER_ARTIFACT] = files
    cm_map = metadata.ClusterMDLoader.get_clusters(p)
    _check_clusters(cm_map, files)
    assert "name1" in cm_map   # stricter than Go: keyed by context name


# --- k8sfiles_test.go / qacaches_test.go (testify suites) -------------------------------------

_LOADERS = {"k8s": (metadata.K8sFilesLoader, "k8s_files"), "qa": (metadata.QACacheLoader, "qa_caches")}


@pytest.mark.parametrize("kind", [pytest.param("k8s", id="TestK8sFilesLoader"),
                                  pytest.param("qa", id="TestQACachesLoader")])
def test_loader_empty_dir(tmp_path, kind):
    loader, _ = _LOADERS[kind]
    p = plantypes.new_plan()
    loader().update_plan(str(tmp_path), p)
    assert_deep_equal(p, plantypes.new_plan())


@pytest.mark.parametrize("kind", [pytest.param("k8s", id="TestK8sFilesLoader"),
                                  pytest.param("qa", id="TestQACachesLoader")])
def test_loader_bad_perm(md_cwd, unprivileged, kind):
    loader, _ = _LOADERS[kind]
    d = os.path.join(unprivileged.tmp, "badperm")
    os.mkdir(d)
    shutil.copy("testdata/%s/valid/valid.yaml" % kind, os.path.join(d, "valid.yml"))
    unprivileged.chown()
    os.chmod(d, 0)

    def check():
        p = plantypes.new_plan()
        with pytest.raises(OSError):
            loader().update_plan(d, p)
        assert_deep_equal(p, plantypes.new_plan())
    unprivileged.run(check)


@pytest.mark.parametrize("kind,d,want", [
    pytest.param("k8s", "invalid", [], id="TestK8sFilesLoader/TestInvalid"),
    pytest.param("k8s", "nonyaml", [], id="TestK8sFilesLoader/TestNonYaml"),
    pytest.param("k8s", "valid", ["testdata/k8s/valid/valid.yaml"], id="TestK8sFilesLoader/TestValid"),
    pytest.param("k8s", "valid_invalid", ["testdata/k8s/valid_invalid/valid.yaml"],
                 id="TestK8sFilesLoader/TestValidInvalid"),
    pytest.param("qa", "invalid", [], id="TestQACachesLoader/TestInvalid"),
    pytest.param("qa", "nonyaml", [], id="TestQACachesLoader/TestNonYaml"),
    pytest.param("qa", "valid", ["testdata/qa/valid/valid.yaml"], id="TestQACachesLoader/TestValid"),
    pytest.param("qa", "valid_invalid", ["testdata/qa/valid_invalid/valid.yaml"],
                 id="TestQACachesLoader/TestValidInvalid"),
    pytest.param("qa", "valid/valid.yaml", ["testdata/qa/valid/valid.yaml"], id="TestQACachesLoader/TestFile"),
])
def test_loader_update_plan(md_cwd, kind, d, want):
    loader, field = _LOADERS[kind]
    p = plantypes.new_plan()
    loader().update_plan("testdata/%s/%s" % (kind, d), p)
    assert_deep_equal(p, _plan_with(**({field: want} if want else {})))


def test_qa_cache_file_without_read_permission_is_skipped(md_cwd, unprivileged):
    """Beyond the Go suite: a cache file with mode 0 in a readable directory."""
    f = os.path.join(unprivileged.tmp, "badfile")
    os.mkdir(f)
    shutil.copy("testdata/qa/valid/valid.yaml", os.path.join(f, "valid.yaml"))
    unprivileged.chown()
    os.chmod(os.path.join(f, "valid.yaml"), 0)

    def check():
        p = plantypes.new_plan()
        metadata.QACacheLoader().update_plan(f, p)
        assert p.qa_caches == []
    unprivileged.run(check)


def test_k8s_files_load_to_ir(md_cwd):
    p = plantypes.new_plan()
    p.k8s_files = ["testdata/k8s/valid/valid.yaml"]
    ir = irtypes.new_ir(p)
    metadata.K8sFilesLoader().load_to_ir(p, ir)
    assert len(ir.cached_objects) == 1


def test_load_to_ir_for_qa(md_cwd):
    """TestQACachesLoader/TestLoadToIRForQA (and, beyond it, the cache engine it registers)."""
    from move2kube_amd import qaengine
    p = plantypes.new_plan()
    p.qa_caches = ["testdata/qa/valid/valid.yaml"]
    metadata.QACacheLoader().load_to_ir(p, irtypes.new_ir(p))
    assert [type(e).__name__ for e in qaengine.engines()] == ["CacheEngine"]
