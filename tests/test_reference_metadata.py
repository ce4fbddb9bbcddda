"""Metadata loader parity (``internal/metadata/*_test.go`` fixtures)."""

import os
import shutil

import pytest

from conftest import ref_path
from move2kube_amd import metadata
from move2kube_amd.models import collection
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import common, yamlio

pytestmark = pytest.mark.reference

MD = ref_path("internal", "metadata")


@pytest.fixture
def md_cwd(tmp_path, monkeypatch):
    """cwd with a copy of the fixtures, so relative fixture paths match the reference's."""
    shutil.copytree(os.path.join(MD, "testdata"), str(tmp_path / "testdata"))
    monkeypatch.chdir(tmp_path)
    return tmp_path


def _dump(p):
    return yamlio.dump(p.to_yaml())


def test_update_plan_no_files(tmp_path):
    p, want = plantypes.new_plan(), plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan(str(tmp_path), p)
    assert _dump(p) == _dump(want)


@pytest.mark.parametrize("d", ["emptyfiles", "invalidfiles"])
def test_update_plan_ignores_bad_files(md_cwd, d):
    p, want = plantypes.new_plan(), plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan("testdata/" + d, p)
    assert _dump(p) == _dump(want)


def test_update_plan_valid_files(md_cwd):
    p = plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan("testdata/validfiles", p)
    assert p.target_info_artifacts[plantypes.K8S_CLUSTER_ARTIFACT] == ["testdata/validfiles/test1.yaml",
                                                                        "testdata/validfiles/test2.yml"]
    assert p.kubernetes.target_cluster_type == "name1"
    assert p.kubernetes.ignore_unsupported_kinds is True


def test_builtin_profiles_match_reference_yamls():
    clusters = metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())
    names = []
    for f in common.get_files_by_ext(os.path.join(MD, "clusters"), [".yml", ".yaml"]):
        cm = collection.ClusterMetadata.from_yaml(common.read_move2kube_yaml(f))
        names.append(cm.name)
        got = clusters[cm.name]
        assert got.spec.storage_classes == (cm.spec.storage_classes or ["default"])
        assert got.spec.api_kind_version_map == cm.spec.api_kind_version_map, cm.name
    assert sorted(names) == sorted(clusters)


def test_load_to_ir_with_empty_plan():
    p = plantypes.new_plan()
    ir = irtypes.new_ir(p)
    metadata.ClusterMDLoader().load_to_ir(p, ir)
    assert ir.target_cluster_spec.storage_classes


@pytest.mark.parametrize("d", ["validfiles", "validfilesnostorageclasses"])
def test_get_clusters_from_filled_plan(md_cwd, d):
    p = plantypes.new_plan()
    p.target_info_artifacts[plantypes.K8S_CLUSTER_ARTIFACT] = ["testdata/%s/test1.yaml" % d, "testdata/%s/test2.yml" % d]
    cm = metadata.ClusterMDLoader.get_clusters(p)
    for k in ("IBM-IKS", "IBM-Openshift", "AWS-EKS", "Kubernetes", "Openshift", "name1"):
        assert k in cm
    for k, v in cm.items():
        assert v.kind == collection.CLUSTER_METADATA_KIND and k == v.name and v.spec.storage_classes


@pytest.mark.parametrize("d,want", [("valid", ["testdata/k8s/valid/valid.yaml"]), ("invalid", []), ("nonyaml", []),
                                    ("valid_invalid", ["testdata/k8s/valid_invalid/valid.yaml"])])
def test_k8s_files_loader(md_cwd, d, want):
    p = plantypes.new_plan()
    metadata.K8sFilesLoader().update_plan("testdata/k8s/" + d, p)
    assert p.k8s_files == want


def test_k8s_files_load_to_ir(md_cwd):
    p = plantypes.new_plan()
    p.k8s_files = ["testdata/k8s/valid/valid.yaml"]
    ir = irtypes.new_ir(p)
    metadata.K8sFilesLoader().load_to_ir(p, ir)
    assert len(ir.cached_objects) == 1


@pytest.mark.parametrize("d,want", [("valid", ["testdata/qa/valid/valid.yaml"]), ("invalid", []), ("nonyaml", []),
                                    ("valid_invalid", ["testdata/qa/valid_invalid/valid.yaml"])])
def test_qa_cache_loader(md_cwd, d, want):
    p = plantypes.new_plan()
    metadata.QACacheLoader().update_plan("testdata/qa/" + d, p)
    assert p.qa_caches == want


def test_qa_cache_loader_unreadable_file(md_cwd, unprivileged):
    """``TestBadPerm`` (qacaches_test.go:77-89): a directory with mode 0 is an
    error and the plan stays empty; a QA cache file with mode 0 inside a
    readable directory is skipped."""
    d = os.path.join(unprivileged.tmp, "badperm")
    os.mkdir(d)
    shutil.copy("testdata/qa/valid/valid.yaml", os.path.join(d, "valid.yml"))
    f = os.path.join(unprivileged.tmp, "badfile")
    os.mkdir(f)
    shutil.copy("testdata/qa/valid/valid.yaml", os.path.join(f, "valid.yaml"))
    unprivileged.chown()
    os.chmod(d, 0)
    os.chmod(os.path.join(f, "valid.yaml"), 0)

    def check():
        p = plantypes.new_plan()
        with pytest.raises(OSError):
            metadata.QACacheLoader().update_plan(d, p)
        assert p.qa_caches == []
        metadata.QACacheLoader().update_plan(f, p)
        assert p.qa_caches == []
    unprivileged.run(check)


def test_qa_cache_load_to_ir_registers_engine(md_cwd):
    from move2kube_amd import qaengine
    p = plantypes.new_plan()
    p.qa_caches = ["testdata/qa/valid/valid.yaml"]
    metadata.QACacheLoader().load_to_ir(p, irtypes.new_ir(p))
    assert [type(e).__name__ for e in qaengine.engines()] == ["CacheEngine"]
