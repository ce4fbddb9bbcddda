"""Metadata loaders off the happy path (reference ``internal/metadata/``):
target-cluster selection errors (``clustermdloader.go:64-98``), cluster
metadata files that are not ClusterMetadata (:121-133), built-in profiles
without storage classes, and Kubernetes files that vanish or change between
plan and translate (``k8sfilesloader.go:62-79``)."""

import os

import pytest

import logparse
from move2kube_amd import metadata
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import log
from move2kube_amd.utils.constants import settings

CM_YAML = """apiVersion: move2kube.konveyor.io/v1alpha1
kind: ClusterMetadata
metadata:
  name: %s
spec:
  storageClasses: %s
  apiKindVersionMap:
    Deployment: [apps/v1]
"""


@pytest.fixture(autouse=True)
def _quiet():
    log.set_verbose(False)


def _ir():
    return irtypes.IR()


@pytest.mark.parametrize("ttype,tpath,err", [
    ("", "", None),
    ("Kubernetes", "/x/c.yaml", "Only one of type or path should be specified for the target cluster. "
                                "Target cluster: {Kubernetes /x/c.yaml}"),
    ("NoSuchProfile", "", "The requested target cluster {NoSuchProfile } was not found"),
])
def test_target_cluster_selection(capsys, ttype, tpath, err):
    p = plantypes.new_plan()
    p.kubernetes.target_cluster_type = ttype
    p.kubernetes.target_cluster_path = tpath
    ir = _ir()
    if err is None:
        metadata.ClusterMDLoader().load_to_ir(p, ir)
        assert ir.target_cluster_spec.get_supported_versions("Deployment")
        assert logparse.logged(capsys.readouterr().err, "Neither type nor path is specified for the target cluster. "
                                                        "Going with the default cluster type: Kubernetes", "warning")
    else:
        with pytest.raises(ValueError) as ei:
            metadata.ClusterMDLoader().load_to_ir(p, ir)
        assert str(ei.value) == err


def test_a_path_target_is_found_only_in_fixed_mode(tmp_path, monkeypatch):
    """The reference keys clusters by name, so a path target is never found
    (SURVEY 2.13); M2K_COMPAT=fixed reads the file."""
    f = tmp_path / "mine.yaml"
    f.write_text(CM_YAML % ("mine", "[fast]"))
    p = plantypes.new_plan()
    p.kubernetes.target_cluster_type = ""
    p.kubernetes.target_cluster_path = str(f)
    with pytest.raises(ValueError, match="was not found"):
        metadata.ClusterMDLoader().load_to_ir(p, _ir())
    monkeypatch.setattr(settings, "compat", "fixed")
    ir = _ir()
    metadata.ClusterMDLoader().load_to_ir(p, ir)
    assert ir.target_cluster_spec.storage_classes == ["fast"]
    p.kubernetes.target_cluster_path = str(tmp_path / "missing.yaml")
    with pytest.raises(ValueError, match="was not found"):
        metadata.ClusterMDLoader().load_to_ir(p, _ir())


def test_collected_cluster_metadata_files(tmp_path, capsys):
    (tmp_path / "good.yaml").write_text(CM_YAML % ("custom", "[]"))
    (tmp_path / "other.yaml").write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\n")
    p = plantypes.new_plan()
    metadata.ClusterMDLoader().update_plan(str(tmp_path), p)
    assert p.target_info_artifacts[plantypes.K8S_CLUSTER_ARTIFACT] == [str(tmp_path / "good.yaml")]
    assert p.kubernetes.target_cluster_type == "custom" and p.kubernetes.ignore_unsupported_kinds
    # a listed file that is no longer ClusterMetadata is an error when the
    # clusters are gathered; an empty storage class list gets "default"
    p.target_info_artifacts[plantypes.K8S_CLUSTER_ARTIFACT].append(str(tmp_path / "other.yaml"))
    clusters = metadata.ClusterMDLoader.get_clusters(p)
    assert clusters["custom"].spec.storage_classes == ["default"]
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, 'Failed to load the cluster metadata at path "%s"' % (tmp_path / "other.yaml"),
                                      "error")
    assert "is not a valid cluster metadata. Expected kind: ClusterMetadata Actual kind: QACache" in err


def test_builtin_profile_without_storage_classes_gets_default(monkeypatch):
    from move2kube_amd import assets
    monkeypatch.setattr(assets, "builtin_clusters", lambda: {"Bare": {"storageClasses": [], "apiKindVersionMap": {}}})
    clusters = metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())
    assert clusters["Bare"].spec.storage_classes == ["default"]


def test_k8s_files_that_change_between_plan_and_translate(tmp_path, capsys):
    good = tmp_path / "svc.yaml"
    good.write_text("apiVersion: v1\nkind: Service\nmetadata:\n  name: s\n")
    gone = tmp_path / "gone.yaml"
    gone.write_text("apiVersion: v1\nkind: Service\nmetadata:\n  name: g\n")
    bad = tmp_path / "bad.yaml"
    bad.write_text("apiVersion: v1\nkind: Service\nmetadata:\n  name: b\n")
    p = plantypes.new_plan()
    metadata.K8sFilesLoader().update_plan(str(tmp_path), p)
    assert sorted(os.path.basename(f) for f in p.k8s_files) == ["bad.yaml", "gone.yaml", "svc.yaml"]
    os.remove(str(gone))
    bad.write_text("kind: [\n")
    ir = _ir()
    metadata.K8sFilesLoader().load_to_ir(p, ir)
    assert [o["metadata"]["name"] for o in ir.cached_objects] == ["s"]
    err = capsys.readouterr().err
    assert logparse.logged(err, 'Failed to read the k8s file at path "%s" Error: "open %s: no such file or directory"'
                           % (gone, gone), "error")
    assert logparse.logged_containing(err, 'Failed to decode the file at path "%s" as a k8s file.' % bad, "error")


@pytest.mark.parametrize("loader", [metadata.ClusterMDLoader, metadata.K8sFilesLoader, metadata.QACacheLoader])
def test_a_missing_source_directory_fails_the_loader(tmp_path, loader):
    with pytest.raises((OSError, ValueError)):
        loader().update_plan(str(tmp_path / "missing"), plantypes.new_plan())


def test_loader_base_is_abstract():
    base = metadata.Loader()
    with pytest.raises(NotImplementedError):
        base.update_plan("", None)
    with pytest.raises(NotImplementedError):
        base.load_to_ir(None, None)
    assert repr(metadata.K8sFilesLoader()) == "*metadata.K8sFilesLoader"
