"""The Helm chart writer off the happy path (reference
``internal/transformer/k8stransformer.go:156-247``): each step of
``generateHelmMetadata`` that cannot write is logged and the rest still
written, and ``operator-sdk`` that is missing, fails or cannot start is a
warning (the chart stays)."""

import os

import pytest

import logparse
from move2kube_amd import transformer
from move2kube_amd.models import output
from move2kube_amd.utils import log


@pytest.fixture(autouse=True)
def _quiet():
    log.set_verbose(True)
    yield
    log.set_verbose(False)


def _t():
    t = transformer.K8sTransformer()
    t.values = output.HelmValues()
    t.exposed_service_paths = {"web": "/web"}
    return t


def test_every_helm_metadata_step_that_fails_is_logged(tmp_path, capsys):
    chart = tmp_path / "proj"
    chart.mkdir()
    (chart / "README.md").mkdir()          # each target path taken by something that cannot be written
    (chart / "Chart.yaml").mkdir()
    (chart / "templates").write_text("a file where the directory goes")
    (chart / "values.yaml").mkdir()
    _t().generate_helm_metadata(str(chart))
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, "Error while writing Readme : ", "error")
    assert logparse.logged_containing(err, "Error while writing Chart.yaml : ", "error")
    assert logparse.logged_containing(err, "Unable to create templates directory : ", "error")
    assert logparse.logged_containing(err, "Error while writing Helm NOTES.txt : ", "error")
    assert logparse.logged_containing(err, "Error in writing Helm values", "warning")
    assert "helm upgrade -i proj proj" in (tmp_path / "helminstall.sh").read_text()   # the last step still ran


def test_helm_metadata_directory_that_cannot_be_made(tmp_path, capsys):
    (tmp_path / "proj").write_text("a file")
    with pytest.raises(OSError):
        _t().generate_helm_metadata(str(tmp_path / "proj"))
    assert logparse.logged_containing(capsys.readouterr().err, "Unable to create Helm Metadata directory", "error")


def _sdk(tmp_path, monkeypatch, body):
    b = tmp_path / "bin"
    b.mkdir(exist_ok=True)
    if body is not None:
        s = b / "operator-sdk"
        s.write_text("#!/bin/sh\n" + body)
        s.chmod(0o755)
    monkeypatch.setenv("PATH", str(b) + os.pathsep + "/usr/bin:/bin")


def test_operator_sdk_missing(tmp_path, monkeypatch, capsys):
    _sdk(tmp_path, monkeypatch, None)
    assert transformer.K8sTransformer.create_operator("proj", str(tmp_path)) is False
    assert logparse.logged(capsys.readouterr().err, 'Unable to find operator-sdk. Skipping operator generation : '
                           'exec: "operator-sdk": executable file not found in $PATH', "warning")


def test_operator_sdk_failure_is_a_warning_with_its_output(tmp_path, monkeypatch, capsys):
    _sdk(tmp_path, monkeypatch, "echo 'FATA[0000] no chart'\nexit 1\n")
    (tmp_path / "proj").mkdir()
    assert transformer.K8sTransformer.create_operator("proj", str(tmp_path)) is False
    assert logparse.logged(capsys.readouterr().err, "Error during operator creation : exit status 1, "
                           "FATA[0000] no chart\n", "warning")


def test_operator_sdk_success_replaces_an_old_operator(tmp_path, monkeypatch):
    _sdk(tmp_path, monkeypatch, "echo ok > PROJECT\n")
    old = tmp_path / "proj-operator"
    old.mkdir()
    (old / "stale").write_text("x")
    assert transformer.K8sTransformer.create_operator("proj", str(tmp_path)) is True
    assert sorted(os.listdir(str(old))) == ["PROJECT"]


def test_operator_sdk_that_cannot_start(tmp_path, monkeypatch, capsys):
    _sdk(tmp_path, monkeypatch, "")
    (tmp_path / "bin" / "operator-sdk").write_bytes(b"\x7fELF not really")   # exec format error
    assert transformer.K8sTransformer.create_operator("proj", str(tmp_path)) is False
    assert logparse.logged(capsys.readouterr().err, "Error during operator creation : fork/exec %s: exec format "
                           "error, " % (tmp_path / "bin" / "operator-sdk"), "warning")


def test_operator_directory_that_cannot_be_made(tmp_path, monkeypatch, capsys):
    _sdk(tmp_path, monkeypatch, "exit 0\n")
    (tmp_path / "proj-operator").mkdir()
    monkeypatch.setattr(transformer, "_mkdir", lambda p: (_ for _ in ()).throw(PermissionError(13, "x", p)))
    assert transformer.K8sTransformer.create_operator("proj", str(tmp_path)) is False
    assert logparse.logged(capsys.readouterr().err, "Unable to create Operator directory %s : mkdir %s: permission "
                           "denied" % (tmp_path / "proj-operator", tmp_path / "proj-operator"), "error")


def _convert(objs, kinds, ignore=False):
    from move2kube_amd.models.collection import ClusterMetadataSpec
    t = transformer.K8sTransformer()
    t.transformed_objects = objs
    t.target_cluster_spec = ClusterMetadataSpec([], kinds)
    t.ignore_unsupported_kinds = ignore
    return t.convert_objects()


def test_a_kind_the_cluster_lacks_is_written_as_it_is_with_the_references_error(capsys):
    """k8stransformer.go:109-138: the version stays GroupVersionKind().String(),
    ParseGroupVersion reads "v1, Kind=..." as the version, and the conversion
    fails with Scheme.New's not-registered error."""
    log.set_verbose(False)
    dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"}}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "s"}}
    assert _convert([dep, svc], {"Pod": ["v1"]}) == [dep, svc]
    err = capsys.readouterr().err
    scheme = "github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46"
    assert logparse.logged(err, 'Error while transforming version : no kind "Deployment" is registered for version '
                                '"apps/v1, Kind=Deployment" in scheme "%s". Writing in original version.' % scheme,
                           "error")
    assert logparse.logged(err, 'Error while transforming version : no kind "Service" is registered for version '
                                '"v1, Kind=Service" in scheme "%s". Writing in original version.' % scheme, "error")


def test_unsupported_kinds_ignored_and_bad_versions_dropped(capsys):
    dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"}}
    assert _convert([dep], {"Pod": ["v1"]}, ignore=True) == []
    assert _convert([dep], {"Deployment": ["a/b/c"]}) == []
    err = capsys.readouterr().err
    assert logparse.logged(err, "Kind Deployment unsupported in target cluster. Will ignore object. "
                                "&TypeMeta{Kind:Deployment,APIVersion:apps/v1,}", "error")
    assert logparse.logged(err, "Unable to parse group version a/b/c : unexpected GroupVersion string: a/b/c",
                           "error")


def test_container_files_that_cannot_be_written(tmp_path, capsys):
    """transformer.go:60-99: a directory that cannot be made skips its file
    with an error line; a file that cannot be written is a warning; the
    scripts are still written."""
    from move2kube_amd.models import ir as irtypes
    c = irtypes.new_container("NewDockerfile", "web:1", True)
    c.add_file("blocked/Dockerfile", "FROM x\n")
    c.add_file("web/web-docker-build.sh", "docker build .\n")
    c.add_file("web/taken", "x")
    out = tmp_path / "out"
    (out / "containers" / "web" / "taken").mkdir(parents=True)      # the file's path is a directory
    (out / "containers" / "blocked").write_text("a file where a directory goes")
    log.set_verbose(False)
    assert transformer.write_containers([c], str(out), str(tmp_path), "quay.io", "ns") is True
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, "Unable to create directory %s : mkdir %s: " % (
        out / "containers" / "blocked", out / "containers" / "blocked"), "error")
    assert logparse.logged(err, "Error writing file at %s : open %s: is a directory" % (
        out / "containers" / "web" / "taken", out / "containers" / "web" / "taken"), "warning")
    assert (out / "containers" / "web" / "web-docker-build.sh").read_text() == "docker build .\n"
    assert (out / "buildimages.sh").exists() and (out / "pushimages.sh").exists() and (out / "copysources.sh").exists()
