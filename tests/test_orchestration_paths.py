"""The error and fallback paths of the orchestration (``move2kube.py``;
reference ``internal/move2kube/planner.go``, ``translator.go``): a planner,
translator, metadata loader or writer that fails is logged with the
reference's text and the run goes on, a ``Fatalf`` stops it, and the old
output tree is removed even when the fast path cannot be taken.  The happy
paths are the expected trees (``tests/test_reference_configs.py``)."""

import os
import shutil

import pytest

import logparse
from move2kube_amd import api, metadata, move2kube, transformer
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source import translator as source_translator
from move2kube_amd.utils import log

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def golang(tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = tmp_path / "golang"
    shutil.copytree(os.path.join(ROOT, "samples", "golang"), str(src))
    log.set_verbose(False)
    return str(src)


class _Broken:
    def __init__(self, exc):
        self.exc = exc

    def __repr__(self):
        return "*source.Broken"

    def get_service_options(self, path, p):
        raise self.exc

    def update_plan(self, path, p):
        raise self.exc

    def load_to_ir(self, p, ir):
        raise self.exc


def test_a_failing_planner_and_metadata_loader_are_skipped(golang, monkeypatch, capsys):
    real = source_translator.get_source_loaders
    monkeypatch.setattr(source_translator, "get_source_loaders", lambda: [_Broken(ValueError("boom"))] + real())
    real_md = metadata.get_loaders
    monkeypatch.setattr(metadata, "get_loaders", lambda: [_Broken(OSError("md"))] + real_md())
    with api.Session() as s:
        p = s.plan(golang)
    assert p.services   # the other translators planned
    err = capsys.readouterr().err
    assert logparse.logged(err, "[*source.Broken] Failed : boom", "warning")
    assert logparse.logged(err, "[*source.Broken] Failed : md", "warning")


@pytest.mark.parametrize("where", ["planner", "metadata"])
def test_a_fatal_planner_stops_the_plan(golang, monkeypatch, where):
    if where == "planner":
        monkeypatch.setattr(source_translator, "get_source_loaders", lambda: [_Broken(log.FatalError("stop"))])
    else:
        monkeypatch.setattr(metadata, "get_loaders", lambda: [_Broken(log.FatalError("stop"))])
    with api.Session() as s:
        with pytest.raises(log.FatalError, match="stop"):
            s.plan(golang)


def test_metadata_loading_failure_into_the_ir_is_a_warning(golang, tmp_path, monkeypatch, capsys):
    with api.Session() as s:
        p = s.plan(golang)
        monkeypatch.setattr(metadata, "get_loaders", lambda: [_Broken(ValueError("ir"))])
        out = s.translate(golang, str(tmp_path / "out"), plan=p)
    assert os.path.exists(os.path.join(out, "myproject", "golang-deployment.yaml")) or os.listdir(out)
    assert logparse.logged(capsys.readouterr().err, "[*source.Broken] Failed : ir", "warning")


def test_a_failing_plan_to_ir_translation_is_fatal(golang, tmp_path, monkeypatch, capsys):
    with api.Session() as s:
        p = s.plan(golang)

        def bad(plan):
            raise ValueError("no ir")
        monkeypatch.setattr(source_translator, "translate", bad)
        with pytest.raises(log.FatalError):
            s.translate(golang, str(tmp_path / "out"), plan=p)
    assert logparse.logged(capsys.readouterr().err,
                           "Failed to translate the plan to intermediate representation. Error: \"no ir\"", "fatal")


def test_curate_without_a_containerization_mode_is_fatal(golang, monkeypatch):
    with api.Session() as s:
        p = s.plan(golang)
        real = move2kube._ask

        def ask(prob):
            if prob.desc.startswith("Select all containerization modes"):
                prob.set_answer([])
                return prob
            return real(prob)
        monkeypatch.setattr(move2kube, "_ask", ask)
        with pytest.raises(log.FatalError, match="No containerization technique was selected"):
            move2kube.curate_plan(p)


def test_curate_ignores_a_service_without_a_selected_mode(golang, monkeypatch, capsys):
    with api.Session() as s:
        p = s.plan(golang)
        for opts in p.services.values():
            for so in opts:
                so.container_build_type = "ReuseDockerfile"
        other = plantypes.Service("other")
        other.container_build_type = "Manual"
        p.services["other"] = [other]
        real = move2kube._ask

        def ask(prob):
            if prob.desc.startswith("Select all containerization modes"):
                prob.set_answer(["Manual"])
                return prob
            return real(prob)
        monkeypatch.setattr(move2kube, "_ask", ask)
        p = move2kube.curate_plan(p)
    assert sorted(p.services) == ["other"]
    assert logparse.logged(capsys.readouterr().err, "Ignoring service golang, since it does not support any "
                                                    "selected containerization technique.", "warning")


def test_curate_asks_for_the_mode_and_keeps_paths_absolute(golang):
    """Two target options of a converted build type: the mode question lists
    them relative to the root and the answer goes back absolute
    (planner.go:147-175)."""
    with api.Session() as s:
        p = s.plan(golang)
        so = p.services["golang"][0]
        so.container_build_type = plantypes.NEW_DOCKERFILE
        so.target_options = [os.path.join(golang, "b"), os.path.join(golang, "a")]
        p = move2kube.curate_plan(p)
    assert p.services["golang"][0].target_options == [os.path.join(golang, "b")]


def test_curate_logs_paths_it_cannot_relativise(golang, monkeypatch, capsys):
    with api.Session() as s:
        p = s.plan(golang)
        so = p.services["golang"][0]
        so.container_build_type = plantypes.NEW_DOCKERFILE
        so.target_options = ["x", "y"]

        def no_rel(path):
            raise ValueError("cannot rel " + path)

        def no_abs(path):
            raise ValueError("cannot abs " + path)
        monkeypatch.setattr(p, "get_relative_path", no_rel)
        monkeypatch.setattr(p, "get_absolute_path", no_abs)
        p = move2kube.curate_plan(p)
    # no option left to offer: ``options[0]`` panics in the reference
    # (planner.go:169); here the service keeps its options and no question is asked
    assert p.services["golang"][0].target_options == ["x", "y"]
    err = capsys.readouterr().err
    assert logparse.logged(err, "Failed to make the option path \"x\" relative to the root directory. "
                                "Error: \"cannot rel x\"", "error")


def test_stale_trash_of_dead_runs_is_removed(tmp_path):
    parent = tmp_path
    dead = parent / ".out.m2k-old-999999999-1"
    alive = parent / (".out.m2k-old-%d-1" % os.getpid())
    odd = parent / ".out.m2k-old-x-1"
    for d in (dead, alive, odd):
        (d / "sub").mkdir(parents=True)
    move2kube._remove_stale_trash(str(parent), "out")
    assert not dead.exists() and alive.exists() and odd.exists()
    move2kube._remove_stale_trash(str(parent / "missing"), "out")   # unreadable parent: nothing to do


def test_output_removal_falls_back_to_a_synchronous_delete(tmp_path, monkeypatch):
    out = tmp_path / "out"
    (out / "a").mkdir(parents=True)

    def no_rename(a, b):
        raise OSError(18, "Invalid cross-device link")
    monkeypatch.setattr(move2kube.os, "rename", no_rename)
    assert move2kube._remove_output(str(out)) is None
    assert not out.exists()


def test_a_failed_removal_is_logged_and_the_run_goes_on(golang, tmp_path, monkeypatch, capsys):
    outdir = tmp_path / "out"
    with api.Session() as s:
        s.translate(golang, str(outdir))

        def cannot(path):
            raise PermissionError(13, "Permission denied", path)
        monkeypatch.setattr(move2kube, "_remove_output", cannot)
        out = s.translate(golang, str(outdir))
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, "Failed to remove the existing file/directory at the output path", "error")
    assert logparse.logged(err, "Anything in the output path will get overwritten.", "error")
    assert os.path.isdir(out)


def test_errors_of_the_background_removal_are_warnings(golang, tmp_path, monkeypatch, capsys):
    import threading
    outdir = tmp_path / "out"
    with api.Session() as s:
        s.translate(golang, str(outdir))
        t = threading.Thread(target=lambda: None)
        t.start()
        monkeypatch.setattr(move2kube, "_remove_output", lambda path: (t, [OSError("late")]))
        s.translate(golang, str(outdir))
    assert logparse.logged(capsys.readouterr().err, "Failed to remove the previous output: late", "warning")


def _fail(exc):
    def f(self, *a, **k):
        raise exc
    return f


@pytest.mark.parametrize("cls,meth,level,text", [
    (transformer.ComposeTransformer, "transform", "error", "Error during translate docker compose file : c"),
    (transformer.ComposeTransformer, "write_objects", "error", "Unable to write docker compose objects : c"),
    (transformer.K8sTransformer, "transform", "fatal", "Error during translate. Error: \"c\""),
    (transformer.K8sTransformer, "write_objects", "fatal", "Unable to write objects Error: \"c\""),
])
def test_transformer_failures(golang, tmp_path, monkeypatch, capsys, cls, meth, level, text):
    monkeypatch.setattr(cls, meth, _fail(ValueError("c")))
    with api.Session() as s:
        if level == "fatal":
            with pytest.raises(log.FatalError):
                s.translate(golang, str(tmp_path / "out"))
        else:
            s.translate(golang, str(tmp_path / "out"))
    assert logparse.logged(capsys.readouterr().err, text, level)


@pytest.mark.parametrize("cls,meth", [(transformer.ComposeTransformer, "transform"),
                                      (transformer.ComposeTransformer, "write_objects"),
                                      (transformer.CICDTransformer, "transform"),
                                      (transformer.CICDTransformer, "write_objects")])
def test_fatal_errors_of_transformers_propagate(golang, tmp_path, monkeypatch, cls, meth):
    monkeypatch.setattr(cls, meth, _fail(log.FatalError("f")))
    with api.Session() as s:
        with pytest.raises(log.FatalError, match="f"):
            s.translate(golang, str(tmp_path / "out"))


@pytest.mark.parametrize("meth,text", [
    ("transform", "Error while genrationg CI/CD resource fomr the IR. Error: \"c\""),
    ("write_objects", "Unable to write the CI/CD artifacts to files. Error: \"c\""),
])
def test_cicd_failures_are_errors(golang, tmp_path, monkeypatch, capsys, meth, text):
    monkeypatch.setattr(transformer.CICDTransformer, meth, _fail(ValueError("c")))
    with api.Session() as s:
        out = s.translate(golang, str(tmp_path / "out"))
    assert logparse.logged(capsys.readouterr().err, text, "error")
    assert os.path.exists(os.path.join(out, "myproject")) or os.listdir(out)


def test_long_version():
    """``version -l``: the VersionInfo YAML; empty fields (no git stamp in a
    source tree) are left out as ``omitempty`` does."""
    import platform
    assert move2kube.get_version(long=True) == "version: v0.1.0\ngoVersion: python%s\n" % platform.python_version()


@pytest.mark.parametrize("file_version,same,warning", [
    ("v0.1.0", True, None),
    ("0.1", True, None),
    ("v0.2.0", False, "The file version (v0.2.0) is newer than the binary version (v0.1.0)."),
    ("v0.0.9", False, "The file version (v0.0.9) is older than the binary version (v0.1.0)."),
    ("v0.1.0-alpha.1", False, "The file version (v0.1.0-alpha.1) is older than the binary version (v0.1.0)."),
    ("bad", False, "Unable to load current version : Invalid Semantic Version"),
])
def test_version_compatibility(capsys, file_version, same, warning):
    """``VersionInfo.IsSameVersion`` with Masterminds/semver ordering."""
    from move2kube_amd.models import info
    log.set_verbose(False)
    assert info.VersionInfo(version=file_version).is_same_version() is same
    err = capsys.readouterr().err
    if warning:
        assert logparse.logged(err, warning, "warning")


@pytest.mark.parametrize("a,b,want", [
    ("v1.0.0-alpha", "v1.0.0-alpha.1", -1), ("v1.0.0-alpha.1", "v1.0.0-alpha.beta", -1),
    ("v1.0.0-beta.2", "v1.0.0-beta.11", -1), ("v1.0.0-rc.1", "v1.0.0", -1), ("v1.0.0-1", "v1.0.0-a", -1),
    ("v1.0.0-a", "v1.0.0-1", 1), ("v1.0.0", "v1.0.0-rc.1", 1), ("v1.0.0-x.1", "v1.0.0-x.1", 0),
])
def test_semver_precedence(a, b, want):
    from move2kube_amd.models import info
    assert info._compare(info._parse_semver(a), info._parse_semver(b)) == want
