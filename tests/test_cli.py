"""CLI verbs and flag semantics, in process (reference ``cmd/move2kube/*.go``):
plan-path resolution (``plan.go:38-80``), translate with and without a plan,
name/root overrides, the plan/source flag rules (``translate.go:93-177``),
QA-cache slices, version output (``version.go``)."""

import os
import re
import shutil

import pytest

import logparse

from move2kube_amd.cli import main as cli
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import yamlio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def work(tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = tmp_path / "src"
    shutil.copytree(os.path.join(ROOT, "samples", "nodejs"), str(src / "nodejs"))
    (src / ".m2kignore").write_text(".\n")
    cwd = tmp_path / "cwd"
    cwd.mkdir()
    monkeypatch.chdir(cwd)
    return tmp_path


def _plan(path):
    return plantypes.read_plan(str(path))


def test_plan_default_file_in_cwd(work):
    assert cli.main(["plan", "-s", str(work / "src")]) == 0
    p = _plan(work / "cwd" / "m2k.plan")
    assert p.name == "myproject" and "nodejs" in p.services
    # the plan stores the root relative to the working directory
    with open(work / "cwd" / "m2k.plan") as f:
        assert "rootDir: ../src" in f.read()


def test_plan_into_existing_directory_and_name(work):
    (work / "plans").mkdir()
    assert cli.main(["plan", "-s", str(work / "src"), "-p", str(work / "plans"), "-n", "shop"]) == 0
    assert _plan(work / "plans" / "m2k.plan").name == "shop"


def test_plan_extensionless_missing_path_is_a_directory(work):
    target = work / "cwd" / "newdir"
    # missing extension-less path -> <path>/m2k.plan; the reference does not
    # create the directory, so the write fails (logged, exit 0)
    assert cli.main(["plan", "-s", str(work / "src"), "-p", str(target)]) == 0
    assert not (target / "m2k.plan").exists()
    assert cli.main(["plan", "-s", str(work / "src"), "-p", str(work / "cwd" / "x.plan")]) == 0
    assert (work / "cwd" / "x.plan").exists()


@pytest.mark.parametrize("bad", ["missing", "file"])
def test_plan_bad_source_is_fatal(work, bad):
    (work / "file").write_text("x")
    assert cli.main(["plan", "-s", str(work / bad)]) == 1


def test_plan_requires_source(work, capsys):
    # cobra MarkFlagRequired (plan.go:102): error + usage, then log.Fatalf
    assert cli.main(["plan"]) == 1
    err = capsys.readouterr().err
    assert err.startswith('Error: required flag(s) "source" not set\nUsage:\n  move2kube plan [flags]\n')
    assert logparse.logged(err, 'Error: "required flag(s) \\"source\\" not set"', "fatal")


def test_translate_without_plan_plans_and_curates(work):
    assert cli.main(["translate", "-s", str(work / "src"), "-o", str(work / "out"), "--qaskip"]) == 0
    out = work / "out" / "myproject"
    assert (out / "myproject" / "nodejs-deployment.yaml").exists()
    assert (out / "m2kqacache.yaml").exists()


def test_translate_needs_plan_or_source(work):
    # no m2k.plan in cwd and no -s: fatal
    assert cli.main(["translate", "--qaskip"]) == 1
    # an explicit plan path that does not exist is fatal even with -s
    assert cli.main(["translate", "-p", str(work / "nope.plan"), "-s", str(work / "src"), "--qaskip"]) == 1


def test_translate_with_plan_name_and_root_overrides(work):
    assert cli.main(["plan", "-s", str(work / "src")]) == 0
    # plan from cwd, renamed
    assert cli.main(["translate", "-n", "renamed", "-o", str(work / "out"), "--qaskip"]) == 0
    assert (work / "out" / "renamed" / "renamed" / "nodejs-deployment.yaml").exists()
    # same plan re-rooted onto a moved copy of the source
    shutil.copytree(str(work / "src"), str(work / "moved"))
    shutil.rmtree(str(work / "src"))
    assert cli.main(["translate", "-s", str(work / "moved"), "-o", str(work / "out2"), "--qaskip"]) == 0
    text = (work / "out2" / "myproject" / "copysources.sh").read_text()
    assert "moved" in text


def test_translate_plan_with_missing_root_is_fatal(work):
    assert cli.main(["plan", "-s", str(work / "src")]) == 0
    shutil.rmtree(str(work / "src"))
    assert cli.main(["translate", "-o", str(work / "out"), "--qaskip"]) == 1


def test_translate_qacache_slices_and_precedence(work):
    def cache(path, answer):
        path.write_text(yamlio.dump({
            "apiVersion": "move2kube.konveyor.io/v1alpha1", "kind": "QACache",
            "spec": {"solutions": [{"description": "Choose the artifact type:",
                                    "solution": {"type": "Select", "answer": [answer]}, "resolved": True}]}}))
        return str(path)
    a = cache(work / "a.yaml", "Helm")
    b = cache(work / "b.yaml", "Knative")
    # comma-joined and repeated -q both work; the LAST cache listed has the
    # highest priority (translate.go reverses the list, AddCaches prepends it)
    assert cli.main(["translate", "-s", str(work / "src"), "-o", str(work / "o1"), "--qaskip", "-q", b + "," + a]) == 0
    assert (work / "o1" / "myproject" / "myproject" / "Chart.yaml").exists()
    assert cli.main(["translate", "-s", str(work / "src"), "-o", str(work / "o2"), "--qaskip", "-q", a, "-q", b]) == 0
    assert "serving.knative.dev" in (work / "o2" / "myproject" / "myproject" / "nodejs-service.yaml").read_text()


def test_translate_output_path_is_a_file(work):
    (work / "out").mkdir()
    (work / "out" / "myproject").write_text("not a dir")
    assert cli.main(["translate", "-s", str(work / "src"), "-o", str(work / "out"), "--qaskip"]) == 1


@pytest.mark.parametrize("argv,want", [
    (["plan", "-s", "{w}/file/x"], "Unable to access source directory : stat {w}/file/x: not a directory"),
    (["plan", "-s", "{w}/src", "-p", "{w}/file/p.yaml"],
     "Error while accessing plan file path {w}/file/p.yaml : stat {w}/file/p.yaml: not a directory "),
    (["translate", "-s", "{w}/file/x", "--qaskip"],
     'Error while accessing the given source directory {w}/file/x Error: "stat {w}/file/x: not a directory"'),
    (["translate", "-s", "{w}/nope", "--qaskip"],
     'The given source directory {w}/nope does not exist. Error: "stat {w}/nope: no such file or directory"'),
    (["translate", "-s", "{w}/src", "-o", "{w}/file", "--qaskip"],
     'Error while accessing output directory at path {w}/file/myproject Error: '
     '"stat {w}/file/myproject: not a directory" . Exiting'),
    (["collect", "-s", "{w}/file/x"], "Error while accessing directory: {w}/file/x. "),
])
def test_stat_errors_are_reported_like_os_stat(work, capsys, argv, want):
    """cmd/move2kube/{plan,translate,collect}.go: only ENOENT is "does not
    exist"; ENOTDIR and the like are access errors, with Go's %q quoting."""
    (work / "file").write_text("x")
    w = str(work)
    assert cli.main([a.format(w=w) for a in argv]) == 1
    assert logparse.logged(capsys.readouterr().err, want.format(w=w), "fatal")


def test_log_quotes_like_go():
    from move2kube_amd.utils import log
    assert log.go_quote('a"b\\c\n\x01\xe9\udce9\u200b') == '"a\\"b\\\\c\\n\\x01\xe9\\xe9\\u200b"'
    assert log._format("%r and %s and %r", ("it's", "x", 3)) == '"it\'s" and x and 3'


def test_version(capsys):
    assert cli.main(["version"]) == 0
    short = capsys.readouterr().out.strip()
    assert short.startswith("v")
    assert cli.main(["version", "-l"]) == 0
    long = yamlio.load(capsys.readouterr().out)
    assert long["version"] == short and long["goVersion"].startswith("python")


def test_no_command_prints_help(capsys):
    assert cli.main([]) == 0
    assert "translate" in capsys.readouterr().out


def test_two_step_flow_matches_one_step_on_reference_samples(tmp_path, monkeypatch):
    """USAGE.md's two flows on the reference's samples/: ``translate -s src``
    (plan + curate inline) and ``plan -s src`` then ``translate`` (the plan is
    used uncurated, translate.go:151-172).  With default answers both write
    the same artifacts; only the QA cache (no curation questions) and
    copysources.sh (output location relative to the sources) differ."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    import refconfigs
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    monkeypatch.setenv("HOME", str(tmp_path))
    shutil.copytree(os.path.join(ROOT, "samples"), str(tmp_path / "samples"))
    monkeypatch.chdir(tmp_path)
    assert cli.main(["translate", "-s", "samples", "--qaskip", "-o", "one"]) == 0
    assert cli.main(["plan", "-s", "samples"]) == 0
    assert cli.main(["translate", "--qaskip"]) == 0
    diff = refconfigs.diff_files(str(tmp_path / "myproject"), str(tmp_path / "one" / "myproject"))
    assert diff == ["copysources.sh", "m2kqacache.yaml"]
    two = yamlio.load(open(str(tmp_path / "myproject" / "m2kqacache.yaml")).read())
    descs = [s["description"] for s in two["spec"]["solutions"]]
    assert "Select all services that are needed:" not in descs
    assert "Select all services that should be exposed:" in descs


def test_verbose_flag_turns_on_debug_lines(work, capsys):
    """`-v` (move2kube.go:41-46, PersistentPreRunE) sets the Debug level for the
    command: the planner's per-file debug lines appear, and go away again."""
    from move2kube_amd.utils import log
    try:
        assert cli.main(["-v", "plan", "-s", str(work / "src"), "-p", str(work / "cwd" / "v.plan")]) == 0
        levels = {lv for lv, _m in logparse.messages(capsys.readouterr().err)}
        assert {"debug", "info"} <= levels
    finally:
        log.set_verbose(False)
    assert cli.main(["plan", "-s", str(work / "src"), "-p", str(work / "cwd" / "q.plan")]) == 0
    assert "debug" not in {lv for lv, _m in logparse.messages(capsys.readouterr().err)}


def test_plan_that_is_a_directory_reads_like_ioutil_readfile(work, capsys):
    """translate.go:131-155 with <dir>/m2k.plan itself a directory: ReadFile
    opens it and fails on the read, so ReadPlan (planutils.go:168) and the
    fatal line carry ``read <path>: is a directory``."""
    (work / "plans" / "m2k.plan").mkdir(parents=True)
    w = str(work)
    assert cli.main(["translate", "-p", w + "/plans", "--qaskip"]) == 1
    err = capsys.readouterr().err
    assert logparse.logged(err, 'Failed to load the plan file at path "%s/plans/m2k.plan" Error '
                           '"read %s/plans/m2k.plan: is a directory"' % (w, w), "error")
    assert logparse.logged(err, 'Unable to read the plan at path %s/plans/m2k.plan Error: '
                           '"read %s/plans/m2k.plan: is a directory"' % (w, w), "fatal")
