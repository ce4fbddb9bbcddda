"""operator-sdk handling of the Helm output (reference
``internal/transformer/k8stransformer.go:215-247``): the tool runs in
``<out>/<project>-operator`` over the absolute chart path; a missing tool or a
failing run is a warning with the tool's stdout, never an error."""

import os
import stat

import pytest

from move2kube_amd.transformer import K8sTransformer
from move2kube_amd.utils import log


def _tool(bindir, body):
    os.makedirs(bindir, exist_ok=True)
    p = os.path.join(bindir, "operator-sdk")
    with open(p, "w") as f:
        f.write("#!/bin/sh\n" + body)
    os.chmod(p, os.stat(p).st_mode | stat.S_IXUSR)


@pytest.fixture
def warnings_seen(monkeypatch):
    seen = []
    monkeypatch.setattr(log, "warning", lambda msg, *a: seen.append(msg % a if a else msg))
    return seen


def test_success_runs_in_operator_dir_with_absolute_chart(tmp_path, monkeypatch, warnings_seen):
    _tool(str(tmp_path / "bin"), 'pwd > where.txt; echo "$@" > args.txt\n')
    monkeypatch.setenv("PATH", str(tmp_path / "bin") + os.pathsep + os.environ["PATH"])
    out = tmp_path / "out"
    (out / "proj").mkdir(parents=True)
    (out / "proj-operator").mkdir()
    (out / "proj-operator" / "stale").write_text("x")
    assert K8sTransformer.create_operator("proj", str(out)) is True
    op = out / "proj-operator"
    assert not (op / "stale").exists()  # os.RemoveAll before the run
    assert os.path.realpath((op / "where.txt").read_text().strip()) == os.path.realpath(str(op))
    assert (op / "args.txt").read_text().split() == [
        "init", "--plugins=helm", "--helm-chart=" + str(out / "proj"), "--domain=io", "--group=proj", "--version=v1alpha1"]
    assert warnings_seen == []


def test_failure_is_a_warning_with_stdout(tmp_path, monkeypatch, warnings_seen):
    _tool(str(tmp_path / "bin"), 'echo "chart invalid"; echo "ignored" >&2; exit 3\n')
    monkeypatch.setenv("PATH", str(tmp_path / "bin") + os.pathsep + os.environ["PATH"])
    (tmp_path / "out" / "proj").mkdir(parents=True)
    assert K8sTransformer.create_operator("proj", str(tmp_path / "out")) is False
    assert warnings_seen == ["Error during operator creation : exit status 3, chart invalid\n"]


def test_missing_tool_is_a_warning(tmp_path, monkeypatch, warnings_seen):
    monkeypatch.setenv("PATH", str(tmp_path / "empty"))
    assert K8sTransformer.create_operator("proj", str(tmp_path)) is False
    assert len(warnings_seen) == 1 and warnings_seen[0].startswith("Unable to find operator-sdk.")
    assert not (tmp_path / "proj-operator").exists()


def test_large_output_does_not_block(tmp_path, monkeypatch, warnings_seen):
    """The tool's stdout goes to a file, so a chatty tool cannot fill a pipe
    while the container files are written."""
    _tool(str(tmp_path / "bin"), 'i=0; while [ $i -lt 3000 ]; do echo "line $i of a long log output"; i=$((i+1)); done; exit 1\n')
    monkeypatch.setenv("PATH", str(tmp_path / "bin") + os.pathsep + os.environ["PATH"])
    (tmp_path / "out" / "proj").mkdir(parents=True)
    started = K8sTransformer.start_operator("proj", str(tmp_path / "out"))
    assert started is not None
    assert K8sTransformer.finish_operator(started) is False
    assert warnings_seen and warnings_seen[0].count("\n") == 3000


def test_previous_output_is_gone_before_operator_sdk_starts(tmp_path, monkeypatch):
    """A Helm translate over an existing output: the old tree, unlinked on a
    thread while the new one is built, is gone before operator-sdk starts
    (the tool copies the chart on the same filesystem)."""
    import sys
    import threading
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
    import refconfigs
    run = refconfigs.Run("helm-openshift", str(tmp_path)).prepare()
    seen = []
    orig = K8sTransformer.start_operator

    def start(project, basepath):
        seen.append([t.name for t in threading.enumerate() if t.name == "m2k-remove-old-output"])
        seen.append([n for n in os.listdir(os.path.dirname(os.path.abspath(basepath))) if ".m2k-old-" in n])
        return orig(project, basepath)
    monkeypatch.setattr(K8sTransformer, "start_operator", staticmethod(start))
    undo = run.apply_env()
    try:
        with run.session() as s:
            run.step(s)
            seen.clear()
            run.step(s)
    finally:
        undo()
    assert seen == [[], []]
    assert refconfigs.diff_files(run.out, refconfigs.golden_dir("helm-openshift"), work=run.work) == []
