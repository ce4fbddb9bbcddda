"""Question order of a Helm translate with new containers in git repos
(reference ``internal/translator/translator.go:92-102``): the CI/CD transform,
whose git secrets ask for known hosts and SSH keys, runs before the main
transformer, so its questions come first and a fatal error among them stops
the run before any of the chart is written or operator-sdk starts.  Only the
write of the Tekton objects waits for operator-sdk (``move2kube.py``)."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402

from move2kube_amd import transformer  # noqa: E402
from move2kube_amd.utils import log, yamlio  # noqa: E402


def _helm_git_run(tmp_path):
    run = refconfigs.Run("git-repos", str(tmp_path)).prepare()
    cache = tmp_path / "helm-qacache.yaml"
    cache.write_text(refconfigs.qacache_text({refconfigs.Q_ARTIFACT: "Helm"}))
    run.caches = [str(cache)]
    return run


def test_cicd_questions_before_the_kubernetes_transform(tmp_path, monkeypatch):
    run = _helm_git_run(tmp_path)
    order = []
    for cls, name in ((transformer.CICDTransformer, "transform"), (transformer.K8sTransformer, "transform"),
                      (transformer.K8sTransformer, "write_objects"), (transformer.CICDTransformer, "write_objects")):
        orig = getattr(cls, name)

        def wrapped(self, *a, _orig=orig, _tag="%s.%s" % (cls.__name__, name)):
            order.append(_tag)
            return _orig(self, *a)
        monkeypatch.setattr(cls, name, wrapped)
    undo = run.apply_env()
    try:
        with run.session() as s:
            out = run.step(s)
    finally:
        undo()
    # the Tekton objects are written inside the chart write's operator-sdk wait
    assert order[:3] == ["CICDTransformer.transform", "K8sTransformer.transform", "K8sTransformer.write_objects"]
    assert "CICDTransformer.write_objects" in order
    assert os.path.exists(os.path.join(out, "myproject", "Chart.yaml"))
    assert os.path.exists(os.path.join(out, "cicd", "myproject-clone-build-push-pipeline.yaml"))
    # the git questions are recorded; the Kubernetes transform asks nothing after them
    cache = yamlio.load(open(os.path.join(out, "m2kqacache.yaml")).read())
    descs = [s["description"] for s in cache["spec"]["solutions"]]
    git = [i for i, d in enumerate(descs) if "public key for the domain" in d or "ssh key" in d.lower()]
    assert git and git[-1] == len(descs) - 1, descs


def test_a_fatal_cicd_question_stops_before_the_chart(tmp_path, monkeypatch):
    run = _helm_git_run(tmp_path)
    started = []

    def fatal(self, ir):
        log.fatal("no answer for the SSH key question")
    monkeypatch.setattr(transformer.CICDTransformer, "transform", fatal)
    monkeypatch.setattr(transformer.K8sTransformer, "transform", lambda self, ir: started.append("k8s"))
    undo = run.apply_env()
    try:
        with run.session() as s:
            with pytest.raises(log.FatalError):
                run.step(s)
    finally:
        undo()
    assert started == []
    assert not os.path.exists(os.path.join(run.out, "myproject", "Chart.yaml"))
    assert not os.path.exists(os.path.join(run.out, "myproject-operator"))
