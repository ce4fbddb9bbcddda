"""Regression: ``translate --qaskip`` of the builder-authored corpus
(``tests/fixtures/extra_samples``: source apps plus a compose app, a CF
manifest and Kubernetes YAMLs the reference's ``samples/`` lacks) must
reproduce ``tests/golden/regression/extra_samples`` byte for byte.

Unlike ``tests/golden/reference`` (derived from the reference, never
regenerated), this tree is our own output: ``M2K_REGEN_GOLDEN=1`` rewrites it
after an intended change (review the diff)."""

import os
import shutil
import sys

import pytest

from move2kube_amd import api

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
import refconfigs  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPUS = os.path.join(ROOT, "tests", "fixtures", "extra_samples")
GOLDEN = os.path.join(ROOT, "tests", "golden", "regression", "extra_samples")


@pytest.fixture
def samples_copy(tmp_path):
    dst = tmp_path / "samples"
    shutil.copytree(CORPUS, str(dst), symlinks=True)
    return str(dst)


def _diff(actual, golden):
    a, g = refconfigs.tree_files(actual), refconfigs.tree_files(golden)
    problems = sorted(set(a) ^ set(g))
    for rel in sorted(set(a) & set(g)):
        with open(a[rel], "rb") as fa, open(g[rel], "rb") as fg:
            if fa.read() != fg.read():
                problems.append(rel)
    return problems


def test_full_samples_tree_matches_golden(samples_copy, tmp_path):
    out = api.translate(samples_copy, str(tmp_path / "out"), name="samples")
    if os.environ.get("M2K_REGEN_GOLDEN") == "1":
        shutil.rmtree(GOLDEN, ignore_errors=True)
        shutil.copytree(out, GOLDEN, symlinks=True)
    assert _diff(out, GOLDEN) == []


def test_single_nodejs_service(tmp_path):
    src = tmp_path / "nodejs"
    shutil.copytree(os.path.join(ROOT, "samples", "nodejs"), str(src))
    out = api.translate(str(src), str(tmp_path / "out"), name="single")
    files = refconfigs.tree_files(out)
    assert "single/nodejs-deployment.yaml" in files
    assert "single/nodejs-service.yaml" in files
    assert "containers/Dockerfile.nodejs" in files
    text = open(files["single/nodejs-deployment.yaml"]).read()
    assert "image: docker.io/single/nodejs:latest" in text
    assert "replicas: 2" in text


def test_translate_is_repeatable_in_process(samples_copy, tmp_path):
    with api.Session() as s:
        o1 = s.translate(samples_copy, str(tmp_path / "o1"), name="samples")
        o2 = s.translate(samples_copy, str(tmp_path / "o2"), name="samples")
    assert _diff(o1, o2) == []


def test_retranslate_replaces_output_and_leaves_nothing_behind(tmp_path):
    """The previous output tree is removed (RemoveAll, translator.go:64) - on a
    background thread that is joined before translate returns."""
    src = tmp_path / "nodejs"
    shutil.copytree(os.path.join(ROOT, "samples", "nodejs"), str(src))
    outdir = tmp_path / "out"
    with api.Session() as s:
        out = s.translate(str(src), str(outdir), name="p")
        stale = os.path.join(out, "p", "stale-file.yaml")
        with open(stale, "w") as f:
            f.write("x")
        s.translate(str(src), str(outdir), name="p")
    assert not os.path.exists(stale)
    assert sorted(os.listdir(str(outdir))) == ["p"]
