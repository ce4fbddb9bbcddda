"""End-to-end: ``translate --qaskip`` of the samples corpus must reproduce the
checked-in expected output tree byte for byte (the BASELINE "manifest diff")."""

import os
import shutil

import pytest

import bench
from move2kube_amd import api

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def samples_copy(tmp_path):
    dst = tmp_path / "samples"
    shutil.copytree(os.path.join(ROOT, "samples"), str(dst), symlinks=True)
    return str(dst)


def _diff(actual, golden):
    a, g = bench.tree_files(actual), bench.tree_files(golden)
    problems = sorted(set(a) ^ set(g))
    for rel in sorted(set(a) & set(g)):
        with open(a[rel], "rb") as fa, open(g[rel], "rb") as fg:
            if fa.read() != fg.read():
                problems.append(rel)
    return problems


def test_full_samples_tree_matches_golden(samples_copy, tmp_path):
    out = api.translate(samples_copy, str(tmp_path / "out"), name="samples")
    assert _diff(out, bench.GOLDEN) == []


def test_single_nodejs_service(tmp_path):
    src = tmp_path / "nodejs"
    shutil.copytree(os.path.join(ROOT, "samples", "nodejs"), str(src))
    out = api.translate(str(src), str(tmp_path / "out"), name="single")
    files = bench.tree_files(out)
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
