"""Container image and CI (reference Dockerfile, scripts/installdeps.sh, .github/workflows):
the image carries operator-sdk installed by installdeps.sh, CI builds it and
runs scripts/image_e2e.sh against it.  No docker here, so the e2e script runs
with the CLI on the host (M2K_E2E_RUNNER) and the operator-sdk stand-in."""

import os
import subprocess
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB_BIN = os.path.join(ROOT, "tests", "fixtures", "configs", "bin")
E2E = os.path.join(ROOT, "scripts", "image_e2e.sh")


def _e2e(path):
    env = dict(os.environ, PATH=path, PYTHONPATH=ROOT, M2K_E2E_RUNNER="%s -m move2kube_amd" % sys.executable)
    return subprocess.run(["bash", E2E], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300)


def test_image_e2e_passes_on_a_correct_translate():
    p = _e2e(STUB_BIN + os.pathsep + os.environ["PATH"])
    out = p.stdout.decode()
    assert p.returncode == 0, out
    assert "0 files differ from tests/golden/reference/helm-openshift" in out


def test_image_e2e_fails_without_operator_sdk(tmp_path):
    # PATH without the stand-in (and without a real operator-sdk)
    path = os.pathsep.join(d for d in os.environ["PATH"].split(os.pathsep)
                           if d and not os.path.exists(os.path.join(d, "operator-sdk")))
    p = _e2e(path)
    assert p.returncode == 1
    assert "operator-sdk did not run" in p.stdout.decode()


def _stages():
    stages, cur = [], None
    for line in open(os.path.join(ROOT, "Dockerfile")):
        if line.startswith("FROM "):
            cur = [line]
            stages.append(cur)
        elif cur is not None:
            cur.append(line)
    return ["".join(s) for s in stages]


def test_dockerfile_installs_and_ships_operator_sdk():
    builder, runtime = _stages()
    assert "scripts/installdeps.sh -y" in builder and "INSTALL_DOCKER=0" in builder
    assert "PYTORCH_ROCM_ARCH=gfx950" in builder
    assert "FROM ${RUNTIME_IMAGE}" in runtime
    text = open(os.path.join(ROOT, "Dockerfile")).read()
    assert "ARG RUNTIME_IMAGE=python:3.10-slim" in text
    assert "/opt/m2k-deps/operator-sdk" in runtime and "/usr/local/bin/" in runtime
    assert "operator-sdk version" in runtime  # the image build fails without a working tool
    assert 'ENTRYPOINT ["move2kube"]' in runtime


def test_ci_builds_the_image_and_runs_e2e():
    wf = yaml.safe_load(open(os.path.join(ROOT, ".github", "workflows", "ci.yml")))
    job = wf["jobs"]["image"]
    runs = " ".join(s.get("run", "") for s in job["steps"])
    assert "make cbuild" in runs and "scripts/image_e2e.sh" in runs and "docker push" in runs
    assert job["needs"] == ["cpu"]


def test_runtime_stage_rebuilds_the_startcache_for_its_interpreter():
    # the builder's python3 and the slim runtime's differ: the cache built in
    # the builder would be ignored (utils/startcache.py interpreter tag)
    text = open(os.path.join(ROOT, "Dockerfile")).read()
    runtime = text[text.index("FROM ${RUNTIME_IMAGE}"):]
    assert "move2kube_amd.ops.startcache_build" in runtime
