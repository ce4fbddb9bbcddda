"""The five BASELINE.json configurations, each checked end to end against an
expected output tree under ``tests/golden/configs/<name>`` ("manifest diff = 0",
SURVEY.md §6):

1. ``golang``   - ``translate -s samples/golang`` (one service, plumbing only)
2. ``compose``  - ``translate -s samples/compose`` (compose -> K8s, multi-service)
3. ``java-cnb`` - samples/java-maven + samples/java-gradle through the CNB
   containerizer (a stand-in for the builder detect phase, as in the reference's
   own any2kube tests, ``internal/source/any2kube_test.go``)
4. ``cf``       - ``collect -a cf`` (stub ``cf`` CLI) + plan + translate of a CF
   manifest, with the collected metadata dropped into the source tree
5. ``helm-openshift`` - the whole samples tree to a Helm chart + operator
   (stub ``operator-sdk``) for the Openshift cluster profile, answers replayed
   from a QA cache (``-q``)

Set ``M2K_REGEN_GOLDEN=1`` to rewrite the expected trees after an intended
output change (then review the diff).
"""

import os
import shutil

import pytest

import bench
from move2kube_amd import api
from move2kube_amd.cli import main as cli_main

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "configs")
FIXTURES = os.path.join(ROOT, "tests", "fixtures")
STUBBIN = os.path.join(FIXTURES, "stubbin")


@pytest.fixture(autouse=True)
def _offline(monkeypatch):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    from move2kube_amd.containerizer.cnb import providers
    providers.reset_providers()
    yield
    providers.reset_providers()


def _copy_samples(dst, *names):
    os.makedirs(dst, exist_ok=True)
    # like samples/.m2kignore: the recursive detectors must not claim the root
    with open(os.path.join(dst, ".m2kignore"), "w") as f:
        f.write(".\n")
    for n in names:
        shutil.copytree(os.path.join(ROOT, "samples", n), os.path.join(dst, n), symlinks=True)
    return dst


def _check(name, out):
    golden = os.path.join(GOLDEN, name)
    if os.environ.get("M2K_REGEN_GOLDEN") == "1":
        shutil.rmtree(golden, ignore_errors=True)
        shutil.copytree(out, golden, symlinks=True)
    a, g = bench.tree_files(out), bench.tree_files(golden)
    problems = sorted(set(a) ^ set(g))
    for rel in sorted(set(a) & set(g)):
        with open(a[rel], "rb") as fa, open(g[rel], "rb") as fg:
            if fa.read() != fg.read():
                problems.append(rel)
    assert problems == [], "output differs from %s" % golden


def test_config_golang(tmp_path):
    src = _copy_samples(str(tmp_path / "src"), "golang")
    out = api.translate(os.path.join(src, "golang"), str(tmp_path / "out"), name="golang")
    files = bench.tree_files(out)
    assert "golang/golang-deployment.yaml" in files
    _check("golang", out)


def test_config_compose(tmp_path):
    src = _copy_samples(str(tmp_path / "src"), "compose")
    out = api.translate(os.path.join(src, "compose"), str(tmp_path / "out"), name="compose")
    files = bench.tree_files(out)
    for svc in ("api", "web", "redis"):
        assert "compose/%s-deployment.yaml" % svc in files
    _check("compose", out)


def test_config_java_cnb(tmp_path, monkeypatch):
    from move2kube_amd.containerizer.cnb import providers

    def supported(path, builder):
        # the Java buildpacks of both builders pass detection on a maven or gradle build
        return any(os.path.isfile(os.path.join(path, m)) for m in ("pom.xml", "build.gradle"))
    monkeypatch.setattr(providers, "is_builder_supported", supported)
    src = _copy_samples(str(tmp_path / "java"), "java-maven", "java-gradle")
    cache = os.path.join(FIXTURES, "configs", "cnb-qacache.yaml")
    out = api.translate(src, str(tmp_path / "out"), name="java", qacaches=[cache])
    files = bench.tree_files(out)
    for svc in ("java-maven", "java-gradle"):
        assert "containers/%s/%s-cnb-build.sh" % (svc, svc) in files
        assert "java/%s-deployment.yaml" % svc in files
    assert not any(f.startswith("containers/Dockerfile") for f in files)
    _check("java-cnb", out)


# buildpack order of the two default builders, as a docker daemon would report
# from their ``io.buildpacks.buildpack.order`` labels
BUILDER_BUILDPACKS = {
    "cloudfoundry/cnb:cflinuxfs3": ["org.cloudfoundry.nodejs", "org.cloudfoundry.python",
                                    "org.cloudfoundry.go", "org.cloudfoundry.staticfile"],
    "gcr.io/buildpacks/builder": ["google.nodejs.runtime", "google.python.runtime", "google.go.runtime"],
}


def test_config_cf(tmp_path, monkeypatch):
    from move2kube_amd.containerizer.cnb import providers
    monkeypatch.setattr(providers, "get_all_buildpacks", lambda builders: dict(BUILDER_BUILDPACKS))
    monkeypatch.setenv("PATH", STUBBIN + os.pathsep + os.environ.get("PATH", ""))
    src = _copy_samples(str(tmp_path / "cf"), "cfapp")
    collected = str(tmp_path / "collect")
    assert cli_main.main(["collect", "-a", "cf", "-s", src, "-o", collected]) == 0
    m2k_collect = os.path.join(collected, "m2k_collect")
    assert os.path.isdir(os.path.join(m2k_collect, "cf"))
    shutil.copytree(m2k_collect, os.path.join(src, "m2k_collect"))
    out = api.translate(src, str(tmp_path / "out"), name="cf")
    files = bench.tree_files(out)
    assert "cf/cf-hello-deployment.yaml" in files
    # app1 only exists in the running instance (cf curl /v2/apps): its nodejs
    # buildpack maps to google.nodejs.runtime (weighted edit distance 21 vs 27)
    with open(files["containers/m2k_collect/cf/app1-cnb-build.sh"]) as f:
        assert "-B gcr.io/buildpacks/builder" in f.read()
    _check("cf", out)


def test_config_helm_openshift(tmp_path, monkeypatch):
    monkeypatch.setenv("PATH", STUBBIN + os.pathsep + os.environ.get("PATH", ""))
    src = str(tmp_path / "samples")
    shutil.copytree(os.path.join(ROOT, "samples"), src, symlinks=True)
    cache = os.path.join(FIXTURES, "configs", "helm-openshift-qacache.yaml")
    out = api.translate(src, str(tmp_path / "out"), name="samples", qacaches=[cache])
    files = bench.tree_files(out)
    assert "samples/Chart.yaml" in files and "samples/values.yaml" in files
    assert "samples-operator/PROJECT" in files
    # Openshift profile: DeploymentConfig + Route instead of Deployment + Ingress
    assert any(f.endswith("-deploymentconfig.yaml") for f in files)
    assert any(f.endswith("-route.yaml") for f in files)
    assert not any(f.endswith("-ingress.yaml") for f in files)
    _check("helm-openshift", out)


@pytest.mark.reference
def test_reference_samples_tree(tmp_path):
    """The reference's own ``samples/`` corpus (read-only fixture) end to end:
    every sample becomes a service with a Deployment and a Service, the compose
    file's api/redis/web and the two Dockerfiles are found as well."""
    from conftest import ref_path
    src = str(tmp_path / "samples")
    shutil.copytree(ref_path("samples"), src, symlinks=True)
    out = api.translate(src, str(tmp_path / "out"), name="refsamples")
    files = set(os.listdir(os.path.join(out, "refsamples")))
    services = {"api", "redis", "web", "docker-compose", "dockerfile", "golang", "java-gradle", "java-maven",
                "nodejs", "php", "python", "ruby", "refsamples-docker-compose-api",
                "refsamples-docker-compose-web", "refsamples-dockerfile"}
    for s in services:
        assert "%s-deployment.yaml" % s in files and "%s-service.yaml" % s in files, s
    assert "refsamples-ingress.yaml" in files
