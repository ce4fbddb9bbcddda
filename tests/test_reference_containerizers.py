"""``internal/containerizer/{dockerfile,s2i,reuse,manual}containerizer_test.go``,
one pytest per Go subtest: the returned container is compared whole with the
fixture's (or ``NewContainer``'s), as ``cmp.Equal`` does."""

import os
import shutil

import pytest

from conftest import ref_path
from goequal import assert_deep_equal
from move2kube_amd.containerizer.base import ContainerizerError
from move2kube_amd.containerizer.dockerfile import DockerfileContainerizer
from move2kube_amd.containerizer.manual import ManualContainerizer
from move2kube_amd.containerizer.reuse import ReuseContainerizer
from move2kube_amd.containerizer.s2i import S2IContainerizer
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import yamlio

pytestmark = pytest.mark.reference

TD = ref_path("internal", "containerizer", "testdata")


@pytest.fixture
def layout(tmp_path, monkeypatch, assets_dir):
    cwd = tmp_path / "internal" / "containerizer"
    cwd.mkdir(parents=True)
    for s in ("dockerfile", "nodejs"):
        shutil.copytree(ref_path("samples", s), str(tmp_path / "samples" / s))
    monkeypatch.chdir(cwd)
    return cwd


def _case(kind, case):
    d = os.path.join(TD, kind, "getcontainer", case)
    plan = plantypes.read_plan(os.path.join(d, "plan.yaml"))
    svc_file = os.path.join(d, "service.yaml")
    service = plantypes.Service.from_yaml(yamlio.load_raw(open(svc_file).read())) if os.path.exists(svc_file) else None
    want = yamlio.load(open(os.path.join(d, "container.yaml")).read()) if os.path.exists(os.path.join(d, "container.yaml")) else None
    return plan, service, want


def _go_yaml_container(d):
    """irtypes.Container as mustreadyaml fills it from container.yaml (go-yaml:
    lowercased field names; RepoInfo keeps its yaml tags)."""
    c = irtypes.Container(d.get("containerbuildtype", ""), "", bool(d.get("new")))
    c.image_names = list(d.get("imagenames") or [])
    c.repo_info = plantypes.RepoInfo.from_yaml(d.get("repoinfo") or {})
    c.new_files = dict(d.get("newfiles") or {})
    c.exposed_ports = list(d.get("exposedports") or [])
    c.user_id = d.get("userid", 0)
    c.accessed_dirs = list(d.get("accesseddirs") or [])
    return c


def test_dockerfile_get_container_for_the_sample_nodejs_app(layout):
    plan, _, want = _case("dockerfilecontainerizer", "normal")
    cont = DockerfileContainerizer().get_container(plan, plan.services["dockerfile"][0])
    assert_deep_equal(cont, _go_yaml_container(want))


@pytest.mark.parametrize("case", [
    pytest.param("incorrectservice", id="get container for the dockerfile sample when the service is wrong"),
    pytest.param("incorrectbuilder", id="get container for the dockerfile sample when the container build type is wrong")])
def test_dockerfile_errors(layout, case):
    plan, service, _ = _case("dockerfilecontainerizer", case)
    with pytest.raises(ContainerizerError):
        DockerfileContainerizer().get_container(plan, service)


def test_s2i_get_container_for_the_sample_nodejs_app(layout):
    plan, _, want = _case("s2icontainerizer", "normal")
    cont = S2IContainerizer().get_container(plan, plan.services["nodejs"][0])
    assert_deep_equal(cont, _go_yaml_container(want))


@pytest.mark.parametrize("case", [
    pytest.param("incorrectservice", id="get container for the nodejs app when the service is wrong"),
    pytest.param("incorrectbuilder", id="get container for the nodejs app when the container build type is wrong")])
def test_s2i_errors(layout, case):
    plan, service, _ = _case("s2icontainerizer", case)
    with pytest.raises(ContainerizerError):
        S2IContainerizer().get_container(plan, service)


def test_reuse_get_container_for_the_sample_nodejs_app(layout):
    plan, service, _ = _case("reusecontainerizer", "normal")
    cont = ReuseContainerizer().get_container(plan, service)
    assert_deep_equal(cont, irtypes.new_container(plantypes.REUSE, service.image, False))


def test_reuse_get_container_when_the_service_is_wrong(layout):
    plan, service, _ = _case("reusecontainerizer", "incorrectservice")
    with pytest.raises(ContainerizerError):
        ReuseContainerizer().get_container(plan, service)


def test_manual_get_container_for_the_sample_nodejs_app(layout):
    plan, service, _ = _case("manualcontainerizer", "normal")
    cont = ManualContainerizer().get_container(plan, service)
    assert_deep_equal(cont, irtypes.new_container(plantypes.MANUAL, service.image, True))


def test_manual_get_container_when_the_service_is_wrong(layout):
    plan, service, _ = _case("manualcontainerizer", "incorrectservice")
    with pytest.raises(ContainerizerError):
        ManualContainerizer().get_container(plan, service)
