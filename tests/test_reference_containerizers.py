"""Containerizer GetContainer parity (``internal/containerizer/*_test.go`` fixtures)."""

import os
import shutil

import pytest

from conftest import ref_path
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


def _check(cont, want):
    assert cont.container_build_type == want["containerbuildtype"]
    assert cont.image_names == want["imagenames"]
    assert cont.new == want["new"]
    assert cont.exposed_ports == want["exposedports"]
    assert cont.user_id == want["userid"]
    assert cont.accessed_dirs == (want.get("accesseddirs") or [])
    assert cont.repo_info.target_path == want["repoinfo"]["targetPath"]
    assert sorted(cont.new_files) == sorted(want["newfiles"])
    # byte for byte, license headers included (the fixtures are the reference's output)
    for k, v in want["newfiles"].items():
        assert cont.new_files[k] == v, k


def test_dockerfile_normal(layout):
    plan, _, want = _case("dockerfilecontainerizer", "normal")
    service = plan.services["dockerfile"][0]
    cz = DockerfileContainerizer()
    cont = cz.get_container(plan, service)
    _check(cont, want)


@pytest.mark.parametrize("case", ["incorrectservice", "incorrectbuilder"])
def test_dockerfile_errors(layout, case):
    plan, service, _ = _case("dockerfilecontainerizer", case)
    with pytest.raises(ContainerizerError):
        DockerfileContainerizer().get_container(plan, service)


def test_s2i_normal(layout):
    plan, _, want = _case("s2icontainerizer", "normal")
    service = plan.services["nodejs"][0]
    cont = S2IContainerizer().get_container(plan, service)
    _check(cont, want)


@pytest.mark.parametrize("case", ["incorrectservice", "incorrectbuilder"])
def test_s2i_errors(layout, case):
    plan, service, _ = _case("s2icontainerizer", case)
    with pytest.raises(ContainerizerError):
        S2IContainerizer().get_container(plan, service)


def test_reuse_normal(layout):
    plan, service, _ = _case("reusecontainerizer", "normal")
    cont = ReuseContainerizer().get_container(plan, service)
    want = irtypes.new_container(plantypes.REUSE, service.image, False)
    assert vars_of(cont) == vars_of(want)


def test_reuse_error(layout):
    plan, service, _ = _case("reusecontainerizer", "incorrectservice")
    with pytest.raises(ContainerizerError):
        ReuseContainerizer().get_container(plan, service)


def test_manual_normal(layout):
    plan, service, _ = _case("manualcontainerizer", "normal")
    cont = ManualContainerizer().get_container(plan, service)
    want = irtypes.new_container(plantypes.MANUAL, service.image, True)
    assert vars_of(cont) == vars_of(want)


def test_manual_error(layout):
    plan, service, _ = _case("manualcontainerizer", "incorrectservice")
    with pytest.raises(ContainerizerError):
        ManualContainerizer().get_container(plan, service)


def vars_of(c):
    return (c.container_build_type, c.image_names, c.new, c.new_files, c.exposed_ports, c.user_id, c.accessed_dirs,
            c.repo_info.to_yaml())
