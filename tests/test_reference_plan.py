"""Plan schema parity with the reference's own fixtures
(``types/plan/planutils_test.go``, ``internal/move2kube/planner_test.go``)."""

import os
import shutil

import pytest

from conftest import ref_path
from goequal import assert_deep_equal
from move2kube_amd import api, move2kube
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import common
from move2kube_amd.utils.constants import settings

pytestmark = pytest.mark.reference


def test_write_plan_roundtrip_is_byte_identical(tmp_path, assets_dir, monkeypatch):
    fixture = ref_path("types", "plan", "testdata", "setrootdir", "nodejsplan.yaml")
    cwd = tmp_path / "types" / "plan"
    cwd.mkdir(parents=True)
    monkeypatch.chdir(cwd)
    p = plantypes.read_plan(fixture)
    out = tmp_path / "actual.yaml"
    plantypes.write_plan(str(out), p)
    assert out.read_text() == open(fixture).read()


def test_set_root_dir_matches_templated_fixture(tmp_path, assets_dir, monkeypatch):
    cwd = tmp_path / "types" / "plan"
    cwd.mkdir(parents=True)
    monkeypatch.chdir(cwd)
    p = plantypes.read_plan(ref_path("types", "plan", "testdata", "setrootdir", "nodejsplan.yaml"))
    new_root = os.path.abspath("new/root/directory")
    p.set_root_dir(new_root)
    assert p.root_dir == new_root
    tpl = open(ref_path("types", "plan", "testdata", "setrootdir", "templatizednodejsplan.yaml")).read()
    want_yaml = common.get_string_from_template(tpl, {"PWD": str(cwd), "TempDir": settings.temp_path})
    from move2kube_amd.utils import yamlio
    want = plantypes.Plan.from_yaml(yamlio.load_raw(want_yaml))
    assert_deep_equal(p, want)


def test_set_root_dir_and_back(tmp_path, assets_dir, monkeypatch):
    cwd = tmp_path / "types" / "plan"
    cwd.mkdir(parents=True)
    monkeypatch.chdir(cwd)
    fixture = ref_path("types", "plan", "testdata", "setrootdir", "nodejsplan.yaml")
    p = plantypes.read_plan(fixture)
    orig = plantypes.read_plan(fixture)
    p.set_root_dir(os.path.abspath("new/root/directory"))
    p.set_root_dir(os.path.abspath("../../samples/nodejs"))
    assert_deep_equal(p, orig)


@pytest.mark.parametrize("with_cache_dir", [
    pytest.param(False, id="create plan for empty app and without the cache folder"),
    pytest.param(True, id="create plan for empty app")])
def test_create_plan_for_empty_dir(tmp_path, assets_dir, with_cache_dir):
    app = tmp_path / "app"
    app.mkdir()
    if with_cache_dir:
        os.makedirs(settings.assets_path, exist_ok=True)
    p = move2kube.create_plan(str(app), "project1")
    want = plantypes.new_plan()
    want.name = "project1"
    want.set_root_dir(str(app))
    assert_deep_equal(p, want)


def test_create_plan_for_reference_nodejs_sample(tmp_path, monkeypatch):
    # layout so that the fixture's relative rootDir (../../samples/nodejs) resolves to our copy
    cwd = tmp_path / "internal" / "move2kube"
    cwd.mkdir(parents=True)
    shutil.copytree(ref_path("samples", "nodejs"), str(tmp_path / "samples" / "nodejs"))
    monkeypatch.chdir(cwd)
    with api.Session() as s:
        want = plantypes.read_plan(ref_path("internal", "move2kube", "testdata", "expectedplanfornodejsapp.yaml"))
        actual = s.plan(os.path.abspath("../../samples/nodejs"), "nodejs-app")
    for services in actual.services.values():
        for svc in services:
            svc.repo_info = plantypes.RepoInfo()
    # the CNB option needs a Docker daemon (the reference test needs one too)
    for name in want.services:
        want.services[name] = [s for s in want.services[name] if s.container_build_type != plantypes.CNB]
    assert_deep_equal(actual, want)


def test_create_plan_for_reference_nodejs_sample_with_cnb(tmp_path, monkeypatch):
    """The whole fixture, CNB option included: the ``podman`` stand-in
    (tests/fixtures/configs/bin) answers the reference's container-runtime
    provider (containerruntimeprovider.go) the way a machine with podman and
    both builder images would, so both builders support the nodejs sample."""
    from move2kube_amd.containerizer import cnb
    cwd = tmp_path / "internal" / "move2kube"
    cwd.mkdir(parents=True)
    shutil.copytree(ref_path("samples", "nodejs"), str(tmp_path / "samples" / "nodejs"))
    monkeypatch.chdir(cwd)
    stubs = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "configs", "bin")
    monkeypatch.setenv("PATH", stubs + os.pathsep + os.environ.get("PATH", ""))
    monkeypatch.setenv("M2K_DISABLE_CNB", "0")
    cnb.reset_cache()
    with api.Session() as s:
        want = plantypes.read_plan(ref_path("internal", "move2kube", "testdata", "expectedplanfornodejsapp.yaml"))
        actual = s.plan(os.path.abspath("../../samples/nodejs"), "nodejs-app")
    for services in actual.services.values():
        for svc in services:
            svc.repo_info = plantypes.RepoInfo()
    assert [s.container_build_type for s in actual.services["nodejs"]] == ["NewDockerfile", "S2I", "CNB"]
    assert_deep_equal(actual, want)
