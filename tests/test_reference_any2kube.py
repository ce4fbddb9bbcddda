"""Any2Kube discovery / translation parity with ``internal/source/any2kube_test.go``."""

import base64
import os
import shutil

import pytest

from conftest import ref_path
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source.any2kube import Any2KubeTranslator
from move2kube_amd.utils import tarutil, yamlio

pytestmark = pytest.mark.reference

SRC_TESTDATA = ref_path("internal", "source", "testdata")


def _svc_dump(services):
    return yamlio.dump([s.to_yaml() for s in services])


def _plan_for(root, name="nodejs-app"):
    p = plantypes.new_plan()
    p.name = name
    p.set_root_dir(root)
    return p


def _strip_repo(services):
    for s in services:
        s.repo_info = plantypes.RepoInfo()
    return services


@pytest.fixture
def fake_cnb(monkeypatch):
    """Stand-in for a Docker daemon running the CNB builders' detect phase: the
    nodejs/java buildpacks pass when a package.json / pom.xml is at the root."""
    from move2kube_amd.containerizer.cnb import providers

    def supported(path, builder):
        return any(os.path.isfile(os.path.join(path, m)) for m in ("package.json", "pom.xml"))
    monkeypatch.setattr(providers, "is_builder_supported", supported)
    monkeypatch.setattr(providers, "is_builder_supported_batch", lambda pairs: [supported(p, b) for p, b in pairs])


@pytest.fixture
def layout(tmp_path, monkeypatch, fake_cnb):
    """tmp/internal/source (cwd) + tmp/samples/nodejs + testdata copies.  Like the
    reference tests, no assets are unpacked, so only CNB options appear."""
    cwd = tmp_path / "internal" / "source"
    cwd.mkdir(parents=True)
    shutil.copytree(ref_path("samples", "nodejs"), str(tmp_path / "samples" / "nodejs"))
    shutil.copytree(SRC_TESTDATA, str(cwd / "testdata"))
    monkeypatch.chdir(cwd)
    return cwd


def test_non_existent_dir(tmp_path, assets_dir):
    services = Any2KubeTranslator().get_service_options(str(tmp_path / "nope"), plantypes.new_plan())
    assert services == []


def test_empty_dir(tmp_path, assets_dir):
    assert Any2KubeTranslator().get_service_options(str(tmp_path), plantypes.new_plan()) == []


def test_unreadable_entries(unprivileged):
    """any2kube_test.go:72-95: a subdirectory with mode 0 and an unreadable
    ``.m2kignore`` give no services and no error."""
    root = unprivileged.tmp
    os.mkdir(os.path.join(root, "nopermstoread"))
    with open(os.path.join(root, ".m2kignore"), "w") as f:
        f.write("foo/")
    unprivileged.chown()
    os.chmod(os.path.join(root, "nopermstoread"), 0)
    os.chmod(os.path.join(root, ".m2kignore"), 0)

    def check():
        from move2kube_amd.utils import fsindex
        fsindex.invalidate()
        assert Any2KubeTranslator().get_service_options(root, plantypes.new_plan()) == []
    unprivileged.run(check)


def test_nodejs_app_empty_plan(layout):
    root = os.path.abspath("../../samples/nodejs")
    want = plantypes.read_plan("testdata/expectedservicesfornodejsapp.yaml").services["nodejs"]
    got = _strip_repo(Any2KubeTranslator().get_service_options(root, _plan_for(root)))
    assert _svc_dump(got) == _svc_dump(want)


def test_nodejs_app_already_containerized(layout):
    root = os.path.abspath("../../samples/nodejs")
    p = _plan_for(root)
    svc1 = plantypes.Service.new("svc1", "Any2Kube")
    svc1.source_artifacts[plantypes.SOURCE_DIRECTORY_ARTIFACT] = [root]
    p.services = {"svc1": [svc1]}
    assert Any2KubeTranslator().get_service_options(root, p) == []


def test_m2kignore_dir_but_not_subdirs(layout):
    root = os.path.abspath("testdata/nodejsappwithm2kignorecase1")
    want = plantypes.read_plan("testdata/expectedservicesfornodejsappwithm2kignorecase1.yaml").services["includeme"]
    got = _strip_repo(Any2KubeTranslator().get_service_options(root, _plan_for(root)))
    assert _svc_dump(got) == _svc_dump(want)


def test_m2kignore_everything_but_one_subdir(layout):
    root = os.path.abspath("testdata/javamavenappwithm2kignorecase2")
    want = plantypes.read_plan("testdata/expectedservicesforjavamavenappwithm2kignorecase2.yaml").services["java-maven"]
    got = _strip_repo(Any2KubeTranslator().get_service_options(root, _plan_for(root, "java-maven-app")))
    assert _svc_dump(got) == _svc_dump(want)


def test_m2kignore_include_dir_ignore_subdirs(tmp_path, assets_dir):
    sub = tmp_path / "includeme" / "excludeme"
    sub.mkdir(parents=True)
    (tmp_path / ".m2kignore").write_bytes(open(os.path.join(SRC_TESTDATA, "m2kignoreforignorecontents"), "rb").read())
    (sub / "package.json").write_text("this is ' invalid json")
    assert Any2KubeTranslator().get_service_options(str(tmp_path), plantypes.new_plan()) == []


def test_multiple_hierarchical_m2kignores(tmp_path, assets_dir):
    with open(os.path.join(SRC_TESTDATA, "testmultiplem2kignores.tar"), "rb") as f:
        tarutil.untar_string(base64.b64encode(f.read()).decode(), str(tmp_path))
    root = str(tmp_path / "testmultiplem2kignores")
    assert Any2KubeTranslator().get_service_options(root, plantypes.new_plan()) == []


def test_translate_no_services(assets_dir):
    p = plantypes.new_plan()
    ir = Any2KubeTranslator().translate([], p)
    assert ir.services == {} and ir.containers == [] and ir.storages == []


def test_translate_nodejs_services_to_ir():
    data = yamlio.load_raw(open(os.path.join(SRC_TESTDATA, "datafortestingtranslate", "servicesfromnodejsapp.yaml")).read())
    services = [plantypes.Service.from_yaml(d) for d in data]
    want = yamlio.load(open(os.path.join(SRC_TESTDATA, "datafortestingtranslate", "expectedirfornodejsapp.yaml")).read())
    ir = Any2KubeTranslator().translate(services, plantypes.new_plan())
    assert ir.name == want["name"]
    assert sorted(ir.services) == sorted(want["services"]) == ["nodejs"]
    s = ir.services["nodejs"]
    ws = want["services"]["nodejs"]
    assert s.containers == [{"name": "nodejs", "image": "nodejs:latest", "ports": [{"containerPort": 8080}]}]
    assert ws["podspec"]["containers"][0]["ports"][0]["containerport"] == 8080
    assert [(f.service_port.number, f.pod_port.number) for f in s.port_forwardings] == [(8080, 8080)]
    assert len(ir.containers) == 1
    c, wc = ir.containers[0], want["containers"][0]
    assert c.container_build_type == wc["containerbuildtype"]
    assert c.image_names == wc["imagenames"]
    assert c.new is True and c.exposed_ports == wc["exposedports"] and c.user_id == wc["userid"]
    assert sorted(c.new_files) == sorted(wc["newfiles"])
    # byte for byte, license header included
    assert c.new_files["nodejs-cnb-build.sh"] == wc["newfiles"]["nodejs-cnb-build.sh"]
    assert ir.kubernetes.artifact_type == want["kubernetes"]["artifactType"]
    assert ir.kubernetes.target_cluster_type == want["kubernetes"]["targetCluster"]["type"]
