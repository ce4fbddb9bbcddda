"""Collectors against stub kubectl / docker / cf executables on PATH."""

import os

import pytest

from move2kube_amd import collector
from move2kube_amd.collector import cf as cfc
from move2kube_amd.collector.cluster import ClusterCollector
from move2kube_amd.collector.images import ImagesCollector, get_image_info
from move2kube_amd.utils import yamlio
from move2kube_amd.utils.constants import settings

STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "stubbin")


@pytest.fixture
def stub_path(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", STUBS + os.pathsep + "/usr/bin:/bin")
    return tmp_path


def _read(path):
    return yamlio.load(open(path).read())


def test_cluster_collector_via_discovery(stub_path):
    out = stub_path / "out"
    ClusterCollector().collect("", str(out))
    files = os.listdir(str(out / "clusters"))
    assert len(files) == 1
    d = _read(str(out / "clusters" / files[0]))
    assert d["kind"] == "ClusterMetadata"
    assert d["metadata"]["name"] == "test-ctx\n"  # the reference keeps kubectl's newline
    assert d["spec"]["storageClasses"] == ["gold", "silver"]
    m = d["spec"]["apiKindVersionMap"]
    assert m["Deployment"] == ["apps/v1", "extensions/v1beta1"]
    assert m["Ingress"] == ["networking.k8s.io/v1", "networking.k8s.io/v1beta1", "extensions/v1beta1"]
    assert m["Route"] == ["route.openshift.io/v1"]
    assert m["Pod"] == ["v1"] and m["Service"] == ["v1"]


def test_cluster_collector_fixed_mode_strips_context(stub_path):
    settings.compat = "fixed"
    ClusterCollector().collect("", str(stub_path / "o"))
    assert os.listdir(str(stub_path / "o" / "clusters"))[0].startswith("test-ctx")


def test_cluster_collector_without_cli(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", str(tmp_path))
    with pytest.raises(RuntimeError):
        ClusterCollector().collect("", str(tmp_path / "o"))


def test_group_order_policy():
    kinds = {"K": ["v1", "zzz.example.com/v1", "apps/v1", "extensions/v1beta1", "x.k8s.io/v1", "a.openshift.io/v1"]}
    ClusterCollector().group_order_policy(kinds)
    assert kinds["K"] == ["a.openshift.io/v1", "x.k8s.io/v1", "apps/v1", "extensions/v1beta1", "zzz.example.com/v1", "v1"]


def test_image_info_parsing():
    info = get_image_info(b'[{"RepoTags":["a:1"],"ContainerConfig":{"ExposedPorts":{"80/tcp":{}},"User":"root","WorkingDir":"/w"}}]')
    assert info.tags == ["a:1"] and info.ports == [80] and info.user_id == -1 and info.accessed_dirs == ["/w"]


def test_images_collector_from_compose(stub_path):
    src = stub_path / "src"
    src.mkdir()
    (src / "docker-compose.yml").write_text("version: '3'\nservices:\n  web:\n    image: app/web:1.0\n  cache:\n    image: redis:6\n")
    ImagesCollector().collect(str(src), str(stub_path / "out"))
    files = os.listdir(str(stub_path / "out" / "images"))
    assert len(files) == 1 and files[0].startswith("web-latest")
    d = _read(str(stub_path / "out" / "images" / files[0]))
    assert d["kind"] == "ImageMetadata"
    assert d["spec"]["ports"] == [443, 8080] and d["spec"]["userID"] == 1001


def test_cf_apps_collector(stub_path):
    cfc.CfAppsCollector().collect("", str(stub_path / "out"))
    files = os.listdir(str(stub_path / "out" / "cf"))
    assert len(files) == 1 and files[0].startswith("instanceapps-ap")
    d = _read(str(stub_path / "out" / "cf" / files[0]))
    apps = d["spec"]["applications"]
    assert [a["name"] for a in apps] == ["app1", "app2"]
    assert apps[0]["buildpack"] == "nodejs_buildpack" and apps[0]["instances"] == 2 and apps[0]["env"] == {"K": "V"}


def test_cf_buildpack_names_from_instance(stub_path):
    # a literal "null" string is passed through like the reference does
    assert cfc.get_cf_buildpack_names("") == ["staticfile_buildpack", "nodejs_buildpack", "null", "python_buildpack"]


def test_cf_container_types_matching():
    options = {"cloudfoundry/cnb:cflinuxfs3": ["org.cloudfoundry.nodejs", "org.cloudfoundry.python"],
               "gcr.io/buildpacks/builder": ["google.nodejs.runtime", "google.go.runtime"]}
    got = cfc.get_buildpack_containerizers(["nodejs_buildpack", "go_buildpack"], options)
    assert [b.buildpack_name for b in got] == ["nodejs_buildpack", "go_buildpack"]
    assert got[1].target_options == ["gcr.io/buildpacks/builder"]


def test_collect_orchestrator_filters_by_annotation(stub_path):
    out = stub_path / "m2k_collect"
    collector.collect("", str(out), ["CF"])
    assert sorted(os.listdir(str(out))) == ["cf"]
