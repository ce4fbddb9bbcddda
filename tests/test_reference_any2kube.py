"""``internal/source/any2kube_test.go``, one pytest per Go subtest, comparing
whole service lists and whole IRs as the Go test does."""

import base64
import os
import shutil

import pytest

from conftest import ref_path
from goequal import assert_deep_equal
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source.any2kube import Any2KubeTranslator
from move2kube_amd.utils import tarutil, yamlio

pytestmark = pytest.mark.reference

SRC_TESTDATA = ref_path("internal", "source", "testdata")


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


# --- TestGetServiceOptions ------------------------------------------------------------

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
    assert_deep_equal(got, want)


def test_nodejs_app_filled_plan(layout):
    """Services of the plan whose source directories lie elsewhere do not hide the app."""
    root = os.path.abspath("../../samples/nodejs")
    p = _plan_for(root)
    svc1 = plantypes.Service.new("svc1", "Any2Kube")
    svc1.source_artifacts[plantypes.SOURCE_DIRECTORY_ARTIFACT] = ["foo/"]
    svc2 = plantypes.Service.new("svc2", "Any2Kube")
    svc2.source_artifacts[plantypes.SOURCE_DIRECTORY_ARTIFACT] = ["bar/"]
    p.services = {"svc1": [svc1], "svc2": [svc2]}
    want = plantypes.read_plan("testdata/expectedservicesfornodejsapp.yaml").services["nodejs"]
    got = _strip_repo(Any2KubeTranslator().get_service_options(root, p))
    assert_deep_equal(got, want)


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
    assert_deep_equal(got, want)


def test_m2kignore_everything_but_one_subdir(layout):
    root = os.path.abspath("testdata/javamavenappwithm2kignorecase2")
    want = plantypes.read_plan("testdata/expectedservicesforjavamavenappwithm2kignorecase2.yaml").services["java-maven"]
    got = _strip_repo(Any2KubeTranslator().get_service_options(root, _plan_for(root, "java-maven-app")))
    assert_deep_equal(got, want)


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


# --- TestTranslate -----------------------------------------------------------------------

def test_translate_no_services(assets_dir):
    p = plantypes.new_plan()
    assert_deep_equal(Any2KubeTranslator().translate([], p), irtypes.new_ir(p))


_GO_K8S_KEYS = {"containers": "containers", "name": "name", "image": "image", "ports": "ports",
                "containerport": "containerPort"}


def _go_yaml_k8s(v):
    """A k8s struct as go-yaml fills it: keys are lowercased Go field names;
    here they go back to the object's JSON names."""
    if isinstance(v, dict):
        return {_GO_K8S_KEYS[k]: _go_yaml_k8s(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_go_yaml_k8s(x) for x in v]
    return v


def _go_yaml_ir(d):
    """irtypes.IR as common.ReadYaml fills it from expectedirfornodejsapp.yaml
    (fields the file leaves out are zero: NewIR's empty values, EquateEmpty)."""
    ir = irtypes.new_ir(plantypes.new_plan())
    ir.name = d["name"]
    for name, sd in d["services"].items():
        s = irtypes.Service(sd["name"])
        s.pod_spec = _go_yaml_k8s(sd["podspec"])
        s.port_forwardings = [irtypes.PortForwarding(irtypes.Port(f["serviceport"]["number"]),
                                                     irtypes.Port(f["podport"]["number"]))
                              for f in sd["servicetopodportforwardings"]]
        ir.services[name] = s
    for cd in d["containers"]:
        c = irtypes.Container(cd["containerbuildtype"], "", cd["new"])
        c.image_names = cd["imagenames"]
        c.new_files = cd["newfiles"]
        c.exposed_ports = cd["exposedports"]
        c.user_id = cd["userid"]
        ir.containers.append(c)
    ir.kubernetes = plantypes.KubernetesOutput.from_yaml(d["kubernetes"])
    return ir


def test_translate_nodejs_services_to_ir():
    td = os.path.join(SRC_TESTDATA, "datafortestingtranslate")
    data = yamlio.load_raw(open(os.path.join(td, "servicesfromnodejsapp.yaml")).read())
    services = [plantypes.Service.from_yaml(d) for d in data]
    want = _go_yaml_ir(yamlio.load(open(os.path.join(td, "expectedirfornodejsapp.yaml")).read()))
    assert_deep_equal(Any2KubeTranslator().translate(services, plantypes.new_plan()), want)
