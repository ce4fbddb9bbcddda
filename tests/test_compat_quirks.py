"""Behaviour switch for the reference's output-affecting quirks.

``M2K_COMPAT=reference`` (the default) keeps the reference's observable behaviour
so that manifests and QA caches match it; ``M2K_COMPAT=fixed`` applies the bug
fix.  Each test pins both sides of one numbered quirk.  Crash/hang quirks are
fixed in both modes and are pinned by their own tests (``test_qa_engines_io.py``
for #12, ``test_collectors.py`` for #8)."""

import os

import pytest

import logparse

from move2kube_amd.apiresourceset import KnativeAPIResourceSet
from move2kube_amd.collector import images
from move2kube_amd.containerizer.base import ContainerizerError, Containerizers
from move2kube_amd.models import plan as plantypes
from move2kube_amd.models import qa
from move2kube_amd.source.compose import v3
from move2kube_amd.utils.constants import settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUBS = os.path.join(ROOT, "tests", "fixtures", "stubbin")

MODES = ["reference", "fixed"]

KSVC = """apiVersion: serving.knative.dev/v1
kind: Service
metadata:
  name: hello
spec:
  template:
    spec:
      containers:
        - image: gcr.io/knative-samples/helloworld-go
"""


@pytest.fixture(params=MODES)
def mode(request, monkeypatch):
    monkeypatch.setattr(settings, "compat", request.param)
    return request.param


def test_default_mode_is_reference(monkeypatch):
    monkeypatch.delenv("M2K_COMPAT", raising=False)
    from move2kube_amd.utils.constants import _Settings
    assert _Settings().compat == "reference" and not _Settings().fixed


def test_q1_knative_services_discovered_only_when_fixed(tmp_path, mode):
    (tmp_path / "ksvc.yaml").write_text(KSVC)
    (tmp_path / "other.yaml").write_text("apiVersion: v1\nkind: ConfigMap\nmetadata:\n  name: c\n")
    p = plantypes.new_plan()
    p.root_dir = str(tmp_path)
    services = KnativeAPIResourceSet().get_service_options(str(tmp_path), p)
    if mode == "reference":
        assert services == []  # inverted type check: real Knative services are skipped
    else:
        assert [s.service_name for s in services] == ["hello"]
        assert services[0].source_artifacts[plantypes.KNATIVE_FILE_ARTIFACT] == [str(tmp_path / "ksvc.yaml")]


def test_q6_compose_v3_zero_value_storages(tmp_path, mode):
    (tmp_path / "s.txt").write_text("s3cret\n")
    (tmp_path / "docker-compose.yaml").write_text(
        'version: "3.7"\nservices:\n  web:\n    image: nginx\n    secrets: [db]\n'
        'secrets:\n  db:\n    file: ./s.txt\n')
    p = plantypes.new_plan()
    p.root_dir = str(tmp_path)
    ir = v3.V3Loader().convert_to_ir(str(tmp_path / "docker-compose.yaml"), p,
                                     plantypes.Service("web", plantypes.COMPOSE2KUBE))
    names = [s.name for s in ir.storages]
    if mode == "reference":
        assert names == ["", "db"]  # make([]Storage, n) then append
    else:
        assert names == ["db"]


def test_q9_image_names_collected_only_when_fixed(monkeypatch, mode):
    monkeypatch.setenv("PATH", STUBS + os.pathsep + "/usr/bin:/bin")
    got = images.get_all_image_names()
    assert got == ([] if mode == "reference" else ["app/web:1.0"])  # "<none>" entries always dropped


def test_q10_cache_merge_duplicates(mode):
    def cache(answer):
        c = qa.Cache("c.yaml")
        p = qa.new_input_problem("Enter the name", [], "")
        p.set_answer([answer])
        c.problems.append(p)
        return c

    a = cache("first")
    a._merge(cache("second"))
    answers = [p.answer[0] for p in a.problems]
    assert answers == (["first", "second"] if mode == "reference" else ["first"])
    # either way the first answer is the one replayed
    q = qa.new_input_problem("Enter the name", [], "")
    assert a.get_solution(q).answer == ["first"]


def test_q15_manual_containerization_dispatch(tmp_path, mode):
    cz = Containerizers()  # registry without Manual, as in the reference
    s = plantypes.Service("app", plantypes.CFMANIFEST2KUBE)
    s.container_build_type = plantypes.MANUAL
    s.image = "app:latest"
    if mode == "reference":
        with pytest.raises(ContainerizerError):
            cz.get_container(plantypes.new_plan(), s)
    else:
        c = cz.get_container(plantypes.new_plan(), s)
        assert c.image_names == ["app:latest"] and c.new


def test_q5_cf_app_path_joined_onto_manifest_file(tmp_path, mode, monkeypatch):
    from move2kube_amd import assets
    from move2kube_amd.source.cfmanifest2kube import CfManifestTranslator
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    assets.setup()
    app = tmp_path / "src" / "app"
    app.mkdir(parents=True)
    (app / "package.json").write_text('{"name": "web", "scripts": {"start": "node index.js"}}\n')
    (tmp_path / "src" / "manifest.yml").write_text("applications:\n- name: web\n  path: app\n")
    p = plantypes.new_plan()
    p.root_dir = str(tmp_path / "src")
    services = CfManifestTranslator().get_service_options(str(tmp_path / "src"), p)
    dockerfile = [s for s in services if s.container_build_type == plantypes.NEW_DOCKERFILE]
    if mode == "reference":
        # <manifest.yml>/app does not exist, so the nodejs detector never sees the app
        assert dockerfile == []
    else:
        assert [s.service_name for s in dockerfile] == ["web"]


def _translate(tmp_path, monkeypatch, files, name="q", curate=True, qacaches=(), ignore_env=True):
    import shutil
    from move2kube_amd import api
    from move2kube_amd.utils import yamlio
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = tmp_path / "src"
    src.mkdir()
    for rel, text in files.items():
        if text is None:
            shutil.copytree(os.path.join(ROOT, "samples", rel), str(src / rel))
        else:
            (src / rel).parent.mkdir(parents=True, exist_ok=True)
            (src / rel).write_text(text)
    with api.Session(qaskip=True, qacaches=qacaches, ignore_env=ignore_env) as session:
        # curate=False keeps the planner's choices (the curator's default cluster is Kubernetes)
        out = session.translate(str(src), str(tmp_path / "out"), name=name, curate=curate)
    objdir = os.path.join(out, name)
    return {f: yamlio.load(open(os.path.join(objdir, f)).read()) for f in sorted(os.listdir(objdir))}


CLUSTER_WITHOUT_HPA = """apiVersion: move2kube.konveyor.io/v1alpha1
kind: ClusterMetadata
metadata:
  name: nohpa
spec:
  storageClasses: [default]
  apiKindVersionMap:
    Deployment: [apps/v1]
    Service: [v1]
    Secret: [v1]
    PersistentVolumeClaim: [v1]
"""

HPA = ("apiVersion: autoscaling/v1\nkind: HorizontalPodAutoscaler\nmetadata:\n  name: web\nspec:\n"
       "  maxReplicas: 3\n  scaleTargetRef:\n    apiVersion: apps/v1\n    kind: Deployment\n    name: nodejs\n")


def test_q3_unsupported_kinds_written_unless_fixed(tmp_path, mode, monkeypatch):
    objs = _translate(tmp_path, monkeypatch, {"nodejs": None, "k8s/hpa.yaml": HPA,
                                             "cluster/nohpa.yaml": CLUSTER_WITHOUT_HPA},
                      curate=False)
    assert "nodejs-deployment.yaml" in objs and "nodejs-service.yaml" in objs
    # the K8s transformer never copies IgnoreUnsupportedKinds from the IR in the reference
    assert ("web-horizontalpodautoscaler.yaml" in objs) == (mode == "reference")


COMPOSE_TWO_VOLUMES = """version: "3.7"
services:
  db:
    image: postgres:13
    volumes:
      - data1:/var/lib/a
      - data2:/var/lib/b
volumes:
  data1: {}
  data2: {}
"""


def test_q4_storage_class_for_all_claims(tmp_path, mode, monkeypatch):
    objs = _translate(tmp_path, monkeypatch, {"docker-compose.yaml": COMPOSE_TWO_VOLUMES})
    pvcs = {f: o for f, o in objs.items() if o.get("kind") == "PersistentVolumeClaim"}
    assert sorted(pvcs) == ["data1-persistentvolumeclaim.yaml", "data2-persistentvolumeclaim.yaml"]
    classes = [o["spec"].get("storageClassName") for o in pvcs.values()]
    # one class chosen for all claims is assigned to a loop copy in the reference
    assert classes == ([None, None] if mode == "reference" else ["default", "default"])


Q13_LOGIN_FROM_CONFIG = """apiVersion: move2kube.konveyor.io/v1alpha1
kind: QACache
spec:
  solutions:
    - description: '[quay.io] What type of container registry login do you want to use?'
      solution:
        type: Select
        answer:
          - Docker login from config
      resolved: true
"""


def _q13(tmp_path, monkeypatch, caches=()):
    import base64
    import json
    cfg = tmp_path / "dockercfg"
    cfg.mkdir()
    (cfg / "config.json").write_text(json.dumps(
        {"auths": {"quay.io": {"auth": base64.b64encode(b"u:p").decode()}}}))
    monkeypatch.setenv("DOCKER_CONFIG", str(cfg))
    monkeypatch.setenv("HOME", str(tmp_path))
    return _translate(tmp_path, monkeypatch, {"docker-compose.yaml":
                                              'version: "3.7"\nservices:\n  web:\n    image: quay.io/org/web:1\n'},
                      qacaches=caches, ignore_env=False)


def _pull_secret_refs_resolve(objs):
    """Every imagePullSecrets entry names a Secret that is written."""
    secrets = {o["metadata"]["name"]: o for o in objs.values() if o.get("kind") == "Secret"}
    refs = []
    for o in objs.values():
        pod = ((o.get("spec") or {}).get("template") or {}).get("spec") or {}
        refs += [e["name"] for e in pod.get("imagePullSecrets", [])]
    return refs, secrets


def test_q13_no_authentication_leaves_no_dangling_pull_secret(tmp_path, mode, monkeypatch):
    """Default answer "No authentication": no Secret, and (fixed) no reference to one."""
    objs = _q13(tmp_path, monkeypatch)
    refs, secrets = _pull_secret_refs_resolve(objs)
    assert refs == [] and secrets == {}


def test_q13_login_from_config_keyed_by_image_registry(tmp_path, mode, monkeypatch):
    """A docker-config login for quay.io, chosen through a QA cache.  The
    reference looks the auth up by the target RegistryURL (docker.io), so the
    option is not offered for quay.io and nothing is emitted; "fixed" emits a
    Secret whose .dockerconfigjson is keyed by quay.io and references it."""
    import base64
    import json
    cache = tmp_path / "q13cache.yaml"
    cache.write_text(Q13_LOGIN_FROM_CONFIG)
    objs = _q13(tmp_path, monkeypatch, caches=[str(cache)])
    refs, secrets = _pull_secret_refs_resolve(objs)
    if mode == "reference":
        assert refs == [] and secrets == {}
        return
    assert len(refs) == 1 and "quay" in refs[0]
    assert set(refs) <= set(secrets)
    sec = secrets[refs[0]]
    assert sec["type"] == "kubernetes.io/dockerconfigjson"
    cfg = json.loads(base64.b64decode(sec["data"][".dockerconfigjson"]))
    assert list(cfg["auths"]) == ["quay.io"]
    assert base64.b64decode(cfg["auths"]["quay.io"]["auth"]) == b"u:p"


def test_session_restores_ignore_environment():
    from move2kube_amd import api
    from move2kube_amd.utils.constants import settings
    before = settings.ignore_environment
    with api.Session(ignore_env=not before) as s:
        s._start()
        assert settings.ignore_environment == (not before)
    assert settings.ignore_environment == before


def test_q2_q15_manual_cf_app_and_manual_images_readme(tmp_path, mode, monkeypatch):
    from move2kube_amd import api
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = tmp_path / "src"
    (src / "app").mkdir(parents=True)
    (src / "app" / "data.bin").write_text("no detector matches this\n")
    (src / "manifest.yml").write_text("applications:\n- name: legacy\n  path: app\n")
    out = api.translate(str(src), str(tmp_path / "out"), name="q")
    readme = os.path.join(out, "Manualimages.md")
    if mode == "reference":
        # Manual is not in the containerizer registry and the readme template gets the wrong struct
        assert not os.path.exists(readme)
    else:
        assert os.path.exists(os.path.join(out, "q", "legacy-deployment.yaml"))
        assert "legacy" in open(readme).read()


def test_q2_write_containers_manual_image(tmp_path, mode, caplog):
    """Quirk #2 directly: a new container without files (a manual image).  The
    reference hands Manualimages.md the wrong struct, so the template fails,
    the error is logged and no file is written; "fixed" writes it and keeps the
    manual image out of pushimages.sh (buildimages.sh never builds it)."""
    from move2kube_amd import transformer
    from move2kube_amd.models import ir as irtypes
    from move2kube_amd.models import plan as plantypes
    manual = irtypes.new_container(plantypes.MANUAL, "legacy:latest", True)
    built = irtypes.new_container(plantypes.NEW_DOCKERFILE, "web:latest", True)
    built.new_files = {"web/Dockerfile.web": "FROM scratch\n", "web/web-docker-build.sh": "docker build .\n"}
    out = str(tmp_path / "out")
    from move2kube_amd.utils import log
    errors = []
    saved = log.error
    log.error = lambda *a, **k: errors.append(a[0] % a[1:] if len(a) > 1 else a[0])
    try:
        assert transformer.write_containers([manual, built], out, str(tmp_path), "docker.io", "ns") is True
    finally:
        log.error = saved
    readme = os.path.join(out, "Manualimages.md")
    push = open(os.path.join(out, "pushimages.sh")).read()
    assert "web:latest" in push
    if mode == "reference":
        assert not os.path.exists(readme)
        assert any("can't evaluate field Images" in e for e in errors)
        assert "legacy:latest" in push
    else:
        assert "legacy:latest" in open(readme).read()
        assert "legacy:latest" not in push


def _registry_questions(tmp_path, monkeypatch, auths):
    """The registry questions of a qaskip translate of a new nodejs image
    with ``auths`` in the docker CLI config, as recorded in m2kqacache.yaml."""
    import json
    from move2kube_amd.utils import yamlio
    cfg = tmp_path / "dockercfg"
    cfg.mkdir()
    (cfg / "config.json").write_text(json.dumps({"auths": auths}))
    monkeypatch.setenv("DOCKER_CONFIG", str(cfg))
    monkeypatch.setenv("HOME", str(tmp_path))
    _translate(tmp_path, monkeypatch, {"nodejs": None}, ignore_env=False)
    cache = yamlio.load(open(os.path.join(str(tmp_path / "out"), "q", "m2kqacache.yaml")).read())
    return {s["description"]: s["solution"] for s in cache["spec"]["solutions"]}


def test_docker_config_auths_are_cleared_by_the_loader(tmp_path, mode, monkeypatch):
    """dockercliconfig.Load decodes each auth and clears it (LoadFromReader),
    so the reference lists the config's registries but never offers the
    docker-config login and keeps docker.io as the default registry; "fixed"
    keeps the auth: the login is offered and its registry is the default."""
    import base64
    good = base64.b64encode(b"user:pw").decode()
    qs = _registry_questions(tmp_path, monkeypatch, {"https://user@quay.io/v1/": {"auth": good},
                                                     "registry.example.com": {}})
    reg = qs["Select the registry where your images are hosted:"]
    assert reg["options"] == ["Other", "quay.io", "registry.example.com", "docker.io"]
    if mode == "reference":
        assert reg["default"] == ["docker.io"] and reg["answer"] == ["docker.io"]
        login = qs["[docker.io] What type of container registry login do you want to use?"]
        assert "Docker login from config" not in login["options"]
    else:
        assert reg["default"] == ["quay.io"] and reg["answer"] == ["quay.io"]
        login = qs["[quay.io] What type of container registry login do you want to use?"]
        assert login["options"][-1] == "Docker login from config"


def test_an_undecodable_docker_config_auth_drops_the_whole_config(tmp_path, monkeypatch):
    """decodeAuth fails (not base64, or no ':'): Load returns the error and the
    reference uses nothing of the file."""
    qs = _registry_questions(tmp_path, monkeypatch, {"quay.io": {"auth": "bm9jb2xvbg=="},   # "nocolon"
                                                     "other.io": {}})
    assert qs["Select the registry where your images are hosted:"]["options"] == ["Other", "docker.io"]


def test_q1_fixed_mode_translates_a_knative_service(tmp_path, monkeypatch):
    """With the type check fixed, a Knative service goes through
    ``KnativeAPIResourceSet.Translate``: its revision template's pod spec
    (container concurrency and timeout dropped) becomes the service's."""
    monkeypatch.setattr(settings, "compat", "fixed")
    ksvc = KSVC.replace("    spec:\n", "    spec:\n      containerConcurrency: 4\n      timeoutSeconds: 30\n")
    objs = _translate(tmp_path, monkeypatch, {"ksvc.yaml": ksvc}, name="k")
    dep = objs["hello-deployment.yaml"]
    spec = dep["spec"]["template"]["spec"]
    assert spec["containers"][0]["image"] == "gcr.io/knative-samples/helloworld-go"
    assert "containerConcurrency" not in spec and "timeoutSeconds" not in spec


def test_q1_knative_translate_skips_what_it_cannot_use(tmp_path, capsys):
    """KnativeAPIResourceSet.Translate: a service without a file, an
    unreadable file, one that no longer decodes, and another kind, each with
    the reference's log line; the rest are translated."""
    from move2kube_amd.utils import log
    log.set_verbose(False)
    good = tmp_path / "good.yaml"
    good.write_text(KSVC)
    bad = tmp_path / "bad.yaml"
    bad.write_text("kind: [\n")
    cfg = tmp_path / "cfg.yaml"
    cfg.write_text("apiVersion: serving.knative.dev/v1\nkind: Configuration\nmetadata:\n  name: c\n")
    p = plantypes.new_plan()
    p.root_dir = str(tmp_path)
    svcs = []
    for name, path in (("nofile", None), ("gone", tmp_path / "gone.yaml"), ("bad", bad), ("cfg", cfg),
                       ("hello", good)):
        s = plantypes.Service(name)
        if path is not None:
            s.source_artifacts[plantypes.KNATIVE_FILE_ARTIFACT] = [str(path)]
        svcs.append(s)
    ir = KnativeAPIResourceSet().translate(svcs, p)
    assert list(ir.services) == ["hello"]
    err = capsys.readouterr().err
    assert logparse.logged(err, "No knative artifacts found in service nofile", "warning")
    assert logparse.logged_containing(err, 'Unable to read the knative file at path "%s"' % (tmp_path / "gone.yaml"),
                                      "error")
    assert logparse.logged_containing(err, 'Failed to decode the knative file at path "%s"' % bad, "error")
    assert logparse.logged(err, 'The knative file at path "%s" does not contain the required type. Expected: '
                                '*v1.Service Actual: *v1.Configuration' % cfg, "error")
