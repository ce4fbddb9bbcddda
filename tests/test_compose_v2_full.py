"""Compose v1/v2 feature coverage (reference ``internal/source/compose/v1v2.go:140-470``):
container name lower-casing, entrypoint/command, ``k=v`` / ``k:v`` / bare env,
``[ip:]svc:pod[/proto]`` ports plus expose, privileged, non-numeric user
(ignored), capabilities, group_add (never attached in the reference),
stop_grace_period, mem_limit, unless-stopped, networks (libcompose real
names), tmpfs, bind volumes (hostPath ``vol<fnv64a>``, read-only) and named
volumes (PVC + RWX/ROX storage; libcompose prefixes top-level declared ones
with the project name)."""

import os
import shutil

from move2kube_amd import api
from move2kube_amd.utils import common, yamlio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "compose_v2_full")


def test_compose_v2_full(tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = str(tmp_path / "proj")
    shutil.copytree(FIXTURE, src)
    out = os.path.join(api.translate(src, str(tmp_path / "out"), name="v2"), "v2")
    objs = {f: yamlio.load(open(os.path.join(out, f)).read()) for f in os.listdir(out)}
    dep = objs["app-deployment.yaml"]
    meta = dep["metadata"]
    assert meta["annotations"]["role"] == "main" and "role" not in meta["labels"]
    assert meta["labels"]["move2kube.konveyor.io/network/proj_backend"] == "true"
    pod = dep["spec"]["template"]["spec"]
    assert pod["hostname"] == "apphost" and pod["subdomain"] == "example.com"
    assert pod["terminationGracePeriodSeconds"] == 90
    assert pod["restartPolicy"] == "Always"
    assert "securityContext" not in pod            # group_add is dropped, as in the reference
    (c,) = pod["containers"]
    assert c["name"] == "app-main"
    assert c["command"] == ["/start.sh"] and c["args"] == ["serve", "--port", "80"]
    assert c["env"] == [{"name": "A", "value": "1"}, {"name": "B", "value": "2"},
                        {"name": "BROKEN", "value": "unknown"}]
    assert c["workingDir"] == "/work" and c["stdin"] is True and c["tty"] is True
    assert c["securityContext"] == {"capabilities": {"add": ["SYS_TIME"]}, "privileged": True}
    assert c["resources"] == {"limits": {"memory": "268435456"}}
    assert [(p["containerPort"], p["protocol"]) for p in c["ports"]] == [(8001, "TCP"), (90, "UDP"), (3000, "TCP"),
                                                                        (4000, "TCP")]
    logs = os.path.join(src, "logs")
    vol = "vol%d" % common.fnv64a(logs.encode())
    assert c["volumeMounts"] == [
        {"mountPath": "/scratch", "name": "app-tmpfs-0"},
        {"mountPath": "/var/log/app", "name": vol, "readOnly": True},
        {"mountPath": "/data", "name": "proj_appdata"},
        {"mountPath": "/shared", "name": "proj_shared", "readOnly": True},
    ]
    assert pod["volumes"] == [
        {"emptyDir": {"medium": "Memory"}, "name": "app-tmpfs-0"},
        {"hostPath": {"path": logs}, "name": vol},
        {"name": "proj_appdata", "persistentVolumeClaim": {"claimName": "proj_appdata"}},
        {"name": "proj_shared", "persistentVolumeClaim": {"claimName": "proj_shared", "readOnly": True}},
    ]
    svc = objs["app-service.yaml"]
    assert [(p["port"], p["targetPort"]) for p in svc["spec"]["ports"]] == [(8001, 8001), (9000, 90), (3000, 3000),
                                                                           (4000, 4000)]
    # named volumes declared at the top level get libcompose's project prefix
    assert objs["proj_appdata-persistentvolumeclaim.yaml"]["spec"]["accessModes"] == ["ReadWriteMany"]
    assert objs["proj_shared-persistentvolumeclaim.yaml"]["spec"]["accessModes"] == ["ReadOnlyMany"]
    assert objs["proj_backend-networkpolicy.yaml"]["metadata"]["name"] == "proj_backend"


def test_compose_v2_unsupported_minor_version_is_skipped(tmp_path, monkeypatch):
    # libcompose accepts 2, 2.0 and 2.1 only; docker/cli's v3 loader rejects 2.x:
    # a 2.4 file yields no services
    from move2kube_amd.source.compose2kube import ComposeTranslator
    from move2kube_amd.models import plan as plantypes
    d = tmp_path / "x"
    d.mkdir()
    (d / "docker-compose.yml").write_text('version: "2.4"\nservices:\n  a:\n    image: busybox\n')
    p = plantypes.new_plan()
    p.root_dir = str(d)
    assert ComposeTranslator().get_service_options(str(d), p) == []


# ---------------------------------------------------------------------------
# libcompose env_file folding and extends (v1v2.go:93-129 -> project.Parse)
# ---------------------------------------------------------------------------

def _write(root, files):
    for rel, text in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)


def _v2_services(root, name="docker-compose.yml"):
    from move2kube_amd.source.compose.v1v2 import parse_v2
    return {s["name"]: s for s in parse_v2(os.path.join(root, name))["services"]}


def _translate_env(tmp_path, files, svc):
    src = str(tmp_path / "proj")
    _write(src, files)
    out = os.path.join(api.translate(src, str(tmp_path / "out"), name="p"), "p")
    dep = yamlio.load(open(os.path.join(out, "%s-deployment.yaml" % svc)).read())
    return dep["spec"]["template"]["spec"]["containers"][0]


def test_v2_env_file_merged_into_environment(tmp_path):
    """The verdict's reproduction: env_file A=1, B=two plus environment [C=3]
    yields C, A, B (explicit entries first, then file lines)."""
    c = _translate_env(tmp_path, {
        "docker-compose.yml": 'version: "2"\nservices:\n  web:\n    image: nginx\n    env_file: app.env\n'
                              '    environment:\n      - C=3\n',
        "app.env": "A=1\nB=two\n"}, "web")
    assert c["env"] == [{"name": "C", "value": "3"}, {"name": "A", "value": "1"}, {"name": "B", "value": "two"}]


def test_v2_env_file_precedence_and_format(tmp_path):
    """Explicit environment wins over files; of two files the later wins (files
    are read last to first); comments/blank lines skipped; lines are verbatim;
    a key is "already set" when an entry starts with ``KEY=``."""
    root = str(tmp_path)
    _write(root, {
        "docker-compose.yml": 'version: "2.1"\nservices:\n  s:\n    image: x\n'
                              '    env_file: [one.env, two.env, missing.env]\n'
                              '    environment:\n      A: explicit\n      AB: 7\n',
        "one.env": "# comment\n\nA=from-one\nB=from-one\nC=from-one\n  D = spaced \nBARE\n",
        "two.env": "B=from-two\nE=\"quoted\"\n"})
    env = _v2_services(root)["s"]["environment"]
    assert env == ["A=explicit", "AB=7", "B=from-two", 'E="quoted"', "C=from-one", "D = spaced", "BARE"]


def test_v2_env_file_string_and_missing(tmp_path):
    root = str(tmp_path)
    _write(root, {"docker-compose.yml": 'version: "2"\nservices:\n  s:\n    image: x\n    env_file: nope.env\n'})
    assert _v2_services(root)["s"]["environment"] == []


def test_v1_env_file(tmp_path):
    root = str(tmp_path)
    _write(root, {"docker-compose.yml": "web:\n  image: x\n  env_file: ./conf/web.env\n  environment:\n    - K=1\n",
                  "conf/web.env": "K=2\nL=3\n"})
    assert _v2_services(root)["web"]["environment"] == ["K=1", "L=3"]


def test_v2_extends_other_file(tmp_path):
    """The verdict's reproduction: web extends base in common.yml (image
    nginx:1.19, port 80) -> image and port come from base."""
    c = _translate_env(tmp_path, {
        "docker-compose.yml": 'version: "2"\nservices:\n  web:\n    extends:\n      file: common.yml\n'
                              '      service: base\n',
        "common.yml": 'version: "2"\nservices:\n  base:\n    image: nginx:1.19\n    ports:\n      - "80:80"\n'}, "web")
    assert c["image"] == "nginx:1.19"
    assert [p["containerPort"] for p in c["ports"]] == [80]


def test_v2_extends_merge_rules_and_chain(tmp_path):
    """Chained extends (same file, then another file): scalars replaced, lists
    appended, maps merged; inherited build contexts and bind sources resolve
    against the file that declared them."""
    root = str(tmp_path)
    _write(root, {
        "docker-compose.yml": 'version: "2"\nservices:\n'
                              '  app:\n    extends: {service: mid}\n    image: app:2\n    ports: ["9000"]\n'
                              '    labels: {tier: app}\n    environment: [X=app]\n'
                              '  mid:\n    extends: {file: lib/base.yml, service: base}\n    ports: ["8000"]\n'
                              '    labels: {team: core}\n',
        "lib/base.yml": 'version: "2"\nservices:\n  base:\n    image: base:1\n    build: ./ctx\n'
                        '    ports: ["7000"]\n    volumes: ["./data:/data"]\n    labels: {tier: base}\n'
                        '    environment: [X=base, Y=base]\n',
    })
    svcs = _v2_services(root)
    app = svcs["app"]
    assert app["image"] == "app:2"
    assert app["ports"] == ["7000", "8000", "9000"]
    assert app["labels"] == {"tier": "app", "team": "core"}
    assert app["environment"] == ["X=base", "Y=base", "X=app"]
    assert app["build_context"] == os.path.join(root, "lib", "ctx")
    assert app["volumes"][0]["source"] == os.path.join(root, "lib", "data")
    assert svcs["mid"]["image"] == "base:1" and svcs["mid"]["ports"] == ["7000", "8000"]


def test_v2_extends_env_file_slice_is_replaced(tmp_path):
    """After env_file folding ``environment`` is a typed slice
    (MaporEqualSlice), which libcompose's merge does not append: the child's
    environment replaces the base's."""
    root = str(tmp_path)
    _write(root, {
        "docker-compose.yml": 'version: "2"\nservices:\n  base:\n    image: b\n    env_file: b.env\n'
                              '  child:\n    extends: {service: base}\n    environment: [C=1]\n',
        "b.env": "B=1\n"})
    svcs = _v2_services(root)
    assert svcs["base"]["environment"] == ["B=1"]
    assert svcs["child"]["environment"] == ["C=1"]


def test_v2_extends_errors(tmp_path):
    import pytest
    from move2kube_amd.source.compose.v3 import ComposeError
    root = str(tmp_path)
    _write(root, {"docker-compose.yml": 'version: "2"\nservices:\n  a:\n    image: x\n    extends: {service: nope}\n'})
    with pytest.raises(ComposeError, match="Failed to find service nope"):
        _v2_services(root)
    _write(root, {"docker-compose.yml": 'version: "2"\nservices:\n  a:\n    image: ia\n    links: [b]\n'
                                        '  b:\n    image: ib\n    extends: {service: a}\n'})
    with pytest.raises(ComposeError, match="cannot be extended"):
        _v2_services(root)
    _write(root, {"docker-compose.yml": 'version: "2"\nservices:\n  a:\n    image: ia\n    extends: {service: b}\n'
                                        '  b:\n    image: ib\n    extends: {service: a}\n'})
    with pytest.raises(ComposeError, match="circular"):
        _v2_services(root)


def test_v2_extends_build_context_plans_reuse_dockerfile(tmp_path):
    """The planner sees the merged service: an inherited ``build`` yields the
    ReuseDockerfile option with the base file's context."""
    from move2kube_amd.source.compose2kube import ComposeTranslator
    from move2kube_amd.models import plan as plantypes
    root = str(tmp_path)
    _write(root, {"docker-compose.yml": 'version: "2"\nservices:\n  web:\n    extends: {file: sub/c.yml, service: b}\n',
                  "sub/c.yml": 'version: "2"\nservices:\n  b:\n    build: ./app\n',
                  "sub/app/Dockerfile": "FROM scratch\n"})
    p = plantypes.new_plan()
    p.root_dir = root
    opts = ComposeTranslator().get_service_options(root, p)
    # sub/c.yml is a compose file of its own too (service b); look at web
    reuse_df = [o for o in opts if o.container_build_type == plantypes.REUSE_DOCKERFILE and o.service_name == "web"]
    assert len(reuse_df) == 1
    assert reuse_df[0].target_options == [os.path.join(root, "sub", "app", "Dockerfile")]


def test_v2_named_volume_names(tmp_path, monkeypatch):
    """handleVolumeConfig: declared with a body -> <project>_<name>; external
    with a name -> that name; external without, bare declaration, or not
    declared -> unchanged.  COMPOSE_PROJECT_NAME overrides the directory name."""
    root = str(tmp_path / "My-App")
    _write(root, {"docker-compose.yml": 'version: "2"\nservices:\n  s:\n    image: x\n    volumes:\n'
                                        '      - a:/a\n      - b:/b\n      - c:/c\n      - d:/d\n      - e:/e\n'
                                        '      - ./f:/f\n'
                                        'volumes:\n  a: {driver: local}\n  b:\n    external:\n      name: real-b\n'
                                        '  c: {external: true}\n  d:\n'})
    srcs = [v["source"] for v in _v2_services(root)["s"]["volumes"]]
    assert srcs == ["myapp_a", "real-b", "c", "d", "e", os.path.join(root, "f")]
    monkeypatch.setenv("COMPOSE_PROJECT_NAME", "Other_Name")
    assert _v2_services(root)["s"]["volumes"][0]["source"] == "othername_a"


def test_v2_group_names_and_negative_grace_period(tmp_path, monkeypatch, capsys):
    """getGroupAdd's cast error, wrapped (v1v2.go:448-459), is the warning
    text; durationInSeconds truncates toward zero as int64(d.Seconds()) does."""
    import logparse
    from move2kube_amd.models import plan as plantypes
    from move2kube_amd.source.compose.v1v2 import V1V2Loader
    from move2kube_amd.utils import log
    monkeypatch.chdir(tmp_path)
    p = tmp_path / "docker-compose.yml"
    p.write_text('version: "2"\nservices:\n  web:\n    image: nginx\n    group_add: ["100", "wheel"]\n'
                 '    stop_grace_period: -1500ms\n')
    plan = plantypes.new_plan()
    plan.root_dir = str(tmp_path)
    svc = plantypes.Service.new("web", plantypes.COMPOSE2KUBE)
    log.set_verbose(False)
    ir = V1V2Loader().convert_to_ir(str(p), plan, svc)
    assert ir.services["web"].pod_spec["terminationGracePeriodSeconds"] == -1
    assert logparse.logged(capsys.readouterr().err, 'GroupAdd should be in gid format, not as group name : unable to '
                           'get group_add: unable to cast "wheel" of type string to int', "warning")
