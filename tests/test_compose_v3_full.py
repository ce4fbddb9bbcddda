"""Compose v3 feature coverage (reference ``internal/source/compose/v3.go:135-651``)
on one file that uses every mapped key: container fields, security context,
pid/hostname/domainname, long and short ports with expose, healthcheck ->
liveness probe, deploy mode/resources/restart_policy/replicas, tmpfs,
secrets and configs (top-level storages and per-service mounts), bind and
named volumes, networks."""

import os
import shutil

import pytest

import logparse

from move2kube_amd import api
from move2kube_amd.source.compose import utils as cutils
from move2kube_amd.utils import common, yamlio
from move2kube_amd.utils.constants import settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "compose_v3_full")


def _translate(tmp_path, monkeypatch, compat):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    monkeypatch.setattr(settings, "compat", compat)
    src = str(tmp_path / "app")
    shutil.copytree(FIXTURE, src)
    out = api.translate(src, str(tmp_path / "out"), name="full")
    objs = {}
    for f in sorted(os.listdir(os.path.join(out, "full"))):
        with open(os.path.join(out, "full", f)) as fh:
            objs[f] = yamlio.load(fh.read())
    return src, out, objs


def test_reference_mode_objects(tmp_path, monkeypatch):
    src, out, objs = _translate(tmp_path, monkeypatch, "reference")
    # the reference's Deployment handler does not list DaemonSet among its kinds,
    # so a deploy.mode=global service gets no workload object (only its Service)
    assert "web-daemonset.yaml" not in objs and "web-service.yaml" in objs
    assert objs["worker-deployment.yaml"]["spec"]["replicas"] == 3
    svc = objs["web-service.yaml"]
    assert [(p["port"], p["targetPort"]) for p in svc["spec"]["ports"]] == [(8080, 80), (8443, 443), (5353, 53), (9000, 9000)]
    assert svc["metadata"]["annotations"]["tier"] == "front"
    # top-level secrets/configs -> Secret/ConfigMap objects
    assert objs["db-pass-secret.yaml"]["data"] == {"db_pass": "czNjcmV0Cg=="}
    assert "data" not in objs["api-key-secret.yaml"]          # external: no content
    assert objs["app-cfg-configmap.yaml"]["data"] == {"app_cfg": "listen=80\n"}
    assert objs["conf-dir-configmap.yaml"]["data"] == {"app.conf": "listen=80\n", "other.ini": "[x]\ny=1\n"}
    assert objs["cache-persistentvolumeclaim.yaml"]["spec"]["storageClassName"] == "default"
    np_ = objs["front-network-networkpolicy.yaml"]
    assert np_["spec"]["podSelector"]["matchLabels"] == {"move2kube.konveyor.io/network/front-network": "true"}


def test_fixed_mode_daemonset(tmp_path, monkeypatch):
    src, out, objs = _translate(tmp_path, monkeypatch, "fixed")
    ds = objs["web-daemonset.yaml"]
    assert ds["kind"] == "DaemonSet"
    pod = ds["spec"]["template"]["spec"]
    assert pod["hostPID"] is True and pod["hostname"] == "webhost" and pod["subdomain"] == "example.org"
    assert pod["restartPolicy"] == "Always"                    # unless-stopped -> Always
    (c,) = pod["containers"]
    assert c["name"] == "web-frontend"                         # container_name, lower-cased
    assert c["command"] == ["/entry.sh"] and c["args"] == ["--port", "80"]
    assert c["workingDir"] == "/srv" and c["stdin"] is True and c["tty"] is True
    assert c["env"] == [{"name": "EMPTY", "value": "unknown"}, {"name": "MODE", "value": "prod"}]
    assert c["securityContext"] == {"capabilities": {"add": ["NET_ADMIN"], "drop": ["ALL"]},
                                    "privileged": True, "runAsUser": 1000}
    assert c["livenessProbe"] == {"exec": {"command": ["curl -f http://localhost"]}, "failureThreshold": 3,
                                  "initialDelaySeconds": 40, "periodSeconds": 30, "timeoutSeconds": 10}
    # memory quantities built with an unknown format print in DecimalExponent form
    assert c["resources"] == {"limits": {"cpu": "500m", "memory": "536870912"},
                              "requests": {"cpu": "250m", "memory": "134217728"}}
    assert [(p["containerPort"], p["protocol"]) for p in c["ports"]] == [(80, "TCP"), (443, "TCP"), (53, "UDP"),
                                                                        (9000, "TCP")]
    mounts = {m["name"]: m for m in c["volumeMounts"]}
    assert mounts["web-tmpfs-0"]["mountPath"] == "/run"
    assert mounts["db_pass"]["mountPath"] == "/var/secrets/db_pass"
    assert mounts["api_key"]["mountPath"] == "/etc/keys/api"
    assert mounts["app-cfg"] == {"mountPath": "/etc/app/app.conf", "name": "app-cfg", "subPath": "app.conf"}
    assert mounts["conf-dir"] == {"mountPath": "/conf_dir", "name": "conf-dir", "subPath": "conf_dir"}
    assert mounts["cache"]["mountPath"] == "/cache"
    vols = {v["name"]: v for v in pod["volumes"]}
    assert vols["web-tmpfs-0"]["emptyDir"] == {"medium": "Memory"}
    assert vols["api_key"]["secret"] == {"defaultMode": 0o400, "items": [{"key": "api_key", "path": "api_key"}],
                                         "secretName": "api_key"}
    assert vols["app-cfg"]["configMap"] == {"defaultMode": 0o440, "items": [{"key": "app.conf", "path": "app.conf"}],
                                            "name": "app-cfg"}
    assert vols["cache"]["persistentVolumeClaim"] == {"claimName": "cache"}
    data = os.path.join(src, "data")
    host = [v for v in pod["volumes"] if "hostPath" in v]
    assert host == [{"hostPath": {"path": data}, "name": "vol%d" % common.fnv64a(data.encode())}]


@pytest.mark.parametrize("value,want", [(536870912, "536870912"), (512000000, "512e6"), (1000, "1e3"),
                                        (1500, "1500"), (0, "0")])
def test_decimal_exponent_quantities(value, want):
    assert cutils.format_quantity_decimal_exponent(value) == want


def test_compose_files_decode_with_go_yaml_v2_rules(tmp_path, monkeypatch):
    """docker/cli and libcompose parse compose files with go-yaml v2: ``yes``/``no``
    are bools, ``1e3`` is a float, ``22:22`` a string; environment mapping values
    are then rendered with fmt.Sprint."""
    from move2kube_amd.source.compose import v3
    p = tmp_path / "docker-compose.yaml"
    p.write_text("version: '3'\nservices:\n  s:\n    image: busybox\n    tty: yes\n    stdin_open: no\n"
                 "    environment:\n      A: yes\n      B: 1e3\n      C: 0777\n      D: 22:22\n      E: 1.5\n")
    parsed = yamlio.load_v2(p.read_text())
    svc = parsed["services"]["s"]
    assert svc["tty"] is True and svc["stdin_open"] is False
    env = v3._mapping_with_equals(svc["environment"])
    assert env == {"A": "true", "B": "1000", "C": "511", "D": "22:22", "E": "1.5"}


@pytest.mark.parametrize("env,where", [("Y: 1", "services.s.environment: true"),
                                       ("1: x", "services.s.environment: 1")])
def test_compose_v3_non_string_keys_fail_the_file(tmp_path, env, where):
    """docker/cli's ParseYAML rejects a document with any non-string mapping key
    (go-yaml v2 reads ``Y`` as a bool), so the v3 loader does not load it."""
    from move2kube_amd.source.compose import v3
    p = tmp_path / "docker-compose.yaml"
    p.write_text("version: '3'\nservices:\n  s:\n    image: busybox\n    environment:\n      %s\n" % env)
    with pytest.raises(v3.ComposeError, match="Non-string key in " + where.replace(".", "\\.")):
        v3.parse_v3(str(p))


@pytest.mark.parametrize("cpus,limit,warning", [
    ("'0.5'", {"cpu": "500m"}, None),
    ("'1_0'", {"cpu": "10"}, None),                       # underscores: Go float syntax
    ("' 0.5'", {}, 'Unable to convert cpu limits resources value : unable to cast " 0.5" of type string to float64'),
    ("'1e400'", {}, 'Unable to convert cpu limits resources value : unable to cast "1e400" of type string to float64'),
    ("'inf'", {"cpu": "-9223372036854775808m"}, None),   # int64(+Inf) on amd64
])
def test_deploy_cpus_parse_like_cast_to_float64(tmp_path, monkeypatch, capsys, cpus, limit, warning):
    """deploy.resources.*.cpus goes through cast.ToFloat64E and int64(x*1000)
    (v3.go:246-269); reservations warn with their own wording."""
    from move2kube_amd.utils import log
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    monkeypatch.setattr(settings, "compat", "fixed")
    src = tmp_path / "app"
    src.mkdir()
    (src / "docker-compose.yaml").write_text(
        "version: '3.7'\nservices:\n  s:\n    image: busybox\n    deploy:\n      resources:\n"
        "        limits:\n          cpus: %s\n        reservations:\n          cpus: 'x'\n" % cpus)
    log.set_verbose(False)
    out = api.translate(str(src), str(tmp_path / "out"), name="c")
    err = capsys.readouterr().err
    dep = yamlio.load(open(os.path.join(out, "c", "s-deployment.yaml")).read())
    res = dep["spec"]["template"]["spec"]["containers"][0]["resources"]
    assert res.get("limits", {}) == limit and res.get("requests", {}) == {}
    assert logparse.logged(err, 'Unable to convert cpu limits reservation value : unable to cast "x" of type string '
                                'to float64', "warning")
    if warning:
        assert logparse.logged(err, warning, "warning")


@pytest.mark.parametrize("content,want", [
    # docker/cli opts.ParseEnvFile: values kept as written, keys trimmed on the left only
    (b"A=1  \n  B=two words \n#C=3\n\xef\xbb\xbfD=4\n", None),
    (b"\xef\xbb\xbfA=1\nB=\n", {"A": "1", "B": ""}),
    (b"A =1\n", "poorly formatted environment: variable 'A ' contains whitespaces"),
    (b"=1\n", "poorly formatted environment: no variable name on line '=1'"),
    (b"A=\xff\n", "contains invalid utf8 bytes at line 1: [65 61 255]"),
])
def test_env_file_lines_parse_like_docker_cli(tmp_path, content, want):
    from move2kube_amd.source.compose.interpolate import EnvFileError, parse_env_file
    p = tmp_path / "app.env"
    p.write_bytes(content)
    if want is None:
        assert parse_env_file(str(p)) == {"A": "1  ", "B": "two words ", "\ufeffD": "4"}
    elif isinstance(want, dict):
        assert parse_env_file(str(p)) == want
    else:
        with pytest.raises(EnvFileError) as ei:
            parse_env_file(str(p))
        assert want in str(ei.value)


def test_env_files_dropped_only_when_missing_or_a_directory(tmp_path, capsys):
    """removeNonExistentEnvFilesV3 (v3.go:46-95): a missing env file or a
    directory is dropped with a warning; every other entry reaches docker/cli's
    opts.ParseEnvFile."""
    from move2kube_amd.source.compose import v3
    from move2kube_amd.utils import log
    (tmp_path / "dir.env").mkdir()
    (tmp_path / "ok.env").write_text("A=1\n")
    p = tmp_path / "docker-compose.yaml"
    p.write_text("version: '3'\nservices:\n  s:\n    image: busybox\n    env_file: [gone.env, dir.env, ok.env]\n")
    log.set_verbose(False)
    cfg = v3.parse_v3(str(p))
    assert cfg["services"][0]["environment"] == {"A": "1"}
    err = capsys.readouterr().err
    for name in ("gone.env", "dir.env"):
        assert logparse.logged(err, "Unable to find env config file %s referred in service s in file %s. Ignoring it."
                               % (tmp_path / name, p), "warning")


@pytest.mark.parametrize("kind", ["fifo", "enotdir"])
def test_an_env_file_that_exists_but_cannot_be_read_fails_the_load(tmp_path, kind):
    """An env file that stat finds but ParseEnvFile cannot read fails the whole
    compose load with the open error, as docker/cli returns it (wrapped by
    ParseV3, v3.go:112-118).  The reference
    blocks forever opening a FIFO, and panics on the nil FileInfo of a stat
    error other than ENOENT (v3.go:61): here both are that error."""
    from move2kube_amd.source.compose import v3
    if kind == "fifo":
        target = tmp_path / "pipe.env"
        os.mkfifo(str(target))
        ref, want = "pipe.env", "open %s: invalid argument" % target
    else:
        (tmp_path / "plain").write_text("x")
        ref, want = "plain/app.env", "open %s: not a directory" % (tmp_path / "plain" / "app.env")
    p = tmp_path / "docker-compose.yaml"
    p.write_text("version: '3'\nservices:\n  s:\n    image: busybox\n    env_file: %s\n" % ref)
    with pytest.raises(v3.ComposeError) as ei:
        v3.parse_v3(str(p))
    assert str(ei.value) == 'Unable to load Compose file at path %s Error: "%s"' % (p, want)   # ParseV3's %q
