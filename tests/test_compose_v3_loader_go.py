"""docker/cli's v3 ``loader.Load`` past the schema (the revision pinned at
``/root/reference/go.mod:47``): ``Transform``'s mapstructure errors,
``resolveVolumePaths``, and the ``external`` rules of ``LoadNetworks``,
``LoadVolumes`` and ``loadFileObjectConfig``; and libcompose's memory
decode for v1/v2.  The reference wraps each as ``Unable to load Compose file
at path <p> Error: <%q>`` (``internal/source/compose/v3.go:93-121``) and logs
it from Compose2Kube (``compose2kube.go:111,170``)."""

import pytest

import logparse
from move2kube_amd.source.compose import v1v2, v3


def _load(tmp_path, body, version="3.7"):
    p = tmp_path / "docker-compose.yaml"
    p.write_text('version: "%s"\n' % version + body)
    return p


def _err(tmp_path, body, version="3.7"):
    p = _load(tmp_path, body, version)
    with pytest.raises(v3.ComposeError) as ei:
        v3.parse_v3(str(p))
    prefix = "Unable to load Compose file at path %s Error: " % p
    assert str(ei.value).startswith(prefix)
    return str(ei.value)[len(prefix):]


def test_transform_errors_are_collected_and_sorted(tmp_path):
    got = _err(tmp_path, "services:\n  web:\n    image: x\n    ports:\n      - 80\n      - abc:80\n"
                         "    volumes:\n      - /ok\n      - a::b:c\n      - vol::x\n"
                         "    deploy:\n      resources:\n        limits:\n          memory: 5zz\n")
    assert got == ('"3 error(s) decoding:\\n\\n'
                   "* error decoding 'Deploy.Resources.Limits.memory': invalid size: '5zz'\\n"
                   "* error decoding 'Ports': Invalid hostPort: abc\\n"
                   "* error decoding 'Volumes[2]': invalid spec: vol::x: empty section between colons\"")


def test_float_port_and_reservation_memory(tmp_path):
    got = _err(tmp_path, "services:\n  web:\n    image: x\n    ports:\n      - 80.5\n"
                         "    deploy:\n      resources:\n        reservations:\n          memory: 1.2.3m\n")
    assert got == ('"2 error(s) decoding:\\n\\n'
                   "* error decoding 'Deploy.Resources.Reservations.memory': strconv.ParseFloat: parsing "
                   '\\"1.2.3\\": invalid syntax\\n'
                   "* error decoding 'Ports': invalid type float64 for port\"")


def test_bind_volume_paths(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", "/home/u")
    p = _load(tmp_path, "services:\n  web:\n    image: x\n    volumes:\n      - ~/d:/a\n      - ./r/../s:/b\n"
                        "      - c:/win:/c\n      - type: bind\n        source: rel\n        target: /d\n")
    (svc,) = v3.parse_v3(str(p))["services"]
    assert [v["source"] for v in svc["volumes"]] == ["/home/u/d", str(tmp_path / "s"), "c:/win",
                                                     str(tmp_path / "rel")]
    got = _err(tmp_path, "services:\n  web:\n    image: x\n    volumes:\n      - type: bind\n        target: /d\n")
    assert got == '"invalid mount config for type \\"bind\\": field Source must not be empty"'


def test_tilde_without_home(tmp_path, monkeypatch, capsys):
    """The lookup is the loader's environment: with --ignoreenv it is empty,
    so ``~`` stays and the path is joined to the file's directory."""
    from move2kube_amd.utils.constants import settings
    monkeypatch.setattr(settings, "ignore_environment", True)
    p = _load(tmp_path, "services:\n  web:\n    image: x\n    volumes:\n      - ~/d:/a\n")
    (svc,) = v3.parse_v3(str(p))["services"]
    assert svc["volumes"][0]["source"] == str(tmp_path / "~" / "d")
    assert logparse.logged(capsys.readouterr().err, "cannot expand '~', because the environment lacks HOME",
                           "warning")


@pytest.mark.parametrize("kind,key,since", [("network", "networks", "3.5"), ("volume", "volumes", "3.4"),
                                            ("secret", "secrets", "3.5"), ("config", "configs", "3.5")])
def test_external_name(tmp_path, capsys, kind, key, since):
    body = "services:\n  web:\n    image: x\n%s:\n  o:\n    external:\n      name: real\n" % key
    cfg = v3.parse_v3(str(_load(tmp_path, body, since)))
    if key != "volumes":
        assert cfg[key]["o"]["name"] == "real"
    msg = "%s o: %s.external.name is deprecated in favor of %s.name" % (kind, kind, kind)
    assert logparse.logged(capsys.readouterr().err, msg, "warning")
    v3.parse_v3(str(_load(tmp_path, body, "3.3")))
    assert "deprecated" not in capsys.readouterr().err
    got = _err(tmp_path, body + "    name: other\n")
    assert got == '"%s o: %s.external.name and %s.name conflict; only use %s.name"' % ((kind,) * 4)


def test_external_volume_conflicts(tmp_path):
    got = _err(tmp_path, "services:\n  web:\n    image: x\nvolumes:\n  v:\n    external: true\n    driver: local\n")
    assert got == '"conflicting parameters \\"external\\" and \\"driver\\" specified for volume \\"v\\""'
    got = _err(tmp_path, "services:\n  web:\n    image: x\nvolumes:\n  v:\n    external: true\n    labels: [a=b]\n")
    assert got == '"conflicting parameters \\"external\\" and \\"labels\\" specified for volume \\"v\\""'


def test_secret_files_are_joined_not_expanded(tmp_path):
    cfg = v3.parse_v3(str(_load(tmp_path, "services:\n  web:\n    image: x\nsecrets:\n  s:\n    file: ~/k\n"
                                          "  e:\n    external: true\nconfigs:\n  c:\n    name: cfg\n")))
    assert cfg["secrets"]["s"]["file"] == str(tmp_path / "~" / "k")
    assert cfg["secrets"]["e"] == {"file": "", "external": True, "name": "e"}
    assert cfg["configs"]["c"]["file"] == str(tmp_path)


def test_warnings_repeat_with_every_parse(tmp_path, capsys):
    """The memo replays a parse's own log lines, as each of the reference's
    parses logs them."""
    from move2kube_amd.utils import fsindex
    p = _load(tmp_path, 'services:\n  web:\n    image: x\n    ports:\n      - "10.0.0.1:80:80"\n')
    with fsindex.scope():
        v3.parse_v3(str(p))
        v3.parse_v3(str(p))
    assert capsys.readouterr().err.count("ignoring IP-address (10.0.0.1:80:80/tcp)") == 2


@pytest.mark.parametrize("mem,err", [("5zz", "invalid size: '5zz'"), ('""', "invalid size: ''"),
                                     ("1.2.3", 'strconv.ParseFloat: parsing \\"1.2.3\\": invalid syntax')])
def test_v2_memory_errors(tmp_path, mem, err):
    """libcompose's MemStringorInt: an int, else RAMInBytes of the scalar's
    text; the error is utils.Convert's, unwrapped."""
    p = _load(tmp_path, "services:\n  web:\n    image: x\n    mem_limit: %s\n" % mem, "2")
    with pytest.raises(v1v2.ComposeError) as ei:
        v1v2.parse_v2(str(p))
    assert str(ei.value) == 'Failed to load docker compose file at path %s Error: "%s"' % (p, err)


def test_empty_environment_values_take_the_loader_environment(tmp_path, monkeypatch):
    """resolveEnvironment / updateEnvironment: ``K``, ``K=`` and ``K: ""``
    (from the service or an env file) take the value the loader's
    environment has for K; a value that is set stays."""
    monkeypatch.setenv("A", "os-a")
    monkeypatch.setenv("B", "os-b")
    monkeypatch.setenv("C", "os-c")
    monkeypatch.delenv("D", raising=False)
    (tmp_path / "e.env").write_text("A=\nE=\n")
    p = _load(tmp_path, "services:\n  web:\n    image: x\n    env_file: e.env\n"
                        "    environment:\n      - B=\n      - C\n      - D=\n      - F=set\n")
    (svc,) = v3.parse_v3(str(p))["services"]
    assert svc["environment"] == {"A": "os-a", "E": "", "B": "os-b", "C": "os-c", "D": "", "F": "set"}


@pytest.mark.parametrize("body,err", [
    ("services:\n  web:\n", "services.web must be a mapping"),
    ('services:\n  "my web":\n    image: x\n', "services Additional property my web is not allowed"),
    ("services:\n  w\u00e9b:\n    image: x\n", "services Additional property w\u00e9b is not allowed"),
    ("services:\n  web:\n    image: x\nhelicopters: {}\n", "(root) Additional property helicopters is not allowed"),
])
def test_schema_service_map(tmp_path, body, err):
    """config_schema_v3.x.json: a service is an object, its name matches
    ``^[a-zA-Z0-9._-]+$`` (additionalProperties false); gojsonschema's root
    context is ``(root)``."""
    assert _err(tmp_path, body) == '"%s"' % err


def test_v2_ports_format(tmp_path):
    """libcompose's "ports" format checker (nat.ParsePortSpecs on string
    entries) refuses the file; a number is not format-checked."""
    p = _load(tmp_path, 'services:\n  web:\n    image: x\n    ports:\n      - 80\n      - "abc:80"\n', "2")
    with pytest.raises(v1v2.ComposeError, match=r"web\.ports\.1 Does not match format 'ports'"):
        v1v2.parse_v2(str(p))
    p = _load(tmp_path, 'services:\n  web:\n    image: x\n    ports:\n      - 80\n      - "8000-8001:80"\n', "2")
    assert v1v2.parse_v2(str(p))["services"][0]["ports"] == ["80", "8000-8001:80"]


def test_probe_without_command_warning(capsys):
    """getHealthCheck's warning prints the HealthCheckTest slice as Go does."""
    from move2kube_amd.source.compose.v3 import V3Loader
    V3Loader.get_health_check({"test": ["NONE"], "timeout": None, "interval": None, "retries": None,
                               "start_period": None})
    V3Loader.get_health_check({"test": [], "timeout": None, "interval": None, "retries": None,
                               "start_period": None})
    err = capsys.readouterr().err
    assert logparse.logged(err, "Could not find command to execute in probe : [NONE]", "warning")
    assert logparse.logged(err, "Could not find command to execute in probe : []", "warning")


@pytest.mark.parametrize("version", ["2", None])
def test_v1v2_service_names(tmp_path, version):
    """libcompose validates the services map against a schema whose service
    names match ^[a-zA-Z0-9._-]+$ (additionalProperties false)."""
    p = tmp_path / "docker-compose.yaml"
    body = '"my web":\n  image: x\n'
    if version:
        p.write_text('version: "2"\nservices:\n' + "".join("  " + ln + "\n" for ln in body.splitlines()))
    else:
        p.write_text(body)
    with pytest.raises(v1v2.ComposeError, match=r"Unsupported config option for \(root\) service: 'my web'"):
        v1v2.parse_v2(str(p))


@pytest.mark.parametrize("key,msg", [
    ("workdir", "Unsupported config option for web service: 'workdir' (did you mean 'working_dir'?)"),
    ("port", "Unsupported config option for web service: 'port' (did you mean 'ports'?)"),
    ("colour", "Unsupported config option for web service: 'colour'"),
])
def test_v2_unsupported_option_hints(tmp_path, key, msg):
    """libcompose's unsupportedConfigMessage adds dockerConfigHints' guess."""
    p = _load(tmp_path, "services:\n  web:\n    image: x\n    %s: y\n" % key, "2")
    with pytest.raises(v1v2.ComposeError) as ei:
        v1v2.parse_v2(str(p))
    assert msg in str(ei.value)
