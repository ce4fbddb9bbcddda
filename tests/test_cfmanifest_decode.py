"""Cloud Foundry manifest decoding (reference ``cfmanifest2kube.go:422-489``
over the CF CLI's ``util/manifest`` Application type): the field forms it
reads, the shapes that make a file "not a CF manifest" (rejected: the error
texts are ours, logged at debug level only, parity unpinned), and the
missing-variable placeholders."""

import pytest

import logparse
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source import cfmanifest
from move2kube_amd.utils import log


def _read(tmp_path, text, name="", kind=plantypes.YAMLS):
    p = tmp_path / "manifest.yml"
    p.write_text(text)
    return cfmanifest.read_application_manifest(str(p), name, kind)


def test_application_fields(tmp_path):
    (a,), variables = _read(tmp_path, """\
applications:
- name: web
  buildpacks: [nodejs_buildpack, 1.5]
  command: npm start
  docker: {image: repo/web:1, username: bob}
  env: {N: 3, F: 2.50, B: true, S: x, Z: null}
  instances: 2
  memory: 1G
  path: ./app
  routes: [{route: web.example.com}, plain.example.com, null]
  services: [db, {name: cache}]
  stack: cflinuxfs3
  no-route: true
  health-check-type: http
""")
    assert variables == []
    assert (a.name, a.buildpacks, a.command.is_set, a.command.value) == ("web", ["nodejs_buildpack", "1.5"], True,
                                                                         "npm start")
    assert (a.docker_image, a.docker_username) == ("repo/web:1", "bob")
    # go-yaml v2 (YAML 1.1): the key N is the boolean false
    assert a.environment_variables == {"false": "3", "F": "2.5", "B": "true", "S": "x", "Z": "<nil>"}
    assert (a.instances.is_set, a.instances.value, a.memory, a.path) == (True, 2, "1G", "./app")
    assert a.routes == ["web.example.com", "plain.example.com", ""]
    assert a.services == ["db", "cache"]
    assert (a.stack_name, a.no_route, a.health_check_type) == ("cflinuxfs3", True, "http")
    assert not a.buildpack.is_set


@pytest.mark.parametrize("value", ["default", "null", "~"])
def test_default_buildpack_is_set_but_empty(tmp_path, value):
    (a,), _ = _read(tmp_path, "applications:\n- name: a\n  buildpack: %s\n" % value)
    assert a.buildpack.is_set and a.buildpack.value == ""


def test_several_applications_filtered_by_service_name(tmp_path):
    text = "applications:\n- name: a\n- name: b\n- name: b\n"
    apps, _ = _read(tmp_path, text)
    assert [x.name for x in apps] == ["a", "b", "b"]
    apps, _ = _read(tmp_path, text, "b")
    assert [x.name for x in apps] == ["b", "b"]
    (only,), _ = _read(tmp_path, "applications:\n- name: a\n", "other")     # one application: no filter
    assert only.name == "a"


@pytest.mark.parametrize("text", ["", "---\n", "other: 1\n", "applications: null\n"])
def test_no_applications(tmp_path, text):
    assert _read(tmp_path, text) == ([], [])


@pytest.mark.parametrize("text", [
    "- a\n- b\n",
    "just text\n",
    "applications: {name: a}\n",
    "applications: [name]\n",
    "applications:\n- name: a\n  buildpacks: nodejs\n",
    "applications:\n- name: a\n  docker: image\n",
    "applications:\n- name: a\n  env: [A]\n",
    "applications:\n- name: a\n  env: {A: {nested: 1}}\n",
    "applications:\n- name: a\n  instances: many\n",
    "applications:\n- name: [a]\n",
])
def test_shapes_that_are_not_a_cf_manifest(tmp_path, text, capsys):
    log.set_verbose(True)
    try:
        with pytest.raises(cfmanifest.ManifestError):
            _read(tmp_path, text)
    finally:
        log.set_verbose(False)
    assert logparse.logged_containing(capsys.readouterr().err, "Unable to read as cf manifest", "debug")


def test_scalar_type_errors_are_go_yaml_texts():
    err = cfmanifest._type_error("a long scalar value", "manifest.Manifest")
    assert err == "yaml: unmarshal errors:\n  line 1: cannot unmarshal !!str `a long ...` into manifest.Manifest"
    assert cfmanifest._type_error([1], "[]manifest.Application").endswith("cannot unmarshal !!seq into "
                                                                          "[]manifest.Application")
    assert "!!bool `true`" in cfmanifest._type_error(True, "x") and "!!float `1.5`" in cfmanifest._type_error(1.5, "x")


def test_unreadable_and_invalid_files(tmp_path):
    with pytest.raises(cfmanifest.ManifestError, match="^open %s: no such file or directory$" % (tmp_path / "none")):
        cfmanifest.get_missing_variables(str(tmp_path / "none"))
    p = tmp_path / "bad.yml"
    p.write_text("applications: [unclosed\n")
    with pytest.raises(cfmanifest.ManifestError, match="^yaml: "):
        cfmanifest.read_application_manifest(str(p))


def test_placeholders(tmp_path):
    """A dotted variable is reported by its first segment; the exact
    ``((a.b))`` scalar then has no value and stays as written, embedded ones
    too (parity unpinned: bosh's own interpolation of dotted names)."""
    (a,), variables = _read(tmp_path, "applications:\n- name: ((name))\n  env:\n    U: ((creds.user))\n"
                                      "    URL: http://((creds.host)):((port))/\n    Q: ((!quiet))\n")
    assert variables == ["creds", "name", "port", "quiet"]
    assert a.name == "{{ $name }}"
    assert a.environment_variables == {"U": "((creds.user))", "URL": "http://((creds.host)):{{ $port }}/",
                                       "Q": "{{ $quiet }}"}


def test_nesting_beyond_the_walks_is_a_manifest_error(tmp_path, monkeypatch):
    monkeypatch.setattr(cfmanifest, "_read_application_manifest",
                        lambda *a: (_ for _ in ()).throw(RecursionError()))
    with pytest.raises(cfmanifest.ManifestError, match="document nested too deeply"):
        cfmanifest.read_application_manifest(str(tmp_path / "m.yml"))
