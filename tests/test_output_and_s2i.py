"""Helm values (reference ``types/output/helmvaluesoutput.go:31-70``) and the
S2I containerizer's failure paths (``internal/containerizer/s2icontainerizer.go``)
with a user-written detector directory: a failing or malformed detect
script, a missing builder, and template files that cannot be read or
rendered (each skipped with the reference's error line)."""

import os

import pytest

import logparse
from move2kube_amd.containerizer.base import ContainerizerError
from move2kube_amd.containerizer.s2i import S2IContainerizer
from move2kube_amd.models import output
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import log, yamlio


def _values(ns="", url="", sc="", globals_=None, services=None):
    h = output.HelmValues()
    h.registry_namespace, h.registry_url, h.storage_class = ns, url, sc
    h.global_variables = dict(globals_ or {})
    h.services = {k: dict(v) for k, v in (services or {}).items()}
    return h


def test_helm_values_merge():
    h = _values("ns", "quay.io", "", {"a": "1"}, {"web": {"web": "v1"}})
    h.merge(_values("", "docker.io", "gold", {"b": "2"}, {"web": {"side": "v2", "web": "v3"}, "db": {"db": "v4"}}))
    assert (h.registry_namespace, h.registry_url, h.storage_class) == ("ns", "docker.io", "gold")
    assert h.global_variables == {"a": "1", "b": "2"}
    assert h.services == {"web": {"web": "v3", "side": "v2"}, "db": {"db": "v4"}}


def test_helm_values_copy_is_deep_and_yaml_keeps_go_field_order():
    h = _values("ns", "quay.io", "gold", {"z": "1", "a": "2"}, {"web": {"web": "v1"}})
    h.ingress_host = "example.com"
    c = h.copy()
    c.services["web"]["web"] = "changed"
    c.global_variables["a"] = "x"
    assert h.services["web"]["web"] == "v1" and h.global_variables["a"] == "2"
    text = yamlio.dump(h.to_yaml())
    assert text == ("ingresshost: example.com\nregistryurl: quay.io\nregistrynamespace: ns\nservices:\n"
                    "  web:\n    containers:\n      web:\n        imagetag: v1\nstorageclass: gold\n"
                    "globalvariables:\n  a: \"2\"\n  z: \"1\"\n")
    # omitempty fields are left out
    assert set(_values().to_yaml()) == {"registryurl", "registrynamespace", "services"}


@pytest.fixture
def s2i_case(tmp_path):
    src = tmp_path / "app"
    src.mkdir()
    (src / "package.json").write_text("{}")
    det = tmp_path / "detector"
    det.mkdir()
    plan = plantypes.new_plan()
    plan.root_dir = str(tmp_path)
    svc = plantypes.Service("app")
    svc.container_build_type = plantypes.S2I
    svc.image = "app:latest"
    svc.target_options = [str(det)]
    svc.source_artifacts[plantypes.SOURCE_DIRECTORY_ARTIFACT] = [str(src)]
    log.set_verbose(False)
    return plan, svc, det


def _detect(det, body):
    s = det / "m2ks2idetect.sh"
    s.write_text("#!/bin/sh\n" + body)
    s.chmod(0o755)


def test_s2i_renders_every_detector_file(s2i_case, capsys):
    plan, svc, det = s2i_case
    _detect(det, "echo '{\"builder\": \"b/node:1\", \"port\": 8080}'\n")
    (det / ".s2i").mkdir()
    (det / ".s2i" / "environment").write_text("IMAGE={{ .image_name }}\n")
    (det / "bad.tpl").write_text("{{ .port | nosuchfunc }}\n")
    os.mkfifo(str(det / "pipe"))
    c = S2IContainerizer().get_container(plan, svc)
    assert c.new_files["app/.s2i/environment"] == "IMAGE=app:latest\n"
    assert "s2i build . b/node:1 app:latest" in c.new_files["app/app-s2i-build.sh"]
    assert "app/bad.tpl" not in c.new_files and "app/pipe" not in c.new_files
    assert c.exposed_ports == [8080]
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, 'Skipping path "%s" . Unable to translate the template to string.'
                                      % (det / "bad.tpl"), "error")
    assert logparse.logged_containing(err, 'Skipping path "%s" . Failed to read the template.' % (det / "pipe"),
                                      "error")


@pytest.mark.parametrize("body,msg", [
    ("exit 3\n", "exit status 3"),
    ("echo 'not json'\n", None),
    ("echo '{\"port\": 80}'\n", "has no builder"),
])
def test_s2i_detect_failures(s2i_case, capsys, body, msg):
    plan, svc, det = s2i_case
    _detect(det, body)
    with pytest.raises(ContainerizerError) as ei:
        S2IContainerizer().get_container(plan, svc)
    if msg:
        assert msg in str(ei.value)
    err = capsys.readouterr().err
    if body.startswith("exit"):
        assert logparse.logged_containing(err, "Detect using S2I containerizer at path", "error")
    elif msg is None:
        assert logparse.logged_containing(err, "Unable to unmarshal the output of the detect script at path", "error")


def test_s2i_needs_a_source_directory(s2i_case):
    plan, svc, det = s2i_case
    svc.source_artifacts = {}
    with pytest.raises(ContainerizerError, match="has no source code directory specified"):
        S2IContainerizer().get_container(plan, svc)
