"""Containerizers off the happy path: the errors ``GetContainer`` returns (and
``Containerizers.GetContainer`` logs as "Error during containerization : %s"),
the detect-output forms ``json.Unmarshal`` into a map accepts or refuses, and
the reuse-Dockerfile containerizer's missing-Dockerfile lines.  Reference:
``internal/containerizer/dockerfilecontainerizer.go:86-170``,
``s2icontainerizer.go:87-110``, ``reusedockerfilecontainerizer.go:40-95``,
``cnbcontainerizer.go:41-115``."""

import os
import sys

import pytest

import logparse
from move2kube_amd.containerizer import cnb
from move2kube_amd.containerizer.base import ContainerizerError
from move2kube_amd.containerizer.dockerfile import DockerfileContainerizer, parse_detect_output
from move2kube_amd.containerizer.reusedockerfile import ReuseDockerfileContainerizer
from move2kube_amd.containerizer.s2i import S2IContainerizer
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import log


@pytest.fixture(autouse=True)
def _verbose():
    log.set_verbose(False)
    yield
    log.set_verbose(False)


def _plan(root):
    p = plantypes.new_plan()
    p.root_dir = str(root)
    return p


def _svc(name, build_type, options, src=None):
    s = plantypes.Service(name)
    s.container_build_type = build_type
    s.image = name + ":latest"
    s.target_options = list(options)
    if src is not None:
        s.source_artifacts[plantypes.SOURCE_DIRECTORY_ARTIFACT] = [str(src)]
    return s


# ---------------------------------------------------------------------------
# detect output
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("text,want", [
    ('{"port": 8080}', {"port": 8080.0}),
    ("null", {}),
    (" {} \n", {}),
])
def test_detect_output_accepted(text, want):
    assert parse_detect_output(text) == want


@pytest.mark.parametrize("text,kind", [("[1]", "array"), ('"x"', "string"), ("5", "number"), ("true", "bool")])
def test_detect_output_that_is_not_an_object(text, kind):
    with pytest.raises(ValueError, match=r"^json: cannot unmarshal %s into Go value of type "
                                         r"map\[string\]interface \{\}$" % kind):
        parse_detect_output(text)


# ---------------------------------------------------------------------------
# Dockerfile containerizer
# ---------------------------------------------------------------------------

@pytest.fixture
def df_case(tmp_path):
    src = tmp_path / "app"
    src.mkdir()
    det = tmp_path / "det"
    det.mkdir()
    (det / "Dockerfile").write_text("FROM base\nEXPOSE {{ .port }}\n")
    (det / "extra.conf").write_text("conf\n")
    return _plan(tmp_path), _svc("app", plantypes.NEW_DOCKERFILE, [str(det)], src), det


def _detect(det, body, name="m2kdfdetect.sh"):
    s = det / name
    s.write_text("#!/bin/sh\n" + body)
    s.chmod(0o755)


def test_dockerfile_container(df_case):
    plan, svc, det = df_case
    _detect(det, "echo '{\"port\": 8080}'\n")
    c = DockerfileContainerizer().get_container(plan, svc)
    assert c.new_files["app/Dockerfile.app"] == "FROM base\nEXPOSE 8080\n"
    assert c.new_files["app/extra.conf"] == "conf\n" and "app/app-docker-build.sh" in c.new_files
    assert "app/m2kdfdetect.sh" not in c.new_files and "app/Dockerfile" not in c.new_files
    assert c.exposed_ports == [8080] and c.repo_info.target_path == "app/Dockerfile.app"


def test_dockerfile_empty_detect_output_keeps_the_template(df_case):
    plan, svc, det = df_case
    _detect(det, "true\n")
    c = DockerfileContainerizer().get_container(plan, svc)
    assert c.new_files["app/Dockerfile.app"] == "FROM base\nEXPOSE {{ .port }}\n" and c.exposed_ports == []


def test_dockerfile_wrong_service(df_case):
    plan, svc, _ = df_case
    for s in (_svc("x", plantypes.S2I, svc.target_options), _svc("x", plantypes.NEW_DOCKERFILE, [])):
        with pytest.raises(ContainerizerError, match="^Unsupported service type for containerization or "
                                                     "insufficient information in service$"):
            DockerfileContainerizer().get_container(plan, s)


def test_dockerfile_missing_template(df_case, capsys):
    plan, svc, det = df_case
    os.remove(str(det / "Dockerfile"))
    with pytest.raises(ContainerizerError):
        DockerfileContainerizer().get_container(plan, svc)
    assert logparse.logged(capsys.readouterr().err, 'Unable to read the Dockerfile template at path "%s" Error: '
                           '"open %s: no such file or directory"' % (det / "Dockerfile", det / "Dockerfile"), "error")


def test_dockerfile_detect_failure_is_the_exit_status(df_case, capsys):
    plan, svc, det = df_case
    _detect(det, "exit 4\n")
    with pytest.raises(ContainerizerError, match="^exit status 4$"):
        DockerfileContainerizer().get_container(plan, svc)
    assert logparse.logged(capsys.readouterr().err, 'Detect using Dockerfile containerizer at path "%s" on the source '
                           'code at path "%s" failed. Error: "exit status 4"' % (det, svc.source_artifacts[
                               plantypes.SOURCE_DIRECTORY_ARTIFACT][0]), "error")


def test_dockerfile_detect_output_not_an_object(df_case, capsys):
    plan, svc, det = df_case
    _detect(det, "echo '[80]'\n")
    with pytest.raises(ContainerizerError, match="cannot unmarshal array"):
        DockerfileContainerizer().get_container(plan, svc)
    assert logparse.logged(capsys.readouterr().err, 'Unable to unmarshal the output of the detect script at path "%s" '
                           'Output: "[80]\\n" Error: "json: cannot unmarshal array into Go value of type '
                           'map[string]interface {}"' % det, "error")


def test_dockerfile_template_failure_writes_an_empty_dockerfile(df_case, capsys):
    plan, svc, det = df_case
    (det / "Dockerfile").write_text("FROM {{ .base | nosuch }}\n")
    _detect(det, "echo '{}'\n")
    c = DockerfileContainerizer().get_container(plan, svc)
    assert c.new_files["app/Dockerfile.app"] == ""
    assert logparse.logged_containing(capsys.readouterr().err, "Template conversion failed : ", "warning")


def test_dockerfile_init_lists_detectors(tmp_path, capsys):
    for d in ("b", "a/x"):
        (tmp_path / d).mkdir(parents=True)
        _detect(tmp_path / d, "true\n")
    log.set_verbose(True)
    c = DockerfileContainerizer()
    c.init(str(tmp_path))
    assert sorted(c.detectors) == [str(tmp_path / "a" / "x"), str(tmp_path / "b")]
    assert logparse.logged_containing(capsys.readouterr().err, "Detected Dockerfile containerization options : [",
                                      "debug")


def test_s2i_detect_failure_and_trimmed_output(tmp_path, capsys):
    src = tmp_path / "app"
    src.mkdir()
    det = tmp_path / "det"
    det.mkdir()
    svc = _svc("app", plantypes.S2I, [str(det)], src)
    _detect(det, "echo '  nope  '\nexit 2\n", "m2ks2idetect.sh")
    with pytest.raises(ContainerizerError, match="^exit status 2$"):
        S2IContainerizer().get_container(_plan(tmp_path), svc)
    _detect(det, "echo '  nope  '\n", "m2ks2idetect.sh")
    with pytest.raises(ContainerizerError):
        S2IContainerizer().get_container(_plan(tmp_path), svc)
    err = capsys.readouterr().err
    assert logparse.logged(err, 'Detect using S2I containerizer at path "%s" on the source code at path "%s" failed. '
                                'Error: "  nope  \\n"' % (det, src), "error")
    assert logparse.logged(err, 'Unable to unmarshal the output of the detect script at path "%s" Output: "nope" '
                                "Error: \"invalid character 'o' in literal null (expecting 'u')\"" % det, "error")
    with pytest.raises(ContainerizerError, match="^Unsupported service type for Containerization"):
        S2IContainerizer().get_container(_plan(tmp_path), _svc("app", plantypes.S2I, []))


# ---------------------------------------------------------------------------
# reuse-Dockerfile containerizer
# ---------------------------------------------------------------------------

def test_reuse_needs_a_target_option(tmp_path):
    with pytest.raises(ContainerizerError, match="^Failed to reuse the Dockerfile. The service web doesn't have any "
                                                 "containerization target options$"):
        ReuseDockerfileContainerizer().get_container(_plan(tmp_path), _svc("web", plantypes.REUSE_DOCKERFILE, []))


def test_reuse_missing_dockerfile_is_assumed_copied(tmp_path, capsys):
    df = tmp_path / "docker" / "Dockerfile"
    svc = _svc("web", plantypes.REUSE_DOCKERFILE, [str(df)])
    svc.build_artifacts[plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT] = [str(tmp_path / "src")]
    c = ReuseDockerfileContainerizer().get_container(_plan(tmp_path), svc)
    script = c.new_files["docker/web-docker-build.sh"]
    assert "-f Dockerfile" in script and "../src" in script
    err = capsys.readouterr().err
    assert logparse.logged(err, 'Unable to find the Dockerfile at path "%s" Error: "stat %s: no such file or '
                                'directory"' % (df, df), "error")
    assert logparse.logged(err, "Will assume the dockerfile will be copied and will proceed.", "error")


def test_reuse_other_stat_errors_pass_silently(tmp_path, capsys):
    (tmp_path / "file").write_text("x")
    df = tmp_path / "file" / "Dockerfile"            # ENOTDIR: not os.IsNotExist
    c = ReuseDockerfileContainerizer().get_container(_plan(tmp_path), _svc("web", plantypes.REUSE_DOCKERFILE, [str(df)]))
    assert "-f Dockerfile" in c.new_files["file/web-docker-build.sh"]
    assert "Unable to find the Dockerfile" not in capsys.readouterr().err


# ---------------------------------------------------------------------------
# CNB containerizer
# ---------------------------------------------------------------------------

def test_cnb_get_container_errors(tmp_path):
    c = cnb.CNBContainerizer()
    plan = _plan(tmp_path)
    with pytest.raises(ContainerizerError, match="^Service a has container build type S2I . Expected CNB$"):
        c.get_container(plan, _svc("a", plantypes.S2I, ["b"]))
    with pytest.raises(ContainerizerError, match="^Service a has no containerization target options$"):
        c.get_container(plan, _svc("a", plantypes.CNB, []))
    with pytest.raises(ContainerizerError, match="^Service a has no source code directory specified$"):
        c.get_container(plan, _svc("a", plantypes.CNB, ["builder"]))
    got = c.get_container(plan, _svc("a", plantypes.CNB, ["my/builder"], tmp_path / "src"))
    assert "my/builder" in got.new_files["src/a-cnb-build.sh"] and got.exposed_ports == [8080]


@pytest.fixture
def chain_off(monkeypatch):
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    monkeypatch.delitem(sys.modules, cnb.__name__ + ".providers", raising=False)
    monkeypatch.setitem(cnb._warned, "not_supported", False)
    monkeypatch.setitem(cnb._warned, "long_wait", False)
    cnb.reset_cache()
    yield
    cnb.reset_cache()


def test_cnb_chain_off(tmp_path, chain_off, capsys):
    c = cnb.CNBContainerizer()
    c.init(str(tmp_path))
    assert c.get_target_options(None, str(tmp_path)) == []
    cnb._cache[str(tmp_path / "x")] = ["cached/builder"]
    assert c.get_target_options(None, str(tmp_path / "x")) == ["cached/builder"]
    assert c.get_all_buildpacks() == {}
    cnb.prefetch_builder_probes()                    # nothing to start
    err = capsys.readouterr().err
    assert err.count("No CNB containerizer method accessible") == 1      # once per process
    assert "This could take a few minutes" not in err                   # the reference's flag starts true


def test_cnb_long_wait_warning_in_fixed_mode(tmp_path, chain_off, capsys, monkeypatch):
    from move2kube_amd.utils.constants import settings
    monkeypatch.setattr(settings, "compat", "fixed")
    out = cnb.CNBContainerizer().get_target_options_batch(None, [str(tmp_path / "a"), str(tmp_path / "b")])
    assert out == [[], []]
    assert capsys.readouterr().err.count("This could take a few minutes to complete.") == 1
