"""The images collector's error paths (reference
``internal/collector/imagescollector.go``): ``docker inspect`` output that is
not JSON, ports and users that do not parse, a docker that is missing or
refuses the socket, ``docker image list`` (whose result the reference
filters and then drops), compose files that are not compose
files, and an output file that cannot be written."""

import os

import pytest

import logparse
from move2kube_amd.collector import images
from move2kube_amd.utils import log
from move2kube_amd.utils.constants import settings


def _docker(tmp_path, monkeypatch, script):
    bindir = tmp_path / "bin"
    bindir.mkdir(exist_ok=True)
    d = bindir / "docker"
    d.write_text("#!/bin/sh\n" + script)
    d.chmod(0o755)
    monkeypatch.setenv("PATH", str(bindir) + os.pathsep + "/usr/bin:/bin")
    log.set_verbose(True)


@pytest.fixture(autouse=True)
def _restore():
    yield
    log.set_verbose(False)


def test_inspect_output_that_is_not_json(capsys):
    log.set_verbose(False)
    info = images.get_image_info(b"not json")
    assert info.tags == [] and info.ports == []
    assert logparse.logged_containing(capsys.readouterr().err, "Unable to unmarshal image info : ", "error")


def test_ports_and_users_that_do_not_parse(capsys):
    log.set_verbose(True)
    info = images.get_image_info(b'[{"RepoTags":["x:1"],"ContainerConfig":{"ExposedPorts":'
                                 b'{"tcp":{},"080/tcp":{},"0123/udp":{},"8080/tcp":{}},"User":"1001"}}]')
    # "080" is not an int (cast.ToIntE reads a leading 0 as octal), "0123" is 83
    assert info.ports == [83, 8080] and info.user_id == 1001
    err = capsys.readouterr().err
    assert logparse.messages(err).count(("debug", "PortNumber not available in image metadata for [x:1]")) == 2


def test_docker_missing(tmp_path, monkeypatch, capsys):
    monkeypatch.setenv("PATH", str(tmp_path / "nobin"))
    log.set_verbose(False)
    with pytest.raises(FileNotFoundError):
        images.get_docker_inspect_result("a:1")
    assert logparse.logged_containing(capsys.readouterr().err, "Error while running docker-inspect: ", "warning")


@pytest.mark.parametrize("out,warnings", [
    ("Got permission denied while trying to connect to the Docker daemon socket",
     ["Error while running docker-inspect due to lack of permissions",
      "Please refer to [https://docs.docker.com/engine/install/linux-postinstall/] to fix this issue"]),
    ("Error: something else", None),
])
def test_docker_inspect_failures(tmp_path, monkeypatch, capsys, out, warnings):
    _docker(tmp_path, monkeypatch, "echo '%s'; exit 1\n" % out)
    log.set_verbose(False)
    with pytest.raises(images.CommandError):
        images.get_docker_inspect_result("a:1")
    err = capsys.readouterr().err
    if warnings:
        for w in warnings:
            assert logparse.logged(err, w, "warning")
    else:
        assert logparse.logged_containing(err, "Error while running docker-inspect: ", "warning")


def test_image_list_is_filtered_and_dropped_as_in_the_reference(tmp_path, monkeypatch, capsys):
    _docker(tmp_path, monkeypatch, "printf 'app/web:1.0\\n<none>:<none>\\nbase:<none>\\n'\n")
    assert images.get_all_image_names() == []
    assert logparse.logged(capsys.readouterr().err, "Ignore image with <none> : <none>:<none>", "debug")
    monkeypatch.setattr(settings, "compat", "fixed")
    assert images.get_all_image_names() == ["app/web:1.0"]


def test_image_list_failure(tmp_path, monkeypatch, capsys):
    _docker(tmp_path, monkeypatch, "exit 3\n")
    with pytest.raises(images.CommandError):
        images.get_all_image_names()
    assert logparse.logged_containing(capsys.readouterr().err, "Error while running docker image list : ", "warning")


def test_compose_image_names_skip_non_compose_yaml(tmp_path):
    (tmp_path / "a.yaml").write_text("services:\n  web: {image: nginx}\n  side: 3\n")
    (tmp_path / "b.yaml").write_text("- just a list\n")
    (tmp_path / "c.yaml").write_text("services: [x]\n")
    (tmp_path / "d.yml").write_text("key: [unclosed\n")
    # a scalar service fails yaml.v3's decode into sourcetypes.DCService: the whole file is skipped
    assert images.get_dc_image_names(str(tmp_path)) == []


def test_collect_skips_failures_and_reports_unwritable_output(tmp_path, monkeypatch, capsys):
    src = tmp_path / "src"
    src.mkdir()
    (src / "docker-compose.yaml").write_text("services:\n  a: {image: ok:1}\n  b: {image: gone:1}\n"
                                            "  c: {image: denied:1}\n")
    _docker(tmp_path, monkeypatch,
            'case "$2" in\n'
            '  ok:1) printf \'[{"RepoTags":["ok:1"],"ContainerConfig":{}}]\' ;;\n'
            '  gone:1) echo "Error: No such object: gone:1"; exit 1 ;;\n'
            '  *) echo "permission denied"; exit 1 ;;\n'
            'esac\n')
    log.set_verbose(False)
    out = tmp_path / "out"
    (out / "images").mkdir(parents=True)
    from move2kube_amd.utils import common
    taken = out / "images" / (common.normalize_for_filename("ok:1") + ".yaml")
    taken.mkdir()                                   # the file's path is taken by a directory
    images.ImagesCollector().collect(str(src), str(out))
    err = capsys.readouterr().err
    assert logparse.logged(err, 'Image [gone:1] not available in local image repo. Run "docker pull gone:1"',
                           "warning")
    assert logparse.logged_containing(err, "Unable to write file %s : " % taken, "error")


def test_collect_re_raises_what_is_not_a_command_failure(tmp_path, monkeypatch):
    src = tmp_path / "src"
    src.mkdir()
    (src / "docker-compose.yaml").write_text("services:\n  a: {image: ok:1}\n")

    def boom(name):
        raise KeyError(name)
    monkeypatch.setattr(images, "get_docker_inspect_result", boom)
    with pytest.raises(KeyError):
        images.ImagesCollector().collect(str(src), str(tmp_path / "out"))


@pytest.mark.parametrize("mode", ["reference", "fixed"])
def test_every_written_image_file_logs_the_nil_write_error_in_reference_mode(tmp_path, monkeypatch, capsys, mode):
    from move2kube_amd.utils import common
    from move2kube_amd.utils.constants import settings
    monkeypatch.setattr(settings, "compat", mode)
    src = tmp_path / "src"
    src.mkdir()
    (src / "docker-compose.yaml").write_text("services:\n  a: {image: ok:1}\n")
    _docker(tmp_path, monkeypatch, "printf '[{\"RepoTags\":[\"ok:1\"],\"ContainerConfig\":{}}]'\n")
    log.set_verbose(False)
    images.ImagesCollector().collect(str(src), str(tmp_path / "out"))
    path = tmp_path / "out" / "images" / (common.normalize_for_filename("ok:1") + ".yaml")
    assert path.is_file()
    logged = logparse.logged(capsys.readouterr().err, "Unable to write file %s : %%!s(<nil>)" % path, "error")
    assert logged == (mode == "reference")


def test_compose_files_the_typed_decode_refuses_are_skipped(tmp_path):
    """sourcetypes.DockerCompose: services must map to mappings (or null)."""
    (tmp_path / "a.yaml").write_text("services:\n  x: {image: one:1}\n  y:\n  z: {image: 3}\n")
    (tmp_path / "b.yaml").write_text("services:\n  x: {image: two:1}\n  y: [not, a, service]\n")
    (tmp_path / "c.yaml").write_text("services:\n  x: {image: {nested: 1}}\n")
    (tmp_path / "d.yaml").write_text("services: [x]\n")
    (tmp_path / "e.yaml").write_text("just: a file\n")
    assert images.get_dc_image_names(str(tmp_path)) == ["one:1", "", "3"]


def test_listing_failure_is_a_warning(tmp_path, monkeypatch, capsys):
    from move2kube_amd.utils import common

    def boom(*a):
        raise OSError(13, "Permission denied", str(tmp_path))
    monkeypatch.setattr(common, "get_files_by_ext", boom)
    assert images.get_dc_image_names(str(tmp_path)) == []
    assert logparse.logged_containing(capsys.readouterr().err, "Unable to fetch yaml files and recognize Docker image "
                                      "yamls : ", "warning")


def test_output_directory_that_cannot_be_made(tmp_path, capsys):
    (tmp_path / "out").mkdir()
    (tmp_path / "out" / "images").write_text("a file")
    with pytest.raises(RuntimeError, match="^mkdir %s: not a directory$" % (tmp_path / "out" / "images")):
        images.ImagesCollector().collect(str(tmp_path / "src"), str(tmp_path / "out"))
    assert logparse.logged(capsys.readouterr().err, "Unable to create output directory %s : mkdir %s: not a directory"
                           % (tmp_path / "out" / "images", tmp_path / "out" / "images"), "error")


def test_docker_missing_for_the_image_list_is_bash_127(tmp_path, monkeypatch, capsys):
    monkeypatch.setenv("PATH", str(tmp_path))
    with pytest.raises(OSError):
        images.get_all_image_names()
    assert logparse.logged(capsys.readouterr().err, "Error while running docker image list : exit status 127", "warning")
