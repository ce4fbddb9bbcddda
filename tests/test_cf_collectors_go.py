"""The Cloud Foundry collectors against what ``cf`` prints (reference
``internal/collector/cfappscollector.go:43-100`` and
``cfcontainertypescollector.go:50-211``): ``cf curl /v2/apps`` is decoded as
``json.Unmarshal`` into ``sourcetypes.CfInstanceApps`` decodes it (Go 1.15
encoding/json: a type mismatch fails the whole document with an
UnmarshalTypeError naming the struct and field path), and each failure is
logged with the caller's own line."""

import os

import pytest

import logparse
from move2kube_amd.collector import cf as cfc
from move2kube_amd.utils import log

ENTITY = "CfSourceApplication.resources.entity."


@pytest.mark.parametrize("text,want", [
    ('{"resources": [{"entity": {"name": "a", "memory": 256, "instances": 2, "ports": [8080],'
     ' "environment_json": {"K": "V", "N": null}, "extra": {"x": [1]}}}], "total_results": 1}',
     [{"name": "a", "memory": 256, "instances": 2, "ports": [8080], "environment_json": {"K": "V", "N": ""}}]),
    # keys match case-insensitively; null leaves a field at its zero value
    ('{"RESOURCES": [{"Entity": {"Name": "b", "BuildPack": null, "DockerImage": "img"}}, null, {}]}',
     [{"name": "b", "dockerimage": "img"}, {}, {}]),
    ("null", []),
    ('{"resources": null}', []),
])
def test_decode(text, want):
    assert cfc.decode_cf_apps(text) == want


@pytest.mark.parametrize("text,err", [
    ("[]", "json: cannot unmarshal array into Go value of type sourcetypes.CfInstanceApps"),
    ('"apps"', "json: cannot unmarshal string into Go value of type sourcetypes.CfInstanceApps"),
    ('{"resources": {}}', "json: cannot unmarshal object into Go struct field CfInstanceApps.resources of type "
                          "[]sourcetypes.CfResource"),
    ('{"resources": [1]}', "json: cannot unmarshal number into Go struct field CfInstanceApps.resources of type "
                           "sourcetypes.CfResource"),
    ('{"resources": [{"entity": "x"}]}', "json: cannot unmarshal string into Go struct field "
                                         "CfResource.resources.entity of type sourcetypes.CfSourceApplication"),
    ('{"resources": [{"entity": {"instances": "2"}}]}',
     "json: cannot unmarshal string into Go struct field " + ENTITY + "instances of type int"),
    ('{"resources": [{"entity": {"memory": 1.5}}]}',
     "json: cannot unmarshal number 1.5 into Go struct field " + ENTITY + "memory of type int64"),
    ('{"resources": [{"entity": {"memory": 1e3}}]}',
     "json: cannot unmarshal number 1e3 into Go struct field " + ENTITY + "memory of type int64"),
    ('{"resources": [{"entity": {"ports": [8080, 4294967296]}}]}',
     "json: cannot unmarshal number 4294967296 into Go struct field " + ENTITY + "ports of type int32"),
    ('{"resources": [{"entity": {"name": 7}}]}',
     "json: cannot unmarshal number into Go struct field " + ENTITY + "name of type string"),
    ('{"resources": [{"entity": {"buildpack": true}}]}',
     "json: cannot unmarshal bool into Go struct field " + ENTITY + "buildpack of type string"),
    ('{"resources": [{"entity": {"environment_json": {"A": 1}}}]}',
     "json: cannot unmarshal number into Go struct field " + ENTITY + "environment_json of type string"),
    ('{"resources": [{"entity": {"environment_json": ["A"]}}]}',
     "json: cannot unmarshal array into Go struct field " + ENTITY + "environment_json of type map[string]string"),
    # the first mismatch in document order is the one reported
    ('{"resources": [{"entity": {"memory": "x", "name": 1}}, {"entity": {"ports": "80"}}]}',
     "json: cannot unmarshal string into Go struct field " + ENTITY + "memory of type int64"),
    ('{"resources": [', "unexpected end of JSON input"),
])
def test_decode_errors(text, err):
    with pytest.raises(ValueError) as ei:
        cfc.decode_cf_apps(text)
    assert str(ei.value) == err


@pytest.fixture
def cf_stub(tmp_path, monkeypatch):
    """A ``cf`` that prints $CF_CURL for ``curl`` and $CF_BPS for
    ``buildpacks``, or fails with $CF_EXIT."""
    b = tmp_path / "bin"
    b.mkdir()
    s = b / "cf"
    s.write_text('#!/bin/sh\n[ -n "$CF_EXIT" ] && exit "$CF_EXIT"\n'
                 'case "$1" in curl) printf "%s" "$CF_CURL";; buildpacks) printf "%s" "$CF_BPS";; esac\n')
    s.chmod(0o755)
    monkeypatch.setenv("PATH", str(b) + os.pathsep + "/usr/bin:/bin")
    log.set_verbose(False)
    return monkeypatch


def test_apps_collector_type_error_skips(cf_stub, tmp_path, capsys):
    cf_stub.setenv("CF_CURL", '{"resources": [{"entity": {"name": "a", "instances": "2"}}]}')
    with pytest.raises(ValueError):
        cfc.CfAppsCollector().collect("", str(tmp_path / "out"))
    err = capsys.readouterr().err
    assert logparse.logged(err, "Error in unmarshalling yaml: json: cannot unmarshal string into Go struct field "
                                + ENTITY + "instances of type int. Skipping.", "error")
    assert len(logparse.messages(err)) == 1                     # logged once
    assert not (tmp_path / "out" / "cf").exists()


def test_apps_collector_command_failure(cf_stub, tmp_path, capsys):
    cf_stub.setenv("CF_EXIT", "3")
    with pytest.raises(Exception, match="^exit status 3$"):
        cfc.CfAppsCollector().collect("", str(tmp_path / "out"))
    assert logparse.logged(capsys.readouterr().err, "exit status 3", "error")


def test_apps_collector_write_failure(cf_stub, tmp_path, capsys):
    cf_stub.setenv("CF_CURL", '{"resources": [{"entity": {"name": "a"}}]}')
    from move2kube_amd.utils import common
    target = tmp_path / "out" / "cf" / (common.normalize_for_filename("instanceapps_a") + ".yaml")
    target.mkdir(parents=True)                                   # the output file's name is taken
    with pytest.raises(RuntimeError):
        cfc.CfAppsCollector().collect("", str(tmp_path / "out"))
    assert logparse.logged(capsys.readouterr().err, "Unable to write collect output : open %s: is a directory"
                           % target, "error")


def test_apps_collector_entities(cf_stub, tmp_path):
    cf_stub.setenv("CF_CURL", '{"resources": [{"entity": {"name": "a", "buildpack": "null", "detected_buildpack": '
                              '"nodejs", "dockerimage": "null", "memory": 64, "ports": null}}]}')
    cfc.CfAppsCollector().collect("", str(tmp_path / "out"))
    (name,) = os.listdir(str(tmp_path / "out" / "cf"))
    text = (tmp_path / "out" / "cf" / name).read_text()
    assert "detectedBuildpack: nodejs" in text and "memory: 64" in text and "ports: []" in text
    assert "buildpack: " not in text.replace("detectedBuildpack", "") and "dockerImage" not in text


def test_buildpack_names_from_the_foundation_log_each_failure(cf_stub, capsys):
    cf_stub.setenv("CF_EXIT", "1")
    assert cfc.get_cf_buildpack_names("") == []
    err = capsys.readouterr().err
    assert logparse.logged(err, "Error while getting buildpacks : exit status 1", "warning")
    assert logparse.logged(err, "Unable to collect buildpacks from cf instance : exit status 1", "warning")
    assert logparse.logged(err, "exit status 1", "error")
    assert logparse.logged(err, "Unable to find used buildpacks : exit status 1", "warning")


def test_buildpack_names_decode_error_has_no_final_period(cf_stub, capsys):
    cf_stub.setenv("CF_BPS", "Getting buildpacks...\n\nbuildpack  position\nruby_buildpack  1\n")
    cf_stub.setenv("CF_CURL", "[1]")
    assert cfc.get_cf_buildpack_names("") == ["ruby_buildpack"]
    assert logparse.logged(capsys.readouterr().err, "Error in unmarshalling yaml: json: cannot unmarshal array into "
                           "Go value of type sourcetypes.CfInstanceApps. Skipping", "error")


def test_used_buildpacks_listing_failure_is_a_warning(tmp_path, monkeypatch, capsys):
    from move2kube_amd.utils import common

    def boom(*a):
        raise OSError(13, "Permission denied", str(tmp_path))
    monkeypatch.setattr(common, "get_files_by_ext", boom)
    assert cfc.get_cf_buildpack_names(str(tmp_path)) == []
    assert logparse.logged_containing(capsys.readouterr().err, "Unable to fetch yaml files and recognize application "
                                      "manifest yamls : ", "warning")


def test_container_types_output_directory_failure(tmp_path, monkeypatch, capsys):
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    (tmp_path / "out").mkdir()
    (tmp_path / "out" / "cf").write_text("a file")
    with pytest.raises(RuntimeError, match="^mkdir %s: not a directory$" % (tmp_path / "out" / "cf")):
        cfc.CFContainerTypesCollector().collect(str(tmp_path / "src"), str(tmp_path / "out"))
    assert logparse.logged(capsys.readouterr().err, "Unable to create output path %s : mkdir %s: not a directory"
                           % (tmp_path / "out" / "cf", tmp_path / "out" / "cf"), "error")


def test_write_failures_are_logged_by_write_yaml_too(cf_stub, tmp_path, capsys):
    """common.WriteYaml logs its own error line before the caller's."""
    cf_stub.setenv("CF_CURL", '{"resources": [{"entity": {"name": "a"}}]}')
    from move2kube_amd.utils import common
    target = tmp_path / "out" / "cf" / (common.normalize_for_filename("instanceapps_a") + ".yaml")
    target.mkdir(parents=True)
    with pytest.raises(RuntimeError):
        cfc.CfAppsCollector().collect("", str(tmp_path / "out"))
    msgs = logparse.messages(capsys.readouterr().err)
    assert msgs == [("error", "Error writing yaml to file. error: open %s: is a directory,  outputPath %s"
                     % (target, target)),
                    ("error", "Unable to write collect output : open %s: is a directory" % target)]
