"""``utils/gojson.py``: json.Unmarshal into typed Go values, and the two
decodes that use it besides the CF apps (``tests/test_cf_collectors_go.py``):
a CNB builder's order label (reference
``internal/containerizer/cnb/provider.go:33-48,94-108``) and the pack
provider's debug lines (``packprovider.go:39-120``)."""

import os

import pytest

import logparse
from move2kube_amd.containerizer.cnb import providers
from move2kube_amd.utils import gojson, log

ORDER = '[{"group": [{"id": "paketo/node", "version": "1.0"}, {"ID": "paketo/npm", "optional": true}]}, {"group": []}]'


def test_order_label():
    assert providers.get_builders_from_label(ORDER) == ["paketo/node", "paketo/npm"]
    assert providers.get_builders_from_label("null") == []
    assert providers.get_builders_from_label('[null, {"group": null}, {"group": [null]}]') == [""]


@pytest.mark.parametrize("label,err", [
    ('{"group": []}', "json: cannot unmarshal object into Go value of type cnb.order"),
    ('["x"]', "json: cannot unmarshal string into Go value of type cnb.orderEntry"),
    ('[{"group": {}}]', "json: cannot unmarshal object into Go struct field orderEntry.group of type "
                        "[]cnb.buildpackRef"),
    ('[{"group": [{"id": 5}]}]', "json: cannot unmarshal number into Go struct field buildpackRef.group.id of "
                                 "type string"),
    ('[{"group": [{"optional": "yes"}]}]', "json: cannot unmarshal string into Go struct field "
                                           "buildpackRef.group.optional of type bool"),
    ("[{", "unexpected end of JSON input"),
])
def test_order_label_errors(label, err, capsys):
    assert providers.get_builders_from_label(label) == []
    assert logparse.logged(capsys.readouterr().err, "Unable to read order : " + err, "warning")


def test_builder_data_debug_line(capsys):
    log.set_verbose(True)
    try:
        providers.get_builders_from_label(ORDER)
    finally:
        log.set_verbose(False)
    assert logparse.logged(capsys.readouterr().err, "Builder data :" + ORDER, "debug")


def test_map_elements_and_ints():
    spec = ("struct", "pkg.T", (("m", ("map", "map[string]int32", ("int", "int32", 32))),
                                ("n", ("int", "uint8", 8))))
    assert gojson.unmarshal('{"m": {"a": 1, "b": null}, "N": -128}', spec) == {"m": {"a": 1, "b": 0}, "n": -128}
    with pytest.raises(ValueError, match=r"^json: cannot unmarshal number 128 into Go struct field T\.n of type "
                                         r"uint8$"):
        gojson.unmarshal('{"n": 128}', spec)
    with pytest.raises(ValueError, match=r"^json: cannot unmarshal bool into Go struct field T\.m of type int32$"):
        gojson.unmarshal('{"m": {"a": true}}', spec)


def _pack(tmp_path, monkeypatch, body):
    b = tmp_path / "bin"
    b.mkdir(exist_ok=True)
    (b / "pack").write_text("#!/bin/sh\n" + body)
    (b / "pack").chmod(0o755)
    monkeypatch.setenv("PATH", str(b) + os.pathsep + "/usr/bin:/bin")


def test_pack_provider_debug_lines(tmp_path, monkeypatch, capsys):
    p = providers.PackProvider()
    monkeypatch.setenv("PATH", str(tmp_path))
    log.set_verbose(True)
    try:
        assert not p.is_available()
        _pack(tmp_path, monkeypatch, "exit 0\n")
        monkeypatch.setattr(providers, "DOCKER_SOCK", str(tmp_path / "no.sock"))
        assert not p.is_available()
        monkeypatch.setattr(providers, "DOCKER_SOCK", str(tmp_path / "bin" / "pack"))
        _pack(tmp_path, monkeypatch, "echo '===> DETECTING'\necho\necho '===> ANALYZING' >&2\nsleep 5\n")
        assert p.is_builder_supported(str(tmp_path), "b") is True
        _pack(tmp_path, monkeypatch, "echo 'No buildpack groups passed detection.'\n")
        assert p.is_builder_supported(str(tmp_path), "b") is False
    finally:
        log.set_verbose(False)
    err = capsys.readouterr().err
    assert logparse.logged(err, 'Unable to find pack : exec: "pack": executable file not found in $PATH', "debug")
    assert logparse.logged(err, "Unable to find pack docker socket, ignoring CNB based containerization approach : "
                                "stat %s: no such file or directory" % (tmp_path / "no.sock"), "debug")
    msgs = [m for lv, m in logparse.messages(err) if lv == "debug"]
    i = msgs.index("===> DETECTING")
    assert msgs[i:i + 3] == ["===> DETECTING", "===> ANALYZING", "Found compatible cnb for %s" % tmp_path]
    assert "No compatible cnb for %s" % tmp_path in msgs
