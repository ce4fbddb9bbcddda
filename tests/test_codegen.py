"""Code generator (``internal/common/generator`` test data shapes)."""

import importlib.util
import os

import pytest

from conftest import ref_path
from move2kube_amd.utils import codegen, tarutil


def _load(path):
    spec = importlib.util.spec_from_file_location("gen_mod", path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.fixture
def data_dir(tmp_path):
    d = tmp_path / "datafortempfilled"
    (d / "testconfigs").mkdir(parents=True)
    (d / "test1.json").write_text('{\n    "foo": "bar"\n}')
    (d / "test2.yml").write_text("---\nkey: `backtick` and '''quotes'''\n")
    (d / "testconfigs" / "test3.yml").write_text("nested: true\n")
    (d / ".hidden").write_text("x")
    (d / "gen.py").write_text("x = 1\n")
    return d


def test_make_constants(data_dir, tmp_path):
    out = tmp_path / "c.py"
    assert codegen.main([str(data_dir), "makeconsts", str(out)]) == 0
    m = _load(str(out))
    assert m.test1_json == '{\n    "foo": "bar"\n}'
    assert "`backtick`" in m.test2_yml
    assert not hasattr(m, "test3_yml") and not hasattr(m, "_hidden")


def test_make_maps(data_dir, tmp_path):
    out = tmp_path / "m.py"
    codegen.main([str(data_dir), "makemaps", str(out)])
    assert sorted(_load(str(out)).CONSTANTS) == ["test1_json", "test2_yml"]


def test_make_tar_roundtrip(data_dir, tmp_path):
    out = tmp_path / "t.py"
    codegen.main([str(data_dir), "maketar", str(out)])
    dst = tmp_path / "x"
    tarutil.untar_string(_load(str(out)).TAR, str(dst))
    assert (dst / "testconfigs" / "test3.yml").read_text() == "nested: true\n"


@pytest.mark.reference
def test_reference_generator_inputs(tmp_path):
    d = ref_path("internal", "common", "generator", "testdata", "datafortempfilled")
    m = _load_str(codegen.make_maps(d), tmp_path)
    assert sorted(m.CONSTANTS) == ["test1_json", "test2_yml"]
    assert m.CONSTANTS["test1_json"] == open(os.path.join(d, "test1.json")).read()


def _load_str(text, tmp_path):
    p = tmp_path / "g.py"
    p.write_text(text)
    return _load(str(p))
