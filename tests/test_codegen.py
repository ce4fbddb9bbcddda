"""Code generator: the Python modules it writes, and (``--go``) the reference's
Go output checked against ``internal/common/generator/testdata``."""

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


# --- internal/common/generator/generator_test.go, one pytest per subtest -------------------
# The Go generator writes Go source; ``--go`` mode writes the same bytes.

GEN_TESTDATA = ref_path("internal", "common", "generator", "testdata")


@pytest.fixture
def gen_cwd(tmp_path, monkeypatch):
    """cwd holding a writable copy of the generator's testdata (the Go test
    writes constants.go into testdata/datafortempfilled)."""
    import shutil
    shutil.copytree(GEN_TESTDATA, str(tmp_path / "testdata"))
    for dp, dns, fns in os.walk(str(tmp_path / "testdata")):
        os.chmod(dp, 0o755)
        for fn in fns:
            os.chmod(os.path.join(dp, fn), 0o644)
    monkeypatch.chdir(tmp_path)
    return tmp_path


def _skip_timestamp(path, want_lines, drop_last=False):
    with open(path) as f:
        lines = f.read().split("\n")
    assert len(lines) == want_lines
    return "\n".join(lines[:2] + lines[3:len(lines) - 1 if drop_last else len(lines)])


@pytest.mark.reference
def test_generate_code_for_non_existent_directory(gen_cwd):
    with pytest.raises(OSError):
        codegen.go_make_constants("testdata/nonexistent", codegen.GO_MAPS)


@pytest.mark.reference
@pytest.mark.parametrize("tpl,fixture", [
    pytest.param("GO_MAPS", "maptempemptyskiptimestamp.txt", id="read empty directory and generate code with maptemp"),
    pytest.param("GO_CONSTS", "conststempemptyskiptimestamp.txt",
                 id="read empty directory and generate code with conststemp")])
def test_generate_code_for_empty_directory(gen_cwd, tpl, fixture):
    d = gen_cwd / "foobar"
    d.mkdir()
    codegen.go_make_constants(str(d), getattr(codegen, tpl))
    with open(os.path.join("testdata", fixture)) as f:
        assert _skip_timestamp(str(d / "constants.go"), 8 + 17) == f.read()


@pytest.mark.reference
@pytest.mark.parametrize("tpl,fixture", [
    pytest.param("GO_MAPS", "maptempfilledskiptimestamp.txt", id="read filled directory and generate code with maptemp"),
    pytest.param("GO_CONSTS", "conststempfilledskiptimestamp.txt",
                 id="read filled directory and generate code with conststemp")])
def test_generate_code_for_filled_directory(gen_cwd, tpl, fixture):
    codegen.go_make_constants("testdata/datafortempfilled", getattr(codegen, tpl))
    with open(os.path.join("testdata", fixture)) as f:
        assert _skip_timestamp("testdata/datafortempfilled/constants.go", 22 + 17) == f.read()


def _unreadable_file_dir(unprivileged):
    p = os.path.join(unprivileged.tmp, "nopermstoread")
    with open(p, "w") as f:
        f.write("no permission to read this file")
    unprivileged.chown()
    os.chmod(p, 0)
    return unprivileged.tmp


def _unwritable_dir(unprivileged):
    d = os.path.join(unprivileged.tmp, "foobar")
    os.mkdir(d)
    unprivileged.chown()
    os.chmod(d, 0o400)
    return d


@pytest.mark.parametrize("make", [
    pytest.param(lambda d: codegen.go_make_constants(d, codegen.GO_CONSTS),
                 id="generate code from directory containing files that we have no permissions to read"),
    pytest.param(codegen.go_make_tar, id="make a tar when the directory has files which we have no permissions to read")])
def test_generate_code_unreadable_file(unprivileged, make):
    d = _unreadable_file_dir(unprivileged)

    def check():
        with pytest.raises((OSError, tarutil.TarError)):
            make(d)
    unprivileged.run(check)


@pytest.mark.parametrize("make", [
    pytest.param(lambda d: codegen.go_make_constants(d, codegen.GO_CONSTS),
                 id="generate code from directory that we have no permissions to write to"),
    pytest.param(codegen.go_make_tar, id="make a tar in a directory that we have no permissions to write to")])
def test_generate_code_unwritable_directory(unprivileged, make):
    d = _unwritable_dir(unprivileged)

    def check():
        with pytest.raises(OSError):
            make(d)
    unprivileged.run(check)


@pytest.mark.reference
def test_make_a_tar_using_a_filled_directory(gen_cwd):
    codegen.go_make_tar("testdata/datafortempfilled")
    with open("testdata/tartempfilledskiptimestampandtar.txt") as f:
        assert _skip_timestamp("testdata/datafortempfilled/constants.go", 6 + 17, drop_last=True) == f.read()
    # the last line holds the tree, without constants.go itself
    with open("testdata/datafortempfilled/constants.go") as f:
        last = f.read().split("\n")[-1]
    assert last.startswith("const Tar =  `") and last.endswith("`")
    names = sorted(m[0] for m in _tar_members(last[len("const Tar =  `"):-1]))
    assert names == [".", "test1.json", "test2.yml", "testconfigs", "testconfigs/test3.yml"]


def _tar_members(b64):
    import base64
    import io
    import tarfile
    with tarfile.open(fileobj=io.BytesIO(base64.b64decode(b64)), mode="r:") as tr:
        return [(m.name, m.size) for m in tr]


@pytest.mark.reference
def test_go_mode_cli(gen_cwd, capsys):
    """``codegen <dir> makemaps --go`` is generator.go's ``main`` (os.Args[2] ==
    "makemaps"); no mode argument writes the consts template."""
    assert codegen.main(["testdata/datafortempfilled", "makemaps", "--go"]) == 0
    with open("testdata/maptempfilledskiptimestamp.txt") as f:
        assert _skip_timestamp("testdata/datafortempfilled/constants.go", 22 + 17) == f.read()
    assert codegen.main(["testdata/datafortempfilled", "--go"]) == 0
    with open("testdata/conststempfilledskiptimestamp.txt") as f:
        assert _skip_timestamp("testdata/datafortempfilled/constants.go", 22 + 17) == f.read()
    assert capsys.readouterr().out.splitlines() == ["testdata/datafortempfilled/constants.go"] * 2
