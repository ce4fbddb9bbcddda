"""``TarAsString`` / ``UnTarString`` against the reference's own fixtures
(``internal/common/tar_test.go:93-330``, data in
``internal/common/testdata/datafortestingtar``)."""

import base64
import io
import json
import os
import shutil
import stat
import tarfile

import pytest

from move2kube_amd.utils import tarutil

from conftest import ref_path

TOBETARRED = ref_path("internal", "common", "testdata", "datafortestingtar", "tobetarred")
UNTAR_JSON = ref_path("internal", "common", "testdata", "datafortestingtar", "untarstring.json")

pytestmark = pytest.mark.reference


def _members(tarstring):
    raw = base64.b64decode(tarstring)
    out = []
    with tarfile.open(fileobj=io.BytesIO(raw), mode="r:") as tr:
        for m in tr:
            data = b"" if m.isdir() else tr.extractfile(m).read()
            out.append((m.name, m.size, m.mode & 0o777, m.isdir(), data))
    return out


def _walk_expected(root, ignored=()):
    """What filepath.Walk reports (lexical order), like the Go test builds it."""
    exp = []

    def visit(p):
        rel = os.path.relpath(p, root)
        if rel in ignored:
            return
        st = os.lstat(p)
        if stat.S_ISDIR(st.st_mode):
            exp.append((rel, 0, st.st_mode & 0o777, True, b""))
            for name in sorted(os.listdir(p)):
                visit(os.path.join(p, name))
        else:
            with open(p, "rb") as f:
                exp.append((rel, st.st_size, st.st_mode & 0o777, False, f.read()))
    visit(root)
    return exp


def test_tar_path_does_not_exist(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    with pytest.raises(tarutil.TarError, match="^lstat foobar: no such file or directory$"):
        tarutil.tar_as_string("foobar", [])


def test_tar_a_single_file(tmp_path):
    src = os.path.join(TOBETARRED, "test1.yaml")
    dst = tmp_path / "test1.yaml"
    shutil.copyfile(src, str(dst))
    os.chmod(str(dst), 0o644)
    data = dst.read_bytes()
    assert _members(tarutil.tar_as_string(str(dst), [])) == [(".", 217, 0o644, False, data)]


def test_tar_an_empty_directory(tmp_path):
    d = tmp_path / "foobar"
    d.mkdir(mode=0o755)
    os.chmod(str(d), 0o755)
    assert _members(tarutil.tar_as_string(str(d), [])) == [(".", 0, 0o755, True, b"")]


def test_tar_a_filled_directory(tmp_path):
    d = str(tmp_path / "tobetarred")
    shutil.copytree(TOBETARRED, d)
    assert _members(tarutil.tar_as_string(d, [])) == _walk_expected(d)


def test_tar_while_ignoring_some_files(tmp_path):
    d = str(tmp_path / "tobetarred")
    shutil.copytree(TOBETARRED, d)
    ignored = ["test2.yml", "versioninfo.json", "foobar.json"]
    got = _members(tarutil.tar_as_string(d, ignored))
    assert got == _walk_expected(d, ignored)
    assert "test2.yml" not in [m[0] for m in got]


def test_tar_unreadable_file_fails(unprivileged):
    """tar_test.go:231-240: a file without read permission cannot be tarred."""
    p = os.path.join(unprivileged.tmp, "nopermstoread")
    with open(p, "w") as f:
        f.write("no permission to read this file")
    unprivileged.chown()
    os.chmod(p, 0)

    def check():
        with pytest.raises(tarutil.TarError, match=r"^open %s: permission denied$" % p):
            tarutil.tar_as_string(p, [])
        with pytest.raises(tarutil.TarError, match=r"^open %s: permission denied$" % p):
            tarutil.tar_as_string(unprivileged.tmp, [])
    unprivileged.run(check)


@pytest.fixture(scope="module")
def untar_data():
    with open(UNTAR_JSON) as f:
        return json.load(f)


def test_untar_valid_then_tar_again(untar_data, tmp_path):
    tarutil.untar_string(untar_data["untar_a_valid_tarstring"], str(tmp_path))
    assert tarutil.tar_as_string(str(tmp_path), [])


def test_untar_invalid_base64(untar_data, tmp_path):
    with pytest.raises(Exception):
        tarutil.untar_string(untar_data["untar_an_invalid_base_64_string"], str(tmp_path))


def test_untar_invalid_tar(untar_data, tmp_path):
    with pytest.raises(Exception):
        tarutil.untar_string(untar_data["untar_an_invalid_tarstring"], str(tmp_path))


@pytest.mark.parametrize("key", [
    pytest.param("untar_into_a_directory_we_dont_have_permission_to_write_to",
                 id="untar into a directory we don't have permission to write to"),
    pytest.param("untar_a_single_file_into_a_directory_we_dont_have_permission_to_write_to",
                 id="untar a single file into a directory we don't have permission to write to")])
def test_untar_into_unwritable_dir(untar_data, unprivileged, key):
    """tar_test.go:281-305: untarring below a directory with mode 0 fails."""
    d = os.path.join(unprivileged.tmp, "nopermstowrite")
    os.mkdir(d)
    unprivileged.chown()
    os.chmod(d, 0)
    data = untar_data[key]

    def check():
        with pytest.raises(OSError):
            tarutil.untar_string(data, os.path.join(d, "foobar"))
    unprivileged.run(check)
