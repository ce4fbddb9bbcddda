"""File discovery and YAML/JSON IO (``internal/common/utils_test.go`` TestGetFilesByExt,
TestGetFilesByName, TestWriteYaml, TestReadYaml, TestWriteJSON, TestReadJSON) and the
typed-file constructors (``types/collection/*_test.go``, ``types/qaengine/cache_test.go``)."""

import os
import shutil

import pytest

from conftest import ref_path
from move2kube_amd.models import collection, qa
from move2kube_amd.utils import common, constants, fsindex, yamlio

pytestmark = pytest.mark.reference

TESTDATA = ref_path("internal", "common", "testdata")


@pytest.fixture
def common_cwd(tmp_path, monkeypatch):
    """cwd holding a copy of the fixtures, so the reference's relative paths apply."""
    shutil.copytree(TESTDATA, str(tmp_path / "testdata"))
    monkeypatch.chdir(tmp_path)
    fsindex.invalidate()
    yield tmp_path
    fsindex.invalidate()


_as_root = hasattr(os, "geteuid") and os.geteuid() == 0


@pytest.mark.parametrize("fn,keys,want", [
    (common.get_files_by_ext, [".yaml", ".yml"],
     ["testdata/validfiles/test1.yaml", "testdata/validfiles/test2.yml", "testdata/validfiles/versioninfo.yaml"]),
    (common.get_files_by_name, ["test1.yaml", "test2.yml"],
     ["testdata/validfiles/test1.yaml", "testdata/validfiles/test2.yml"]),
])
def test_get_files(common_cwd, fn, keys, want):
    with pytest.raises(OSError):
        fn("foobar", keys)
    # a file path is returned as itself
    assert fn("testdata/validfiles/test1.yaml", keys) == ["testdata/validfiles/test1.yaml"]
    assert fn("testdata/validfiles", keys) == want
    os.mkdir("empty")
    assert fn("empty", keys) == []


@pytest.mark.parametrize("fn,keys", [(common.get_files_by_ext, [".yaml", ".yml"]), (common.get_files_by_name, ["a.yaml"])])
def test_get_files_unreadable_directory(unprivileged, fn, keys):
    """utils_test.go:76-87: a directory without permissions is an error."""
    d = os.path.join(unprivileged.tmp, "app1")
    os.mkdir(d)
    unprivileged.chown()
    os.chmod(d, 0)

    def check():
        fsindex.invalidate()
        with pytest.raises(OSError):
            fn(d, keys)
    unprivileged.run(check)


def test_write_yaml(tmp_path):
    with pytest.raises(OSError):
        common.write_yaml("/this/does/not/exist/foobar.yaml", "contents1")
    p = str(tmp_path / "foobar.yaml")
    common.write_yaml(p, {"foo": "contents1", "bar": 42})
    # go-yaml v3 keeps struct field order; maps written from structs keep insertion order here
    assert open(p).read() == "foo: contents1\nbar: 42\n"

    class GivesYamlError:
        def to_yaml(self):
            raise ValueError("Can't marshal this type to yaml.")

    with pytest.raises(ValueError):
        common.write_yaml(str(tmp_path / "bad.yaml"), GivesYamlError())


def test_read_yaml(common_cwd):
    with pytest.raises(OSError):
        common.read_yaml("foobar")
    with pytest.raises(yamlio.YAMLError):
        common.read_yaml("testdata/invalidfiles/test1.yaml")
    data = common.read_yaml("testdata/validfiles/test1.yaml")
    # keys a struct does not declare stay absent (Name/Tag keep their defaults in Go)
    assert "Name" not in data and "Tag" not in data
    assert (data["kind"], data["contextName"]) == ("ClusterMetadata", "name1")
    # version strings stay strings, not floats
    v = common.read_yaml("testdata/validfiles/versioninfo.yaml")
    assert v == {"version": "0.0.0", "gitCommit": "1.0.0", "gitTreeState": "1.1.0", "goVersion": "1.1.1"}


def test_write_json(tmp_path):
    with pytest.raises(OSError):
        common.write_json("/this/does/not/exist/foobar.json", "contents1")
    p = str(tmp_path / "foobar.json")
    common.write_json(p, {"Foo": "contents1", "Bar": 42})
    assert open(p).read() == '{"Foo":"contents1","Bar":42}\n'
    with pytest.raises(TypeError):
        common.write_json(str(tmp_path / "bad.json"), object())


def test_read_json(common_cwd):
    with pytest.raises(OSError):
        common.read_json("foobar")
    with pytest.raises(ValueError):
        common.read_json("testdata/invalidfiles/test1.json")
    assert common.read_json("testdata/validfiles/test1.json") == {"name": "name1", "foo": 42, "bar": ["bar"]}
    assert common.read_json("testdata/validfiles/versioninfo.json") == {
        "Version": "0.0.0", "GitCommit": "1.0.0", "GitTreeState": "1.1.0", "GoVersion": "1.1.1"}


@pytest.mark.parametrize("obj,kind", [
    (collection.ImageInfo(), collection.IMAGE_METADATA_KIND),
    (collection.CfContainerizers(), collection.CF_CONTAINERIZERS_KIND),
    (collection.CfInstanceApps(), collection.CF_INSTANCE_APPS_KIND),
    (qa.Cache("cache.yaml"), qa.QACACHE_KIND),
])
def test_new_typed_files(obj, kind):
    assert obj.kind == kind
    assert obj.api_version == constants.SCHEME_GROUP_VERSION == "move2kube.konveyor.io/v1alpha1"
    doc = obj.to_yaml()
    assert doc["kind"] == kind and doc["apiVersion"] == constants.SCHEME_GROUP_VERSION
