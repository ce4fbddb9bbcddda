"""``internal/common/utils_test.go``, one pytest per Go subtest (the ids are the
Go subtest names; ``tests/reference_ledger.json`` maps each one).  Each test
checks what the Go subtest checks, with the same inputs and the same expected
values; where Go decodes into a struct, ``_decode`` below fills the struct's
fields the way the Go decoder does, from the document this package read.

Relative paths are the reference's: the tests run from a copy of
``internal/common/testdata``'s parent."""

import os
import shutil

import pytest

from conftest import ref_path
from goequal import assert_deep_equal, subtests
from move2kube_amd.utils import common, fsindex, gotemplate, yamlio

pytestmark = pytest.mark.reference

TESTDATA = ref_path("internal", "common", "testdata")


@pytest.fixture
def common_cwd(tmp_path, monkeypatch):
    shutil.copytree(TESTDATA, str(tmp_path / "testdata"))
    monkeypatch.chdir(tmp_path)
    fsindex.invalidate()
    yield tmp_path
    fsindex.invalidate()


class Struct:
    """An anonymous Go struct value: fields in declaration order."""

    def __init__(self, **fields):
        self.__dict__.update(fields)

    def __eq__(self, other):
        return type(other) is Struct and list(self.__dict__.items()) == list(other.__dict__.items())

    def __repr__(self):
        return "{%s}" % " ".join("%s:%r" % kv for kv in self.__dict__.items())


def _decode(doc, into, keys, fold):
    """Decode the mapping ``doc`` into the struct ``into`` as go-yaml v3
    (``fold`` False: key = tag, else the lowercased field name, exact match)
    or encoding/json (``fold`` True: exact key first, then EqualFold) does:
    fields without a key keep their value."""
    for field, key in keys.items():
        if key in doc:
            setattr(into, field, doc[key])
        elif fold:
            for k, v in doc.items():
                if k.lower() == key.lower():
                    setattr(into, field, v)
                    break
    return into


def _unreadable_dir(unprivileged):
    d = os.path.join(unprivileged.tmp, "app1")
    os.mkdir(d)
    unprivileged.chown()
    os.chmod(d, 0)
    return d


# --- TestGetFilesByExt / TestGetFilesByName -------------------------------------

_BY = {"ext": (common.get_files_by_ext, [".yaml", ".yml"],
               ["testdata/validfiles/test1.yaml", "testdata/validfiles/test2.yml",
                "testdata/validfiles/versioninfo.yaml"]),
       "name": (common.get_files_by_name, ["test1.yaml", "test2.yml"],
                ["testdata/validfiles/test1.yaml", "testdata/validfiles/test2.yml"])}


@pytest.mark.parametrize("by", subtests(("get files by extension when the path doesn't exist", "ext"),
                                        ("get files by name when the path doesn't exist", "name")))
def test_get_files_path_does_not_exist(common_cwd, by):
    fn, keys, _ = _BY[by]
    with pytest.raises(OSError):
        fn("foobar", keys)


@pytest.mark.parametrize("by", subtests(("get files by extension when the path is a file", "ext"),
                                        ("get files by name when the path is a file", "name")))
def test_get_files_path_is_a_file(common_cwd, by):
    fn, keys, _ = _BY[by]
    assert_deep_equal(fn("testdata/validfiles/test1.yaml", keys), ["testdata/validfiles/test1.yaml"])


@pytest.mark.parametrize("by", subtests(("get files by extension in the normal use case", "ext"),
                                        ("get files by name in the normal use case", "name")))
def test_get_files_normal_use_case(common_cwd, by):
    fn, keys, want = _BY[by]
    assert_deep_equal(fn("testdata/validfiles", keys), want)


@pytest.mark.parametrize("by", subtests(("get files by extension when the directory is empty", "ext"),
                                        ("get files by name when the directory is empty", "name")))
def test_get_files_directory_is_empty(tmp_path, by):
    fn, keys, _ = _BY[by]
    fsindex.invalidate()
    assert_deep_equal(fn(str(tmp_path), keys), [])


@pytest.mark.parametrize("by", subtests(
    ("get files by extension when you don't have permissions for the directory", "ext"),
    ("get files by name when you don't have permissions for the directory", "name")))
def test_get_files_no_permissions_for_the_directory(unprivileged, by):
    fn, keys, _ = _BY[by]
    d = _unreadable_dir(unprivileged)

    def check():
        fsindex.invalidate()
        with pytest.raises(OSError):
            fn(d, keys)
    unprivileged.run(check)


# --- TestYamlAttrPresent -----------------------------------------------------------

@pytest.mark.parametrize("path,attr,want", subtests(
    ("get attribute from non existent path", "foobar", "attr1", None),
    ("get attribute from invalid yaml file", "testdata/invalidfiles/test1.yaml", "attr1", None),
    ("get non existent attribute from yaml file", "testdata/validfiles/test1.yaml", "attr1", None),
    ("get attribute from yaml file", "testdata/validfiles/test1.yaml", "kind", "ClusterMetadata")))
def test_yaml_attr_present(common_cwd, path, attr, want):
    ok, val = common.yaml_attr_present(path, attr)
    if want is None:
        assert ok is False
    else:
        assert (ok, val) == (True, want)


# --- TestGetImageNameAndTag ----------------------------------------------------------

@pytest.mark.parametrize("image,want", subtests(
    ("get imagename and tag", "konveyor/getting-started:1.2.3-alpha.beta.gamma+hello.123.world",
     ("getting-started", "1.2.3-alpha.beta.gamma+hello.123.world")),
    ("get imagename and tag when there is no tag", "konveyor/getting-started", ("getting-started", "latest"))))
def test_get_image_name_and_tag(image, want):
    assert common.get_image_name_and_tag(image) == want


# --- TestWriteYaml / TestReadYaml ------------------------------------------------------

class GivesYamlError:
    def to_yaml(self):
        raise ValueError("Can't marshal this type to yaml.")


class GivesJSONError:
    def __json__(self):
        raise ValueError("Can't marshal this type to json.")


def test_write_yaml_to_an_invalid_path():
    with pytest.raises(OSError):
        common.write_yaml("/this/does/not/exist/foobar.yaml", "contents1")


def test_write_yaml_to_a_yaml_file(tmp_path):
    path1 = str(tmp_path) + "foobar.yaml"   # t.TempDir() + "foobar.yaml": a sibling of the temp dir
    try:
        common.write_yaml(path1, {"foo": "contents1", "bar": 42})   # struct{Foo string; Bar int}
        with open(path1) as f:
            assert f.read() == "foo: contents1\nbar: 42\n"
    finally:
        if os.path.exists(path1):
            os.remove(path1)


def test_write_yaml_data_that_cannot_be_encoded(tmp_path):
    with pytest.raises(ValueError):
        common.write_yaml(str(tmp_path / "foobar.yaml"), GivesYamlError())


_NAME_TAG = {"Name": "name", "Tag": "tag"}


def test_read_yaml_from_non_existent_path(common_cwd):
    with pytest.raises(OSError):
        common.read_yaml("foobar")


def test_read_yaml_from_invalid_yaml_file(common_cwd):
    with pytest.raises(yamlio.YAMLError):
        common.read_yaml("testdata/invalidfiles/test1.yaml")


def test_read_yaml_non_existent_keys(common_cwd):
    data1 = _decode(common.read_yaml("testdata/validfiles/test1.yaml"), Struct(Name="foo", Tag="bar"), _NAME_TAG, False)
    assert data1 == Struct(Name="foo", Tag="bar")


def test_read_yaml_some_data(common_cwd):
    data1 = _decode(common.read_yaml("testdata/validfiles/test1.yaml"), Struct(Kind="foo", ContextName="bar"),
                    {"Kind": "kind", "ContextName": "contextName"}, False)
    assert data1 == Struct(Kind="ClusterMetadata", ContextName="name1")


_VERSION_YAML = {"Version": "version", "GitCommit": "gitCommit", "GitTreeState": "gitTreeState", "GoVersion": "goVersion"}
_VERSION_JSON = {k: k for k in _VERSION_YAML}


def _version_info(version, commit, tree, go):
    return Struct(Version=version, GitCommit=commit, GitTreeState=tree, GoVersion=go)


def test_read_yaml_version_info(common_cwd):
    data1 = _decode(common.read_yaml("testdata/validfiles/versioninfo.yaml"),
                    _version_info("0.0.0", "0.0.0", "0.0.0", "0.0.0"), _VERSION_YAML, False)
    assert data1 == _version_info("0.0.0", "1.0.0", "1.1.0", "1.1.1")


# --- TestWriteJSON / TestReadJSON ----------------------------------------------------------

def test_write_json_to_an_invalid_path():
    with pytest.raises(OSError):
        common.write_json("/this/does/not/exist/foobar.json", "contents1")


def test_write_json_to_a_json_file(tmp_path):
    path1 = str(tmp_path) + "foobar.json"
    try:
        common.write_json(path1, {"Foo": "contents1", "Bar": 42})
        with open(path1) as f:
            assert f.read() == '{"Foo":"contents1","Bar":42}\n'
    finally:
        if os.path.exists(path1):
            os.remove(path1)


def test_write_json_data_that_cannot_be_encoded(tmp_path):
    with pytest.raises((TypeError, ValueError)):
        common.write_json(str(tmp_path / "foobar.json"), GivesJSONError())


_NAME_FOO_BAR = {"Name": "Name", "Foo": "Foo", "Bar": "Bar"}


def test_read_json_from_non_existent_path(common_cwd):
    with pytest.raises(OSError):
        common.read_json("foobar")


def test_read_json_from_invalid_json_file(common_cwd):
    with pytest.raises(ValueError):
        common.read_json("testdata/invalidfiles/test1.json")


def test_read_json_non_existent_keys(common_cwd):
    data1 = _decode(common.read_json("testdata/validfiles/test1.json"), Struct(Key1="foo", Key2="bar"),
                    {"Key1": "Key1", "Key2": "Key2"}, True)
    assert data1 == Struct(Key1="foo", Key2="bar")


def test_read_json_some_data(common_cwd):
    data1 = _decode(common.read_json("testdata/validfiles/test1.json"), Struct(Name="", Foo=0, Bar=None),
                    _NAME_FOO_BAR, True)
    assert_deep_equal(data1, Struct(Name="name1", Foo=42, Bar=["bar"]))


def test_read_json_version_info(common_cwd):
    data1 = _decode(common.read_json("testdata/validfiles/versioninfo.json"),
                    _version_info("0.0.0", "0.0.0", "0.0.0", "0.0.0"), _VERSION_JSON, True)
    assert data1 == _version_info("0.0.0", "1.0.0", "1.1.0", "1.1.1")


# --- table tests -------------------------------------------------------------------------------

@pytest.mark.parametrize("inp,out", subtests(
    ("normalize an invalid filename", "foobar%${/2\n\tinv.json.yaml.", "2-inv.json.yaml-d65d80a1c389718f"),
    ("normalize a valid filename", "foobar", "foobar-534a426c0464b01e"),
    ("normalize a long valid filename", "thisisalongfilenamefoobar", "thisisalongfile-730bb88a395ce114"),
    ("normalize a valid filename with an extension", "foobar.json", "foobar.json-f161da8efa921f1f"),
    ("normalize a valid filepath", "path/to/a/file/foobar.json", "foobar.json-b1760918996ebb3")))
def test_normalize_for_filename(inp, out):
    assert common.normalize_for_filename(inp) == out


@pytest.mark.parametrize("inp,out", subtests(
    ("normalize an invalid service name", "foobar.website.registration.", "foobar-website-registration-"),
    ("normalize a valid service name", "foobar", "foobar"),
    ("normalize a long valid service name", "thisisalongservicenamefoobar", "thisisalongservicenamefoobar")))
def test_normalize_for_service_name(inp, out):
    assert common.normalize_for_service_name(inp) == out


@pytest.mark.parametrize("arr,query,out", subtests(
    ("find a string in the array", ["foo", "bar"], "foo", True),
    ("find a non existent string in the array", ["foo", "bar"], "str1", False)))
def test_is_string_present(arr, query, out):
    assert common.is_string_present(arr, query) is out


@pytest.mark.parametrize("arr,query,out", subtests(
    ("find a int in an empty array", [], 0, False),
    ("find a int in an array", [100, 0, 1, -1, -42], 0, True),
    ("find a non existent int in an array", [100, 0, 1, -1, -42], 200, False),
    ("find a int in an array when there are duplicates", [100, 0, -42, -42, 1], -42, True)))
def test_is_int_present(arr, query, out):
    assert common.is_int_present(arr, query) is out


@pytest.mark.parametrize("a,b,out", subtests(
    ("merge 2 empty arrays", [], [], []),
    ("merge a filled array into an empty array", [], ["foo", "bar"], ["foo", "bar"]),
    ("merge an empty array into a filled array", ["foo", "bar"], [], ["foo", "bar"]),
    ("merge 2 filled arrays", ["foo", "bar"], ["foo", "bar", "item1", "item2"], ["foo", "bar", "item1", "item2"])))
def test_merge_string_slices(a, b, out):
    assert_deep_equal(common.merge_string_slices(a, b), out)


@pytest.mark.parametrize("a,b,out", subtests(
    ("merge 2 empty arrays", [], [], []),
    ("merge a filled array into an empty array", [], [100, 0], [100, 0]),
    ("merge an empty array into a filled array", [100, -42, -1, 0], [], [100, -42, -1, 0]),
    ("merge 2 filled arrays", [100, -42, -1, 0], [10, -1, -1, 0, 2], [100, -42, -1, 0, 10, 2])))
def test_merge_int_slices(a, b, out):
    assert_deep_equal(common.merge_int_slices(a, b), out)


class EmptyStruct:
    """``struct{}{}``: no fields, so ``{{.Name}}`` cannot be evaluated."""


_HELLO = "Hello! My name is {{.Name}} and my ID is {{.ID}}"
_TEMPLATE_CASES = (
    ("fill an empty template with an empty string", "", "", "", False),
    ("fill an empty template with an empty struct with no fields", "", EmptyStruct(), "", False),
    ("fill an empty template with an empty struct", "", Struct(Name="", ID=0), "", False),
    ("fill an empty template with a filled struct", "", Struct(Name="foobar", ID=42), "", False),
    ("fill a template with an empty struct with no fields", _HELLO, EmptyStruct(), "", True),
    ("fill a template with an empty struct", _HELLO, Struct(Name="", ID=0), "Hello! My name is  and my ID is 0", False),
    ("fill a template with a filled struct", _HELLO, Struct(Name="foobar", ID=42),
     "Hello! My name is foobar and my ID is 42", False),
)


@pytest.mark.parametrize("tpl,data,out,err", subtests(*_TEMPLATE_CASES))
def test_get_string_from_template(tpl, data, out, err):
    if err:
        with pytest.raises(gotemplate.TemplateError):
            common.get_string_from_template(tpl, data)
    else:
        assert common.get_string_from_template(tpl, data) == out


@pytest.mark.parametrize("tpl,data,out,err", subtests(*_TEMPLATE_CASES))
def test_write_template_to_file(tmp_path, tpl, data, out, err):
    path = str(tmp_path / "test1.go")
    if err:
        with pytest.raises(gotemplate.TemplateError):
            common.write_template_to_file(tpl, data, path, 0o777)
    else:
        common.write_template_to_file(tpl, data, path, 0o777)
        with open(path) as f:
            assert f.read() == out


def test_write_template_to_file_when_the_path_does_not_exist():
    with pytest.raises(OSError):
        common.write_template_to_file(_HELLO, Struct(Name="foobar", ID=42), "/this/path/does/not/exist/foobar", 0o777)


@pytest.mark.parametrize("arr,query,out", subtests(
    ("find the closest in an empty array", [], "foo", ""),
    ("find the closest in the array when the string exists", ["foo", "bar"], "foo", "foo"),
    ("find the closest in the array when the string doesn't exist", ["foo", "bar"], "bar2", "bar")))
def test_get_closest_matching_string(arr, query, out):
    assert common.get_closest_matching_string(arr, query) == out


@pytest.mark.parametrize("m1,m2,out", subtests(
    ("merge 2 empty maps", {}, {}, {}),
    ("merge a filled map into an empty map", {}, {"key1": "val1"}, {"key1": "val1"}),
    ("merge an empty map into a filled map", {"key1": "val1"}, {}, {"key1": "val1"}),
    ("merge 2 filled maps", {"key1": "val1", "key2": "val2"}, {"key2": "newval2", "key3": "val3"},
     {"key1": "val1", "key2": "newval2", "key3": "val3"})))
def test_merge_string_maps(m1, m2, out):
    assert_deep_equal(common.merge_string_maps(m1, m2), out)


@pytest.mark.parametrize("inp,out", subtests(
    ("normalize an empty name", "", ""),
    ("normalize an invalid name", "foo\n123.bar%4.inv#22.-", "foo-123.bar-4.inv-22.-"),
    ("normalize an invalid name", "foo/bar/", "bar"),
    ("normalize an invalid name", "path/prefix/foo_bar_baz", "foo-bar-baz"),
    ("normalize a valid name", "foo.bar.baz", "foo.bar.baz"),
    ("normalize a valid long name", "0123456789" * 8, "0123456789" * 8)))
def test_make_file_name_compliant(inp, out):
    assert common.make_file_name_compliant(inp) == out


@pytest.mark.parametrize("inp,out", subtests(
    ("find common directory when list is empty", [], ""),
    ("normal use case", ["/foo/bar/baz", "/foo/bar", "/foo"], "/foo"),
    ("normal use case and common directory is root", ["/foo/bar/baz", "/foo/bar", "/app1/service1/module1"], "/"),
    ("find common directory when list has unclean paths",
     ["/app1/./service1/", "/app1/service1/module2/", "/app1/./service1/../service1/module1"], "/app1/service1"),
    ("find common directory when list has unclean paths and common directory is root",
     ["/foo/bar///baz", "/foo/bar///.", "/app1/./service1/../service1/module1"], "/"),
    ("list has identical paths", ["/foo/bar/baz"] * 3, "/foo/bar/baz"),
    ("list contains root", ["/", "/.", "/..", "/.app/.bar", "/.app/.bar"], "/"),
    ("list contains root", ["/foo/bar", "/", "/foo/bar/baz"], "/"),
    ("list has identical but unclean paths", ["/foo/bar/baz////", "/foo/bar/baz", "/foo/bar/baz/././../baz/"],
     "/foo/bar/baz")))
def test_clean_and_find_common_directory(inp, out):
    assert common.clean_and_find_common_directory(inp) == out


@pytest.mark.parametrize("inp,out", subtests(
    ("find common directory when list is empty", [], ""),
    ("normal use case", ["/foo/bar/baz", "/foo/bar", "/foo"], "/foo"),
    ("normal use case and common directory is root", ["/foo/bar/baz", "/foo/bar", "/app1/service1/module1"], "/"),
    ("list has identical paths", ["/foo/bar/baz"] * 3, "/foo/bar/baz")))
def test_find_common_directory(inp, out):
    assert common.find_common_directory(inp) == out


@pytest.mark.parametrize("inp,out", subtests(
    ("Empty input slice", [], []),
    ("No duplicates", ["foo", "bar", "baz"], ["foo", "bar", "baz"]),
    ("Some duplicates", ["abc", "foo", "bar", "foo", "baz", "foo", "abc", "abc"], ["abc", "foo", "bar", "baz"]),
    ("Only duplicates", ["foo"] * 7, ["foo"])))
def test_unique_strings(inp, out):
    assert_deep_equal(common.unique_strings(inp), out)
