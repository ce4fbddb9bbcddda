"""YAML decode errors worded as go-yaml reports them (``yaml: line N:
<libyaml problem>``; v3 names the context line, v2 the problem line, scanner
lines one later; ``unknown anchor``), and single-document loads that decode
the first document of a stream as ``yaml.Unmarshal`` does."""

import pytest

from move2kube_amd.utils import yamlio


@pytest.mark.parametrize("text,v3,v2", [
    ("a: b: c\n", "yaml: mapping values are not allowed in this context",
     "yaml: mapping values are not allowed in this context"),
    ("k: v\nk2: v2\n  bad: 3\n", "yaml: line 3: mapping values are not allowed in this context",
     "yaml: line 3: mapping values are not allowed in this context"),
    ("a: 1\nb: [1, 2\n", "yaml: line 1: did not find expected ',' or ']'",
     "yaml: line 2: did not find expected ',' or ']'"),
    ("key: 'unterminated\n", "yaml: line 2: found unexpected end of stream",
     "yaml: line 2: found unexpected end of stream"),
    ("a: &x 1\nb: *y\n", "yaml: unknown anchor 'y' referenced", "yaml: unknown anchor 'y' referenced"),
    # decode.go mapping(): a sequence or mapping key is failf("invalid map key: %#v");
    # v3 decodes an all-string mapping into map[string]interface{}, v2 never does
    ("a:\n  ? [1, 'x', 1.5, true, null, 2.0]\n  : 2\n",
     'yaml: invalid map key: []interface {}{1, "x", 1.5, true, interface {}(nil), 2}',
     'yaml: invalid map key: []interface {}{1, "x", 1.5, true, interface {}(nil), 2}'),
    ("? {b: 1, a: [yes]}\n: x\n", 'yaml: invalid map key: map[string]interface {}{"a":[]interface {}{"yes"}, "b":1}',
     'yaml: invalid map key: map[interface {}]interface {}{"a":[]interface {}{true}, "b":1}'),
    ("x: {? {[1]: 2} : 3}\n", "yaml: invalid map key: []interface {}{1}", "yaml: invalid map key: []interface {}{1}"),
])
def test_parse_errors_read_like_go_yaml(text, v3, v2):
    with pytest.raises(yamlio.YAMLError) as ei:
        yamlio.load(text)
    assert str(ei.value) == v3
    with pytest.raises(yamlio.YAMLError) as ei:
        yamlio.load_v2(text)
    assert str(ei.value) == v2
    with yamlio.parse_cache():  # one memoised parse, both wordings
        for load, want in ((yamlio.load, v3), (yamlio.load_v2, v2), (yamlio.load, v3)):
            with pytest.raises(yamlio.YAMLError) as ei:
                load(text)
            assert str(ei.value) == want


def test_single_loads_decode_the_first_document():
    assert yamlio.load("a: 1\n---\nb: 2\n") == {"a": 1}
    assert yamlio.load_v2("a: yes\n---\n[unclosed\n") == {"a": True}
    assert yamlio.load_raw("a: 1\n---\nb: 2\n") == {"a": "1"}
    assert yamlio.load_all("a: 1\n---\nb: 2\n") == [{"a": 1}, {"b": 2}]


def test_plan_read_error_is_worded_like_the_reference(tmp_path):
    from move2kube_amd.models import plan as plantypes
    p = tmp_path / "m2k.plan"
    p.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: Plan\nmetadata:\n  name: a\n    bad: 1\n")
    with pytest.raises(Exception) as ei:
        plantypes.read_plan(str(p))
    assert str(ei.value) == "yaml: line 5: mapping values are not allowed in this context"


@pytest.mark.parametrize("text,want", [
    # resolve.go resolvableTag: a tag go-yaml does not resolve decodes by node kind
    ("a: !foo bar\n", {"a": "bar"}),
    ("a: !!foo 12\n", {"a": "12"}),
    ("a: !foo [1, {b: 2}]\n", {"a": [1, {"b": 2}]}),
    ("a: !!set {x}\n", {"a": {"x": None}}),
    ("a: !!omap [x: 1]\n", {"a": [{"x": 1}]}),
    ("a: !!python/tuple [1]\n", {"a": [1]}),
    # decode.go scalar(): !!binary is decoded into a string
    ("a: !!binary aGVsbG8=\n", {"a": "hello"}),
])
def test_tags_decode_like_go_yaml(text, want):
    assert yamlio.load(text) == want
    assert yamlio.load_v2(text) == want


@pytest.mark.parametrize("text,want", [
    ("a: !!binary aGVsbG8\n", "yaml: !!binary value contains invalid base64 data"),
    # readerc.go: reader errors carry no mark, so no line number
    ("a: b\x01\n", "yaml: control characters are not allowed"),
    ("a: b\udcff\n", "yaml: invalid leading UTF-8 octet"),          # a lone 0xff byte
    ("a: b\udce9\udc80\n", "yaml: invalid trailing UTF-8 octet"),   # 0xe9 0x80 then a newline
    ("a: b\udce9\udc80", "yaml: incomplete UTF-8 octet sequence"),
    ("a: \udcc0\udc80\n", "yaml: invalid length of a UTF-8 sequence"),   # overlong NUL
    ("a: \udced\udca0\udc80\n", "yaml: invalid Unicode character"),      # an encoded surrogate
])
def test_decode_failures_read_like_go_yaml(text, want):
    for load in (yamlio.load, yamlio.load_v2, yamlio.load_raw):
        with pytest.raises(yamlio.YAMLError) as ei:
            load(text)
        assert str(ei.value) == want


def test_nel_is_not_printable_for_the_emitter():
    """yamlprivateh.go is_printable leaves out NEL (U+0085): a string holding
    one is written double-quoted with the \\N escape (PyYAML's emitter would
    write it raw, and the reader turns a raw NEL into a line break)."""
    for v in ("a\x85b", "\x85", "a\nb\x85c"):
        text = yamlio.dump({"k": [v]})
        assert "\x85" not in text and "\\N" in text
        assert yamlio.load(text) == {"k": [v]}


def test_line_and_paragraph_separators_in_a_literal_scalar():
    """emitterc.go write_break writes a break other than LF as itself and the
    next line's indentation follows it, so LS/PS inside a literal block read
    back unchanged (splitting lines there turned them into LF)."""
    for v in ("a\u2028b\nc", "x\u2029y\nz", "a\nb\u2028c"):
        text = yamlio.dump({"k": [v]})
        assert text.startswith("k:\n  - |-\n") and ("\u2028" in text or "\u2029" in text)
        assert yamlio.load(text) == {"k": [v]}


def test_line_separator_in_a_single_quoted_scalar():
    """write_single_quoted_scalar: LS/PS are written as themselves and the next
    character follows the indentation, so '--- x' after one is not read as a
    document marker at column 0."""
    for doc in ({"k": ["true\u2028--- x"]}, {"k": "a\u2029b"}, {"a": {"b": ["x\u2028\u2028y"]}}):
        text = yamlio.dump(doc)
        assert "'" in text and "\u2028\n" not in text
        assert yamlio.load(text) == doc
