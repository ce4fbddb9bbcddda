"""``utils/fastjson.py``: decoding as Go's ``encoding/json`` decodes, and
``go_encode`` as ``json.NewEncoder(w).Encode`` writes (Go 1.15,
``encoding/json/encode.go``: ``encodeState.string``, ``floatEncoder.encode``).
No Go toolchain is here; each expected value cites the code it follows
(parity beyond that source is unpinned)."""

import math

import pytest

from move2kube_amd.utils import fastjson


@pytest.mark.parametrize("v,want", [
    # floatEncoder: shortest 'f' in [1e-6, 1e21), shortest 'e' outside, e-09 -> e-9
    (1e-7, "1e-7"),
    (1.5e-10, "1.5e-10"),
    (1e-6, "0.000001"),
    (1.5, "1.5"),
    (100.0, "100"),
    (-0.0, "-0"),
    (1e20, "100000000000000000000"),
    (1e21, "1e+21"),
    (123456789.125, "123456789.125"),
    (3, "3"),
    # encodeState.string: HTML-safe escapes, raw UTF-8, � for a bad byte
    ("<a&b>", '"\\u003ca\\u0026b\\u003e"'),
    ("café ", '"café\\u2028"'),
    ("a\udcffb", '"a\\ufffdb"'),
    ("\x01\b\f\n\r\t", '"\\u0001\\u0008\\u000c\\n\\r\\t"'),
    ({"b": [1, None], "a": True}, '{"b":[1,null],"a":true}'),   # struct field order kept
])
def test_go_encode(v, want):
    assert fastjson.go_encode(v) == (want + "\n").encode("utf-8")


@pytest.mark.parametrize("f,text", [(math.nan, "NaN"), (math.inf, "+Inf"), (-math.inf, "-Inf")])
def test_go_encode_unsupported_values(f, text):
    # floatEncoder: e.error(&UnsupportedValueError{v, strconv.FormatFloat(f, 'g', -1, 64)})
    with pytest.raises(fastjson.UnsupportedValueError, match="^json: unsupported value: %s$" % text.replace("+", "\\+")):
        fastjson.go_encode([f])


@pytest.mark.parametrize("text,want", [
    ('{"port": 8080}', {"port": 8080}),
    ("[1.5, null, true]", [1.5, None, True]),
    ('"\\u00e9"', "é"),
])
def test_loads(text, want):
    assert fastjson.loads(text) == want


@pytest.mark.parametrize("text,err", [
    ("NaN", "invalid character 'N' looking for beginning of value"),
    ('{"a" 1}', "invalid character '1' after object key"),
    ("[1,", "unexpected end of JSON input"),
])
def test_loads_errors_are_go_texts(text, err):
    with pytest.raises(ValueError) as ei:
        fastjson.loads(text)
    assert str(ei.value) == err


@pytest.mark.parametrize("text,want", [
    # encoding/json decode.go unquote: a surrogate escape that is not half of a
    # pair decodes to U+FFFD, as a byte that is not UTF-8 does
    ('"\\ud800"', "�"),
    ('"\\udc80x"', "�x"),
    ('"\\ud83d\\ude00"', "\U0001F600"),
    ('{"\\ude00\\ud83d": ["a", "\\ud801"]}', {"��": ["a", "�"]}),
    ('"\udcff"', "�"),          # a surrogate-escaped byte of a file read as text
    (b'"\xff"', "�"),
])
def test_lone_surrogates_decode_to_the_replacement_character(text, want):
    assert fastjson.loads(text) == want


def test_errors_inside_containers_without_the_json_package():
    """A cold command never imports ``json``; the C scanner's errors inside an
    object or array then surface as SystemError and must still become Go's
    text (truncated detector output, a half-written docker config)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    texts = ['{"port": 80', "[1 2]", '{"a": [1,]}', '{"a" 1}']
    code = "\n".join([
        "import sys",
        "sys.path.insert(0, %r)" % root,
        "from move2kube_amd.utils import fastjson",
        "assert 'json.decoder' not in sys.modules",
        "for t in %r:" % texts,
        "    try:",
        "        fastjson.loads(t, parse_int=float)",
        "    except ValueError as e:",
        "        print(e)"])
    out = subprocess.run([sys.executable, "-S", "-c", code], capture_output=True, text=True, check=True).stdout
    assert out.splitlines() == ["unexpected end of JSON input", "invalid character '2' after array element",
                                "invalid character ']' looking for beginning of value",
                                "invalid character '1' after object key"]


def test_go_marshal_indent():
    """json.MarshalIndent(v, "", "\\t") as docker/cli's SaveToWriter writes a
    config file (configfile/file.go): Go's escapes, no trailing newline,
    empty containers kept compact."""
    from move2kube_amd.utils import fastjson
    got = fastjson.go_marshal_indent({"auths": {"r<é>&": {}, "b": {"auth": "x"}}, "l": [], "n": [1, None]}, "\t")
    assert got == ('{\n\t"auths": {\n\t\t"r\\u003cé\\u003e\\u0026": {},\n\t\t"b": {\n\t\t\t"auth": "x"\n\t\t}\n\t},'
                   '\n\t"l": [],\n\t"n": [\n\t\t1,\n\t\tnull\n\t]\n}').encode()
    assert fastjson.go_marshal_indent({}, "  ") == b"{}"
