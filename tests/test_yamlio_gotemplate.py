"""go-yaml v3 emitter and Go text/template semantics the outputs depend on."""

import pytest

from move2kube_amd.utils import gotemplate, yamlio


@pytest.mark.parametrize("value,out", [
    ("plain", "plain"), ("true", '"true"'), ("yes", '"yes"'), ("123", '"123"'), ("1.5", '"1.5"'),
    ("", '""'), ("a: b", "'a: b'"), ("- x", "'- x'"), ("#c", "'#c'"), (" lead", "' lead'"),
    ("null", '"null"'), ("~", '"~"'), ("0x1F", '"0x1F"'), ("1e3", '"1e3"'), ("12:30", '"12:30"'),
    ("2001-12-14", '"2001-12-14"'), ("it's", "it's"), ("{x}", "'{x}'"), ("a\tb", '"a\\tb"'),
    ("{{ .Release.Name }}-{{ .Values.ingresshost }}", "'{{ .Release.Name }}-{{ .Values.ingresshost }}'"),
])
def test_scalar_styles(value, out):
    assert yamlio.dump({"k": value}) == "k: %s\n" % out


def test_literal_blocks():
    assert yamlio.dump({"k": "a\nb\n"}) == "k: |\n  a\n  b\n"
    assert yamlio.dump({"k": "a\nb"}) == "k: |-\n  a\n  b\n"
    assert yamlio.dump({"k": "a\nb\n\n"}) == "k: |+\n  a\n  b\n\n"
    assert yamlio.dump({"k": "a \nb"}) == 'k: "a \\nb"\n'


def test_sequences_indented_and_empty_collections():
    assert yamlio.dump({"a": [1, 2], "b": {}, "c": [], "d": None}) == "a:\n  - 1\n  - 2\nb: {}\nc: []\nd: null\n"


def test_go_map_ordering_and_numbers():
    d = yamlio.GoMap({"b": 1, "a": 2.5, "a10": 1e-7, "a2": 1000000.0, "A": True})
    assert yamlio.dump(d) == "A: true\na: 2.5\na2: 1e+06\na10: 1e-07\nb: 1\n"


def test_k8s_dump_sorts_all_maps():
    assert yamlio.dumps_k8s({"z": 1, "a": {"x": 1, "b": 2}}) == "a:\n  b: 2\n  x: 1\nz: 1\n"
    # go-yaml v3 quotes YAML 1.1 booleans such as "y" even as keys
    assert yamlio.dumps_k8s({"y": 1}) == '"y": 1\n'


def test_loader_is_yaml12ish():
    d = yamlio.load("a: yes\nb: on\nc: 2001-12-14\nd: 0x10\ne: true\n")
    assert d == {"a": "yes", "b": "on", "c": "2001-12-14", "d": 16, "e": True}


@pytest.mark.parametrize("tpl,data,out", [
    ("{{ .A }}-{{ .B }}", {"A": 1, "B": "x"}, "1-x"),
    ("{{- if .A }} yes {{- else }} no {{- end }}", {"A": False}, " no"),
    ("{{- if .A }} yes {{- else -}} no {{- end }}", {"A": False}, "no"),
    ("{{ range $k, $v := . }}{{ $k }}={{ $v }};{{ end }}", {"b": 2, "a": 1}, "a=1;b=2;"),
    ("{{ range . }}[{{ . }}]{{ else }}empty{{ end }}", [], "empty"),
    ("{{ with .A }}{{ . }}{{ end }}", {"A": "w"}, "w"),
    ('{{ index .M "k" }}', {"M": {"k": "v"}}, "v"),
    ("{{ printf \"%s-%d\" .S .N }}", {"S": "s", "N": 3}, "s-3"),
    ("{{ len .L }}", {"L": [1, 2, 3]}, "3"),
    ("{{ if and .A (not .B) }}ok{{ end }}", {"A": 1, "B": 0}, "ok"),
    ("{{ if eq .A \"x\" \"y\" }}ok{{ end }}", {"A": "y"}, "ok"),
    ("{{/* comment */}}x", {}, "x"),
    ('{{"{{ .Release.Name }}"}}', {}, "{{ .Release.Name }}"),
    ("{{ .Missing }}", {}, "<no value>"),
    ("{{ define \"t\" }}T{{ . }}{{ end }}{{ template \"t\" .X }}", {"X": 1}, "T1"),
    ("{{ $x := 1 }}{{ if true }}{{ $x = 2 }}{{ end }}{{ $x }}", {}, "2"),
])
def test_templates(tpl, data, out):
    assert gotemplate.render(tpl, data) == out


def test_template_errors():
    with pytest.raises(gotemplate.TemplateError):
        gotemplate.render("{{ .A", {})
    with pytest.raises(gotemplate.TemplateError):
        gotemplate.render("{{ if }}x{{ end }}", {})


def test_parse_cache_returns_private_copies_and_reraises():
    from move2kube_amd.utils import yamlio as y
    text = "a:\n  b: [1, 2]\n"
    bad = "a: [\n"
    with y.parse_cache():
        d1 = y.load(text)
        d1["a"]["b"].append(3)
        d2 = y.load(text)
        assert d2 == {"a": {"b": [1, 2]}}
        assert y.load_raw("x: 1\n") == {"x": "1"}      # loaders are cached separately
        assert y.load("x: 1\n") == {"x": 1}
        for _ in range(2):
            try:
                y.load(bad)
            except y.YAMLError:
                pass
            else:
                raise AssertionError("expected a YAML error")
    assert y._memo is None


GO_TEMPLATE_CASES = [
    # (template, data, output of Go's text/template + fmt)
    ("{{- /* c */ -}} a", {}, "a"),
    ("{{range $i, $e := .L}}{{$i}}={{$e}};{{end}}", {"L": ["x", "y"]}, "0=x;1=y;"),
    ("{{range .L}}{{.}}{{else}}empty{{end}}", {"L": []}, "empty"),
    ("{{with .A}}{{.}}{{else}}none{{end}}", {"A": ""}, "none"),
    ("{{or .A .B}}|{{and .A .B}}", {"A": 0, "B": "z"}, "z|0"),
    ('{{printf "%q" .S}}', {"S": 'a"b'}, '"a\\"b"'),
    ('{{printf "%5d|%-4s|%x" 42 "ab" 255}}', {}, "   42|ab  |ff"),
    ("{{eq .A 1 2 3}}", {"A": 3}, "true"),
    ('{{.A | printf "%s-%s" "x"}}', {"A": "y"}, "x-y"),
    ('{{define "t"}}[{{.}}]{{end}}{{template "t" .A}}', {"A": "q"}, "[q]"),
    ("a  {{- 1 -}}  b", {}, "a1b"),
    # fmt.Sprint: a space only between operands when neither is a string
    ('{{print 1 2 "a" 3 "b" "c"}}', {}, "1 2a3bc"),
    ('{{println 1 "a"}}', {}, "1 a\n"),
    ('{{html "<a&b>"}}|{{urlquery "a b&c"}}|{{js "a\'b"}}', {}, "&lt;a&amp;b&gt;|a+b%26c|a\\'b"),
    ("{{.M}}|{{.L}}", {"M": {"b": 1, "a": 2}, "L": [1, "x", True]}, "map[a:2 b:1]|[1 x true]"),
    ("{{$x := 1}}{{if true}}{{$x = 2}}{{end}}{{$x}}", {}, "2"),
    ('{{slice "abcdef" 1 3}}|{{.Missing}}', {}, "bc|<no value>"),
    ("{{ 3.5 }} {{ 1e3 }} {{ 0x10 }} {{ 'a' }}", {}, "3.5 1000 16 97"),
    # fmt's bad-verb and nil renderings
    ('{{printf "%d|%d|%d" true 1.5 "x"}}', {}, "%!d(bool=true)|%!d(float64=1.5)|%!d(string=x)"),
    ('{{printf "%s|%s|%t|%t" 5 true 1 false}}', {}, "%!s(int=5)|%!s(bool=true)|%!t(int=1)|false"),
    ('{{printf "%T %T %T %T" 1 "a" .M .L}}', {"M": {}, "L": []}, "int string map[string]interface {} []interface {}"),
    ('{{printf "%v|%d|%s" nil nil nil}}', {}, "<nil>|%!d(<nil>)|%!s(<nil>)"),
    ('{{printf "%05d|%-3d|%3s" 42 7 "ab"}}', {}, "00042|7  | ab"),
    ('{{printf "%.2f|%e|%g" 3.14159 1234.5 0.000001}}', {}, "3.14|1.234500e+03|1e-06"),
]


@pytest.mark.parametrize("src,data,want", GO_TEMPLATE_CASES)
def test_go_template_semantics(src, data, want):
    from move2kube_amd.utils.gotemplate import Template
    assert Template(src).execute(data) == want


# plain scalar -> (go-yaml v3 value, go-yaml v2 value) decoding into interface{}
GO_YAML_SCALARS = [
    ("22:22", "22:22", "22:22"),        # no YAML 1.1 base-60 ints in go-yaml
    ("190:20:30", "190:20:30", "190:20:30"),
    ("1:30.5", "1:30.5", "1:30.5"),
    ("1e3", 1000.0, 1000.0),            # yamlStyleFloat: exponent without a dot
    ("0o17", 15, 15),
    ("0777", 511, 511),                 # ParseInt base 0: leading 0 is octal
    ("09", 9.0, 9.0),                   # not octal -> yamlStyleFloat
    ("1__0", 10, 10),                   # every '_' removed first
    ("0x_1F", 31, 31),
    ("_1", "_1", "_1"),
    ("+12", 12, 12),
    (".5", 0.5, 0.5),
    ("1.", 1.0, 1.0),
    ("1e400", "1e400", "1e400"),        # ParseFloat range error -> string
    ("18446744073709551615", 18446744073709551615, 18446744073709551615),   # uint64
    ("2001-12-14", "2001-12-14", "2001-12-14"),   # timestamps stay strings
    ("yes", "yes", True),
    ("Off", "Off", False),
    ("y", "y", True),
    ("TRUE", True, True),
    ("1.2.3", "1.2.3", "1.2.3"),
]


@pytest.mark.parametrize("text,v3,v2", GO_YAML_SCALARS)
def test_go_yaml_scalar_resolution(text, v3, v2):
    assert yamlio.load("a: " + text)["a"] == v3
    assert yamlio.load_v2("a: " + text)["a"] == v2
    # the emitter agrees with the v3 decoder about which strings need quotes
    if isinstance(v3, str):
        assert yamlio.load(yamlio.dump({"a": text}))["a"] == text


def test_go_yaml_special_floats():
    import math
    assert math.isnan(yamlio.load("a: .NaN")["a"])
    assert yamlio.load("a: -.inf")["a"] == float("-inf")
    assert yamlio.load("a: +.Inf")["a"] == float("inf")
