"""The closure-compiled Go template executor (utils/gotemplate.py, the
default) against the tree-walking interpreter it was derived from
(``M2K_TEMPLATE_INTERPRET=1``): same output, or the same error, on every
packaged template and on a corpus that covers every node and operand kind and
the error paths."""

import os

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from move2kube_amd.utils import gotemplate

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(ROOT, "move2kube_amd", "assets")


def _both(src, data, funcs=None):
    results = []
    for interpret in (True, False):
        old = gotemplate.INTERPRET, gotemplate.COMPILE_AFTER
        gotemplate.INTERPRET, gotemplate.COMPILE_AFTER = interpret, 0
        try:
            t = gotemplate.Template(src)  # a fresh tree each time: no compiled state shared
            results.append(("ok", t.execute(data, funcs)))
        except gotemplate.TemplateError as e:
            results.append(("error", str(e)))
        finally:
            gotemplate.INTERPRET, gotemplate.COMPILE_AFTER = old
    return results


def _packaged():
    out = []
    for dp, _, fns in os.walk(ASSETS):
        for fn in sorted(fns):
            if fn.endswith((".tpl", ".txt")) or fn in ("Dockerfile", "environment"):
                with open(os.path.join(dp, fn)) as f:
                    out.append((os.path.relpath(os.path.join(dp, fn), ASSETS), f.read()))
    return out


_DATA = [
    {},
    {"IsHelm": True, "ExposedServicePaths": {"api": "/api", "web": "/"}, "Project": "p", "NewImages": True,
     "Helm": True, "AddCopySourcesWarning": True, "Images": ["a", "b"], "RegistryURL": "quay.io",
     "RegistryNamespace": "ns", "IngressHost": "h.example.com", "Builder": "b", "ImageName": "img",
     "port": 8080, "app_name": "app", "binding": "0.0.0.0:8080", "main_script_rel_path": "main.py",
     "war_path": "x.war", "ant_cmd": "ant all", "app_file": "app.py", "RelRootDir": "..", "Dst": "containers",
     "Name": "chart"},
    {"IsHelm": False, "ExposedServicePaths": {}, "Images": [], "NewImages": False, "port": "80"},
]


@pytest.mark.parametrize("name,src", _packaged(), ids=[n for n, _ in _packaged()])
def test_packaged_templates(name, src):
    for data in _DATA:
        a, b = _both(src, data)
        assert a == b, (name, data)


_CORPUS = [
    '{{define "row"}}{{.}}|{{end}}{{block "b" .X}}[{{.}}]{{end}}{{range $i, $v := .L}}{{if eq $v 2}}{{continue}}'
    '{{else if eq $v 4}}{{break}}{{end}}{{template "row" $v}}{{end}}{{with .M}}{{.k}}{{else}}none{{end}}',
    '{{$x := (printf "%d-%s" 3 "z")}}{{$x = print $x "!"}}{{$x}} {{len .L | printf "%03d"}}',
    '{{range .M}}{{.}}{{else}}empty{{end}}{{range $k, $v := .M}}{{$k}}={{$v}};{{end}}{{range 3}}{{.}}{{end}}',
    '{{if and .A .B}}both{{else if or .A .B}}one{{else}}none{{end}}{{not .A}}',
    '{{index .L 1}} {{index .M "k"}} {{slice .S 1 3}} {{len .S}} {{html "<a&b>"}} {{js "x\'y"}} {{urlquery "a b"}}',
    '{{.Missing}} {{.M.missing}} {{.M.k.deeper}}',
    '{{nil | print}} {{true}} {{1.5}} {{0x1F}} {{-3}} {{\'a\'}} {{`raw`}}',
    '{{template "nope"}}',
    '{{.L.x}}',
    '{{$u}}',
    '{{$u = 1}}',
    '{{nofunc 1}}',
    '{{index .L 9}}',
    '{{range .S}}{{.}}{{end}}',
    '{{.A 1}}',
    '{{1 | .A}}',
    '{{call .F 2}} {{call .F}}',
    '{{$a := 1}}{{if true}}{{$a := 2}}{{$a}}{{end}}{{$a}}',
    '{{with $v := .M}}{{$v.k}}{{end}}{{range $i := .L}}{{$i}}{{end}}',
    '{{eq .A 1 2 true}}',
    '{{lt 1 "a"}}',
    '{{printf "%v %q %5.2f %x" .L "s" 3.14159 255}}',
    '{{- " trimmed " -}} {{/* c */}} x',
]
_CORPUS_DATA = {"A": True, "B": False, "L": [1, 2, 3, 4, 5], "M": {"k": "v", "z": 2}, "S": "hello", "X": "x",
                "F": lambda *a: "f%d" % len(a)}


@pytest.mark.parametrize("src", _CORPUS)
def test_corpus_agrees(src):
    a, b = _both(src, _CORPUS_DATA)
    assert a == b


_PIECES = ["text ", "{{.A}}", "{{.L}}", "{{.M.k}}", "{{$}}", "{{len .L}}", "{{index .L 0}}",
           "{{if .A}}", "{{if .B}}", "{{else}}", "{{end}}", "{{range .L}}", "{{range $i, $v := .M}}", "{{with .M}}",
           "{{$x := .S}}", "{{$x}}", "{{$x = 1}}", "{{.}}", "{{print . .A}}", "{{else if .A}}",
           "{{printf \"%v\" .}}", "{{- \" \" -}}", "{{not .}}", "{{eq . 2}}", "{{eq . 2.0}}", "{{lt . \"a\"}}",
           "{{index .M \"z\"}}", "{{.M.k.x}}", "{{(.M).k}}", "{{and .A .Missing}}", "{{template \"t\" .}}",
           "{{define \"t\"}}<{{.}}>{{end}}", "{{nil}}", "{{$i}}"]


@settings(max_examples=300, deadline=None)
@given(st.lists(st.sampled_from(_PIECES), max_size=12))
def test_random_templates_agree(pieces):
    src = "".join(pieces)
    try:
        gotemplate.Template(src)
    except gotemplate.TemplateError:
        return  # does not parse: nothing to execute
    a, b = _both(src, _CORPUS_DATA)
    assert a == b, src


def test_break_and_continue_are_not_go115_keywords():
    # Go 1.15's lexer has no break/continue keywords (parse/lex.go key map;
    # they came with Go 1.18): the parser sees an undefined function
    for src in ("{{break}}", "{{range .L}}{{continue}}{{end}}"):
        with pytest.raises(gotemplate.TemplateError, match='function "(break|continue)" not defined'):
            gotemplate.Template(src)


def test_undefined_template_error_text():
    # exec.go walkTemplate + ErrorContext: the name token's position, the
    # node's String() cut to 20 runes
    want = 'template: :1:11: executing "" at <{{template "nope" .}...>: template "nope" not defined'
    assert [r for r in _both('{{template "nope" .}}', {})] == [("error", want)] * 2


def test_a_template_is_compiled_on_its_second_execution():
    t = gotemplate.Template("{{range .L}}{{.}}{{end}}")
    assert t.execute({"L": [1, 2]}) == "12" and "_run" not in t.__dict__
    assert t.execute({"L": [3]}) == "3" and "_run" in t.__dict__
    assert t.execute({"L": []}) == ""
