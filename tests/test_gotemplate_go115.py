"""Go 1.15 ``text/template`` semantics (``utils/gotemplate.py``), case by case.

The reference renders user templates with ``template.New("").Parse`` and
``Execute`` (``internal/common/utils.go:347-374``) under go1.15
(``go.mod:3``).  No Go toolchain is here, so each expected value follows the
Go 1.15 source named next to it: ``text/template/funcs.go`` (builtins,
``basicKind``), ``exec.go`` (evaluation, ``evalField``, ``walkRange``,
``validateType``, ``idealConstant``, ``errorf`` / ``ErrorContext``),
``parse/parse.go`` and ``parse/lex.go``; parity beyond that source is
unpinned.  Data is what ``json.Unmarshal`` gives a detector's output: numbers
are float64 (Python floats), null is a nil interface (None).

Each case runs through the interpreter and the compiled closures.
"""

import os
import stat

import pytest

from move2kube_amd.utils import gotemplate

DATA = {"port": 8080.0, "s": "hi", "n": 2.0, "one": 1.0, "zero": 0.0, "b": True, "l": [1, 2, 3],
        "e": [], "m": {"k": "v", "z": 2}, "em": {}, "nullkey": None, "a": {"b": "v"}}

OK = "ok"
ERR = "error"   # an execution error; the expected value is the message after "executing ... at <...>: "
PARSE = "parse"  # a parse error; the expected value is the message after "template: :LINE: "

CASES = [
    # -- funcs.go eq/ne/lt/le/gt/ge: basicKind ----------------------------------
    ("{{if eq .port 8080}}a{{end}}", ERR, "error calling eq: incompatible types for comparison"),
    ("{{if eq .port 8080.0}}a{{end}}", OK, "a"),          # idealConstant: a "." makes a float64
    ("{{if eq .port 8080}}a{{else}}b{{end}}", ERR, "error calling eq: incompatible types for comparison"),
    ('{{eq .s "x" "hi"}}', OK, "true"),                    # eq a b c: a == b || a == c
    ("{{eq .l .l}}", ERR, "error calling eq: invalid type for comparison"),    # slices are not basic kinds
    ("{{eq .m .m}}", ERR, "error calling eq: invalid type for comparison"),
    ('{{eq .missing "x"}}', ERR, "error calling eq: invalid type for comparison"),   # the zero Value
    ('{{eq .nullkey "x"}}', ERR, "error calling eq: invalid type for comparison"),   # nil interface
    ("{{eq nil nil}}", ERR, "error calling eq: invalid type for comparison"),
    ('{{eq 1 "1"}}', ERR, "error calling eq: incompatible types for comparison"),
    ("{{eq .s}}", ERR, "error calling eq: missing argument for comparison"),
    ("{{eq .b true}}", OK, "true"),
    ("{{eq (index .s 0) 104}}", OK, "true"),              # uint8 against int: the sign special case
    ("{{lt true false}}", ERR, "error calling lt: invalid type for comparison"),   # bools do not order
    ('{{lt 1 2}} {{lt "a" "b"}} {{lt .one 2.5}}', OK, "true true true"),
    ("{{lt 1.5 2}}", ERR, "error calling lt: incompatible types for comparison"),
    ("{{le 2 2}} {{gt 3 2}} {{ge 2 3}} {{ne 1 2}}", OK, "true true false true"),
    ('{{ne "a" 1}}', ERR, "error calling ne: incompatible types for comparison"),
    ("{{ne 1}}", ERR, "wrong number of args for ne: want 2 got 1"),            # evalCall arity
    # -- parse.go / lex.go: what Go 1.15 rejects ----------------------------------
    ("{{break}}", PARSE, 'function "break" not defined'),                     # no break keyword before 1.18
    ("{{range .l}}{{continue}}{{end}}", PARSE, 'function "continue" not defined'),
    ("{{with .s}}x{{else with .n}}y{{end}}", PARSE, "unexpected <with> in else"),   # else-with is 1.23
    ("{{range .l}}x{{else if .b}}y{{end}}", PARSE, "unexpected <if> in input"),     # else-if only in if
    ("{{with .s}}x{{else if .b}}y{{end}}", PARSE, "unexpected <if> in input"),
    ("{{foo}}", PARSE, 'function "foo" not defined'),                         # checked while parsing
    ("{{if false}}{{foo}}{{end}}", PARSE, 'function "foo" not defined'),
    ("{{$x}}", PARSE, 'undefined variable "$x"'),
    ("{{if true}}{{$x := 1}}{{end}}{{$x}}", PARSE, 'undefined variable "$x"'),    # scope ends at {{end}}
    ("{{.s\n}}", PARSE, "unclosed action"),                                    # no newlines in actions (1.16)
    ("{{.s | 1}}", PARSE, "non executable command in pipeline stage 2"),
    ("{{true.x}}", PARSE, 'unexpected . after term "true"'),
    ("{{.s}}{{end}}", PARSE, "unexpected {{end}}"),
    ("{{if .s}}", PARSE, "unexpected EOF"),
    ('{{define "a"}}x{{end}}{{define "a"}}y{{end}}', PARSE, 'template: multiple definition of template "a"'),
    ("{{ /* c */ }}", PARSE, 'unexpected "/" in command'),                   # comments only right after {{
    ('{{"\\\'"}}', PARSE, "invalid syntax"),                                   # strconv.Unquote: \' in "..."
    ("{{99999999999999999999}}", PARSE, 'integer overflow: "99999999999999999999"'),   # newNumber
    ("{{$a, $b := .l}}", PARSE, "too many declarations in command"),
    ("{{range $a, 3}}{{end}}", PARSE, "range can only initialize variables"),
    ("{{if}}{{end}}", PARSE, "missing value for if"),
    ("{{.s.}}", PARSE, "unexpected <.> in operand"),
    # -- exec.go: walkRange / evalCommand / evalField ---------------------------
    ("{{range 3}}x{{end}}", ERR, "range can't iterate over 3"),              # range over an int is 1.22
    ("{{range .s}}x{{end}}", ERR, "range can't iterate over hi"),
    ("{{range .n}}x{{end}}", ERR, "range can't iterate over 2"),
    ("{{range .nullkey}}x{{else}}none{{end}}", OK, "none"),                  # nil: the else branch
    ("{{nil}}", ERR, "nil is not a command"),
    ('{{.missing | printf "%v"}}', OK, "<nil>"),           # a missing key given to a function is nil
    ('{{printf "%v" .missing}}|{{printf "%v" .nullkey}}', OK, "<nil>|<nil>"),
    ("{{.missing}}|{{.nullkey}}|{{.missing.x}}", OK, "<no value>|<no value>|<no value>"),
    ("{{.nullkey.x}}", ERR, "nil pointer evaluating interface {}.x"),
    ("{{.s.x}}", ERR, "can't evaluate field x in type interface {}"),
    ("{{.s 1}}", ERR, "s is not a method but has arguments"),
    ("{{1 | .s}}", ERR, "s is not a method but has arguments"),
    ('{{"a" "b"}}', ERR, 'can\'t give argument to non-function "a"'),
    ("{{.a.b}} {{(.m).k}} {{$.s}}", OK, "v v hi"),
    ('{{index .m "missing"}}|{{printf "%v" (index .m "missing")}}', OK, "<no value>|<nil>"),
    ("{{18446744073709551615}}", ERR, "18446744073709551615 overflows int"),   # idealConstant
    ('{{template "a"}}{{define "a"}}[{{.}}]{{end}}', OK, "[<no value>]"),   # no pipeline: no data
    ('{{block "b" .s}}<{{.}}>{{end}}', OK, "<hi>"),
    ("{{$x := 1}}{{$x = 2}}{{$x}}", OK, "2"),
    ("{{range $i, $v := .l}}{{$i}}:{{$v}} {{end}}", OK, "0:1 1:2 2:3 "),
    ("{{range $v := .e}}{{else}}{{$v}}{{end}}", OK, "[]"),   # the variable holds the whole value in else
    ("{{range $k, $v := .m}}{{$k}}={{$v}};{{end}}", OK, "k=v;z=2;"),
    ("{{with $x := .s}}{{$x}}{{.}}{{end}}", OK, "hihi"),
    ("{{if .zero}}y{{else}}n{{end}}{{if .em}}y{{else}}n{{end}}{{if .e}}y{{else}}n{{end}}", OK, "nnn"),
    ("{{$}}", OK, None),   # checked below: the whole map
    # -- funcs.go: the other builtins ---------------------------------------------
    ("{{len \"héllo\"}} {{index \"héllo\" 1}}", OK, "6 195"),              # a string's bytes
    ("{{slice .l 1}} {{slice .l 1 2}} {{slice \"abc\" 1}}", OK, "[2 3] [2] bc"),
    ("{{index .l 5}}", ERR, "error calling index: index out of range: 5"),
    ("{{index .l .one}}", ERR, "error calling index: cannot index slice/array with type float64"),
    ("{{index .m 1}}", ERR, "error calling index: value has type int; should be string"),
    ("{{slice .l 2 1}}", ERR, "error calling slice: invalid slice index: 2 > 1"),
    ('{{slice "abc" 0 1 2}}', ERR, "error calling slice: cannot 3-index slice a string"),
    ("{{len .n}}", ERR, "error calling len: len of type float64"),
    ("{{and 1 0 .s}} {{or 0 \"\" \"z\"}} {{not .l}}", OK, "0 z false"),
    ("{{and 0 .nullkey.x}}", ERR, "nil pointer evaluating interface {}.x"),   # 1.15: no short circuit
    ("{{html \"<a href='x'>\\\"&\"}}", OK, "&lt;a href=&#39;x&#39;&gt;&#34;&amp;"),   # HTMLEscape
    ("{{html .missing}}", OK, "&lt;no value&gt;"),        # evalArgs: a nil operand prints <no value>
    ('{{urlquery "a b/c?d"}}', OK, "a+b%2Fc%3Fd"),
    ('{{print 1 2}} {{print "a" 1 2 "b"}}', OK, "1 2 a1 2b"),
    ("{{println .missing}}", OK, "<nil>\n"),
    ("{{printf}}", ERR, "wrong number of args for printf: want at least 1 got 0"),
    ("{{printf 3}}", ERR, "expected string; found 3"),     # evalString
    ("{{printf .n}}", ERR, "wrong type for value; expected string; got float64"),   # validateType
    ("{{printf .missing}}", ERR, "invalid value; expected string"),
    ("{{printf nil}}", ERR, "cannot assign nil to string"),
    ("{{not}}", ERR, "wrong number of args for not: want 1 got 0"),
    ('{{printf "%d %s %v" .n .port .l}}', OK, "%!d(float64=2) %!s(float64=8080) [1 2 3]"),
    ('{{index .m "k" | printf "%q"}}', OK, '"v"'),
    # -- literals: newNumber / idealConstant / strconv.Unquote -------------------
    ('{{"\\u00e9\\x41\\101"}}', OK, "éAA"),
    ("{{'\\n'}} {{'a'}}", OK, "10 97"),
    ("{{0x10}} {{1e2}} {{1_000}} {{017}} {{0o17}} {{-3}} {{.5}}", OK, "16 100 1000 15 15 -3 0.5"),
    ("{{1i}}", OK, "(0+1i)"),
    ("{{`a\rb`}}", OK, "ab"),                             # Unquote drops \r from raw strings
    # -- lex.go trimming and comments ----------------------------------------------
    ("a  {{- .s -}}  b", OK, "ahib"),
    ("a {{- /* c\n d */ -}} b", OK, "ab"),
    ("{{.s  -}} x", OK, "hix"),
]


def _run(src, data, interpret):
    old = gotemplate.INTERPRET, gotemplate.COMPILE_AFTER
    gotemplate.INTERPRET, gotemplate.COMPILE_AFTER = interpret, 0
    try:
        t = gotemplate.Template(src)
    except gotemplate.TemplateError as e:
        return ("parse", str(e))
    finally:
        gotemplate.INTERPRET, gotemplate.COMPILE_AFTER = old
    gotemplate.INTERPRET, gotemplate.COMPILE_AFTER = interpret, 0
    try:
        return ("ok", t.execute(data))
    except gotemplate.TemplateError as e:
        return ("error", str(e))
    finally:
        gotemplate.INTERPRET, gotemplate.COMPILE_AFTER = old


@pytest.mark.parametrize("src,kind,want", CASES, ids=[c[0][:40] for c in CASES])
@pytest.mark.parametrize("interpret", [True, False], ids=["interpreted", "compiled"])
def test_go115_semantics(src, kind, want, interpret):
    got_kind, got = _run(src, DATA, interpret)
    assert got_kind == kind, (src, got)
    if want is None:
        return
    if kind == OK:
        assert got == want
    elif kind == ERR:
        assert got.startswith('template: :1:') and ': executing "" at <' in got, got
        assert got.split(">: ", 1)[1] == want
    else:
        assert got.startswith("template: :"), got
        assert got.split(": ", 2)[2] == want, got


def test_case_count():
    assert len(CASES) >= 80


def test_whole_data_prints_as_a_go_map():
    assert _run("{{$}}", {"b": 1.0, "a": [1.0, None]}, False) == ("ok", "map[a:[1 <nil>] b:1]")


@pytest.mark.parametrize("src,want", [
    # exec.go errorf + parse.Tree.ErrorContext: line, byte column (on line 1 the
    # column is the byte offset itself), the node's String() cut to 20 runes
    ("{{if eq .port 8080}}x{{end}}",
     'template: :1:5: executing "" at <eq .port 8080>: error calling eq: incompatible types for comparison'),
    ("a\n{{if eq .port 8080}}x{{end}}",
     'template: :2:5: executing "" at <eq .port 8080>: error calling eq: incompatible types for comparison'),
    ("é{{lt 1 \"a\"}}",
     'template: :1:4: executing "" at <lt 1 "a">: error calling lt: incompatible types for comparison'),
    ('{{printf "%d" .port | printf "%s" | eq 1}}',
     'template: :1:36: executing "" at <eq 1>: error calling eq: incompatible types for comparison'),
    # a field chain .x.y is positioned at its second field (parse.go operand: newChain(t.peek().pos))
    ('{{define "t"}}{{.x.y}}{{end}}{{template "t" .}}',
     'template: :1:18: executing "t" at <.x.y>: nil pointer evaluating interface {}.y'),
    # exec.go walkTemplate: unbounded {{template}} recursion stops at maxExecDepth,
    # reported at the call inside the recursing template, positioned at its
    # name token (parse.go templateControl: newTemplate(token.pos, ...)); this
    # stack runs out before depth 100000: the text is Go's, the depth is not
    ('{{define "a"}}x{{template "a" .}}{{end}}{{template "a" .}}',
     'template: :1:26: executing "a" at <{{template "a" .}}>: exceeded maximum template depth (100000)'),
])
def test_error_location_and_context(src, want):
    data = {"port": 8080.0, "x": None}
    for interpret in (True, False):
        assert _run(src, data, interpret) == ("error", want)


def test_parse_error_line():
    assert _run("a\nb\n{{foo}}", {}, False) == ("parse", 'template: :3: function "foo" not defined')


# -- end to end: a user detector whose Dockerfile template Go rejects ----------

DETECT = """#!/bin/sh
if [ -f "$1/app.txt" ]; then echo '{"port": 8080, "name": "web"}'; else exit 1; fi
"""


def _translate_with_detector(tmp_path, monkeypatch, template):
    from move2kube_amd import api
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = tmp_path / "src"
    (src / "app").mkdir(parents=True)
    (src / "app" / "app.txt").write_text("x\n")
    det = src / "detectors" / "mine"
    det.mkdir(parents=True)
    (det / "m2kdfdetect.sh").write_text(DETECT)
    os.chmod(str(det / "m2kdfdetect.sh"), stat.S_IRWXU)
    (det / "Dockerfile").write_text(template)
    with api.Session(qaskip=True) as session:
        out = session.translate(str(src), str(tmp_path / "out"), name="p")
    found = []
    for dp, _, fns in os.walk(out):
        for fn in fns:
            if fn.startswith("Dockerfile."):
                found.append(os.path.join(dp, fn))
    return found


def test_user_detector_template_go_rejects_writes_an_empty_dockerfile(tmp_path, monkeypatch, capsys):
    # dockerfilecontainerizer.go:113-127: the JSON port is float64, the
    # literal 8080 an int, so eq fails; the reference logs "Template
    # conversion failed" and writes the Dockerfile with empty contents
    found = _translate_with_detector(tmp_path, monkeypatch, "FROM x\n{{if eq .port 8080}}EXPOSE 8080{{end}}\n")
    err = capsys.readouterr().err
    assert "Template conversion failed" in err
    assert "incompatible types for comparison" in err
    assert len(found) == 1 and open(found[0]).read() == ""


def test_user_detector_template_go_accepts_renders(tmp_path, monkeypatch, capsys):
    found = _translate_with_detector(tmp_path, monkeypatch,
                                     "FROM x\n{{if eq .port 8080.0}}EXPOSE {{.port}}{{end}} {{printf \"%q\" .name}}\n")
    assert "Template conversion failed" not in capsys.readouterr().err
    assert len(found) == 1 and open(found[0]).read() == 'FROM x\nEXPOSE 8080 "web"\n'


def test_user_detector_template_nested_beyond_the_stack_fails_cleanly(tmp_path, monkeypatch, capsys):
    """Go's parser has no nesting limit (its stacks grow); this one stops at
    the interpreter's recursion limit.  Such a template is a template error
    (logged, empty Dockerfile), not a crash of the command (DEVIATIONS.md 6)."""
    deep = "FROM x\n{{" + "(" * 2000 + ".port" + ")" * 2000 + "}}\n"
    with pytest.raises(gotemplate.TemplateError, match="nested too deeply to parse"):
        gotemplate.Template(deep)
    found = _translate_with_detector(tmp_path, monkeypatch, deep)
    err = capsys.readouterr().err
    assert "Template conversion failed" in err and "nested too deeply" in err
    assert len(found) == 1 and open(found[0]).read() == ""
