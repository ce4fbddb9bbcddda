"""The Go 1.15 ``text/template`` lexer (``gotemplate._lex``): item kinds,
values and positions as ``src/text/template/parse/lex.go`` produces them, and
its error texts.  No Go toolchain is here: each case cites the lex.go code it
follows (parity beyond that source is unpinned)."""

import glob
import os

import pytest
from hypothesis import given, settings, strategies as st

from move2kube_amd.utils import gotemplate as g

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kinds(src):
    return [(k, v) for k, v, _ in g._lex(src) if k != g.I_SPACE]


@pytest.mark.parametrize("src,want", [
    # lexText / lexLeftDelim / lexRightDelim
    ("a{{.x}}b", [(g.I_TEXT, "a"), (g.I_LDELIM, "{{"), (g.I_FIELD, ".x"), (g.I_RDELIM, "}}"), (g.I_TEXT, "b"),
                  (g.I_EOF, "")]),
    # trim markers need a space or tab next to the dash (hasLeftTrimMarker / hasRightTrimMarker)
    ("a \n{{- 1 -}} \n b", [(g.I_TEXT, "a"), (g.I_LDELIM, "{{"), (g.I_NUMBER, "1"), (g.I_RDELIM, "}}"),
                            (g.I_TEXT, "b"), (g.I_EOF, "")]),
    # lexFieldOrVariable: ".a.b" is two field items, "$" alone is a variable
    ("{{.a.b $ $x.y}}", [(g.I_LDELIM, "{{"), (g.I_FIELD, ".a"), (g.I_FIELD, ".b"), (g.I_VARIABLE, "$"),
                         (g.I_VARIABLE, "$x"), (g.I_FIELD, ".y"), (g.I_RDELIM, "}}"), (g.I_EOF, "")]),
    # keywords of Go 1.15 (no break / continue), bools, nil, dot
    ("{{if true}}{{else}}{{end}}{{break}}", [
        (g.I_LDELIM, "{{"), (g.I_IF, "if"), (g.I_BOOL, "true"), (g.I_RDELIM, "}}"),
        (g.I_LDELIM, "{{"), (g.I_ELSE, "else"), (g.I_RDELIM, "}}"),
        (g.I_LDELIM, "{{"), (g.I_END, "end"), (g.I_RDELIM, "}}"),
        (g.I_LDELIM, "{{"), (g.I_IDENT, "break"), (g.I_RDELIM, "}}"), (g.I_EOF, "")]),
    # scanNumber: Go 1.13 literals, complex numbers
    ("{{0x1F 0b101 0o17 1_000 .5 1e3 0x1p-2 1i 1+2i -3}}", [
        (g.I_LDELIM, "{{"), (g.I_NUMBER, "0x1F"), (g.I_NUMBER, "0b101"), (g.I_NUMBER, "0o17"),
        (g.I_NUMBER, "1_000"), (g.I_NUMBER, ".5"), (g.I_NUMBER, "1e3"), (g.I_NUMBER, "0x1p-2"),
        (g.I_NUMBER, "1i"), (g.I_COMPLEX, "1+2i"), (g.I_NUMBER, "-3"), (g.I_RDELIM, "}}"), (g.I_EOF, "")]),
    # lexQuote / lexRawQuote / lexChar; punctuation; := and =
    ('{{$x := "a\\"b" `r\nr` \'c\' | ( ) , = }}', [
        (g.I_LDELIM, "{{"), (g.I_VARIABLE, "$x"), (g.I_DECLARE, ":="), (g.I_STRING, '"a\\"b"'),
        (g.I_RAWSTRING, "`r\nr`"), (g.I_CHARCONST, "'c'"), (g.I_PIPE, "|"), (g.I_LPAREN, "("),
        (g.I_RPAREN, ")"), (g.I_CHAR, ","), (g.I_ASSIGN, "="), (g.I_RDELIM, "}}"), (g.I_EOF, "")]),
    # lexComment: right after the delimiter, trim markers on both sides
    ("a {{- /* c\n */ -}} b", [(g.I_TEXT, "a"), (g.I_TEXT, "b"), (g.I_EOF, "")]),
    # two spaces before a trim-marked right delimiter (lexSpace backs up)
    ("{{1  -}} x", [(g.I_LDELIM, "{{"), (g.I_NUMBER, "1"), (g.I_RDELIM, "}}"), (g.I_TEXT, "x"), (g.I_EOF, "")]),
])
def test_items(src, want):
    assert kinds(src) == want


def test_positions_are_offsets_into_the_source():
    items = g._lex("ab{{ .x  | printf }}")
    assert [(k, p) for k, _, p in items if k in (g.I_LDELIM, g.I_FIELD, g.I_PIPE, g.I_IDENT, g.I_RDELIM)] == [
        (g.I_LDELIM, 2), (g.I_FIELD, 5), (g.I_PIPE, 9), (g.I_IDENT, 11), (g.I_RDELIM, 18)]


@pytest.mark.parametrize("src,err", [
    ("{{.x\n}}", "unclosed action"),                      # lexInsideAction: isEndOfLine (Go 1.15)
    ("{{.x", "unclosed action"),                          # eof
    ("{{/* x }}", "unclosed comment"),                    # lexComment
    ("{{/* x */ }}", "comment ends before closing delimiter"),
    ('{{"abc}}', "unterminated quoted string"),           # lexQuote
    ("{{`abc}}", "unterminated raw quoted string"),       # lexRawQuote
    ("{{'a}}", "unterminated character constant"),       # lexChar
    ("{{(1}}", "unclosed left paren"),
    ("{{1)}}", "unexpected right paren U+0029 ')'"),
    ("{{a:b}}", "expected :="),
    ("{{1x}}", 'bad number syntax: "1x"'),                # scanNumber: next must not be alphanumeric
    ("{{.x#}}", "bad character U+0023 '#'"),              # atTerminator
    ("{{\x01}}", "unrecognized character in action: U+0001"),
    ("{{-\n1}}", "unclosed action"),                      # "-\n" is no trim marker in Go 1.15
])
def test_lex_errors(src, err):
    items = g._lex(src)
    assert items[-1][0] == g.I_ERROR and items[-1][1] == err


def test_template_assets_lex_without_errors():
    files = sorted(glob.glob(os.path.join(ROOT, "move2kube_amd", "assets", "templates", "*")))
    files += sorted(glob.glob(os.path.join(ROOT, "move2kube_amd", "assets", "m2kassets", "**", "Dockerfile"),
                              recursive=True))
    assert files
    for f in files:
        with open(f) as fh:
            items = g._lex(fh.read())
        assert items[-1][0] == g.I_EOF, (f, items[-1])


_PIECES = st.sampled_from(["0x1F", "0b", "0o7", "0x", "1_0", "1.", ".5", "1.5e-3", "2e", "3i", "-", "+", "+.5",
                           "-1", "e5", "\"a\\\"b\"", "\"", "'c'", "''", "'\\", "`raw`", "`", "/*c*/", "/*", "/",
                           ":=", ":", "=", "|", "(", ")", ",", "$", "$x", "$x.Y", ".", ".A.b_1", "..", ".1", "abc",
                           "_x", " ", "\t", "\n", "é", "١", "\\", "*", "x0", "{{", "}}", "{{- ", " -}}"])


@settings(max_examples=1500, deadline=None)
@given(st.lists(_PIECES, min_size=1, max_size=8).map("".join))
def test_generated_inputs_end_in_eof_or_one_error(src):
    items = g._lex(src)
    assert items[-1][0] in (g.I_EOF, g.I_ERROR)
    assert all(k != g.I_ERROR for k, _, _ in items[:-1])
    # positions increase and point at the item's text
    last = -1
    for k, v, p in items:
        assert p >= last
        last = p
        if k not in (g.I_EOF, g.I_ERROR, g.I_TEXT):
            assert src.startswith(v, p), (src, k, v, p)
