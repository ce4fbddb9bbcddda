"""Go 1.15 ``fmt.Sprintf`` (``utils/gofmt.py``), case by case.

No Go toolchain is available here, so every expected value is derived from
the Go 1.15 source named next to it (``src/fmt/print.go``,
``src/fmt/format.go``, ``src/strconv/quote.go``, ``src/strconv/ftoa.go``);
parity beyond those sources is unpinned.  Arguments are the Python values
that stand for Go values (``float`` is float64, a JSON number; ``int`` is
int; ``None`` a nil interface; lists ``[]interface {}``; dicts
``map[string]interface {}``).
"""

import math

import pytest

from move2kube_amd.utils import gofmt
from move2kube_amd.utils.gotemplate import go_sprintf

INF = math.inf

CASES = [
    # -- integers: format.go fmtInteger ---------------------------------------
    ("%d", [42], "42"),
    ("%+d", [42], "+42"),                                   # f.plus
    ("% d", [42], " 42"),                                   # f.space
    ("%05d", [-42], "-0042"),                               # zero pad leaves room for the sign
    ("%-5d|", [42], "42   |"),                              # f.minus
    ("%-+5d|", [3], "+3   |"),
    ("%x|%X|%#x|%#X", [255, 255, 255, 255], "ff|FF|0xff|0XFF"),
    ("%#08x", [255], "0x000000ff"),                         # zero padding is a precision, then 0x
    ("%x", [-255], "-ff"),
    ("%o|%#o|%O", [8, 8, 8], "10|010|0o10"),                # Go 1.13 %O
    ("%b|%#b", [5, 5], "101|0b101"),
    ("%.3d|%.0d|%5.0d|", [7, 0, 0], "007||     |"),         # precision 0 and value 0 print nothing
    ("%c|%c", [65, 0x1F600], "A|\U0001F600"),               # fmtC
    ("%c", [-1], "�"),                                 # > MaxRune -> RuneError
    ("%q|%q|%+q", [65, 0x263A, 0x263A], "'A'|'☺'|'\\u263a'"),   # fmtQc: QuoteRune / ToASCII
    ("%U|%U|%#U", [65, 0x1F600, 0x263A], "U+0041|U+1F600|U+263A '☺'"),   # fmtUnicode
    # -- floats: format.go fmtFloat, strconv.FormatFloat ----------------------
    ("%8.3f|%-8.3f|", [3.14159, 3.14159], "   3.142|3.142   |"),
    ("%08.3f", [-3.14159], "-003.142"),                     # sign written before the zero padding
    ("%+.2f|% .2f", [3.0, 3.0], "+3.00| 3.00"),
    ("%e|%E", [1234.5678, 1234.5678], "1.234568e+03|1.234568E+03"),
    ("%e", [0.0], "0.000000e+00"),
    ("%.0f|%.0f", [2.5, 3.5], "2|4"),                       # round half to even (exact decimal)
    ("%g|%g|%g|%v", [1e21, 100000.0, 1000000.0, 1e-7], "1e+21|100000|1e+06|1e-07"),   # shortest, eprec 6
    ("%.3g|%.3g|%G", [1234.0, 0.0001234, 1e-10], "1.23e+03|0.000123|1E-10"),
    ("%v|%v|%v", [8080.0, 0.5, -0.0], "8080|0.5|-0"),
    ("%6.2v|", [3.14159], "   3.1|"),                       # %v with a precision is %g
    ("%x|%X|%.1x|%x", [1.0, 3.0, 1.0, 0.0], "0x1p+00|0X1.8P+01|0x1.0p+00|0x0p+00"),   # ftoa.go fmtX
    ("%b", [1.0], "4503599627370496p-52"),                  # ftoa.go fmtB
    ("%#g|%#.3g|%#v", [1.0, 2.0, 1.0], "1.00000|2.00|1"),   # sharp keeps trailing zeros
    ("%v|%f|%+f|%06v|", [INF, math.nan, math.nan, INF], "+Inf|NaN|+NaN|  +Inf|"),   # no zero pad for Inf/NaN
    ("%F", [1.5], "1.500000"),
    # -- strings: fmtS / fmtQ / fmtSbx -----------------------------------------
    ("%s|%.2s|%7s|", ["héllo", "héllo", "héllo"], "héllo|hé|  héllo|"),   # width and precision count runes
    ("%6.3s|", ["abcdef"], "   abc|"),
    ("%05s", ["ab"], "000ab"),                              # zero padding applies to strings too
    ("%q", ['a"b\n\x01\x7f'], '"a\\"b\\n\\x01\\u007f"'),    # strconv.Quote
    ("%q|%+q", ["héllo", "héllo"], '"héllo"|"h\\u00e9llo"'),
    ("%#q|%#q", ["ab", "a`b"], '`ab`|"a`b"'),              # CanBackquote
    ("%x|% x|%#x|%# x|%X", ["hi", "hi", "hi", "hi", "hi"], "6869|68 69|0x6869|0x68 0x69|6869"),
    ("%x", ["é"], "c3a9"),                                  # the string's UTF-8 bytes
    ("%v|%#v", ["x", "x"], 'x|"x"'),
    # -- bool ------------------------------------------------------------------
    ("%t|%v|%-6v|", [True, False, True], "true|false|true  |"),
    # -- bad verbs and operands: print.go badVerb -------------------------------
    ("%d|%d|%d", [True, 1.5, "x"], "%!d(bool=true)|%!d(float64=1.5)|%!d(string=x)"),
    ("%d|%s", [3.0, 8080.0], "%!d(float64=3)|%!s(float64=8080)"),   # JSON numbers are float64
    ("%q", [1.5], "%!q(float64=1.5)"),
    ("%z", [1], "%!z(int=1)"),
    ("%v|%s|%7v|", [None, None, None], "<nil>|%!s(<nil>)|  <nil>|"),
    ("%T|%T|%T|%10T|", [1.5, None, "s", 1], "float64|<nil>|string|       int|"),
    # -- composite values: print.go printValue ----------------------------------
    ("%v", [[1, "a", None]], "[1 a <nil>]"),
    ("%d|%03d", [[1, 2], [1, 2]], "[1 2]|[001 002]"),       # the verb applies to each element
    ("%s", [["a", 1]], "[a %!s(int=1)]"),
    ("%q|%x", [["a", "b"], ["hi", 255]], '["a" "b"]|[6869 ff]'),
    ("%v", [{"b": 1, "a": [1]}], "map[a:[1] b:1]"),         # fmtsort: keys in order
    ("%#v", [{"b": 1, "a": [1]}], 'map[string]interface {}{"a":[]interface {}{1}, "b":1}'),
    ("%#v|%#v|%#v", [42, [None], None], "42|[]interface {}{interface {}(nil)}|<nil>"),
    ("%d", [[None]], "[<nil>]"),                            # a nil interface element prints <nil> for any verb
    # -- argument handling: doPrintf / argNumber / intFromArg -------------------
    ("%[2]d %[1]d", [1, 2], "2 1"),
    ("%[3]*.[2]*[1]f", [12.0, 2, 6], " 12.00"),             # the print.go documentation example
    ("%[3]d", [1], "%!d(BADINDEX)"),
    ("%*d|%-*d|%*d|", [5, 42, 3, 7, -3, 7], "   42|7  |7  |"),   # negative width means '-'
    ("%*d", ["x", 7], "%!(BADWIDTH)7"),
    ("%.*f|%.*d", [2, 3.14159, -1, 5], "3.14|%!(BADPREC)5"),   # a negative precision is BADPREC
    ("%d %d", [1], "1 %!d(MISSING)"),
    ("%d", [1, 2], "1%!(EXTRA int=2)"),
    ("%d", [1, "a", None, [1]], "1%!(EXTRA string=a, <nil>, []interface {}=[1])"),
    ("abc%", [], "abc%!(NOVERB)"),
    ("%%|%5%|%-%", [], "%|%|%"),                            # %% ignores width and absorbs no operand
    ("%!", [1], "%!!(int=1)"),
    ("%[1]d %d", [1, 2], "1 2"),                            # after an index, the next arg follows it
    ("%[2]d", [1, 2], "2"),                                 # reordered: no EXTRA check
]


@pytest.mark.parametrize("fmt,args,want", CASES, ids=[c[0] for c in CASES])
def test_sprintf(fmt, args, want):
    assert go_sprintf(fmt, args) == want


def test_case_count():
    assert len(CASES) >= 60


@pytest.mark.parametrize("args,want", [
    ([1, 2, "a", 3, "b", "c"], "1 2a3bc"),       # print.go doPrint: a space between two non-strings
    ([None, None], "<nil> <nil>"),
    (["a", None], "a<nil>"),
    ([1.5, [1]], "1.5 [1]"),
])
def test_sprint(args, want):
    assert gofmt.sprint(args) == want


def test_sprintln():
    assert gofmt.sprintln(["a", 1, None]) == "a 1 <nil>\n"


@pytest.mark.parametrize("s,want", [
    ("abc", '"abc"'),
    ("a\tb", '"a\\tb"'),
    ("\a\b\f\v\r", '"\\a\\b\\f\\v\\r"'),
    ("­", '"\\u00ad"'),              # soft hyphen is not printable (IsPrint Latin-1 table)
    (" ", '"\\u2028"'),              # line separator: Zl
    ("\U0001F600", '"\U0001F600"'),       # printable beyond the BMP
    ("\udcff", '"\\xff"'),                # a byte that was not UTF-8
    ("\\", '"\\\\"'),
])
def test_strconv_quote(s, want):
    assert gofmt.quote(s) == want


@pytest.mark.parametrize("v,fmt,prec,want", [
    (123456789.0, "g", -1, "1.23456789e+08"),
    (0.000012, "g", -1, "1.2e-05"),
    (0.0001, "g", -1, "0.0001"),
    (123.0, "e", 2, "1.23e+02"),
    (5e-324, "g", -1, "5e-324"),
    (1.7976931348623157e308, "g", -1, "1.7976931348623157e+308"),
    (0.1, "x", -1, "0x1.999999999999ap-04"),
    (1.0, "x", 0, "0x1p+00"),
    (1.5, "x", 0, "0x1p+01"),             # 0x1.8 rounds half to even: up to 0x2p+00 = 0x1p+01
    (2.0 ** 100, "x", -1, "0x1p+100"),
    (-2.0, "b", -1, "-4503599627370496p-51"),
])
def test_strconv_format_float(v, fmt, prec, want):
    assert gofmt.format_float(v, fmt, prec) == want
