"""Go 1.15 ``fmt`` (``Sprintf`` / ``Sprint`` / ``Sprintln``) and the
``strconv`` quoting and float formatting it relies on.

The reference is built with go1.15 (``/root/reference/go.mod:3``,
``/root/reference/Dockerfile:20``).  Its templates call ``printf``/``print``
(``text/template`` maps them to ``fmt.Sprintf``/``fmt.Sprint``), and its log
lines are ``fmt`` formats, so this module follows the Go 1.15 sources verb for
verb: ``src/fmt/print.go`` (``doPrintf``, ``printArg``, ``printValue``,
``badVerb``, ``argNumber``, ``intFromArg``), ``src/fmt/format.go``
(``fmtInteger``, ``fmtFloat``, ``fmtQ``, ``fmtSbx``, ``fmtUnicode``, ``pad``)
and ``src/strconv`` (``quote.go``: ``Quote``/``QuoteRune``/``CanBackquote``;
``ftoa.go``: ``%e %f %g %b %x`` of a float64).  No Go toolchain is available
here, so parity beyond those sources is unpinned; ``tests/test_gofmt.py``
cites the source line each expected value follows.

Values: Python stands in for the Go values a template or a JSON document
produces -- ``None`` is a nil interface, ``bool``/``int``/``float``/``complex``/
``str`` are ``bool``/``int``/``float64``/``complex128``/``string``,
:class:`GoUint8` is a ``uint8`` (a byte indexed out of a string), ``bytes`` a
``[]byte``, ``list``/``tuple`` a ``[]interface {}``, ``dict`` a
``map[string]interface {}``, any other object a struct (its ``vars()``).
``NO_VALUE`` is the zero ``reflect.Value`` (a missing map key).
"""

import math
import struct

LDIGITS = "0123456789abcdefx"
UDIGITS = "0123456789ABCDEFX"
_MASK64 = (1 << 64) - 1
_MAX_RUNE = 0x10FFFF
_RUNE_ERROR = 0xFFFD


class _NoValue:
    """The zero reflect.Value (a missing map key): prints ``<no value>``."""

    __slots__ = ()

    def __repr__(self):
        return "<no value>"

    def __bool__(self):
        return False


NO_VALUE = _NoValue()


class GoUint8(int):
    """A Go ``uint8``: what ``index`` returns for a string (one byte)."""

    __slots__ = ()


# ---------------------------------------------------------------------------
# Types
# ---------------------------------------------------------------------------

_TYPE_NAMES = {bool: "bool", int: "int", float: "float64", complex: "complex128", str: "string",
               GoUint8: "uint8", bytes: "[]uint8", bytearray: "[]uint8", list: "[]interface {}",
               tuple: "[]interface {}", dict: "map[string]interface {}"}


def type_string(v):
    """``reflect.TypeOf(v).String()`` of a value (``%T``); ``<nil>`` for nil."""
    if v is None or v is NO_VALUE:
        return "<nil>"
    name = _TYPE_NAMES.get(type(v))
    if name is not None:
        return name
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if isinstance(v, (list, tuple)):
        return "[]interface {}"
    if isinstance(v, dict):
        return "map[string]interface {}"
    if callable(v):
        return "func(...interface {}) interface {}"
    return type(v).__name__


def _sort_key(k):
    """internal/fmtsort order of map keys: numbers by value, strings by bytes."""
    if isinstance(k, (int, float)) and not isinstance(k, bool):
        return (0, k, "")
    if isinstance(k, bool):
        return (1, int(k), "")
    return (2, 0, k if isinstance(k, str) else str(k))


def sorted_keys(d):
    try:
        return sorted(d.keys())
    except TypeError:
        return sorted(d.keys(), key=_sort_key)


# ---------------------------------------------------------------------------
# strconv: quoting (src/strconv/quote.go)
# ---------------------------------------------------------------------------

def is_print(r):
    """strconv.IsPrint: letters, marks, numbers, punctuation, symbols and the
    ASCII space (quote.go: IsPrint; the Latin-1 fast path is exact, above it
    the categories of Python's Unicode tables stand in for Go 1.15's)."""
    if r <= 0xFF:
        return 0x20 <= r <= 0x7E or (0xA1 <= r <= 0xFF and r != 0xAD)
    if 0xD800 <= r <= 0xDFFF or r > _MAX_RUNE:
        return False
    import unicodedata
    return unicodedata.category(chr(r))[0] in "LMNPS"


_ESC = {7: "\\a", 8: "\\b", 12: "\\f", 10: "\\n", 13: "\\r", 9: "\\t", 11: "\\v"}


def _append_escaped_rune(out, r, quote, ascii_only):
    """quote.go: appendEscapedRune (graphicOnly false)."""
    if r == ord(quote) or r == 0x5C:
        out.append("\\" + chr(r))
        return
    if ascii_only:
        if r < 0x80 and is_print(r):
            out.append(chr(r))
            return
    elif is_print(r):
        out.append(chr(r))
        return
    e = _ESC.get(r)
    if e is not None:
        out.append(e)
    elif r < 0x20:
        out.append("\\x%02x" % r)
    else:
        if r > _MAX_RUNE:
            r = _RUNE_ERROR
        if r < 0x10000:
            out.append("\\u%04x" % r)
        else:
            out.append("\\U%08x" % r)


def quote_with(s, quote='"', ascii_only=False):
    """quote.go: appendQuotedWith.  A byte that was not UTF-8
    (surrogateescape, U+DC80..U+DCFF) is written ``\\xNN``."""
    if s.isascii() and s.isprintable() and quote not in s and "\\" not in s:
        return quote + s + quote
    out = [quote]
    for ch in s:
        r = ord(ch)
        if 0xDC80 <= r <= 0xDCFF:
            out.append("\\x%02x" % (r - 0xDC00))
            continue
        if 0xD800 <= r <= 0xDFFF:
            r = _RUNE_ERROR
        _append_escaped_rune(out, r, quote, ascii_only)
    out.append(quote)
    return "".join(out)


def quote(s):
    """strconv.Quote."""
    return quote_with(s, '"', False)


def quote_to_ascii(s):
    """strconv.QuoteToASCII."""
    return quote_with(s, '"', True)


def quote_rune(r, ascii_only=False):
    """strconv.QuoteRune / QuoteRuneToASCII (invalid runes become U+FFFD)."""
    if r < 0 or r > _MAX_RUNE or 0xD800 <= r <= 0xDFFF:
        r = _RUNE_ERROR
    out = ["'"]
    _append_escaped_rune(out, r, "'", ascii_only)
    out.append("'")
    return "".join(out)


def can_backquote(s):
    """strconv.CanBackquote."""
    for ch in s:
        r = ord(ch)
        if r >= 0x80:
            if r == 0xFEFF or 0xD800 <= r <= 0xDFFF:
                return False
            continue
        if (r < 0x20 and r != 9) or r == 0x60 or r == 0x7F:
            return False
    return True


def utf8_bytes(s):
    """The Go string's bytes (surrogateescape for bytes that were not UTF-8)."""
    return s.encode("utf-8", "surrogateescape")


# ---------------------------------------------------------------------------
# strconv: float formatting (src/strconv/ftoa.go)
# ---------------------------------------------------------------------------

def _shortest(a):
    """(digits, dp) of the shortest decimal that round-trips a (> 0):
    0.d1d2...dn x 10^dp, as ftoa.go's Ryu/Grisu shortest mode."""
    r = repr(a)
    mant, _, exp = r.partition("e")
    e = int(exp) if exp else 0
    ip, _, fp = mant.partition(".")
    if fp == "0":
        fp = ""
    digits = (ip + fp).lstrip("0")
    lead = len(ip + fp) - len((ip + fp).lstrip("0"))
    dp = len(ip) + e - lead
    digits = digits.rstrip("0")
    if not digits:
        return "0", 0
    return digits, dp


def _fmt_e(neg, digits, dp, prec, fmt):
    """ftoa.go: fmtE of a decimal (digits, dp) with prec digits after the point."""
    out = "-" if neg else ""
    out += digits[0] if digits else "0"
    if prec > 0:
        frac = digits[1:1 + prec]
        out += "." + frac + "0" * (prec - len(frac))
    exp = dp - 1 if digits and digits != "0" else 0
    out += fmt
    if exp < 0:
        out += "-"
        exp = -exp
    else:
        out += "+"
    out += "%02d" % exp
    return out


def _fmt_f(neg, digits, dp, prec):
    """ftoa.go: fmtF."""
    out = "-" if neg else ""
    if dp > 0:
        ip = digits[:dp]
        out += ip + "0" * (dp - len(ip))
    else:
        out += "0"
    if prec > 0:
        frac = []
        for i in range(1, prec + 1):
            j = dp + i - 1
            frac.append(digits[j] if 0 <= j < len(digits) else "0")
        out += "." + "".join(frac)
    return out


def _bits(v):
    b = struct.unpack("<Q", struct.pack("<d", v))[0]
    neg = b >> 63 != 0
    exp = (b >> 52) & 0x7FF
    mant = b & ((1 << 52) - 1)
    return neg, exp, mant


def _fmt_b(v):
    """ftoa.go: fmtB, -ddddp±ddd."""
    neg, exp, mant = _bits(v)
    if exp == 0:
        exp += 1
    else:
        mant |= 1 << 52
    exp += -1023
    exp -= 52
    return ("-" if neg else "") + str(mant) + "p" + ("+" if exp >= 0 else "") + str(exp)


def _fmt_x(v, prec, fmt):
    """ftoa.go: fmtX, -0x1.yyyyp±dd."""
    neg, exp, mant = _bits(v)
    if exp == 0:
        exp += 1
    else:
        mant |= 1 << 52
    exp += -1023
    if mant == 0:
        exp = 0
    mant <<= 60 - 52
    while mant != 0 and mant & (1 << 60) == 0:
        mant <<= 1
        exp -= 1
    if 0 <= prec < 15:
        shift = prec * 4
        extra = (mant << shift) & ((1 << 60) - 1)
        mant >>= 60 - shift
        if extra | (mant & 1) > 1 << 59:
            mant += 1
        mant <<= 60 - shift
        if mant & (1 << 61):
            mant >>= 1
            exp += 1
    hexd = "0123456789ABCDEF" if fmt == "X" else "0123456789abcdef"
    out = ["-"] if neg else []
    out += ["0", fmt, chr(ord("0") + ((mant >> 60) & 1))]
    mant = (mant << 4) & _MASK64
    if prec < 0 and mant != 0:
        out.append(".")
        while mant != 0:
            out.append(hexd[(mant >> 60) & 15])
            mant = (mant << 4) & _MASK64
    elif prec > 0:
        out.append(".")
        for _ in range(prec):
            out.append(hexd[(mant >> 60) & 15])
            mant = (mant << 4) & _MASK64
    out.append("P" if fmt == "X" else "p")
    if exp < 0:
        out.append("-")
        exp = -exp
    else:
        out.append("+")
    out.append("%02d" % exp if exp < 100 else str(exp))
    return "".join(out)


def format_float(v, fmt, prec):
    """strconv.FormatFloat(v, fmt, prec, 64) for fmt in ``b e E f g G x X``."""
    if v != v:
        return "NaN"
    if v in (math.inf, -math.inf):
        return "+Inf" if v > 0 else "-Inf"
    if fmt == "b":
        return _fmt_b(v)
    if fmt in "xX":
        return _fmt_x(v, prec, fmt)
    neg = math.copysign(1.0, v) < 0
    a = -v if neg else v
    if prec < 0:
        if a == 0:
            digits, dp = "0", 1
            nd = 1
        else:
            digits, dp = _shortest(a)
            nd = len(digits)
        if fmt in "eE":
            return _fmt_e(neg, digits if a else "0", dp, nd - 1, fmt)
        if fmt == "f":
            return _fmt_f(neg, digits if a else "", dp if a else 0, max(nd - dp, 0) if a else 0)
        # %g shortest: eprec 6
        exp = dp - 1 if a else 0
        if exp < -4 or exp >= 6:
            return _fmt_e(neg, digits, dp, nd - 1, "e" if fmt == "g" else "E")
        if a == 0:
            return "-0" if neg else "0"
        return _fmt_f(neg, digits, dp, max(nd - dp, 0))
    if fmt in "eE":
        s = "%.*e" % (prec, a)
        return ("-" if neg else "") + (s.upper() if fmt == "E" else s)
    if fmt == "f":
        return ("-" if neg else "") + "%.*f" % (prec, a)
    # %g / %G with a precision: Python's %g applies the same rule
    # (ftoa.go: %e when exp < -4 || exp >= eprec; trailing zeros dropped)
    if prec == 0:
        prec = 1
    s = "%.*g" % (prec, a)
    if fmt == "G":
        s = s.upper()
    return ("-" if neg else "") + s


def format_float_g(f):
    """strconv.FormatFloat(f, 'g', -1, 64): fmt's %v of a float64."""
    return format_float(f, "g", -1)


# ---------------------------------------------------------------------------
# The printer (src/fmt/print.go, src/fmt/format.go)
# ---------------------------------------------------------------------------


def _printer():
    from .gofmt_printer import _Printer
    return _Printer()



def sprintf(fmt, args):
    """fmt.Sprintf(fmt, args...)."""
    p = _printer()
    p.do_printf(fmt, args)
    return "".join(p.buf)


def sprint_one(v):
    """fmt.Sprint(v) of one operand (%v)."""
    t = type(v)
    if t is str:
        return v
    if t is int:
        return str(v)
    if t is bool:
        return "true" if v else "false"
    if t is float:
        if v != v or v in (math.inf, -math.inf):
            return "NaN" if v != v else ("+Inf" if v > 0 else "-Inf")
        return format_float(v, "g", -1)
    if v is None:
        return "<nil>"
    if v is NO_VALUE:
        return "<no value>"
    p = _printer()
    p.print_arg(v, "v")
    return "".join(p.buf)


def sprint(args):
    """fmt.Sprint: a space between operands when neither is a string."""
    out = []
    prev_string = False
    for i, a in enumerate(args):
        is_string = isinstance(a, str)
        if i > 0 and not is_string and not prev_string:
            out.append(" ")
        out.append(sprint_one(a))
        prev_string = is_string
    return "".join(out)


def sprintln(args):
    """fmt.Sprintln: spaces between all operands, a newline at the end."""
    return " ".join(sprint_one(a) for a in args) + "\n"
