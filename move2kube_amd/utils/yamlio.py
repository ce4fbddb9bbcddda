"""YAML reading and a byte-compatible re-implementation of go-yaml v3 output.

Every file the reference writes goes through ``gopkg.in/yaml.v3`` with
``SetIndent(2)`` (``internal/common/utils.go:159-177``,
``internal/transformer/transformer.go:162-204``).  Plans, QA caches, cluster
metadata and the generated Kubernetes manifests must round-trip
byte-for-byte (the reference's ``TestWritePlan`` compares bytes), so this
module re-implements the parts of the libyaml emitter that go-yaml v3 uses:

* scalar style selection (``yaml_emitter_analyze_scalar`` +
  ``yaml_emitter_select_scalar_style`` + go-yaml's ``stringv`` resolve check),
* block mappings/sequences with sequences indented under their key,
* literal block scalars with chomping/indentation hints,
* the natural key order go-yaml uses for Go maps (``sorter.go``).

Ordering model: a plain ``dict`` is emitted in insertion order (Go struct
field order) unless ``sort_maps=True``; a :class:`GoMap` is always sorted with
the go-yaml key comparator (Go maps).
"""

import functools
import math
import re
import threading
from .lazyre import lazy as _lazy_re

# PyYAML is imported on the first parse (``_lz()``), not at start-up: a CLI
# run over a source tree without YAML files never pays for it.

__all__ = [
    "GoMap", "dump", "dumps_k8s", "load", "load_raw", "load_all", "go_key_sorted",
    "YAMLError",
]


def __getattr__(name):
    # ``except yamlio.YAMLError`` only evaluates the name when an exception
    # reaches the clause, i.e. after a parse has imported PyYAML
    if name == "YAMLError":
        return _lz().yaml.YAMLError
    raise AttributeError(name)


class GoMap(dict):
    """A mapping that go-yaml would encode with sorted keys (a Go map)."""


# ---------------------------------------------------------------------------
# go-yaml key ordering (yaml.v3 sorter.go keyList.Less)
# ---------------------------------------------------------------------------

def _kind_rank(v):
    # reflect.Kind order used when kinds differ: Bool(1) < Int(2..) < Uint < Float(13/14) < String(24)
    if isinstance(v, bool):
        return 1
    if isinstance(v, int):
        return 2
    if isinstance(v, float):
        return 14
    if isinstance(v, str):
        return 24
    return 30


def _go_key_cmp(a, b):
    if not isinstance(a, str) or not isinstance(b, str):
        ka, kb = _kind_rank(a), _kind_rank(b)
        if ka != kb:
            return -1 if ka < kb else 1
        if isinstance(a, (int, float)) and isinstance(b, (int, float)):
            return (a > b) - (a < b)
        return 0
    ar, br = a, b
    digits = False
    n = min(len(ar), len(br))
    for i in range(n):
        if ar[i] == br[i]:
            digits = ar[i].isdigit()
            continue
        al = ar[i].isalpha()
        bl = br[i].isalpha()
        if al and bl:
            return -1 if ar[i] < br[i] else 1
        if al or bl:
            if digits:
                return -1 if al else 1
            return -1 if bl else 1
        an = bn = 0
        if ar[i] == "0" or br[i] == "0":
            j = i - 1
            while j >= 0 and ar[j].isdigit():
                if ar[j] != "0":
                    an = bn = 1
                    break
                j -= 1
        ai = i
        while ai < len(ar) and ar[ai].isdigit():
            an = an * 10 + (ord(ar[ai]) - 48)
            ai += 1
        bi = i
        while bi < len(br) and br[bi].isdigit():
            bn = bn * 10 + (ord(br[bi]) - 48)
            bi += 1
        if an != bn:
            return -1 if an < bn else 1
        if ai != bi:
            return -1 if ai < bi else 1
        return -1 if ar[i] < br[i] else 1
    return (len(ar) > len(br)) - (len(ar) < len(br))


_go_key = functools.cmp_to_key(_go_key_cmp)


def go_key_sorted(keys):
    """Sort keys the way go-yaml v3 sorts Go map keys."""
    return sorted(keys, key=_go_key)


# ---------------------------------------------------------------------------
# Plain-scalar resolution (what a plain scalar would decode to)
# ---------------------------------------------------------------------------

_YAML_FLOAT = _lazy_re(r"^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$")
_TIMESTAMP_FORMATS = [
    _lazy_re(r"^\d{4}-\d{1,2}-\d{1,2}[Tt]\d{1,2}:\d{1,2}:\d{1,2}(\.\d+)?(Z|[+-]\d{1,2}(:\d{2})?)$"),
    _lazy_re(r"^\d{4}-\d{1,2}-\d{1,2} \d{1,2}:\d{1,2}:\d{1,2}(\.\d+)?$"),
    _lazy_re(r"^\d{4}-\d{1,2}-\d{1,2}$"),
]
_NULLS = {"", "~", "null", "Null", "NULL"}
_BOOLS = {"true", "True", "TRUE", "false", "False", "FALSE"}
_OLD_BOOLS = {"y", "Y", "yes", "Yes", "YES", "on", "On", "ON",
              "n", "N", "no", "No", "NO", "off", "Off", "OFF"}
_SPECIAL_FLOATS = {".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF",
                   "-.inf", "-.Inf", "-.INF", ".nan", ".NaN", ".NAN"}
# characters a _YAML_FLOAT match can contain ("$" also matches before a final
# newline); a string with any other character is ruled out without the regex
_DROP_FLOAT_CHARS = str.maketrans("", "", "0123456789.eE+-\n")


def _maybe_float(s):
    return not s.translate(_DROP_FLOAT_CHARS)


_BASE60 = _lazy_re(r"^[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+(?:\.[0-9_]*)?$")


def _is_base60(s):
    return ":" in s and _BASE60.match(s) is not None


def _go_parse_int(s):
    """strconv.ParseInt(s, 0, 64) acceptance (after '_' removal)."""
    t = s
    if t[:1] in "+-":
        t = t[1:]
    if not t:
        return False
    low = t.lower()
    try:
        if low.startswith("0x"):
            int(t[2:], 16)
            return len(t) > 2
        if low.startswith("0o"):
            int(t[2:], 8)
            return len(t) > 2
        if low.startswith("0b"):
            int(t[2:], 2)
            return len(t) > 2
        if len(t) > 1 and t[0] == "0":
            int(t[1:], 8)
            return True
        if not t.isdigit():
            return False
        return True
    except ValueError:
        return False


def resolves_to_string(s):
    """True if ``s`` written as a plain scalar would decode back as a string."""
    if s in _NULLS or s in _BOOLS:
        return False
    if not s:
        return False
    c = s[0]
    if c.isdigit() or c in "+-.":
        if s in _SPECIAL_FLOATS:
            return False
        if c.isdigit() and len(s) >= 8 and s[4] == "-":  # every format starts \d{4}-
            for rx in _TIMESTAMP_FORMATS:
                if rx.match(s):
                    return False
        plain = s.replace("_", "")
        if _go_parse_int(plain):
            return False
        if _maybe_float(plain) and _YAML_FLOAT.match(plain):
            return False
        if c == "." :
            try:
                float(s)
                return False
            except ValueError:
                pass
    if s.startswith("<<") and s == "<<":
        return False
    return True


# ---------------------------------------------------------------------------
# libyaml scalar analysis
# ---------------------------------------------------------------------------

def _is_break(ch):
    return ch in "\r\n\x85  "


def _is_space(ch):
    return ch == " "


def _is_printable(ch):
    """yamlprivateh.go is_printable: NEL (U+0085) is not printable for the
    emitter (PyYAML's emitter counts it), so a string holding one is written
    double-quoted with ``\\N`` and reads back unchanged."""
    o = ord(ch)
    return (o == 0x0A or 0x20 <= o <= 0x7E or 0xA0 <= o <= 0xD7FF
            or 0xE000 <= o <= 0xFFFD and o != 0xFEFF or 0x10000 <= o <= 0x10FFFF)


def _analyze(value):
    """Return (multiline, block_plain_allowed, single_quoted_allowed, block_allowed)."""
    if value == "":
        return False, True, True, False
    block_indicators = flow_indicators = False
    line_breaks = special = tabs = False
    leading_space = leading_break = trailing_space = trailing_break = False
    break_space = space_break = False
    previous_space = previous_break = False
    if value.startswith("---") or value.startswith("..."):
        block_indicators = flow_indicators = True
    preceded_by_ws = True
    n = len(value)
    for i, ch in enumerate(value):
        followed_by_ws = i + 1 >= n or value[i + 1] in " \t\r\n\x85  "
        if i == 0:
            if ch in "#,[]{}&*!|>'\"%@`":
                flow_indicators = block_indicators = True
            elif ch in "?:":
                flow_indicators = True
                if followed_by_ws:
                    block_indicators = True
            elif ch == "-":
                if followed_by_ws:
                    flow_indicators = block_indicators = True
        else:
            if ch in ",?[]{}":
                flow_indicators = True
            elif ch == ":":
                flow_indicators = True
                if followed_by_ws:
                    block_indicators = True
            elif ch == "#":
                if preceded_by_ws:
                    flow_indicators = block_indicators = True
        if ch == "\t":
            tabs = True
        elif not _is_printable(ch):
            special = True
        if _is_space(ch):
            if i == 0:
                leading_space = True
            if i == n - 1:
                trailing_space = True
            if previous_break:
                break_space = True
            previous_space, previous_break = True, False
        elif _is_break(ch):
            line_breaks = True
            if i == 0:
                leading_break = True
            if i == n - 1:
                trailing_break = True
            if previous_space:
                space_break = True
            previous_space, previous_break = False, True
        else:
            previous_space = previous_break = False
        preceded_by_ws = ch in " \t\r\n\x85  \x00"
    block_plain = True
    single_quoted = True
    block_allowed = True
    if leading_space or leading_break or trailing_space or trailing_break:
        block_plain = False
    if trailing_space:
        block_allowed = False
    if break_space:
        block_plain = False
        single_quoted = False
    if space_break or tabs or special:
        block_plain = False
        single_quoted = False
    if space_break or special:
        block_allowed = False
    if line_breaks:
        block_plain = False
    if block_indicators:
        block_plain = False
    return line_breaks, block_plain, single_quoted, block_allowed


_ESCAPES = {
    "\x00": "\\0", "\x07": "\\a", "\x08": "\\b", "\t": "\\t", "\n": "\\n",
    "\x0b": "\\v", "\x0c": "\\f", "\r": "\\r", "\x1b": "\\e", '"': '\\"',
    "\\": "\\\\", "\x85": "\\N", "\xa0": "\\_", " ": "\\L", " ": "\\P",
}


def _double_quoted(s):
    out = ['"']
    for ch in s:
        if ch in _ESCAPES:
            out.append(_ESCAPES[ch])
        elif not _is_printable(ch) or ch == "﻿":
            o = ord(ch)
            if o <= 0xFF:
                out.append("\\x%02X" % o)
            elif o <= 0xFFFF:
                out.append("\\u%04X" % o)
            else:
                out.append("\\U%08X" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _single_quoted(s, indent=0):
    """emitterc.go write_single_quoted_scalar: quotes doubled; a break (LS or
    PS: LF and the unprintable ones never get this style) is written as
    itself and the next character starts after the indentation."""
    if "\u2028" not in s and "\u2029" not in s:
        return "'" + s.replace("'", "''") + "'"
    out = ["'"]
    breaks = False
    for ch in s:
        if ch in "\u2028\u2029":
            out.append(ch)
            breaks = True
            continue
        if breaks:
            out.append(" " * indent)
            breaks = False
        out.append("''" if ch == "'" else ch)
    out.append("'")
    return "".join(out)


PLAIN, SINGLE, DOUBLE, LITERAL = range(4)


# strings that libyaml's analysis always allows as block plain scalars: no
# indicators, no leading/trailing space, no breaks, printable ASCII only
_SIMPLE_SCALAR = _lazy_re(r"[A-Za-z0-9_/](?:[A-Za-z0-9_./ -]*[A-Za-z0-9_./-])?\Z")
_DROP_SIMPLE_CHARS = str.maketrans("", "", "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_./ -")


def _is_simple_scalar(s):
    """``_SIMPLE_SCALAR.match(s)`` with string operations (no compile in a cold process)."""
    return (s != "" and not s.translate(_DROP_SIMPLE_CHARS) and s[0] not in ". -" and s[-1] != " ")
_style_cache = {}


def _string_style(s, key=False):
    """Style go-yaml v3 would emit for a Go string value ``s`` (memoised)."""
    k = (s, key)
    st = _style_cache.get(k)
    if st is None:
        if _is_simple_scalar(s):
            can_plain = resolves_to_string(s) and not _is_base60(s) and s not in _OLD_BOOLS
            st = PLAIN if can_plain else DOUBLE
        else:
            st = _string_style_slow(s, key)
        if len(_style_cache) > 200000:
            _style_cache.clear()
        _style_cache[k] = st
    return st


def _string_style_slow(s, key=False):
    can_plain = resolves_to_string(s) and not _is_base60(s) and s not in _OLD_BOOLS
    if "\n" in s:
        style = LITERAL
    elif can_plain:
        style = PLAIN
    else:
        style = DOUBLE
    multiline, block_plain, single_ok, block_ok = _analyze(s)
    if key and multiline:
        style = DOUBLE
    if style == PLAIN:
        if not block_plain:
            style = SINGLE
        if s == "" and key:
            style = SINGLE
    if style == SINGLE and not single_ok:
        style = DOUBLE
    if style == LITERAL and (not block_ok or key):
        style = DOUBLE
    return style


def _literal(s, indent):
    hint = ""
    if s and (s[0] == " " or _is_break(s[0])):
        hint += "2"
    if s == "" or not _is_break(s[-1]):
        hint += "-"
    elif len(s) == 1 or _is_break(s[-2]):
        hint += "+"
    lines = ["|" + hint]
    pad = " " * indent
    buf = []
    breaks = True
    for ch in s:
        if ch == "\n":
            lines.append("".join(buf))
            buf = []
            breaks = True
        elif _is_break(ch):
            # emitterc.go write_break: a break other than LF (LS, PS: the
            # printable ones that reach a literal) is written as itself, and
            # the next line's indentation follows it on the same output line
            buf.append(ch)
            breaks = True
        else:
            if breaks:
                buf.append(pad)
                breaks = False
            buf.append(ch)
    if buf:
        lines.append("".join(buf))
    # the first element is the header; content lines follow, each terminated by \n
    return lines


def _format_float(f):
    if math.isnan(f):
        return ".nan"
    if math.isinf(f):
        return ".inf" if f > 0 else "-.inf"
    return go_format_float(f)


def go_format_float(f):
    """strconv.FormatFloat(f, 'g', -1, 64)."""
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    neg = f < 0
    a = -f if neg else f
    # shortest round-trip decimal digits (Python's repr is shortest round-trip)
    s = "%.17e" % a
    for prec in range(1, 18):
        s = "%.*e" % (prec - 1, a)
        if float(s) == a:
            break
    mant, e = s.split("e")
    e = int(e)
    digits = mant.replace(".", "").rstrip("0") or "0"
    nd = len(digits)
    # Go: with shortest formatting eprec is 6; %e when exp < -4 || exp >= eprec
    if e < -4 or e >= 6:
        m = digits[0] + ("." + digits[1:] if nd > 1 else "")
        out = "%se%s%02d" % (m, "-" if e < 0 else "+", abs(e))
    elif e >= nd - 1:
        out = digits + "0" * (e - nd + 1)
    elif e >= 0:
        out = digits[:e + 1] + "." + digits[e + 1:]
    else:
        out = "0." + "0" * (-e - 1) + digits
    return ("-" if neg else "") + out


# ---------------------------------------------------------------------------
# Emitter
# ---------------------------------------------------------------------------

class _Emitter:
    def __init__(self, sort_maps):
        self.sort_maps = sort_maps
        self.out = []

    def _keys(self, d):
        if isinstance(d, GoMap) or self.sort_maps:
            return go_key_sorted(d.keys())
        return list(d.keys())

    def scalar(self, v, indent, key=False):
        """Return list of lines; first line is the inline part."""
        if v is None:
            return ["null"]
        if v is True:
            return ["true"]
        if v is False:
            return ["false"]
        if isinstance(v, int):
            return [str(v)]
        if isinstance(v, float):
            return [_format_float(v)]
        if isinstance(v, bytes):
            import base64
            return ["!!binary " + base64.b64encode(v).decode()]
        s = str(v)
        style = _string_style(s, key=key)
        if style == PLAIN:
            return [s]
        if style == SINGLE:
            return [_single_quoted(s, indent)]
        if style == DOUBLE:
            return [_double_quoted(s)]
        return _literal(s, indent)

    @staticmethod
    def _is_coll(v):
        return isinstance(v, (dict, list, tuple))

    def emit_map(self, d, indent, first_prefix=None):
        pad = " " * indent
        first = True
        for k in self._keys(d):
            v = d[k]
            kl = self.scalar(k, indent, key=True)[0]
            prefix = first_prefix if (first and first_prefix is not None) else pad
            first = False
            self._emit_value(prefix + kl + ":", v, indent)

    def emit_seq(self, seq, indent, first_prefix=None):
        pad = " " * indent
        first = True
        for item in seq:
            prefix = first_prefix if (first and first_prefix is not None) else pad
            first = False
            if isinstance(item, dict) and item:
                self.emit_map(item, indent + 2, first_prefix=prefix + "- ")
            elif isinstance(item, (list, tuple)) and item:
                self.emit_seq(item, indent + 2, first_prefix=prefix + "- ")
            elif isinstance(item, dict):
                self.out.append(prefix + "- {}")
            elif isinstance(item, (list, tuple)):
                self.out.append(prefix + "- []")
            else:
                lines = self.scalar(item, indent + 2)
                self.out.append(prefix + "- " + lines[0])
                self.out.extend(lines[1:])

    def _emit_value(self, head, v, indent):
        if isinstance(v, dict):
            if not v:
                self.out.append(head + " {}")
            else:
                self.out.append(head)
                self.emit_map(v, indent + 2)
        elif isinstance(v, (list, tuple)):
            if not v:
                self.out.append(head + " []")
            else:
                self.out.append(head)
                self.emit_seq(v, indent + 2)
        else:
            lines = self.scalar(v, indent + 2)
            self.out.append(head + " " + lines[0])
            self.out.extend(lines[1:])

    def document(self, data):
        if isinstance(data, dict):
            if data:
                self.emit_map(data, 0)
            else:
                self.out.append("{}")
        elif isinstance(data, (list, tuple)):
            if data:
                self.emit_seq(data, 0)
            else:
                self.out.append("[]")
        else:
            lines = self.scalar(data, 2)
            self.out.append(lines[0])
            self.out.extend(lines[1:])
        return "\n".join(self.out) + "\n"


def dump_py(data, sort_maps=False):
    """The pure-Python emitter: the executable specification of the native one."""
    return _Emitter(sort_maps).document(data)


_scalar_lines = _Emitter(False).scalar
_native_dump = None


def _native():
    global _native_dump
    if _native_dump is None:
        from ..ops import native
        m = native.module()
        _native_dump = getattr(m, "yaml_dump", None) or False
    return _native_dump


def dump(data, sort_maps=False):
    """Encode ``data`` like go-yaml v3 ``Encoder`` with ``SetIndent(2)``.

    Runs the native emitter (``ops/csrc/yaml_emit.cpp``) when the extension is
    built; it defers floats, non-ASCII text and numeric-looking strings to the
    Python helpers below, so both paths emit identical bytes."""
    nd = _native()
    if nd:
        return nd(data, sort_maps, GoMap, _scalar_lines, _string_style, go_key_sorted)
    return _Emitter(sort_maps).document(data)


def dumps_k8s(obj):
    """Encode a JSON-shaped object the way the reference writes manifests
    (json.Marshal -> yaml.Unmarshal into interface{} -> yaml.v3 encode): every
    mapping becomes a Go map, so keys are sorted."""
    return dump(obj, sort_maps=True)


# ---------------------------------------------------------------------------
# Loading
# ---------------------------------------------------------------------------

_INT64_MIN, _INT64_MAX, _UINT64_MAX = -(1 << 63), (1 << 63) - 1, (1 << 64) - 1
_DOT_FLOAT = _lazy_re(r"^\.[0-9][0-9_]*(?:[eE][-+]?[0-9]+)?$")


def _go_int_value(t):
    """Value of a string accepted by :func:`_go_parse_int` (base-0 Go syntax)."""
    neg = t[:1] == "-"
    if t[:1] in "+-":
        t = t[1:]
    low = t[:2].lower()
    if low == "0x":
        v = int(t[2:], 16)
    elif low == "0o":
        v = int(t[2:], 8)
    elif low == "0b":
        v = int(t[2:], 2)
    elif len(t) > 1 and t[0] == "0":
        v = int(t[1:], 8)
    else:
        v = int(t)
    return -v if neg else v


def go_resolve_number(s):
    """go-yaml (v2 and v3) ``resolve()`` of a plain scalar whose first byte is
    a sign, a digit or a dot: an int (``strconv.ParseInt(plain, 0, 64)``, then
    ``ParseUint``, with every ``_`` removed), a float (``yamlStyleFloat``) or
    the scalar itself as a string.  Unlike PyYAML's YAML 1.1 resolvers there
    are no base-60 numbers (``22:22`` stays a string) and ``1e3``/``0o17``
    are numbers."""
    if s in _SPECIAL_FLOATS:
        low = s.lower()
        return float("nan") if "nan" in low else float("-inf" if low[0] == "-" else "inf")
    if s[0] == ".":
        if _DOT_FLOAT.match(s):
            return float(s)
        return s
    plain = s.replace("_", "")
    if _go_parse_int(plain):
        v = _go_int_value(plain)
        if _INT64_MIN <= v <= _INT64_MAX or (0 <= v <= _UINT64_MAX and plain[:1] not in "+-"):
            return v
    if _maybe_float(plain) and _YAML_FLOAT.match(plain):
        v = float(plain)
        if not math.isinf(v):
            return v
    return s


def _construct_go_number(loader, node):
    return go_resolve_number(node.value)


_GONUM_TAG = "tag:move2kube:go-number"
_GONUM_FIRST = _lazy_re(r"^[-+0-9.]")


_TRUE_WORDS = {"y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON"}


def _construct_v2_bool(loader, node):
    return node.value in _TRUE_WORDS


def _construct_raw_scalar(loader, node):
    return node.value


def _construct_untagged(loader, node):
    """A node whose tag go-yaml does not resolve (``!foo``, ``!!foo``,
    ``!!set``, ``!!omap``, ``!!pairs``, ``!!timestamp``, ``!!python/...``):
    decode.go decodes it by kind, a scalar as its text (resolve.go
    ``resolvableTag``; an explicit ``!!timestamp`` would be a time.Time there,
    its text here: parity unpinned)."""
    import yaml
    if isinstance(node, yaml.MappingNode):
        return loader.construct_mapping(node, deep=True)
    if isinstance(node, yaml.SequenceNode):
        return loader.construct_sequence(node, deep=True)
    return node.value


def _construct_go_binary(loader, node):
    """decode.go scalar(): ``!!binary`` is base64.StdEncoding (line breaks
    ignored) decoded into a string; bad data is ``failf("!!binary value
    contains invalid base64 data")``."""
    import base64
    import binascii
    try:
        data = base64.b64decode(loader.construct_scalar(node).replace("\r", "").replace("\n", ""), validate=True)
    except (binascii.Error, ValueError):
        raise _GoDecodeError("!!binary value contains invalid base64 data") from None
    return data.decode("utf-8", errors="surrogateescape")


class _GoDecodeError(Exception):
    """A go-yaml decoder failf(): the text after ``yaml: ``."""


class _Loaders:
    """PyYAML plus the three go-yaml flavoured loaders, built once."""

    def __init__(self):
        import yaml
        self.yaml = yaml
        base = getattr(yaml, "CSafeLoader", yaml.SafeLoader)

        def make(name, keep_resolvers):
            cls = type(name, (base,), {})
            cls.yaml_implicit_resolvers = {}
            for ch, resolvers in yaml.SafeLoader.yaml_implicit_resolvers.items():
                kept = [(tag, rx) for tag, rx in resolvers if tag in keep_resolvers]
                if kept:
                    cls.yaml_implicit_resolvers[ch] = kept
            return cls

        def go_scalars(cls, bools):
            cls.add_implicit_resolver("tag:yaml.org,2002:bool", re.compile("^(?:" + "|".join(bools) + ")$"),
                                      sorted({b[0] for b in bools}))
            cls.add_implicit_resolver(_GONUM_TAG, _GONUM_FIRST, list("-+0123456789."))
            cls.add_constructor(_GONUM_TAG, _construct_go_number)

        # go-yaml v3 into interface{}: bools are only true/false, no timestamps
        # (kept as strings for interface{} targets), go-yaml's int/float rules.
        self.typed = make("_TypedLoader", {"tag:yaml.org,2002:null", "tag:yaml.org,2002:merge"})
        go_scalars(self.typed, ["true", "True", "TRUE", "false", "False", "FALSE"])
        # go-yaml v2 (what docker/cli's compose v3 loader and libcompose parse
        # compose files with): v3's rules plus the YAML 1.1 y/yes/on, n/no/off bools.
        self.v2 = make("_V2Loader", {"tag:yaml.org,2002:null", "tag:yaml.org,2002:merge"})
        go_scalars(self.v2, ["y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON",
                             "n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF"])
        self.v2.add_constructor("tag:yaml.org,2002:bool", _construct_v2_bool)
        # Every scalar is kept as its source text (what go-yaml does when decoding
        # a scalar into a Go string field); only nulls resolve.
        self.raw = make("_RawLoader", {"tag:yaml.org,2002:null"})
        for tag in ("tag:yaml.org,2002:int", "tag:yaml.org,2002:float", "tag:yaml.org,2002:bool",
                    "tag:yaml.org,2002:timestamp"):
            self.raw.add_constructor(tag, _construct_raw_scalar)
        for cls in (self.typed, self.v2, self.raw):
            cls.add_constructor(None, _construct_untagged)
            for tag in ("set", "omap", "pairs") + (("timestamp",) if cls is not self.raw else ()):
                cls.add_constructor("tag:yaml.org,2002:" + tag, _construct_untagged)
            cls.add_constructor("tag:yaml.org,2002:binary", _construct_go_binary)


_loaders = None
_loaders_lock = threading.Lock()


def _lz():
    global _loaders
    if _loaders is None:
        with _loaders_lock:
            if _loaders is None:
                _loaders = _Loaders()
    return _loaders


# Command-scoped parse memo.  Every planner/loader of the reference decodes
# every YAML file of the source tree on its own (compose v3, compose v1/v2, CF
# manifest, knative, kube, k8s-files, QA-cache and cluster loaders: 8-10
# parses of each file per translate).  Inside ``parse_cache()`` each distinct
# (loader, text) pair is parsed once and callers get private copies.  Keyed by
# content, so it can never serve a stale document.
_memo = None
_memo_depth = 0
_memo_lock = threading.Lock()


class parse_cache:
    """Memoize YAML parses for the duration of one command (nestable)."""

    __slots__ = ()

    def __enter__(self):
        global _memo, _memo_depth
        with _memo_lock:
            if _memo_depth == 0:
                _memo = {}
            _memo_depth += 1

    def __exit__(self, *exc):
        global _memo, _memo_depth
        with _memo_lock:
            _memo_depth -= 1
            if _memo_depth == 0:
                _memo = None
        return False


_ATOMS = (str, int, float, bool, type(None))


def _tree_copy(o):
    t = type(o)
    if t is dict:
        return {k: (v if type(v) in _ATOMS else _tree_copy(v)) for k, v in o.items()}
    if t is list:
        return [v if type(v) in _ATOMS else _tree_copy(v) for v in o]
    if t in _ATOMS:
        return o
    import copy
    return copy.deepcopy(o)


def _memoized(kind, text, parse):
    memo = _memo
    if memo is None or not isinstance(text, str):
        return parse(text)
    key = (kind, text)
    hit = memo.get(key, _MISS)
    if hit is _MISS:
        try:
            hit = (True, parse(text))
        except _lz().yaml.YAMLError as e:
            hit = (False, e)
        memo[key] = hit
    ok, val = hit
    if not ok:
        raise val.with_traceback(None)
    # (self-containing anchors were refused by _check_aliasing; a document too
    # deep to copy raises RecursionError and its caller skips the file)
    docs, dups = val
    return _tree_copy(docs), dups


_MISS = object()


# Native decode (ops/csrc/yaml_parse.cpp): a strict block-YAML subset parser
# that resolves scalars like the three loader classes above and answers
# _UNSUPPORTED for anything else (anchors, tags, multi-line flow/quoted/plain
# scalars, malformed input, ...), which then goes through PyYAML.  Most files a
# command reads never import PyYAML.  M2K_NATIVE_YAML=0 turns it off.
_TYPED, _V2, _RAW = 0, 1, 2
_UNSUPPORTED = object()
_native_load = None


def _allowed_alias_ratio(decoded):
    """go-yaml v3 decode.go allowedAliasRatio: 99% of the nodes may come
    through aliases up to 400k decoded nodes, falling to 10% at 4M."""
    if decoded <= 400000:
        return 0.99
    if decoded >= 4000000:
        return 0.10
    return 0.99 - 0.89 * (decoded - 400000) / 3600000.0


def _check_aliasing(doc, error):
    """Reject a document the way go-yaml v3 does before it is walked: an
    anchor that contains itself, or aliases that expand it far beyond its text
    ("billion laughs").  PyYAML shares one object per anchor, so the load is
    cheap, but every later walk (copies, conversions, emission) would expand
    it.  Counted on the loaded tree: every container object is one node
    however often it is referenced; ``decoded`` counts each reference's
    subtree again, as go-yaml's decoder does.  (The reference checks the
    ratio while decoding; checked here once over the whole document.)"""
    if not isinstance(doc, (dict, list)):
        return
    expanded = {}          # id -> nodes decoded for one reference to it
    unique = 0
    on_path = set()
    stack = [(doc, False)]
    while stack:
        o, done = stack.pop()
        i = id(o)
        if done:
            on_path.discard(i)
            n = 1
            if isinstance(o, dict):
                for k, v in o.items():
                    n += 1 + (expanded[id(v)] if isinstance(v, (dict, list)) else 1)
            else:
                for v in o:
                    n += expanded[id(v)] if isinstance(v, (dict, list)) else 1
            expanded[i] = n
            if n > 4000000 * 4:
                break
            continue
        if i in expanded:
            continue
        if i in on_path:
            raise error("anchor value contains itself")
        on_path.add(i)
        vals = o.values() if isinstance(o, dict) else o
        unique += 1 + (len(o) if isinstance(o, dict) else 0) + sum(1 for v in vals if not isinstance(v, (dict, list)))
        stack.append((o, True))
        for v in vals:
            if isinstance(v, (dict, list)) and id(v) not in expanded:
                if id(v) in on_path:
                    raise error("anchor value contains itself")
                stack.append((v, False))
    decoded = expanded.get(id(doc))
    if decoded is None:  # stopped early: far past any allowed expansion
        raise error("document contains excessive aliasing")
    aliased = decoded - unique
    if aliased > 100 and decoded > 1000 and aliased / decoded > _allowed_alias_ratio(decoded):
        raise error("document contains excessive aliasing")


def _native_loader():
    global _native_load
    if _native_load is None:
        import os
        fn = False
        if os.environ.get("M2K_NATIVE_YAML", "1") != "0":
            from ..ops import native
            fn = getattr(native.module(), "yaml_load", None) or False
        _native_load = fn
    return _native_load


MAX_DEPTH = 10000  # go-yaml v2/v3: max_flow_level and max_indents


def _too_deep(text, limit=MAX_DEPTH):
    """Cheap upper-bound check of the nesting a parser would have to recurse
    through: flow brackets (outside quotes) plus block levels (indentation
    steps and compact ``- `` entries).  PyYAML's C composer recurses once per
    level and overflows the C stack on deep documents (``'[' * 200000``), so
    such a document is refused before it reaches PyYAML, with go-yaml's error.
    The count only ever over-estimates the real depth by the quoted-bracket
    approximation, and only documents of more than ``limit`` bytes are scanned."""
    if len(text) <= limit:
        return False
    if text.count("[") + text.count("{") > limit:
        flow = 0
        quote = ""
        prev = "\n"
        escaped = False
        for ch in text:
            if quote:
                if quote == "#":
                    if ch == "\n":
                        quote = ""
                elif escaped:
                    escaped = False
                elif ch == "\\" and quote == '"':
                    escaped = True
                elif ch == quote:
                    quote = ""
                prev = ch
                continue
            if ch in "[{":
                flow += 1
                if flow > limit:
                    return True
            elif ch in "]}":
                flow -= 1 if flow else 0
            elif ch in "\"'" and prev in " \t\n:[{,-?":
                quote = ch          # a quoted scalar starts only where a node can start
            elif ch == "#" and prev in " \t\n":
                quote = "#"
            prev = ch
    stack = []
    for line in text.split("\n"):
        body = line.lstrip(" ")
        if not body or body[0] == "#":
            continue
        col = len(line) - len(body)
        while stack and stack[-1] >= col:
            stack.pop()
        stack.append(col)
        while body.startswith("- ") or body == "-":
            col += 2
            body = body[2:].lstrip(" ")
            stack.append(col)
        if len(stack) > limit:
            return True
    return False


def _duplicate_keys(root):
    """go-yaml v3 ``decoder.mapping`` duplicate-key errors of one composed
    document, in its decode order: within a mapping every later key with the
    same node kind and value as an earlier one (``line 5: mapping key "a"
    already defined at line 2``); a mapping that has such keys is not
    descended into.  Nodes shared through aliases are looked at once."""
    import yaml
    out = []
    seen = set()

    def ident(node):
        return (type(node).__name__, node.value if isinstance(node, yaml.ScalarNode) else "")

    stack = [root]
    while stack:
        node = stack.pop()
        if id(node) in seen:
            continue
        seen.add(id(node))
        if isinstance(node, yaml.MappingNode):
            pairs = node.value
            first = {}
            errs = []
            for j, (k, _v) in enumerate(pairs):
                key = ident(k)
                for i, ki in first.get(key, ()):
                    errs.append((i, j, "line %d: mapping key %s already defined at line %d"
                                 % (k.start_mark.line + 1, _go_quote(k.value if key[1] else ""),
                                    ki.start_mark.line + 1)))
                first.setdefault(key, []).append((j, k))
            if errs:
                out.extend(e for _i, _j, e in sorted(errs, key=lambda x: (x[0], x[1])))
                continue
            stack.extend(v for _k, v in reversed(pairs))
        elif isinstance(node, yaml.SequenceNode):
            stack.extend(reversed(node.value))
    return out


def _go_quote(s):
    from .log import go_quote
    return go_quote(s)


_SHORT_TAGS = {bool: "!!bool", int: "!!int", float: "!!float", str: "!!str", list: "!!seq"}


def go_unmarshal_type_error(text, value, into="map[string]interface {}"):
    """go-yaml v3's ``yaml: unmarshal errors:`` text for a document whose
    top-level node (decoded here as ``value``) cannot go into ``into``: the
    node's line, short tag and, for a scalar, its text (``decoder.terror``)."""
    import yaml
    line, raw = 1, ""
    try:
        node = yaml.compose(text, Loader=getattr(yaml, "CSafeLoader", yaml.SafeLoader))
    except yaml.YAMLError:
        node = None
    if node is not None:
        line = node.start_mark.line + 1
        if isinstance(node, yaml.ScalarNode):
            raw = node.value
    tag = _SHORT_TAGS.get(type(value), "!!str")
    shown = ""
    if tag != "!!seq":
        shown = " `" + (raw[:7] + "..." if len(raw) > 10 else raw) + "`"
    return "yaml: unmarshal errors:\n  line %d: cannot unmarshal %s%s into %s" % (line, tag, shown, into)


class _InvalidMapKey(Exception):
    """A sequence or mapping used as a mapping key (PyYAML's "found unhashable
    key"); ``key`` is the key's decoded value."""

    def __init__(self, key):
        super().__init__(key)
        self.key = key


def _first_invalid_key(node):
    """The first collection key node in go-yaml's decode order (a key is
    decoded, then checked, then its value), or None."""
    import yaml
    stack = [node]
    seen = set()
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if isinstance(n, yaml.MappingNode):
            todo = []
            for k, v in n.value:
                todo.append(("key", k))
                todo.append(("val", v))
            for what, child in reversed(todo):
                stack.append(child)
                if what == "key" and isinstance(child, (yaml.MappingNode, yaml.SequenceNode)) and \
                        not (isinstance(child, yaml.ScalarNode) and child.value == "<<"):
                    stack.append(("check", child))
        elif isinstance(n, yaml.SequenceNode):
            stack.extend(reversed(n.value))
        elif isinstance(n, tuple):
            inner = _first_invalid_key(n[1])
            return inner if inner is not None else n[1]
    return None


def _go_sharp_v(v, v2):
    """``fmt.Sprintf("%#v", v)`` of a value go-yaml decoded into interface{}
    (an element: a nil is ``interface {}(nil)``)."""
    from . import gofmt
    if v is None:
        return "interface {}(nil)"
    if isinstance(v, list):
        return "[]interface {}{" + ", ".join(_go_sharp_v(x, v2) for x in v) + "}"
    if isinstance(v, dict):
        # decode.go mapping(): v3 makes map[string]interface{} when every key is
        # a string; v2 always map[interface{}]interface{}
        typ = "map[string]interface {}" if not v2 and all(isinstance(k, str) for k in v) else \
            "map[interface {}]interface {}"
        return typ + "{" + ", ".join("%s:%s" % (_go_sharp_v(k, v2), _go_sharp_v(v[k], v2))
                                      for k in gofmt.sorted_keys(v)) + "}"
    return gofmt.sprintf("%#v", [v])


def _construct(loader, node):
    """construct_document, turning "found unhashable key" into
    :class:`_InvalidMapKey` with the offending key decoded."""
    import yaml
    try:
        return loader.construct_document(node)
    except yaml.constructor.ConstructorError as e:
        if e.problem != "found unhashable key":
            raise
        key = _first_invalid_key(node)
        if key is None:
            raise
        loader.constructed_objects = {}
        loader.recursive_objects = {}
        raise _InvalidMapKey(loader.construct_object(key, deep=True)) from None


def _pyyaml_load(loader_cls, text, multi):
    """``yaml.load_all``, or for a single load the first document only (go-yaml's
    ``Unmarshal`` decodes the first document of a stream and never reads the
    rest), with the duplicate-key scan of each composed document before it is
    constructed."""
    loader = loader_cls(text)
    dups = []
    try:
        if multi:
            docs = []
            while loader.check_node():
                node = loader.get_node()
                dups.extend(_duplicate_keys(node))
                docs.append(_construct(loader, node))
        else:
            docs = None
            if loader.check_node():
                node = loader.get_node()
                if node is not None:
                    dups = _duplicate_keys(node)
                    docs = _construct(loader, node)
    finally:
        loader.dispose()
    return docs, dups


def _go_error_texts(e, text):
    """(go-yaml v3 text, go-yaml v2 text) of a PyYAML parse error, or None.
    Both libraries are ports of libyaml, whose problem strings PyYAML's C
    loader reports verbatim; they differ in the line they name (``parser.fail``:
    v3 prefers the context mark, v2 the problem mark; scanner marks are one
    line behind).  Marks are 0-based and line 0 is not printed."""
    import yaml
    if not isinstance(e, yaml.MarkedYAMLError):
        return None
    problem = e.problem or "unknown problem parsing YAML content"
    if isinstance(e, yaml.composer.ComposerError) and problem.startswith("found undefined alias"):
        name = ""
        if e.problem_mark is not None and isinstance(text, str):
            i = e.problem_mark.index + 1
            j = i
            while j < len(text) and text[j] not in " \t\r\n,[]{}":
                j += 1
            name = text[i:j]
        msg = "yaml: unknown anchor '%s' referenced" % name
        return msg, msg
    scanner = isinstance(e, yaml.scanner.ScannerError)
    cm = e.context_mark if e.context_mark is not None else (e.problem_mark if scanner else None)
    cl = cm.line if cm is not None else 0
    pl = e.problem_mark.line if e.problem_mark is not None else 0
    bump = 1 if scanner else 0
    v3 = cl + bump if cl else (pl + bump if pl else 0)
    v2 = pl + bump if pl else cl

    def fmt(line):
        return "yaml: " + ("line %d: " % line if line else "") + problem
    return fmt(v3), fmt(v2)


def _go_utf8_problem(text):
    """The first problem readerc.go ``yaml_parser_update_buffer`` finds in the
    bytes of ``text`` (surrogate-escaped where they are not UTF-8)."""
    raw = text.encode("utf-8", errors="surrogateescape") if isinstance(text, str) else bytes(text)
    i, n = 0, len(raw)
    while i < n:
        b = raw[i]
        width = 1 if b & 0x80 == 0 else 2 if b & 0xE0 == 0xC0 else 3 if b & 0xF0 == 0xE0 else \
            4 if b & 0xF8 == 0xF0 else 0
        if width == 0:
            return "invalid leading UTF-8 octet"
        if i + width > n:
            return "incomplete UTF-8 octet sequence"
        value = b & (0x7F if width == 1 else 0x1F if width == 2 else 0x0F if width == 3 else 0x07)
        for k in range(1, width):
            c = raw[i + k]
            if c & 0xC0 != 0x80:
                return "invalid trailing UTF-8 octet"
            value = (value << 6) + (c & 0x3F)
        if not (width == 1 or (width == 2 and value >= 0x80) or (width == 3 and value >= 0x800) or
                (width == 4 and value >= 0x10000)):
            return "invalid length of a UTF-8 sequence"
        if 0xD800 <= value <= 0xDFFF or value > 0x10FFFF:
            return "invalid Unicode character"
        if not (value in (0x09, 0x0A, 0x0D, 0x85) or 0x20 <= value <= 0x7E or 0xA0 <= value <= 0xD7FF or
                0xE000 <= value <= 0xFFFD or 0x10000 <= value <= 0x10FFFF):
            return "control characters are not allowed"
        i += width
    return "invalid leading UTF-8 octet"


def _parse(text, mode, multi):
    """-> (document(s), go-yaml v3 duplicate-key errors).  Only the v3 entry
    points raise on the second part: go-yaml v2 (compose files, and Kubernetes
    objects through sigs.k8s.io/yaml) keeps the last value of a repeated key."""
    nl = _native_loader()
    if nl and isinstance(text, str):
        try:
            r = nl(text, mode, multi, go_resolve_number, _UNSUPPORTED)
        except UnicodeError:
            r = _UNSUPPORTED
        except ValueError as e:   # nesting past go-yaml's limit (yaml_parse.cpp TooDeep)
            raise _lz().yaml.YAMLError(str(e)) from None
        if r is not _UNSUPPORTED:   # (it never decodes a document with repeated keys)
            return r, ()
    if isinstance(text, str) and _too_deep(text):
        raise _lz().yaml.YAMLError("yaml: exceeded max depth of %d" % MAX_DEPTH)
    lz = _lz()
    loader = (lz.typed, lz.v2, lz.raw)[mode]
    try:
        docs, dups = _pyyaml_load(loader, text, multi)
        if "*" in text:
            for d in (docs if multi else (docs,)):
                _check_aliasing(d, lz.yaml.YAMLError)
        return docs, tuple(dups)
    except lz.yaml.MarkedYAMLError as e:
        texts = _go_error_texts(e, text)
        if texts is None:
            raise
        err = lz.yaml.YAMLError(texts[1] if mode == _V2 else texts[0])
        err.go_v2 = texts[1]
        raise err from None
    except _InvalidMapKey as e:
        # decode.go mapping(): failf("invalid map key: %#v", k.Interface())
        v3, v2 = ("yaml: invalid map key: " + _go_sharp_v(e.key, flavour) for flavour in (False, True))
        err = lz.yaml.YAMLError(v2 if mode == _V2 else v3)
        err.go_v2 = v2
        raise err from None
    except _GoDecodeError as e:
        raise lz.yaml.YAMLError("yaml: %s" % e) from None
    except lz.yaml.reader.ReaderError as e:
        # readerc.go yaml_parser_set_reader_error: no mark, so parser.fail()
        # prints the problem alone
        raise lz.yaml.YAMLError("yaml: " + (e.reason or "unknown problem parsing YAML content")) from None
    except UnicodeError:
        # bytes that are not UTF-8 (kept as surrogates by read_text): a parse
        # error of this document worded as go-yaml's reader - callers skip the
        # file instead of losing the whole planner
        raise lz.yaml.YAMLError("yaml: " + _go_utf8_problem(text)) from None


def _v3(result):
    """The decoded document(s) of a go-yaml v3 ``Unmarshal``: repeated keys
    fail the whole decode (``*yaml.TypeError``)."""
    docs, dups = result
    if dups:
        raise _lz().yaml.YAMLError("yaml: unmarshal errors:\n  " + "\n  ".join(dups))
    return docs


def _v2(result):
    return result[0]


def _as_v2(memoized, kind, text, parse):
    """A shared v3-flavoured parse answering a v2 caller: parse errors name
    the line go-yaml v2 would."""
    try:
        return memoized(kind, text, parse)
    except _lz().yaml.YAMLError as e:
        v2 = getattr(e, "go_v2", None)
        if v2 is None:
            raise
        raise _lz().yaml.YAMLError(v2) from None


def load(text):
    """Decode like go-yaml v3 into ``interface{}``."""
    return _v3(_memoized("typed", text, lambda t: _parse(t, _TYPED, False)))


def load_all(text):
    return _v3(_memoized("typed*", text, lambda t: _parse(t, _TYPED, True)))


_V2_ONLY_WORDS = _lazy_re(r"\b(?:[yYnN]|yes|Yes|YES|no|No|NO|on|On|ON|off|Off|OFF)\b")


def load_v2(text):
    """Decode like go-yaml v2 into ``interface{}`` (compose files).  The two
    decoders differ only in the YAML 1.1 bool words, so a document that does
    not contain one anywhere shares the v3 parse (and its memo entry)."""
    if isinstance(text, str) and not _V2_ONLY_WORDS.search(text):
        return _v2(_as_v2(_memoized, "typed", text, lambda t: _parse(t, _TYPED, False)))
    return _v2(_memoized("typed-v2", text, lambda t: _parse(t, _V2, False)))


def load_all_v2(text):
    if isinstance(text, str) and not _V2_ONLY_WORDS.search(text):
        return _v2(_as_v2(_memoized, "typed*", text, lambda t: _parse(t, _TYPED, True)))
    return _v2(_memoized("typed-v2*", text, lambda t: _parse(t, _V2, True)))


def load_raw(text):
    """Decode keeping scalars as raw strings (for typed struct decoding)."""
    return _v3(_memoized("raw", text, lambda t: _parse(t, _RAW, False)))
