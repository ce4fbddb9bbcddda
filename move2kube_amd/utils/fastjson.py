"""JSON decoding straight on the C scanner (``_json.make_scanner``), the one
the stdlib ``json`` package wraps, so the read paths of a command (cluster
profiles, detector output, ``~/.docker/config.json``) do not import the
four-module ``json`` package.  :func:`go_encode` writes what Go's
``json.NewEncoder(w).Encode`` writes (the REST QA engine's responses).

What is accepted and the error text follow Go's ``encoding/json`` (what the
reference decodes detector output, ``docker inspect`` and the CLI tools' JSON
with): ``NaN``/``Infinity`` and a byte-order mark are syntax errors, invalid
UTF-8 inside a string becomes U+FFFD per byte, and a failure raises
``ValueError`` with the message Go's scanner gives (``invalid character 'x'
looking for beginning of value``, ``unexpected end of JSON input``), found by
re-scanning the input the way ``encoding/json/scanner.go`` does.
"""

import _json


class _GoRejects(Exception):
    """NaN / Infinity: valid for Python's scanner, not for Go's."""


def _reject_constant(name):
    raise _GoRejects(name)


class _Context:
    """The attributes ``_json.make_scanner`` reads from a ``JSONDecoder``."""

    def __init__(self, parse_int=int, parse_float=float):
        self.strict = True
        self.object_hook = None
        self.object_pairs_hook = None
        self.parse_float = parse_float
        self.parse_int = parse_int
        self.parse_constant = _reject_constant
        self.memo = {}


_scanners = {}
_WS = " \t\n\r"


def _text(s):
    """str of the input; invalid UTF-8 bytes become one U+FFFD each, as Go's
    decoder replaces them."""
    if not isinstance(s, (bytes, bytearray)):
        return s
    try:
        return bytes(s).decode("utf-8")
    except UnicodeDecodeError:
        t = bytes(s).decode("utf-8", "surrogateescape")
        return "".join("\ufffd" if "\udc80" <= c <= "\udcff" else c for c in t)


def loads(s, parse_int=int, parse_float=float):
    text = _text(s)
    scan = _scanners.get((parse_int, parse_float))
    if scan is None:
        scan = _scanners[parse_int, parse_float] = _json.make_scanner(_Context(parse_int, parse_float))
    i, n = 0, len(text)
    while i < n and text[i] in _WS:
        i += 1
    try:
        obj, end = scan(text, i)
        while end < n and text[end] in _WS:
            end += 1
        if end != n:
            raise ValueError("extra data")
    except (StopIteration, ValueError, _GoRejects, RecursionError, SystemError):
        # SystemError: CPython 3.10's scanner reports an error inside an object
        # or array through json.decoder.JSONDecodeError, looked up in
        # sys.modules only; in a process that never imported json (a cold
        # command) it returns NULL with no exception set
        raw = s if isinstance(s, (bytes, bytearray)) else s.encode("utf-8", "surrogatepass")
        raise ValueError(go_syntax_error(bytes(raw)) or "invalid JSON") from None
    if "\\u" in text or (text is s and not _valid_utf8(text)):
        obj = _no_lone_surrogates(obj)
    return obj


def _valid_utf8(t):
    try:
        t.encode("utf-8")
        return True
    except UnicodeEncodeError:
        return False


def _no_lone_surrogates(o):
    """decode.go unquote: a ``\\uD800``-range escape that is not half of a
    pair, like a byte that is not UTF-8, becomes U+FFFD (the scanner has
    already joined the pairs, so every surrogate left is a lone one)."""
    if isinstance(o, str):
        if _valid_utf8(o):
            return o
        return "".join("\ufffd" if "\ud800" <= c <= "\udfff" else c for c in o)
    if isinstance(o, list):
        return [_no_lone_surrogates(x) for x in o]
    if isinstance(o, dict):
        return {_no_lone_surrogates(k): _no_lone_surrogates(v) for k, v in o.items()}
    return o


def load(f, parse_int=int):
    return loads(f.read(), parse_int)


# ---------------------------------------------------------------------------
# Go's encoder (encoding/json encodeState, escapeHTML on)
# ---------------------------------------------------------------------------

_GO_ENC_ESC = {'"': '\\"', "\\": "\\\\", "\n": "\\n", "\r": "\\r", "\t": "\\t",
               "<": "\\u003c", ">": "\\u003e", "&": "\\u0026",
               "\u2028": "\\u2028", "\u2029": "\\u2029"}


def _go_string(s):
    """``encodeState.string`` (Go 1.15): compact escapes only for quote,
    backslash, newline, carriage return and tab, ``\\u00XX`` for the other
    control characters (``\\b`` and ``\\f`` included), ``<``, ``>``, ``&`` and
    U+2028/U+2029 as ``\\uXXXX``, every other character raw UTF-8; a byte
    that was not UTF-8 (surrogateescape) is written as the escape text
    ``\\ufffd``."""
    out = []
    for ch in s:
        e = _GO_ENC_ESC.get(ch)
        if e is not None:
            out.append(e)
        elif ch < " ":
            out.append("\\u%04x" % ord(ch))
        elif "\ud800" <= ch <= "\udfff":
            out.append("\\ufffd")
        else:
            out.append(ch)
    return '"' + "".join(out) + '"'


class UnsupportedValueError(ValueError):
    """encoding/json UnsupportedValueError (NaN and infinities)."""


def _go_float(f):
    """floatEncoder.encode (Go 1.15, 64 bits): the shortest 'f' form, or the
    shortest 'e' form below 1e-6 and from 1e21 on, with e-09 written e-9."""
    from .gofmt import format_float
    if f != f or f in (float("inf"), float("-inf")):
        raise UnsupportedValueError("json: unsupported value: " + format_float(f, "g", -1))
    a = abs(f)
    fmt = "e" if a != 0 and (a < 1e-6 or a >= 1e21) else "f"
    b = format_float(f, fmt, -1)
    if fmt == "e" and len(b) >= 4 and b[-4] == "e" and b[-3] == "-" and b[-2] == "0":
        b = b[:-2] + b[-1]
    return b


def _go_value(v, out):
    if v is None:
        out.append("null")
    elif v is True:
        out.append("true")
    elif v is False:
        out.append("false")
    elif isinstance(v, int):
        out.append(str(v))
    elif isinstance(v, float):
        out.append(_go_float(v))
    elif isinstance(v, str):
        out.append(_go_string(v))
    elif isinstance(v, dict):
        out.append("{")
        for i, (k, x) in enumerate(v.items()):
            if i:
                out.append(",")
            out.append(_go_string(str(k)))
            out.append(":")
            _go_value(x, out)
        out.append("}")
    elif isinstance(v, (list, tuple)):
        out.append("[")
        for i, x in enumerate(v):
            if i:
                out.append(",")
            _go_value(x, out)
        out.append("]")
    else:
        raise TypeError("json: unsupported type: %s" % type(v).__name__)


def _go_value_indent(v, out, indent, depth):
    if isinstance(v, dict) and v:
        inner = "\n" + indent * (depth + 1)
        out.append("{")
        for i, (k, x) in enumerate(v.items()):
            out.append(("," if i else "") + inner + _go_string(str(k)) + ": ")
            _go_value_indent(x, out, indent, depth + 1)
        out.append("\n" + indent * depth + "}")
    elif isinstance(v, (list, tuple)) and v:
        inner = "\n" + indent * (depth + 1)
        out.append("[")
        for i, x in enumerate(v):
            out.append(("," if i else "") + inner)
            _go_value_indent(x, out, indent, depth + 1)
        out.append("\n" + indent * depth + "]")
    else:
        _go_value(v, out)


def go_marshal_indent(v, indent):
    """``json.MarshalIndent(v, "", indent)``: Go's escaping, ``": "`` after a
    key, an empty object or array kept as ``{}`` / ``[]``, no trailing
    newline; UTF-8 bytes.  Dicts are written in their own order (a Go map's
    keys sorted, a struct's fields in declaration order: the caller's job)."""
    out = []
    _go_value_indent(v, out, indent, 0)
    return "".join(out).encode("utf-8")


def go_encode(v):
    """``json.NewEncoder(w).Encode(v)`` of a value whose dicts hold the Go
    struct's fields in declaration order: compact, HTML-escaped, one trailing
    newline; returned as UTF-8 bytes."""
    out = []
    _go_value(v, out)
    out.append("\n")
    return "".join(out).encode("utf-8")


# ---------------------------------------------------------------------------
# Go's scanner, for the error text only
# ---------------------------------------------------------------------------

def _quote_char(c):
    """``quoteChar`` of encoding/json: the byte as a Go character literal."""
    if c == 0x27:
        return "'\\''"
    if c == 0x22:
        return "'\"'"
    from .log import go_quote
    return "'" + go_quote(chr(c))[1:-1] + "'"


_SPACE = b" \t\r\n"
_DIGITS = b"0123456789"
_HEX = b"0123456789abcdefABCDEF"
_MAX_DEPTH = 10000


def go_syntax_error(data):
    """The ``SyntaxError`` text ``json.Unmarshal`` returns for ``data``, or
    None when Go's scanner accepts it."""
    stack = []          # "obj" / "arr": what the value being scanned belongs to
    i, n = 0, len(data)

    def err(c, context):
        return "invalid character %s %s" % (_quote_char(c), context)

    # state: "value" (begin value), "value_or_close" (after '['), "key_or_close"
    # (after '{'), "key" (after ','), "colon" (after a key), "end" (after a value)
    state = "value"
    while True:
        if state in ("value", "value_or_close", "key_or_close", "key", "colon", "end"):
            while i < n and data[i] in _SPACE:
                i += 1
            if i >= n:
                if state == "end" and not stack:
                    return None
                return "unexpected end of JSON input"
            c = data[i]
        if state == "value_or_close":
            if c == 0x5D:   # ]
                i += 1
                stack.pop()
                state = "end"
                continue
            state = "value"
        if state == "key_or_close":
            if c == 0x7D:   # }
                i += 1
                stack.pop()
                state = "end"
                continue
            state = "key"
        if state == "key":
            if c != 0x22:
                return err(c, "looking for beginning of object key string")
            r = _scan_string(data, i + 1)
            if isinstance(r, str):
                return r
            i = r
            state = "colon"
            continue
        if state == "colon":
            if c != 0x3A:
                return err(c, "after object key")
            i += 1
            state = "value"
            continue
        if state == "end":
            if not stack:
                return err(c, "after top-level value")
            if stack[-1] == "obj":
                if c == 0x2C:
                    i += 1
                    state = "key"
                    continue
                if c == 0x7D:
                    i += 1
                    stack.pop()
                    continue
                return err(c, "after object key:value pair")
            if c == 0x2C:
                i += 1
                state = "value"
                continue
            if c == 0x5D:
                i += 1
                stack.pop()
                continue
            return err(c, "after array element")
        # state == "value"
        if c in (0x7B, 0x5B):
            if len(stack) >= _MAX_DEPTH:
                return "exceeded max depth"
            stack.append("obj" if c == 0x7B else "arr")
            i += 1
            state = "key_or_close" if c == 0x7B else "value_or_close"
            continue
        if c == 0x22:
            r = _scan_string(data, i + 1)
            if isinstance(r, str):
                return r
            i = r
        elif c == 0x2D or c in _DIGITS:
            r = _scan_number(data, i)
            if isinstance(r, str):
                return r
            i = r
        elif c in b"tfn":
            word = {0x74: b"true", 0x66: b"false", 0x6E: b"null"}[c]
            for j in range(1, len(word)):
                if i + j >= n:
                    return "unexpected end of JSON input"
                if data[i + j] != word[j]:
                    return err(data[i + j], "in literal %s (expecting %s)" % (word.decode(), _quote_char(word[j])))
            i += len(word)
        else:
            return err(c, "looking for beginning of value")
        state = "end"


def _scan_string(data, i):
    """Index after the closing quote of a string whose body starts at i, or
    the error text."""
    n = len(data)
    while i < n:
        c = data[i]
        if c == 0x22:
            return i + 1
        if c == 0x5C:
            i += 1
            if i >= n:
                break
            e = data[i]
            if e == 0x75:   # u
                for j in range(1, 5):
                    if i + j >= n:
                        return "unexpected end of JSON input"
                    if data[i + j] not in _HEX:
                        return "invalid character %s in \\u hexadecimal character escape" % _quote_char(data[i + j])
                i += 5
                continue
            if e not in b'bfnrt\\/"':
                return "invalid character %s in string escape code" % _quote_char(e)
            i += 1
            continue
        if c < 0x20:
            return "invalid character %s in string literal" % _quote_char(c)
        i += 1
    return "unexpected end of JSON input"


def _scan_number(data, i):
    """Index after a number starting at i, or the error text."""
    n = len(data)
    if data[i] == 0x2D:
        i += 1
        if i >= n:
            return "unexpected end of JSON input"
        if data[i] not in _DIGITS:
            return "invalid character %s in numeric literal" % _quote_char(data[i])
    if data[i] == 0x30:
        i += 1
    else:
        while i < n and data[i] in _DIGITS:
            i += 1
    if i < n and data[i] == 0x2E:
        i += 1
        if i >= n:
            return "unexpected end of JSON input"
        if data[i] not in _DIGITS:
            return "invalid character %s after decimal point in numeric literal" % _quote_char(data[i])
        while i < n and data[i] in _DIGITS:
            i += 1
    if i < n and data[i] in b"eE":
        i += 1
        if i < n and data[i] in b"+-":
            i += 1
        if i >= n:
            return "unexpected end of JSON input"
        if data[i] not in _DIGITS:
            return "invalid character %s in exponent of numeric literal" % _quote_char(data[i])
        while i < n and data[i] in _DIGITS:
            i += 1
    return i
