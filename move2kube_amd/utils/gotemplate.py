"""Go 1.15 ``text/template``.

Go templates are part of the reference's user-facing extension ABI: the
Dockerfile/S2I detector directories carry ``Dockerfile`` and
``.s2i/environment`` templates rendered with the JSON a detect script prints
(``internal/containerizer/dockerfilecontainerizer.go:113-127``,
``s2icontainerizer.go:160``), and every output script/readme is a Go template
(``internal/transformer/templates/*``), all executed by
``common.GetStringFromTemplate`` (``internal/common/utils.go:347-374``:
``template.New("").Parse`` with no extra functions).  The reference is built
with go1.15 (``go.mod:3``, ``Dockerfile:20``), so this follows the Go 1.15
sources of ``text/template``:

* ``parse/lex.go``: one action per line (a newline inside an action is
  "unclosed action"; multi-line actions came with Go 1.16), trim markers
  ``{{- `` / `` -}}`` with a space or tab, comments right after the
  delimiter, Go 1.13 number literals, the 1.15 keywords (no ``break`` /
  ``continue``: Go 1.18);
* ``parse/parse.go``: functions and variables are checked while parsing
  (``function "x" not defined``, ``undefined variable "$x"``), ``{{else if}}``
  only inside ``{{if}}`` (``{{else with}}`` is Go 1.23), ``{{define}}`` only
  at the top level, operands separated by spaces;
* ``exec.go``: ``reflect``-style evaluation -- a missing map key is the zero
  ``reflect.Value`` (printed ``<no value>``, passed to a function as a nil
  interface), a nil interface value is dug out of every pipeline stage,
  ``range`` over an integer, string or number is "range can't iterate over",
  ``nil`` is not a command, errors carry Go's ``template: :LINE:COL:
  executing "" at <CONTEXT>:`` prefix;
* ``funcs.go``: the builtins with their 1.15 signatures (``and``/``or``
  evaluate every argument), ``eq``/``ne``/``lt``/``le``/``gt``/``ge`` on
  ``basicKind`` (float64 against int is "incompatible types for comparison",
  slices, maps, nil and missing values are "invalid type for comparison",
  ``lt`` on booleans is an error), ``index``/``slice``/``len`` on the bytes
  of a string, ``html``/``js``/``urlquery`` escapers;
* ``fmt`` through :mod:`.gofmt`.

Values are the ones :mod:`.gofmt` describes (JSON numbers are ``float``; a
template literal ``8080`` is an ``int``).  A template is parsed once per
process (or comes from the build's start-up cache) and, from its second
execution on, runs as closures compiled from the parse tree; both paths share
the evaluation helpers and ``tests/test_gotemplate_compiled.py`` checks they
agree.  ``tests/test_gotemplate_go115.py`` pins the behaviour case by case
against the Go source lines it follows (parity unpinned beyond them: no Go
toolchain here).
"""

import os

from .gofmt import (NO_VALUE, GoUint8, quote as go_quote, sorted_keys, sprint, sprint_one,
                    sprintf, sprintln, type_string)

INTERPRET = os.environ.get("M2K_TEMPLATE_INTERPRET", "") == "1"  # the tree walker instead of closures
COMPILE_AFTER = 1  # executions of a template interpreted before it is compiled to closures
MAX_EXEC_DEPTH = 100000  # exec.go: maxExecDepth


class TemplateError(Exception):
    pass


class _GoError(Exception):
    """An error a builtin returns (``error calling NAME: ...``)."""


_MISSING = object()  # exec.go: missingVal (no final value in a pipeline)


# ---------------------------------------------------------------------------
# Formatting entry points (kept for callers)
# ---------------------------------------------------------------------------

def go_sprint(v, top=True):
    """fmt.Sprint of one value (``%v``); a missing value prints ``<no value>``."""
    return sprint_one(v)


def go_sprintf(fmt, args):
    """fmt.Sprintf."""
    return sprintf(fmt, [None if a is NO_VALUE else a for a in args])


def go_type_name(v):
    """fmt's %T of a value."""
    return type_string(v)


# ---------------------------------------------------------------------------
# Lexer (parse/lex.go, Go 1.15)
# ---------------------------------------------------------------------------

(I_ERROR, I_BOOL, I_CHAR, I_CHARCONST, I_COMPLEX, I_ASSIGN, I_DECLARE, I_EOF, I_FIELD, I_IDENT,
 I_LDELIM, I_LPAREN, I_NUMBER, I_PIPE, I_RAWSTRING, I_RDELIM, I_RPAREN, I_SPACE, I_STRING, I_TEXT,
 I_VARIABLE, I_KEYWORD, I_BLOCK, I_DOT, I_DEFINE, I_ELSE, I_END, I_IF, I_NIL, I_RANGE, I_TEMPLATE,
 I_WITH) = range(32)

_KEYWORDS = {"block": I_BLOCK, "define": I_DEFINE, "else": I_ELSE, "end": I_END, "if": I_IF,
             "nil": I_NIL, "range": I_RANGE, "template": I_TEMPLATE, "with": I_WITH}
_SPACE = " \t"          # lex.go (1.15): isSpace
_EOL = "\r\n"           # lex.go (1.15): isEndOfLine
_TRIM = " \t\r\n"       # lex.go: spaceChars (what a trim marker removes)


def _alnum(c):
    """lex.go: isAlphaNumeric (unicode.IsLetter / unicode.IsDigit)."""
    return c == "_" or c.isalpha() or c.isdecimal()


def _has_left_trim(src, p):
    return p + 1 < len(src) and src[p] == "-" and src[p + 1] in _SPACE


def _at_right_delim(src, p, right):
    """lex.go: atRightDelim -> (delim, trimSpaces)."""
    if p + 1 < len(src) and src[p] in _SPACE and src[p + 1] == "-" and src.startswith(right, p + 2):
        return True, True
    if src.startswith(right, p):
        return True, False
    return False, False


def _at_terminator(src, p, right):
    """lex.go: atTerminator."""
    if p >= len(src):
        return True
    c = src[p]
    return c in _SPACE or c in _EOL or c in ".,|:)(" or c == right[0]


def _fmt_U(c):
    """%#U of a rune."""
    from .gofmt import is_print
    r = ord(c)
    h = "U+%04X" % r
    return h + " '" + c + "'" if is_print(r) else h


def _scan_number(src, p):
    """lex.go: scanNumber -> (ok, end)."""
    n = len(src)
    i = p
    if i < n and src[i] in "+-":
        i += 1
    digits = "0123456789_"
    if i < n and src[i] == "0":
        i += 1
        if i < n and src[i] in "xX":
            i += 1
            digits = "0123456789abcdefABCDEF_"
        elif i < n and src[i] in "oO":
            i += 1
            digits = "01234567_"
        elif i < n and src[i] in "bB":
            i += 1
            digits = "01_"
    while i < n and src[i] in digits:
        i += 1
    if i < n and src[i] == ".":
        i += 1
        while i < n and src[i] in digits:
            i += 1
    if len(digits) == 11 and i < n and src[i] in "eE":
        i += 1
        if i < n and src[i] in "+-":
            i += 1
        while i < n and src[i] in "0123456789_":
            i += 1
    if len(digits) == 23 and i < n and src[i] in "pP":
        i += 1
        if i < n and src[i] in "+-":
            i += 1
        while i < n and src[i] in "0123456789_":
            i += 1
    if i < n and src[i] == "i":
        i += 1
    if i < n and _alnum(src[i]):
        return False, i + 1
    return True, i


def _lex(src, left="{{", right="}}"):
    """The items of ``src``: (kind, value, pos); lexing stops at the first
    error, which is an I_ERROR item (the parser reports it when it gets
    there, as Go's concurrent lexer does)."""
    items = []
    emit = items.append
    n = len(src)
    pos = 0
    while True:
        # lexText
        x = src.find(left, pos)
        if x < 0:
            if pos < n:
                emit((I_TEXT, src[pos:], pos))
            emit((I_EOF, "", n))
            return items
        end_text = x
        if _has_left_trim(src, x + len(left)):
            end_text = pos + len(src[pos:x].rstrip(_TRIM))
        if end_text > pos:
            emit((I_TEXT, src[pos:end_text], pos))
        # lexLeftDelim
        p = x + len(left)
        trim = _has_left_trim(src, p)
        after = 2 if trim else 0
        if src.startswith("/*", p + after):
            # lexComment
            p += after + 2
            i = src.find("*/", p)
            if i < 0:
                emit((I_ERROR, "unclosed comment", x))
                return items
            p = i + 2
            delim, trim_r = _at_right_delim(src, p, right)
            if not delim:
                emit((I_ERROR, "comment ends before closing delimiter", p))
                return items
            if trim_r:
                p += 2
            p += len(right)
            if trim_r:
                p = n - len(src[p:].lstrip(_TRIM))
            pos = p
            continue
        emit((I_LDELIM, left, x))
        p += after
        paren = 0
        # lexInsideAction
        while True:
            delim, trim_r = _at_right_delim(src, p, right)
            if delim:
                if paren == 0:
                    if trim_r:
                        p += 2
                    emit((I_RDELIM, right, p))
                    p += len(right)
                    if trim_r:
                        p = n - len(src[p:].lstrip(_TRIM))
                    pos = p
                    break
                emit((I_ERROR, "unclosed left paren", p))
                return items
            if p >= n:
                emit((I_ERROR, "unclosed action", p))
                return items
            c = src[p]
            if c in _EOL:
                emit((I_ERROR, "unclosed action", p))
                return items
            if c in _SPACE:
                # lexSpace (a trim-marked right delimiter after the run is not space)
                j = p
                while j < n and src[j] in _SPACE:
                    j += 1
                spaces = j - p
                if src.startswith("-" + right, j):
                    j -= 1
                    if spaces == 1:
                        p = j
                        continue
                emit((I_SPACE, src[p:j], p))
                p = j
                continue
            if c == "=":
                emit((I_ASSIGN, "=", p))
                p += 1
            elif c == ":":
                if src.startswith(":=", p):
                    emit((I_DECLARE, ":=", p))
                    p += 2
                else:
                    emit((I_ERROR, "expected :=", p))
                    return items
            elif c == "|":
                emit((I_PIPE, "|", p))
                p += 1
            elif c == '"':
                j = p + 1
                while True:
                    if j >= n or src[j] == "\n":
                        emit((I_ERROR, "unterminated quoted string", p))
                        return items
                    if src[j] == "\\":
                        if j + 1 >= n or src[j + 1] == "\n":
                            emit((I_ERROR, "unterminated quoted string", p))
                            return items
                        j += 2
                        continue
                    if src[j] == '"':
                        break
                    j += 1
                emit((I_STRING, src[p:j + 1], p))
                p = j + 1
            elif c == "`":
                j = src.find("`", p + 1)
                if j < 0:
                    emit((I_ERROR, "unterminated raw quoted string", p))
                    return items
                emit((I_RAWSTRING, src[p:j + 1], p))
                p = j + 1
            elif c == "$" or (c == "." and not (p + 1 < n and "0" <= src[p + 1] <= "9")):
                # lexVariable / lexField -> lexFieldOrVariable
                kind = I_VARIABLE if c == "$" else I_FIELD
                j = p + 1
                if _at_terminator(src, j, right):
                    emit((kind if c == "$" else I_DOT, c, p))
                    p = j
                    continue
                while j < n and _alnum(src[j]):
                    j += 1
                if not _at_terminator(src, j, right):
                    emit((I_ERROR, "bad character %s" % _fmt_U(src[j]), j))
                    return items
                emit((kind, src[p:j], p))
                p = j
            elif c == "'":
                j = p + 1
                while True:
                    if j >= n or src[j] == "\n":
                        emit((I_ERROR, "unterminated character constant", p))
                        return items
                    if src[j] == "\\":
                        if j + 1 >= n or src[j + 1] == "\n":
                            emit((I_ERROR, "unterminated character constant", p))
                            return items
                        j += 2
                        continue
                    if src[j] == "'":
                        break
                    j += 1
                emit((I_CHARCONST, src[p:j + 1], p))
                p = j + 1
            elif c in "+-." or "0" <= c <= "9":
                ok, j = _scan_number(src, p)
                if not ok:
                    emit((I_ERROR, "bad number syntax: %s" % go_quote(src[p:j]), p))
                    return items
                if j < n and src[j] in "+-":
                    ok, k = _scan_number(src, j)
                    if not ok or src[k - 1] != "i":
                        emit((I_ERROR, "bad number syntax: %s" % go_quote(src[p:k]), p))
                        return items
                    emit((I_COMPLEX, src[p:k], p))
                    p = k
                else:
                    emit((I_NUMBER, src[p:j], p))
                    p = j
            elif _alnum(c):
                j = p + 1
                while j < n and _alnum(src[j]):
                    j += 1
                if not _at_terminator(src, j, right):
                    emit((I_ERROR, "bad character %s" % _fmt_U(src[j]), j))
                    return items
                word = src[p:j]
                kw = _KEYWORDS.get(word)
                if kw is not None:
                    emit((kw, word, p))
                elif word in ("true", "false"):
                    emit((I_BOOL, word, p))
                else:
                    emit((I_IDENT, word, p))
                p = j
            elif c == "(":
                emit((I_LPAREN, "(", p))
                paren += 1
                p += 1
            elif c == ")":
                paren -= 1
                if paren < 0:
                    emit((I_ERROR, "unexpected right paren %s" % _fmt_U(c), p))
                    return items
                emit((I_RPAREN, ")", p))
                p += 1
            elif ord(c) <= 0x7F and 0x20 <= ord(c) < 0x7F:
                emit((I_CHAR, c, p))
                p += 1
            else:
                emit((I_ERROR, "unrecognized character in action: %s" % _fmt_U(c), p))
                return items


def _item_str(it):
    """lex.go: item.String."""
    kind, val = it[0], it[1]
    if kind == I_EOF:
        return "EOF"
    if kind == I_ERROR:
        return val
    if kind > I_KEYWORD:
        return "<%s>" % val
    if len(val) > 10:
        return go_quote(val[:10]) + "..."
    return go_quote(val)


# ---------------------------------------------------------------------------
# strconv.Unquote / UnquoteChar and number literals (parse/node.go: newNumber)
# ---------------------------------------------------------------------------

_SIMPLE_ESC = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92}


def _unquote_char(s, i, quote):
    """strconv.UnquoteChar at s[i]: (rune or byte, is_byte, next index)."""
    c = s[i]
    if c == quote and quote in "'\"":
        raise ValueError("invalid syntax")
    if c != "\\":
        return ord(c), False, i + 1
    if i + 1 >= len(s):
        raise ValueError("invalid syntax")
    c = s[i + 1]
    i += 2
    if c in _SIMPLE_ESC:
        return _SIMPLE_ESC[c], False, i
    if c in "xuU":
        n = {"x": 2, "u": 4, "U": 8}[c]
        h = s[i:i + n]
        if len(h) < n or any(ch not in "0123456789abcdefABCDEF" for ch in h):
            raise ValueError("invalid syntax")
        v = int(h, 16)
        if c == "x":
            return v, True, i + n
        if v > 0x10FFFF or 0xD800 <= v <= 0xDFFF:
            raise ValueError("invalid syntax")
        return v, False, i + n
    if "0" <= c <= "7":
        o = s[i - 1:i + 2]
        if len(o) < 3 or any(ch not in "01234567" for ch in o):
            raise ValueError("invalid syntax")
        v = int(o, 8)
        if v > 255:
            raise ValueError("invalid syntax")
        return v, True, i + 2
    if c in "'\"":
        if c != quote:
            raise ValueError("invalid syntax")
        return ord(c), False, i
    raise ValueError("invalid syntax")


def _unquote(text):
    """strconv.Unquote of a "..." or `...` literal."""
    if text[0] == "`":
        return text[1:-1].replace("\r", "")
    body = text[1:-1]
    if "\\" not in body:
        return body
    out = bytearray()
    i = 0
    while i < len(body):
        v, is_byte, i = _unquote_char(body, i, '"')
        if is_byte:
            out.append(v)
        else:
            out += chr(v).encode("utf-8", "surrogatepass")
    return out.decode("utf-8", "surrogateescape")


def _underscore_ok(s):
    """strconv: underscoreOK."""
    saw = "^"
    i = 0
    if s[:1] in ("-", "+"):
        s = s[1:]
    hexa = False
    if len(s) >= 2 and s[0] == "0" and s[1].lower() in "box":
        i = 2
        saw = "0"
        hexa = s[1].lower() == "x"
    while i < len(s):
        c = s[i]
        if "0" <= c <= "9" or (hexa and "a" <= c.lower() <= "f"):
            saw = "0"
        elif c == "_":
            if saw != "0":
                return False
            saw = "_"
        else:
            if saw == "_":
                return False
            saw = "!"
        i += 1
    return saw != "_"


def _parse_uint0(s):
    """strconv.ParseUint(s, 0, 64), None on error."""
    if not s or s[0] in "+-":
        return None
    s0 = s
    base = 10
    if s[0] == "0":
        if len(s) >= 3 and s[1].lower() == "b":
            base, s = 2, s[2:]
        elif len(s) >= 3 and s[1].lower() == "o":
            base, s = 8, s[2:]
        elif len(s) >= 3 and s[1].lower() == "x":
            base, s = 16, s[2:]
        else:
            base, s = 8, s[1:]
    if "_" in s0 and not _underscore_ok(s0):
        return None
    t = s.replace("_", "")
    if not t and base == 8 and s0.replace("_", "") == "0":
        return 0
    if not t:
        return None
    try:
        v = int(t, base)
    except ValueError:
        return None
    return v if v < 1 << 64 else None


def _parse_int0(s):
    """strconv.ParseInt(s, 0, 64), None on error."""
    neg = s[:1] == "-"
    body = s[1:] if s[:1] in "+-" else s
    u = _parse_uint0(body)
    if u is None:
        return None
    v = -u if neg else u
    return v if -(1 << 63) <= v < 1 << 63 else None


def _parse_float(s):
    """strconv.ParseFloat(s, 64) for the literals the lexer produces."""
    if "_" in s and not _underscore_ok(s):
        return None
    t = s.replace("_", "")
    body = t.lstrip("+-")
    try:
        if body[:2] in ("0x", "0X"):
            if "p" not in body.lower():
                return None
            v = float.fromhex(body)
        else:
            v = float(body)
    except (ValueError, OverflowError):
        return None
    if v in (float("inf"),):
        return None  # out of range
    return -v if t.startswith("-") else v


def _ideal_constant(text, kind):
    """(value, error) of a number node as exec.go's idealConstant sees it:
    int unless the text has ``. e E p P`` (and is not a hex int or a rune)."""
    if kind == I_CHARCONST:
        body = text[1:-1]
        try:
            v, is_byte, j = _unquote_char(body, 0, "'")
        except (ValueError, IndexError):
            return None, "invalid syntax", True
        if j != len(body):
            return None, "malformed character constant: %s" % text, True
        return v, None, False
    if kind == I_COMPLEX or text.endswith("i"):
        if text.endswith("i") and kind != I_COMPLEX:
            f = _parse_float(text[:-1])
            if f is not None:
                return complex(0, f), None, False
        # a+bi
        for k in range(len(text) - 2, 0, -1):
            if text[k] in "+-" and text[k - 1] not in "eEpP":
                re_ = _parse_float(text[:k])
                im = _parse_float(text[k:-1])
                if re_ is not None and im is not None:
                    return complex(re_, im), None, False
                break
        return None, "illegal number syntax: %s" % go_quote(text), True
    u = _parse_uint0(text)
    i = _parse_int0(text)
    is_hex_int = len(text) > 2 and text[0] == "0" and text[1] in "xX" and not any(c in "pP" for c in text)
    is_float_text = any(c in ".eEpP" for c in text)
    if i is not None or u is not None:
        if is_float_text and not is_hex_int:
            return float(i if i is not None else u), None, False
        if i is not None:
            return i, None, False
        return None, "%s overflows int" % text, False   # exec-time error
    f = _parse_float(text)
    if f is None:
        return None, "illegal number syntax: %s" % go_quote(text), True
    if not is_float_text:
        return None, "integer overflow: %s" % go_quote(text), True
    return f, None, False


# ---------------------------------------------------------------------------
# Parse tree (parse/node.go)
# ---------------------------------------------------------------------------

class _Text:
    __slots__ = ("pos", "text")

    def __init__(self, pos, text):
        self.pos, self.text = pos, text


class _Action:
    __slots__ = ("pos", "pipe")

    def __init__(self, pos, pipe):
        self.pos, self.pipe = pos, pipe


class _Pipe:
    __slots__ = ("pos", "decls", "cmds", "is_assign")

    def __init__(self, pos, decls, cmds, is_assign):
        self.pos, self.decls, self.cmds, self.is_assign = pos, decls, cmds, is_assign


class _Command:
    __slots__ = ("pos", "args")

    def __init__(self, pos, args):
        self.pos, self.args = pos, args


class _Field:
    __slots__ = ("pos", "idents")

    def __init__(self, pos, idents):
        self.pos, self.idents = pos, idents


class _Variable:
    __slots__ = ("pos", "idents")

    def __init__(self, pos, idents):
        self.pos, self.idents = pos, idents


class _Chain:
    __slots__ = ("pos", "node", "fields")

    def __init__(self, pos, node, fields):
        self.pos, self.node, self.fields = pos, node, fields


class _Ident:
    __slots__ = ("pos", "name")

    def __init__(self, pos, name):
        self.pos, self.name = pos, name


class _Dot:
    __slots__ = ("pos",)

    def __init__(self, pos):
        self.pos = pos


class _Nil:
    __slots__ = ("pos",)

    def __init__(self, pos):
        self.pos = pos


class _Bool:
    __slots__ = ("pos", "value")

    def __init__(self, pos, value):
        self.pos, self.value = pos, value


class _Number:
    __slots__ = ("pos", "text", "value", "error")

    def __init__(self, pos, text, value, error):
        self.pos, self.text, self.value, self.error = pos, text, value, error


class _String:
    __slots__ = ("pos", "quoted", "text")

    def __init__(self, pos, quoted, text):
        self.pos, self.quoted, self.text = pos, quoted, text


class _Branch:
    """if / range / with."""
    __slots__ = ("pos", "kind", "pipe", "body", "else_body")

    def __init__(self, pos, kind, pipe, body, else_body):
        self.pos, self.kind, self.pipe, self.body, self.else_body = pos, kind, pipe, body, else_body


class _TemplateCall:
    __slots__ = ("pos", "name", "pipe")

    def __init__(self, pos, name, pipe):
        self.pos, self.name, self.pipe = pos, name, pipe


class _End:
    __slots__ = ("pos",)

    def __init__(self, pos):
        self.pos = pos


class _Else:
    __slots__ = ("pos",)

    def __init__(self, pos):
        self.pos = pos


_NODE_TYPES = (_Text, _Action, _Pipe, _Command, _Field, _Variable, _Chain, _Ident, _Dot, _Nil, _Bool,
               _Number, _String, _Branch, _TemplateCall)
_NODE_TAG = {t: i for i, t in enumerate(_NODE_TYPES)}


def _node_str(n):
    """parse/node.go: the String() of a node (exec error contexts)."""
    t = type(n)
    if t is _Field:
        return "".join("." + x for x in n.idents)
    if t is _Variable:
        return ".".join(n.idents)
    if t is _Ident:
        return n.name
    if t is _Dot:
        return "."
    if t is _Nil:
        return "nil"
    if t is _Bool:
        return "true" if n.value else "false"
    if t is _Number:
        return n.text
    if t is _String:
        return n.quoted
    if t is _Chain:
        s = _node_str(n.node)
        if type(n.node) is _Pipe:
            s = "(" + s + ")"
        return s + "".join("." + f for f in n.fields)
    if t is _Command:
        return " ".join("(" + _node_str(a) + ")" if type(a) is _Pipe else _node_str(a) for a in n.args)
    if t is _Pipe:
        decl = ", ".join(n.decls) + " := " if n.decls else ""
        return decl + " | ".join(_node_str(c) for c in n.cmds)
    if t is _Action:
        return "{{" + _node_str(n.pipe) + "}}"
    if t is _TemplateCall:
        if n.pipe is None:
            return "{{template %s}}" % go_quote(n.name)
        return "{{template %s %s}}" % (go_quote(n.name), _node_str(n.pipe))
    if t is _Branch:
        s = "{{%s %s}}%s" % (n.kind, _node_str(n.pipe), _list_str(n.body))
        if n.else_body is not None:
            s += "{{else}}" + _list_str(n.else_body)
        return s + "{{end}}"
    if t is _Text:
        return n.text
    if t is _End:
        return "{{end}}"
    if t is _Else:
        return "{{else}}"
    return "?"


def _list_str(nodes):
    return "".join(_node_str(n) for n in nodes)


# ---------------------------------------------------------------------------
# Parser (parse/parse.go, Go 1.15)
# ---------------------------------------------------------------------------

_TERM_START = frozenset((I_BOOL, I_CHARCONST, I_COMPLEX, I_DOT, I_FIELD, I_IDENT, I_NUMBER, I_NIL,
                         I_RAWSTRING, I_STRING, I_VARIABLE, I_LPAREN))


class _Parser:
    def __init__(self, src, items, funcs, name):
        self.src = src
        self.items = items
        self.i = 0
        self.funcs = funcs
        self.name = name
        self.vars = ["$"]
        self.defines = {}
        self.last = items[0] if items else (I_EOF, "", 0)

    # -- tokens ----------------------------------------------------------------
    def next(self):
        it = self.items[self.i] if self.i < len(self.items) else self.items[-1]
        self.i += 1
        self.last = it
        return it

    def backup(self, k=1):
        self.i -= k

    def peek(self):
        return self.items[self.i] if self.i < len(self.items) else self.items[-1]

    def next_non_space(self):
        while True:
            it = self.next()
            if it[0] != I_SPACE:
                return it

    def peek_non_space(self):
        it = self.next_non_space()
        self.backup()
        return it

    def errorf(self, msg):
        line = self.src.count("\n", 0, self.last[2]) + 1
        raise TemplateError("template: %s:%d: %s" % (self.name, line, msg))

    def expect(self, kind, context):
        it = self.next_non_space()
        if it[0] != kind:
            self.unexpected(it, context)
        return it

    def unexpected(self, it, context):
        if it[0] == I_ERROR:
            self.errorf(it[1])
        self.errorf("unexpected %s in %s" % (_item_str(it), context))

    # -- structure -------------------------------------------------------------
    def parse(self):
        root = []
        while self.peek()[0] != I_EOF:
            if self.peek()[0] == I_LDELIM:
                mark = self.i
                self.next()
                if self.next_non_space()[0] == I_DEFINE:
                    self.parse_definition()
                    continue
                self.i = mark
            n = self.text_or_action()
            if type(n) in (_End, _Else):
                self.errorf("unexpected %s" % _node_str(n))
            root.append(n)
        return root

    def add_define(self, name, body):
        """parse.go: Tree.add (a later non-empty definition of a name is an error)."""
        old = self.defines.get(name)
        if old is not None and _nonempty(old) and _nonempty(body):
            self.errorf("template: multiple definition of template %s" % go_quote(name))
        if old is None or not _nonempty(old):
            self.defines[name] = body

    def parse_definition(self):
        context = "define clause"
        it = self.next_non_space()
        if it[0] not in (I_STRING, I_RAWSTRING):
            self.unexpected(it, context)
        name = self._unquote(it)
        self.expect(I_RDELIM, context)
        saved = self.vars
        self.vars = ["$"]
        body, end = self.item_list()
        self.vars = saved
        if type(end) is not _End:
            self.errorf("unexpected %s in %s" % (_node_str(end), context))
        self.add_define(name, body)

    def item_list(self):
        nodes = []
        while self.peek_non_space()[0] != I_EOF:
            n = self.text_or_action()
            if type(n) in (_End, _Else):
                return nodes, n
            nodes.append(n)
        self.errorf("unexpected EOF")

    def text_or_action(self):
        it = self.next_non_space()
        if it[0] == I_TEXT:
            return _Text(it[2], it[1])
        if it[0] == I_LDELIM:
            return self.action()
        self.unexpected(it, "input")

    def action(self):
        it = self.next_non_space()
        k = it[0]
        if k == I_BLOCK:
            return self.block_control()
        if k == I_ELSE:
            return self.else_control()
        if k == I_END:
            return _End(self.expect(I_RDELIM, "end")[2])
        if k == I_IF:
            return self.control("if", True)
        if k == I_RANGE:
            return self.control("range", False)
        if k == I_TEMPLATE:
            return self.template_control()
        if k == I_WITH:
            return self.control("with", False)
        self.backup()
        pos = self.peek()[2]
        return _Action(pos, self.pipeline("command"))

    def control(self, kind, allow_else_if):
        """parse.go: parseControl (variables declared here end at {{end}})."""
        nvars = len(self.vars)
        pipe = self.pipeline(kind)
        body, nxt = self.item_list()
        else_body = None
        if type(nxt) is _Else:
            if allow_else_if and self.peek()[0] == I_IF:
                # {{if a}}_{{else if b}}_{{end}} is {{if a}}_{{else}}{{if b}}_{{end}}{{end}}
                self.next()
                else_body = [self.control("if", True)]
            else:
                else_body, nxt = self.item_list()
                if type(nxt) is not _End:
                    self.errorf("expected end; found %s" % _node_str(nxt))
        del self.vars[nvars:]
        return _Branch(pipe.pos, kind, pipe, body, else_body)

    def else_control(self):
        peek = self.peek_non_space()
        if peek[0] == I_IF:
            return _Else(peek[2])   # "else if": the if stays pending
        return _Else(self.expect(I_RDELIM, "else")[2])

    def block_control(self):
        context = "block clause"
        it = self.next_non_space()
        name = self.template_name(it, context)
        pipe = self.pipeline(context)
        saved = self.vars
        self.vars = ["$"]
        body, end = self.item_list()
        self.vars = saved
        if type(end) is not _End:
            self.errorf("unexpected %s in %s" % (_node_str(end), context))
        self.add_define(name, body)
        return _TemplateCall(it[2], name, pipe)

    def template_control(self):
        context = "template clause"
        it = self.next_non_space()
        name = self.template_name(it, context)
        pipe = None
        if self.next_non_space()[0] != I_RDELIM:
            self.backup()
            pipe = self.pipeline(context)
        return _TemplateCall(it[2], name, pipe)

    def template_name(self, it, context):
        if it[0] in (I_STRING, I_RAWSTRING):
            return self._unquote(it)
        self.unexpected(it, context)

    def _unquote(self, it):
        try:
            return _unquote(it[1])
        except (ValueError, IndexError):
            self.errorf("invalid syntax")

    # -- pipelines -------------------------------------------------------------
    def pipeline(self, context):
        pos = self.peek_non_space()[2]
        decls = []
        is_assign = False
        while True:  # decls:
            v = self.peek_non_space()
            if v[0] == I_VARIABLE:
                vi = self.i
                self.next_non_space()
                nxt = self.peek_non_space()
                if nxt[0] in (I_ASSIGN, I_DECLARE):
                    is_assign = nxt[0] == I_ASSIGN
                    self.next_non_space()
                    decls.append(v[1])
                    self.vars.append(v[1])
                elif nxt[0] == I_CHAR and nxt[1] == ",":
                    self.next_non_space()
                    decls.append(v[1])
                    self.vars.append(v[1])
                    if context == "range" and len(decls) < 2:
                        if self.peek_non_space()[0] in (I_VARIABLE, I_RDELIM, I_RPAREN):
                            continue
                        self.errorf("range can only initialize variables")
                    self.errorf("too many declarations in %s" % context)
                else:
                    self.i = vi
            break
        cmds = []
        while True:
            it = self.next_non_space()
            k = it[0]
            if k in (I_RDELIM, I_RPAREN):
                if not cmds:
                    self.errorf("missing value for %s" % context)
                for n, c in enumerate(cmds[1:]):
                    if type(c.args[0]) in (_Bool, _Dot, _Nil, _Number, _String):
                        self.errorf("non executable command in pipeline stage %d" % (n + 2))
                if k == I_RPAREN:
                    self.backup()
                return _Pipe(pos, decls, cmds, is_assign)
            if k in _TERM_START:
                self.backup()
                cmds.append(self.command())
            else:
                self.unexpected(it, context)

    def command(self):
        pos = self.peek_non_space()[2]
        args = []
        while True:
            self.peek_non_space()
            op = self.operand()
            if op is not None:
                args.append(op)
            it = self.next()
            k = it[0]
            if k == I_SPACE:
                continue
            if k == I_ERROR:
                self.errorf(it[1])
            if k in (I_RDELIM, I_RPAREN):
                self.backup()
            elif k != I_PIPE:
                self.errorf("unexpected %s in operand" % _item_str(it))
            break
        if not args:
            self.errorf("empty command")
        return _Command(pos, args)

    def operand(self):
        node = self.term()
        if node is None:
            return None
        if self.peek()[0] == I_FIELD:
            cpos = self.peek()[2]
            fields = []
            while self.peek()[0] == I_FIELD:
                fields.append(self.next()[1][1:])
            t = type(node)
            if t is _Field:
                return _Field(cpos, node.idents + tuple(fields))
            if t is _Variable:
                return _Variable(cpos, node.idents + tuple(fields))
            if t in (_Bool, _String, _Number, _Nil, _Dot):
                self.errorf("unexpected . after term %s" % go_quote(_node_str(node)))
            return _Chain(cpos, node, tuple(fields))
        return node

    def term(self):
        it = self.next_non_space()
        k, val, pos = it
        if k == I_ERROR:
            self.errorf(val)
        if k == I_IDENT:
            if val not in self.funcs:
                self.errorf("function %s not defined" % go_quote(val))
            return _Ident(pos, val)
        if k == I_DOT:
            return _Dot(pos)
        if k == I_NIL:
            return _Nil(pos)
        if k == I_VARIABLE:
            name = val
            if name not in self.vars:
                self.errorf("undefined variable %s" % go_quote(name))
            return _Variable(pos, (name,))
        if k == I_FIELD:
            return _Field(pos, (val[1:],))
        if k == I_BOOL:
            return _Bool(pos, val == "true")
        if k in (I_CHARCONST, I_COMPLEX, I_NUMBER):
            value, err, at_parse = _ideal_constant(val, k)
            if err is not None and at_parse:
                self.errorf(err)
            return _Number(pos, val, value, err)
        if k == I_LPAREN:
            pipe = self.pipeline("parenthesized pipeline")
            it2 = self.next()
            if it2[0] != I_RPAREN:
                self.errorf("unclosed right paren: unexpected %s" % _item_str(it2))
            return pipe
        if k in (I_STRING, I_RAWSTRING):
            return _String(pos, val, self._unquote(it))
        self.backup()
        return None


def _nonempty(nodes):
    """parse.go: IsEmptyTree is false (anything but space-only text)."""
    for n in nodes:
        if type(n) is not _Text or n.text.strip(" \t\r\n"):
            return True
    return False


# ---------------------------------------------------------------------------
# Parse trees as plain data (utils/startcache.py)
# ---------------------------------------------------------------------------

def _to_data(n):
    """A node as a tuple (tag, pos, fields...); node lists as lists."""
    if n is None:
        return None
    if type(n) is list:
        return [_to_data(e) for e in n]
    t = type(n)
    tag = _NODE_TAG[t]
    if t is _Text:
        return (tag, n.pos, n.text)
    if t is _Action:
        return (tag, n.pos, _to_data(n.pipe))
    if t is _Pipe:
        return (tag, n.pos, tuple(n.decls), [_to_data(c) for c in n.cmds], n.is_assign)
    if t is _Command:
        return (tag, n.pos, [_to_data(a) for a in n.args])
    if t is _Chain:
        return (tag, n.pos, _to_data(n.node), n.fields)
    if t is _Branch:
        return (tag, n.pos, n.kind, _to_data(n.pipe), _to_data(n.body), _to_data(n.else_body))
    if t is _TemplateCall:
        return (tag, n.pos, n.name, _to_data(n.pipe))
    # leaves: every slot is a constant
    return (tag,) + tuple(getattr(n, a) for a in t.__slots__)


def _from_data(d):
    if d is None:
        return None
    if type(d) is list:
        return [_from_data(e) for e in d]
    return _DECODE[d[0]](d)


def _dec_leaf(cls):
    return lambda d: cls(*d[1:])


_DECODE = [
    _dec_leaf(_Text),
    lambda d: _Action(d[1], _from_data(d[2])),
    lambda d: _Pipe(d[1], list(d[2]), [_from_data(c) for c in d[3]], d[4]),
    lambda d: _Command(d[1], [_from_data(a) for a in d[2]]),
    _dec_leaf(_Field), _dec_leaf(_Variable),
    lambda d: _Chain(d[1], _from_data(d[2]), d[3]),
    _dec_leaf(_Ident), _dec_leaf(_Dot), _dec_leaf(_Nil), _dec_leaf(_Bool), _dec_leaf(_Number), _dec_leaf(_String),
    lambda d: _Branch(d[1], d[2], _from_data(d[3]), _from_data(d[4]), _from_data(d[5])),
    lambda d: _TemplateCall(d[1], d[2], _from_data(d[3])),
]


# ---------------------------------------------------------------------------
# Template
# ---------------------------------------------------------------------------

class Template:
    """A parsed Go 1.15 text/template (``template.New(name).Parse(src)``)."""

    def __init__(self, src, name="", funcs=None):
        self.name = name
        self.text = src
        names = _BUILTIN_NAMES if not funcs else _BUILTIN_NAMES | frozenset(funcs)
        p = _Parser(src, _lex(src), names, name)
        self.root = p.parse()
        self.defines = p.defines

    # -- the parsed form as plain data (utils/startcache.py) -----------------
    def to_data(self):
        """The parse tree as nested tuples, lists and constants (marshal-able)."""
        return (_to_data(self.root), {k: _to_data(v) for k, v in self.defines.items()})

    @classmethod
    def from_data(cls, data, name="", src=""):
        """The template :meth:`to_data` described, without parsing."""
        t = cls.__new__(cls)
        t.name = name
        t.text = src
        root, defines = data
        t.root = _from_data(root)
        t.defines = {k: _from_data(v) for k, v in defines.items()}
        return t

    # -- execution ---------------------------------------------------------
    def execute(self, data, funcs=None):
        """exec.go: Template.Execute; raises TemplateError with Go's text."""
        st = _State(self, self.name, funcs)
        out = st.out
        if data is None:
            data = NO_VALUE   # Execute(w, nil): reflect.ValueOf(nil) is the zero Value
        st.vars = [("$", data)]
        try:
            run = self.__dict__.get("_run")
            if run is None:
                # compiling costs about three executions: a template a process
                # executes once (most of them, in a cold CLI run) is interpreted
                runs = self.__dict__.get("_runs", 0)
                if INTERPRET or runs < COMPILE_AFTER:
                    self._runs = runs + 1
                    st.walk_list(data, self.root)
                    return "".join(out)
                run = self._run = _c_list(self.root)
            run(st, data)
        except RecursionError:
            raise TemplateError("template: %s: exceeded maximum template depth (%d)" % (self.name, MAX_EXEC_DEPTH))
        return "".join(out)

    def compiled_define(self, name):
        """The compiled body of ``{{define name}}``, or None."""
        cache = self.__dict__.setdefault("_defines_run", {})
        run = cache.get(name)
        if run is None:
            body = self.defines.get(name)
            if body is None:
                return None
            run = cache[name] = _c_list(body)
        return run


# ---------------------------------------------------------------------------
# Execution helpers shared by the interpreter and the closures (exec.go)
# ---------------------------------------------------------------------------

def _utf8_len(s):
    return len(s.encode("utf-8", "surrogateescape"))


def _exec_error(st, node, msg):
    """exec.go: state.errorf with the node's location and context."""
    text = st.tmpl.text or ""
    pos = node.pos if node is not None else 0
    prefix = text[:pos]
    nl = prefix.rfind("\n")
    col = _utf8_len(prefix) if nl < 0 else _utf8_len(prefix[nl + 1:])
    line = 1 + prefix.count("\n")
    ctx = _node_str(node) if node is not None else ""
    if len(ctx) > 20:
        ctx = ctx[:20] + "..."
    return TemplateError("template: %s:%d:%d: executing %s at <%s>: %s"
                         % (st.tmpl.name, line, col, go_quote(st.name), ctx, msg))


class _State:
    __slots__ = ("tmpl", "name", "vars", "depth", "out", "funcs")

    def __init__(self, tmpl, name, funcs=None, out=None, depth=0):
        self.tmpl = tmpl
        self.name = name
        self.vars = None
        self.depth = depth
        self.out = [] if out is None else out
        self.funcs = funcs

    # -- variables -------------------------------------------------------------
    def var_value(self, node, name):
        for k in range(len(self.vars) - 1, -1, -1):
            if self.vars[k][0] == name:
                return self.vars[k][1]
        raise _exec_error(self, node, "undefined variable: %s" % name)

    def set_var(self, node, name, value):
        for k in range(len(self.vars) - 1, -1, -1):
            if self.vars[k][0] == name:
                self.vars[k] = (name, value)
                return
        raise _exec_error(self, node, "undefined variable: %s" % name)

    # -- the tree walker ---------------------------------------------------------
    def walk_list(self, dot, nodes):
        for n in nodes:
            t = type(n)
            if t is _Text:
                self.out.append(n.text)
            elif t is _Action:
                val = self.eval_pipeline(dot, n.pipe)
                if not n.pipe.decls:
                    self.out.append(_print_value(self, n, val))
            elif t is _Branch:
                if n.kind == "range":
                    self.walk_range(dot, n)
                else:
                    self.walk_if_or_with(dot, n)
            else:
                self.walk_template(dot, n)

    def walk_if_or_with(self, dot, n):
        mark = len(self.vars)
        val = self.eval_pipeline(dot, n.pipe)
        if _truth(val):
            self.walk_list(val if n.kind == "with" else dot, n.body)
        elif n.else_body is not None:
            self.walk_list(dot, n.else_body)
        del self.vars[mark:]

    def walk_range(self, dot, n):
        mark0 = len(self.vars)
        val = self.eval_pipeline(dot, n.pipe)
        items = _range_items(self, n, val)
        mark = len(self.vars)
        ndecl = len(n.pipe.decls)
        if items:
            for k, v in items:
                if ndecl > 0:
                    self.vars[mark - 1] = (self.vars[mark - 1][0], v)
                if ndecl > 1:
                    self.vars[mark - 2] = (self.vars[mark - 2][0], k)
                self.walk_list(v, n.body)
                del self.vars[mark:]
        elif n.else_body is not None:
            self.walk_list(dot, n.else_body)
        del self.vars[mark0:]

    def walk_template(self, dot, n):
        body = self.tmpl.defines.get(n.name)
        if body is None:
            raise _exec_error(self, n, "template %s not defined" % go_quote(n.name))
        if self.depth >= MAX_EXEC_DEPTH:
            raise _exec_error(self, n, "exceeded maximum template depth (%d)" % MAX_EXEC_DEPTH)
        # {{template "x"}} runs with the zero Value as its data
        newdot = self.eval_pipeline(dot, n.pipe) if n.pipe is not None else NO_VALUE
        st = _State(self.tmpl, n.name, self.funcs, self.out, self.depth + 1)
        st.vars = [("$", newdot)]
        st.walk_list(newdot, body)

    # -- pipelines -------------------------------------------------------------
    def eval_pipeline(self, dot, pipe):
        val = _MISSING
        for cmd in pipe.cmds:
            val = self.eval_command(dot, cmd, val)
            if val is None:
                val = NO_VALUE   # a nil interface dug out: the zero Value
        if pipe.decls:
            for name in pipe.decls:
                if pipe.is_assign:
                    self.set_var(pipe, name, val)
                else:
                    self.vars.append((name, val))
        return val

    def eval_command(self, dot, cmd, final):
        first = cmd.args[0]
        t = type(first)
        if t is _Field:
            return self.eval_field_chain(dot, dot, first, first.idents, cmd.args, final)
        if t is _Ident:
            return self.eval_function(dot, first, cmd, cmd.args, final)
        if t is _Variable:
            return self.eval_variable(dot, first, cmd.args, final)
        if t is _Chain:
            return self.eval_chain(dot, first, cmd.args, final)
        if t is _Pipe:
            _not_a_function(self, first, cmd.args, final)
            return self.eval_pipeline(dot, first)
        _not_a_function(self, first, cmd.args, final)
        return _literal_command(self, first, dot)

    def eval_field_chain(self, dot, receiver, node, idents, args, final):
        for name in idents[:-1]:
            receiver = _field(self, node, name, False, receiver, None)
        has_args = (args is not None and len(args) > 1) or final is not _MISSING
        margs = None
        if has_args:
            margs = lambda: [self.eval_arg(dot, "I", a) for a in args[1:]] + ([] if final is _MISSING else [final])  # noqa: E731
        return _field(self, node, idents[-1], has_args, receiver, margs)

    def eval_chain(self, dot, chain, args, final):
        if type(chain.node) is _Nil:
            raise _exec_error(self, chain, "indirection through explicit nil in %s" % _node_str(chain))
        recv = self.eval_arg(dot, None, chain.node)
        return self.eval_field_chain(dot, recv, chain, chain.fields, args, final)

    def eval_variable(self, dot, var, args, final):
        value = self.var_value(var, var.idents[0])
        if len(var.idents) == 1:
            _not_a_function(self, var, args, final)
            return value
        return self.eval_field_chain(dot, value, var, var.idents[1:], args, final)

    def eval_function(self, dot, ident, node, args, final):
        spec = _spec(self, ident)
        argnodes = args[1:] if args is not None else ()
        nin = len(argnodes) + (final is not _MISSING)
        fixed, variadic = spec[1], spec[2]
        _check_arity(self, ident, spec, len(argnodes), nin)
        vals = []
        for i, a in enumerate(argnodes):
            vals.append(self.eval_arg(dot, fixed[i] if i < len(fixed) else variadic, a))
        if final is not _MISSING:
            vals.append(_validate(self, node, final, _final_type(spec, nin)))
        return _invoke(self, spec, ident.name, node, vals)

    def eval_arg(self, dot, typ, n):
        """exec.go: evalArg for a parameter of type typ ('V' reflect.Value,
        'I' interface{}, 'S' string, None untyped)."""
        t = type(n)
        if t is _Dot:
            return _validate(self, n, dot, typ)
        if t is _Nil:
            return _nil_arg(self, n, typ)
        if t is _Field:
            return _validate(self, n, self.eval_field_chain(dot, dot, n, n.idents, None, _MISSING), typ)
        if t is _Variable:
            return _validate(self, n, self.eval_variable(dot, n, None, _MISSING), typ)
        if t is _Pipe:
            return _validate(self, n, self.eval_pipeline(dot, n), typ)
        if t is _Ident:
            return _validate(self, n, self.eval_function(dot, n, n, None, _MISSING), typ)
        if t is _Chain:
            return _validate(self, n, self.eval_chain(dot, n, None, _MISSING), typ)
        return _literal_arg(self, n, typ)


def _not_a_function(st, node, args, final):
    if (args is not None and len(args) > 1) or final is not _MISSING:
        raise _exec_error(st, node, "can't give argument to non-function %s" % _node_str(args[0]))


def _literal_command(st, n, dot):
    t = type(n)
    if t is _Bool:
        return n.value
    if t is _Dot:
        return dot
    if t is _Nil:
        raise _exec_error(st, n, "nil is not a command")
    if t is _Number:
        return _number_value(st, n)
    if t is _String:
        return n.text
    raise _exec_error(st, n, "can't evaluate command %s" % go_quote(_node_str(n)))


def _number_value(st, n):
    if n.error is not None:
        raise _exec_error(st, n, n.error)
    return n.value


def _literal_arg(st, n, typ):
    """evalArg's typed branch for a literal (evalString / evalEmptyInterface)."""
    t = type(n)
    if typ == "S":
        if t is _String:
            return n.text
        raise _exec_error(st, n, "expected string; found %s" % _node_str(n))
    if t is _Bool:
        return n.value
    if t is _Number:
        return _number_value(st, n)
    if t is _String:
        return n.text
    raise _exec_error(st, n, "can't handle assignment of %s to empty interface argument" % _node_str(n))


def _nil_arg(st, n, typ):
    if typ == "V":
        return NO_VALUE
    if typ == "I" or typ is None:
        return None
    raise _exec_error(st, n, "cannot assign nil to string")


def _validate(st, node, value, typ):
    """exec.go: validateType."""
    if typ == "I":
        return None if value is NO_VALUE else value
    if typ == "S":
        if type(value) is str:
            return value
        if value is NO_VALUE:
            raise _exec_error(st, node, "invalid value; expected string")
        got = "interface {}" if value is None else type_string(value)
        raise _exec_error(st, node, "wrong type for value; expected string; got %s" % got)
    return value


def _field(st, node, name, has_args, receiver, margs):
    """exec.go: evalField (a missing map key is the zero Value)."""
    if receiver is NO_VALUE:
        return NO_VALUE
    if receiver is None:
        raise _exec_error(st, node, "nil pointer evaluating interface {}.%s" % name)
    if type(receiver) is dict or isinstance(receiver, dict):
        if has_args:
            raise _exec_error(st, node, "%s is not a method but has arguments" % name)
        return receiver.get(name, NO_VALUE)
    if not isinstance(receiver, (str, int, float, complex, list, tuple, bytes)) and not name.startswith("_"):
        attr = getattr(receiver, name, _MISSING)
        if attr is not _MISSING:
            if callable(attr) and not isinstance(attr, type):
                try:
                    return attr(*(margs() if margs is not None else ()))
                except TemplateError:
                    raise
                except Exception as e:  # noqa: BLE001
                    raise _exec_error(st, node, "error calling %s: %s" % (name, e))
            if has_args:
                raise _exec_error(st, node, "%s has arguments but cannot be invoked as function" % name)
            return attr
    raise _exec_error(st, node, "can't evaluate field %s in type %s" % (name, _receiver_type(receiver)))


def _receiver_type(v):
    if isinstance(v, (str, int, float, complex, list, tuple, bytes, dict)):
        return "interface {}"
    return type(v).__name__


def _truth(v):
    """exec.go: isTrue(indirectInterface(v))."""
    if v is NO_VALUE or v is None:
        return False
    t = type(v)
    if t is bool:
        return v
    if t is str or t is list or t is dict or t is tuple or t is bytes:
        return len(v) > 0
    if t is int or t is float or t is complex or t is GoUint8:
        return v != 0
    if isinstance(v, (str, list, dict, tuple, bytes)):
        return len(v) > 0
    return True


def _range_items(st, n, val):
    """exec.go: walkRange's switch over the value's kind."""
    t = type(val)
    if t is list or t is tuple or isinstance(val, (list, tuple)):
        return list(enumerate(val))
    if t is dict or isinstance(val, dict):
        return [(k, val[k]) for k in sorted_keys(val)]
    if val is NO_VALUE or val is None:
        return []
    if t is bytes:
        return [(i, GoUint8(b)) for i, b in enumerate(val)]
    raise _exec_error(st, _range_context(n), "range can't iterate over %s" % sprint_one(val))


def _range_context(n):
    """The node exec.go's state points at after evaluating a range pipeline."""
    cmd = n.pipe.cmds[-1]
    first = cmd.args[0]
    if type(first) in (_Field, _Variable, _Chain):
        return first
    if type(first) is _Ident:
        return cmd if len(cmd.args) == 1 else cmd.args[-1]
    return first


def _print_value(st, node, v):
    """exec.go: printValue (the zero Value prints ``<no value>``)."""
    t = type(v)
    if t is str:
        return v
    if v is NO_VALUE or v is None:
        return "<no value>"
    if callable(v) and not isinstance(v, (list, dict, tuple)) and t not in (int, float, bool):
        raise _exec_error(st, node, "can't print %s of type %s" % (_node_str(node), type_string(v)))
    return sprint_one(v)


# ---------------------------------------------------------------------------
# Builtins (funcs.go, Go 1.15)
# ---------------------------------------------------------------------------

def _b_and(arg0, *args):
    if not _truth(arg0):
        return arg0
    for a in args:
        arg0 = a
        if not _truth(a):
            break
    return arg0


def _b_or(arg0, *args):
    if _truth(arg0):
        return arg0
    for a in args:
        arg0 = a
        if _truth(a):
            break
    return arg0


def _b_not(arg):
    return not _truth(arg)


_BAD_TYPE = "invalid type for comparison"        # funcs.go: errBadComparisonType
_BAD_CMP = "incompatible types for comparison"   # funcs.go: errBadComparison
_NO_CMP = "missing argument for comparison"      # funcs.go: errNoComparison


def _basic_kind(v):
    """funcs.go: basicKind -> 'bool' | 'int' | 'uint' | 'float' | 'complex' | 'string'."""
    t = type(v)
    if t is str:
        return "string"
    if t is int:
        return "int"
    if t is float:
        return "float"
    if t is bool:
        return "bool"
    if t is GoUint8:
        return "uint"
    if t is complex:
        return "complex"
    raise _GoError(_BAD_TYPE)


def _b_eq(arg1, *arg2):
    k1 = _basic_kind(arg1)
    if not arg2:
        raise _GoError(_NO_CMP)
    for b in arg2:
        k2 = _basic_kind(b)
        if k1 != k2:
            if {k1, k2} == {"int", "uint"}:
                truth = arg1 == b and (arg1 >= 0 and b >= 0)
            else:
                raise _GoError(_BAD_CMP)
        else:
            truth = arg1 == b
        if truth:
            return True
    return False


def _b_ne(arg1, arg2):
    return not _b_eq(arg1, arg2)


def _b_lt(arg1, arg2):
    k1 = _basic_kind(arg1)
    k2 = _basic_kind(arg2)
    if k1 != k2:
        if k1 == "int" and k2 == "uint":
            return arg1 < 0 or arg1 < arg2
        if k1 == "uint" and k2 == "int":
            return arg2 >= 0 and arg1 < arg2
        raise _GoError(_BAD_CMP)
    if k1 in ("bool", "complex"):
        raise _GoError(_BAD_TYPE)
    return arg1 < arg2


def _b_le(arg1, arg2):
    if _b_lt(arg1, arg2):
        return True
    return _b_eq(arg1, arg2)


def _b_gt(arg1, arg2):
    return not _b_le(arg1, arg2)


def _b_ge(arg1, arg2):
    return not _b_lt(arg1, arg2)


def _index_arg(index, cap_):
    """funcs.go: indexArg."""
    if index is NO_VALUE or index is None:
        raise _GoError("cannot index slice/array with nil")
    if type(index) not in (int, GoUint8):
        raise _GoError("cannot index slice/array with type %s" % type_string(index))
    if index < 0 or index > cap_:
        raise _GoError("index out of range: %d" % index)
    return index


def _b_index(item, *indexes):
    """funcs.go: index (a string indexes its bytes; a missing key is nil)."""
    if item is NO_VALUE or item is None:
        raise _GoError("index of untyped nil")
    for index in indexes:
        if item is None:
            raise _GoError("index of nil pointer")
        t = type(item)
        if t is str or t is list or t is tuple or t is bytes:
            b = item.encode("utf-8", "surrogateescape") if t is str else item
            x = _index_arg(index, len(b))
            if x == len(b):
                raise _GoError("reflect: %s index out of range" % ("string" if t is str else "slice"))
            item = GoUint8(b[x]) if t in (str, bytes) else item[x]
        elif isinstance(item, dict):
            if index is NO_VALUE:
                index = None
            if type(index) is not str:
                if index is None:
                    raise _GoError("value is nil; should be of type string")
                raise _GoError("value has type %s; should be string" % type_string(index))
            item = item.get(index)
        else:
            raise _GoError("can't index item of type %s" % type_string(item))
    return item


def _b_slice(item, *indexes):
    """funcs.go: slice."""
    if item is NO_VALUE or item is None:
        raise _GoError("slice of untyped nil")
    if len(indexes) > 3:
        raise _GoError("too many slice indexes: %d" % len(indexes))
    t = type(item)
    if t is str:
        if len(indexes) == 3:
            raise _GoError("cannot 3-index slice a string")
        seq = item.encode("utf-8", "surrogateescape")
    elif t in (list, tuple, bytes):
        seq = item
    else:
        raise _GoError("can't slice item of type %s" % type_string(item))
    cap_ = len(seq)
    idx = [0, len(seq), len(seq)]
    for i, index in enumerate(indexes):
        idx[i] = _index_arg(index, cap_)
    if idx[0] > idx[1]:
        raise _GoError("invalid slice index: %d > %d" % (idx[0], idx[1]))
    if len(indexes) == 3 and idx[1] > idx[2]:
        raise _GoError("invalid slice index: %d > %d" % (idx[1], idx[2]))
    out = seq[idx[0]:idx[1]]
    if t is str:
        return out.decode("utf-8", "surrogateescape")
    return list(out) if t is tuple else out


def _b_len(item):
    """funcs.go: length (a string's length is its byte count)."""
    if item is None:
        raise _GoError("len of nil pointer")
    if item is NO_VALUE:
        raise _GoError("reflect: call of reflect.Value.Type on zero Value")
    t = type(item)
    if t is str:
        return len(item.encode("utf-8", "surrogateescape"))
    if t in (list, tuple, dict, bytes) or isinstance(item, (list, dict)):
        return len(item)
    raise _GoError("len of type %s" % type_string(item))


def _b_call(fn, *args):
    """funcs.go: call."""
    if fn is NO_VALUE or fn is None:
        raise _GoError("call of nil")
    if not callable(fn) or isinstance(fn, type):
        raise _GoError("non-function of type %s" % type_string(fn))
    return fn(*[None if a is NO_VALUE else a for a in args])


def _eval_args(args):
    """funcs.go: evalArgs (one string passes through; nil prints <no value>)."""
    if len(args) == 1 and type(args[0]) is str:
        return args[0]
    return sprint([("<no value>" if a is None or a is NO_VALUE else a) for a in args])


_HTML_ESC = {'"': "&#34;", "'": "&#39;", "&": "&amp;", "<": "&lt;", ">": "&gt;", "\x00": "\ufffd"}


def _b_html(*args):
    """funcs.go: HTMLEscapeString."""
    s = _eval_args(args)
    if not any(c in s for c in "\"'&<>\x00"):
        return s
    return "".join(_HTML_ESC.get(c, c) for c in s)


def _b_js(*args):
    """funcs.go: JSEscapeString (parity unpinned for < > & =: \\u003C form)."""
    from .gofmt import is_print
    s = _eval_args(args)
    out = []
    for ch in s:
        o = ord(ch)
        if ch in "\\'\"":
            out.append("\\" + ch)
        elif ch in "<>&=":
            out.append("\\u%04X" % o)
        elif o < 0x20:
            out.append("\\u00%02X" % o)
        elif o >= 0x80 and not is_print(o):
            out.append("\\u%04X" % o)
        else:
            out.append(ch)
    return "".join(out)


def _b_urlquery(*args):
    """funcs.go: URLQueryEscaper (url.QueryEscape)."""
    import urllib.parse
    return urllib.parse.quote_plus(_eval_args(args).encode("utf-8", "surrogateescape"), safe="")


def _b_print(*args):
    return sprint(args)


def _b_println(*args):
    return sprintln(args)


def _b_printf(fmt, *args):
    return sprintf(fmt, list(args))


# name -> (function, fixed parameter types, variadic element type or None)
_SPECS = {
    "and": (_b_and, "V", "V"), "or": (_b_or, "V", "V"), "not": (_b_not, "V", None),
    "len": (_b_len, "V", None), "index": (_b_index, "V", "V"), "slice": (_b_slice, "V", "V"),
    "call": (_b_call, "V", "V"), "html": (_b_html, "", "I"), "js": (_b_js, "", "I"),
    "urlquery": (_b_urlquery, "", "I"), "print": (_b_print, "", "I"), "println": (_b_println, "", "I"),
    "printf": (_b_printf, "S", "I"),
    "eq": (_b_eq, "V", "V"), "ne": (_b_ne, "VV", None), "lt": (_b_lt, "VV", None),
    "le": (_b_le, "VV", None), "gt": (_b_gt, "VV", None), "ge": (_b_ge, "VV", None),
}
_BUILTIN_NAMES = frozenset(_SPECS)


def _user_spec(fn):
    return (fn, "", "I")


def _spec(st, ident):
    spec = _SPECS.get(ident.name)
    if spec is None and st.funcs and ident.name in st.funcs:
        spec = _user_spec(st.funcs[ident.name])
    if spec is None:
        raise _exec_error(st, ident, "%s is not a defined function" % go_quote(ident.name))
    return spec


def _check_arity(st, ident, spec, nargs, nin):
    """exec.go: evalCall's argument count checks."""
    fixed, variadic = spec[1], spec[2]
    if variadic is not None:
        if nin < len(fixed):
            raise _exec_error(st, ident, "wrong number of args for %s: want at least %d got %d"
                              % (ident.name, len(fixed), nargs))
    elif nin != len(fixed):
        raise _exec_error(st, ident, "wrong number of args for %s: want %d got %d" % (ident.name, len(fixed), nin))


def _final_type(spec, nin):
    fixed, variadic = spec[1], spec[2]
    if variadic is not None:
        return fixed[nin - 1] if nin - 1 < len(fixed) else variadic
    return fixed[-1]


def _invoke(st, spec, name, node, vals):
    try:
        return spec[0](*vals)
    except _GoError as e:
        raise _exec_error(st, node, "error calling %s: %s" % (name, e))
    except TemplateError:
        raise
    except RecursionError:
        raise
    except Exception as e:  # noqa: BLE001 - a panic in a function: safeCall
        raise _exec_error(st, node, "error calling %s: %s" % (name, e))


# ---------------------------------------------------------------------------
# Compilation to closures
# ---------------------------------------------------------------------------
# Each node becomes a Python closure once per parsed template, so executing it
# does no per-node dispatch on node kinds.  The closures follow _State's
# walk_* / eval_* methods step for step (same evaluation order, same helpers,
# same errors).  A template is compiled on its second execution
# (COMPILE_AFTER); M2K_TEMPLATE_INTERPRET=1 keeps the interpreter, and
# tests/test_gotemplate_compiled.py checks the two agree on every packaged
# template and the template test corpus.

def _c_list(nodes):
    fns = tuple(_c_node(n) for n in nodes)
    if len(fns) == 1:
        return fns[0]

    def run(st, dot):
        for f in fns:
            f(st, dot)
    return run


def _c_node(n):
    t = type(n)
    if t is _Text:
        text = n.text

        def text_node(st, dot):
            st.out.append(text)
        return text_node
    if t is _Action:
        pipe = _c_pipe(n.pipe)
        if n.pipe.decls:
            def declare_node(st, dot):
                pipe(st, dot)
            return declare_node

        def action_node(st, dot):
            v = pipe(st, dot)
            st.out.append(v if type(v) is str else _print_value(st, n, v))
        return action_node
    if t is _Branch:
        return _c_range(n) if n.kind == "range" else _c_if_or_with(n)
    return _c_template(n)


def _c_if_or_with(n):
    pipe = _c_pipe(n.pipe)
    body = _c_list(n.body)
    else_body = None if n.else_body is None else _c_list(n.else_body)
    is_with = n.kind == "with"

    def cond_node(st, dot):
        mark = len(st.vars)
        val = pipe(st, dot)
        if _truth(val):
            body(st, val if is_with else dot)
        elif else_body is not None:
            else_body(st, dot)
        del st.vars[mark:]
    return cond_node


def _c_range(n):
    pipe = _c_pipe(n.pipe)
    body = _c_list(n.body)
    else_body = None if n.else_body is None else _c_list(n.else_body)
    ndecl = len(n.pipe.decls)

    def range_node(st, dot):
        vars_ = st.vars
        mark0 = len(vars_)
        val = pipe(st, dot)
        items = _range_items(st, n, val)
        mark = len(vars_)
        if items:
            for k, v in items:
                if ndecl > 0:
                    vars_[mark - 1] = (vars_[mark - 1][0], v)
                if ndecl > 1:
                    vars_[mark - 2] = (vars_[mark - 2][0], k)
                body(st, v)
                del vars_[mark:]
        elif else_body is not None:
            else_body(st, dot)
        del vars_[mark0:]
    return range_node


def _c_template(n):
    name = n.name
    pipe = _c_pipe(n.pipe) if n.pipe is not None else None

    def call_node(st, dot):
        body = st.tmpl.compiled_define(name)
        if body is None:
            raise _exec_error(st, n, "template %s not defined" % go_quote(name))
        if st.depth >= MAX_EXEC_DEPTH:
            raise _exec_error(st, n, "exceeded maximum template depth (%d)" % MAX_EXEC_DEPTH)
        newdot = pipe(st, dot) if pipe is not None else NO_VALUE
        sub = _State(st.tmpl, name, st.funcs, st.out, st.depth + 1)
        sub.vars = [("$", newdot)]
        body(sub, newdot)
    return call_node


def _c_pipe(pipe):
    """fn(st, dot) -> value of the pipeline, declaring or assigning its
    variables (exec.go: evalPipeline)."""
    cmds = tuple(_c_cmd(c, i > 0) for i, c in enumerate(pipe.cmds))
    decls = tuple(pipe.decls)
    if not decls and len(cmds) == 1:
        only = cmds[0]

        def single(st, dot):
            v = only(st, dot, _MISSING)
            return NO_VALUE if v is None else v
        return single
    is_assign = pipe.is_assign

    def run(st, dot):
        val = _MISSING
        for c in cmds:
            val = c(st, dot, val)
            if val is None:
                val = NO_VALUE
        for name in decls:
            if is_assign:
                st.set_var(pipe, name, val)
            else:
                st.vars.append((name, val))
        return val
    return run


def _c_cmd(cmd, has_final):
    """fn(st, dot, final) of one command of a pipeline (exec.go: evalCommand)."""
    first = cmd.args[0]
    t = type(first)
    args = cmd.args
    if t is _Field:
        return _c_field_chain(first, first.idents, args, has_final, None)
    if t is _Ident:
        return _c_function(first, cmd, args, has_final)
    if t is _Variable:
        return _c_variable(first, args, has_final)
    if t is _Chain:
        return _c_chain(first, args, has_final)
    if t is _Pipe:
        sub = _c_pipe(first)
        if len(args) > 1 or has_final:
            def refuse_pipe(st, dot, final):
                _not_a_function(st, first, args, final)
            return refuse_pipe
        return lambda st, dot, final: sub(st, dot)
    if len(args) > 1 or has_final:
        def refuse(st, dot, final):
            _not_a_function(st, first, args, final)
        return refuse
    if t is _Bool or t is _String or (t is _Number and first.error is None):
        v = first.value if t is not _String else first.text
        return lambda st, dot, final: v
    if t is _Dot:
        return lambda st, dot, final: dot
    return lambda st, dot, final: _literal_command(st, first, dot)


def _c_field_chain(node, idents, args, has_final, recv):
    """exec.go: evalFieldChain; recv is fn(st, dot) of the receiver (None: dot)."""
    head = tuple(idents[:-1])
    last = idents[-1]
    nargs = len(args) if args is not None else 0
    method_args = tuple(_c_arg(a, "I") for a in args[1:]) if nargs > 1 else ()

    def chain(st, dot, final):
        r = dot if recv is None else recv(st, dot)
        for name in head:
            r = _field(st, node, name, False, r, None)
        has_args = nargs > 1 or final is not _MISSING
        margs = None
        if has_args:
            def margs():
                return [a(st, dot) for a in method_args] + ([] if final is _MISSING else [final])
        return _field(st, node, last, has_args, r, margs)

    if recv is None and not head and nargs <= 1 and not has_final:
        def field_fast(st, dot, final):
            if type(dot) is dict:
                return dot.get(last, NO_VALUE)
            return _field(st, node, last, False, dot, None)
        return field_fast
    return chain


def _c_variable(var, args, has_final):
    name = var.idents[0]
    if len(var.idents) == 1:
        def variable(st, dot, final):
            value = st.var_value(var, name)
            _not_a_function(st, var, args, final)
            return value
        return variable

    def recv(st, dot):
        return st.var_value(var, name)
    return _c_field_chain(var, var.idents[1:], args, has_final, recv)


def _c_chain(chain, args, has_final):
    if type(chain.node) is _Nil:
        def nil_chain(st, dot, final):
            raise _exec_error(st, chain, "indirection through explicit nil in %s" % _node_str(chain))
        return nil_chain
    recv = _c_arg(chain.node, None)
    return _c_field_chain(chain, chain.fields, args, has_final, recv)


def _c_function(ident, node, args, has_final):
    """exec.go: evalFunction / evalCall with the builtin's parameter types."""
    name = ident.name
    argnodes = args[1:] if args is not None else ()
    compiled = {}

    def arg_fns(spec):
        fns = compiled.get(id(spec))
        if fns is None:
            fixed, variadic = spec[1], spec[2]
            fns = compiled[id(spec)] = tuple(_c_arg(a, fixed[i] if i < len(fixed) else variadic)
                                             for i, a in enumerate(argnodes))
        return fns

    spec0 = _SPECS.get(name)
    if spec0 is not None:
        fixed, variadic = spec0[1], spec0[2]
        nin = len(argnodes) + has_final
        ok = (nin >= len(fixed)) if variadic is not None else (nin == len(fixed))
        if ok:
            fns = arg_fns(spec0)
            fn = spec0[0]
            ftype = _final_type(spec0, nin) if has_final else None

            def call_builtin(st, dot, final):
                vals = [f(st, dot) for f in fns]
                if has_final:
                    vals.append(_validate(st, node, final, ftype))
                try:
                    return fn(*vals)
                except _GoError as e:
                    raise _exec_error(st, node, "error calling %s: %s" % (name, e))
                except (TemplateError, RecursionError):
                    raise
                except Exception as e:  # noqa: BLE001
                    raise _exec_error(st, node, "error calling %s: %s" % (name, e))
            return call_builtin

    def call(st, dot, final):
        spec = _spec(st, ident)
        nin = len(argnodes) + (final is not _MISSING)
        _check_arity(st, ident, spec, len(argnodes), nin)
        vals = [f(st, dot) for f in arg_fns(spec)]
        if final is not _MISSING:
            vals.append(_validate(st, node, final, _final_type(spec, nin)))
        return _invoke(st, spec, name, node, vals)
    return call


def _c_arg(n, typ):
    """fn(st, dot) of exec.go's evalArg for a parameter of type typ."""
    t = type(n)
    if t is _Dot:
        if typ == "V":
            return lambda st, dot: dot
        return lambda st, dot: _validate(st, n, dot, typ)
    if t is _Nil:
        return lambda st, dot: _nil_arg(st, n, typ)
    if t in (_Field, _Variable, _Chain, _Ident, _Pipe):
        if t is _Field:
            inner = _c_field_chain(n, n.idents, None, False, None)
        elif t is _Variable:
            inner = _c_variable(n, (n,), False)
        elif t is _Chain:
            inner = _c_chain(n, None, False)
        elif t is _Ident:
            inner = _c_function(n, n, None, False)
        else:
            sub = _c_pipe(n)
            inner = lambda st, dot, final: sub(st, dot)  # noqa: E731
        if typ == "V" or typ is None:
            return lambda st, dot: inner(st, dot, _MISSING)
        return lambda st, dot: _validate(st, n, inner(st, dot, _MISSING), typ)
    if typ == "S" and t is _String:
        text = n.text
        return lambda st, dot: text
    if typ != "S" and (t is _Bool or t is _String or (t is _Number and n.error is None)):
        v = n.text if t is _String else n.value
        return lambda st, dot: v
    return lambda st, dot: _literal_arg(st, n, typ)


# ---------------------------------------------------------------------------
# Entry points
# ---------------------------------------------------------------------------

_CACHE = {}


def compiled(src):
    """The parsed template of ``src`` (cached); a parse error raises.  A
    packaged template comes from the build's start-up cache
    (``utils/startcache.py``) instead of being parsed in every process."""
    t = _CACHE.get(src)
    if t is None:
        from . import startcache
        data = startcache.template(src)
        t = Template(src) if data is None else Template.from_data(data, src=src)
        if len(_CACHE) < 512:
            _CACHE[src] = t
    return t


def render(src, data, funcs=None):
    """Parse (cached) and execute a Go template against ``data``."""
    if funcs:
        return Template(src, funcs=funcs).execute(data, funcs)
    return compiled(src).execute(data, funcs)
