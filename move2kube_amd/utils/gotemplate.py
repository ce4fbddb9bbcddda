"""A Go ``text/template`` interpreter (the subset the reference relies on).

Go templates are part of the reference's user-facing extension ABI: the
Dockerfile/S2I detector directories carry ``Dockerfile`` and
``.s2i/environment`` templates rendered with the JSON a detect script prints
(``internal/containerizer/dockerfilecontainerizer.go:134``,
``s2icontainerizer.go:160``), and every output script/readme is a Go
template (``internal/transformer/templates/*``).  Users who wrote custom
detectors for the reference must be able to reuse them unchanged, so this is
a faithful interpreter, not a Jinja translation.

Supported: text/actions with ``{{-``/``-}}`` trimming, comments, ``if`` /
``else if`` / ``else`` / ``with`` / ``range`` (with ``$k, $v :=``) /
``define`` / ``template`` / ``block`` / ``break`` / ``continue``, variables
and assignment, field chains on maps and objects, pipelines, parenthesised
pipelines, literals, and the builtin functions (and, or, not, len, index,
slice, print, printf, println, eq, ne, lt, le, gt, ge, html, js, urlquery,
call).  Values print with Go ``fmt`` ``%v`` semantics.
"""

import math
import os
import re

from . import fastjson
from .lazyre import lazy as _lazy_re
from .yamlio import go_format_float


INTERPRET = os.environ.get("M2K_TEMPLATE_INTERPRET", "") == "1"  # the tree walker instead of closures
COMPILE_AFTER = 1  # executions of a template interpreted before it is compiled to closures


class TemplateError(Exception):
    pass


class _NoValue:
    """The zero reflect.Value (a missing map key): prints ``<no value>``."""

    def __repr__(self):
        return "<no value>"

    def __bool__(self):
        return False


NO_VALUE = _NoValue()


# ---------------------------------------------------------------------------
# Formatting (fmt %v)
# ---------------------------------------------------------------------------

def go_sprint(v, top=True):
    if v is NO_VALUE:
        return "<no value>"
    if v is None:
        return "<nil>"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if math.isinf(v):
            return "+Inf" if v > 0 else "-Inf"
        if math.isnan(v):
            return "NaN"
        return go_format_float(v)
    if isinstance(v, str):
        return v
    if isinstance(v, bytes):
        return "[" + " ".join(str(b) for b in v) + "]"
    if isinstance(v, dict):
        items = []
        for k in sorted(v.keys(), key=_sort_key):
            items.append("%s:%s" % (go_sprint(k, False), go_sprint(v[k], False)))
        return "map[" + " ".join(items) + "]"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(go_sprint(x, False) for x in v) + "]"
    if hasattr(v, "__dict__"):
        return "{" + " ".join(go_sprint(x, False) for x in vars(v).values()) + "}"
    return str(v)


_GO_TYPE_NAMES = {bool: "bool", int: "int", float: "float64", str: "string", list: "[]interface {}",
                  tuple: "[]interface {}", dict: "map[string]interface {}", bytes: "[]uint8"}


def _go_type_name(v):
    """reflect type name of a decoded value in Go's error texts (JSON numbers
    are float64, objects map[string]interface {})."""
    return _GO_TYPE_NAMES.get(type(v), type(v).__name__)


def _sort_key(k):
    if isinstance(k, (int, float)) and not isinstance(k, bool):
        return (0, k, "")
    return (1, 0, str(k))


def _truth(v):
    if v is NO_VALUE or v is None:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v != 0
    if isinstance(v, (str, bytes, list, tuple, dict)):
        return len(v) > 0
    return True


def go_type_name(v):
    """Go's %T of a value decoded from YAML/JSON or produced by a template."""
    if v is None:
        return "<nil>"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, int):
        return "int"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if isinstance(v, dict):
        return "map[string]interface {}"
    if isinstance(v, (list, tuple)):
        return "[]interface {}"
    return type(v).__name__


def _bad_verb(verb, a):
    """fmt's rendering of an operand the verb does not apply to: %!d(string=x)."""
    return "%!" + verb + "(" + go_type_name(a) + "=" + go_sprint(a) + ")"


def go_sprintf(fmt, args):
    out = []
    i = 0
    ai = 0
    n = len(fmt)
    while i < n:
        c = fmt[i]
        if c != "%":
            out.append(c)
            i += 1
            continue
        i += 1
        if i >= n:
            out.append("%!(NOVERB)")
            break
        flags = ""
        while i < n and fmt[i] in "+-# 0":
            flags += fmt[i]
            i += 1
        width = ""
        while i < n and fmt[i].isdigit():
            width += fmt[i]
            i += 1
        prec = None
        if i < n and fmt[i] == ".":
            i += 1
            prec = ""
            while i < n and fmt[i].isdigit():
                prec += fmt[i]
                i += 1
        if i >= n:
            break
        verb = fmt[i]
        i += 1
        if verb == "%":
            out.append("%")
            continue
        if ai >= len(args):
            out.append("%!" + verb + "(MISSING)")
            continue
        a = args[ai]
        ai += 1
        if a is None and verb not in "vT":
            # fmt prints a nil operand as %!verb(<nil>) for every verb but %v/%T
            s = "%!" + verb + "(<nil>)"
        elif verb == "v":
            s = go_sprint(a)
        elif verb == "s":
            if isinstance(a, (bool, int, float)):
                s = _bad_verb(verb, a)
            else:
                s = go_sprint(a)
                if prec:
                    s = s[:int(prec)]
        elif verb == "q":
            if isinstance(a, bool) or isinstance(a, float):
                s = _bad_verb(verb, a)
            elif isinstance(a, int):
                s = "'%s'" % chr(a)
            else:
                import json
                s = json.dumps(go_sprint(a))
        elif verb == "d":
            s = str(a) if isinstance(a, int) and not isinstance(a, bool) else _bad_verb(verb, a)
        elif verb in "xX":
            if isinstance(a, bool):
                s = _bad_verb(verb, a)
            elif isinstance(a, int):
                s = format(a, verb)
            else:
                s = go_sprint(a).encode().hex()
                if verb == "X":
                    s = s.upper()
        elif verb in "feEgG":
            if not isinstance(a, (int, float)) or isinstance(a, bool):
                s = _bad_verb(verb, a)
            else:
                p = int(prec) if prec else 6
                if verb == "g":
                    s = go_format_float(float(a)) if prec is None else ("%." + str(p) + "g") % a
                else:
                    s = ("%." + str(p) + verb) % a
        elif verb == "t":
            s = go_sprint(a) if isinstance(a, bool) else _bad_verb(verb, a)
        elif verb == "T":
            s = go_type_name(a)
        else:
            s = _bad_verb(verb, a)
        if width:
            w = int(width)
            if "-" in flags:
                s = s.ljust(w)
            elif "0" in flags and verb in "dxXfeEgG":
                s = s.rjust(w, "0")
            else:
                s = s.rjust(w)
        out.append(s)
    if ai < len(args):
        out.append("%!(EXTRA " + ", ".join(go_sprint(a) for a in args[ai:]) + ")")
    return "".join(out)


# ---------------------------------------------------------------------------
# Lexer
# ---------------------------------------------------------------------------

# The token grammar; _scan_token implements it by hand (compiling this costs a
# cold process ~1 ms) and tests/test_gotemplate_lexer.py checks the two agree.
_INT_RE = _lazy_re(r"^[-+]?\d+$")
_TOKEN_RE = _lazy_re(r"""
    (?P<ws>\s+)
  | (?P<comment>/\*.*?\*/)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<raw>`[^`]*`)
  | (?P<char>'(?:[^'\\]|\\.)+')
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<pipe>\|)
  | (?P<lparen>\()
  | (?P<rparen>\))
  | (?P<comma>,)
  | (?P<var>\$[A-Za-z0-9_]*)
  | (?P<field>(?:\.[A-Za-z_][A-Za-z0-9_]*)+)
  | (?P<dot>\.)
  | (?P<num>[-+]?(?:0[xX][0-9a-fA-F_]+|0[bB][01_]+|0[oO][0-7_]+|(?:\d[\d_]*)?\.?\d[\d_]*(?:[eE][-+]?\d+)?)i?)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
""", re.S | re.X)


_IDENT_START = frozenset("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ_")
_IDENT_CHARS = _IDENT_START | frozenset("0123456789")
_HEX_ = frozenset("0123456789abcdefABCDEF_")
_BIN_ = frozenset("01_")
_OCT_ = frozenset("01234567_")
_SINGLE = {":=": "decl"}
_PUNCT = {"=": "assign", "|": "pipe", "(": "lparen", ")": "rparen", ",": "comma"}


def _skip_digits(src, i, n, underscore=True):
    while i < n and (src[i].isdecimal() or (underscore and src[i] == "_")):
        i += 1
    return i


def _scan_quoted(src, pos, n, quote, at_least_one):
    i = pos + 1
    while i < n:
        c = src[i]
        if c == "\\":
            if i + 1 >= n:
                return -1
            i += 2
            continue
        if c == quote:
            return -1 if (at_least_one and i == pos + 1) else i + 1
        i += 1
    return -1


def _scan_num(src, pos, n):
    i = pos
    if i < n and src[i] in "+-":
        i += 1
    if i + 2 < n and src[i] == "0" and src[i + 1] in "xXbBoO":
        digits = _HEX_ if src[i + 1] in "xX" else _BIN_ if src[i + 1] in "bB" else _OCT_
        if src[i + 2] in digits:
            j = i + 3
            while j < n and src[j] in digits:
                j += 1
            return j + 1 if j < n and src[j] == "i" else j
    if i < n and src[i].isdecimal():
        j = _skip_digits(src, i + 1, n)
        if j + 1 < n and src[j] == "." and src[j + 1].isdecimal():
            j = _skip_digits(src, j + 2, n)
    elif i + 1 < n and src[i] == "." and src[i + 1].isdecimal():
        j = _skip_digits(src, i + 2, n)
    else:
        return -1
    if j < n and src[j] in "eE":
        k = j + 1
        if k < n and src[k] in "+-":
            k += 1
        if k < n and src[k].isdecimal():
            j = _skip_digits(src, k + 1, n, underscore=False)
    return j + 1 if j < n and src[j] == "i" else j


def _scan_token(src, pos):
    """(kind, end) of the action token at ``pos``, or None: the first
    alternative of ``_TOKEN_RE`` that matches, without compiling it."""
    n = len(src)
    c = src[pos]
    if c.isspace():
        j = pos + 1
        while j < n and src[j].isspace():
            j += 1
        return "ws", j
    if c == "/":
        if src.startswith("/*", pos):
            e = src.find("*/", pos + 2)
            if e >= 0:
                return "comment", e + 2
        return None
    if c == '"':
        e = _scan_quoted(src, pos, n, '"', False)
        return ("str", e) if e >= 0 else None
    if c == "`":
        e = src.find("`", pos + 1)
        return ("raw", e + 1) if e >= 0 else None
    if c == "'":
        e = _scan_quoted(src, pos, n, "'", True)
        return ("char", e) if e >= 0 else None
    if c == ":":
        return ("decl", pos + 2) if src.startswith(":=", pos) else None
    kind = _PUNCT.get(c)
    if kind is not None:
        return kind, pos + 1
    if c == "$":
        j = pos + 1
        while j < n and src[j] in _IDENT_CHARS:
            j += 1
        return "var", j
    if c == ".":
        j = pos
        while j + 1 < n and src[j] == "." and src[j + 1] in _IDENT_START:
            j += 2
            while j < n and src[j] in _IDENT_CHARS:
                j += 1
        return ("field", j) if j > pos else ("dot", pos + 1)
    if c in "+-" or c.isdecimal():
        e = _scan_num(src, pos, n)
        return ("num", e) if e >= 0 else None
    if c in _IDENT_START:
        j = pos + 1
        while j < n and src[j] in _IDENT_CHARS:
            j += 1
        return "ident", j
    return None


def _lex_action(src, pos, right_delim):
    """Tokenise an action starting at pos; returns (tokens, end_pos_after_delim, trim_right)."""
    toks = []
    n = len(src)
    while True:
        if pos >= n:
            raise TemplateError("unclosed action")
        # closing delimiter (optionally with trim marker)
        if src.startswith(" -" + right_delim, pos) or (src.startswith("-" + right_delim, pos) and pos > 0 and src[pos - 1].isspace()):
            off = 2 if src[pos] == " " else 1
            return toks, pos + off + len(right_delim), True
        if src.startswith(right_delim, pos):
            return toks, pos + len(right_delim), False
        tok = _scan_token(src, pos)
        if tok is None:
            raise TemplateError("unexpected %r in action" % src[pos:pos + 10])
        kind, end = tok
        if kind == "ws":
            pos = end
            continue
        start, pos = pos, end
        text = src[start:end]
        # a field chain directly after a closing paren or variable: (x).Field, $x.Field
        if kind == "field" and toks and toks[-1][0] in ("rparen", "var") and src[start] == ".":
            if toks[-1][0] == "var":
                toks[-1] = ("var", toks[-1][1] + text)
            else:
                toks.append(("chain", text))
            continue
        if kind == "var" and pos < n and src[pos] == ".":
            # $x.Field.Sub
            kind2, end2 = _scan_token(src, pos)
            if kind2 == "field":
                text += src[pos:end2]
                pos = end2
        toks.append((kind, text))


# ---------------------------------------------------------------------------
# AST
# ---------------------------------------------------------------------------

class _Text:
    __slots__ = ("text",)

    def __init__(self, text):
        self.text = text


class _Action:
    __slots__ = ("pipe",)

    def __init__(self, pipe):
        self.pipe = pipe


class _If:
    def __init__(self, kind, pipe, body, else_body):
        self.kind, self.pipe, self.body, self.else_body = kind, pipe, body, else_body


class _TemplateCall:
    def __init__(self, name, pipe):
        self.name, self.pipe = name, pipe


class _Break:
    pass


class _Continue:
    pass


class _BreakSignal(Exception):
    pass


class _ContinueSignal(Exception):
    pass


class _Pipe:
    def __init__(self, decls, cmds, is_assign=False):
        self.decls, self.cmds, self.is_assign = decls, cmds, is_assign


# operands: ("field", [names]), ("var", name, [fields]), ("dot",), ("lit", value),
# ("ident", name), ("pipe", _Pipe, [fields]), ("nil",)

def _parse_string(tok):
    kind, text = tok
    if kind == "raw":
        return text[1:-1]
    if kind == "char":
        return ord(fastjson.loads('"' + text[1:-1].replace('"', '\\"') + '"'))
    try:
        return fastjson.loads(text)
    except ValueError:
        return text[1:-1].encode().decode("unicode_escape")


def _parse_number(text):
    t = text.replace("_", "")
    if t.endswith("i"):
        raise TemplateError("complex numbers unsupported")
    low = t.lower().lstrip("+-")
    sign = -1 if t.startswith("-") else 1
    if low.startswith("0x"):
        return sign * int(low[2:], 16)
    if low.startswith("0b"):
        return sign * int(low[2:], 2)
    if low.startswith("0o"):
        return sign * int(low[2:], 8)
    if _INT_RE.match(t):
        if len(low) > 1 and low.startswith("0"):
            return sign * int(low, 8)
        return int(t)
    return float(t)


class _Parser:
    def __init__(self, toks):
        self.toks = toks
        self.i = 0

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else (None, None)

    def next(self):
        t = self.peek()
        self.i += 1
        return t

    def done(self):
        return self.i >= len(self.toks)

    def pipeline(self, allow_decl=True, stop=None):
        decls = []
        is_assign = False
        if allow_decl:
            # $x := ... | $k, $v := ... | $x = ...
            j = self.i
            vs = []
            while j < len(self.toks) and self.toks[j][0] == "var" and "." not in self.toks[j][1]:
                vs.append(self.toks[j][1])
                j += 1
                if j < len(self.toks) and self.toks[j][0] == "comma":
                    j += 1
                    continue
                break
            if vs and j < len(self.toks) and self.toks[j][0] in ("decl", "assign"):
                is_assign = self.toks[j][0] == "assign"
                decls = vs
                self.i = j + 1
        cmds = []
        while True:
            cmd = self.command(stop)
            if not cmd:
                raise TemplateError("missing command")
            cmds.append(cmd)
            k, _ = self.peek()
            if k == "pipe":
                self.next()
                continue
            break
        return _Pipe(decls, cmds, is_assign)

    def command(self, stop=None):
        args = []
        while not self.done():
            k, t = self.peek()
            if k in ("pipe", "rparen") or k == stop:
                break
            args.append(self.operand())
        return args

    def operand(self):
        k, t = self.next()
        if k == "field":
            return ("field", t[1:].split("."))
        if k == "dot":
            return ("dot",)
        if k == "var":
            parts = t.split(".")
            return ("var", parts[0], parts[1:])
        if k in ("str", "raw", "char"):
            return ("lit", _parse_string((k, t)))
        if k == "num":
            return ("lit", _parse_number(t))
        if k == "ident":
            if t == "true":
                return ("lit", True)
            if t == "false":
                return ("lit", False)
            if t == "nil":
                return ("nil",)
            return ("ident", t)
        if k == "lparen":
            p = self.pipeline(allow_decl=False)
            k2, _ = self.next()
            if k2 != "rparen":
                raise TemplateError("unclosed parenthesis")
            fields = []
            if self.peek()[0] == "chain":
                fields = self.next()[1][1:].split(".")
            return ("pipe", p, fields)
        raise TemplateError("unexpected token %r" % (t,))


def _split_template(src, left="{{", right="}}"):
    """Yield ('text', str) and ('action', tokens, trim_left, trim_right)."""
    items = []
    pos = 0
    n = len(src)
    while pos < n:
        j = src.find(left, pos)
        if j < 0:
            items.append(["text", src[pos:]])
            break
        items.append(["text", src[pos:j]])
        k = j + len(left)
        trim_left = False
        if src.startswith("- ", k) or (src.startswith("-", k) and k + 1 < n and src[k + 1] in "\t\r\n"):
            trim_left = True
            k += 1
        # comment
        rest = src[k:].lstrip(" \t\r\n") if trim_left else src[k:]
        kk = k + (len(src[k:]) - len(rest))
        if rest.startswith("/*"):
            end = src.find("*/", kk)
            if end < 0:
                raise TemplateError("unclosed comment")
            p = end + 2
            trim_right = False
            while p < n and src[p] in " \t\r\n" and not src.startswith(right, p):
                p += 1
            if src.startswith("-" + right, p):
                trim_right = True
                p += 1
            if not src.startswith(right, p):
                raise TemplateError("comment ends before closing delimiter")
            items.append(["comment", None, trim_left, trim_right])
            pos = p + len(right)
            continue
        toks, pos, trim_right = _lex_action(src, k, right)
        items.append(["action", toks, trim_left, trim_right])
    # apply trimming
    for idx, it in enumerate(items):
        if it[0] in ("action", "comment"):
            if it[2] and idx > 0 and items[idx - 1][0] == "text":
                items[idx - 1][1] = items[idx - 1][1].rstrip(" \t\r\n")
            if it[3] and idx + 1 < len(items) and items[idx + 1][0] == "text":
                items[idx + 1][1] = items[idx + 1][1].lstrip(" \t\r\n")
    return items


class Template:
    """A parsed Go text/template."""

    def __init__(self, src, name=""):
        self.name = name
        self.defines = {}
        items = _split_template(src)
        self._items = items
        self._i = 0
        self._range_depth = 0  # {{break}} / {{continue}} only inside a range body (Go's parse.Tree.rangeDepth)
        body, term = self._parse_list(())
        if term is not None:
            raise TemplateError("unexpected {{%s}}" % term)
        self.root = body

    # -- parsing -----------------------------------------------------------
    def _parse_list(self, terminators):
        nodes = []
        while self._i < len(self._items):
            it = self._items[self._i]
            self._i += 1
            if it[0] == "text":
                if it[1]:
                    nodes.append(_Text(it[1]))
                continue
            if it[0] == "comment":
                continue
            toks = it[1]
            if not toks:
                raise TemplateError("missing value for command")
            k, t = toks[0]
            if k == "ident" and t in ("end", "else"):
                if t not in terminators:
                    raise TemplateError("unexpected {{%s}}" % t)
                return nodes, (t, toks[1:])
            if k == "ident" and t in ("if", "with", "range"):
                p = _Parser(toks[1:])
                pipe = p.pipeline(allow_decl=True)
                depth = 1 if t == "range" else 0
                self._range_depth += depth
                body, term = self._parse_list(("end", "else"))
                self._range_depth -= depth
                nodes.append(_If(t, pipe, body, self._parse_else(t, term)))
                continue
            if k == "ident" and t in ("define", "block"):
                name = _parse_string(toks[1])
                pipe = None
                if t == "block":
                    pipe = _Parser(toks[2:]).pipeline(allow_decl=False) if len(toks) > 2 else None
                body, _ = self._parse_list(("end",))
                self.defines[name] = body
                if t == "block":
                    nodes.append(_TemplateCall(name, pipe))
                continue
            if k == "ident" and t == "template":
                name = _parse_string(toks[1])
                pipe = _Parser(toks[2:]).pipeline(allow_decl=False) if len(toks) > 2 else None
                nodes.append(_TemplateCall(name, pipe))
                continue
            if k == "ident" and t in ("break", "continue"):
                if not self._range_depth:
                    raise TemplateError("{{%s}} outside {{range}}" % t)
                nodes.append(_Break() if t == "break" else _Continue())
                continue
            p = _Parser(toks)
            pipe = p.pipeline(allow_decl=True)
            if not p.done():
                raise TemplateError("unexpected %r in operand" % (p.peek()[1],))
            nodes.append(_Action(pipe))
        if terminators:
            raise TemplateError("unexpected EOF")
        return nodes, None

    def _parse_else(self, kind, term):
        """Parse what follows ``{{else ...}}``; ``{{else if x}}`` is sugar for a
        nested if sharing the outer ``{{end}}``."""
        if term[0] == "end":
            return None
        rest = term[1]
        if rest and rest[0][0] == "ident" and rest[0][1] in ("if", "with") and kind != "range":
            sub = rest[0][1]
            pipe = _Parser(rest[1:]).pipeline(allow_decl=True)
            body, term2 = self._parse_list(("end", "else"))
            return [_If(sub, pipe, body, self._parse_else(sub, term2))]
        body, _ = self._parse_list(("end",))
        return body

    # -- the parsed form as plain data (utils/startcache.py) -----------------
    def to_data(self):
        """The parse tree as nested tuples, lists and constants (marshal-able)."""
        return (_nodes_data(self.root), {k: _nodes_data(v) for k, v in self.defines.items()})

    @classmethod
    def from_data(cls, data, name=""):
        """The template :meth:`to_data` described, without parsing."""
        t = cls.__new__(cls)
        t.name = name
        root, defines = data
        t.root = _nodes_from(root)
        t.defines = {k: _nodes_from(v) for k, v in defines.items()}
        return t

    # -- execution ---------------------------------------------------------
    def execute(self, data, funcs=None):
        out = []
        st = _State(self, data, funcs or {})
        run = self.__dict__.get("_run")
        if run is None:
            # compiling costs about three executions: a template a process
            # executes once (most of them, in a cold CLI run) is interpreted
            runs = self.__dict__.get("_runs", 0)
            if INTERPRET or runs < COMPILE_AFTER:
                self._runs = runs + 1
                st.walk(self.root, data, [("$", data)], out)
                return "".join(out)
            run = self._run = _c_nodes(self.root)
        run(st, data, [("$", data)], out)
        return "".join(out)

    def compiled_define(self, name):
        """The compiled body of ``{{define name}}``, or None."""
        cache = self.__dict__.setdefault("_defines_run", {})
        run = cache.get(name)
        if run is None:
            body = self.defines.get(name)
            if body is None:
                return None
            run = cache[name] = _c_nodes(body)
        return run


def _pipe_data(p):
    return None if p is None else (tuple(p.decls), [[_operand_data(a) for a in c] for c in p.cmds], p.is_assign)


def _operand_data(a):
    return ("pipe", _pipe_data(a[1]), a[2]) if a[0] == "pipe" else a


def _nodes_data(nodes):
    out = []
    for n in nodes:
        if isinstance(n, _Text):
            out.append(("t", n.text))
        elif isinstance(n, _Action):
            out.append(("a", _pipe_data(n.pipe)))
        elif isinstance(n, _If):
            out.append(("i", n.kind, _pipe_data(n.pipe), _nodes_data(n.body),
                        None if n.else_body is None else _nodes_data(n.else_body)))
        elif isinstance(n, _TemplateCall):
            out.append(("c", n.name, _pipe_data(n.pipe)))
        elif isinstance(n, _Break):
            out.append(("b",))
        elif isinstance(n, _Continue):
            out.append(("k",))
        else:
            raise TypeError("unknown template node %r" % (n,))
    return out


def _pipe_from(d):
    if d is None:
        return None
    decls, cmds, is_assign = d
    return _Pipe(list(decls), [[_operand_from(a) for a in c] for c in cmds], is_assign)


def _operand_from(a):
    return ("pipe", _pipe_from(a[1]), a[2]) if a[0] == "pipe" else a


def _nodes_from(data):
    out = []
    for d in data:
        k = d[0]
        if k == "t":
            out.append(_Text(d[1]))
        elif k == "a":
            out.append(_Action(_pipe_from(d[1])))
        elif k == "i":
            out.append(_If(d[1], _pipe_from(d[2]), _nodes_from(d[3]), None if d[4] is None else _nodes_from(d[4])))
        elif k == "c":
            out.append(_TemplateCall(d[1], _pipe_from(d[2])))
        elif k == "b":
            out.append(_Break())
        elif k == "k":
            out.append(_Continue())
        else:
            raise ValueError("unknown template node %r" % (k,))
    return out


class _State:
    def __init__(self, tmpl, root, funcs):
        self.tmpl = tmpl
        self.root = root
        self.funcs = dict(_BUILTINS)
        self.funcs.update(funcs)

    def walk(self, nodes, dot, scope, out):
        mark = len(scope)
        try:
            for node in nodes:
                if isinstance(node, _Text):
                    out.append(node.text)
                elif isinstance(node, _Action):
                    val = self.eval_pipe(node.pipe, dot, scope)
                    if not node.pipe.decls:
                        out.append(go_sprint(val))
                elif isinstance(node, _If):
                    self.walk_control(node, dot, scope, out)
                elif isinstance(node, _TemplateCall):
                    body = self.tmpl.defines.get(node.name)
                    if body is None:
                        raise TemplateError(go_sprintf("template %q not defined", [node.name]))
                    newdot = self.eval_pipe(node.pipe, dot, scope) if node.pipe else None
                    self.walk(body, newdot, [("$", newdot)], out)
                elif isinstance(node, _Break):
                    raise _BreakSignal()
                elif isinstance(node, _Continue):
                    raise _ContinueSignal()
        finally:
            del scope[mark:]

    def walk_control(self, node, dot, scope, out):
        mark = len(scope)
        try:
            if node.kind == "range":
                val = self.eval_pipe(node.pipe, dot, scope, declare=False)
                items = []
                if isinstance(val, dict):
                    items = [(k, val[k]) for k in sorted(val.keys(), key=_sort_key)]
                elif isinstance(val, (list, tuple, str, bytes)):
                    if isinstance(val, str):
                        raise TemplateError("range can't iterate over %s" % val)
                    items = list(enumerate(val))
                elif isinstance(val, int) and not isinstance(val, bool):
                    items = [(i, i) for i in range(val)]
                elif val is None or val is NO_VALUE:
                    items = []
                else:
                    raise TemplateError("range can't iterate over %s" % go_sprint(val))
                if not items:
                    if node.else_body is not None:
                        self.walk(node.else_body, dot, scope, out)
                    return
                decls = node.pipe.decls
                for k, v in items:
                    inner = len(scope)
                    if len(decls) == 1:
                        scope.append((decls[0], v))
                    elif len(decls) == 2:
                        scope.append((decls[0], k))
                        scope.append((decls[1], v))
                    try:
                        self.walk(node.body, v, scope, out)
                    except _BreakSignal:
                        break
                    except _ContinueSignal:
                        pass
                    finally:
                        del scope[inner:]
                return
            val = self.eval_pipe(node.pipe, dot, scope)
            if _truth(val):
                self.walk(node.body, val if node.kind == "with" else dot, scope, out)
            elif node.else_body is not None:
                self.walk(node.else_body, dot, scope, out)
        finally:
            del scope[mark:]

    # -- pipelines -----------------------------------------------------------
    def eval_pipe(self, pipe, dot, scope, declare=True):
        val = None
        final = None
        for i, cmd in enumerate(pipe.cmds):
            val = self.eval_cmd(cmd, dot, scope, final if i > 0 else None, has_final=i > 0)
            final = val
        if pipe.decls and declare:
            if pipe.is_assign:
                for name in pipe.decls:
                    for idx in range(len(scope) - 1, -1, -1):
                        if scope[idx][0] == name:
                            scope[idx] = (name, val)
                            break
                    else:
                        raise TemplateError("undefined variable: %s" % name)
            else:
                scope.append((pipe.decls[0], val))
        return val

    def eval_cmd(self, cmd, dot, scope, final, has_final):
        first = cmd[0]
        if first[0] == "ident":
            name = first[1]
            fn = self.funcs.get(name)
            if fn is None:
                raise TemplateError('function "%s" not defined' % name)
            if name in ("and", "or"):
                args = cmd[1:]
                vals = [self.eval_arg(a, dot, scope) for a in args]
                if has_final:
                    vals.append(final)
                return fn(*vals)
            args = [self.eval_arg(a, dot, scope) for a in cmd[1:]]
            if has_final:
                args.append(final)
            try:
                return fn(*args)
            except TemplateError:
                raise
            except Exception as e:  # noqa: BLE001
                raise TemplateError("error calling %s: %s" % (name, e))
        if len(cmd) > 1 or has_final:
            # method-style calls with args are not supported on data values
            if first[0] in ("field",) and (len(cmd) > 1 or has_final):
                raise TemplateError("can't give argument to non-function %s" % ".".join(first[1]))
        return self.eval_arg(first, dot, scope)

    def eval_arg(self, a, dot, scope):
        kind = a[0]
        if kind == "lit":
            return a[1]
        if kind == "nil":
            return None
        if kind == "dot":
            return dot
        if kind == "field":
            return self.fields(dot, a[1])
        if kind == "var":
            name = a[1]
            for idx in range(len(scope) - 1, -1, -1):
                if scope[idx][0] == name:
                    return self.fields(scope[idx][1], a[2])
            raise TemplateError("undefined variable: %s" % name)
        if kind == "pipe":
            v = self.eval_pipe(a[1], dot, scope, declare=False)
            return self.fields(v, a[2])
        if kind == "ident":
            fn = self.funcs.get(a[1])
            if fn is None:
                raise TemplateError('function "%s" not defined' % a[1])
            return fn()
        raise TemplateError("bad operand")

    @staticmethod
    def fields(val, names):
        for name in names:
            if val is NO_VALUE or val is None:
                if val is None:
                    raise TemplateError("nil pointer evaluating .%s" % name)
                return NO_VALUE
            if isinstance(val, dict):
                val = val.get(name, NO_VALUE)
            elif hasattr(val, name):
                val = getattr(val, name)
                if callable(val):
                    val = val()
            else:
                raise TemplateError("can't evaluate field %s in type %s" % (name, _go_type_name(val)))
        return val


# ---------------------------------------------------------------------------
# Compilation to closures
# ---------------------------------------------------------------------------
# Each node becomes a Python closure once per parsed template, so executing it
# does no per-node dispatch on node and operand kinds.  The closures follow
# _State.walk / walk_control / eval_pipe / eval_cmd / eval_arg step for step
# (same evaluation order, same errors).  A template is compiled on its second
# execution (COMPILE_AFTER); M2K_TEMPLATE_INTERPRET=1 keeps the interpreter,
# and tests/test_gotemplate_compiled.py checks the two agree on every packaged
# template and the template test corpus.

def _c_nodes(nodes):
    fns = tuple(_c_node(n) for n in nodes)
    declares = any(isinstance(n, _Action) and n.pipe.decls for n in nodes)

    if not declares:  # nothing at this level adds to the scope
        def run(st, dot, scope, out):
            for f in fns:
                f(st, dot, scope, out)
        return run

    def run_scoped(st, dot, scope, out):
        mark = len(scope)
        try:
            for f in fns:
                f(st, dot, scope, out)
        finally:
            del scope[mark:]
    return run_scoped


def _c_node(n):
    if isinstance(n, _Text):
        text = n.text

        def text_node(st, dot, scope, out):
            out.append(text)
        return text_node
    if isinstance(n, _Action):
        pipe = _c_pipe(n.pipe, True)
        if n.pipe.decls:
            def declare_node(st, dot, scope, out):
                pipe(st, dot, scope)
            return declare_node

        def action_node(st, dot, scope, out):
            out.append(go_sprint(pipe(st, dot, scope)))
        return action_node
    if isinstance(n, _If):
        return _c_control(n)
    if isinstance(n, _TemplateCall):
        name = n.name
        pipe = _c_pipe(n.pipe, True) if n.pipe else None

        def call_node(st, dot, scope, out):
            body = st.tmpl.compiled_define(name)
            if body is None:
                raise TemplateError(go_sprintf("template %q not defined", [name]))
            newdot = pipe(st, dot, scope) if pipe is not None else None
            body(st, newdot, [("$", newdot)], out)
        return call_node
    if isinstance(n, _Break):
        def break_node(st, dot, scope, out):
            raise _BreakSignal()
        return break_node
    if isinstance(n, _Continue):
        def continue_node(st, dot, scope, out):
            raise _ContinueSignal()
        return continue_node
    raise TypeError("unknown template node %r" % (n,))


def _c_control(node):
    body = _c_nodes(node.body)
    else_body = None if node.else_body is None else _c_nodes(node.else_body)
    if node.kind == "range":
        pipe = _c_pipe(node.pipe, False)
        decls = tuple(node.pipe.decls)

        def range_node(st, dot, scope, out):
            mark = len(scope)
            try:
                val = pipe(st, dot, scope)
                items = []
                if isinstance(val, dict):
                    items = [(k, val[k]) for k in sorted(val.keys(), key=_sort_key)]
                elif isinstance(val, (list, tuple, str, bytes)):
                    if isinstance(val, str):
                        raise TemplateError("range can't iterate over %s" % val)
                    items = list(enumerate(val))
                elif isinstance(val, int) and not isinstance(val, bool):
                    items = [(i, i) for i in range(val)]
                elif val is None or val is NO_VALUE:
                    items = []
                else:
                    raise TemplateError("range can't iterate over %s" % go_sprint(val))
                if not items:
                    if else_body is not None:
                        else_body(st, dot, scope, out)
                    return
                for k, v in items:
                    inner = len(scope)
                    if len(decls) == 1:
                        scope.append((decls[0], v))
                    elif len(decls) == 2:
                        scope.append((decls[0], k))
                        scope.append((decls[1], v))
                    try:
                        body(st, v, scope, out)
                    except _BreakSignal:
                        break
                    except _ContinueSignal:
                        pass
                    finally:
                        del scope[inner:]
            finally:
                del scope[mark:]
        return range_node
    pipe = _c_pipe(node.pipe, True)
    is_with = node.kind == "with"

    def cond_node(st, dot, scope, out):
        mark = len(scope)
        try:
            val = pipe(st, dot, scope)
            if _truth(val):
                body(st, val if is_with else dot, scope, out)
            elif else_body is not None:
                else_body(st, dot, scope, out)
        finally:
            del scope[mark:]
    return cond_node


def _c_pipe(pipe, declare):
    """fn(st, dot, scope) -> value of the pipeline (declaring or assigning its
    variables when ``declare``, as eval_pipe does)."""
    cmds = [_c_cmd(c, i > 0) for i, c in enumerate(pipe.cmds)]
    decls = tuple(pipe.decls) if declare else ()
    if not decls and len(cmds) == 1:
        only = cmds[0]

        def single(st, dot, scope):
            return only(st, dot, scope, None)
        return single
    is_assign = pipe.is_assign

    def run(st, dot, scope):
        val = None
        for c in cmds:
            val = c(st, dot, scope, val)
        if decls:
            if is_assign:
                for name in decls:
                    for idx in range(len(scope) - 1, -1, -1):
                        if scope[idx][0] == name:
                            scope[idx] = (name, val)
                            break
                    else:
                        raise TemplateError("undefined variable: %s" % name)
            else:
                scope.append((decls[0], val))
        return val
    return run


def _c_cmd(cmd, has_final):
    """fn(st, dot, scope, final) of one command of a pipeline."""
    first = cmd[0]
    if first[0] == "ident":
        name = first[1]
        args = tuple(_c_arg(a) for a in cmd[1:])
        wrap = name not in ("and", "or")

        def call(st, dot, scope, final):
            fn = st.funcs.get(name)
            if fn is None:
                raise TemplateError('function "%s" not defined' % name)
            vals = [a(st, dot, scope) for a in args]
            if has_final:
                vals.append(final)
            if not wrap:
                return fn(*vals)
            try:
                return fn(*vals)
            except TemplateError:
                raise
            except Exception as e:  # noqa: BLE001
                raise TemplateError("error calling %s: %s" % (name, e))
        return call
    arg = _c_arg(first)
    if first[0] == "field" and (len(cmd) > 1 or has_final):
        message = "can't give argument to non-function %s" % ".".join(first[1])

        def refuse(st, dot, scope, final):
            raise TemplateError(message)
        return refuse

    def value(st, dot, scope, final):
        return arg(st, dot, scope)
    return value


def _c_arg(a):
    kind = a[0]
    fields = _State.fields
    if kind == "lit":
        v = a[1]
        return lambda st, dot, scope: v
    if kind == "nil":
        return lambda st, dot, scope: None
    if kind == "dot":
        return lambda st, dot, scope: dot
    if kind == "field":
        names = a[1]
        return lambda st, dot, scope: fields(dot, names)
    if kind == "var":
        name, names = a[1], a[2]

        def var(st, dot, scope):
            for idx in range(len(scope) - 1, -1, -1):
                if scope[idx][0] == name:
                    return fields(scope[idx][1], names)
            raise TemplateError("undefined variable: %s" % name)
        return var
    if kind == "pipe":
        sub = _c_pipe(a[1], False)
        names = a[2]
        return lambda st, dot, scope: fields(sub(st, dot, scope), names)
    if kind == "ident":
        name = a[1]

        def ident(st, dot, scope):
            fn = st.funcs.get(name)
            if fn is None:
                raise TemplateError('function "%s" not defined' % name)
            return fn()
        return ident

    def bad(st, dot, scope):
        raise TemplateError("bad operand")
    return bad


# ---------------------------------------------------------------------------
# Builtins
# ---------------------------------------------------------------------------

def _and(*args):
    v = True
    for v in args:
        if not _truth(v):
            return v
    return v


def _or(*args):
    v = False
    for v in args:
        if _truth(v):
            return v
    return v


def _basic(v):
    if v is NO_VALUE:
        return None
    return v


def _eq(a, *bs):
    if not bs:
        raise TemplateError("missing argument for comparison")
    a = _basic(a)
    for b in bs:
        b = _basic(b)
        if isinstance(a, bool) != isinstance(b, bool) and a is not None and b is not None:
            raise TemplateError("incompatible types for comparison")
        if a == b:
            return True
    return False


def _ne(a, b):
    return not _eq(a, b)


def _cmp(op):
    def f(a, b):
        a, b = _basic(a), _basic(b)
        try:
            return op(a, b)
        except TypeError:
            raise TemplateError("incompatible types for comparison")
    return f


def _index(item, *idx):
    v = item
    for i in idx:
        if v is NO_VALUE or v is None:
            raise TemplateError("index of untyped nil")
        if isinstance(v, dict):
            v = v.get(i, NO_VALUE)
        elif isinstance(v, (list, tuple, str, bytes)):
            if not isinstance(i, int) or i < 0 or i >= len(v):
                raise TemplateError("index out of range: %s" % (i,))
            v = v[i]
            if isinstance(v, str) and len(v) == 1 and isinstance(item, str):
                v = ord(v)
        else:
            raise TemplateError("can't index item of type %s" % type(v).__name__)
    return v


def _slice(item, *idx):
    if len(idx) == 0:
        return item
    if len(idx) == 1:
        return item[idx[0]:]
    return item[idx[0]:idx[1]]


def _len(v):
    if v is NO_VALUE or v is None:
        raise TemplateError("len of nil pointer")
    try:
        return len(v)
    except TypeError:
        raise TemplateError("len of type %s" % type(v).__name__)


def _print(*args):
    # fmt.Sprint: spaces between operands when neither is a string
    out = []
    prev_str = True
    for i, a in enumerate(args):
        is_str = isinstance(a, str)
        if i > 0 and not is_str and not prev_str:
            out.append(" ")
        out.append(go_sprint(a))
        prev_str = is_str
    return "".join(out)


def _println(*args):
    return " ".join(go_sprint(a) for a in args) + "\n"


def _printf(fmt, *args):
    return go_sprintf(fmt, list(args))


def _html_escape(*args):
    import html as _html
    return _html.escape(_print(*args), quote=True).replace("&#x27;", "&#39;")


def _js_escape(*args):
    s = _print(*args)
    out = []
    for ch in s:
        if ch in "\\'\"<>&=":
            out.append("\\u%04X" % ord(ch) if ch in "<>&=" else "\\" + ch)
        elif ord(ch) < 0x20:
            out.append("\\u%04X" % ord(ch))
        else:
            out.append(ch)
    return "".join(out)


def _urlquery(*args):
    import urllib.parse
    return urllib.parse.quote_plus(_print(*args))


def _call(fn, *args):
    return fn(*args)


_BUILTINS = {
    "and": _and, "or": _or, "not": lambda v: not _truth(v), "len": _len, "index": _index,
    "slice": _slice, "print": _print, "println": _println, "printf": _printf,
    "eq": _eq, "ne": _ne,
    "lt": _cmp(lambda a, b: a < b), "le": _cmp(lambda a, b: a <= b),
    "gt": _cmp(lambda a, b: a > b), "ge": _cmp(lambda a, b: a >= b),
    "html": _html_escape, "js": _js_escape, "urlquery": _urlquery, "call": _call,
}


_CACHE = {}


def compiled(src):
    """The parsed template of ``src`` (cached); a parse error raises.  A
    packaged template comes from the build's start-up cache
    (``utils/startcache.py``) instead of being parsed in every process."""
    t = _CACHE.get(src)
    if t is None:
        from . import startcache
        data = startcache.template(src)
        t = Template(src) if data is None else Template.from_data(data)
        if len(_CACHE) < 512:
            _CACHE[src] = t
    return t


def render(src, data, funcs=None):
    """Parse (cached) and execute a Go template against ``data``."""
    return compiled(src).execute(data, funcs)
