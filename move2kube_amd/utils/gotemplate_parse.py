"""Go 1.15 ``text/template`` lexer and parser (``parse/lex.go``,
``parse/parse.go``, ``parse/node.go`` newNumber, ``strconv.Unquote``) for
``utils/gotemplate.py``.  A separate module: a command whose templates all come
from the build's start-up cache (every packaged one) never imports it.
"""

from .gofmt import quote as go_quote
from .gotemplate import (TemplateError, _Action, _Bool, _Branch, _Chain, _Command, _Dot, _Else, _End, _Field,
                         _Ident, _Nil, _Number, _Pipe, _String, _TemplateCall, _Text, _Variable, _node_str)


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




def parse(src, funcs, name=""):
    """(root nodes, {name: nodes} of the definitions) of ``src``; a parse
    error raises TemplateError with Go's text."""
    p = _Parser(src, _lex(src), funcs, name)
    root = p.parse()
    return root, p.defines
