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
COMPILE_AFTER = int(os.environ.get("M2K_TEMPLATE_COMPILE_AFTER", "1"))  # interpreted runs before compiling
MAX_EXEC_DEPTH = 100000  # exec.go: maxExecDepth


class TemplateError(Exception):
    pass


class _GoError(Exception):
    """An error a builtin returns (``error calling NAME: ...``)."""


class _TooDeep(Exception):
    """The interpreter's stack ran out inside a ``{{template}}`` call; carries
    that call (``st``, ``node``) so :meth:`Template.execute` reports Go's
    depth error at it.  Built without a Python ``__init__``: it is raised
    where the stack has no room left."""


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
        from .gotemplate_parse import parse
        names = _BUILTIN_NAMES if not funcs else _BUILTIN_NAMES | frozenset(funcs)
        try:
            self.root, self.defines = parse(src, names, name)
        except RecursionError:
            # Go's recursive-descent parser has no depth limit (its stacks grow);
            # this one stops at the interpreter's recursion limit (DEVIATIONS.md 6)
            raise TemplateError("template: %s: nested too deeply to parse (recursion limit)" % name) from None

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
                from .gotemplate_compile import _c_list
                run = self._run = _c_list(self.root)
            run(st, data)
        except _TooDeep as e:
            # exec.go walkTemplate: s.depth == maxExecDepth, reported at the call
            raise _exec_error(e.st, e.node, "exceeded maximum template depth (%d)" % MAX_EXEC_DEPTH) from None
        except RecursionError:
            # nesting (not {{template}} calls) deeper than the interpreter's stack
            raise TemplateError("template: %s: nested too deeply to execute (recursion limit)" % self.name) from None
        return "".join(out)

    def compiled_define(self, name):
        """The compiled body of ``{{define name}}``, or None."""
        cache = self.__dict__.setdefault("_defines_run", {})
        run = cache.get(name)
        if run is None:
            body = self.defines.get(name)
            if body is None:
                return None
            from .gotemplate_compile import _c_list
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
        for n, v in reversed(self.vars):   # exec.go varValue: innermost first
            if n == name:
                return v
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
        try:
            st.walk_list(newdot, body)
        except RecursionError:
            e = _TooDeep()
            e.st, e.node = self, n
            raise e

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


def __getattr__(name):
    """The lexer/parser and compiler names (``_lex``, ``I_*``, ``_c_*``, ...)
    live in modules loaded on use; tests reach them through this module.
    Dunder names are never forwarded: the import system probes ``__path__``
    on every ``from gotemplate import X``, and answering it would load both
    modules in every process."""
    if name.startswith("__"):
        raise AttributeError("module %r has no attribute %r" % (__name__, name))
    for mod in ("gotemplate_parse", "gotemplate_compile"):
        import importlib
        m = importlib.import_module("." + mod, __package__)
        if hasattr(m, name):
            return getattr(m, name)
    raise AttributeError("module %r has no attribute %r" % (__name__, name))
