"""Go templates compiled to closures (``utils/gotemplate.py``): imported on a
template's second execution, so a command that runs each template once
(most of them, in a cold CLI run) never loads it.
"""

from .gofmt import quote as go_quote
from .gotemplate import (MAX_EXEC_DEPTH, NO_VALUE, TemplateError, _Action, _Bool, _Branch, _Chain, _Dot, _Field,
                         _GoError, _Ident, _TooDeep, _MISSING, _Nil, _Number, _Pipe, _SPECS, _State, _String, _Text,
                         _Variable, _check_arity, _exec_error, _field, _final_type, _invoke, _literal_arg,
                         _literal_command, _nil_arg, _node_str, _not_a_function, _print_value, _range_items, _spec,
                         _truth, _validate)


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
        try:
            body(sub, newdot)
        except RecursionError:
            e = _TooDeep()
            e.st, e.node = st, n
            raise e
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


