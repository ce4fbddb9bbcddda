"""Writer of the start-up cache (``move2kube_amd/_startcache.bin``); the
reader and the reasons are in ``utils/startcache.py``.

* templates: every file under ``assets/templates`` and every non-script file
  under ``assets/m2kassets`` (the containerizers' Dockerfile and ``.s2i``
  templates) that parses as a Go template, keyed by its text as the runtime
  reads it (``assets.template``: text mode; the containerizers: UTF-8 bytes).
* regular expressions: every pattern the package's sources pass as a string
  literal to ``lazyre.lazy``/``_lazy_re``, ``LazyPattern`` or a ``re``
  function, found by walking their syntax trees (nothing is imported or run).

Format: ``marshal.dumps((interpreter tag, (mtime_s, size, sha1) of
utils/gotemplate.py, {template text: marshal.dumps(parse tree)},
{(pattern, flags): marshal.dumps(_sre.compile arguments)}))``.
"""

import ast
import hashlib
import marshal
import os
import re
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(PKG, "assets")
_RE_FUNCS = {"compile", "match", "fullmatch", "search", "sub", "subn", "split", "findall", "finditer"}
_LAZY_FUNCS = {"lazy", "_lazy_re", "LazyPattern"}


def target():
    from ..utils import startcache
    return startcache.PATH


def _template_files():
    out = []
    tdir = os.path.join(ASSETS, "templates")
    for fn in sorted(os.listdir(tdir)):
        p = os.path.join(tdir, fn)
        if os.path.isfile(p):
            out.append(p)
    for dp, dns, fns in os.walk(os.path.join(ASSETS, "m2kassets")):
        dns.sort()
        for fn in sorted(fns):
            if not fn.endswith(".sh"):
                out.append(os.path.join(dp, fn))
    return out


def _template_texts(path):
    with open(path, "rb") as f:
        raw = f.read()
    texts = {raw.decode("utf-8", errors="surrogateescape")}
    try:
        with open(path) as f:
            texts.add(f.read())
    except (UnicodeDecodeError, OSError):
        pass
    return texts


def _flags_value(node):
    """Value of a flags argument made of int literals and ``re.X`` names."""
    if node is None:
        return 0
    if isinstance(node, ast.Constant) and isinstance(node.value, int):
        return node.value
    if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id == "re":
        v = getattr(re, node.attr, None)
        if isinstance(v, int):
            return int(v)
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.BitOr):
        a, b = _flags_value(node.left), _flags_value(node.right)
        if a is not None and b is not None:
            return a | b
    return None


def _call_name(func):
    if isinstance(func, ast.Name):
        return func.id, None
    if isinstance(func, ast.Attribute):
        base = func.value.id if isinstance(func.value, ast.Name) else None
        return func.attr, base
    return None, None


def _patterns_in(src):
    """(pattern, flags) of the regex literals of one module's source."""
    out = set()
    for node in ast.walk(ast.parse(src)):
        if not isinstance(node, ast.Call) or not node.args:
            continue
        name, base = _call_name(node.func)
        if name in _LAZY_FUNCS:
            flags_node = node.args[1] if len(node.args) > 1 else None
        elif base == "re" and name in _RE_FUNCS:
            pos = 1 if name == "compile" else {"sub": 4, "subn": 4, "split": 3}.get(name, 2)
            flags_node = node.args[pos] if len(node.args) > pos else None
        else:
            continue
        for kw in node.keywords:
            if kw.arg == "flags":
                flags_node = kw.value
        first = node.args[0]
        if not (isinstance(first, ast.Constant) and isinstance(first.value, str)):
            continue
        flags = _flags_value(flags_node)
        if flags is not None:
            out.add((first.value, flags))
    return out


def _package_sources():
    for dp, dns, fns in os.walk(PKG):
        dns[:] = sorted(d for d in dns if d != "__pycache__")
        for fn in sorted(fns):
            if fn.endswith(".py"):
                yield os.path.join(dp, fn)


def sre_args(pattern, flags):
    """What ``sre_compile.compile(pattern, flags)`` passes to
    ``_sre.compile`` - or None unless a pattern compiled from it equals
    ``re.compile(pattern, flags)``."""
    import _sre
    import sre_compile
    import sre_parse
    try:
        p = sre_parse.parse(pattern, flags)
        code = sre_compile._code(p, flags)
    except (re.error, TypeError, ValueError, OverflowError, RecursionError):
        return None
    groupindex = dict(p.state.groupdict)
    indexgroup = [None] * p.state.groups
    for k, i in groupindex.items():
        indexgroup[i] = k
    args = (int(flags | p.state.flags), [int(c) for c in code], p.state.groups - 1, groupindex, tuple(indexgroup))
    try:
        same = _sre.compile(pattern, *args) == re.compile(pattern, flags)
    except (re.error, TypeError, ValueError, RuntimeError):
        return None
    return args if same else None


def _inputs():
    """What the cache is built from: sources and asset files (path, mtime, size)."""
    paths = list(_package_sources()) + _template_files()
    return sorted((os.path.relpath(p, PKG), int(os.stat(p).st_mtime), os.stat(p).st_size) for p in paths)


def collect():
    """(templates {text: marshalled tree}, regexes {(pattern, flags):
    marshalled _sre.compile arguments}): both unmarshalled per entry, when used."""
    from ..utils import gotemplate
    templates = {}
    for path in _template_files():
        for text in _template_texts(path):
            try:
                t = gotemplate.Template(text)
            except gotemplate.TemplateError:
                continue  # not a template (or a broken one): parsed, and raising, at run time
            templates[text] = marshal.dumps(t.to_data())
    patterns = set()
    for path in _package_sources():
        with open(path, encoding="utf-8") as f:
            patterns |= _patterns_in(f.read())
    regexes = {}
    for pattern, flags in sorted(patterns):
        args = sre_args(pattern, flags)
        if args is not None:
            regexes[(pattern, flags)] = marshal.dumps(args)
    return templates, regexes


def _gotemplate_stamp():
    from ..utils import startcache
    mtime, size = startcache.source_stamp(startcache.parser_sources())
    return mtime, size, startcache.source_digest(startcache.parser_sources())


def write(out=None):
    """Build the cache and write it atomically; returns its path."""
    from ..utils import startcache
    out = out or target()
    templates, regexes = collect()
    blob = marshal.dumps((startcache.interpreter_tag(), _gotemplate_stamp(), templates, regexes))
    with open(out + ".tmp", "wb") as f:
        f.write(blob)
    with open(out + ".inputs.tmp", "wb") as f:
        f.write(marshal.dumps(_inputs()))
    os.replace(out + ".tmp", out)
    os.replace(out + ".inputs.tmp", out + ".inputs")
    return out


def stale(out=None):
    """True unless the cache exists for this interpreter and was built from
    the current sources and assets."""
    from ..utils import startcache
    out = out or target()
    try:
        with open(out, "rb") as f:
            tag = marshal.loads(f.read())[0]
        with open(out + ".inputs", "rb") as f:
            inputs = marshal.loads(f.read())
    except (OSError, ValueError, EOFError, TypeError, IndexError):
        return True
    return tag != startcache.interpreter_tag() or inputs != _inputs()


if __name__ == "__main__":
    print(write())
    sys.exit(0)
