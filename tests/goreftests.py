"""The test names of the reference's Go test files (``*_test.go``): each
``func TestX(t *testing.T)`` without subtests is ``TestX``; each subtest is
``TestX/<name>`` with the name as written in ``t.Run("<name>", ...)``, or, for
a table-driven ``t.Run(tc.name, ...)``, each ``name: "<name>"`` of the table
in that function.  ``tests/test_reference_ledger.py`` checks that every one
is mapped to a pytest in ``tests/reference_ledger.json``."""

import os
import re

_FUNC = re.compile(r"^func (Test\w+)\(t \*testing\.T\) \{", re.M)
_RUN_LIT = re.compile(r't\.Run\("((?:[^"\\]|\\.)*)"')
_RUN_VAR = re.compile(r"t\.Run\((\w+)\.(\w+),")
_GO_STR = re.compile(r'"((?:[^"\\]|\\.)*)"')


def _body(src, start):
    """The text of the function whose opening brace ends at ``start``."""
    depth, i = 1, start
    in_str = in_raw = in_line_comment = in_block_comment = False
    while i < len(src) and depth:
        c = src[i]
        if in_line_comment:
            in_line_comment = c != "\n"
        elif in_block_comment:
            if src.startswith("*/", i):
                in_block_comment = False
                i += 1
        elif in_str:
            if c == "\\":
                i += 1
            elif c == '"':
                in_str = False
        elif in_raw:
            in_raw = c != "`"
        elif src.startswith("//", i):
            in_line_comment = True
        elif src.startswith("/*", i):
            in_block_comment = True
        elif c == '"':
            in_str = True
        elif c == "`":
            in_raw = True
        elif c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
        i += 1
    return src[start:i]


def _unquote(s):
    return s.encode("latin-1", "backslashreplace").decode("unicode_escape")


def test_names(path):
    with open(path, encoding="utf-8") as f:
        src = f.read()
    out = []
    for m in _FUNC.finditer(src):
        name = m.group(1)
        body = _body(src, m.end())
        subs = [_unquote(s) for s in _RUN_LIT.findall(body)]
        for var, field in _RUN_VAR.findall(body):
            subs += [_unquote(s) for s in re.findall(r"\b%s:\s*\"((?:[^\"\\]|\\.)*)\"" % re.escape(field), body)]
        if subs:
            seen = {}
            for s in subs:   # testing.T: a repeated subtest name gets #01, #02, ...
                n = seen.get(s, 0)
                seen[s] = n + 1
                out.append("%s/%s%s" % (name, s, "#%02d" % n if n else ""))
        else:
            out.append(name)
    return out


def all_test_names(root):
    """{relative path of the _test.go file: [names]} under ``root``."""
    found = {}
    for dp, dns, fns in os.walk(root):
        dns[:] = sorted(d for d in dns if not d.startswith(".") and d != "vendor")
        for fn in sorted(fns):
            if fn.endswith("_test.go"):
                p = os.path.join(dp, fn)
                found[os.path.relpath(p, root)] = test_names(p)
    return found
