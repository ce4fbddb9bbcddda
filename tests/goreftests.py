"""The test names of the reference's Go test files (``*_test.go``): each
``func TestX(t *testing.T)`` without subtests is ``TestX``; each subtest is
``TestX/<name>`` with the name as written in ``t.Run("<name>", ...)``, or, for
a table-driven ``t.Run(tc.name, ...)``, each ``name: "<name>"`` of the table
in that function; a testify ``suite.Run(t, new(S))`` has one subtest per
``Test*`` method of ``S``.  ``tests/test_reference_ledger.py`` checks that every one
is mapped to a pytest in ``tests/reference_ledger.json``."""

import os
import re

_FUNC = re.compile(r"^func (Test\w+)\(t \*testing\.T\) \{", re.M)
_RUN_LIT = re.compile(r't\.Run\("((?:[^"\\]|\\.)*)"')
_RUN_VAR = re.compile(r"t\.Run\((\w+)\.(\w+),")
_SUITE = re.compile(r"suite\.Run\(t, (?:new\((\w+)\)|&(\w+)\{\})")
_TABLE = re.compile(r"\w+\s*:?=\s*\[\]struct\s*\{")
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


def _strip_comments(src):
    """``src`` with every comment blanked (newlines kept): a test inside
    ``/* ... */`` is not compiled, so go test never runs it."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            out.append(" " * (j - i))
            i = j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append(re.sub(r"[^\n]", " ", src[i:j]))
            i = j
        elif c in "\"`":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if (c == '"' and src[j] == "\\") else 1
            out.append(src[i:j + 1])
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _unquote(s):
    return s.encode("latin-1", "backslashreplace").decode("unicode_escape")


def _table_names(body, field):
    """The ``field`` of each row of the ``[]struct{...}{...}`` table literal in
    ``body``: ``field: "x"`` in a keyed row, else (field first in the struct)
    the row's first string literal."""
    m = _TABLE.search(body)
    if not m:
        return []
    decl = _body(body, m.end())                  # struct type body, up to its "}"
    first = re.match(r"\s*(\w+)", decl).group(1)
    lit = body.index("{", m.end() + len(decl))
    rows_src = _body(body, lit + 1)
    names, i = [], 0
    while True:
        j = rows_src.find("{", i)
        if j < 0:
            break
        row = _body(rows_src, j + 1)
        keyed = re.search(r"\b%s:\s*\"((?:[^\"\\]|\\.)*)\"" % re.escape(field), row)
        if keyed:
            names.append(_unquote(keyed.group(1)))
        elif first == field:
            s = _GO_STR.search(row)
            if s:
                names.append(_unquote(s.group(1)))
        i = j + 1 + len(row)
    return names


def test_names(path):
    with open(path, encoding="utf-8") as f:
        src = _strip_comments(f.read())
    out = []
    for m in _FUNC.finditer(src):
        name = m.group(1)
        body = _body(src, m.end())
        runs = []   # (offset, [names]) in source order, as the subtests run
        for r in _RUN_LIT.finditer(body):
            runs.append((r.start(), [_unquote(r.group(1))]))
        for r in _RUN_VAR.finditer(body):
            runs.append((r.start(), _table_names(body, r.group(2))))
        subs = [s for _, names in sorted(runs) for s in names]
        suite = _SUITE.search(body)
        if suite:   # testify: one subtest per Test* method, in reflect's (sorted) method order
            subs += sorted(re.findall(r"^func \(\w+ \*%s\) (Test\w+)\(\)" % (suite.group(1) or suite.group(2)), src, re.M))
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
