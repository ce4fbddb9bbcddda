"""Dockerfile recognition (reference ``internal/source/dockerfile2kube.go:117-144``).

The reference feeds *every* file of the source tree to buildkit's Dockerfile
parser and accepts it if the first instruction that is not ``ARG`` is a
``FROM`` whose original line matches ``FROM_RE``.  The scan of the first
instructions (comments, parser directives, line continuations with the
configurable escape character, 64 KiB line limit) is done natively and in
parallel by ``ops/csrc/m2k_native.cpp:sniff_dockerfiles``; this module holds the
exact pure-Python equivalent and the final regex check.
"""

from ..utils.lazyre import lazy as _lazy_re

FROM_RE = _lazy_re(r"(?i)FROM\s+(--platform=[^\s]+)?[^\s]+(\s+AS\s+[^\s]+)?\s*(#.+)?$")
_MAX_LINE = 64 * 1024
_DIRECTIVE_RE = _lazy_re(r"^#\s*([a-zA-Z][a-zA-Z0-9]*)\s*=\s*(.+?)\s*$")


def _trim_continuation(line, esc):
    s = line.rstrip(" \t")
    if s.endswith(esc):
        return s[:-1], True
    return line, False


def sniff_first_from(path):
    """Original line of the first non-ARG instruction if it is FROM, else ''."""
    from ..utils.common import read_bytes
    try:
        data = read_bytes(path)
    except OSError:
        return ""
    text = data.decode("utf-8", errors="surrogateescape")
    if text.startswith("﻿"):
        text = text[1:]
    lines = text.split("\n")
    if text.endswith("\n"):
        lines.pop()
    esc = "\\"
    directives_open = True
    i = 0
    n = len(lines)
    while i < n:
        phys = lines[i].rstrip("\r")
        i += 1
        if len(phys) > _MAX_LINE:
            return ""
        line = phys.lstrip()
        if directives_open:
            if line.startswith("#"):
                m = _DIRECTIVE_RE.match(line)
                if m:
                    if m.group(1).lower() == "escape" and m.group(2) in ("`", "\\"):
                        esc = m.group(2)
                    continue
                directives_open = False
            elif line:
                directives_open = False
        if not line or line.startswith("#"):
            continue
        line, cont = _trim_continuation(line, esc)
        while cont and i < n:
            nxt = lines[i].rstrip("\r")
            i += 1
            if len(nxt) > _MAX_LINE:
                return ""
            t = nxt.lstrip()
            if not t or t.startswith("#"):
                continue
            nxt, cont = _trim_continuation(nxt, esc)
            line += nxt
        cmd = line.split(None, 1)[0].lower() if line.split() else ""
        if cmd == "arg":
            continue
        return line if cmd == "from" else ""
    return ""


def is_dockerfile_line(original):
    return bool(original) and FROM_RE.search(original) is not None


def is_dockerfile(path):
    return is_dockerfile_line(sniff_first_from(path))
