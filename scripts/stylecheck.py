#!/usr/bin/env python3
"""Minimal style gate: every Python source has a module docstring, no tabs in
Python indentation, no trailing whitespace, and no line exceeds 160 columns
(reference CI runs golangci-lint + a license-header check)."""

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_COL = 160


def main():
    bad = []
    for base in ("move2kube_amd", "scripts"):
        for dp, dns, fns in os.walk(os.path.join(ROOT, base)):
            dns[:] = [d for d in dns if d != "__pycache__"]
            for fn in fns:
                if not fn.endswith(".py"):
                    continue
                p = os.path.join(dp, fn)
                src = open(p, encoding="utf-8").read()
                rel = os.path.relpath(p, ROOT)
                if src.strip() and ast.get_docstring(ast.parse(src)) is None and fn != "__main__.py":
                    bad.append("%s: missing module docstring" % rel)
                for i, line in enumerate(src.splitlines(), 1):
                    if line.rstrip() != line:
                        bad.append("%s:%d: trailing whitespace" % (rel, i))
                    if line.startswith("\t"):
                        bad.append("%s:%d: tab indentation" % (rel, i))
                    if len(line) > MAX_COL and "noqa: E501" not in line:
                        bad.append("%s:%d: line longer than %d" % (rel, i, MAX_COL))
    for b in bad:
        print(b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
