"""Module-level regular expressions compiled on first use.

A cold CLI process pays ``sre_compile`` for every ``re.compile`` that runs at
import time - about a fifth of a cold ``translate`` was spent there, mostly on
patterns the run never used (YAML timestamp forms, compose durations, semver).
:class:`LazyPattern` has the ``re.Pattern`` interface and compiles on the first
attribute access; after that the compiled pattern's bound methods are instance
attributes, so the hot path is a plain attribute lookup.  Patterns the
build's start-up cache holds skip ``sre_compile`` altogether (:func:`compile`).
"""

import re

_FORWARDED = ("match", "fullmatch", "search", "sub", "subn", "split", "findall", "finditer",
              "pattern", "flags", "groups", "groupindex")


def compile(pattern, flags=0):
    """``re.compile``, served from the build's start-up cache when it holds
    the pattern (``utils/startcache.py``: no ``sre_compile`` in the process)."""
    from . import startcache
    rx = startcache.regex(pattern, flags)
    return rx if rx is not None else re.compile(pattern, flags)


class LazyPattern:
    def __init__(self, pattern, flags=0):
        self._args = (pattern, flags)

    def compiled(self):
        return compile(*self._args)

    def __getattr__(self, name):
        if name.startswith("__") or name == "_args":
            raise AttributeError(name)
        rx = compile(*self._args)
        for n in _FORWARDED:
            setattr(self, n, getattr(rx, n))
        return getattr(rx, name)

    def __repr__(self):
        return "LazyPattern(%r)" % (self._args[0],)


def lazy(pattern, flags=0):
    return LazyPattern(pattern, flags)


class LazyModule:
    """Stand-in for a module imported on first attribute access (``subprocess``
    costs a cold process ~1 ms and most runs never fork)."""

    def __init__(self, name):
        self._name = name

    def __getattr__(self, attr):
        if attr.startswith("__") or attr == "_name":
            raise AttributeError(attr)
        import sys
        __import__(self._name)  # not importlib.import_module: importlib costs another ~0.3 ms cold
        return getattr(sys.modules[self._name], attr)
