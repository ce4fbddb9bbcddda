"""Loader for the native runtime extension (``_m2k_native``).

The extension is built in-tree by ``move2kube_amd.ops.build`` (called from
``__graft_entry__.build()``).  Every entry point has an exact pure-Python
fallback so the framework still runs where the extension was not built; set
``M2K_REQUIRE_NATIVE=1`` to make a missing extension an error.
"""

import os

_mod = None
_tried = False


def _load():
    global _mod, _tried
    if _tried:
        return _mod
    _tried = True
    if os.environ.get("M2K_DISABLE_NATIVE"):
        return None
    try:
        from . import _m2k_native as m  # noqa: F401
        _mod = m
    except ImportError:
        if os.environ.get("M2K_REQUIRE_NATIVE"):
            raise
        _mod = None
    return _mod


def available():
    return _load() is not None


def module():
    return _load()


def walk(root):
    return _load().walk(root)


def crc64_ecma(data):
    m = _load()
    if m is not None:
        return m.crc64_ecma(data)
    from ..utils.common import crc64_ecma_py
    return crc64_ecma_py(data)


def fnv64a(data):
    m = _load()
    if m is not None:
        return m.fnv64a(data)
    from ..utils.common import fnv64a_py
    return fnv64a_py(data)


def sniff_dockerfiles(paths, nthreads=8):
    m = _load()
    if m is not None:
        return m.sniff_dockerfiles(paths, nthreads)
    from ..source.dockerfile_parser import sniff_first_from
    return [sniff_first_from(p) for p in paths]


def run_commands(argvs, cwds, parallel=8, timeout_s=0.0):
    m = _load()
    if m is not None:
        return m.run_commands(argvs, cwds, parallel, timeout_s)
    return None
