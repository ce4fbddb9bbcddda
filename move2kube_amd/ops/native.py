"""Loader for the native runtime extension (``_m2k_native``).

The extension is built in-tree by ``move2kube_amd.ops.build`` (called from
``__graft_entry__.build()``).  Every entry point has an exact pure-Python
fallback so the framework still runs where the extension was not built; set
``M2K_REQUIRE_NATIVE=1`` to make a missing extension an error.
"""

import _thread
import os

_mod = None
_tried = False
_lock = _thread.RLock()


def _load():
    """The extension module, or None.  Loaded once under a lock: a second
    thread asking while the first is still importing waits for it instead of
    being told there is none (collector and probe threads start together)."""
    global _mod, _tried
    if _tried:
        return _mod
    with _lock:
        if not _tried:
            mod = None
            if not os.environ.get("M2K_DISABLE_NATIVE"):
                try:
                    from . import _m2k_native as mod  # noqa: F811
                except ImportError:
                    if os.environ.get("M2K_REQUIRE_NATIVE"):
                        raise
                    mod = None
            _mod = mod
            _tried = True
    return _mod


def available():
    return _load() is not None


def module():
    return _load()


# Paths cross into C++ as bytes (os.fsencode: a file name that is not UTF-8
# arrives in Python with surrogates and goes back out as the same bytes);
# paths coming back are decoded the same way (m2k_native.cpp:walk).
_fsencode = os.fsencode


def walk(root):
    return _load().walk(_fsencode(root))


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
        return m.sniff_dockerfiles([_fsencode(p) for p in paths], nthreads)
    from ..source.dockerfile_parser import sniff_first_from
    return [sniff_first_from(p) for p in paths]


def remove_tree(path):
    """``os.RemoveAll``-like delete of ``path`` (symlinks unlinked, not followed);
    raises OSError on the first failure."""
    m = _load()
    if m is None:
        import shutil
        if os.path.isdir(path) and not os.path.islink(path):
            shutil.rmtree(path)
        else:
            os.remove(path)
        return
    err, where = m.remove_tree(_fsencode(path))
    if err:
        raise OSError(err, os.strerror(err), os.fsdecode(where))


_write_threads = None


def write_files(items, nthreads=None):
    """Write ``[(path, text_or_bytes, mode)]``; returns ``[OSError or None]`` per
    item.  Native: parallel (up to 8 threads, within this rank's CPU share), GIL
    released; a repeated path keeps its last content."""
    global _write_threads
    if nthreads is None:
        if _write_threads is None:
            from ..utils.constants import host_threads
            _write_threads = host_threads(8)
        nthreads = _write_threads
    datas = [d.encode("utf-8", errors="surrogateescape") if isinstance(d, str) else bytes(d) for _, d, _ in items]
    m = _load()
    if m is not None:
        paths = [p for p, _, _ in items]
        errs = m.write_files([_fsencode(p) for p in paths], datas, [int(md) for _, _, md in items], nthreads)
        return [OSError(e, os.strerror(e), p) if e else None for p, e in zip(paths, errs)]
    out = []
    for (p, _, md), data in zip(items, datas):
        try:
            with open(os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_CLOEXEC, md), "wb") as f:
                f.write(data)
            out.append(None)
        except OSError as e:
            out.append(e)
    return out


def run_commands(argvs, cwds, parallel=8, timeout_s=0.0):
    m = _load()
    if m is not None:
        return m.run_commands([[_fsencode(a) for a in argv] for argv in argvs], [_fsencode(c) for c in cwds],
                              parallel, timeout_s)
    return None
