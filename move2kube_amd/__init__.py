"""move2kube_amd - a from-scratch re-implementation of the move2kube migration
tool (collect / plan / translate of docker-compose, Cloud Foundry, Dockerfile,
source-directory and Kubernetes/Knative inputs into Kubernetes/Helm/Knative/
Tekton artifacts) with a native runtime: a C++ extension for directory
indexing, Dockerfile sniffing, hashing, batched edit distance and a parallel
detector-process pool, plus a gfx950 HIP kernel for large all-pairs fuzzy
matching.  See SURVEY.md for the component map.
"""

import _imp
import marshal as _marshal
import os as _os
import sys as _sys
from _frozen_importlib import ModuleSpec as _ModuleSpec


class _BytecodeBundle:
    """Meta-path finder/loader serving this package's modules from
    ``_bytecode.bin`` (written by ``ops/bytecode.py``): the index is read once
    per process and each module's code with one ``pread``, instead of a
    lookup, stat and pyc read per module.  A module whose source
    no longer has the recorded mtime and size is left to the normal finders."""

    def __init__(self, root, mods, fd, base):
        self._root = root
        self._mods = mods
        self._fd = fd      # the bundle file, kept open: code is read per module
        self._base = base  # where the code section starts

    def find_spec(self, name, path=None, target=None):
        rec = self._mods.get(name)
        if rec is None:
            return None
        origin = _os.path.join(self._root, rec[1])
        try:
            st = _os.stat(origin)
        except OSError:
            return None
        if int(st.st_mtime) != rec[2] or st.st_size != rec[3]:
            return None
        spec = _ModuleSpec(name, self, origin=origin, is_package=rec[0])
        spec.has_location = True
        if rec[0]:
            spec.submodule_search_locations = [_os.path.dirname(origin)]
        return spec

    def create_module(self, spec):
        return None

    def exec_module(self, module):
        exec(self.get_code(module.__spec__.name), module.__dict__)

    def get_code(self, name):
        rec = self._mods[name]
        code = _marshal.loads(_os.pread(self._fd, rec[5], self._base + rec[4]))
        _imp._fix_co_filename(code, _os.path.join(self._root, rec[1]))
        return code

    def get_filename(self, name):
        return _os.path.join(self._root, self._mods[name][1])

    def get_source(self, name):
        with open(self.get_filename(name), "rb") as f:
            return f.read().decode()

    def is_package(self, name):
        return self._mods[name][0]


def _install_bytecode_bundle():
    if _os.environ.get("M2K_BYTECODE_BUNDLE", "1") == "0":
        return
    from _frozen_importlib_external import MAGIC_NUMBER
    root = _os.path.dirname(_os.path.abspath(__file__))
    try:
        fd = _os.open(_os.path.join(root, "_bytecode.bin"), _os.O_RDONLY | _os.O_CLOEXEC)
    except OSError:
        return
    try:  # header: b"M2KB", its length, marshalled index (ops/bytecode.py)
        head = _os.pread(fd, 8, 0)
        if head[:4] != b"M2KB" or len(head) != 8:
            raise ValueError
        n = int.from_bytes(head[4:], "big")
        tag, optimize, mods = _marshal.loads(_os.pread(fd, n, 8))
        if tag != MAGIC_NUMBER + b"m2k2" or optimize != _sys.flags.optimize:
            raise ValueError
    except (OSError, ValueError, EOFError, TypeError):
        _os.close(fd)
        return
    # a re-import of the package (tests drop it from sys.modules) replaces its finder
    _sys.meta_path[:] = [f for f in _sys.meta_path if type(f).__name__ != "_BytecodeBundle"]
    _sys.meta_path.insert(0, _BytecodeBundle(root, mods, fd, 8 + n))


_install_bytecode_bundle()


def _cli_process():
    """Start-up trims for a process that is the CLI (``python -m
    move2kube_amd`` and the release launcher call it first; a program that
    imports the package as a library does not).  The cyclic garbage collector
    is off for the whole process (the entry freezes what the imports created):
    neither the ~20 collections an import sequence of this size triggers nor
    the one at interpreter exit walk those objects (2 ms of a cold start on the
    MI355X hosts), and a command's objects live until it ends, so collections
    during it would only re-walk a growing heap (``api.gc_paused``).  ``shutil`` is imported
    without its optional ``bz2``/``lzma`` archive formats, which this tool never
    asks ``shutil`` for (0.7 ms of a cold start on the MI355X hosts; ``tarfile``
    still imports them when it needs them), and ``msvcrt`` is recorded as
    absent so that ``subprocess`` does not search ``sys.path`` for it."""
    import gc
    gc.disable()
    mods = _sys.modules
    if "shutil" not in mods:
        blocked = [m for m in ("bz2", "lzma") if m not in mods]
        for m in blocked:
            mods[m] = None
        try:
            import shutil  # noqa: F401
        finally:
            for m in blocked:
                del mods[m]
    if _sys.platform != "win32":
        mods.setdefault("msvcrt", None)


def _cli_exit(rc):
    """End the CLI process the way ``sys.exit(rc)`` would, without the
    interpreter's teardown of every module and object (3 ms and more of a cold
    ``translate``, ``profiles/tools/exit_ab.py``): wait for non-daemon threads, run
    the ``atexit`` handlers (the QA write-cache flush, the trace file,
    multiprocessing's clean-up), flush the standard streams, then ``_exit``.
    Every file the commands write is closed by then (the runs emit no
    ``ResourceWarning`` under ``-X dev``, ``tests/test_cold_imports.py``)."""
    code = 0 if rc is None else rc if isinstance(rc, int) else 1
    if not isinstance(rc, (int, type(None))):
        print(rc, file=_sys.stderr)
    threading = _sys.modules.get("threading")
    shutdown = getattr(threading, "_shutdown", None)
    if shutdown is not None:
        shutdown()
    import atexit
    atexit._run_exitfuncs()
    for stream in (_sys.stdout, _sys.stderr):
        try:
            stream.flush()
        except (OSError, ValueError, AttributeError) as e:
            # CPython reports a failed flush of stdout at exit (EPIPE, ENOSPC
            # on a redirect) and exits with 120 unless the command failed
            if stream is _sys.stdout and not isinstance(e, AttributeError):
                try:
                    print("Exception ignored in: %r\n%s: %s" % (stream, type(e).__name__, e), file=_sys.stderr)
                except (OSError, ValueError):
                    pass
                if code == 0:
                    code = 120
    _os._exit(code & 0xFF)

from .models.info import VERSION as __version__  # noqa: E402,F401
