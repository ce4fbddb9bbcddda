"""Writer of the package's bytecode bundle (``move2kube_amd/_bytecode.bin``).

Every CLI invocation is a cold process, and most of what it costs above a bare
interpreter is importing ~80 modules of this package.  The ordinary path does,
per module, a directory-cache lookup over the candidate suffixes, a ``stat`` of
the source, an ``open``/``read``/``close`` of its ``__pycache__`` file and the
header checks; served from the bundle, a cold ``translate`` on the MI355X hosts
is 1.2-2.5 ms faster (``profiles/tools/cold_ab.py``,
``profiles/r03_cold_bundle/cold_ab.jsonl``).  The bundle
holds the compiled code of every module in one file that the package reads once
(``move2kube_amd/__init__.py`` installs the finder); a module is served from it
only while its source still has the size and mtime (whole seconds, the
``.pyc`` rule) it was compiled from, so an edited or added file falls back to
the normal import path by itself, exactly as a stale ``.pyc`` is recompiled.

Format: ``b"M2KB"``, the header's length (4 bytes, big-endian), the header
``marshal.dumps((tag, optimize, {name: (is_pkg, relpath, mtime_s, size,
offset, length)}))``, then every module's marshalled code at ``offset``
(from the end of the header).  A process reads the small header once and each
module's code when that module is imported (``os.pread``), not the whole file.
``tag`` = the interpreter's pyc magic number + ``b"m2k2"``; an interpreter
with another magic number, or another ``-O`` level, ignores the file.

Built with the native targets (``ops/build.py``, ``__graft_entry__.build``);
``M2K_BYTECODE_BUNDLE=0`` turns the finder off.
"""

import marshal
import os
import struct
import sys
from importlib.util import MAGIC_NUMBER

TAG = MAGIC_NUMBER + b"m2k2"
MAGIC = b"M2KB"
PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILENAME = "_bytecode.bin"


def target():
    return os.path.join(PKG, FILENAME)


def _modules(pkg_dir):
    """(module name, path, is_package) of every module of the package: .py files
    in directories that are packages (an ``__init__.py`` all the way up)."""
    base = os.path.basename(pkg_dir)
    for dp, dns, fns in os.walk(pkg_dir):
        dns[:] = sorted(d for d in dns if os.path.isfile(os.path.join(dp, d, "__init__.py")))
        rel = os.path.relpath(dp, pkg_dir)
        prefix = base if rel == "." else base + "." + rel.replace(os.sep, ".")
        for fn in sorted(fns):
            if not fn.endswith(".py"):
                continue
            path = os.path.join(dp, fn)
            if fn == "__init__.py":
                yield prefix, path, True
            else:
                yield prefix + "." + fn[:-3], path, False


def write(pkg_dir=PKG, out=None):
    """Compile every module and write the bundle atomically; returns its path.
    The package's own ``__init__`` is left out (it is what reads the bundle)."""
    out = out or os.path.join(pkg_dir, FILENAME)
    mods = {}
    blobs = []
    offset = 0
    base = os.path.basename(pkg_dir)
    for name, path, is_pkg in _modules(pkg_dir):
        if name == base:
            continue
        st = os.stat(path)
        with open(path, "rb") as f:
            src = f.read()
        blob = marshal.dumps(compile(src, path, "exec", dont_inherit=True))
        mods[name] = (is_pkg, os.path.relpath(path, pkg_dir), int(st.st_mtime), st.st_size, offset, len(blob))
        blobs.append(blob)
        offset += len(blob)
    header = marshal.dumps((TAG, sys.flags.optimize, mods))
    with open(out + ".tmp", "wb") as f:
        f.write(MAGIC + struct.pack(">I", len(header)) + header)
        for blob in blobs:
            f.write(blob)
    os.replace(out + ".tmp", out)
    return out


def read_header(path):
    """(tag, optimize, {name: record}) of a bundle file, and the offset its
    code section starts at."""
    with open(path, "rb") as f:
        head = f.read(8)
        if len(head) != 8 or head[:4] != MAGIC:
            raise ValueError("not a bytecode bundle")
        n = struct.unpack(">I", head[4:])[0]
        return marshal.loads(f.read(n)), 8 + n


def stale(pkg_dir=PKG, out=None):
    """True when a module is missing from the bundle or its source changed."""
    out = out or os.path.join(pkg_dir, FILENAME)
    try:
        (tag, optimize, mods), _ = read_header(out)
    except (OSError, ValueError, EOFError, TypeError):
        return True
    if tag != TAG or optimize != sys.flags.optimize:
        return True
    base = os.path.basename(pkg_dir)
    names = set()
    for name, path, _ in _modules(pkg_dir):
        if name == base:
            continue
        names.add(name)
        rec = mods.get(name)
        st = os.stat(path)
        if rec is None or (rec[2], rec[3]) != (int(st.st_mtime), st.st_size):
            return True
    return names != set(mods)


if __name__ == "__main__":
    print(write())
