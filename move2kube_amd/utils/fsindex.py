"""Single-walk file index shared by all planners.

The reference walks the whole source tree once per planner/loader
(``common.GetFilesByExt``/``GetFilesByName`` at ``internal/common/utils.go:47-120``,
called by the compose, CF, knative, kube, cluster-metadata, k8s-files and
QA-cache planners plus every containerizer ``Init``): >=8 full walks.  Here the
tree is walked once (natively, see ``ops/csrc/m2k_native.cpp``) and every
query filters the cached listing.  Walk order and error semantics match Go's
``filepath.Walk``: lexical order, symlinks not followed (a symlink is listed as
a non-directory), unreadable sub-directories are skipped with a warning, an
unreadable/missing root is an error.

Caching is explicit: inside ``with fsindex.scope():`` (the planner and the
translator open one) indexes are reused; outside a scope each query walks
afresh so callers never observe stale listings.
"""

import contextlib
import os
import threading

from . import log

FILE, DIR, SYMLINK, OTHER = 0, 1, 2, 3

_local = threading.local()


def _cache():
    return getattr(_local, "cache", None)


@contextlib.contextmanager
def scope():
    """Reuse file indexes for the duration of the block (nestable)."""
    prev = _cache()
    if prev is None:
        _local.cache = {}
    try:
        yield
    finally:
        if prev is None:
            _local.cache = None
            _local.aux = None


def invalidate():
    c = _cache()
    if c is not None:
        c.clear()
    aux = getattr(_local, "aux", None)
    if aux is not None:
        aux.clear()


def scoped_cache(name):
    """A dict that lives as long as the enclosing :func:`scope` (None outside one)."""
    if _cache() is None:
        return None
    aux = getattr(_local, "aux", None)
    if aux is None:
        aux = _local.aux = {}
    return aux.setdefault(name, {})


class FileIndex:
    """The result of one ``filepath.Walk``-equivalent traversal."""

    __slots__ = ("root", "paths", "kinds", "errors")

    def __init__(self, root, paths, kinds, errors):
        self.root = root
        self.paths = paths
        self.kinds = kinds
        self.errors = errors

    def files(self):
        return [p for p, k in zip(self.paths, self.kinds) if k != DIR]

    def dirs(self):
        return [p for p, k in zip(self.paths, self.kinds) if k == DIR]

    def files_by_ext(self, exts):
        exts = list(exts)
        out = []
        for p, k in zip(self.paths, self.kinds):
            if k == DIR:
                continue
            base = p.rsplit("/", 1)[-1]
            i = base.rfind(".")
            ext = base[i:] if i >= 0 else ""
            for e in exts:
                if ext == e:
                    out.append(p)
        return out

    def files_by_name(self, names):
        names = list(names)
        out = []
        for p, k in zip(self.paths, self.kinds):
            if k == DIR:
                continue
            base = p.rsplit("/", 1)[-1]
            for n in names:
                if base == n:
                    out.append(p)
        return out

    def sub_index(self, sub_root):
        """Listing of a sub-directory derived from this index (no new walk)."""
        prefix = sub_root.rstrip("/") + "/"
        paths, kinds = [], []
        for p, k in zip(self.paths, self.kinds):
            if p == sub_root or p.startswith(prefix):
                paths.append(p)
                kinds.append(k)
        errors = [e for e in self.errors if e[0] == sub_root or e[0].startswith(prefix)]
        return FileIndex(sub_root, paths, kinds, errors)


def _walk_py(root):
    paths, kinds, errors = [], [], []
    try:
        st = os.lstat(root)
    except OSError as e:
        raise FileNotFoundError(str(e))
    import stat as _stat
    if not _stat.S_ISDIR(st.st_mode):
        paths.append(root)
        kinds.append(SYMLINK if _stat.S_ISLNK(st.st_mode) else FILE)
        return paths, kinds, errors

    def rec(d):
        paths.append(d)
        kinds.append(DIR)
        try:
            with os.scandir(d) as it:
                entries = sorted((e.name, e) for e in it)
        except OSError as e:
            errors.append((d, str(e)))
            return
        for name, e in entries:
            p = d + "/" + name if d != "/" else "/" + name
            try:
                if e.is_symlink():
                    paths.append(p)
                    kinds.append(SYMLINK)
                elif e.is_dir(follow_symlinks=False):
                    rec(p)
                else:
                    paths.append(p)
                    kinds.append(FILE)
            except OSError as ex:
                errors.append((p, str(ex)))
    rec(root)
    return paths, kinds, errors


def walk(root):
    """Walk ``root`` and return a :class:`FileIndex` (native walker when built)."""
    from ..ops import native
    root = root.rstrip("/") or "/"
    if native.available():
        paths, kinds, errors = native.walk(root)
    else:
        paths, kinds, errors = _walk_py(root)
    for p, msg in errors:
        if p == root:
            raise PermissionError(msg)
        log.warning("Skipping path %r due to error: %r", p, msg)
    return FileIndex(root, paths, kinds, errors)


def get_index(root):
    if not os.path.exists(root):
        log.warning("Error in walking through files due to : %r", "lstat %s: no such file or directory" % root)
        raise FileNotFoundError(root)
    if not os.path.isdir(root):
        log.warning("The path %r is not a directory.", root)
    root = root.rstrip("/") or "/"
    cache = _cache()
    if cache is None:
        return walk(root)
    idx = cache.get(root)
    if idx is not None:
        return idx
    for r, parent in cache.items():
        if root.startswith(r.rstrip("/") + "/"):
            idx = parent.sub_index(root)
            cache[root] = idx
            return idx
    idx = walk(root)
    cache[root] = idx
    return idx
