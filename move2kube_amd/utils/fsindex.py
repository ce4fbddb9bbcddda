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

import os
import re
import threading

from . import log

FILE, DIR, SYMLINK, OTHER = 0, 1, 2, 3
MISSING = -1
# "*.<ext>" with ext in [A-Za-z0-9_+-]: characters deleted by this table
_DROP_SUFFIX_CHARS = str.maketrans("", "", "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_+-")


def _is_suffix_pattern(pattern):
    return len(pattern) > 2 and pattern.startswith("*.") and not pattern[2:].translate(_DROP_SUFFIX_CHARS)

_local = threading.local()


def _cache():
    return getattr(_local, "cache", None)


class scope:
    """Reuse file indexes for the duration of the block (nestable).

    ``keep_for=root``: when this (outermost) scope ends, its listings and
    scoped caches are kept for one later ``scope(adopt=root)`` on this thread
    - the plan and the translate of one ``translate`` command, which walk the
    same unchanged tree (see :func:`handoff_allowed`).  Anything kept and not
    adopted is dropped by the next keeping scope or :func:`drop_kept`."""

    __slots__ = ("keep_for", "adopt", "prev")

    def __init__(self, keep_for=None, adopt=None):
        self.keep_for = keep_for
        self.adopt = adopt

    def __enter__(self):
        self.prev = prev = _cache()
        if prev is None:
            kept = getattr(_local, "kept", None)
            _local.kept = None
            if self.adopt is not None and kept is not None and kept[0] == self.adopt:
                _local.cache, _local.aux = kept[1], kept[2]
            else:
                _local.cache = {}

    def __exit__(self, *exc):
        if self.prev is None:
            if self.keep_for is not None:
                _local.kept = (self.keep_for, _local.cache, getattr(_local, "aux", None))
            _local.cache = None
            _local.aux = None
        return False


def drop_kept():
    _local.kept = None


def handoff_allowed(src_root, out_path):
    """The plan's listings may serve the translate of the same command only
    when nothing the command writes in between lands inside the source tree:
    the output directory (created with its QA cache before translating) must
    lie outside it."""
    src = os.path.realpath(src_root)
    out = _realpath_of_nearest(out_path)
    return not (out == src or out.startswith(src.rstrip(os.sep) + os.sep))


def _realpath_of_nearest(path):
    """``realpath`` of ``path``, resolved through its nearest existing ancestor
    when it does not exist yet (an output directory reached through a symlink
    into the source tree must compare as inside it)."""
    p = os.path.abspath(path)
    tail = []
    while not os.path.lexists(p):
        parent, name = os.path.split(p)
        if parent == p:
            break
        tail.append(name)
        p = parent
    return os.path.join(os.path.realpath(p), *reversed(tail))


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
    """The result of one ``filepath.Walk``-equivalent traversal.

    Walk order is depth-first pre-order with sorted names, so every
    directory's subtree is one contiguous range of ``paths``.  Sub-indexes are
    sliced out of that range (no rescans) and remember their offset in the
    base index, which lets recursive "any entry named like X below here?"
    queries use one precomputed position list per pattern (``has_match``).
    """

    __slots__ = ("root", "paths", "kinds", "errors", "base", "lo", "_pos", "_end", "_match", "_by_ext", "_by_name")

    def __init__(self, root, paths, kinds, errors, base=None, lo=0):
        self.root = root
        self.paths = paths
        self.kinds = kinds
        self.errors = errors
        self.base = base
        self.lo = lo
        self._pos = None
        self._end = None
        self._match = None
        self._by_ext = None
        self._by_name = None

    def _file_maps(self):
        """ext -> [positions], basename -> [positions] of non-directories (one pass)."""
        if self._by_ext is None:
            by_ext, by_name = {}, {}
            for i, (p, k) in enumerate(zip(self.paths, self.kinds)):
                if k == DIR:
                    continue
                base = p.rsplit("/", 1)[-1]
                j = base.rfind(".")
                by_ext.setdefault(base[j:] if j >= 0 else "", []).append(i)
                by_name.setdefault(base, []).append(i)
            self._by_ext, self._by_name = by_ext, by_name
        return self._by_ext, self._by_name

    def _select(self, which, keys):
        """Entries listed under ``keys`` in the base index's ext/name map,
        restricted to this index's range (sub-indexes share the base maps)."""
        import bisect
        base = self.base or self
        table = base._file_maps()[which]
        lo, hi = self.lo, self.lo + len(self.paths)
        whole = base is self
        pos = []
        for key in keys:
            ps = table.get(key)
            if not ps:
                continue
            if whole:
                pos.extend(ps)
            else:
                pos.extend(ps[bisect.bisect_left(ps, lo):bisect.bisect_left(ps, hi)])
        if len(keys) > 1:
            pos.sort()
        bp = base.paths
        return [bp[i] for i in pos]

    def files(self):
        return [p for p, k in zip(self.paths, self.kinds) if k != DIR]

    def dirs(self):
        return [p for p, k in zip(self.paths, self.kinds) if k == DIR]

    def files_by_ext(self, exts):
        """Non-directories whose extension (Go ``filepath.Ext``) is in ``exts``, in walk order."""
        return self._select(0, list(dict.fromkeys(exts)))

    def files_by_name(self, names):
        """Non-directories whose base name is in ``names``, in walk order."""
        return self._select(1, list(dict.fromkeys(names)))

    # -- subtree ranges -------------------------------------------------------
    def _positions(self):
        if self._pos is None:
            self._pos = {p: i for i, p in enumerate(self.paths)}
        return self._pos

    def _ends(self):
        """end[i] = one past the last descendant of entry i."""
        if self._end is None:
            n = len(self.paths)
            end = list(range(1, n + 1))
            stack = []  # (prefix, index) of open directories
            for i, (p, k) in enumerate(zip(self.paths, self.kinds)):
                while stack and not p.startswith(stack[-1][0]):
                    end[stack.pop()[1]] = i
                if k == DIR:
                    stack.append((p.rstrip("/") + "/", i))
            for _, j in stack:
                end[j] = n
            self._end = end
        return self._end

    def sub_index(self, sub_root):
        """Listing of a sub-directory derived from this index (no new walk).
        Positions and subtree ends come from the base index (computed once),
        so deriving many nested sub-indexes costs one slice each."""
        base = self.base or self
        i = base._positions().get(sub_root)
        if i is None or not self.lo <= i < self.lo + len(self.paths):
            return FileIndex(sub_root, [], [], [], base, self.lo)
        j = base._ends()[i]
        prefix = sub_root.rstrip("/") + "/"
        errors = [e for e in self.errors if e[0] == sub_root or e[0].startswith(prefix)]
        return FileIndex(sub_root, base.paths[i:j], base.kinds[i:j], errors, base, i)

    def child_kind(self, name):
        """Kind of the entry ``<root>/<name>`` as of the walk (``MISSING`` when
        the root listing had no such name), or None when the index cannot
        answer: the root is not a directory (a symlinked root is not followed
        by the walk, but ``test -f root/name`` follows it) or the entry could
        not be stat'ed.  Lets detectors answer ``test -f`` without a syscall."""
        if not self.kinds or self.kinds[0] != DIR:
            return None
        base = self.base or self
        p = self.root + "/" + name if self.root != "/" else "/" + name
        i = base._positions().get(p)
        if i is not None:
            return base.kinds[i]
        if self.errors and any(e[0] == p for e in self.errors):
            return None
        return MISSING

    def children_matching(self, pattern):
        """Sorted names of the root's direct children (any kind) whose name
        matches the shell ``pattern`` and does not start with a dot - what
        ``for f in <pattern>`` expands to in that directory."""
        base = self.base or self
        prefix = self.root.rstrip("/") + "/"
        pos = base._pattern_positions(pattern)
        import bisect
        lo, hi = self.lo + 1, self.lo + len(self.paths)
        out = []
        for k in range(bisect.bisect_left(pos, lo), bisect.bisect_left(pos, hi)):
            rest = base.paths[pos[k]][len(prefix):]
            if "/" not in rest and not rest.startswith("."):
                out.append(rest)
        return sorted(out)

    def _pattern_positions(self, pattern):
        """Positions (in this base index) of entries whose basename matches ``pattern``."""
        if self._match is None:
            self._match = {}
        pos = self._match.get(pattern)
        if pos is None:
            if _is_suffix_pattern(pattern):
                # "*.go"-style: the basename ends with the suffix iff the path does
                suffix = pattern[1:]
                pos = [i for i, p in enumerate(self.paths) if p.endswith(suffix)]
            else:
                import fnmatch
                rx = re.compile(fnmatch.translate(pattern))
                pos = [i for i, p in enumerate(self.paths) if rx.match(p.rsplit("/", 1)[-1])]
            self._match[pattern] = pos
        return pos

    def has_match(self, pattern, include_root=False):
        """True if some entry of this index (other than its root unless asked)
        has a basename matching the shell ``pattern`` (``find -name``)."""
        import bisect
        base = self.base or self
        pos = base._pattern_positions(pattern)
        lo = self.lo if include_root else self.lo + 1
        hi = self.lo + len(self.paths)
        k = bisect.bisect_left(pos, lo)
        return k < len(pos) and pos[k] < hi


def _go_errno_text(code):
    from .common import go_errno_text
    return go_errno_text(code)


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
                entries = sorted(((e.name, e) for e in it), key=lambda ne: os.fsencode(ne[0]))   # Go: byte order
        except OSError as e:
            errors.append((d, "open %s: %s" % (d, _go_errno_text(e.errno))))
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
                    kinds.append(FILE if e.is_file(follow_symlinks=False) else OTHER)
            except OSError as ex:
                errors.append((p, "lstat %s: %s" % (p, _go_errno_text(ex.errno))))
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


def peek_index(root):
    """The index of ``root`` if the enclosing scope already has it or one of
    its ancestors (derived without a walk); None otherwise.  Never walks."""
    cache = _cache()
    if cache is None:
        return None
    idx = cache.get(root)
    if idx is not None:
        return idx
    root = root.rstrip("/") or "/"
    idx = cache.get(root)
    if idx is not None:
        return idx
    anc = root
    while True:
        parent_dir = os.path.dirname(anc)
        if parent_dir == anc:
            return None
        anc = parent_dir
        parent = cache.get(anc)
        if parent is not None:
            if (parent.base or parent)._positions().get(root) is None:
                return None
            idx = parent.sub_index(root)
            cache[root] = idx
            return idx


def get_index(root):
    cache = _cache()
    if cache is not None:
        # a cached root existed when it was walked: skip the stat checks
        idx = cache.get(root.rstrip("/") or "/")
        if idx is not None:
            return idx
    if not os.path.exists(root):
        log.warning("Error in walking through files due to : %r", "stat %s: no such file or directory" % root)
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
    # nearest cached ancestor (O(depth) lookups instead of scanning the cache)
    anc = root
    while True:
        parent_dir = os.path.dirname(anc)
        if parent_dir == anc:
            break
        anc = parent_dir
        parent = cache.get(anc)
        if parent is not None:
            idx = parent.sub_index(root)
            cache[root] = idx
            return idx
    idx = walk(root)
    cache[root] = idx
    return idx
