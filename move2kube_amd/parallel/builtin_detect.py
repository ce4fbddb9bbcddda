"""In-process evaluation of the built-in containerizer detectors.

Every detector shipped in ``assets/m2kassets`` is a few lines of POSIX sh
(``test -f``, ``find -name``, a ``*.war`` glob, ``grep -lR __main__``).  Running
them means fork+exec of ``sh`` plus its ``find``/``wc``/``head`` children for
every (detector x directory) pair - on a 17-service tree that is ~70% of a
whole ``translate``.  This module evaluates the *unmodified* built-in scripts
natively against the already-built directory index and returns exactly the
exit status and stdout the script prints.

A script is only evaluated in-process when it lives under the unpacked assets
directory **and** its bytes hash to the packaged original; user-supplied or
edited detectors (and everything with ``M2K_NATIVE_DETECT=0``) always run as
real processes through :mod:`move2kube_amd.parallel.detect_pool`.

Known, documented difference: with several ``__main__`` files the python
detectors report the lexically first one, while ``grep -R`` reports the first
in readdir order (file-system dependent in the reference too).
"""

import os

from ..utils import common, fsindex
from ..utils.constants import settings

_HERE = os.path.dirname(os.path.abspath(__file__))
_ASSETS_SRC = os.path.join(os.path.dirname(_HERE), "assets", "m2kassets")


class Dir:
    """One target directory of a detect batch: its index is looked up once for
    all the detectors run against it (they run back to back)."""

    __slots__ = ("src", "idx", "_full")

    def __init__(self, src):
        self.src = src
        self.idx = fsindex.peek_index(src)  # never walks
        self._full = False

    def index(self):
        """``fsindex.get_index(src)`` (walks if the scope does not cover src);
        None when src cannot be listed."""
        if self._full is False:
            try:
                self._full = fsindex.get_index(self.src)
            except (OSError, FileNotFoundError):
                self._full = None
        return self._full


def _exists_file(d, name):
    """``test -f "$src/name"``, answered from the scope's directory index when
    it covers ``src`` (the plan/translate scopes always do) - no stat per
    (detector x directory) pair; symlinks and unknowns still go to the FS."""
    idx = d.idx
    if idx is not None:
        k = idx.child_kind(name)
        if k == fsindex.FILE:
            return True
        if k in (fsindex.MISSING, fsindex.DIR, fsindex.OTHER):
            return False
    return os.path.isfile(os.path.join(d.src, name))


def _find_any(d, pattern):
    """``find "$src"/. -name pattern -print | head -n1 | wc -l`` == 1."""
    idx = d.index()
    return idx is not None and idx.has_match(pattern)


def _find_main(d):
    """``grep -lRe __main__ "$src" | awk '/.py$/' | head -n1`` -> relative path."""
    src = d.src
    idx = d.index()
    if idx is None:
        return ""
    for p, k in zip(idx.paths, idx.kinds):
        if k == fsindex.DIR:
            continue
        shown = src + p[len(idx.root):] if p.startswith(idx.root) else p
        if len(shown) < 3 or not shown.endswith("py"):  # awk '/.py$/': any character, then "py"
            continue
        try:
            if b"__main__" not in common.read_bytes(p):
                continue
        except OSError:
            continue
        try:
            return os.path.relpath(os.path.realpath(shown), os.path.realpath(src))
        except ValueError:
            return ""
    return ""


def _ok(s):
    return 0, s.encode("utf-8", "surrogateescape")


_FAIL = (1, b"")


def _simple(marker, out):
    def fn(d):
        return _ok(out) if _exists_file(d, marker) else _FAIL
    return fn


def _recursive(pattern, out):
    def fn(d):
        return _ok(out) if _find_any(d, pattern) else _FAIL
    return fn


def _war(port):
    def fn(d):
        src, idx = d.src, d.idx
        if idx is not None and idx.kinds and idx.kinds[0] == fsindex.DIR:
            wars = idx.children_matching("*.war")
        else:
            try:
                wars = sorted(n for n in os.listdir(src) if n.endswith(".war") and not n.startswith("."))
            except OSError:
                wars = []
        # the script's loop exits 1 unless the first (sorted) match exists
        if not wars or not os.path.exists(os.path.join(src, wars[0])):
            return _FAIL
        return _ok('{"port":%d, "war_path":"%s"}' % (port, wars[0]))
    return fn


_PY_MARKERS = ("requirements.txt", "setup.py", "environment.yml", "Pipfile")


def _python_df(d):
    for m in _PY_MARKERS:
        if _exists_file(d, m):
            return _ok('{"main_script_rel_path": "%s", "app_name": "app", "port": 8080}' % _find_main(d))
    return _FAIL


def _python_s2i(d):
    for m in _PY_MARKERS:
        if _exists_file(d, m):
            return _ok('{"builder": "%s", "app_file": "%s", "app_name": "app", "port": 8080}'
                       % ("registry.access.redhat.com/rhscl/python-36-rhel7:latest", _find_main(d)))
    return _FAIL


def _golang_s2i(d):
    if not _exists_file(d, "go.mod") and not _find_any(d, "*.go"):
        return _FAIL
    return _ok('{"builder": "%s", "port": 8080}\n' % "registry.access.redhat.com/ubi8/go-toolset:latest")


def _java_s2i(d):
    if _exists_file(d, "build.gradle") or _exists_file(d, "build.xml"):
        return _FAIL
    if _exists_file(d, "pom.xml"):
        return _ok('{"builder": "%s", "port": 8080}\n' % "registry.access.redhat.com/jboss-eap-6/eap64-openshift:latest")
    if not _find_any(d, "*.java"):
        return _FAIL
    return _ok('{"builder": "%s", "port": 8080}\n'
               % "registry.access.redhat.com/redhat-openjdk-18/openjdk18-openshift:latest")


DETECTORS = {
    ("dockerfiles/django", "m2kdfdetect.sh"): _simple("Pipfile", '{"port": 8080, "binding": "0.0.0.0:8080"}\n'),
    ("dockerfiles/golang", "m2kdfdetect.sh"): _recursive("*.go", '{"port": 8080, "app_name": "app-bin"}\n'),
    ("dockerfiles/java-war-jboss", "m2kdfdetect.sh"): _war(8080),
    ("dockerfiles/java-war-liberty", "m2kdfdetect.sh"): _war(9080),
    ("dockerfiles/java-war-tomcat", "m2kdfdetect.sh"): _war(8080),
    ("dockerfiles/javaant", "m2kdfdetect.sh"): _simple(
        "build.xml", '{"port": 8080, "ant_cmd": "ant all", "app_name": "simplewebapp"}\n'),
    ("dockerfiles/javagradle", "m2kdfdetect.sh"): _simple("build.gradle", '{"port": 8080, "app_name": "simplewebapp"}\n'),
    ("dockerfiles/javamaven", "m2kdfdetect.sh"): _simple("pom.xml", '{"port": 8080, "app_name": "app"}\n'),
    ("dockerfiles/nodejs", "m2kdfdetect.sh"): _simple("package.json", '{"port": 8080, "app_name": "app"}\n'),
    ("dockerfiles/php", "m2kdfdetect.sh"): _recursive(
        "*.php", '{"port": 8080, "binding": "0.0.0.0:8080", "app_name": "app"}\n'),
    ("dockerfiles/python", "m2kdfdetect.sh"): _python_df,
    ("dockerfiles/ruby", "m2kdfdetect.sh"): _simple("Gemfile", '{"port": 8080, "app_name": "app"}\n'),
    ("s2i/golang", "m2ks2idetect.sh"): _golang_s2i,
    ("s2i/java", "m2ks2idetect.sh"): _java_s2i,
    ("s2i/nodejs", "m2ks2idetect.sh"): _simple(
        "package.json", '{"builder": "%s", "port": 8080}\n' % "registry.access.redhat.com/ubi8/nodejs-10"),
    ("s2i/php", "m2ks2idetect.sh"): _recursive(
        "*.php", '{"builder": "%s", "port": 8080}\n' % "registry.access.redhat.com/rhscl/php-72-rhel7:latest"),
    ("s2i/python", "m2ks2idetect.sh"): _python_s2i,
    ("s2i/ruby", "m2ks2idetect.sh"): _simple(
        "Gemfile", '{"builder": "%s", "port": 8080}\n' % "registry.access.redhat.com/rhscl/ruby-25-rhel7:latest"),
}


def _read(path):
    with open(path, "rb") as f:
        return f.read()


_MISSING = object()
_packaged = {}  # (rel, script) -> bytes of the packaged original (read on first use)


def _packaged_bytes(key):
    b = _packaged.get(key)
    if b is None:
        try:
            b = _read(os.path.join(_ASSETS_SRC, key[0], key[1]))
        except OSError:
            b = _MISSING
        _packaged[key] = b
    return None if b is _MISSING else b

_verified = {}  # (path, mtime_ns, size) -> bool


def enabled():
    return os.environ.get("M2K_NATIVE_DETECT", "1") not in ("0", "")


def lookup(script_dir, script):
    """The in-process implementation for this detector, or None."""
    if not enabled():
        return None
    # within one plan/translate scope the assets directory does not change:
    # resolve and hash-check each detector once per scope
    memo = fsindex.scoped_cache("builtin-detect")
    if memo is not None:
        key = (script_dir, script, settings.assets_path)
        fn = memo.get(key, False)
        if fn is False:
            fn = memo[key] = _lookup(script_dir, script)
        return fn
    return _lookup(script_dir, script)


_resolved = {}  # (script_dir, script, assets_path), all absolute -> (key, path) or None


def _resolve(script_dir, script, assets_path):
    """(detector key, script path) when ``script_dir`` lies in the assets tree
    and names a built-in detector, else None (pure path arithmetic)."""
    assets = os.path.abspath(assets_path)
    d = os.path.abspath(script_dir)
    if not d.startswith(assets + os.sep):
        return None
    key = (os.path.relpath(d, assets), script)
    if key not in DETECTORS:
        return None
    return key, os.path.join(d, script)


def _lookup(script_dir, script):
    assets_path = settings.assets_path
    if os.path.isabs(script_dir) and os.path.isabs(assets_path):
        mk = (script_dir, script, assets_path)
        r = _resolved.get(mk, _MISSING)
        if r is _MISSING:
            r = _resolved[mk] = _resolve(script_dir, script, assets_path)
    else:  # relative to the working directory: nothing to remember
        r = _resolve(script_dir, script, assets_path)
    if r is None:
        return None
    key, path = r
    fn = DETECTORS[key]
    want = _packaged_bytes(key)
    if want is None:
        return None
    try:
        st = os.stat(path)
    except OSError:
        return None
    vk = (path, st.st_mtime_ns, st.st_size)
    ok = _verified.get(vk)
    if ok is None:
        try:
            ok = _read(path) == want  # byte-identical to the packaged detector
        except OSError:
            ok = False
        _verified[vk] = ok
    return fn if ok else None
