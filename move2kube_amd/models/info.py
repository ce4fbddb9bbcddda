"""Version information (reference ``types/info/versioninfo.go``)."""


from ..utils import log
from ..utils.lazyre import lazy as _lazy_re

VERSION = "v0.1.0"
BUILD_METADATA = ""
GIT_COMMIT = ""
GIT_TREE_STATE = ""
try:  # stamped into release archives by scripts/builddist.py (the reference's -ldflags -X, Makefile:40-56)
    from .._buildinfo import BUILD_METADATA, GIT_COMMIT, GIT_TREE_STATE, VERSION  # noqa: F401
except ImportError:
    pass


def get_version():
    if not BUILD_METADATA:
        return VERSION
    return VERSION + "+" + BUILD_METADATA


class VersionInfo:
    def __init__(self, version="", git_commit="", git_tree_state="", runtime_version=""):
        self.version = version
        self.git_commit = git_commit
        self.git_tree_state = git_tree_state
        self.runtime_version = runtime_version

    def to_yaml(self):
        d = {}
        if self.version:
            d["version"] = self.version
        if self.git_commit:
            d["gitCommit"] = self.git_commit
        if self.git_tree_state:
            d["gitTreeState"] = self.git_tree_state
        if self.runtime_version:
            d["goVersion"] = self.runtime_version
        return d

    def is_same_version(self):
        try:
            binary = _parse_semver(get_version())
        except ValueError as e:
            log.warning("Unable to load current version of binary : %s", e)
            return False
        try:
            obj = _parse_semver(self.version)
        except ValueError as e:
            log.warning("Unable to load current version : %s", e)
            return False
        c = _compare(binary, obj)
        if c == 0:
            return True
        if c < 0:
            log.warning("The file version (%s) is newer than the binary version (%s).", self.version, get_version())
        else:
            log.warning("The file version (%s) is older than the binary version (%s).", self.version, get_version())
        return False


def get_version_info():
    import platform  # only `version -l` needs it (CLI start-up time)
    return VersionInfo(get_version(), GIT_COMMIT, GIT_TREE_STATE, "python" + platform.python_version())


_SEMVER = _lazy_re(r"^v?(\d+)(?:\.(\d+))?(?:\.(\d+))?(?:-([0-9A-Za-z\-.]+))?(?:\+([0-9A-Za-z\-.]+))?$")


def _parse_semver(s):
    """Masterminds/semver NewVersion (lenient: optional v, minor, patch)."""
    m = _SEMVER.match(s or "")
    if not m:
        raise ValueError("Invalid Semantic Version")
    major, minor, patch, pre, _ = m.groups()
    return int(major), int(minor or 0), int(patch or 0), pre or ""


def _compare(a, b):
    if a[:3] != b[:3]:
        return -1 if a[:3] < b[:3] else 1
    pa, pb = a[3], b[3]
    if pa == pb:
        return 0
    if pa == "":
        return 1
    if pb == "":
        return -1
    ia, ib = pa.split("."), pb.split(".")
    for x, y in zip(ia, ib):
        if x == y:
            continue
        if x.isdigit() and y.isdigit():
            return -1 if int(x) < int(y) else 1
        if x.isdigit():
            return -1
        if y.isdigit():
            return 1
        return -1 if x < y else 1
    return (len(ia) > len(ib)) - (len(ia) < len(ib))
