import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# the read-only reference checkout; CI has none (M2K_REFERENCE_DIR=/nonexistent
# reproduces that here: the `reference` tests skip)
REFERENCE = os.environ.get("M2K_REFERENCE_DIR", "/root/reference")

# deterministic offline runs everywhere
os.environ.setdefault("M2K_NO_NETWORK", "1")
os.environ.setdefault("M2K_DISABLE_CNB", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "reference: needs the read-only reference checkout for its fixtures")


def pytest_collection_modifyitems(config, items):
    if os.path.isdir(REFERENCE):
        return
    skip = pytest.mark.skip(reason="reference fixtures not available")
    for item in items:
        if "reference" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _fresh_state():
    """Every test starts with no QA engines, no caches and default settings."""
    from move2kube_amd import api
    from move2kube_amd.utils.constants import settings
    api.reset_state()
    saved = (settings.compat, settings.ignore_environment, settings.temp_path, settings.assets_path)
    yield
    api.reset_state()
    settings.compat, settings.ignore_environment, settings.temp_path, settings.assets_path = saved


@pytest.fixture
def assets_dir(monkeypatch):
    """A private unpacked copy of m2kassets (tests may edit detectors; the CLI
    itself uses the packaged tree read-only)."""
    from move2kube_amd import assets
    from move2kube_amd.utils.constants import settings
    monkeypatch.setenv("M2K_UNPACK_ASSETS", "1")
    tmp = assets.setup()
    yield settings.assets_path
    assets.cleanup(tmp)


def ref_path(*parts):
    return os.path.join(REFERENCE, *parts)


# -- fault injection as an unprivileged user ----------------------------------
#
# The reference's permission tests (chmod-0 files and directories) mean
# nothing to root, which reads and writes them anyway, and this suite runs as
# root in the build containers.  ``unprivileged`` runs the checking part of
# such a test in a forked child that has dropped to nobody/nogroup, over a
# tree in a directory that user owns and can reach.

NOBODY = 65534


def _preload_package():
    """Import every module of the package in the parent: the child cannot read
    the repository (its parent directories are private to root), so a lazy
    import inside the code under test must find its module in sys.modules."""
    import importlib
    import pkgutil
    import move2kube_amd
    for m in pkgutil.walk_packages(move2kube_amd.__path__, "move2kube_amd."):
        if m.name.endswith("__main__") or ".ops.gpu" in m.name or ".ops.lib" in m.name:
            continue  # the CLI entry, the GPU path, the HIP library (not a Python module)
        importlib.import_module(m.name)


class Unprivileged:
    def __init__(self, base):
        self.tmp = base
        self.as_root = os.geteuid() == 0

    def chown(self, *paths):
        """Give a tree built by the parent to the child's user (root only)."""
        if not self.as_root:
            return
        for p in paths or (self.tmp,):
            for dp, dns, fns in os.walk(p):
                os.lchown(dp, NOBODY, NOBODY)
                for n in dns + fns:
                    os.lchown(os.path.join(dp, n), NOBODY, NOBODY)

    def run(self, fn):
        """``fn()`` with uid/gid 65534 (in-process when not root); an exception
        in it fails the test with the child's traceback."""
        if not self.as_root:
            fn()
            return
        import traceback
        _preload_package()
        r, w = os.pipe()
        pid = os.fork()
        if pid == 0:  # child: never returns into pytest
            code, msg = 0, b""
            try:
                os.close(r)
                try:
                    os.setgroups([])
                    os.setresgid(NOBODY, NOBODY, NOBODY)
                    os.setresuid(NOBODY, NOBODY, NOBODY)
                except OSError as e:
                    code, msg = 2, str(e).encode()
                else:
                    os.chdir(self.tmp)
                    fn()
            except BaseException:  # noqa: BLE001
                code, msg = 1, traceback.format_exc().encode("utf-8", "replace")
            try:
                os.write(w, msg)
            finally:
                os._exit(code)
        os.close(w)
        chunks = []
        while True:
            b = os.read(r, 65536)
            if not b:
                break
            chunks.append(b)
        os.close(r)
        _, status = os.waitpid(pid, 0)
        out = b"".join(chunks).decode("utf-8", "replace")
        if os.WIFSIGNALED(status):
            pytest.fail("unprivileged child killed by signal %d" % os.WTERMSIG(status))
        code = os.WEXITSTATUS(status)
        if code == 2:
            pytest.skip("cannot drop to an unprivileged user: " + out)
        if code != 0:
            pytest.fail("in the unprivileged child:\n" + out, pytrace=False)


@pytest.fixture
def unprivileged():
    """A directory the unprivileged child owns (under a world-traversable
    parent) plus ``run(fn)``; see :class:`Unprivileged`."""
    import shutil
    import tempfile
    base = tempfile.mkdtemp(prefix="m2k-nobody-", dir="/tmp" if os.path.isdir("/tmp") else None)
    os.chmod(base, 0o755)
    u = Unprivileged(base)
    u.chown()
    try:
        yield u
    finally:
        for dp, dns, _fns in os.walk(base):
            for d in dns:
                try:
                    os.chmod(os.path.join(dp, d), 0o755)
                except OSError:
                    pass
        shutil.rmtree(base, ignore_errors=True)
