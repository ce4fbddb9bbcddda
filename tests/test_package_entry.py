"""The package's process entry (``move2kube_amd/__init__.py``): the bytecode
bundle finder's fallbacks, the CLI start-up trims and the fast exit's exit
codes (``sys.exit`` semantics without the interpreter teardown).  The bundle
against edited trees is ``tests/test_bytecode_bundle.py``."""

import os
import subprocess
import sys

import pytest

import move2kube_amd as pkg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(code, flags=(), stdout=subprocess.PIPE):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.run([sys.executable] + list(flags) + ["-c", code], env=env, stdout=stdout,
                          stderr=subprocess.PIPE)


def test_exit_with_a_message_is_status_1():
    p = _py("import move2kube_amd as m; m._cli_exit('Error: bad flag')")
    assert p.returncode == 1 and p.stderr.decode() == "Error: bad flag\n"


def test_exit_status_is_taken_modulo_256():
    assert _py("import move2kube_amd as m; m._cli_exit(257)").returncode == 1
    assert _py("import move2kube_amd as m; m._cli_exit(None)").returncode == 0


def test_a_failed_stdout_flush_exits_120():
    """CPython's rule at exit: a stdout that cannot be flushed (ENOSPC on
    ``/dev/full``) is reported and turns status 0 into 120."""
    if not os.path.exists("/dev/full"):
        pytest.skip("no /dev/full")
    with open("/dev/full", "w") as full:
        p = _py("import move2kube_amd as m, sys; sys.stdout.write('x' * 10); m._cli_exit(0)", stdout=full)
    assert p.returncode == 120
    assert "Exception ignored in" in p.stderr.decode() and "No space left on device" in p.stderr.decode()
    with open("/dev/full", "w") as full:
        p = _py("import move2kube_amd as m, sys; sys.stdout.write('x'); m._cli_exit(3)", stdout=full)
    assert p.returncode == 3          # a failing command keeps its own status


def test_cli_process_trims():
    """As the release launcher starts it (``python -S``, nothing of shutil's
    imported yet): no garbage collector, shutil without bz2/lzma."""
    p = _py("import sys; import move2kube_amd as m; m._cli_process(); import gc; "
            "print(gc.isenabled(), 'shutil' in sys.modules, 'bz2' in sys.modules, 'lzma' in sys.modules, "
            "sys.modules.get('msvcrt', 1))", flags=["-S"])
    assert p.stdout.decode().split() == ["False", "True", "False", "False", "None"]


def _bundle():
    for f in sys.meta_path:
        if type(f).__name__ == "_BytecodeBundle":
            return f
    pytest.skip("no bytecode bundle in this tree (make build)")


def test_bundle_loader_protocol():
    b = _bundle()
    spec = b.find_spec("move2kube_amd.utils.common")
    if spec is None:
        pytest.skip("utils/common.py changed since the bundle was built")
    assert spec.origin == os.path.join(ROOT, "move2kube_amd", "utils", "common.py") and spec.loader is b
    assert b.get_filename("move2kube_amd.utils.common") == spec.origin
    with open(spec.origin) as f:
        assert b.get_source("move2kube_amd.utils.common") == f.read()
    assert b.is_package("move2kube_amd.utils") and not b.is_package("move2kube_amd.utils.common")
    pspec = b.find_spec("move2kube_amd.utils")
    assert pspec.submodule_search_locations == [os.path.join(ROOT, "move2kube_amd", "utils")]
    assert b.create_module(spec) is None
    assert b.find_spec("not_ours") is None


def test_bundle_skips_a_module_whose_source_is_gone(monkeypatch):
    b = _bundle()
    name = "move2kube_amd.utils.common"
    rec = list(b._mods[name])
    rec[1] = os.path.join("utils", "no_such_module.py")
    monkeypatch.setitem(b._mods, name, tuple(rec))
    assert b.find_spec(name) is None


@pytest.mark.parametrize("content", [b"", b"XXXX\x00\x00\x00\x04abcd", b"M2KB\x00\x00\x00\x03abc"])
def test_a_broken_bundle_is_ignored(tmp_path, monkeypatch, content):
    bad = tmp_path / "_bytecode.bin"
    bad.write_bytes(content)
    real_open = pkg._os.open
    before = list(sys.meta_path)
    monkeypatch.setattr(pkg._os, "open", lambda path, flags, *a: real_open(str(bad), flags, *a))
    pkg._install_bytecode_bundle()
    assert sys.meta_path == before


def test_a_missing_bundle_is_ignored(monkeypatch):
    before = list(sys.meta_path)

    def missing(path, flags, *a):
        raise FileNotFoundError(path)
    monkeypatch.setattr(pkg._os, "open", missing)
    pkg._install_bytecode_bundle()
    assert sys.meta_path == before
