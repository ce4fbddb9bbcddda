"""The package's bytecode bundle (``ops/bytecode.py`` writes it,
``move2kube_amd/__init__.py`` serves from it): modules load from it while their
sources are unchanged, an edited, added or removed file takes the normal
import path, a bundle of another interpreter or ``-O`` level is ignored, and
tracebacks still show the source lines.  Each case runs in a fresh interpreter
over a private copy of the package."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def tree(tmp_path):
    dst = tmp_path / "move2kube_amd"
    shutil.copytree(os.path.join(ROOT, "move2kube_amd"), str(dst),
                    ignore=shutil.ignore_patterns("__pycache__", "_bytecode.bin", "csrc"))
    sys.path.insert(0, ROOT)
    try:
        from move2kube_amd.ops import bytecode
        bytecode.write(str(dst))
        assert not bytecode.stale(str(dst))
    finally:
        sys.path.remove(ROOT)
    return tmp_path


def _py(tree, code, *flags, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "M2K_BYTECODE_BUNDLE")}
    e.update(env or {})
    p = subprocess.run([sys.executable, "-S"] + list(flags) + ["-c", code], cwd=str(tree), env=e,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    assert p.returncode == 0, p.stderr
    return p.stdout.split()


LOADERS = ("import sys\nsys.path.insert(0, '.')\nimport move2kube_amd.cli.main, move2kube_amd.utils.common\n"
           "for n in ('move2kube_amd.cli.main', 'move2kube_amd.utils.common', 'move2kube_amd.cli'):\n"
           "    print(type(sys.modules[n].__loader__).__name__)\n")


def test_modules_come_from_the_bundle(tree):
    assert _py(tree, LOADERS) == ["_BytecodeBundle"] * 3
    assert _py(tree, LOADERS, env={"M2K_BYTECODE_BUNDLE": "0"}) == ["SourceFileLoader"] * 3


def test_edited_module_falls_back_to_its_source(tree):
    p = tree / "move2kube_amd" / "utils" / "common.py"
    p.write_text(p.read_text() + "\nEDITED = 1\n")
    code = LOADERS + "print(move2kube_amd.utils.common.EDITED)\n"
    assert _py(tree, code) == ["_BytecodeBundle", "SourceFileLoader", "_BytecodeBundle", "1"]


def test_same_size_edit_with_a_new_mtime_falls_back(tree):
    p = tree / "move2kube_amd" / "models" / "info.py"
    text = p.read_text()
    p.write_text(text.replace('VERSION = "v', 'VERSION = "w', 1))
    st = os.stat(str(p))
    os.utime(str(p), (st.st_atime, st.st_mtime + 5))
    code = "import sys\nsys.path.insert(0, '.')\nimport move2kube_amd\nprint(move2kube_amd.__version__[0])\n"
    assert _py(tree, code) == ["w"]


def test_added_and_removed_modules(tree):
    (tree / "move2kube_amd" / "utils" / "newmod.py").write_text("X = 42\n")
    os.unlink(str(tree / "move2kube_amd" / "utils" / "sshkeys.py"))
    code = ("import sys\nsys.path.insert(0, '.')\nimport move2kube_amd.utils.newmod as m\nprint(m.X)\n"
            "try:\n    import move2kube_amd.utils.sshkeys\nexcept ModuleNotFoundError:\n    print('gone')\n")
    assert _py(tree, code) == ["42", "gone"]
    sys.path.insert(0, ROOT)
    try:
        from move2kube_amd.ops import bytecode
        assert bytecode.stale(str(tree / "move2kube_amd"))
    finally:
        sys.path.remove(ROOT)


def test_bundle_of_another_optimize_level_is_ignored(tree):
    assert _py(tree, LOADERS, "-O") == ["SourceFileLoader"] * 3


def test_python_m_and_tracebacks(tree):
    e = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    p = subprocess.run([sys.executable, "-m", "move2kube_amd", "version"], cwd=str(tree), env=e,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    assert p.returncode == 0 and p.stdout.startswith("v"), p.stderr
    # the code objects carry the unpacked tree's paths: tracebacks show the source lines
    code = ("import sys, traceback\nsys.path.insert(0, '.')\nfrom move2kube_amd.utils import fastjson\n"
            "try:\n    fastjson.loads('')\nexcept ValueError:\n    tb = traceback.format_exc()\n"
            "print(type(fastjson.__loader__).__name__)\nprint(repr(tb))\n")
    e = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    p = subprocess.run([sys.executable, "-S", "-c", code], cwd=str(tree), env=e, stdout=subprocess.PIPE, text=True)
    loader, tb = p.stdout.splitlines()
    assert loader == "_BytecodeBundle"
    assert repr(os.path.join(str(tree), "move2kube_amd", "utils", "fastjson.py"))[1:-1] in tb
    assert "raise ValueError(" in tb
