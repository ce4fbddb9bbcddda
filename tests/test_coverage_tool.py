"""``scripts/coverage.py``: line coverage without a coverage package (the
reference's ``go test -coverprofile``, ``Makefile:105-106``).  The C tracer
must see lines run in worker threads and in the CLI processes a test starts,
and the floor check must catch a drop."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import coverage as m2kcov  # noqa: E402  (scripts/coverage.py, not the PyPI package)


def test_executable_lines_come_from_code_objects(tmp_path):
    p = tmp_path / "m.py"
    p.write_text('"""doc"""\n\nX = 1\n\n\ndef f(a):\n    # comment\n    return a + 1\n\n\nclass C:\n    y = 2\n')
    assert m2kcov.executable_lines(str(p)) == {1, 3, 6, 8, 11, 12}


def test_ranges():
    assert m2kcov._ranges({1, 2, 3, 5, 7, 8}) == ["1-3", "5", "7-8"]


def test_threads_and_cli_processes_are_counted(tmp_path):
    probe = tmp_path / "test_probe.py"
    probe.write_text(
        "import os, subprocess, sys, threading\n"
        "def test_probe():\n"
        "    from move2kube_amd.utils import common\n"
        "    t = threading.Thread(target=common.go_trim_space, args=(' x ',))\n"
        "    t.start(); t.join()\n"
        "    subprocess.run([sys.executable, '-m', 'move2kube_amd', 'version'], check=True,\n"
        "                   stdout=subprocess.DEVNULL)\n")
    data = tmp_path / "data"
    out = tmp_path / "out"
    res = m2kcov.run([str(probe), "-q", "-p", "no:cacheprovider"], str(out), keep_data=str(data))
    assert res["pytest_exit"] == 0
    assert res["processes"] >= 2           # pytest and the CLI process
    mods = res["modules"]
    trim = _def_line(os.path.join(ROOT, "move2kube_amd", "utils", "common.py"), "def go_trim_space")
    hits = m2kcov.merge(str(data))
    common_hits = hits[os.path.realpath(os.path.join(ROOT, "move2kube_amd", "utils", "common.py"))]
    assert trim + 3 in common_hits         # the body's return line ran on the worker thread
    assert mods["move2kube_amd/cli/main.py"]["hit"] > 0   # only the CLI process ran the CLI
    with open(out / "coverage.json") as f:
        assert json.load(f)["total"]["hit"] > 0
    assert (out / "coverage.txt").read_text().splitlines()[-1].startswith("TOTAL")


def _def_line(path, prefix):
    with open(path) as f:
        for i, line in enumerate(f, 1):
            if line.startswith(prefix):
                return i
    raise AssertionError(prefix)


def test_floor_check(tmp_path):
    res = {"total": {"percent": 80.0}, "modules": {"a.py": {"percent": 50.0}, "b.py": {"percent": 90.0}}}
    floor = tmp_path / "floor.json"
    m2kcov.write_floor(res, str(floor))
    assert m2kcov.check_floor(res, str(floor)) == []
    res["modules"]["a.py"]["percent"] = 48.5
    res["total"]["percent"] = 79.5
    assert m2kcov.check_floor(res, str(floor)) == ["a.py 48.5% < floor 50.0%"]


def test_committed_floor_covers_every_module():
    with open(os.path.join(ROOT, "scripts", "coverage_floor.json")) as f:
        floor = json.load(f)
    mods = set(m2kcov.product_modules())
    listed = set(floor["modules"])
    assert listed <= mods
    assert {m for m in mods if m2kcov.executable_lines(os.path.join(ROOT, m))} == listed


def test_cli_help():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "coverage.py"), "--help"],
                       stdout=subprocess.PIPE, check=True)
    assert b"run" in p.stdout and b"report" in p.stdout
