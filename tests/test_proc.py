"""utils/proc.py: external tools through the native posix_spawn runtime
(ops/csrc/proc_spawn.cpp), with subprocess semantics, and the same calls on
the subprocess fallback."""

import os
import subprocess
import sys
import time

import pytest

from move2kube_amd.ops import native
from move2kube_amd.utils import common, proc


@pytest.fixture(params=["native", "fallback"])
def mode(request, monkeypatch):
    if request.param == "native":
        if not native.available() or not hasattr(native.module(), "proc_spawn"):
            pytest.skip("native extension not built")
    else:
        monkeypatch.setattr(native, "module", lambda: None)
    return request.param


def test_stdout_stderr_modes(mode):
    sh = ["/bin/sh", "-c", "echo out; echo err >&2; exit 3"]
    r = proc.run(sh, stdout=proc.PIPE, stderr=proc.PIPE)
    assert (r.returncode, r.stdout, r.stderr) == (3, b"out\n", b"err\n")
    r = proc.run(sh, stdout=proc.PIPE, stderr=proc.STDOUT)
    assert sorted(r.stdout.splitlines()) == [b"err", b"out"] and r.stderr is None
    r = proc.run(sh, stdout=proc.PIPE, stderr=proc.DEVNULL)
    assert r.stdout == b"out\n"
    r = proc.run(["/bin/sh", "-c", "cat; echo done"], stdout=proc.PIPE)  # stdin is /dev/null
    assert r.stdout == b"done\n"


def test_missing_executable_is_file_not_found(mode):
    with pytest.raises(FileNotFoundError) as ei:
        proc.run(["m2k-no-such-tool-xyz", "a"])
    assert ei.value.filename == "m2k-no-such-tool-xyz"
    with pytest.raises(OSError) as ei:
        common.run_tool(["m2k-no-such-tool-xyz"])
    assert str(ei.value) == 'exec: "m2k-no-such-tool-xyz": executable file not found in $PATH'


def test_cwd_and_file_stdout(mode, tmp_path):
    with open(tmp_path / "out.txt", "w+b") as f:
        r = proc.spawn(["/bin/sh", "-c", "pwd"], cwd=str(tmp_path), stdout=f).wait()
        assert r.returncode == 0 and r.stdout is None
        f.seek(0)
        assert f.read().decode().strip() == os.path.realpath(str(tmp_path))


def test_signal_return_code_and_sigpipe_default(mode):
    r = proc.run(["/bin/sh", "-c", "kill -TERM $$"])
    assert r.returncode == -15
    assert common.go_exit_status(r.returncode) == "signal: terminated"
    # Python ignores SIGPIPE; a child gets the default back (as with subprocess),
    # so `yes` dies quietly when `head` goes away
    r = proc.run(["/bin/sh", "-c", "yes | head -n 1"], stdout=proc.PIPE, stderr=proc.PIPE)
    assert (r.returncode, r.stdout, r.stderr) == (0, b"y\n", b"")


def test_timeout_kills_and_raises(mode):
    t = time.monotonic()
    with pytest.raises(subprocess.TimeoutExpired):
        proc.run(["/bin/sh", "-c", "exec sleep 5"], timeout=0.3)
    assert time.monotonic() - t < 3
    c = proc.spawn(["/bin/sh", "-c", "exec sleep 5"]).wait(0.2)
    assert c.timed_out


def test_child_that_closes_stdout_early_is_still_reaped(mode):
    r = proc.run(["/bin/sh", "-c", "exec >&- 2>&-; sleep 0.2; exit 4"], stdout=proc.PIPE, timeout=10)
    assert r.returncode == 4 and r.stdout == b""


def test_large_output_is_drained(mode):
    r = proc.run([sys.executable, "-c", "import sys; sys.stdout.write('x' * 3000000); sys.stderr.write('e' * 300000)"],
                 stdout=proc.PIPE, stderr=proc.PIPE)
    assert r.returncode == 0 and len(r.stdout) == 3000000 and len(r.stderr) == 300000


def test_run_many_is_concurrent_and_ordered(mode):
    cmds = [["/bin/sh", "-c", "sleep 0.4; echo %d" % i] for i in range(4)] + [["m2k-no-such-tool-xyz"]]
    t = time.monotonic()
    out = proc.run_many(cmds, stdout=proc.PIPE)
    assert time.monotonic() - t < 1.4
    assert [r.stdout for r in out[:4]] == [b"0\n", b"1\n", b"2\n", b"3\n"]
    assert isinstance(out[4], FileNotFoundError)
    out = common.run_tools([["m2k-no-such-tool-xyz"]])
    assert str(out[0]) == 'exec: "m2k-no-such-tool-xyz": executable file not found in $PATH'
    out = proc.run_many([["/bin/sh", "-c", "exec sleep 5"], ["/bin/echo", "ok"]], stdout=proc.PIPE, timeout=0.3)
    assert isinstance(out[0], subprocess.TimeoutExpired) and out[1].stdout == b"ok\n"


def test_bounded_parallelism(mode, tmp_path):
    # with parallel=1 the children never overlap: each sees no marker of another
    marker = tmp_path / "busy"
    script = "[ -e %s ] && exit 9; : > %s; sleep 0.05; rm %s" % (marker, marker, marker)
    out = proc.run_many([["/bin/sh", "-c", script]] * 4, parallel=1)
    assert [r.returncode for r in out] == [0, 0, 0, 0]


def test_run_many_drains_every_child_and_refills_slots(mode):
    # a later child writing more than a pipe holds is not blocked behind a
    # slow earlier one (its pipe drains while the first is waited for) ...
    big = [sys.executable, "-c", "import sys; sys.stdout.write('x' * 1000000)"]
    out = proc.run_many([["/bin/sh", "-c", "sleep 1; echo slow"], big], stdout=proc.PIPE, timeout=5)
    assert out[0].stdout == b"slow\n" and len(out[1].stdout) == 1000000
    # ... and with two slots, the quick children go through the slot the
    # first quick one frees while the slow one still runs
    cmds = [["/bin/sh", "-c", "sleep 1.2; echo a"]] + [["/bin/sh", "-c", "sleep 0.3; echo %d" % i] for i in range(3)]
    t = time.monotonic()
    out = proc.run_many(cmds, parallel=2, stdout=proc.PIPE)
    assert time.monotonic() - t < 1.9          # serial head-of-line waiting would take 1.2 + 0.6 + ...
    assert [r.stdout for r in out] == [b"a\n", b"0\n", b"1\n", b"2\n"]


def test_cold_tool_paths_do_not_import_subprocess(tmp_path):
    """The CNB podman probe, operator-sdk and the collectors run their tools
    without importing subprocess (its import is the cost this module avoids)."""
    if not native.available():
        pytest.skip("native extension not built")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from move2kube_amd.utils import common, proc\n"
            "r = common.run_tool(['/bin/echo', 'hi'], stdout=proc.PIPE)\n"
            "assert r.stdout == b'hi\\n'\n"
            "rs = proc.run_many([['/bin/echo', 'a'], ['/bin/echo', 'b']], parallel=1)\n"
            "assert [x.stdout for x in rs] == [b'a\\n', b'b\\n']\n"
            "print([m for m in ('subprocess', 'queue') if m in sys.modules])\n" % root)
    p = subprocess.run([sys.executable, "-S", "-c", code], stdout=subprocess.PIPE, check=True)
    assert p.stdout.strip() == b"[]"   # run_many waits natively: no thread per child


def test_child_gets_only_the_standard_descriptors(mode):
    """As subprocess's close_fds: an inheritable descriptor of ours does not
    reach the tool."""
    r, w = os.pipe()
    high = os.dup2(w, 77)  # dup2 makes an inheritable copy
    try:
        res = proc.run(["/bin/sh", "-c", "ls /proc/$$/fd"], stdout=proc.PIPE)
        fds = {int(x) for x in res.stdout.split()}
        assert {0, 1, 2} <= fds and high not in fds
    finally:
        for fd in (r, w, high):
            os.close(fd)
