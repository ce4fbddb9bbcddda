"""External tools without the ``subprocess`` module.

The reference runs its external tools with Go's ``os/exec``:
``operator-sdk`` (``internal/transformer/k8stransformer.go:226-247``), the
container runtime of the CNB provider chain
(``internal/containerizer/cnb/containerruntimeprovider.go:45-130``) and the
``cf``/``kubectl``/``docker`` CLIs of the collectors (``internal/collector/``).
In a cold CLI process ``import subprocess`` alone costs about as much as one
of those tools, so the commands go through the native runtime's
``proc_spawn``/``proc_wait`` (``ops/csrc/proc_spawn.cpp``: ``posix_spawnp``,
pipes drained and the child reaped with the GIL released).  Where the
extension is not built the same calls run on ``subprocess.Popen``.

Semantics follow ``subprocess``: stdin is ``/dev/null``; a missing executable
raises ``FileNotFoundError`` with ``filename`` = ``argv[0]``; a negative
return code is the signal that ended the child; :func:`run` raises
``subprocess.TimeoutExpired`` after killing a child that overran.
"""

import os

from ..ops import native

PIPE = -1
DEVNULL = -2
INHERIT = -3
STDOUT = -4  # stderr only: into stdout


class Completed:
    """What ``subprocess.run`` returns (``args``, ``returncode``, ``stdout``,
    ``stderr``), plus ``timed_out``."""
    __slots__ = ("args", "returncode", "stdout", "stderr", "timed_out")

    def __init__(self, args, returncode, stdout, stderr, timed_out=False):
        self.args = args
        self.returncode = returncode
        self.stdout = stdout
        self.stderr = stderr
        self.timed_out = timed_out


def _fd(x):
    if isinstance(x, int):
        return x
    return x.fileno()  # a file object


class Child:
    """A started tool; :meth:`wait` collects it once."""

    def __init__(self, args, pid=None, out_fd=-1, err_fd=-1, popen=None, pipes=(False, False)):
        self.args = args
        self.pid = pid if popen is None else popen.pid
        self._out_fd = out_fd
        self._err_fd = err_fd
        self._popen = popen
        self._pipes = pipes
        self._done = None

    def wait(self, timeout=None):
        """Wait (drain the pipes, reap); a child still running after
        ``timeout`` seconds is killed and ``timed_out`` is set."""
        if self._done is not None:
            return self._done
        if self._popen is None:
            # proc_wait closes the descriptors whatever happens (an interrupt
            # included): hand them over once, never twice
            ofd, efd, self._out_fd, self._err_fd = self._out_fd, self._err_fd, -1, -1
            rc, out, err, timed_out = native.module().proc_wait(self.pid, ofd, efd, float(timeout or 0))
            self._done = Completed(self.args, rc, out if self._pipes[0] else None,
                                   err if self._pipes[1] else None, timed_out)
            return self._done
        import subprocess
        p = self._popen
        try:
            out, err = p.communicate(timeout=timeout)
            timed_out = False
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
            timed_out = True
        self._done = Completed(self.args, p.returncode, out, err, timed_out)
        return self._done


def spawn(argv, cwd=None, stdout=PIPE, stderr=DEVNULL):
    """Start ``argv`` (PATH search as ``execvp``) with stdin on ``/dev/null``.
    ``stdout``/``stderr``: :data:`PIPE`, :data:`DEVNULL`, :data:`INHERIT`, a
    file object or descriptor; ``stderr`` may also be :data:`STDOUT`."""
    args = list(argv)
    m = native.module()
    if m is not None and hasattr(m, "proc_spawn"):
        out_mode = stdout if isinstance(stdout, int) and stdout < 0 else _fd(stdout)
        err_mode = stderr if isinstance(stderr, int) and stderr < 0 else _fd(stderr)
        pid, ofd, efd = m.proc_spawn([os.fsencode(a) for a in args], None if cwd is None else os.fsencode(cwd),
                                     out_mode, err_mode)
        return Child(args, pid, ofd, efd, pipes=(stdout == PIPE, stderr == PIPE))
    import subprocess
    conv = {PIPE: subprocess.PIPE, DEVNULL: subprocess.DEVNULL, INHERIT: None, STDOUT: subprocess.STDOUT}
    p = subprocess.Popen(args, cwd=cwd, stdin=subprocess.DEVNULL,
                         stdout=conv.get(stdout, stdout) if isinstance(stdout, int) else stdout,
                         stderr=conv.get(stderr, stderr) if isinstance(stderr, int) else stderr)
    return Child(args, popen=p)


def _timeout_error(c, timeout):
    import subprocess
    return subprocess.TimeoutExpired(c.args, timeout, output=c.stdout, stderr=c.stderr)


def run(argv, cwd=None, stdout=PIPE, stderr=DEVNULL, timeout=None):
    """``subprocess.run(argv, stdin=DEVNULL, ...)``."""
    c = spawn(argv, cwd=cwd, stdout=stdout, stderr=stderr).wait(timeout)
    if c.timed_out:
        raise _timeout_error(c, timeout)
    return c


def run_many(argvs, parallel=None, cwd=None, stdout=PIPE, stderr=DEVNULL, timeout=None):
    """``[run(a, ...) for a in argvs]`` with up to ``parallel`` children alive
    at once (all of them by default); a raised error is returned in its slot.
    Every live child's pipes drain at once, its deadline counts from its start,
    and a slot is refilled as soon as any child exits: natively one poll loop
    over all of them (``procgroup_*``, ``ops/csrc/proc_spawn.cpp``), otherwise
    one waiting thread per child."""
    n = len(argvs)
    if parallel is None or parallel < 1:
        parallel = n
    m = native.module()
    if m is not None and hasattr(m, "procgroup_new"):
        return _run_many_native(m, argvs, parallel, cwd, stdout, stderr, timeout)
    return _run_many_threads(argvs, parallel, cwd, stdout, stderr, timeout)


def _run_many_native(m, argvs, parallel, cwd, stdout, stderr, timeout):
    n = len(argvs)
    out = [None] * n
    group = m.procgroup_new()
    live = 0
    nxt = 0
    while nxt < n or live:
        while nxt < n and live < parallel:
            try:
                c = spawn(argvs[nxt], cwd=cwd, stdout=stdout, stderr=stderr)
            except OSError as e:
                out[nxt] = e
            else:
                ofd, efd, c._out_fd, c._err_fd = c._out_fd, c._err_fd, -1, -1   # the group owns them now
                m.procgroup_add(group, nxt, c.pid, ofd, efd, float(timeout or 0))
                out[nxt] = c
                live += 1
            nxt += 1
        if live:
            i, rc, o, e, timed_out = m.procgroup_wait_any(group)
            c = out[i]
            r = c._done = Completed(c.args, rc, o if c._pipes[0] else None, e if c._pipes[1] else None, timed_out)
            out[i] = _timeout_error(r, timeout) if timed_out else r
            live -= 1
    return out


def _run_many_threads(argvs, parallel, cwd, stdout, stderr, timeout):
    import queue
    import threading
    n = len(argvs)
    out = [None] * n
    done = queue.SimpleQueue()

    def waiter(i, c):
        try:
            r = c.wait(timeout)
            done.put((i, _timeout_error(r, timeout) if r.timed_out else r))
        except BaseException as e:  # noqa: BLE001 - reported in the child's slot
            done.put((i, e))

    live = 0
    nxt = 0
    while nxt < n or live:
        while nxt < n and live < parallel:
            try:
                c = spawn(argvs[nxt], cwd=cwd, stdout=stdout, stderr=stderr)
            except OSError as e:
                out[nxt] = e
            else:
                threading.Thread(target=waiter, args=(nxt, c), name="m2k-proc-wait", daemon=True).start()
                live += 1
            nxt += 1
        if live:
            i, r = done.get()
            out[i] = r
            live -= 1
    return out
