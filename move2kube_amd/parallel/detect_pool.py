"""Parallel execution of containerizer detect scripts.

The reference runs ``/bin/sh <detector> <dir>`` serially for every
(detector x directory) pair during planning and again during translation
(``internal/containerizer/dockerfilecontainerizer.go:76-83``,
``s2icontainerizer.go:76-83``).  Here a batch of detect jobs is executed by the
native bounded posix_spawn pool (``ops/csrc/m2k_native.cpp:run_commands``,
GIL released) with ``settings.workers`` concurrent children, results are
returned in submission order, and results are memoised for the lifetime of the
enclosing ``fsindex.scope()`` so the translate phase does not re-run detectors
the plan phase already ran in the same process.  Unmodified built-in detectors
are evaluated in-process (:mod:`.builtin_detect`) without spawning anything.
"""

import os

from ..ops import native
from . import builtin_detect
from ..utils import fsindex, log, trace
from ..utils.constants import settings

DETECT_TIMEOUT_S = float(os.environ.get("M2K_DETECT_TIMEOUT", "300"))


class DetectResult:
    __slots__ = ("code", "stdout")

    def __init__(self, code, stdout):
        self.code = code
        self.stdout = stdout

    @property
    def ok(self):
        return self.code == 0


def _run_py(jobs):
    def one(job):
        script_dir, script, target = job
        try:
            import subprocess
            p = subprocess.run(["/bin/sh", script, target], cwd=script_dir, stdout=subprocess.PIPE,
                               stdin=subprocess.DEVNULL, timeout=DETECT_TIMEOUT_S)
            return DetectResult(p.returncode, p.stdout.decode("utf-8", "replace"))
        except (OSError, subprocess.TimeoutExpired) as e:
            log.debug("detect %s failed: %s", job, e)
            return DetectResult(-1, "")
    if len(jobs) == 1:
        return [one(jobs[0])]
    from concurrent.futures import ThreadPoolExecutor  # imports logging: keep it off the start-up path
    with ThreadPoolExecutor(max_workers=settings.workers) as ex:
        return list(ex.map(one, jobs))


def run_detect_jobs(jobs):
    """Run [(script_dir, script_name, target_dir), ...]; returns DetectResults in order."""
    if not jobs:
        return []
    with trace.span("detect-batch", "detect", jobs=len(jobs)):
        return _run_detect_jobs(jobs)


def _run_detect_jobs(jobs):
    cache = fsindex.scoped_cache("detect")
    todo, todo_idx = [], []
    results = [None] * len(jobs)
    for i, job in enumerate(jobs):
        if cache is not None and job in cache:
            results[i] = cache[job]
        else:
            todo.append(job)
            todo_idx.append(i)
    if todo:
        spawn, spawn_idx = [], []
        fns = {}
        shared = {}  # (code, stdout bytes) -> one read-only DetectResult
        cur = None  # builtin_detect.Dir of the current target (jobs come grouped by target)
        for k, job in enumerate(todo):
            d, script, target = job
            fn = fns.get((d, script), False)
            if fn is False:
                fn = fns[(d, script)] = builtin_detect.lookup(d, script)
            if fn is None:
                spawn.append(job)
                spawn_idx.append(k)
                continue
            if cur is None or cur.src != target:
                cur = builtin_detect.Dir(target)
            key = fn(cur)
            r = shared.get(key)
            if r is None:
                r = shared[key] = DetectResult(key[0], key[1].decode("utf-8", "replace"))
            results[todo_idx[k]] = r
            if cache is not None:
                cache[job] = r
        todo = spawn
        todo_idx = [todo_idx[k] for k in spawn_idx]
    if todo:
        if native.available():
            raw = native.run_commands([["/bin/sh", script, target] for (_, script, target) in todo],
                                      [d for (d, _, _) in todo], settings.workers, DETECT_TIMEOUT_S)
            res = [DetectResult(code, out.decode("utf-8", "replace")) for code, out in raw]
        else:
            res = _run_py(todo)
        for i, job, r in zip(todo_idx, todo, res):
            results[i] = r
            if cache is not None:
                cache[job] = r
    return results


def run_detect(script_dir, script, target):
    return run_detect_jobs([(script_dir, script, target)])[0]
