"""Warm A/B of when the previous output tree is deleted in a helm-openshift
step (``move2kube.py:_remove_output``), interleaved in one process:

* ``thread``   - renamed aside, deleted on a thread from the start (the default);
* ``sync``     - deleted before anything is written;
* ``join``     - the thread, joined before ``operator-sdk`` is spawned;
* ``overlap``  - renamed aside, deleted by the main thread while
  ``operator-sdk`` runs.

Per variant: median step time and the median time ``proc.spawn`` of
``operator-sdk`` takes (posix_spawn with vfork returns when the child has
exec'd; a tree being unlinked on another thread can slow that).  One JSON line.

    python benchmarks/remove_ab.py [--pairs 40]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
sys.path.insert(0, ROOT)
import refconfigs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=40)
    a = ap.parse_args()
    from move2kube_amd import move2kube as M
    from move2kube_amd import transformer as T
    from move2kube_amd.ops import native
    from move2kube_amd.utils import proc

    orig_remove, orig_start, orig_finish = M._remove_output, T.K8sTransformer.start_operator, \
        T.K8sTransformer.finish_operator
    orig_spawn = proc.spawn
    threads, trash, spawn_ms = [], [], []

    def spawn_timed(*args, **kw):
        t = time.perf_counter()
        try:
            return orig_spawn(*args, **kw)
        finally:
            spawn_ms.append((time.perf_counter() - t) * 1000)

    def remove_sync(outpath):
        native.remove_tree(outpath)

    def remove_keep(outpath):
        r = orig_remove(outpath)
        if r:
            threads.append(r[0])
        return r

    def remove_aside(outpath):
        parent, base = os.path.split(os.path.abspath(outpath))
        t = os.path.join(parent, ".%s.m2k-old-%d-ab" % (base, os.getpid()))
        os.rename(outpath, t)
        trash.append(t)

    def start_joined(project, basepath):
        while threads:
            threads.pop().join()
        return orig_start(project, basepath)

    def finish_after_delete(started):
        while trash:
            native.remove_tree(trash.pop())
        return orig_finish(started)

    variants = {
        "thread": (orig_remove, orig_start, orig_finish),
        "sync": (remove_sync, orig_start, orig_finish),
        "join": (remove_keep, start_joined, orig_finish),
        "overlap": (remove_aside, orig_start, finish_after_delete),
    }
    root, fs = refconfigs.workdir_root("auto")
    work = tempfile.mkdtemp(prefix="m2k-rmab-", dir=root)
    run = refconfigs.Run("helm-openshift", work).prepare()
    undo = run.apply_env()
    proc.spawn = spawn_timed
    steps = {k: [] for k in variants}
    spawns = {k: [] for k in variants}
    try:
        with run.session() as s:
            for _ in range(5):
                run.step(s)
            for i in range(a.pairs):
                order = list(variants) if i % 2 == 0 else list(reversed(list(variants)))
                for k in order:
                    M._remove_output = variants[k][0]
                    T.K8sTransformer.start_operator = staticmethod(variants[k][1])
                    T.K8sTransformer.finish_operator = staticmethod(variants[k][2])
                    run.step(s)   # leaves this variant's tree behind for the timed step
                    del spawn_ms[:]
                    t = time.perf_counter()
                    run.step(s)
                    steps[k].append((time.perf_counter() - t) * 1000)
                    spawns[k].append(sum(spawn_ms))
    finally:
        proc.spawn = orig_spawn
        M._remove_output = orig_remove
        T.K8sTransformer.start_operator, T.K8sTransformer.finish_operator = \
            staticmethod(orig_start), staticmethod(orig_finish)
        undo()
    print(json.dumps({"pairs": a.pairs, "workdir_fs": fs,
                      "step_p50_ms": {k: round(statistics.median(v), 3) for k, v in steps.items()},
                      "spawn_p50_ms": {k: round(statistics.median(v), 3) for k, v in spawns.items()}}), flush=True)


if __name__ == "__main__":
    main()
