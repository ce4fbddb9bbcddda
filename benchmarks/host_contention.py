#!/usr/bin/env python3
"""How much CPU a fixed piece of work costs each of N concurrent processes on
this host, N = 1, 2, 4, 8 - the control experiment for the weak-scaling
rehearsal (``scripts/scale_rehearsal.sh``), where CPU per rank-step grows with
the rank count.  No move2kube code runs here, so what grows here is the host:

* ``cpu``   - pure-Python work (dict/str/JSON churn, like the translate
  step's own Python): user CPU per iteration;
* ``fs``    - the output tree's file churn on the tmpfs the bench uses:
  create a tree of 200 files of 2 KiB in 20 directories, then delete it (the
  headline step writes and removes about 170 files plus the operator's copy
  of the chart): system CPU per iteration;
* ``spawn`` - start and reap ``/bin/sh -c :`` through the same native
  ``posix_spawnp`` runner the CLI uses for ``operator-sdk`` (one per step).

Every process runs each phase for the same number of iterations, all
processes start together (a shared barrier file), and each reports user and
system CPU and wall time per iteration from ``getrusage``.  One JSON line per
N: the per-process means and their ratio to N=1.

    python benchmarks/host_contention.py [--ranks 1,2,4,8] [--iters 200]
"""

import argparse
import json
import os
import resource
import shutil
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _usage():
    a, b = resource.getrusage(resource.RUSAGE_SELF), resource.getrusage(resource.RUSAGE_CHILDREN)
    return a.ru_utime + b.ru_utime, a.ru_stime + b.ru_stime, time.perf_counter()


def _delta(t0, t1, n):
    return {"user_ms": round((t1[0] - t0[0]) * 1e3 / n, 4), "sys_ms": round((t1[1] - t0[1]) * 1e3 / n, 4),
            "wall_ms": round((t1[2] - t0[2]) * 1e3 / n, 4)}


def _cpu_work():
    d = {}
    for i in range(400):
        k = "svc-%d" % i
        d[k] = {"name": k, "ports": [i, i + 1], "labels": {"app": k.upper()}}
    s = json.dumps(d, sort_keys=True)
    back = json.loads(s)
    return sum(len(v["name"]) for v in back.values()) + len(s.replace("svc", "SVC").split(","))


def _fs_work(root, blob):
    d = os.path.join(root, "tree")
    os.mkdir(d)
    for i in range(20):
        sub = os.path.join(d, "d%d" % i)
        os.mkdir(sub)
        for j in range(10):
            with open(os.path.join(sub, "f%d.yaml" % j), "wb") as f:
                f.write(blob)
    shutil.rmtree(d)


def worker(gate, root, iters):
    sys.path.insert(0, ROOT)
    from move2kube_amd.utils import proc
    blob = b"x" * 2048
    while not os.path.exists(gate):   # every process starts together
        time.sleep(0.0005)
    out = {}
    t0 = _usage()
    for _ in range(iters):
        _cpu_work()
    out["cpu"] = _delta(t0, _usage(), iters)
    t0 = _usage()
    for _ in range(iters):
        _fs_work(root, blob)
    out["fs"] = _delta(t0, _usage(), iters)
    n = max(1, iters // 4)
    t0 = _usage()
    for _ in range(n):
        proc.run(["/bin/sh", "-c", ":"], stdout=proc.DEVNULL)
    out["spawn"] = _delta(t0, _usage(), n)
    print(json.dumps(out), flush=True)


def run_n(n, iters, base):
    tmp = tempfile.mkdtemp(prefix="m2k-contention-", dir=base)
    gate = os.path.join(tmp, "go")
    try:
        procs = []
        for r in range(n):
            root = os.path.join(tmp, "r%d" % r)
            os.mkdir(root)
            procs.append(subprocess.Popen([sys.executable, __file__, "--worker", gate, root, str(iters)],
                                          stdout=subprocess.PIPE))
        time.sleep(0.3)   # let every interpreter start before the gate opens
        open(gate, "w").close()
        rows = []
        for p in procs:
            out, _ = p.communicate(timeout=600)
            if p.returncode != 0:
                raise RuntimeError("worker failed")
            rows.append(json.loads(out.decode().strip().splitlines()[-1]))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    mean = {}
    for phase in ("cpu", "fs", "spawn"):
        mean[phase] = {k: round(sum(r[phase][k] for r in rows) / len(rows), 4) for k in ("user_ms", "sys_ms",
                                                                                          "wall_ms")}
    return mean


def main(argv=None):
    if argv is None:
        argv = sys.argv[1:]
    if argv and argv[0] == "--worker":
        worker(argv[1], argv[2], int(argv[3]))
        return 0
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--workdir", default="/dev/shm" if os.access("/dev/shm", os.W_OK) else None)
    a = ap.parse_args(argv)
    first = None
    for n in [int(x) for x in a.ranks.split(",")]:
        m = run_n(n, a.iters, a.workdir)
        if first is None:
            first = m
        ratio = {ph: {k: round(m[ph][k] / first[ph][k], 3) if first[ph][k] else None for k in m[ph]}
                 for ph in m}
        print(json.dumps({"n": n, "iters": a.iters, "per_process": m, "ratio_to_first": ratio}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
