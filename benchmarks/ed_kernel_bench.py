#!/usr/bin/env python3
"""Micro-benchmark of the batched fuzzy-matching path: gfx950 kernel vs the
native multi-threaded CPU implementation, on a synthetic "CF foundation"
(N app/buildpack names x M builder buildpack ids).  Prints one JSON line."""

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from move2kube_amd.ops import gpu, native  # noqa: E402


def words(rng, n, lo, hi):
    alpha = "abcdefghijklmnopqrstuvwxyz_-0123456789"
    return ["".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--options", type=int, default=200000)
    ap.add_argument("--queries", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu", action="store_true", help="also time the native CPU path")
    ap.add_argument("--qmax", type=int, default=64, help="longest query (buildpack names are mostly <= 32)")
    a = ap.parse_args()
    rng = random.Random(0)
    opts = words(rng, a.options, 4, 40)
    qs = words(rng, a.queries, 4, a.qmax)
    res = {"options": a.options, "queries": a.queries, "qmax": a.qmax, "pairs": a.options * a.queries}
    cells = sum(len(o) for o in opts) * a.queries  # option bytes x queries = bit-parallel steps
    if gpu.available():
        gpu.ed_closest(opts[:1024], qs[:8])  # warm-up / context creation
        for name, fn in (("closest", gpu.ed_closest), ("matrix", gpu.ed_matrix)):
            t = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                r = fn(opts, qs)
                t.append(time.perf_counter() - t0)
            res["gpu_%s_s" % name] = min(t)
            res["gpu_%s_breakdown" % name] = gpu.last_timings()
            res["gpu_%s_gsteps_per_s" % name] = cells / min(t) / 1e9
        res["arch"] = gpu.device_arch()
        gi, gd = gpu.ed_closest(opts, qs)
    if a.cpu and native.available():
        th = min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        ci, cd = native.module().closest_batch(opts, qs, th)
        res["cpu_native_closest_s"] = time.perf_counter() - t0
        res["cpu_threads"] = th
        if gpu.available():
            res["gpu_cpu_agree"] = bool((gi == ci).all() and (gd == cd).all())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
