#!/usr/bin/env python3
"""GPU vs native-CPU crossover for the closest-match dispatcher
(``ops/editdistance.py``): times both paths over a range of batch sizes and
prints one JSON line per size, plus the smallest size where the GPU wins."""

import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from move2kube_amd.ops import editdistance, gpu, native  # noqa: E402


def words(rng, n, lo, hi):
    alpha = "abcdefghijklmnopqrstuvwxyz_-0123456789"
    return ["".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def best(fn, reps=5):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


COLD = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
from move2kube_amd.ops import gpu
t0 = time.perf_counter()
gpu.ed_closest(["nodejs_buildpack", "java_buildpack"], ["node"])
t1 = time.perf_counter()
gpu.ed_closest(["nodejs_buildpack", "java_buildpack"], ["node"])
t2 = time.perf_counter()
print("%.3f %.3f" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3))
"""


def cold_start_ms():
    """First GPU call in a fresh process (HIP runtime + code object load) vs the second."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", COLD, root], stdout=subprocess.PIPE, text=True, timeout=300)
    first, second = (float(x) for x in p.stdout.split())
    return first, second


def main():
    first, second = cold_start_ms()
    print(json.dumps({"cold_first_call_ms": round(first, 3), "warm_second_call_ms": round(second, 3)}), flush=True)
    rng = random.Random(0)
    m = native.module()
    th = editdistance._threads()
    crossover = None
    gpu.ed_closest(words(rng, 1024, 4, 40), words(rng, 8, 4, 20))  # context + arena warm-up
    for n_opts, n_q in ((20, 8), (50, 16), (100, 16), (200, 32), (500, 32), (1000, 64), (2000, 64), (5000, 64), (10000, 128), (20000, 256),
                        (50000, 512), (100000, 1024)):
        opts, qs = words(rng, n_opts, 4, 40), words(rng, n_q, 4, 24)
        c = best(lambda: m.closest_batch(opts, qs, th))
        g = best(lambda: gpu.ed_closest(opts, qs))
        pairs = n_opts * n_q
        if crossover is None and g < c:
            crossover = pairs
        print(json.dumps({"options": n_opts, "queries": n_q, "pairs": pairs, "cpu_ms": round(c * 1e3, 3),
                          "gpu_ms": round(g * 1e3, 3), "cpu_threads": th}), flush=True)
    print(json.dumps({"crossover_pairs": crossover}), flush=True)


if __name__ == "__main__":
    main()
