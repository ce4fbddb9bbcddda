"""Weighted edit distance (smetrics.WagnerFischer(a, b, 1, 1, 2)) with dispatch.

Small problems (the common case: a handful of options) run on the CPU; large
all-pairs batches (CF foundation exports: thousands of app buildpack names x
builder buildpack lists) are offloaded to the MI355X kernel in
``ed_kernel.hip`` when a GPU is present.
"""

import os

from . import gpu, native

GPU_MIN_PAIRS = int(os.environ.get("M2K_GPU_MIN_PAIRS", "65536"))


def wagner_fischer_py(a, b, icost=1, dcost=1, scost=2):
    if isinstance(a, str):
        a = a.encode()
    if isinstance(b, str):
        b = b.encode()
    row1 = [j * icost for j in range(len(b) + 1)]
    for i in range(1, len(a) + 1):
        row2 = [i * dcost] + [0] * len(b)
        ai = a[i - 1]
        for j in range(1, len(b) + 1):
            if ai == b[j - 1]:
                row2[j] = row1[j - 1]
            else:
                ins = row2[j - 1] + icost
                dele = row1[j] + dcost
                sub = row1[j - 1] + scost
                if ins < dele and ins < sub:
                    row2[j] = ins
                elif dele < sub:
                    row2[j] = dele
                else:
                    row2[j] = sub
        row1 = row2
    return row1[len(b)]


def matrix(options, queries, device="auto"):
    """Distance matrix [len(options)][len(queries)].

    device: "auto" | "cpu" | "gpu"."""
    na, nb = len(options), len(queries)
    use_gpu = device == "gpu" or (
        device == "auto" and na * nb >= GPU_MIN_PAIRS and gpu.gpu_host())
    if use_gpu and all(len(q.encode() if isinstance(q, str) else q) <= 64 for q in queries):
        return gpu.ed_matrix(options, queries)
    if use_gpu and device == "gpu":
        raise gpu.GpuUnavailable("queries longer than 64 bytes are not supported on the GPU path")
    m = native.module()
    if m is not None:
        flat = m.edit_distance_batch(list(options), list(queries), 1, 1, 2, 8)
        return [flat[i * nb:(i + 1) * nb] for i in range(na)]
    return [[wagner_fischer_py(o, q) for q in queries] for o in options]


def distances(options, search):
    """Distances of each option to one search string."""
    return [row[0] for row in matrix(options, [search])] if options else []


def closest(options, search):
    best, best_d = "", 2 ** 31 - 1
    for o, d in zip(options, distances(options, search)):
        if d < best_d:
            best, best_d = o, d
    return best
