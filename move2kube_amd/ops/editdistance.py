"""Weighted edit distance (smetrics.WagnerFischer(a, b, 1, 1, 2)) with dispatch.

Small problems (the common case: a handful of options) run on the CPU; large
all-pairs batches (CF foundation exports: thousands of app buildpack names x
builder buildpack lists) are offloaded to the MI355X kernel in
``ed_kernel.hip`` when a GPU is present.
"""

import os
import sys

from . import native

# numpy and the HIP wrapper (which needs numpy) are imported on first use:
# importing numpy costs more than the handful of matches a CLI run makes
# (``closest_index_list``).


def _np():
    import numpy
    return numpy


def _gpu():
    from . import gpu
    return gpu

# Crossover measured on MI355X (profiles/r01_ed_crossover.log): once the HIP
# runtime is up, the GPU wins from ~8k pairs (0.09 ms vs 0.09-0.22 ms on 16
# threads); the first HIP call of a process costs ~280 ms, which the CPU path
# only exceeds around 10^8 pairs.
GPU_MIN_PAIRS = int(os.environ.get("M2K_GPU_MIN_PAIRS", "8192"))
GPU_MIN_PAIRS_COLD = int(os.environ.get("M2K_GPU_MIN_PAIRS_COLD", "100000000"))


def _gpu_warm():
    """True when this process already paid the HIP start-up (our library ran,
    or torch initialised the device)."""
    if "move2kube_amd.ops.gpu" in sys.modules and _gpu().warm():
        return True
    torch = sys.modules.get("torch")
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:  # noqa: BLE001
        return False


def wagner_fischer_py(a, b, icost=1, dcost=1, scost=2):
    if isinstance(a, str):
        a = a.encode("utf-8", "surrogateescape")
    if isinstance(b, str):
        b = b.encode("utf-8", "surrogateescape")
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


def _use_gpu(pairs, device, queries):
    if device == "cpu":
        return False
    if device != "gpu" and pairs < GPU_MIN_PAIRS:
        return False
    gpu = _gpu()
    fits = all(len(q.encode("utf-8", "surrogateescape") if isinstance(q, str) else q) <= 64 for q in queries)
    if device == "gpu":
        if not fits:
            raise gpu.GpuUnavailable("queries longer than 64 bytes are not supported on the GPU path")
        return True
    if not fits or pairs < GPU_MIN_PAIRS or not gpu.gpu_host():
        return False
    return pairs >= GPU_MIN_PAIRS_COLD or _gpu_warm()


def _threads():
    from ..utils.constants import host_threads
    return host_threads(16)


def matrix(options, queries, device="auto"):
    """Distance matrix, int32 array of shape [len(options), len(queries)].

    device: "auto" | "cpu" | "gpu"."""
    na, nb = len(options), len(queries)
    if _use_gpu(na * nb, device, queries):
        gpu = _gpu()
        try:
            return gpu.ed_matrix(options, queries)
        except gpu.GpuUnsupportedInput:
            if device == "gpu":
                raise
    m = native.module()
    if m is not None:
        return m.edit_distance_batch(list(options), list(queries), 1, 1, 2, _threads())
    np = _np()
    return np.array([[wagner_fischer_py(o, q) for q in queries] for o in options], dtype=np.int32).reshape(na, nb)


def closest_indices(options, queries, device="auto"):
    """For every query the index of the first option with the minimum distance
    and that distance (int32 arrays; -1 when there are no options).  The argmin
    is fused into the distance computation (GPU kernel or native CPU)."""
    na, nb = len(options), len(queries)
    np = _np()
    if na == 0 or nb == 0:
        return np.full(nb, -1, dtype=np.int32), np.full(nb, -1, dtype=np.int32)
    if _use_gpu(na * nb, device, queries):
        gpu = _gpu()
        try:
            return gpu.ed_closest(options, queries)
        except gpu.GpuUnsupportedInput:
            if device == "gpu":
                raise
    m = native.module()
    if m is not None:
        return m.closest_batch(list(options), list(queries), _threads())
    idx, dist = _closest_py(options, queries)
    return np.array(idx, dtype=np.int32), np.array(dist, dtype=np.int32)


def _closest_py(options, queries):
    idx, dist = [], []
    for q in queries:
        bi, bd = -1, -1
        for i, o in enumerate(options):
            d = wagner_fischer_py(o, q)
            if bi < 0 or d < bd:
                bi, bd = i, d
        idx.append(bi)
        dist.append(bd)
    return idx, dist


def closest_index_list(options, queries, device="auto"):
    """:func:`closest_indices` as two Python lists.  Below the GPU threshold
    this path never imports numpy (the native ``closest_list``)."""
    na, nb = len(options), len(queries)
    if na == 0 or nb == 0:
        return [-1] * nb, [-1] * nb
    if _use_gpu(na * nb, device, queries):
        idx, dist = closest_indices(options, queries, device)
        return [int(i) for i in idx], [int(d) for d in dist]
    m = native.module()
    if m is not None:
        return m.closest_list(list(options), list(queries), _threads())
    return _closest_py(options, queries)


def distances(options, search):
    """Distances of each option to one search string."""
    return [int(x) for x in matrix(options, [search])[:, 0]] if options else []


def closest(options, search):
    if not options:
        return ""
    idx, _ = closest_index_list(options, [search])
    return options[idx[0]]
