"""Numerics of the gfx950 batched edit-distance kernels vs the plain CPU
Wagner-Fischer reference (ins=1, del=1, sub=2)."""

import os
import random

import numpy as np
import pytest

from move2kube_amd.ops import editdistance, gpu, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _rand_strings(rng, n, lo, hi, alphabet="abcdefghij_-0123"):
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def _ref_matrix(opts, qs):
    return np.array([[editdistance.wagner_fischer_py(o, q) for q in qs] for o in opts], dtype=np.int32)


def test_gpu_library_loads():
    assert gpu.gpu_host(), "no /dev/kfd on a GPU test run"
    assert gpu.available(), "libm2k_ed_hip.so must load on the GPU box"
    assert gpu.device_arch().startswith("gfx950")


def test_ed_matrix_matches_cpu_small():
    rng = random.Random(1)
    opts = _rand_strings(rng, 300, 0, 40) + ["", "x" * 200]
    qs = _rand_strings(rng, 37, 0, 64) + ["", "y" * 64]
    got = gpu.ed_matrix(opts, qs)
    assert got.shape == (len(opts), len(qs))
    assert np.array_equal(got, _ref_matrix(opts, qs))


def test_ed_matrix_matches_native_large():
    rng = random.Random(7)
    opts = _rand_strings(rng, 4096 + 77, 1, 48, alphabet="abcdefghijklmnopqrstuvwxyz_")
    qs = _rand_strings(rng, 96, 1, 64, alphabet="abcdefghijklmnopqrstuvwxyz_")
    got = gpu.ed_matrix(opts, qs)
    want = native.module().edit_distance_batch(opts, qs, 1, 1, 2, 8)
    assert np.array_equal(got, want)


def test_ed_closest_matches_cpu_with_ties():
    rng = random.Random(11)
    # few distinct option strings -> many exact ties; the first index must win
    base = _rand_strings(rng, 40, 1, 20, alphabet="abcd")
    opts = [base[rng.randrange(len(base))] for _ in range(5000)]
    qs = _rand_strings(rng, 300, 0, 64, alphabet="abcd")
    gi, gd = gpu.ed_closest(opts, qs)
    ci, cd = native.module().closest_batch(opts, qs, 8)
    assert np.array_equal(gd, cd)
    assert np.array_equal(gi, ci)
    for j in (0, 17, 299):
        row = [editdistance.wagner_fischer_py(o, qs[j]) for o in opts]
        assert gd[j] == min(row) and gi[j] == row.index(min(row))


def test_ed_closest_many_query_slabs():
    # more than 65535 queries exercises the gridDim.y slabbing
    rng = random.Random(5)
    opts = _rand_strings(rng, 64, 1, 12)
    qs = _rand_strings(rng, 70000, 0, 10)
    gi, gd = gpu.ed_closest(opts, qs)
    ci, cd = native.module().closest_batch(opts, qs, 8)
    assert np.array_equal(gi, ci) and np.array_equal(gd, cd)


def test_dispatch_uses_gpu_for_large_batches(monkeypatch):
    gpu.ed_closest(["warm"], ["up"])  # a warm runtime uses the small-batch threshold
    assert editdistance._gpu_warm()
    calls = []
    real = gpu.ed_closest

    def spy(o, q):
        calls.append((len(o), len(q)))
        return real(o, q)

    monkeypatch.setattr(gpu, "ed_closest", spy)
    rng = random.Random(3)
    opts = _rand_strings(rng, 2048, 1, 30)
    qs = _rand_strings(rng, 64, 1, 30)
    idx, dist = editdistance.closest_indices(opts, qs)
    assert calls == [(2048, 64)]
    row = [editdistance.wagner_fischer_py(o, qs[7]) for o in opts]
    assert dist[7] == min(row) and idx[7] == row.index(min(row))


def test_closest_matching_strings_gpu_batch():
    from move2kube_amd.utils import common
    opts = ["nodejs_buildpack", "java_buildpack", "python_buildpack", "go_buildpack", "ruby_buildpack"] * 1000
    names = ["node", "javaa", "pythn", "golang", "rubyy"] * 20
    got = common.get_closest_matching_strings(opts, names)
    want = [editdistance.closest(opts, n) for n in names]
    assert got == [opts[0], opts[1], opts[2], opts[3], opts[4]] * 20
    assert got == want


def test_all_byte_values_fall_back_to_cpu():
    # every byte value in use leaves no code for padding: the kernel refuses and
    # the dispatcher answers on the CPU
    base = [bytes(range(i, min(256, i + 32))) for i in range(0, 256, 32)]
    opts = base * 3000
    qs = [bytes([1, 2, 3]), bytes([250, 251])] * 20
    with pytest.raises(gpu.GpuUnsupportedInput):
        gpu.ed_closest(opts, qs)
    idx, dist = editdistance.closest_indices(opts, qs)
    for j in (0, 1):
        row = [editdistance.wagner_fischer_py(o, qs[j]) for o in base]
        assert dist[j] == min(row) and idx[j] == row.index(min(row))


def test_uneven_lengths_and_padding_slots():
    # nA not a multiple of the 512-option panel, lengths spanning many 16-byte blocks
    rng = random.Random(9)
    opts = _rand_strings(rng, 1537, 0, 200, alphabet="ab")
    qs = _rand_strings(rng, 33, 0, 64, alphabet="abc")
    assert np.array_equal(gpu.ed_matrix(opts, qs), _ref_matrix(opts, qs))
    gi, gd = gpu.ed_closest(opts, qs)
    ci, cd = native.module().closest_batch(opts, qs, 8)
    assert np.array_equal(gi, ci) and np.array_equal(gd, cd)


def test_tile_classes_boundaries_and_wide_alphabet():
    """Query lengths at every tile-class edge (8 x 16-bit, 4 x 32-bit, 2 x 64-bit
    per workgroup) with partially filled tiles, on a > 63-symbol alphabet (the
    unscaled-code kernels) and on a small one (scaled codes)."""
    rng = random.Random(21)
    for alphabet in ("".join(chr(c) for c in range(32, 127)), "acgt"):
        opts = _rand_strings(rng, 1100, 0, 70, alphabet=alphabet)
        qs = []
        for n in (0, 1, 15, 16, 17, 31, 32, 33, 63, 64):
            qs += _rand_strings(rng, 3, n, n, alphabet=alphabet)
        rng.shuffle(qs)
        assert np.array_equal(gpu.ed_matrix(opts, qs), _ref_matrix(opts, qs))
        gi, gd = gpu.ed_closest(opts, qs)
        ci, cd = native.module().closest_batch(opts, qs, 8)
        assert np.array_equal(gi, ci) and np.array_equal(gd, cd)


def test_cold_process_keeps_small_batches_on_cpu():
    """In a fresh process the first HIP call costs ~280 ms: a batch above the
    warm threshold but far below the cold one stays on the CPU."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from move2kube_amd.ops import editdistance, gpu\n"
            "calls = []\n"
            "real = gpu.ed_closest\n"
            "gpu.ed_closest = lambda o, q: calls.append(1) or real(o, q)\n"
            "opts = ['buildpack-%%d' %% i for i in range(4000)]\n"
            "editdistance.closest_indices(opts, ['node', 'java', 'go'] * 10)\n"
            "print(len(calls), gpu.warm())\n") % (ROOT,)
    p = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True, timeout=300)
    assert p.stdout.split() == ["0", "False"]

