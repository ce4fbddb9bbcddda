"""Numerics of the gfx950 batched edit-distance kernel vs the plain CPU
Wagner-Fischer reference (ins=1, del=1, sub=2)."""

import random

import pytest

from move2kube_amd.ops import editdistance, gpu

pytestmark = pytest.mark.gpu


def _rand_strings(rng, n, lo, hi, alphabet="abcdefghij_-0123"):
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


def test_gpu_library_loads():
    assert gpu.gpu_host(), "no /dev/kfd on a GPU test run"
    assert gpu.available(), "libm2k_ed_hip.so must load on the GPU box"
    assert gpu.device_arch().startswith("gfx950")


def test_ed_kernel_matches_cpu_small():
    rng = random.Random(1)
    opts = _rand_strings(rng, 300, 0, 40) + ["", "x" * 200]
    qs = _rand_strings(rng, 37, 0, 64) + ["", "y" * 64]
    got = gpu.ed_matrix(opts, qs)
    want = [[editdistance.wagner_fischer_py(o, q) for q in qs] for o in opts]
    assert got == want


def test_ed_kernel_matches_native_large():
    from move2kube_amd.ops import native
    rng = random.Random(7)
    opts = _rand_strings(rng, 4096, 1, 48, alphabet="abcdefghijklmnopqrstuvwxyz_")
    qs = _rand_strings(rng, 96, 1, 64, alphabet="abcdefghijklmnopqrstuvwxyz_")
    got = gpu.ed_matrix(opts, qs)
    m = native.module()
    assert m is not None
    flat = m.edit_distance_batch(opts, qs, 1, 1, 2, 8)
    want = [flat[i * len(qs):(i + 1) * len(qs)] for i in range(len(opts))]
    assert got == want


def test_dispatch_uses_gpu_for_large_batches(monkeypatch):
    calls = []
    real = gpu.ed_matrix

    def spy(o, q):
        calls.append((len(o), len(q)))
        return real(o, q)

    monkeypatch.setattr(gpu, "ed_matrix", spy)
    rng = random.Random(3)
    opts = _rand_strings(rng, 2048, 1, 30)
    qs = _rand_strings(rng, 64, 1, 30)
    m = editdistance.matrix(opts, qs)
    assert calls == [(2048, 64)]
    assert m[5][7] == editdistance.wagner_fischer_py(opts[5], qs[7])


def test_closest_matching_strings_gpu_batch():
    from move2kube_amd.utils import common
    opts = ["nodejs_buildpack", "java_buildpack", "python_buildpack", "go_buildpack", "ruby_buildpack"] * 1000
    names = ["node", "javaa", "pythn", "golang", "rubyy"] * 20
    got = common.get_closest_matching_strings(opts, names)
    want = [common.get_closest_matching_string(opts, n) for n in names]
    assert got == want
