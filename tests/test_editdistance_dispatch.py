"""The edit-distance dispatcher on the CPU (``ops/editdistance.py``; the GPU
paths themselves run in ``tests/test_gpu_kernels.py`` on the MI355X): when it
sends work to the GPU, falling back to the CPU for input the kernel does not
take, and the pure-Python twin when the native extension is absent (the
reference's ``smetrics.WagnerFischer(a, b, 1, 1, 2)``)."""

import sys

import pytest

from move2kube_amd.ops import editdistance as ed
from move2kube_amd.ops import native

OPTS = ["nodejs_buildpack", "java_buildpack", "go_buildpack", "python_buildpack"]
QS = ["nodejs", "golang", "ruby", ""]


def _want():
    return [[ed.wagner_fischer_py(o, q) for q in QS] for o in OPTS]


@pytest.fixture
def no_native(monkeypatch):
    monkeypatch.setattr(native, "module", lambda: None)


def test_pure_python_twin(no_native):
    assert ed.matrix(OPTS, QS).tolist() == _want()
    idx, dist = ed.closest_indices(OPTS, QS)
    for j in range(len(QS)):
        col = [row[j] for row in _want()]
        assert dist[j] == min(col) and idx[j] == col.index(min(col))
    assert ed.closest_index_list(OPTS, QS) == (list(idx), list(dist))
    assert ed.closest(OPTS, "golang") == "go_buildpack"
    assert ed.distances(OPTS, "go") == [ed.wagner_fischer_py(o, "go") for o in OPTS]


def test_empty_inputs():
    assert ed.closest_indices([], ["a"])[0].tolist() == [-1]
    assert ed.closest_index_list([], ["a", "b"]) == ([-1, -1], [-1, -1])
    assert ed.closest([], "a") == "" and ed.distances([], "a") == []


class _FakeGpu:
    """Stands in for ``ops/gpu.py`` to observe the dispatch decisions."""

    class GpuUnavailable(RuntimeError):
        pass

    class GpuUnsupportedInput(GpuUnavailable):
        pass

    def __init__(self, host=True, warm=False, unsupported=False):
        self.host, self._warm, self.unsupported, self.calls = host, warm, unsupported, []

    def gpu_host(self):
        return self.host

    def warm(self):
        return self._warm

    def ed_matrix(self, options, queries):
        self.calls.append("matrix")
        if self.unsupported:
            raise self.GpuUnsupportedInput("no")
        import numpy
        return numpy.zeros((len(options), len(queries)), dtype=numpy.int32)

    def ed_closest(self, options, queries):
        self.calls.append("closest")
        if self.unsupported:
            raise self.GpuUnsupportedInput("no")
        import numpy
        return numpy.zeros(len(queries), dtype=numpy.int32), numpy.zeros(len(queries), dtype=numpy.int32)


@pytest.fixture
def fake_gpu(monkeypatch):
    def make(**kw):
        g = _FakeGpu(**kw)
        monkeypatch.setattr(ed, "_gpu", lambda: g)
        monkeypatch.setitem(sys.modules, "move2kube_amd.ops.gpu", g)
        return g
    return make


def test_auto_stays_on_the_cpu_below_the_thresholds(fake_gpu, monkeypatch):
    g = fake_gpu(host=True, warm=False)
    monkeypatch.setattr(ed, "GPU_MIN_PAIRS", 4)
    monkeypatch.setattr(ed, "GPU_MIN_PAIRS_COLD", 10 ** 9)
    assert ed.matrix(OPTS, QS).tolist() == _want()            # 16 pairs: over the warm threshold, not the cold one
    assert g.calls == []
    g._warm = True                                            # HIP already up in this process
    assert ed.matrix(OPTS, QS).tolist() == [[0] * 4] * 4 and g.calls == ["matrix"]
    g.host = False
    assert ed.matrix(OPTS, QS).tolist() == _want() and g.calls == ["matrix"]


def test_auto_goes_to_the_gpu_above_the_cold_threshold(fake_gpu, monkeypatch):
    g = fake_gpu(host=True)
    monkeypatch.setattr(ed, "GPU_MIN_PAIRS", 4)
    monkeypatch.setattr(ed, "GPU_MIN_PAIRS_COLD", 16)
    assert ed.closest_index_list(OPTS, QS) == ([0] * 4, [0] * 4) and g.calls == ["closest"]
    assert ed.matrix(OPTS, QS + ["x" * 65]).tolist() != []    # a query the kernel cannot take: CPU
    assert g.calls == ["closest"]


def test_forced_gpu(fake_gpu):
    g = fake_gpu(host=True)
    assert ed.matrix(OPTS, QS, device="gpu").tolist() == [[0] * 4] * 4
    with pytest.raises(g.GpuUnavailable, match="longer than 64 bytes"):
        ed.matrix(OPTS, ["y" * 65], device="gpu")
    g.unsupported = True
    with pytest.raises(g.GpuUnsupportedInput):
        ed.closest_indices(OPTS, QS, device="gpu")
    assert ed.matrix(OPTS, QS, device="cpu").tolist() == _want()


def test_unsupported_input_on_auto_falls_back_to_the_cpu(fake_gpu, monkeypatch):
    g = fake_gpu(host=True, warm=True, unsupported=True)
    monkeypatch.setattr(ed, "GPU_MIN_PAIRS", 1)
    assert ed.matrix(OPTS, QS).tolist() == _want()
    idx, dist = ed.closest_indices(OPTS, QS)
    assert g.calls == ["matrix", "closest"] and list(dist) == [min(r[j] for r in _want()) for j in range(4)]


def test_gpu_warm_through_torch(monkeypatch):
    class _Cuda:
        @staticmethod
        def is_initialized():
            return True

    class _Torch:
        cuda = _Cuda()
    monkeypatch.delitem(sys.modules, "move2kube_amd.ops.gpu", raising=False)
    monkeypatch.setitem(sys.modules, "torch", _Torch())
    assert ed._gpu_warm() is True
    _Cuda.is_initialized = staticmethod(lambda: (_ for _ in ()).throw(RuntimeError("no driver")))
    assert ed._gpu_warm() is False
