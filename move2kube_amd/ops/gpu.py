"""ctypes binding for the MI355X batched fuzzy-matching kernel (``ed_kernel.hip``).

The HIP library is built in-tree for gfx950 (``libm2k_ed_hip.so``).  On a
machine that exposes an AMD GPU (``/dev/kfd``) a missing library is an error
(``GpuUnavailable``) rather than a silent CPU fallback; on CPU-only hosts the
callers use the native CPU path.
"""

import _thread
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libm2k_ed_hip.so")

_lib = None
_state = None  # None=untried, True=ok, False=unavailable
_lock = _thread.RLock()


class GpuUnavailable(RuntimeError):
    pass


class GpuUnsupportedInput(GpuUnavailable):
    """The kernel cannot take this input (query > 64 bytes, all 256 byte values used)."""


_RC_UNSUPPORTED = (-2, -8)


def gpu_host():
    """True on a host exposing an AMD GPU to this process."""
    if os.environ.get("M2K_FORCE_CPU"):
        return False
    return os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK)


def _load():
    if _state is not None:
        return _lib
    with _lock:   # one thread loads; the others wait for it
        return _load_locked()


def _load_locked():
    """Load the library (under ``_lock``).  ``_lib`` is set before ``_state``
    and ``_state`` only when the outcome is known, so the lock-free check in
    :func:`_load` never hands a thread a provisional None while another
    thread is still loading (the round-4 race of ``ops/native.py``)."""
    global _state
    if _state is not None:
        return _lib
    ok = False
    try:
        ok = _open_library()
    finally:
        _state = ok
    return _lib


def _open_library():
    global _lib
    if not os.path.exists(LIB_PATH):
        if gpu_host():
            raise GpuUnavailable("HIP library %s not built (run __graft_entry__.build())" % LIB_PATH)
        return False
    lib = ctypes.CDLL(LIB_PATH)
    i64p = ctypes.POINTER(ctypes.c_int64)
    i32p = ctypes.POINTER(ctypes.c_int32)
    for fn in (lib.m2k_ed_matrix, lib.m2k_ed_closest):
        fn.restype = ctypes.c_int
    lib.m2k_ed_matrix.argtypes = [ctypes.c_char_p, i64p, ctypes.c_int, ctypes.c_char_p, i64p, ctypes.c_int, i32p]
    lib.m2k_ed_closest.argtypes = [ctypes.c_char_p, i64p, ctypes.c_int, ctypes.c_char_p, i64p, ctypes.c_int, i32p,
                                   i32p]
    lib.m2k_ed_last_timings.restype = None
    lib.m2k_ed_last_timings.argtypes = [ctypes.POINTER(ctypes.c_double)]
    lib.m2k_gpu_device_count.restype = ctypes.c_int
    lib.m2k_gpu_arch.restype = ctypes.c_char_p
    _lib = lib
    return True


def available():
    try:
        lib = _load()
    except OSError:
        return False
    return lib is not None and lib.m2k_gpu_device_count() > 0


_warm = False


def warm():
    """A kernel call has completed in this process (HIP runtime initialised)."""
    return _warm


def last_timings():
    """{prep, h2d, kernel, d2h} milliseconds of the last ed_matrix/ed_closest call."""
    lib = _lib_or_raise()
    buf = (ctypes.c_double * 4)()
    lib.m2k_ed_last_timings(buf)
    return dict(zip(("prep_ms", "h2d_ms", "kernel_ms", "d2h_ms"), (round(x, 3) for x in buf)))


def device_arch():
    lib = _load()
    return lib.m2k_gpu_arch().decode() if lib is not None else ""


def _pack(strings):
    """(packed bytes, int64 offsets[n+1], max length)."""
    from . import native
    m = native.module()
    if m is not None and isinstance(strings, list):
        data, off, maxlen = m.pack_strings(strings)
        return data, off, int(maxlen)
    bs = [s.encode("utf-8", "surrogateescape") if isinstance(s, str) else bytes(s) for s in strings]
    lens = np.fromiter((len(b) for b in bs), dtype=np.int64, count=len(bs))
    off = np.zeros(len(bs) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return b"".join(bs), off, int(lens.max()) if len(bs) else 0


def _ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _lib_or_raise():
    lib = _load()
    if lib is None:
        raise GpuUnavailable("HIP library not available")
    return lib


def ed_matrix(options, queries):
    """Distance matrix, shape [len(options), len(queries)] (int32 numpy view of a
    query-major device result).  Every query must be <= 64 bytes."""
    lib = _lib_or_raise()
    na, nb = len(options), len(queries)
    if na == 0 or nb == 0:
        return np.zeros((na, nb), dtype=np.int32)
    a, offa, _ = _pack(options)
    q, offb, qmax = _pack(queries)
    if qmax > 64:
        raise GpuUnsupportedInput("queries longer than 64 bytes are not supported on the GPU path")
    outT = np.empty((nb, na), dtype=np.int32)
    rc = lib.m2k_ed_matrix(a, _ptr(offa, ctypes.c_int64), na, q, _ptr(offb, ctypes.c_int64), nb,
                           _ptr(outT, ctypes.c_int32))
    if rc in _RC_UNSUPPORTED:
        raise GpuUnsupportedInput("m2k_ed_matrix cannot take this input (code %d)" % rc)
    if rc != 0:
        raise GpuUnavailable("m2k_ed_matrix failed with code %d" % rc)
    global _warm
    _warm = True
    return outT.T


def ed_closest(options, queries):
    """(index, distance) int32 arrays: for every query the first option with the
    minimum distance (-1, -1 when there are no options)."""
    lib = _lib_or_raise()
    na, nb = len(options), len(queries)
    idx = np.full(nb, -1, dtype=np.int32)
    dist = np.full(nb, -1, dtype=np.int32)
    if nb == 0 or na == 0:
        return idx, dist
    a, offa, _ = _pack(options)
    q, offb, qmax = _pack(queries)
    if qmax > 64:
        raise GpuUnsupportedInput("queries longer than 64 bytes are not supported on the GPU path")
    rc = lib.m2k_ed_closest(a, _ptr(offa, ctypes.c_int64), na, q, _ptr(offb, ctypes.c_int64), nb,
                            _ptr(idx, ctypes.c_int32), _ptr(dist, ctypes.c_int32))
    if rc in _RC_UNSUPPORTED:
        raise GpuUnsupportedInput("m2k_ed_closest cannot take this input (code %d)" % rc)
    if rc != 0:
        raise GpuUnavailable("m2k_ed_closest failed with code %d" % rc)
    global _warm
    _warm = True
    return idx, dist
