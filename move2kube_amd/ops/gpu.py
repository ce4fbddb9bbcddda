"""ctypes binding for the MI355X batched fuzzy-matching kernel (``ed_kernel.hip``).

The HIP library is built in-tree for gfx950 (``libm2k_ed_hip.so``).  On a
machine that exposes an AMD GPU (``/dev/kfd``) a missing library is an error
(``GpuUnavailable``) rather than a silent CPU fallback; on CPU-only hosts the
callers use the native CPU path.
"""

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libm2k_ed_hip.so")

_lib = None
_state = None  # None=untried, True=ok, False=unavailable


class GpuUnavailable(RuntimeError):
    pass


def gpu_host():
    """True on a host exposing an AMD GPU to this process."""
    if os.environ.get("M2K_FORCE_CPU"):
        return False
    return os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK)


def _load():
    global _lib, _state
    if _state is not None:
        return _lib
    _state = False
    if not os.path.exists(LIB_PATH):
        if gpu_host():
            raise GpuUnavailable("HIP library %s not built (run __graft_entry__.build())" % LIB_PATH)
        return None
    lib = ctypes.CDLL(LIB_PATH)
    lib.m2k_ed_batch.restype = ctypes.c_int
    lib.m2k_ed_batch.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                 ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_int)]
    lib.m2k_gpu_device_count.restype = ctypes.c_int
    lib.m2k_gpu_arch.restype = ctypes.c_char_p
    _lib = lib
    _state = True
    return _lib


def available():
    try:
        lib = _load()
    except OSError:
        return False
    return lib is not None and lib.m2k_gpu_device_count() > 0


def device_arch():
    lib = _load()
    return lib.m2k_gpu_arch().decode() if lib is not None else ""


def ed_matrix(options, queries):
    """Distance matrix [len(options)][len(queries)] computed on the GPU.

    Every query must be <= 64 bytes.  Raises GpuUnavailable on failure."""
    lib = _load()
    if lib is None:
        raise GpuUnavailable("HIP library not available")
    ob = [o.encode() if isinstance(o, str) else o for o in options]
    qb = [q.encode() if isinstance(q, str) else q for q in queries]
    na, nb = len(ob), len(qb)
    if na == 0 or nb == 0:
        return [[0] * nb for _ in range(na)]
    lena = (ctypes.c_int * na)(*[len(o) for o in ob])
    lenb = (ctypes.c_int * nb)(*[len(q) for q in qb])
    out = (ctypes.c_int * (na * nb))()
    rc = lib.m2k_ed_batch(b"".join(ob), lena, na, b"".join(qb), lenb, nb, out)
    if rc != 0:
        raise GpuUnavailable("m2k_ed_batch failed with code %d" % rc)
    flat = list(out)
    return [flat[i * nb:(i + 1) * nb] for i in range(na)]
