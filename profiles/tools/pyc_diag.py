"""Which modules of a cold ``move2kube translate`` run from a stale or missing
bytecode cache on this host (their source is compiled again by every process
that cannot write the cache, e.g. a non-root user and a system Python).

usage: python scripts/pyc_diag.py [src_dir]   (prints one JSON line)
"""
import importlib.util
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pyc_state(mod):
    spec = getattr(mod, "__spec__", None)
    origin = getattr(spec, "origin", None) if spec else None
    if not origin or not origin.endswith(".py") or not os.path.isfile(origin):
        return None
    cached = importlib.util.cache_from_source(origin)
    try:
        with open(cached, "rb") as f:
            head = f.read(16)
    except OSError:
        return "missing"
    flags = struct.unpack("<I", head[4:8])[0]
    if flags & 1:
        return "hash-based"
    mtime, size = struct.unpack("<II", head[8:16])
    st = os.stat(origin)
    if mtime != (int(st.st_mtime) & 0xFFFFFFFF) or size != (st.st_size & 0xFFFFFFFF):
        return "stale"
    return "ok"


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "samples", "golang")
    t0 = time.perf_counter()
    from move2kube_amd.cli import main as climain
    import tempfile
    out = tempfile.mkdtemp(prefix="m2k-pycdiag-")
    climain.main(["translate", "-s", src, "-o", out, "--qaskip"])
    dt = time.perf_counter() - t0
    states = {}
    for name, mod in sorted(sys.modules.items()):
        s = pyc_state(mod)
        if s is not None:
            states.setdefault(s, []).append(name)
    print(json.dumps({"run_ms": round(dt * 1e3, 2), "uid": os.getuid(), "executable": sys.executable,
                      "pycache_prefix": sys.pycache_prefix,
                      "counts": {k: len(v) for k, v in states.items()},
                      "not_ok": {k: v for k, v in states.items() if k != "ok"}}))


if __name__ == "__main__":
    main()
