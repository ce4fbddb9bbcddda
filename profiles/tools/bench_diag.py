"""bench.py with per-step timings printed per rank (stderr) and optional
switches for contention diagnosis: M2K_DIAG_NO_OPERATOR=1 skips operator-sdk."""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "benchmarks"))
import refconfigs  # noqa: E402
import bench  # noqa: E402

times = []
_step = refconfigs.Run.step


def step(self, session):
    t = time.perf_counter()
    try:
        return _step(self, session)
    finally:
        times.append((time.perf_counter() - t) * 1e3)


refconfigs.Run.step = step
if os.environ.get("M2K_DIAG_NO_OPERATOR") == "1":
    from move2kube_amd.transformer import K8sTransformer
    K8sTransformer.start_operator = staticmethod(lambda project, basepath: None)
try:
    bench.main()
finally:
    s = sorted(times)
    if s:
        print("rank %s steps %d p50 %.1f p90 %.1f max %.1f min %.1f" % (
            os.environ.get("RANK", "0"), len(s), s[len(s) // 2], s[int(len(s) * 0.9)], s[-1], s[0]), file=sys.stderr)
