"""cProfile of warm in-process steps of one BASELINE configuration.

usage: python scripts/profile_step.py [config=helm-openshift] [sort=tottime] [steps=20]
"""
import cProfile
import os
import pstats
import shutil
import sys
import tempfile
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

import refconfigs  # noqa: E402
from move2kube_amd.utils import log  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else refconfigs.HEADLINE
    sort = sys.argv[2] if len(sys.argv) > 2 else "tottime"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    log.set_quiet()
    work = tempfile.mkdtemp(prefix="m2k-prof-")
    run = refconfigs.Run(name, work).prepare()
    undo = run.apply_env()
    try:
        with run.session() as s:
            for _ in range(5):
                run.step(s)
            times = []
            for _ in range(steps):
                t0 = time.perf_counter()
                run.step(s)
                times.append((time.perf_counter() - t0) * 1e3)
            times.sort()
            print("%s: p50 %.3f ms, min %.3f ms over %d steps" % (name, times[len(times) // 2], times[0], steps))
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(steps):
                run.step(s)
            pr.disable()
            pstats.Stats(pr).sort_stats(sort).print_stats(45)
    finally:
        undo()
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
