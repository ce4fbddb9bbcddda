"""cProfile of one cold CLI process of a BASELINE configuration (after an
untimed priming run, bytecode cached): import time, total time and the
profile of ``main()``.

usage: python scripts/cold_profile.py [config=golang] [sort=cumulative]
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

import refconfigs  # noqa: E402

_CHILD = """
import cProfile, pstats, time, sys
t0 = time.perf_counter()
from move2kube_amd.cli import main
t1 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
try:
    main.main(%r)
except SystemExit:
    pass
pr.disable()
print("import ms %%.2f, total ms %%.2f" %% ((t1 - t0) * 1e3, (time.perf_counter() - t0) * 1e3))
pstats.Stats(pr).sort_stats(%r).print_stats(50)
"""


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "golang"
    sort = sys.argv[2] if len(sys.argv) > 2 else "cumulative"
    work = tempfile.mkdtemp(prefix="m2k-coldprof-")
    try:
        run = refconfigs.Run(name, work).prepare()
        extra = {"PYTHONPYCACHEPREFIX": os.path.join(work, "pycache")}
        run.run_cli(extra_env=extra)  # primes the bytecode cache; collect output for cf
        env = run.env()
        env.update(extra)
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        argv = run.cli_commands()[-1]
        p = subprocess.run([sys.executable, "-c", _CHILD % (argv, sort)], env=env, cwd=work,
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
        sys.stdout.write(p.stdout.decode())
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
