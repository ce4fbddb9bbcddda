"""Where a cold CLI process spends its time: per run, the interpreter start
until the entry script runs, the import of ``move2kube_amd.cli.main``, the
first ``main()`` (with the time of the imports it triggers) and a second and
third ``main()`` in the same process (warm).  Median over N processes, one
JSON line.

    python scripts/cold_phases.py golang [--runs 15]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402

CHILD = r'''
import time
t_entry = time.perf_counter()
import builtins, os, sys
sys.path.insert(0, ROOT)
n0 = len(sys.modules)
from move2kube_amd.cli.main import main
t_imported = time.perf_counter()
n1 = len(sys.modules)
import shutil
orig = builtins.__import__
depth = [0]
acc = [0.0]
def imp(name, *a, **k):
    depth[0] += 1
    t = time.perf_counter()
    try:
        return orig(name, *a, **k)
    finally:
        depth[0] -= 1
        if depth[0] == 0:
            acc[0] += time.perf_counter() - t
def run(argv):
    shutil.rmtree(OUT, ignore_errors=True)
    # a CLI process starts its QA engines once (package globals, as in the
    # reference); drop the previous run's before the next main()
    eng = sys.modules.get("move2kube_amd.qaengine.engine")
    if eng is not None:
        eng.reset()
    t = time.perf_counter()
    try:
        main(argv)
    except SystemExit:
        pass
    return (time.perf_counter() - t) * 1e3
builtins.__import__ = imp
first = run(ARGV)
builtins.__import__ = orig
n2 = len(sys.modules)
second = run(ARGV)
third = run(ARGV)
import json  # not before: its system pyc is stale on the MI355X image
with open(RESULT, "a") as f:
    f.write(json.dumps({"start_to_entry": (t_entry - T0) * 1e3, "import_cli": (t_imported - t_entry) * 1e3,
                        "first_main": first, "first_main_imports": acc[0] * 1e3, "second_main": second,
                        "third_main": third, "modules": [n0, n1, n2]}) + "\n")
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--runs", type=int, default=15)
    ap.add_argument("--command", type=int, default=-1,
                    help="which of the configuration's CLI commands to time (cf: 0 = collect, 1 = translate)")
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="m2k-phases-")
    run = refconfigs.Run(a.config, work).prepare()
    env = run.env()
    argv = run.cli_commands()[a.command]
    result = os.path.join(work, "phases.jsonl")
    child = os.path.join(work, "child.py")
    import time
    for i in range(a.runs + 1):  # the first run warms the pyc files and page cache
        with open(child, "w") as f:
            f.write("import sys\nT0 = float(sys.argv[1])\nROOT = %r\nARGV = %r\nOUT = %r\nRESULT = %r\n" % (
                ROOT, argv, run.outdir, result if i else os.devnull) + CHILD)
        # T0: the parent's clock just before the spawn (perf_counter is
        # CLOCK_MONOTONIC, the same clock in every process)
        subprocess.run([sys.executable, "-S", child, repr(time.perf_counter())], env=env, cwd=work,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
    rows = [json.loads(line) for line in open(result)]
    out = {"config": a.config, "command": argv[0], "runs": len(rows)}
    for k in rows[0]:
        if k == "modules":
            out[k] = rows[0][k]
            continue
        v = sorted(r[k] for r in rows)
        out[k] = round(v[len(v) // 2], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
