#!/usr/bin/env python3
"""Where a cold CLI command spends its time: ``--runs`` cold processes of a
BASELINE configuration's last command with ``M2K_TRACE`` on
(``utils/trace.py``), the median duration of every traced span, the process
wall time and its first span's start (the imports before the command runs).
One JSON line.

    python benchmarks/cold_trace.py helm-openshift [--runs 15]
"""
import argparse
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refconfigs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--runs", type=int, default=15)
    ap.add_argument("--tree", default=refconfigs.ROOT, help="the source tree to run (e.g. .ab_base/r04)")
    a = ap.parse_args()
    root, _ = refconfigs.workdir_root("auto")
    work = tempfile.mkdtemp(prefix="m2k-coldtrace-", dir=root)
    try:
        run = refconfigs.Run(a.config, work).prepare()
        env = run.env()
        env["PYTHONPATH"] = os.path.abspath(a.tree)
        cmds = run.cli_commands()
        spans, walls = {}, []
        for i in range(a.runs + 1):  # the first run primes the bytecode and page caches
            trace_file = os.path.join(work, "trace.json")
            for argv in cmds[:-1]:
                subprocess.run([sys.executable, "-m", "move2kube_amd"] + argv, env=env, cwd=work,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
            e = dict(env, M2K_TRACE=trace_file)
            t0 = time.perf_counter()
            subprocess.run([sys.executable, "-m", "move2kube_amd"] + cmds[-1], env=e, cwd=work,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
            wall = (time.perf_counter() - t0) * 1e3
            if i == 0:
                continue
            walls.append(wall)
            with open(trace_file) as f:
                ev = json.load(f)
            ev = ev["traceEvents"] if isinstance(ev, dict) else ev
            per = {}
            for x in ev:
                if x.get("ph") == "X":
                    per[x["name"]] = per.get(x["name"], 0.0) + x.get("dur", 0) / 1000.0
            for k, v in per.items():
                spans.setdefault(k, []).append(v)
        med = {k: round(statistics.median(v + [0.0] * (len(walls) - len(v))), 3) for k, v in spans.items()}
        top = dict(sorted(med.items(), key=lambda kv: -kv[1]))
        print(json.dumps({"config": a.config, "command": cmds[-1][0], "runs": len(walls),
                          "wall_p50_ms": round(statistics.median(walls), 3), "span_p50_ms": top}), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
