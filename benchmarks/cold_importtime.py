#!/usr/bin/env python3
"""``python -X importtime`` of one cold CLI command of a BASELINE
configuration (its last command), after an untimed priming run: every module
imported after ``site``, self and cumulative microseconds, median of
``--runs`` processes, largest self time first.  One JSON line.

    python benchmarks/cold_importtime.py helm-openshift [--runs 9] [--tree .ab_base/r04]
"""
import argparse
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refconfigs  # noqa: E402


def one(env, work, argv):
    p = subprocess.run([sys.executable, "-X", "importtime", "-m", "move2kube_amd"] + argv, env=env, cwd=work,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, check=True)
    lines = [ln for ln in p.stderr.splitlines() if ln.startswith("import time:")]
    site = max(i for i, ln in enumerate(lines) if ln.rstrip().endswith("| site"))
    out = {}
    for ln in lines[site + 1:]:
        parts = ln[len("import time:"):].split("|")
        try:
            out[parts[2].strip()] = (int(parts[0]), int(parts[1]))
        except ValueError:
            continue
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--runs", type=int, default=9)
    ap.add_argument("--tree", default=refconfigs.ROOT, help="the source tree to import (e.g. .ab_base/r04)")
    a = ap.parse_args()
    root, _ = refconfigs.workdir_root("auto")
    work = tempfile.mkdtemp(prefix="m2k-imptime-", dir=root)
    try:
        run = refconfigs.Run(a.config, work).prepare()
        env = run.env()
        env["PYTHONPATH"] = os.path.abspath(a.tree)
        argv = run.cli_commands()[-1]
        for argv0 in run.cli_commands()[:-1]:  # e.g. cf's collect, so translate sees its output
            subprocess.run([sys.executable, "-m", "move2kube_amd"] + argv0, env=env, cwd=work,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
        one(env, work, argv)
        runs = [one(env, work, argv) for _ in range(a.runs)]
        names = set().union(*runs)
        med = {n: (statistics.median(r.get(n, (0, 0))[0] for r in runs),
                   statistics.median(r.get(n, (0, 0))[1] for r in runs)) for n in names}
        ours = sum(v[0] for n, v in med.items() if n.startswith("move2kube_amd"))
        other = sum(v[0] for n, v in med.items() if not n.startswith("move2kube_amd"))
        top = sorted(med.items(), key=lambda kv: -kv[1][0])
        print(json.dumps({"config": a.config, "command": argv[0], "runs": a.runs,
                          "self_us_ours": ours, "self_us_stdlib_after_site": other, "modules": len(med),
                          "self_cum_us": {n: [int(s), int(c)] for n, (s, c) in top}}), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
