#!/usr/bin/env python3
"""Interleaved same-box A/B of the headline ``bench.py`` between two trees.

A headline shift between two driver records can be box noise (another host,
another disk, another neighbour) or a code change; only runs of both trees on
one box, alternated so drift hits both alike, tell them apart.  ``--base`` is
a checkout of the older tree (``git archive <rev> | tar -x -C DIR``; its
native libraries may be copied from this tree when the sources agree), the
current tree is ``--head`` (default: this repository).

Each pair runs both trees once, in alternating order, as separate processes:
``bench.py --steps S --warmup W --check-runs 0 --large-tree ""``.  Prints one
JSON line per run and a summary line: per tree the ms/step of every run, the
median, and ``head_over_base`` (median ratio; < 1 means the head is faster).

``--cold CONFIGS`` compares cold CLI starts instead: each pair runs
``benchmarks/baseline_configs.py --configs CONFIGS`` in both trees and records
per configuration ``cold_over_floor_p50_ms`` (CLI processes minus a bare
interpreter started next to them); the summary has the median per tree.
"""

import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def run_bench(tree, steps, warmup, timeout):
    cmd = [sys.executable, "-u", "bench.py", "--steps", str(steps), "--warmup", str(warmup),
           "--check-runs", "0", "--large-tree", ""]
    p = subprocess.run(cmd, cwd=tree, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout)
    line = [x for x in p.stdout.decode().splitlines() if x.startswith("{")]
    if p.returncode != 0 or not line:
        raise RuntimeError("bench.py in %s failed (%d): %s" % (tree, p.returncode, p.stderr.decode()[-2000:]))
    return json.loads(line[-1])


def run_cold(tree, configs, runs, timeout):
    cmd = [sys.executable, "-u", os.path.join("benchmarks", "baseline_configs.py"), "--runs", str(runs),
           "--emulation-runs", "0", "--configs", configs]
    p = subprocess.run(cmd, cwd=tree, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout)
    rows = [json.loads(x) for x in p.stdout.decode().splitlines() if x.startswith("{")]
    rows = [r for r in rows if "config" in r]
    if p.returncode != 0 or not rows:
        raise RuntimeError("baseline_configs.py in %s failed (%d): %s" % (tree, p.returncode,
                                                                          p.stderr.decode()[-2000:]))
    return {r["config"]: r["cold_over_floor_p50_ms"] for r in rows}


def main_cold(args, trees):
    per = {"base": {}, "head": {}}
    out = open(args.out, "a") if args.out else None
    try:
        for i in range(args.pairs):
            order = ("base", "head") if i % 2 == 0 else ("head", "base")
            for label in order:
                d = run_cold(trees[label], args.cold, args.runs, args.timeout)
                for k, v in d.items():
                    per[label].setdefault(k, []).append(v)
                line = json.dumps({"pair": i, "tree": label, "cold_over_floor_p50_ms": d})
                print(line, flush=True)
                if out:
                    out.write(line + "\n")
                    out.flush()
        med = {t: {k: statistics.median(v) for k, v in per[t].items()} for t in per}
        line = json.dumps({"summary": True, "cold_over_floor_p50_ms": per, "median_ms": med})
        print(line, flush=True)
        if out:
            out.write(line + "\n")
    finally:
        if out:
            out.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", required=True, help="checkout of the older tree")
    ap.add_argument("--head", default=ROOT)
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=240, help="seconds per bench.py run")
    ap.add_argument("--out", default=None, help="also append the JSON lines to this file")
    ap.add_argument("--cold", default="", help="configurations whose cold CLI start to compare instead")
    ap.add_argument("--runs", type=int, default=9, help="cold runs per configuration and tree per pair")
    args = ap.parse_args()
    trees = {"base": os.path.abspath(args.base), "head": os.path.abspath(args.head)}
    if args.cold:
        return main_cold(args, trees)
    ms = {"base": [], "head": []}
    out = open(args.out, "a") if args.out else None
    try:
        for i in range(args.pairs):
            order = ("base", "head") if i % 2 == 0 else ("head", "base")
            for label in order:
                d = run_bench(trees[label], args.steps, args.warmup, args.timeout)
                ms[label].append(d["ms_per_step"])
                rec = {"pair": i, "tree": label, "ms_per_step": d["ms_per_step"], "value": d["value"],
                       "step_ms": d.get("step_ms"), "manifest_diff_vs_ref": d.get("manifest_diff_vs_ref"),
                       "workdir_fs": d.get("workdir_fs")}
                line = json.dumps(rec)
                print(line, flush=True)
                if out:
                    out.write(line + "\n")
                    out.flush()
        med = {k: statistics.median(v) for k, v in ms.items()}
        summary = {"summary": True, "ms_per_step": ms, "median_ms": med,
                   "head_over_base": round(med["head"] / med["base"], 3) if med["base"] else None}
        line = json.dumps(summary)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
    finally:
        if out:
            out.close()


if __name__ == "__main__":
    main()
