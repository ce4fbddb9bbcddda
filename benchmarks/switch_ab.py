"""Interleaved cold-CLI A/B of one environment switch (e.g. M2K_STARTCACHE):
PAIRS pairs of `python -m move2kube_amd <the configuration's last command>`
with the switch at OFF and ON, alternating which goes first; prints the
median of each side and the median of the paired differences (off - on).

    python benchmarks/switch_ab.py M2K_STARTCACHE 0 1 helm-openshift,golang --pairs 60
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("var")
    ap.add_argument("off")
    ap.add_argument("on")
    ap.add_argument("configs")
    ap.add_argument("--pairs", type=int, default=40)
    a = ap.parse_args()
    root, _ = refconfigs.workdir_root("auto")
    for cfg in a.configs.split(","):
        work = tempfile.mkdtemp(prefix="m2k-swab-", dir=root)
        run = refconfigs.Run(cfg, work).prepare()
        env = run.env()
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        argv = [sys.executable, "-m", "move2kube_amd"] + run.cli_commands()[-1]
        res = {a.off: [], a.on: []}
        for i in range(a.pairs + 1):
            for v in ((a.off, a.on) if i % 2 else (a.on, a.off)):
                t = time.perf_counter()
                subprocess.run(argv, env=dict(env, **{a.var: v}), cwd=work, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL, check=True)
                if i:  # the first pair primes the caches
                    res[v].append((time.perf_counter() - t) * 1e3)
        diffs = [x - y for x, y in zip(res[a.off], res[a.on])]
        print(json.dumps({"config": cfg, "var": a.var, "pairs": a.pairs,
                          "median_ms": {k: round(statistics.median(v), 3) for k, v in res.items()},
                          "paired_diff_off_minus_on_median_ms": round(statistics.median(diffs), 3)}), flush=True)


if __name__ == "__main__":
    main()
