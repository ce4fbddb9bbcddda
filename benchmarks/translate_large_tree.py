#!/usr/bin/env python3
"""``translate`` on large synthetic source trees: per-service cost vs tree size.

The tree generator is ``plan_large_tree.make_tree`` (nodejs / python / golang /
java / ruby / php / Dockerfile / compose apps).  For each ``--apps`` value the
whole command runs in-process (plan + curate with defaults + translate +
write), after one untimed warm-up on a small tree so imports and the assets
unpack are not charged to the first size; each size is timed ``--repeat``
times on a fresh copy of its tree and the fastest run is kept.  Trees live on
a tmpfs when one is writable (``refconfigs.workdir_root``: on the GPU hosts'
scratch disks the 42k-file trees of an earlier step slow later writes).
Prints one JSON line with the
per-service milliseconds at every size and the ratio largest/smallest, which
is 1.0 for a linear pipeline (VERDICT r2 asks for <= 1.5 at 2000 vs 100 apps).
"""

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
os.environ.setdefault("M2K_NO_NETWORK", "1")
os.environ.setdefault("M2K_DISABLE_CNB", "1")

import plan_large_tree  # noqa: E402


def run_once(work, apps, depth, files, profile=None):
    from move2kube_amd import api
    src = os.path.join(work, "src-%d" % apps)
    out = os.path.join(work, "out-%d" % apps)
    plan_large_tree.make_tree(src, apps, depth, files)
    with api.Session(qaskip=True) as s:
        if profile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        s.translate(src, out, name="bigtree")
        dt = time.perf_counter() - t0
        if profile:
            prof.disable()
            prof.dump_stats(profile)
        n = len(s.plan(src, "bigtree").services)
    shutil.rmtree(src, ignore_errors=True)
    shutil.rmtree(out, ignore_errors=True)
    return dt, n


def measure(sizes, depth=2, files=3, workdir=None, profile_largest=None, repeat=3):
    if workdir is None:
        import refconfigs
        workdir = refconfigs.workdir_root("auto")[0]
    work = tempfile.mkdtemp(prefix="m2k-bigtranslate-", dir=workdir)
    try:
        run_once(work, 16, depth, files)          # warm-up: imports, assets
        rows = []
        for i, apps in enumerate(sizes):
            prof = profile_largest if (profile_largest and i == len(sizes) - 1) else None
            runs = [run_once(work, apps, depth, files, prof if r == 0 else None) for r in range(max(1, repeat))]
            dt, n = min(runs)
            rows.append({"apps": apps, "services": n, "translate_s": round(dt, 3),
                         "ms_per_service": round(1000.0 * dt / max(n, 1), 3),
                         "runs_s": [round(r[0], 3) for r in runs]})
        return rows
    finally:
        shutil.rmtree(work, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--apps", default="100,400,1000,2000", help="comma-separated tree sizes")
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--files", type=int, default=3)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--profile", default=None, help="write a cProfile of the largest size here")
    ap.add_argument("--repeat", type=int, default=3, help="timed runs per size; the fastest is kept")
    args = ap.parse_args()
    sizes = [int(x) for x in args.apps.split(",")]
    rows = measure(sizes, args.depth, args.files, args.workdir, args.profile, args.repeat)
    ratio = rows[-1]["ms_per_service"] / rows[0]["ms_per_service"]
    print(json.dumps({"metric": "large_tree_translate_ms_per_service", "depth": args.depth, "files": args.files,
                      "sizes": rows, "ratio_largest_vs_smallest": round(ratio, 3)}))


if __name__ == "__main__":
    main()
