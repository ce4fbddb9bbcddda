"""Interleaved cold-start A/B of one configuration's translate command: the
release launcher (``python -S bin/m2k_main.py``) and ``python -m
move2kube_amd``, each with and without the bytecode bundle
(``M2K_BYTECODE_BUNDLE=0``), next to the two bare-interpreter floors.  Prints
one JSON line of p25/p50 per variant (ms).

    python scripts/cold_ab.py golang [--runs 31]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--runs", type=int, default=31)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="m2k-coldab-")
    run = refconfigs.Run(a.config, work).prepare()
    env = run.env()
    env["PYTHONPATH"] = ROOT
    launcher = refconfigs.release_launcher(work)
    argv = run.cli_commands()[-1]
    nob = dict(env, M2K_BYTECODE_BUNDLE="0")
    variants = {
        "launcher": (launcher + argv, env),
        "launcher_nobundle": (launcher + argv, nob),
        "module": ([sys.executable, "-m", "move2kube_amd"] + argv, env),
        "module_nobundle": ([sys.executable, "-m", "move2kube_amd"] + argv, nob),
        "floor_nosite": ([sys.executable, "-S", "-c", "pass"], env),
        "floor_site": ([sys.executable, "-c", "pass"], env),
    }
    times = {k: [] for k in variants}
    for i in range(a.runs + 2):
        for k, (cmd, e) in variants.items():
            t0 = time.perf_counter()
            p = subprocess.run(cmd, env=e, cwd=work, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            dt = (time.perf_counter() - t0) * 1e3
            if p.returncode != 0:
                raise SystemExit("%s failed: %s" % (k, p.stderr.decode(errors="replace")[-1000:]))
            if i >= 2:  # two warm-up rounds (pyc writes, page cache)
                times[k].append(dt)
    out = {"config": a.config, "runs": a.runs}
    for k, v in times.items():
        v.sort()
        out[k] = {"p25": round(v[len(v) // 4], 2), "p50": round(v[len(v) // 2], 2)}
    for k in ("launcher", "launcher_nobundle"):
        out[k]["over_floor_p50"] = round(out[k]["p50"] - out["floor_nosite"]["p50"], 2)
    for k in ("module", "module_nobundle"):
        out[k]["over_floor_p50"] = round(out[k]["p50"] - out["floor_site"]["p50"], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
