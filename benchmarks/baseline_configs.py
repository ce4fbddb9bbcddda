#!/usr/bin/env python3
"""Per-configuration wall clock for the five BASELINE.json configurations
(``benchmarks/refconfigs.py``), on the reference's own ``samples/`` corpus.

BASELINE.md ("Baseline this repo will measure", item 2) asks for the
``translate --qaskip`` time of each configuration as the p50 of 5 runs with
CNB disabled (the java-cnb and cf configurations probe CNB through a
``podman`` stand-in instead of a container engine).  For every configuration
this reports:

* ``warm_p50_ms`` / ``warm_iqr_ms`` - p50 and interquartile range of
  ``--runs`` in-process runs of the configuration's commands (assets
  unpacked once; nothing else reused between runs: fresh file index,
  detectors, QA engines, output directory);
* ``cold_p50_ms``  - p50 of ``--runs`` sets of complete CLI processes
  (``python -m move2kube_amd collect|translate ...``: interpreter start,
  imports, asset unpack, the command, cleanup) - what a user of the Go binary
  compares against; byte-compiled modules cached as in an installed package
  (``cold_iqr_ms`` / ``cold_over_floor_iqr_ms``: the interquartile ranges);
  ``cold_cpu_p50_ms`` is their CPU time and ``cold_over_floor_p50_ms`` the
  time above a bare ``python -c pass`` per process, paired run by run;
* ``cold_launcher_p50_ms`` / ``cold_launcher_over_floor_p50_ms`` - the same
  commands through the release archive's launcher (``python3 -S
  bin/m2k_main.py``, ``scripts/builddist.py``), and its time above a bare
  ``python -S -c pass``;
* ``python_emulation_of_reference_fork_model_p50_ms`` - p50 of in-process runs
  with every detector forked as ``/bin/sh`` one at a time on one worker, the
  way ``dockerfilecontainerizer.go:76-83`` runs them.  This is a Python
  emulation of the reference's execution model, not the Go tool (no Go
  toolchain here); it is reported for context only;
* ``samples_yamls_warm_p50_ms`` / ``helm_openshift_over_samples_yamls`` -
  the headline corpus translated with every default (Yamls, Kubernetes
  profile, no operator) and the headline configuration's warm p50 over it: the
  cost of the Helm chart, the Openshift group/versions and the operator-sdk
  run per service of the same corpus;
* ``manifest_diff_vs_ref`` - files differing from the reference-derived
  expected tree ``tests/golden/reference/<config>`` (0 = identical), checked
  on the first warm run, every emulation run and every cold run.

Usage: ``python benchmarks/baseline_configs.py [--runs 5] [--json out.json]``.
Host CPU only; no GPU is involved.
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
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import refconfigs  # noqa: E402


def _p50(xs):
    return round(statistics.median(xs), 3)


def _iqr(xs):
    """Interquartile range (q75 - q25, linear interpolation); 0 for one run."""
    if len(xs) < 2:
        return 0.0
    q = statistics.quantiles(xs, n=4, method="inclusive")
    return round(q[2] - q[0], 3)


def warm_runs(name, runs, emulation_runs=0):
    """In-process timings of one configuration; returns a result dict."""
    from move2kube_amd.utils import log
    from move2kube_amd.utils.constants import settings
    log.set_quiet()
    work = tempfile.mkdtemp(prefix="m2k-cfgbench-")
    run = refconfigs.Run(name, work).prepare()
    undo = run.apply_env()
    res = {"config": name}
    try:
        with run.session() as s:
            out = run.step(s)
            res["manifest_diff_vs_ref"] = refconfigs.manifest_diff_vs_ref(name, out)
            times = []
            for _ in range(runs):
                t0 = time.perf_counter()
                run.step(s)
                times.append((time.perf_counter() - t0) * 1e3)
            res["warm_p50_ms"] = _p50(times)
            res["warm_iqr_ms"] = _iqr(times)
            res["warm_min_ms"] = round(min(times), 3)
            if emulation_runs > 0:
                saved = (os.environ.get("M2K_NATIVE_DETECT"), settings.workers)
                os.environ["M2K_NATIVE_DETECT"] = "0"
                settings.workers = 1
                try:
                    times = []
                    for _ in range(emulation_runs):
                        t0 = time.perf_counter()
                        out = run.step(s)
                        times.append((time.perf_counter() - t0) * 1e3)
                    res["python_emulation_of_reference_fork_model_p50_ms"] = _p50(times)
                    res["manifest_diff_vs_ref"] += refconfigs.manifest_diff_vs_ref(name, out) or 0
                finally:
                    if saved[0] is None:
                        os.environ.pop("M2K_NATIVE_DETECT", None)
                    else:
                        os.environ["M2K_NATIVE_DETECT"] = saved[0]
                    settings.workers = saved[1]
    finally:
        undo()
        shutil.rmtree(work, ignore_errors=True)
    return res


def _children_cpu_ms():
    import resource
    r = resource.getrusage(resource.RUSAGE_CHILDREN)
    return (r.ru_utime + r.ru_stime) * 1e3


def cold_stats(name, runs):
    """``runs`` sets of CLI processes (plus one untimed priming run), each
    preceded by a bare interpreter start in the same environment, so a noisy
    host shows up in both.  Returns p50 wall and CPU (user+sys of the child
    processes, stand-in tools included) of the sets, p50 of the per-pair
    difference to the bare interpreter, and the total manifest diff."""
    work = tempfile.mkdtemp(prefix="m2k-cfgcold-")
    try:
        run = refconfigs.Run(name, work).prepare()
        # Bytecode goes to a private PYTHONPYCACHEPREFIX primed by the untimed
        # run - the state of an installed package (pip / scripts/install.sh
        # byte-compile at install time).
        extra = {"PYTHONPYCACHEPREFIX": os.path.join(work, "pycache")}
        env = run.env()
        env.update(extra)
        launcher = refconfigs.release_launcher(work)
        walls, cpus, over, diff = [], [], [], 0
        lwalls, lover = [], []
        ncmd = len(run.cli_commands())
        for i in range(-1, runs):
            t0 = time.perf_counter()
            subprocess.run([sys.executable, "-c", "pass"], env=env)
            floor = (time.perf_counter() - t0) * 1e3
            c0 = _children_cpu_ms()
            t0 = time.perf_counter()
            out = run.run_cli(extra_env=extra)
            wall = (time.perf_counter() - t0) * 1e3
            if i >= 0:
                walls.append(wall)
                cpus.append(_children_cpu_ms() - c0)
                over.append(wall - floor * ncmd)
            diff += refconfigs.manifest_diff_vs_ref(name, out) or 0
            t0 = time.perf_counter()
            subprocess.run([sys.executable, "-S", "-c", "pass"], env=env)
            floor = (time.perf_counter() - t0) * 1e3
            t0 = time.perf_counter()
            out = run.run_cli(extra_env=extra, launcher=launcher)
            wall = (time.perf_counter() - t0) * 1e3
            if i >= 0:
                lwalls.append(wall)
                lover.append(wall - floor * ncmd)
            diff += refconfigs.manifest_diff_vs_ref(name, out) or 0
        return {"cold_p50_ms": _p50(walls), "cold_iqr_ms": _iqr(walls), "cold_cpu_p50_ms": _p50(cpus),
                "cold_over_floor_p50_ms": _p50(over), "cold_over_floor_iqr_ms": _iqr(over),
                "cold_launcher_p50_ms": _p50(lwalls), "cold_launcher_over_floor_p50_ms": _p50(lover),
                "manifest_diff_vs_ref": diff}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def cold_runs(name, runs):
    """(cold stats without the diff, total manifest diff vs ref) - see :func:`cold_stats`."""
    st = cold_stats(name, runs)
    return st, st.pop("manifest_diff_vs_ref")


def bench_config(name, runs, emulation_runs):
    res = warm_runs(name, runs, emulation_runs)
    cold = cold_stats(name, runs)
    res["manifest_diff_vs_ref"] += cold.pop("manifest_diff_vs_ref")
    res.update(cold)
    return res


def interpreter_floor(runs, flags=()):
    """p50 of a bare ``python -c pass`` (the cold-run floor no Python CLI can beat)."""
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        subprocess.run([sys.executable] + list(flags) + ["-c", "pass"])
        times.append((time.perf_counter() - t0) * 1e3)
    return _p50(times)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--emulation-runs", type=int, default=3,
                    help="runs of the Python emulation of the reference's fork-per-detector model (0 = skip)")
    ap.add_argument("--configs", default=",".join(refconfigs.CONFIGS))
    ap.add_argument("--json", default=None, help="also write the results here")
    ap.add_argument("--workdir", default="auto",
                    help="root for inputs and outputs: auto (tmpfs if available), disk, or a path (see bench.py)")
    args = ap.parse_args()
    root, workdir_fs = refconfigs.workdir_root(args.workdir)
    if root is not None:
        tempfile.tempdir = root
    results = {"runs": args.runs, "workdir_fs": workdir_fs, "python_floor_ms": interpreter_floor(args.runs),
               "python_floor_nosite_ms": interpreter_floor(args.runs, ["-S"]), "configs": []}
    # the headline corpus with default answers (Yamls, Kubernetes): what the
    # Helm + Openshift + operator output of the same 15 services costs on top
    yamls = warm_runs("samples-yamls", args.runs)
    results["samples_yamls_warm_p50_ms"] = yamls["warm_p50_ms"]
    for name in args.configs.split(","):
        r = bench_config(name, args.runs, args.emulation_runs)
        results["configs"].append(r)
        print(json.dumps(r), flush=True)
    ho = [r for r in results["configs"] if r["config"] == refconfigs.HEADLINE]
    if ho and yamls["warm_p50_ms"]:
        results["helm_openshift_over_samples_yamls"] = round(ho[0]["warm_p50_ms"] / yamls["warm_p50_ms"], 3)
    print(json.dumps({k: v for k, v in results.items() if k != "configs"}), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)
    return 0 if all(r["manifest_diff_vs_ref"] == 0 for r in results["configs"]) else 1


if __name__ == "__main__":
    sys.exit(main())
