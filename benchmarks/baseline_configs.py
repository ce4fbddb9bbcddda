#!/usr/bin/env python3
"""Per-configuration wall clock for the five BASELINE.json configurations.

BASELINE.md ("Baseline this repo will measure", item 2) asks for the
``translate --qaskip`` time of each configuration as the p50 of 5 runs with
CNB disabled.  For every configuration this script reports:

* ``warm_p50_ms``  - p50 of ``--runs`` in-process translates (assets unpacked
  once, nothing else reused between runs: fresh file index, detectors, QA
  engines, output directory);
* ``cold_p50_ms``  - p50 of ``--runs`` complete CLI processes
  (``python -m move2kube_amd translate ...``: interpreter start, imports,
  asset unpack, translate, cleanup) - what a user of the Go binary compares
  against; byte-compiled modules cached as in an installed package;
* ``refmodel_p50_ms`` - p50 of in-process runs in the reference's execution
  model (every detector forked as ``/bin/sh`` one at a time, one worker),
  a same-machine proxy for the Go tool's fork-dominated cost;
* ``manifest_diff`` - files differing from ``tests/golden/configs/<name>``
  (0 = identical), checked on the first warm run and on every cold run.

Configurations (same set-up as ``tests/test_baseline_configs.py``):
golang, compose, java-cnb (CNB builder detect stubbed as in the reference's
own any2kube tests), cf (``collect -a cf`` through the stub ``cf`` CLI, then
translate) and helm-openshift (whole samples tree, Openshift profile, answers
replayed from a QA cache, stub ``operator-sdk``).

Usage: ``python benchmarks/baseline_configs.py [--runs 5] [--json out.json]``.
The script runs on the host CPU only; no GPU is involved.
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SAMPLES = os.path.join(ROOT, "samples")
GOLDEN = os.path.join(ROOT, "tests", "golden", "configs")
FIXTURES = os.path.join(ROOT, "tests", "fixtures")
STUBBIN = os.path.join(FIXTURES, "stubbin")

os.environ["M2K_NO_NETWORK"] = "1"
os.environ["M2K_DISABLE_CNB"] = "1"

BUILDER_BUILDPACKS = {
    "cloudfoundry/cnb:cflinuxfs3": ["org.cloudfoundry.nodejs", "org.cloudfoundry.python",
                                    "org.cloudfoundry.go", "org.cloudfoundry.staticfile"],
    "gcr.io/buildpacks/builder": ["google.nodejs.runtime", "google.python.runtime", "google.go.runtime"],
}

# name -> (sample dirs copied under a root with a ".m2kignore" of ".", source
#          subdir translated (None = the root), project name, QA cache fixture,
#          root directory name - as in the tests, since copysources.sh embeds
#          the source path relative to the output directory)
CONFIGS = {
    "golang": (["golang"], "golang", "golang", None, "src"),
    "compose": (["compose"], "compose", "compose", None, "src"),
    "java-cnb": (["java-maven", "java-gradle"], None, "java", "cnb-qacache.yaml", "java"),
    "cf": (["cfapp"], None, "cf", None, "cf"),
    "helm-openshift": (None, None, "samples", "helm-openshift-qacache.yaml", "samples"),
}


def _patch(name):
    """Stand-ins for the external tools each configuration talks to; returns
    a function that undoes them (configurations run one after another in the
    same process)."""
    from move2kube_amd.containerizer.cnb import providers
    saved = (os.environ.get("PATH", ""), providers.is_builder_supported, providers.get_all_buildpacks)

    def restore():
        os.environ["PATH"] = saved[0]
        providers.is_builder_supported, providers.get_all_buildpacks = saved[1], saved[2]
        providers.reset_providers()

    os.environ["PATH"] = STUBBIN + os.pathsep + saved[0]
    if name == "java-cnb":
        providers.is_builder_supported = lambda path, builder: any(
            os.path.isfile(os.path.join(path, m)) for m in ("pom.xml", "build.gradle"))
    elif name == "cf":
        providers.get_all_buildpacks = lambda builders: dict(BUILDER_BUILDPACKS)
    return restore


def prepare(name, work):
    """Copy the configuration's sources into ``work``; returns (src, project, caches)."""
    dirs, sub, project, cache, rootname = CONFIGS[name]
    root = os.path.join(work, rootname)
    if dirs is None:
        shutil.copytree(SAMPLES, root, symlinks=True)
    else:
        os.makedirs(root)
        with open(os.path.join(root, ".m2kignore"), "w") as f:
            f.write(".\n")
        for d in dirs:
            shutil.copytree(os.path.join(SAMPLES, d), os.path.join(root, d), symlinks=True)
    caches = [os.path.join(FIXTURES, "configs", cache)] if cache else []
    if name == "cf":
        from move2kube_amd.cli import main as cli_main
        collected = os.path.join(work, "collect")
        rc = cli_main.main(["collect", "-a", "cf", "-s", root, "-o", collected])
        if rc != 0:
            raise RuntimeError("collect failed")
        shutil.copytree(os.path.join(collected, "m2k_collect"), os.path.join(root, "m2k_collect"))
    src = os.path.join(root, sub) if sub else root
    return src, project, caches


def manifest_diff(out, name):
    import bench
    return bench.manifest_diff(out, os.path.join(GOLDEN, name))


def child(name, src, project, out, caches):
    """One cold CLI process (``--child``): stubs, then ``translate`` via the CLI."""
    _patch(name)
    from move2kube_amd.cli import main as cli_main
    argv = ["translate", "-s", src, "-o", out, "-n", project, "--qaskip"]
    for c in caches:
        argv += ["-q", c]
    return cli_main.main(argv)


def bench_config(name, runs, refmodel_runs):
    from move2kube_amd import api
    from move2kube_amd.utils import log
    from move2kube_amd.utils.constants import settings
    log.set_quiet()
    restore = _patch(name)
    work = tempfile.mkdtemp(prefix="m2k-cfgbench-")
    try:
        src, project, caches = prepare(name, work)
        res = {"config": name}
        with api.Session(qaskip=True, qacaches=caches) as s:
            outdir = os.path.join(work, "out")
            out = s.translate(src, outdir, name=project)
            res["manifest_diff"] = manifest_diff(out, name)
            times = []
            for _ in range(runs):
                t0 = time.perf_counter()
                s.translate(src, outdir, name=project)
                times.append((time.perf_counter() - t0) * 1e3)
            res["warm_p50_ms"] = round(statistics.median(times), 3)
            res["warm_min_ms"] = round(min(times), 3)
            if refmodel_runs > 0:
                saved = (os.environ.get("M2K_NATIVE_DETECT"), settings.workers)
                os.environ["M2K_NATIVE_DETECT"] = "0"
                settings.workers = 1
                try:
                    times = []
                    for _ in range(refmodel_runs):
                        t0 = time.perf_counter()
                        out = s.translate(src, outdir, name=project)
                        times.append((time.perf_counter() - t0) * 1e3)
                    res["refmodel_p50_ms"] = round(statistics.median(times), 3)
                    res["manifest_diff"] += manifest_diff(out, name)
                finally:
                    if saved[0] is None:
                        os.environ.pop("M2K_NATIVE_DETECT", None)
                    else:
                        os.environ["M2K_NATIVE_DETECT"] = saved[0]
                    settings.workers = saved[1]
        # cold CLI processes.  Bytecode goes to a private PYTHONPYCACHEPREFIX,
        # primed by one untimed run - the state of an installed package
        # (pip / scripts/install.sh byte-compile at install time); without it
        # every run of a read-only checkout recompiles ~140 modules (~75 ms).
        env = dict(os.environ, PYTHONPYCACHEPREFIX=os.path.join(work, "pycache"))
        times = []
        for i in range(-1, runs):
            out = os.path.join(work, "cold%d" % i)
            cmd = [sys.executable, os.path.abspath(__file__), "--child", name, src, project, out] + caches
            t0 = time.perf_counter()
            p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=work, env=env)
            if i >= 0:
                times.append((time.perf_counter() - t0) * 1e3)
            if p.returncode != 0:
                raise RuntimeError("cold run failed: %s" % p.stderr.decode(errors="replace")[-2000:])
            res["manifest_diff"] += manifest_diff(os.path.join(out, project), name)
        res["cold_p50_ms"] = round(statistics.median(times), 3)
        if res.get("refmodel_p50_ms"):
            res["speedup_vs_refmodel"] = round(res["refmodel_p50_ms"] / res["warm_p50_ms"], 1)
        return res
    finally:
        restore()
        shutil.rmtree(work, ignore_errors=True)


def interpreter_floor(runs):
    """p50 of a bare ``python -c pass`` (the cold-run floor no Python CLI can beat)."""
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        subprocess.run([sys.executable, "-c", "pass"])
        times.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(times), 3)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        name, src, project, out = sys.argv[2:6]
        sys.exit(child(name, src, project, out, sys.argv[6:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--refmodel-runs", type=int, default=3)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--json", default=None, help="also write the results here")
    args = ap.parse_args()
    results = {"runs": args.runs, "python_floor_ms": interpreter_floor(args.runs), "configs": []}
    for name in args.configs.split(","):
        r = bench_config(name, args.runs, args.refmodel_runs)
        results["configs"].append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps({"python_floor_ms": results["python_floor_ms"]}), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)
    return 0 if all(r["manifest_diff"] == 0 for r in results["configs"]) else 1


if __name__ == "__main__":
    sys.exit(main())
