#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json configuration 5 on the reference's own
``samples/`` corpus.

The reference (a Go CLI) publishes no performance numbers; BASELINE.json names
the fallback metric "translate wall-clock + manifest diff vs ref on samples/"
and five configurations.  The headline step is configuration 5, "full samples/
tree -> Helm chart + Operator output with target-cluster GroupVersion
customize": ``move2kube translate -s samples --qaskip -q
helm-openshift-qacache.yaml`` (Helm artifacts, Openshift cluster profile, so
every object goes through the profile's group/version selection:
DeploymentConfig, Route, ImageStream), including the operator-sdk call
(stand-in on ``PATH``).  One step = plan + curate (answers replayed from the QA
cache, defaults otherwise) + translate + write of every artifact, in process;
nothing is cached between steps (fresh file index, detector runs, QA engines,
output directory).  ``benchmarks/refconfigs.py`` defines the commands.

Multi-GPU: one rank per GPU (torch.distributed over RCCL; joined whenever a
launcher set RANK and MASTER_ADDR, one rank included), each rank translating
its own copy of the corpus (weak scaling); the timed region is bracketed by a
barrier and ``torch.cuda.synchronize()`` and the slowest rank's time is
reported.  ``value`` = translated services per second summed over all ranks.

Work tree: inputs and output trees live on a tmpfs (``/dev/shm``) when one is
available (``--workdir``, reported as ``workdir_fs``): every step rewrites the
output tree, and on the hosts' discard-mounted scratch disks that churn slows
every later run (see README "Why tmpfs").

Host accounting (``host``): CPU ms per step over all ranks, context switches,
and ``per_rank`` user / sys CPU, step p50 / p90 and context switches per step,
so that a CPU-share limit on a shared node can be told from a code change.
``--pin-cores`` (rehearsal only) pins each rank to its own physical cores and
``M2K_HOST_THREADS=1`` sizes every host pool to one thread
(``scripts/scale_rehearsal.sh`` runs the three variants).

Correctness (untimed, rank 0): ``manifest_diff_vs_ref`` is the number of
files that differ from the reference-derived expected trees
(``tests/golden/reference/<config>``) over all five configurations, and
``per_config`` gives each configuration's diff plus its warm in-process and
cold CLI-process p50 and interquartile range over ``--check-runs`` (default 9)
runs; ``per_config_vs_prev`` divides them by the
previous round's driver line (``benchmarks/prev_round_bench.json``).  The
reference's execution model is only emulated in Python
(``benchmarks/baseline_configs.py``), so nothing here is a measured
comparison with the Go tool and ``vs_baseline`` is null.
"""

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (HERE, os.path.join(HERE, "benchmarks")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import refconfigs  # noqa: E402

BASELINE_CONFIG = "full samples/ tree → Helm chart + Operator output with target-cluster GroupVersion customize"


def _dist_env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def tree_files(root):
    return refconfigs.tree_files(root)


def per_config_checks(runs):
    """Untimed: every configuration's diff vs the reference-derived tree and its
    warm / cold p50 and interquartile range (``benchmarks/baseline_configs.py``)."""
    import baseline_configs
    out = {}
    for name in refconfigs.CONFIGS:
        r = baseline_configs.warm_runs(name, runs)
        cold, cold_diff = baseline_configs.cold_runs(name, runs)
        out[name] = {"manifest_diff_vs_ref": r["manifest_diff_vs_ref"] + cold_diff, "runs": runs,
                     "warm_p50_ms": r["warm_p50_ms"], "warm_iqr_ms": r["warm_iqr_ms"],
                     "cold_p50_ms": cold["cold_p50_ms"], "cold_iqr_ms": cold["cold_iqr_ms"],
                     "cold_over_floor_p50_ms": cold["cold_over_floor_p50_ms"],
                     "cold_over_floor_iqr_ms": cold["cold_over_floor_iqr_ms"],
                     "cold_launcher_p50_ms": cold["cold_launcher_p50_ms"]}
    return out


# the previous round's driver line (BENCH_r05.json, stdout verbatim; kept out
# of profiles/, which does not travel to the GPU box)
PREV_BENCH = os.path.join(HERE, "benchmarks", "prev_round_bench.json")


def per_config_vs_prev(per_config, prev_path):
    """Ratio now / previous round for each configuration's warm p50 and cold
    p50 over the interpreter floor (> 1 = slower), next to the previous
    values, so that a shifted median shows in the bench line itself; compare
    a ratio with ``*_iqr_ms`` / p50 before calling it a regression."""
    try:
        with open(prev_path) as f:
            prev = json.load(f)
    except (OSError, ValueError):
        return None
    out = {"prev": os.path.relpath(prev_path, HERE), "prev_ms_per_step": prev.get("ms_per_step")}
    for name, now in (per_config or {}).items():
        was = (prev.get("per_config") or {}).get(name)
        if not was or "warm_p50_ms" not in now:
            continue
        row = {}
        for k in ("warm", "cold_over_floor"):
            if was.get(k + "_p50_ms") and now.get(k + "_p50_ms") is not None:
                row[k + "_ratio"] = round(now[k + "_p50_ms"] / was[k + "_p50_ms"], 3)
                row[k + "_prev_p50_ms"] = was[k + "_p50_ms"]
        out[name] = row
    return out


def large_tree_check(sizes):
    """Untimed: per-service ``translate`` cost on synthetic trees of growing
    size (the scaling axis of this workload); a ratio near 1 means linear."""
    saved = {k: os.environ.get(k) for k in ("M2K_NO_NETWORK", "M2K_DISABLE_CNB")}
    os.environ.update({"M2K_NO_NETWORK": "1", "M2K_DISABLE_CNB": "1"})
    try:
        import translate_large_tree
        rows = translate_large_tree.measure(sizes)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    per = {str(r["apps"]): r["ms_per_service"] for r in rows}
    return {"large_tree_translate_ms_per_service": per,
            "services": {str(r["apps"]): r["services"] for r in rows},
            "ratio_largest_vs_smallest": round(rows[-1]["ms_per_service"] / rows[0]["ms_per_service"], 3)}


def step_spread(step_s):
    """Rank 0's per-step wall times: min / p50 / p90 / max in ms, so that box
    noise (a slow tail) can be told from a regression (a shifted p50)."""
    if not step_s:
        return None
    ms = sorted(x * 1000.0 for x in step_s)

    def q(f):
        return round(ms[min(len(ms) - 1, int(f * (len(ms) - 1) + 0.5))], 3)
    return {"min": round(ms[0], 3), "p50": q(0.5), "p90": q(0.9), "max": round(ms[-1], 3), "n": len(ms)}


def _cpu_s():
    """(user, system) CPU seconds of this process and its reaped children
    (the operator-sdk stand-in, detector scripts), and their (voluntary,
    involuntary) context switches."""
    import resource
    a, b = resource.getrusage(resource.RUSAGE_SELF), resource.getrusage(resource.RUSAGE_CHILDREN)
    return (a.ru_utime + b.ru_utime, a.ru_stime + b.ru_stime,
            a.ru_nvcsw + b.ru_nvcsw, a.ru_nivcsw + b.ru_nivcsw)


def pin_to_cores(local_rank, local_world):
    """Weak-scaling rehearsal knob (``--pin-cores``): restrict this rank to its
    own physical cores - the CPUs of this job's affinity mask grouped by
    (package, core id) from sysfs, cores dealt round-robin to the local ranks,
    every SMT sibling of a dealt core kept.  Runs before anything touches the
    GPU.  Returns the CPU list, or None where the topology cannot be read."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    cores = {}
    for c in allowed:
        base = "/sys/devices/system/cpu/cpu%d/topology/" % c
        try:
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
            with open(base + "core_id") as f:
                core = f.read().strip()
        except OSError:
            return None
        cores.setdefault((pkg, core), []).append(c)
    keys = sorted(cores, key=lambda k: min(cores[k]))
    mine = [c for i, k in enumerate(keys) if i % max(1, local_world) == local_rank % max(1, local_world)
            for c in cores[k]]
    if not mine:   # more ranks than cores: share by rank modulo core count
        mine = cores[keys[local_rank % len(keys)]]
    os.sched_setaffinity(0, mine)
    return mine


def _cgroup_throttled_us():
    """Time the container's CPU quota held its tasks back (cgroup v2 cpu.stat);
    None where it cannot be read."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                if line.startswith("throttled_usec"):
                    return int(line.split()[1])
    except (OSError, ValueError):
        pass
    return None


def _host_cpus():
    """CPUs this job may use: the affinity mask within the cgroup quota."""
    from move2kube_amd.utils.constants import _cgroup_cpu_limit
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    limit = _cgroup_cpu_limit()
    return n if limit is None else min(n, limit)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=refconfigs.HEADLINE,
                    choices=sorted(refconfigs.CONFIGS) + sorted(refconfigs.EXTRA_CONFIGS))
    ap.add_argument("--check-runs", type=int, default=9,
                    help="warm/cold runs per configuration in the untimed per-config check (0 = skip)")
    ap.add_argument("--prev", default=PREV_BENCH,
                    help="previous round's bench line (JSON) for per_config_vs_prev; empty = skip")
    ap.add_argument("--pin-cores", action="store_true",
                    help="rehearsal knob: pin each rank to its own physical cores (LOCAL_RANK) before any GPU call")
    ap.add_argument("--large-tree", default="100,1000,5000",
                    help="untimed: translate synthetic trees of these app counts and report ms per service "
                         "(benchmarks/translate_large_tree.py); empty = skip")
    ap.add_argument("--keep", action="store_true", help="keep the work directory")
    ap.add_argument("--workdir", default="auto",
                    help="root for the input copies and output trees: auto (tmpfs if available), disk, or a path")
    args = ap.parse_args()

    world, rank, local_rank = _dist_env()
    pinned = None
    if args.pin_cores:
        pinned = pin_to_cores(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", world) or world))
    import torch
    dist = None
    have_cuda = torch.cuda.is_available()
    if have_cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ):  # launched by torchrun, one rank too
        import torch.distributed as dist
        dist.init_process_group(backend="nccl" if have_cuda else "gloo")

    def barrier():
        if dist is not None:
            if have_cuda:
                dist.barrier(device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier()
        if have_cuda:
            torch.cuda.synchronize()

    from move2kube_amd.utils import log
    log.set_quiet()
    root, workdir_fs = refconfigs.workdir_root(args.workdir)
    if root is not None:
        tempfile.tempdir = root  # also for the per-configuration checks below

    work = tempfile.mkdtemp(prefix="m2k-bench-r%d-" % rank)
    run = refconfigs.Run(args.config, work).prepare()
    undo = run.apply_env()
    n_services = 0
    step_s = []
    diff_headline = None
    phase_ms = None
    try:
        with run.session() as s:
            out = run.step(s)  # first (warm-up) step doubles as the correctness gate
            n_services = len(s.plan(run.src, refconfigs.PROJECT).services)
            if rank == 0:
                diff_headline = refconfigs.manifest_diff_vs_ref(args.config, out)
            for _ in range(max(0, args.warmup - 1)):
                run.step(s)
            barrier()
            step_s = []
            thr0, cpu0 = _cgroup_throttled_us(), _cpu_s()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ts = time.perf_counter()
                run.step(s)
                step_s.append(time.perf_counter() - ts)
            barrier()
            elapsed = time.perf_counter() - t0
            cpu1, thr1 = _cpu_s(), _cgroup_throttled_us()
            cpu_s = tuple(b - a for a, b in zip(cpu0, cpu1))
            if rank == 0:
                # untimed: one traced step for the per-phase breakdown (utils/trace.py)
                from move2kube_amd.utils import trace
                trace.enable("")
                try:
                    run.step(s)
                    phase_ms = {k: round(v, 3) for k, v in list(trace.summary().items())[:12]}
                finally:
                    trace._events = None
    finally:
        undo()
        if not args.keep:
            shutil.rmtree(work, ignore_errors=True)

    per_config = None
    if rank == 0 and args.check_runs > 0:
        per_config = per_config_checks(args.check_runs)
    if rank == 0 and args.large_tree:
        per_config = dict(per_config or {})
        per_config["large-tree"] = large_tree_check([int(x) for x in args.large_tree.split(",")])

    spread = step_spread(step_s)
    slowest_p50 = spread["p50"] if spread else 0.0
    k = max(1, args.steps)
    # this rank's accounting per timed step: user / sys CPU ms, step p50 / p90,
    # voluntary / involuntary context switches, CPUs it may run on
    mine = [cpu_s[0] * 1e3 / k, cpu_s[1] * 1e3 / k, slowest_p50, spread["p90"] if spread else 0.0,
            cpu_s[2] / k, cpu_s[3] / k, float(_host_cpus() if pinned is None else len(pinned))]
    per_rank = [mine]
    if dist is not None:
        dev = torch.device("cuda", torch.cuda.current_device()) if have_cuda else torch.device("cpu")
        t = torch.tensor([elapsed, slowest_p50], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, slowest_p50 = float(t[0].item()), float(t[1].item())
        c = torch.tensor(list(cpu_s), dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        cpu_s = tuple(float(x) for x in c.tolist())
        rows = [torch.zeros(len(mine), dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(rows, torch.tensor(mine, dtype=torch.float64, device=dev))
        per_rank = [r.tolist() for r in rows]
    ms = elapsed * 1000.0 / max(1, args.steps)
    value = world * n_services * args.steps / elapsed if elapsed > 0 else 0.0
    if rank == 0:
        total_diff = diff_headline
        if per_config is not None and total_diff is not None:
            total_diff = sum(v["manifest_diff_vs_ref"] for v in per_config.values() if "manifest_diff_vs_ref" in v)
        print(json.dumps({
            "metric": "translate_throughput (BASELINE fallback: translate wall-clock + manifest diff vs ref on samples/)",
            "value": round(value, 3),
            "unit": "services/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "step_ms": spread,
            # host-side accounting of the timed region, to tell a CPU-share
            # limit from a code change when N ranks share one node's CPUs:
            # CPU ms per step summed over ranks (children included), the
            # slowest rank's median step, and the cgroup's quota throttling
            "host": {"cpus": _host_cpus(),
                     "cpu_ms_per_step_all_ranks": round((cpu_s[0] + cpu_s[1]) * 1000.0 / max(1, args.steps), 3),
                     "cpu_sys_ms_per_step_all_ranks": round(cpu_s[1] * 1000.0 / max(1, args.steps), 3),
                     "slowest_rank_step_p50_ms": round(slowest_p50, 3),
                     "cgroup_throttled_ms": None if thr0 is None or thr1 is None else round((thr1 - thr0) / 1000.0, 3),
                     "ctx_switches_per_step_all_ranks": {"voluntary": round(cpu_s[2] / k, 2),
                                                         "involuntary": round(cpu_s[3] / k, 2)},
                     "pinned": pinned is not None,
                     "per_rank": [dict(zip(("user_ms", "sys_ms", "step_p50_ms", "step_p90_ms", "nvcsw", "nivcsw",
                                            "cpus"), (round(x, 3) for x in r))) for r in per_rank]},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "n/a",
            "data": "reference samples/ corpus (%d services), in-process plan+curate+translate per step, "
                    "output tree rewritten each step on %s; stand-ins for operator-sdk; no container engine"
                    % (n_services, workdir_fs),
            "workdir_fs": workdir_fs,
            "manifest_diff_vs_ref": total_diff,
            "manifest_diff_vs_ref_headline": diff_headline,
            "per_config": per_config,
            "per_config_vs_prev": per_config_vs_prev(per_config, args.prev) if per_config and args.prev else None,
            "phase_ms_one_step": phase_ms,
            "config": {"model": BASELINE_CONFIG, "command": "move2kube translate -s samples --qaskip -q "
                       "helm-openshift-qacache.yaml" if args.config == refconfigs.HEADLINE else args.config,
                       "global_batch": world, "seq_len": n_services, "parallelism": "dp%d" % world},
        }), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
