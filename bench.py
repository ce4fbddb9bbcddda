#!/usr/bin/env python3
"""Headline benchmark: end-to-end ``translate --qaskip`` of the samples corpus.

The reference (a Go CLI) publishes no performance numbers; BASELINE.json names
the fallback metric "translate wall-clock + manifest diff vs ref on samples/".
One *step* is a complete in-process ``plan`` + ``curate`` (default answers) +
``translate`` of the whole ``samples/`` tree (13 services: 7 source-directory
apps, a Dockerfile app, a 3-service compose app, a CF manifest app and a
Kubernetes YAML app), writing every artifact (k8s YAMLs, compose, Tekton, build
scripts, QA cache) to a private output directory.  Nothing is cached between
steps (fresh file index, fresh detector runs, fresh QA engines).

Multi-GPU: one rank per GPU (torch.distributed), each rank translating its own
copy of the corpus (weak scaling); the timed region is bracketed by a barrier
and ``torch.cuda.synchronize()`` and the slowest rank's time is reported.
``value`` = total translated services per second over all ranks.

Before timing, rank 0 checks the output of one step against the checked-in
expected tree (``tests/golden/samples``) and reports ``manifest_diff`` (number
of differing/missing/extra files; 0 = identical).

After timing, a couple of untimed steps rerun in the reference's execution
model (every detector forked as ``/bin/sh`` one at a time, as
``internal/containerizer/dockerfilecontainerizer.go:76-83`` does) and report
``reference_model_ms_per_step`` - a same-machine proxy for the Go tool, whose
cost is dominated by those forks; the reference publishes no numbers, so
``vs_baseline`` stays null.
"""

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
SAMPLES = os.path.join(HERE, "samples")
GOLDEN = os.path.join(HERE, "tests", "golden", "samples")

# deterministic, offline runs: no ssh-keyscan, no docker/podman/pack probing
os.environ.setdefault("M2K_NO_NETWORK", "1")
os.environ.setdefault("M2K_DISABLE_CNB", "1")


def _dist_env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def tree_files(root):
    out = {}
    for dp, _dn, fns in os.walk(root):
        for fn in fns:
            p = os.path.join(dp, fn)
            out[os.path.relpath(p, root)] = p
    return out


def manifest_diff(actual_root, golden_root):
    """Count of files that differ, are missing or are extra vs the golden tree."""
    if not os.path.isdir(golden_root):
        return None
    a, g = tree_files(actual_root), tree_files(golden_root)
    diff = 0
    for rel in set(a) | set(g):
        if rel not in a or rel not in g:
            diff += 1
            continue
        with open(a[rel], "rb") as fa, open(g[rel], "rb") as fg:
            if fa.read() != fg.read():
                diff += 1
    return diff


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--src", default=SAMPLES)
    ap.add_argument("--keep", action="store_true", help="keep the output directory")
    ap.add_argument("--reference-model-steps", type=int, default=2,
                    help="untimed steps in the reference's serial fork-per-detector mode (0 = skip)")
    args = ap.parse_args()

    world, rank, local_rank = _dist_env()
    import torch
    dist = None
    have_cuda = torch.cuda.is_available()
    if have_cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1:
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

    sys.path.insert(0, HERE)
    from move2kube_amd import api
    from move2kube_amd.utils import log
    log.set_quiet()

    work = tempfile.mkdtemp(prefix="m2k-bench-r%d-" % rank)
    n_services = 0
    phase_ms = None
    try:
        # private copy outside any git checkout, so output is location independent
        src = os.path.join(work, "samples")
        shutil.copytree(args.src, src, symlinks=True)
        with api.Session(qaskip=True) as s:
            def step():
                out = s.translate(src, os.path.join(work, "out"), name="samples")
                return out

            # correctness gate (rank 0) + service count
            out = step()
            plan = s.plan(src, "samples")
            n_services = len(plan.services)
            diff = manifest_diff(out, GOLDEN) if rank == 0 else None
            for _ in range(max(0, args.warmup - 1)):
                step()
            barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            barrier()
            elapsed = time.perf_counter() - t0
            # Untimed: one traced step for the per-phase breakdown (utils/trace.py)
            phase_ms = None
            if rank == 0:
                from move2kube_amd.utils import trace
                trace.enable("")
                try:
                    step()
                    phase_ms = {k: round(v, 3) for k, v in list(trace.summary().items())[:12]}
                finally:
                    trace._events = None
            # Untimed ablation: the reference's execution model (every detector
            # forked as a shell process, one at a time), same output required.
            ref_ms = None
            if args.reference_model_steps > 0 and rank == 0:
                from move2kube_amd.utils.constants import settings
                saved = (os.environ.get("M2K_NATIVE_DETECT"), settings.workers)
                os.environ["M2K_NATIVE_DETECT"] = "0"
                settings.workers = 1
                try:
                    out_ref = step()
                    t1 = time.perf_counter()
                    for _ in range(args.reference_model_steps):
                        step()
                    ref_ms = (time.perf_counter() - t1) * 1000.0 / args.reference_model_steps
                    if rank == 0 and diff is not None:
                        diff += manifest_diff(out_ref, GOLDEN)
                finally:
                    if saved[0] is None:
                        os.environ.pop("M2K_NATIVE_DETECT", None)
                    else:
                        os.environ["M2K_NATIVE_DETECT"] = saved[0]
                    settings.workers = saved[1]
    finally:
        if not args.keep:
            shutil.rmtree(work, ignore_errors=True)

    if dist is not None:
        dev = torch.device("cuda", torch.cuda.current_device()) if have_cuda else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed * 1000.0 / max(1, args.steps)
    value = world * n_services * args.steps / elapsed if elapsed > 0 else 0.0
    if rank == 0:
        print(json.dumps({
            "metric": "translate_throughput_samples",
            "value": round(value, 3),
            "unit": "services/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "n/a",
            "data": "samples/ corpus (%d services), in-process translate --qaskip, CNB disabled" % n_services,
            "manifest_diff": diff,
            "reference_model_ms_per_step": None if ref_ms is None else round(ref_ms, 3),
            "speedup_vs_reference_model": None if not ref_ms else round(ref_ms / ms, 2),
            "phase_ms_one_step": phase_ms,
            "config": {"model": "move2kube translate samples/ (full tree)", "global_batch": world,
                       "seq_len": n_services, "parallelism": "dp%d" % world},
        }), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
