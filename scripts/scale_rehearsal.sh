# Weak-scaling rehearsal of bench.py on one box's CPUs (gloo, no GPU touched):
# N = 1, 2, 4, 8 ranks and then 1 rank again, one JSON line each into
# gpurun_out/$RUN/, plus a summary line per run with the host accounting that
# bench.py reports (CPU ms per step over all ranks and per rank, context
# switches, the box's CPU share, the slowest rank's median step, cgroup
# throttling).
#   VARIANTS  space-separated subset of
#             base    bench.py as the driver runs it
#             pinned  --pin-cores: each rank on its own physical cores
#             thr1    M2K_HOST_THREADS=1 M2K_WORKERS=1: one thread per host pool
#             (default: all three, interleaved per N so box drift hits each)
#   gpurun -- 'RUN=r06_scale bash scripts/scale_rehearsal.sh'
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
RUN=${RUN:-scale}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
VARIANTS=${VARIANTS:-base pinned thr1}
STEPS=${STEPS:-30}
k=0
for n in ${NS:-1 2 4 8 1}; do
  for v in $VARIANTS; do
    k=$((k + 1))
    extra=()
    envs=()
    case "$v" in
      base) ;;
      pinned) extra=(--pin-cores) ;;
      thr1) envs=(M2K_HOST_THREADS=1 M2K_WORKERS=1) ;;
      *) echo "unknown variant $v" >&2; exit 2 ;;
    esac
    log="$OUT/scale_${k}_${v}_n${n}.log"
    env "${envs[@]}" timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + k)) bench.py --gpus $n --steps "$STEPS" --warmup 3 \
      --check-runs 0 --large-tree "" "${extra[@]}" > "$log" 2>&1
    grep '^{"metric"' "$log" | VARIANT=$v python -c '
import json, os, sys
d = json.loads(sys.stdin.read())
h = d["host"]
pr = h["per_rank"]
def avg(k):
    return round(sum(r[k] for r in pr) / len(pr), 3)
print(json.dumps({"variant": os.environ["VARIANT"], "n": d["n_gpus"], "ms_per_step": d["ms_per_step"],
                  "value": d["value"], "step_ms": d["step_ms"], "cpus": h["cpus"],
                  "cpu_ms_per_step_all_ranks": h["cpu_ms_per_step_all_ranks"],
                  "cpu_sys_ms_per_step_all_ranks": h["cpu_sys_ms_per_step_all_ranks"],
                  "cpu_demand": round(h["cpu_ms_per_step_all_ranks"] / d["ms_per_step"], 2),
                  "rank_user_ms": avg("user_ms"), "rank_sys_ms": avg("sys_ms"),
                  "rank_step_p50_ms": avg("step_p50_ms"), "rank_step_p90_ms": avg("step_p90_ms"),
                  "rank_nvcsw": avg("nvcsw"), "rank_nivcsw": avg("nivcsw"), "rank_cpus": avg("cpus"),
                  "slowest_rank_step_p50_ms": h["slowest_rank_step_p50_ms"],
                  "cgroup_throttled_ms": h["cgroup_throttled_ms"]}))' | tee -a "$OUT/scale_summary.jsonl"
  done
done
# the box's CPU topology, for reading the pinned variant
python - > "$OUT/topology.json" <<'EOF'
import json, os
cpus = sorted(os.sched_getaffinity(0))
rows = {}
for c in cpus:
    b = "/sys/devices/system/cpu/cpu%d/topology/" % c
    try:
        rows[c] = {k: open(b + k).read().strip() for k in ("physical_package_id", "core_id", "thread_siblings_list")}
    except OSError as e:
        rows[c] = str(e)
print(json.dumps({"affinity": cpus, "nproc_machine": os.cpu_count(), "topology": rows}))
EOF
