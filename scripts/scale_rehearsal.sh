# Weak-scaling rehearsal of bench.py on one box's CPUs (gloo, no GPU touched):
# N = 1, 2, 4, 8 ranks and then 1 rank again, one JSON line each into
# gpurun_out/$RUN/, plus a summary line per run with the host accounting that
# bench.py reports (CPU ms per step over all ranks, the box's CPU share, the
# slowest rank's median step, cgroup throttling).
#   gpurun -- 'RUN=r04_scale bash scripts/scale_rehearsal.sh'
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
RUN=${RUN:-scale}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
k=0
for n in 1 2 4 8 1; do
  k=$((k + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + k)) bench.py --gpus $n --steps 30 --warmup 3 --check-runs 0 --large-tree "" \
    > "$OUT/scale_${k}_n${n}.log" 2>&1
  grep '^{"metric"' "$OUT/scale_${k}_n${n}.log" | python -c '
import json, sys
d = json.loads(sys.stdin.read())
h = d["host"]
print(json.dumps({"n": d["n_gpus"], "ms_per_step": d["ms_per_step"], "value": d["value"], "step_ms": d["step_ms"],
                  "cpus": h["cpus"], "cpu_ms_per_step_all_ranks": h["cpu_ms_per_step_all_ranks"],
                  "cpu_sys_ms_per_step_all_ranks": h["cpu_sys_ms_per_step_all_ranks"],
                  "cpu_demand": round(h["cpu_ms_per_step_all_ranks"] / d["ms_per_step"], 2),
                  "slowest_rank_step_p50_ms": h["slowest_rank_step_p50_ms"],
                  "cgroup_throttled_ms": h["cgroup_throttled_ms"]}))' | tee -a "$OUT/scale_summary.jsonl"
done
