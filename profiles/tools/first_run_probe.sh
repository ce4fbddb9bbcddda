# Is the first bench.py process on a box slower than the next ones, and does a
# burst of short CLI processes (the cold benchmarks) make the next one slow?
# Three back-to-back bench.py runs on the fresh box, then 60 cold CLI runs
# (benchmarks/cold_trace.py), then three bench.py runs again; one summary line
# each (ms/step, step p50/p90, CPU ms per step user+sys and sys).
#   gpurun -- 'RUN=r04_first_run bash scripts/first_run_probe.sh'
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
RUN=${RUN:-first_run}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
summary() {
  python -c '
import json, sys
d = [json.loads(l) for l in sys.stdin if l.startswith("{\"metric\"")][-1]
h = d["host"]
print(json.dumps({"label": sys.argv[1], "ms_per_step": d["ms_per_step"], "p50": d["step_ms"]["p50"],
                  "p90": d["step_ms"]["p90"], "cpu_ms": h["cpu_ms_per_step_all_ranks"],
                  "sys_ms": h["cpu_sys_ms_per_step_all_ranks"]}))' "$1" | tee -a "$OUT/first_run.jsonl"
}
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 3 --check-runs 0 --large-tree "" 2> /dev/null | summary "fresh_$i"
done
timeout -k 10 180 python -u benchmarks/cold_trace.py helm-openshift --runs 60 > "$OUT/burst.json"
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 3 --check-runs 0 --large-tree "" 2> /dev/null | summary "after_burst_$i"
done
