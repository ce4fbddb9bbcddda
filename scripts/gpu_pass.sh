# One pass on the GPU box into gpurun_out/$RUN/:
#   pytest -m gpu, smoke(), bench.py with its default checks (per-config diffs,
#   warm/cold p50s, large-tree ratio), rocprofv3 kernel stats of smoke(), and,
#   when AB names a tree under .ab_base/, the interleaved same-box A/B of the
#   headline against it (benchmarks/ab_bench.py).
# Every GPU step has its own time limit; the first failure ends the pass.
#   COLD_AB=<tree> adds the same A/B of cold CLI starts (ab_bench.py --cold),
#   PHASES=1 the per-configuration cold phase split (scripts/cold_phases.py),
#   TRACE=1 the traced spans of cold CLI runs (benchmarks/cold_trace.py),
#   BUDGET=1 the whole-process cold budget split (benchmarks/cold_budget.py),
#   COV=1 the line coverage of `pytest -m gpu` (scripts/coverage.py; merge its
#         cov_gpu_data/ with the CPU suite's: coverage.py report --data A --data B),
#   SKIP_BENCH=1 leaves out the GPU tests, smoke, bench and rocprof steps.
#   RUN=r04_x AB=r03 gpurun --timeout 1200 -- bash scripts/gpu_pass.sh
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
RUN=${RUN:-pass}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_BENCH" ]; then
echo "pytest -m gpu"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -1 "$OUT/pytest_gpu.log"
echo "smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "bench"
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["step_ms"], d["manifest_diff_vs_ref"], d["per_config"]["large-tree"]["ratio_largest_vs_smallest"])' "$OUT/bench.json"
echo "rocprof smoke"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof" -o smoke -- python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/rocprof_smoke.log" 2>&1
fi
if [ -n "$COV" ]; then
  echo "gpu test coverage"
  timeout -k 10 400 python -u scripts/coverage.py run --out "$OUT/cov_gpu" --data "$OUT/cov_gpu_data" \
    -- tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/cov_gpu.log" 2>&1
  tail -1 "$OUT/cov_gpu.log"
fi
if [ -n "$AB" ]; then
  echo "A/B vs $AB"
  timeout -k 10 900 python -u benchmarks/ab_bench.py --base ".ab_base/$AB" --pairs "${AB_PAIRS:-4}" --out "$OUT/ab.jsonl"
fi
if [ -n "$COLD_AB" ]; then
  echo "cold A/B vs $COLD_AB"
  timeout -k 10 900 python -u benchmarks/ab_bench.py --base ".ab_base/$COLD_AB" --cold "${COLD_CONFIGS:-golang,java-cnb,cf,helm-openshift}" \
    --pairs "${COLD_PAIRS:-2}" --runs 9 --timeout 400 --out "$OUT/cold_ab.jsonl"
fi
if [ -n "$PHASES" ]; then
  echo "cold phases"
  for c in golang docker-compose java-cnb cf helm-openshift; do
    timeout -k 10 120 python -u scripts/cold_phases.py "$c" --runs 15 >> "$OUT/cold_phases.jsonl"
  done
  timeout -k 10 120 python -u scripts/cold_phases.py cf --command 0 --runs 15 >> "$OUT/cold_phases.jsonl"
  cat "$OUT/cold_phases.jsonl"
fi
if [ -n "$TRACE" ]; then
  echo "cold traces"
  for c in golang java-cnb cf helm-openshift; do
    timeout -k 10 180 python -u benchmarks/cold_trace.py "$c" --runs 15 | tee -a "$OUT/cold_trace.jsonl"
    timeout -k 10 180 python -u benchmarks/cold_importtime.py "$c" --runs 9 >> "$OUT/cold_importtime.jsonl"
  done
fi
if [ -n "$BUDGET" ]; then
  echo "cold budget"
  timeout -k 10 600 python -u benchmarks/cold_budget.py "${BUDGET_CONFIGS:-golang,java-cnb,cf,helm-openshift}" --runs "${BUDGET_RUNS:-30}" | tee "$OUT/cold_budget.jsonl"
fi
echo done
