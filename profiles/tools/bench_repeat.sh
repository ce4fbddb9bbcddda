# bench.py five times back to back on one box (default settings, no per-config
# checks) - the spread of the headline number on one host.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-benchrepeat}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --check-runs 0 > $OUT/bench_$i.log 2>&1
  grep metric $OUT/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["workdir_fs"])' | tee -a $OUT/summary.txt
done
