# Round-3 GPU-box pass into gpurun_out/$RUN/: pytest -m gpu, bench.py, the
# per-configuration bench, smoke() (plain and under rocprofv3 kernel trace),
# large-tree translate scaling and an -X importtime of one cold CLI translate.
set -e
cd $GRAFT_REPO_ROOT
RUN=${RUN:-r03}
export RUN
bash scripts/gpu_configs.sh
OUT=gpurun_out/$RUN
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/rocprof -o smoke -- python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/rocprof_smoke.log 2>&1
timeout -k 10 400 python -u benchmarks/translate_large_tree.py --apps 100,400,1000,2000 > $OUT/translate_large_tree.json 2> $OUT/translate_large_tree.err
W=$(mktemp -d)
cp -r samples/golang $W/src
( cd $W && PYTHONPATH=$GRAFT_REPO_ROOT M2K_NO_NETWORK=1 M2K_DISABLE_CNB=1 timeout -k 10 60 python -X importtime -m move2kube_amd translate -s src -o out --qaskip > /dev/null 2> importtime.txt ) || true
cp $W/importtime.txt $OUT/importtime_golang.txt || true
rm -rf $W
echo done
