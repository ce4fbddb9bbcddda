# GPU-box validation: pytest -m gpu, smoke() and bench.py into gpurun_out/$RUN/
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-validate}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 > $OUT/bench.log 2>&1
echo done
