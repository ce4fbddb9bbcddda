set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1b
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1b/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1b/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 > gpurun_out/r1b/bench.log 2>&1
echo done
