set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1c
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1c/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 > gpurun_out/r1c/bench.log 2>&1
timeout -k 10 500 python -u benchmarks/baseline_configs.py --runs 5 --json gpurun_out/r1c/baseline_configs.json > gpurun_out/r1c/baseline_configs.log 2>&1
nproc > gpurun_out/r1c/host.txt; cat /proc/cpuinfo | grep "model name" | head -1 >> gpurun_out/r1c/host.txt; df -T /tmp >> gpurun_out/r1c/host.txt
echo done
