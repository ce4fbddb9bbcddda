# GPU-box validation: pytest -m gpu, bench.py and the per-config benchmark into gpurun_out/$RUN/
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${RUN:-latest}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${RUN:-latest}/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 > gpurun_out/${RUN:-latest}/bench.log 2>&1
timeout -k 10 500 python -u benchmarks/baseline_configs.py --runs 5 --json gpurun_out/${RUN:-latest}/baseline_configs.json > gpurun_out/${RUN:-latest}/baseline_configs.log 2>&1
nproc > gpurun_out/${RUN:-latest}/host.txt; cat /proc/cpuinfo | grep "model name" | head -1 >> gpurun_out/${RUN:-latest}/host.txt; df -T /tmp >> gpurun_out/${RUN:-latest}/host.txt
echo done
