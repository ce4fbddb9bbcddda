# GPU-box performance pass into gpurun_out/$RUN/: per-config cold/warm bench (9 runs),
# warm cProfile of the headline configuration, cold cProfiles of golang and helm-openshift
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-perf}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 > $OUT/bench.log 2>&1
timeout -k 10 600 python -u benchmarks/baseline_configs.py --runs 9 --json $OUT/baseline_configs.json > $OUT/baseline_configs.log 2>&1
timeout -k 10 120 python -u scripts/profile_step.py helm-openshift cumulative 20 > $OUT/profile_warm_helm_openshift.txt 2>&1
timeout -k 10 120 python -u scripts/cold_profile.py golang tottime > $OUT/cold_profile_golang.txt 2>&1
timeout -k 10 120 python -u scripts/cold_profile.py helm-openshift cumulative > $OUT/cold_profile_helm_openshift.txt 2>&1
nproc > $OUT/host.txt; grep -m1 "model name" /proc/cpuinfo >> $OUT/host.txt
echo done
