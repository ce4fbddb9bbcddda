# Cold-start pass on the GPU box into gpurun_out/$RUN/: the per-configuration
# bench (warm, cold `python -m`, cold release launcher), importtime of a cold
# golang translate through the launcher and through -m, and the stale-pyc probe.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-cold}
mkdir -p $OUT
export M2K_NO_NETWORK=1 M2K_DISABLE_CNB=1
timeout -k 10 500 python -u benchmarks/baseline_configs.py --runs 9 --emulation-runs 0 --json $OUT/baseline_configs.json > $OUT/baseline_configs.log 2>&1
timeout -k 10 60 python -u scripts/pyc_diag.py > $OUT/pyc_diag.json 2> $OUT/pyc_diag.err
W=$(mktemp -d)
cp -r samples/golang $W/src
python - $W <<'PY'
import sys
sys.path.insert(0, "scripts")
import builddist
open(sys.argv[1] + "/m2k_main.py", "w").write(builddist.ENTRY.replace("os.path.dirname(os.path.dirname(os.path.abspath(__file__)))", repr(__import__("os").getcwd())))
PY
cd $W
for i in 1 2 3; do rm -rf out; timeout -k 5 60 python -S -X importtime m2k_main.py translate -s src -o out --qaskip > /dev/null 2> imp_launcher.txt; done
for i in 1 2 3; do rm -rf out; PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 5 60 python -X importtime -m move2kube_amd translate -s src -o out --qaskip > /dev/null 2> imp_module.txt; done
cp imp_launcher.txt imp_module.txt $GRAFT_REPO_ROOT/$OUT/
cd $GRAFT_REPO_ROOT
rm -rf $W
echo done
