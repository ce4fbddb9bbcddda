set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cold
export M2K_NO_NETWORK=1 M2K_DISABLE_CNB=1
cp -r samples/golang /tmp/golang_src
cd /tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
for i in 1 2 3; do python -X importtime -c "pass" 2> $GRAFT_REPO_ROOT/gpurun_out/cold/floor_imp$i.txt; done
for i in 1 2 3; do timeout -k 5 60 python -X importtime -m move2kube_amd translate -s golang_src -o out$i --qaskip > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/cold/imp$i.txt; done
timeout -k 5 60 python -c "
import cProfile,pstats,sys,time
t0=time.perf_counter()
pr=cProfile.Profile(); pr.enable()
sys.path.insert(0,'$GRAFT_REPO_ROOT')
from move2kube_amd.cli import main
t1=time.perf_counter()
main.main(['translate','-s','golang_src','-o','outp','--qaskip'])
pr.disable()
print('import',t1-t0,'total',time.perf_counter()-t0)
pstats.Stats(pr).sort_stats('cumulative').print_stats(60)
pstats.Stats(pr).sort_stats('tottime').print_stats(30)
" > $GRAFT_REPO_ROOT/gpurun_out/cold/prof.txt 2>&1
cat /proc/self/status | grep -i cpus_allowed_list > $GRAFT_REPO_ROOT/gpurun_out/cold/aff.txt
echo done
