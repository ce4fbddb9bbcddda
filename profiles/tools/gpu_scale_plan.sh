# GPU-box pass: large-tree planning benchmark and the gloo weak-scaling rehearsal of bench.py
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-scaleplan}
mkdir -p $OUT
timeout -k 10 300 python -u benchmarks/plan_large_tree.py --apps 2000 --depth 4 --files 5 > $OUT/plan_large_tree.json 2> $OUT/plan_large_tree.err
bash scripts/scale_rehearsal.sh > $OUT/scale_rehearsal.txt 2>&1
cp gpurun_out/scale/*.log $OUT/ || true
echo done
