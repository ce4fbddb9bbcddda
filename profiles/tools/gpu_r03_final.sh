# Round-3 full pass on the GPU box into gpurun_out/$RUN/: pytest -m gpu, smoke(),
# bench.py (+ per-config and large-tree checks), bench.py under torchrun/RCCL
# with one rank, rocprofv3 kernel stats of smoke(), large-tree plan, and the
# gloo weak-scaling series (1/2/4/8 ranks on the box's CPU share).
set -e
cd $GRAFT_REPO_ROOT
RUN=${RUN:-r03_final}
export RUN
bash scripts/gpu_configs.sh
OUT=gpurun_out/$RUN
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
RUN=$RUN bash scripts/gpu_dist1.sh > /dev/null
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o smoke -- python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/rocprof_smoke.log 2>&1
timeout -k 10 300 python -u benchmarks/plan_large_tree.py --apps 2000 --depth 4 --files 5 > $OUT/plan_large_tree.json 2> $OUT/plan_large_tree.err
timeout -k 10 400 python -u benchmarks/translate_large_tree.py --apps 100,400,1000,2000 > $OUT/translate_large_tree.json 2> $OUT/translate_large_tree.err
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
for n in 1 2 4 8; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 30 --warmup 3 --check-runs 0 --large-tree "" > $OUT/scale_n$n.log 2>&1
  grep metric $OUT/scale_n$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["n_gpus"], d["ms_per_step"], d["value"])' >> $OUT/scale_summary.txt
done
cat $OUT/scale_summary.txt
echo done
