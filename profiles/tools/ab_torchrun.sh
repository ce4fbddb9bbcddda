# A/B on one box: bench.py plain vs under torchrun (1 rank, RCCL), alternating.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-ab_torchrun}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --check-runs 0 --large-tree "" > $OUT/plain_$i.log 2>&1
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $((29520 + i)) bench.py --gpus 1 --steps 30 --warmup 3 --check-runs 0 --large-tree "" > $OUT/torchrun_$i.log 2>&1
  for f in plain_$i torchrun_$i; do
    grep metric $OUT/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["ms_per_step"], d["phase_ms_one_step"]["plan"], d["phase_ms_one_step"]["translate"])' $f >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
