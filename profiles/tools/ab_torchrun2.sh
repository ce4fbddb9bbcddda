# Isolate the torchrun slowdown: plain / 1-rank RCCL without torchrun / torchrun / torchrun --monitor-interval 5 / torchrun with gloo-only barriers
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-ab_torchrun2}
mkdir -p $OUT
S="--steps 30 --warmup 3 --check-runs 0 --large-tree"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $S "" > $OUT/plain_$i.log 2>&1
  RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29540 + i)) timeout -k 10 200 python -u bench.py $S "" > $OUT/manualenv_$i.log 2>&1
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29550 + i)) bench.py $S "" > $OUT/torchrun_$i.log 2>&1
  timeout -k 10 200 python -m torch.distributed.run --monitor-interval 5 --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29560 + i)) bench.py $S "" > $OUT/torchrun_mon5_$i.log 2>&1
  for f in plain_$i manualenv_$i torchrun_$i torchrun_mon5_$i; do
    grep metric $OUT/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["ms_per_step"], d["phase_ms_one_step"]["plan"], d["phase_ms_one_step"]["translate"])' $f >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
