# Weak-scaling rehearsal of bench.py on the box's CPUs (gloo, no GPU touched):
# N = 1, 2, 4, 8 ranks, one JSON line each into gpurun_out/scale/.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scale
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
for n in 1 2 4 8; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 30 --warmup 3 --check-runs 0 \
    > gpurun_out/scale/n$n.log 2>&1
  grep metric gpurun_out/scale/n$n.log
done
