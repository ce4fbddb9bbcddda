# bench.py through torchrun with one rank on the GPU: init_process_group("nccl")
# (RCCL), barrier with device_ids, MAX all-reduce of the timer on the device -
# the code path of the driver's multi-GPU runs, on the one GPU a box has.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-dist1}
mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --check-runs 0 > $OUT/bench_torchrun_n1.log 2>&1
grep metric $OUT/bench_torchrun_n1.log
