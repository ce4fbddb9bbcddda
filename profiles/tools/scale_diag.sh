# Weak-scaling check of bench.py on the box's CPUs (gloo, no GPU): N = 1, 2, 4, 8
# on tmpfs, then N = 1 again on tmpfs and on disk; per-rank step percentiles.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-scalediag}
mkdir -p $OUT
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
(df -T /dev/shm /tmp; cat /sys/fs/cgroup/cpu.max) > $OUT/env.txt 2>&1 || true
run() {  # name n args...
  name=$1; n=$2; shift 2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 200)) scripts/bench_diag.py --gpus $n --steps 30 --warmup 3 --check-runs 0 "$@" > $OUT/$name.log 2>&1
  echo "$name $(grep metric $OUT/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["workdir_fs"])')"
  grep "^rank" $OUT/$name.log | sort | head -2 | sed "s/^/  /"
}
run n1 1
run n2 2
run n4 4
run n8 8
run n1_again 1
run n1_disk 1 --workdir disk
run n8_disk 8 --workdir disk
run n1_disk_after 1 --workdir disk
