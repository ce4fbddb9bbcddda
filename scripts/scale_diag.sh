# Diagnose weak-scaling contention of bench.py on the box's CPUs (gloo, no GPU):
# the same 8-rank run three times, with process/load snapshots in between.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-scalediag}
mkdir -p $OUT
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES=
snap() {
  echo "== $1: $(cat /proc/loadavg)" >> $OUT/snap.txt
  ps -eo pid,ppid,stat,pcpu,etimes,comm --sort=-pcpu | head -15 >> $OUT/snap.txt
  grep -E "usage_usec|system_usec|throttled_usec" /sys/fs/cgroup/cpu.stat >> $OUT/snap.txt 2>/dev/null || true
  ls /tmp | wc -l >> $OUT/snap.txt
}
run() {  # name n extra-env...
  name=$1; n=$2; shift 2
  env "$@" timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 200)) scripts/bench_diag.py --gpus $n --steps 20 --warmup 3 --check-runs 0 $CFG > $OUT/$name.log 2>&1
  echo "$name $(grep metric $OUT/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["phase_ms_one_step"].get("translate"))')"
  grep "^rank" $OUT/$name.log | sort | head -2 | sed "s/^/  /"
}
snap start
CFG="" run ho_n8_a 8 M2K_X=1
snap after_a
sleep 5
snap after_sleep
CFG="" run ho_n8_b 8 M2K_X=1
snap after_b
CFG="" run ho_n8_c 8 M2K_X=1
snap after_c
