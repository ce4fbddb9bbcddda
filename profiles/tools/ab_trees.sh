# A/B of warm in-process steps on the GPU box: the tree in .ab_base (A, an
# older revision unpacked by the caller) vs this tree (B), interleaved.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-abtrees}
mkdir -p $OUT
export TMPDIR=/dev/shm
for i in 1 2 3 4 5; do
  GRAFT_REPO_ROOT=$PWD/.ab_base timeout -k 10 120 python -u .ab_base/scripts/profile_step.py ${CONFIG:-helm-openshift} tottime 40 2>&1 | sed -n 1p | sed "s/^/A /" >> $OUT/ab.txt
  timeout -k 10 120 python -u scripts/profile_step.py ${CONFIG:-helm-openshift} tottime 40 2>&1 | sed -n 1p | sed "s/^/B /" >> $OUT/ab.txt
done
cat $OUT/ab.txt
