# A/B of warm in-process steps on the GPU box: ENV_A vs ENV_B, interleaved, 5 rounds each
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${RUN:-ab}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  env ${ENV_A:-M2K_AB=a} timeout -k 10 120 python -u scripts/profile_step.py ${CONFIG:-helm-openshift} tottime 40 2>&1 | sed -n 1p | sed "s/^/A /" >> $OUT/ab.txt
  env ${ENV_B:-M2K_AB=b} timeout -k 10 120 python -u scripts/profile_step.py ${CONFIG:-helm-openshift} tottime 40 2>&1 | sed -n 1p | sed "s/^/B /" >> $OUT/ab.txt
done
cat $OUT/ab.txt
