# Interleaved cold traces and import times of one configuration, HEAD vs an
# A/B base tree under .ab_base/ (benchmarks/cold_trace.py, cold_importtime.py):
#   RUN=r05_cc CONFIG=cf BASE=r04 gpurun -- bash scripts/cold_compare.sh
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-cold_compare}
mkdir -p "$OUT"
export TMPDIR=/tmp
C=${CONFIG:-cf}
for i in 1 2 3; do
  for t in head base; do
    extra=""; [ "$t" = base ] && extra="--tree .ab_base/${BASE:-r04}"
    echo "trace $C $t $i"
    timeout -k 10 180 python -u benchmarks/cold_trace.py "$C" --runs 11 $extra | sed "s/^{/{\"tree\": \"$t\", /" >> "$OUT/cold_trace.jsonl"
  done
done
for t in head base; do
  extra=""; [ "$t" = base ] && extra="--tree .ab_base/${BASE:-r04}"
  timeout -k 10 180 python -u benchmarks/cold_importtime.py "$C" --runs 9 $extra | sed "s/^{/{\"tree\": \"$t\", /" >> "$OUT/cold_importtime.jsonl"
done
echo done
