#!/usr/bin/env bash
# End-to-end check of a built image (CI job `image`; the reference's
# build.yml hands its image to an external test repository instead):
# `translate --qaskip` of the whole samples/ corpus to a Helm chart for the
# Openshift profile inside the container, compared with the expected tree
# tests/golden/reference/helm-openshift.
#
#   scripts/image_e2e.sh <image>
#
# The operator directory is not compared file by file: the expected tree was
# made with the operator-sdk stand-in (DEVIATIONS.md §3), the image carries
# the real tool.  It must exist and hold the PROJECT file operator-sdk writes.
#
# M2K_E2E_RUNNER replaces `docker run ... <image>` (the test suite runs this
# script with the CLI on the host: M2K_E2E_RUNNER="python3 -m move2kube_amd").
set -euo pipefail

ROOT="$(cd "$(dirname "$0")/.." && pwd)"
IMAGE="${1:-}"
if [ -z "${M2K_E2E_RUNNER:-}" ] && [ -z "$IMAGE" ]; then
  echo "usage: image_e2e.sh <image>" >&2
  exit 2
fi
WORK="$(mktemp -d)"
trap 'rm -rf "$WORK"' EXIT
cp -R "$ROOT/samples" "$WORK/samples"
cp "$ROOT/tests/fixtures/configs/helm-openshift-qacache.yaml" "$WORK/"

ARGS=(translate -s samples --qaskip -q helm-openshift-qacache.yaml -o out)
if [ -n "${M2K_E2E_RUNNER:-}" ]; then
  (cd "$WORK" && M2K_DISABLE_CNB=1 M2K_NO_NETWORK=1 $M2K_E2E_RUNNER "${ARGS[@]}") > "$WORK/translate.log" 2>&1 || {
    tail -20 "$WORK/translate.log"; exit 1; }
else
  docker run --rm -u "$(id -u):$(id -g)" -e HOME=/tmp -e M2K_DISABLE_CNB=1 -e M2K_NO_NETWORK=1 \
    -v "$WORK:/wksps" "$IMAGE" "${ARGS[@]}" > "$WORK/translate.log" 2>&1 || {
    tail -20 "$WORK/translate.log"; exit 1; }
fi

OUT="$WORK/out/myproject"  # translate writes <-o>/<project name>
if [ ! -f "$OUT/myproject-operator/PROJECT" ]; then
  echo "FAIL: operator-sdk did not run (no myproject-operator/PROJECT)"
  grep -i operator "$WORK/translate.log" || true
  exit 1
fi
python3 - "$OUT" "$ROOT" <<'PY'
import sys
sys.path.insert(0, sys.argv[2] + "/benchmarks")
import refconfigs
bad = [p for p in refconfigs.diff_files(sys.argv[1], refconfigs.golden_dir("helm-openshift"))
       if not p.startswith("myproject-operator/")]
for p in bad:
    print("differs:", p)
print("%d files differ from tests/golden/reference/helm-openshift (operator directory excluded)" % len(bad))
sys.exit(1 if bad else 0)
PY
