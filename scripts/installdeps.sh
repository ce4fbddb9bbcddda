#!/usr/bin/env bash
# Report (and where possible explain how to install) the optional tools
# move2kube_amd shells out to (reference scripts/installdeps.sh).
#   docker / podman   CNB detection, `collect` image inspection
#   pack              CNB builds/detection fallback
#   kubectl / oc      `collect` cluster metadata
#   cf                `collect` Cloud Foundry apps and buildpacks
#   operator-sdk      Helm-based operator generation
#   ssh-keygen        PEM conversion of private keys for CI/CD git secrets
#   hipcc (ROCm)      building the gfx950 fuzzy-matching kernel
set -uo pipefail
missing=0
for tool in docker podman pack kubectl oc cf operator-sdk ssh-keygen hipcc g++; do
  if command -v "$tool" >/dev/null 2>&1; then
    printf '  %-13s %s\n' "$tool" "$(command -v "$tool")"
  else
    printf '  %-13s MISSING\n' "$tool"
    missing=$((missing + 1))
  fi
done
python3 - <<'PY'
import importlib
for m in ("yaml", "numpy", "pybind11", "torch"):
    try:
        importlib.import_module(m)
        print("  %-13s ok" % ("py:" + m))
    except Exception:
        print("  %-13s MISSING" % ("py:" + m))
PY
echo "${missing} optional tool(s) missing; every one of them is only needed by the feature listed above."
