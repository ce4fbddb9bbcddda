#!/usr/bin/env bash
# Install move2kube_amd from a release archive (reference scripts/install.sh).
#   install.sh <archive.tar.gz> [prefix]      default prefix: /usr/local
# Verifies the archive against its .sha256sum (when present next to it), unpacks
# it under <prefix>/lib/move2kube-amd and links <prefix>/bin/move2kube.
set -euo pipefail

archive="${1:?usage: install.sh <archive.tar.gz> [prefix]}"
prefix="${2:-/usr/local}"

if [ -f "${archive}.sha256sum" ]; then
  (cd "$(dirname "$archive")" && sha256sum -c "$(basename "$archive").sha256sum")
else
  echo "warning: no checksum file next to ${archive}; skipping verification" >&2
fi

dest="${prefix}/lib/move2kube-amd"
mkdir -p "$dest" "${prefix}/bin"
tar -xzf "$archive" -C "$dest" --strip-components=1
ln -sf "${dest}/bin/move2kube" "${prefix}/bin/move2kube"
# byte-compile once at install time: a fresh tree otherwise recompiles every
# module on each (read-only) run, which more than doubles CLI start-up
python3 -m compileall -q -j 0 "${dest}/move2kube_amd" >/dev/null || \
  echo "warning: byte-compilation failed; start-up will be slower" >&2
if ! python3 -c "import yaml, numpy" 2>/dev/null; then
  echo "warning: python3 with pyyaml and numpy is required" >&2
fi
echo "installed: ${prefix}/bin/move2kube -> ${dest}"
"${prefix}/bin/move2kube" version
