#!/usr/bin/env bash
# Install the external tools move2kube_amd drives (reference:
# scripts/installdeps.sh, which the reference's image build runs with -y).
#
#   installdeps.sh [-y] [--check]
#
#   -y        no prompts: install everything missing and put the install
#             directory at the front of PATH in ~/.bash_profile (run with sudo when docker is wanted)
#   --check   only report what is present / missing, install nothing
#
# Tools and what uses them:
#   docker          CNB detection (socket or CLI), `collect` image inspection
#   pack            CNB detection fallback
#   kubectl         `collect` cluster metadata
#   operator-sdk    the Helm chart's operator (`translate`, Helm artifacts);
#                   must be a v1 release - an older one is replaced
#
# Everything goes to $MOVE2KUBE_DEP_INSTALL_PATH (default: ./bin).  Versions and
# download locations can be pinned or pointed at a mirror:
#   PACK_VERSION (v0.12.0)          PACK_URL
#   KUBECTL_VERSION (stable.txt)    KUBECTL_URL
#   OPERATOR_SDK_VERSION (v1.0.0)   OPERATOR_SDK_URL
#   INSTALL_DOCKER=0                never run the docker convenience script
#   FORCE_INSTALL=1                 install pack, kubectl and operator-sdk into
#                                   the install directory even when PATH has
#                                   them (the image build copies all three)
set -eu

QUIET=false
CHECK_ONLY=false
for arg in "$@"; do
  case "$arg" in
    -y) QUIET=true ;;
    --check) CHECK_ONLY=true ;;
    *)
      echo "Invalid args: $*"
      echo "Usage: installdeps.sh [-y] [--check]"
      exit 1 ;;
  esac
done

DEST="${MOVE2KUBE_DEP_INSTALL_PATH:-$PWD/bin}"
PACK_VERSION="${PACK_VERSION:-v0.12.0}"
OPERATOR_SDK_VERSION="${OPERATOR_SDK_VERSION:-v1.0.0}"
INSTALL_DOCKER="${INSTALL_DOCKER:-1}"
FORCE_INSTALL="${FORCE_INSTALL:-0}"

have() { command -v "$1" >/dev/null 2>&1; }

# present <tool>: on PATH and not to be (re)installed into $DEST
present() { [ "$FORCE_INSTALL" != 1 ] && have "$1"; }

# operator-sdk v0 cannot scaffold a Helm operator with `init --plugins=helm`
sdk_is_v1() {
  have operator-sdk || return 1
  operator-sdk version 2>/dev/null | cut -d, -f1 | grep -q 'operator-sdk version: "v1'
}

in_container() {
  [ -f /.dockerenv ] || [ -f /run/.containerenv ] || grep -qs container_t /proc/1/attr/current
}

report() {
  local missing=0 t
  for t in docker pack kubectl operator-sdk; do
    if have "$t"; then
      printf '  %-13s %s\n' "$t" "$(command -v "$t")"
    else
      printf '  %-13s MISSING\n' "$t"
      missing=$((missing + 1))
    fi
  done
  if have operator-sdk && ! sdk_is_v1; then
    echo "  operator-sdk is not a v1 release; Helm operators will not be generated"
  fi
  echo "${missing} tool(s) missing; each is needed only by the feature listed in the header of this script."
}

if [ "$CHECK_ONLY" = true ]; then
  report
  exit 0
fi

WORK=""
on_exit() {
  local rc=$?
  [ -n "$WORK" ] && rm -rf "$WORK"
  if [ "$rc" != 0 ]; then
    echo "Failed to install the dependencies (exit status $rc)."
  fi
}
trap on_exit EXIT

OS="$(uname -s | tr '[:upper:]' '[:lower:]')"
case "$(uname -m)" in
  x86_64 | amd64) ARCH=amd64; SDK_ARCH=x86_64 ;;
  aarch64 | arm64) ARCH=arm64; SDK_ARCH=aarch64 ;;
  *) echo "Unsupported architecture: $(uname -m)"; exit 1 ;;
esac
case "$OS" in
  linux) PACK_OS=linux; SDK_OS=linux-gnu ;;
  darwin) PACK_OS=macos; SDK_OS=apple-darwin
          echo "Install Docker Desktop separately: https://docs.docker.com/docker-for-mac/install/" ;;
  *) echo "Unsupported platform: $OS"; exit 1 ;;
esac

confirm() {  # confirm <question>: yes under -y
  [ "$QUIET" = true ] && return 0
  local reply
  read -r -p "$1 [y/N]: " reply
  [ "$reply" = y ] || [ "$reply" = Y ]
}

echo "move2kube_amd dependencies: docker (Linux only), pack, kubectl, operator-sdk -> $DEST"
if ! confirm "Proceed?"; then
  echo "Not confirmed; nothing installed."
  exit 1
fi
mkdir -p "$DEST"
WORK="$(mktemp -d)"

fetch() {  # fetch <url> <file>
  echo "  GET $1"
  curl -fsSL -o "$2" "$1"
}

if ! have docker && [ "$OS" = linux ] && [ "$INSTALL_DOCKER" != 0 ]; then
  if in_container; then
    echo "Skipping docker: running inside a container (mount the host's /var/run/docker.sock instead)."
  else
    echo "Installing docker..."
    fetch "${DOCKER_SCRIPT_URL:-https://get.docker.com}" "$WORK/get-docker.sh"
    if [ "$QUIET" = true ] || [ "$(id -u)" = 0 ]; then sh "$WORK/get-docker.sh"; else sudo sh "$WORK/get-docker.sh"; fi
  fi
fi

if ! present pack; then
  echo "Installing pack ${PACK_VERSION}..."
  fetch "${PACK_URL:-https://github.com/buildpacks/pack/releases/download/${PACK_VERSION}/pack-${PACK_VERSION}-${PACK_OS}.tgz}" "$WORK/pack.tgz"
  tar -xzf "$WORK/pack.tgz" -C "$WORK"
  install -m 0755 "$WORK/pack" "$DEST/pack"
fi

if ! present kubectl; then
  if [ -z "${KUBECTL_URL:-}" ]; then
    KUBECTL_VERSION="${KUBECTL_VERSION:-$(curl -fsSL https://storage.googleapis.com/kubernetes-release/release/stable.txt)}"
    KUBECTL_URL="https://storage.googleapis.com/kubernetes-release/release/${KUBECTL_VERSION}/bin/${OS}/${ARCH}/kubectl"
  fi
  echo "Installing kubectl ${KUBECTL_VERSION:-}..."
  fetch "$KUBECTL_URL" "$WORK/kubectl"
  install -m 0755 "$WORK/kubectl" "$DEST/kubectl"
fi

if [ "$FORCE_INSTALL" = 1 ] || ! sdk_is_v1; then
  have operator-sdk && ! sdk_is_v1 && echo "operator-sdk on PATH is not v1 ($(command -v operator-sdk)); installing ${OPERATOR_SDK_VERSION} ahead of it"
  echo "Installing operator-sdk ${OPERATOR_SDK_VERSION}..."
  fetch "${OPERATOR_SDK_URL:-https://github.com/operator-framework/operator-sdk/releases/download/${OPERATOR_SDK_VERSION}/operator-sdk-${OPERATOR_SDK_VERSION}-${SDK_ARCH}-${SDK_OS}}" "$WORK/operator-sdk"
  install -m 0755 "$WORK/operator-sdk" "$DEST/operator-sdk"
  if ! "$DEST/operator-sdk" version 2>/dev/null | cut -d, -f1 | grep -q 'operator-sdk version: "v1'; then
    echo "The downloaded operator-sdk does not report a v1 version."
    exit 1
  fi
fi

echo "Installed the dependencies to $DEST"
case ":$PATH:" in
  *":$DEST:"*)
    echo "$DEST is already on \$PATH"
    if [ -x "$DEST/operator-sdk" ] && [ "$(command -v operator-sdk)" != "$DEST/operator-sdk" ]; then
      echo "Warning: $(command -v operator-sdk) comes before $DEST/operator-sdk on \$PATH"
    fi ;;
  *)
    # ahead of the rest of PATH, so a replaced pre-v1 operator-sdk does not shadow the new one
    if confirm "Put $DEST at the front of \$PATH in ~/.bash_profile?"; then
      echo "PATH=\"$DEST:\$PATH\"" >> ~/.bash_profile
      echo "Added $DEST to \$PATH in ~/.bash_profile; open a new shell or source it."
    else
      echo "~/.bash_profile not modified; add $DEST to \$PATH yourself."
    fi ;;
esac
echo "Done."
