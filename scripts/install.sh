#!/usr/bin/env bash
# Install move2kube_amd from a release (reference scripts/install.sh:27-235).
#
#   install.sh [latest | <tag> | <archive.tar.gz>] [prefix]
#
#   latest (default)   resolve the newest release tag from the release page
#   <tag>              a pinned release, e.g. v0.3.1
#   <archive.tar.gz>   an archive already on disk (its .sha256sum next to it
#                      is checked when present)
#
# Environment (the reference's knobs, plus a mirrorable release location):
#   MOVE2KUBE_RELEASE_URL   release page base (default: the project's GitHub
#                           releases); archives are fetched from
#                           $MOVE2KUBE_RELEASE_URL/download/<tag>/<archive>
#   MOVE2KUBE_INSTALL_PREFIX  install prefix (default /usr/local; the second
#                           argument wins): the tree goes to
#                           <prefix>/lib/move2kube-amd, the launcher to
#                           <prefix>/bin/move2kube
#   USE_SUDO=true           use sudo for the install steps, and only when the
#                           prefix is not writable by the current user
#   VERIFY_CHECKSUM=true    check the archive's sha256 (sha256sum, or openssl)
#   BINARY_NAME=move2kube   DEBUG=false
#
# Downloads with curl, or wget when curl is missing.  Exits non-zero, saying
# why, on an unsupported OS/arch, a missing download tool, a failed download
# or a checksum mismatch; nothing is installed then.

[[ $DEBUG ]] || DEBUG='false'
[[ $BINARY_NAME ]] || BINARY_NAME='move2kube'
[[ $USE_SUDO ]] || USE_SUDO='true'
[[ $VERIFY_CHECKSUM ]] || VERIFY_CHECKSUM='true'
[[ $MOVE2KUBE_RELEASE_URL ]] || MOVE2KUBE_RELEASE_URL='https://github.com/rahulansible72/move2kube-amd/releases'
[[ $MOVE2KUBE_INSTALL_PREFIX ]] || MOVE2KUBE_INSTALL_PREFIX='/usr/local'

REQUEST="${1:-latest}"
PREFIX="${2:-$MOVE2KUBE_INSTALL_PREFIX}"
TAG=''
ARCHIVE_PATH=''
SUM_PATH=''

has() { type "$1" &>/dev/null && echo true || echo false; }
HAS_CURL="$(has curl)"
HAS_WGET="$(has wget)"
HAS_OPENSSL="$(has openssl)"
HAS_SHA256SUM="$(has sha256sum)"

initArch() {
    ARCH="$(uname -m)"
    case $ARCH in
    armv5*) ARCH="armv5" ;;
    armv6*) ARCH="armv6" ;;
    armv7*) ARCH="arm" ;;
    aarch64) ARCH="arm64" ;;
    x86) ARCH="386" ;;
    x86_64) ARCH="amd64" ;;
    i686) ARCH="386" ;;
    i386) ARCH="386" ;;
    esac
}

initOS() {
    OS="$(uname | tr '[:upper:]' '[:lower:]')"
    case "$OS" in
    mingw*) OS='windows' ;;
    esac
}

# The archives carry native libraries built for Linux on x86-64.
verifySupported() {
    local supported="linux-amd64"
    if ! echo "${supported}" | grep -q "${OS}-${ARCH}"; then
        echo "No prebuilt archive for ${OS}-${ARCH}."
        echo "To build from source: make build && make dist"
        exit 1
    fi
    if [ -z "$ARCHIVE_PATH" ] && [ "${HAS_CURL}" != "true" ] && [ "${HAS_WGET}" != "true" ]; then
        echo "Either curl or wget is required"
        exit 1
    fi
    if [ "${VERIFY_CHECKSUM}" == "true" ] && [ "${HAS_OPENSSL}" != "true" ] && [ "${HAS_SHA256SUM}" != "true" ]; then
        echo "In order to verify checksum, sha256sum or openssl must first be installed."
        echo "Please install sha256sum or openssl or set VERIFY_CHECKSUM=false in your environment."
        exit 1
    fi
}

# fetch URL [FILE]: the body to FILE (or stdout); non-zero on an HTTP error.
fetch() {
    if [ "${HAS_CURL}" == "true" ]; then
        if [ -n "${2:-}" ]; then curl -fsSL -o "$2" "$1"; else curl -fsSL "$1"; fi
    else
        if [ -n "${2:-}" ]; then wget -q -O "$2" "$1"; else wget -q -O - "$1"; fi
    fi
}

# getLatestVersion: the first release tag linked from the release page.
getLatestVersion() {
    local page
    if ! page="$(fetch "$MOVE2KUBE_RELEASE_URL")"; then
        echo "Unable to read the release page ${MOVE2KUBE_RELEASE_URL}"
        exit 1
    fi
    TAG="$(printf '%s\n' "$page" | grep -o 'releases/tag/v[^"<> ]*' | head -n 1 | sed 's|.*/||')"
    if [ -z "$TAG" ]; then
        echo "No release tag found at ${MOVE2KUBE_RELEASE_URL}"
        exit 1
    fi
}

# checkInstalledVersion: 0 when the installed move2kube already is $TAG.
checkInstalledVersion() {
    local bin="$PREFIX/bin/$BINARY_NAME"
    if [ -x "$bin" ] || type "$BINARY_NAME" &>/dev/null; then
        [ -x "$bin" ] || bin="$BINARY_NAME"
        local version
        version="$("$bin" version 2>/dev/null)" || version=''
        if [[ "$version" == "$TAG" ]]; then
            echo "Move2Kube ${version} is already the latest"
            return 0
        fi
        if [ -n "$version" ]; then
            echo "Move2Kube ${TAG} is available. Changing from version ${version}."
        fi
    fi
    return 1
}

downloadFile() {
    DIST="move2kube-amd-$TAG-$OS-$ARCH.tar.gz"
    DOWNLOAD_URL="$MOVE2KUBE_RELEASE_URL/download/$TAG/$DIST"
    TMP_ROOT="$(mktemp -d -t move2kube-installer-XXXXXX)"
    ARCHIVE_PATH="$TMP_ROOT/$DIST"
    SUM_PATH="$ARCHIVE_PATH.sha256sum"
    echo "Downloading $DOWNLOAD_URL"
    if [ "${VERIFY_CHECKSUM}" == "true" ] && ! fetch "$DOWNLOAD_URL.sha256sum" "$SUM_PATH"; then
        echo "Unable to download $DOWNLOAD_URL.sha256sum"
        exit 1
    fi
    if ! fetch "$DOWNLOAD_URL" "$ARCHIVE_PATH"; then
        echo "Unable to download $DOWNLOAD_URL"
        exit 1
    fi
}

verifyChecksum() {
    if [ "${VERIFY_CHECKSUM}" != "true" ]; then
        return 0
    fi
    if [ ! -f "$SUM_PATH" ]; then
        echo "warning: no checksum file next to ${ARCHIVE_PATH}; skipping verification" >&2
        return 0
    fi
    printf "Verifying checksum... "
    local expected sum
    expected="$(awk '{print $1}' <"$SUM_PATH")"
    if [ "$HAS_SHA256SUM" == "true" ]; then
        sum="$(sha256sum "$ARCHIVE_PATH" | awk '{print $1}')"
    else
        sum="$(openssl sha1 -sha256 "$ARCHIVE_PATH" | awk '{print $NF}')"
    fi
    if [ "$sum" != "$expected" ]; then
        echo "SHA sum of ${ARCHIVE_PATH} does not match. Aborting."
        exit 1
    fi
    echo "Done."
}

# writable DIR: DIR (or the first existing parent) is writable by this user.
writable() {
    local d="$1"
    while [ ! -e "$d" ]; do d="$(dirname "$d")"; done
    [ -w "$d" ]
}

# runAsRoot CMD...: sudo only when the prefix is not writable and USE_SUDO allows it.
runAsRoot() {
    if [ "$NEED_SUDO" == "true" ]; then
        sudo "$@"
    else
        "$@"
    fi
}

installFile() {
    NEED_SUDO=false
    if [ "$(id -u)" != "0" ] && [ "$USE_SUDO" == "true" ] && ! writable "$PREFIX"; then
        NEED_SUDO=true
    fi
    local dest="$PREFIX/lib/move2kube-amd"
    echo "Preparing to install $BINARY_NAME into ${PREFIX}"
    runAsRoot mkdir -p "$PREFIX/lib" "$PREFIX/bin"
    runAsRoot rm -rf "$dest.new"
    runAsRoot mkdir -p "$dest.new"
    runAsRoot tar -xzf "$ARCHIVE_PATH" -C "$dest.new" --strip-components=1
    runAsRoot rm -rf "$dest"
    runAsRoot mv "$dest.new" "$dest"
    runAsRoot ln -sf "$dest/bin/move2kube" "$PREFIX/bin/$BINARY_NAME"
    # byte-compile once at install time: a fresh tree otherwise recompiles every
    # module on each (read-only) run, which more than doubles CLI start-up
    runAsRoot python3 -m compileall -q -j 0 "$dest/move2kube_amd" >/dev/null ||
        echo "warning: byte-compilation failed; start-up will be slower" >&2
    if ! python3 -c "import yaml, numpy" 2>/dev/null; then
        echo "warning: python3 with pyyaml and numpy is required" >&2
    fi
    echo "Successfully installed $BINARY_NAME into $PREFIX/bin/$BINARY_NAME"
}

testVersion() {
    if ! "$PREFIX/bin/$BINARY_NAME" version; then
        echo "$PREFIX/bin/$BINARY_NAME does not run"
        exit 1
    fi
    if ! command -v "$BINARY_NAME" >/dev/null; then
        echo "$BINARY_NAME not found. Is $PREFIX/bin on your "'$PATH?'
    fi
}

cleanup() {
    if [[ -d "${TMP_ROOT:-}" ]]; then
        rm -rf "$TMP_ROOT"
    fi
}

fail_trap() {
    result=$?
    if [ "$result" != "0" ]; then
        echo "Failed to install $BINARY_NAME"
        echo -e "\tFor support, see README.md"
    fi
    cleanup
    exit $result
}

main() {
    echo 'Installing move2kube'
    case "$REQUEST" in
    *.tar.gz)
        ARCHIVE_PATH="$REQUEST"
        [ -f "$ARCHIVE_PATH.sha256sum" ] && SUM_PATH="$ARCHIVE_PATH.sha256sum"
        ;;
    latest) ;;
    *) TAG="$REQUEST" ;;
    esac
    initArch
    initOS
    verifySupported
    if [ -n "$ARCHIVE_PATH" ]; then
        if [ ! -f "$ARCHIVE_PATH" ]; then
            echo "No archive at $ARCHIVE_PATH"
            exit 1
        fi
        verifyChecksum
        installFile
    else
        [ -n "$TAG" ] || getLatestVersion
        if ! checkInstalledVersion; then
            downloadFile
            verifyChecksum
            installFile
        fi
    fi
    testVersion
    echo 'Done!'
}

trap "fail_trap" EXIT
set -e
set -u
if [ "${DEBUG}" == "true" ]; then
    set -x
fi

main
