"""SSH known_hosts parsing and host-key retrieval (reference
``internal/common/knownhosts/knownhosts.go``).

``get_known_hosts_line`` fetches a host's public key by starting an SSH
handshake to port 22 (as user ``git``) - done here with the ``ssh-keyscan``
tool when available, since no SSH library ships with the runtime.  Network
access is bounded by a short timeout and can be disabled with
``M2K_NO_NETWORK=1``.
"""

import base64
import os
import shutil
import subprocess

from . import log

MARKER_CERT = "@cert-authority"
MARKER_REVOKED = "@revoked"

_KEY_TYPES = {"ssh-rsa", "ssh-dss", "ssh-ed25519", "ecdsa-sha2-nistp256", "ecdsa-sha2-nistp384",
              "ecdsa-sha2-nistp521", "sk-ssh-ed25519@openssh.com", "sk-ecdsa-sha2-nistp256@openssh.com"}


class KnownHostsError(ValueError):
    pass


def _valid_key_blob(blob):
    try:
        raw = base64.b64decode(blob, validate=True)
    except ValueError:
        return False
    if len(raw) < 4:
        return False
    n = int.from_bytes(raw[:4], "big")
    if n <= 0 or 4 + n > len(raw):
        return False
    return raw[4:4 + n].decode("ascii", "replace") in _KEY_TYPES


def parse_known_hosts_line(line):
    """(should_ignore, host, line)."""
    parts = line.split()
    ignore = False
    if parts and parts[0] in (MARKER_CERT, MARKER_REVOKED):
        ignore = True
        parts = parts[1:]
    if len(parts) < 2:
        raise KnownHostsError("knownhosts: missing host pattern")
    if len(parts) < 3:
        raise KnownHostsError("knownhosts: missing key type pattern")
    if not _valid_key_blob(parts[2]):
        raise KnownHostsError("knownhosts: invalid key blob")
    return ignore, parts[0], line


def parse_known_hosts(path):
    out = {}
    with open(path) as f:
        for n, raw in enumerate(f, 1):
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            try:
                ignore, host, text = parse_known_hosts_line(line)
            except KnownHostsError as e:
                raise KnownHostsError("Error occurred parsing known_hosts file at path %r on line no. %d Error: %r" % (path, n, str(e)))
            if ignore or host.startswith("|"):
                continue
            for h in host.split(","):
                if h:
                    out.setdefault(h, []).append(text)
    return out


def get_known_hosts_line(host, timeout=5):
    """``host algo base64key`` for the host, or '' when it cannot be fetched."""
    if os.environ.get("M2K_NO_NETWORK") or shutil.which("ssh-keyscan") is None:
        log.debug("Cannot fetch the ssh host key of %s (no ssh-keyscan or network disabled)", host)
        return ""
    try:
        p = subprocess.run(["ssh-keyscan", "-T", str(timeout), "-t", "rsa", host], stdout=subprocess.PIPE,
                           stderr=subprocess.DEVNULL, timeout=timeout + 2)
    except (OSError, subprocess.TimeoutExpired):
        return ""
    for line in p.stdout.decode("utf-8", "replace").splitlines():
        line = line.strip()
        if line and not line.startswith("#"):
            return line
    return ""
