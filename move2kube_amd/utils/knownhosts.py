"""SSH known_hosts parsing and host-key retrieval (reference
``internal/common/knownhosts/knownhosts.go``).

``get_known_hosts_line`` fetches a host's public key by starting an SSH
handshake to port 22, as ``GetKey`` does: in process (``utils/sshwire.py``:
the transport up to the verified key-exchange reply), with the
``ssh-keyscan`` tool as the fallback when that fails.  Network access is
bounded by a short timeout and can be disabled with ``M2K_NO_NETWORK=1``.
"""

import base64
import os
import shutil

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


# golang.org/x/crypto/ssh supportedHostKeyAlgos (plain keys): the client offers
# these in this order and the server picks the first one it has, so this is
# the key ``GetKey`` (knownhosts.go:137-155) ends up with.
GO_HOST_KEY_ORDER = ("ecdsa-sha2-nistp256", "ecdsa-sha2-nistp384", "ecdsa-sha2-nistp521", "ssh-rsa", "ssh-dss",
                     "ssh-ed25519")


def pick_host_key_line(lines, host):
    """From ``ssh-keyscan`` output, the line for the key a Go ssh client would
    negotiate, as ``knownhosts.Line([host], key)`` writes it: ``host algo key``."""
    best = None
    for line in lines:
        parts = line.split()
        if len(parts) < 3 or line.startswith("#") or parts[1] not in GO_HOST_KEY_ORDER:
            continue
        rank = GO_HOST_KEY_ORDER.index(parts[1])
        if best is None or rank < best[0]:
            best = (rank, "%s %s %s" % (host, parts[1], parts[2]))
    return best[1] if best else ""


def fetch_line_in_process(host, timeout=5, port=22):
    """``knownhosts.Line([host], key)`` for the key ``host`` proves it holds in
    an SSH key exchange (``GetKey``, knownhosts.go:137-155), or '' on failure."""
    from . import sshwire
    try:
        ktype, blob = sshwire.fetch_host_key(host, port=port, timeout=timeout)
    except (OSError, sshwire.SSHError, ValueError) as e:
        log.debug("In-process ssh handshake with %s failed : %s", host, e)
        return ""
    log.debug("host %s on port %d has the key of type %s", host, port, ktype)
    return "%s %s %s" % (host, ktype, base64.b64encode(blob).decode("ascii"))


def get_known_hosts_line(host, timeout=5):
    """``host algo base64key`` for the host, or '' when it cannot be fetched.
    The key is the one a Go client would negotiate (:data:`GO_HOST_KEY_ORDER`),
    fetched in process; ``ssh-keyscan`` (every key type scanned, the same one
    kept) is the fallback."""
    if os.environ.get("M2K_NO_NETWORK"):
        log.debug("Cannot fetch the ssh host key of %s (network disabled)", host)
        return ""
    line = fetch_line_in_process(host, timeout)
    if line:
        return line
    if shutil.which("ssh-keyscan") is None:
        log.debug("Cannot fetch the ssh host key of %s (handshake failed, no ssh-keyscan)", host)
        return ""
    import subprocess
    try:
        p = subprocess.run(["ssh-keyscan", "-T", str(timeout), "-t", "rsa,ecdsa,ed25519,dsa", host],
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, stdin=subprocess.DEVNULL,
                           timeout=timeout + 2)
    except (OSError, subprocess.SubprocessError):
        return ""
    return pick_host_key_line(p.stdout.decode("utf-8", "replace").splitlines(), host)
