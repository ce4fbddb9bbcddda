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
from .common import go_scan_lines, go_trim_space

MARKER_CERT = "@cert-authority"
MARKER_REVOKED = "@revoked"

class KnownHostsError(ValueError):
    pass


def go_std_b64decode(s):
    """``base64.StdEncoding.DecodeString`` (Go 1.15 ``decodeQuantum``): padded,
    CR and LF skipped, anything else outside the alphabet is
    ``illegal base64 data at input byte N``."""
    src = s.encode("utf-8", errors="surrogateescape") if isinstance(s, str) else bytes(s)
    n = len(src)

    def corrupt(i):
        return KnownHostsError("illegal base64 data at input byte %d" % i)
    out = bytearray()
    si = 0
    while True:
        dbuf = [0, 0, 0, 0]
        dlen, j, end = 4, 0, False
        while j < 4:
            if si == n:
                if j == 0:
                    return bytes(out)
                raise corrupt(si - j)
            c = src[si]
            si += 1
            v = _B64_DECODE[c]
            if v >= 0:
                dbuf[j] = v
                j += 1
                continue
            if c in (10, 13):                      # '\n', '\r'
                continue
            if c != 61 or j in (0, 1):             # not '=', or padding too early
                raise corrupt(si - 1)
            if j == 2:                             # "==" expected
                while si < n and src[si] in (10, 13):
                    si += 1
                if si == n:
                    raise corrupt(n)
                if src[si] != 61:
                    raise corrupt(si - 1)
                si += 1
            while si < n and src[si] in (10, 13):
                si += 1
            if si < n:
                raise corrupt(si)                  # trailing garbage
            dlen, end = j, True
            break
        val = dbuf[0] << 18 | dbuf[1] << 12 | dbuf[2] << 6 | dbuf[3]
        out += bytes(((val >> 16) & 0xFF, (val >> 8) & 0xFF, val & 0xFF))[:dlen - 1]
        if end:
            return bytes(out)


_B64_DECODE = [-1] * 256
for _i, _c in enumerate(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"):
    _B64_DECODE[_c] = _i

# crypto/elliptic curve parameters (p, b, byte length): elliptic.Unmarshal's
# on-curve check
_CURVES = {
    "nistp256": (0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff,
                 0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b, 32),
    "nistp384": (0xfffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffeffffffff0000000000000000ffffffff,
                 0xb3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef,
                 48),
    "nistp521": ((1 << 521) - 1,
                 0x0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1bf073573df883d2c34f1ef451fd46b503f00,
                 66),
}


def _ssh_string(b, i):
    if len(b) - i < 4:
        raise KnownHostsError("ssh: short read")
    n = int.from_bytes(b[i:i + 4], "big")
    if len(b) - i - 4 < n:
        raise KnownHostsError("ssh: short read")
    return b[i + 4:i + 4 + n], i + 4 + n


def _ssh_mpint(b, i):
    v, i = _ssh_string(b, i)
    x = int.from_bytes(v, "big")
    if v and v[0] & 0x80:
        x -= 1 << (8 * len(v))
    return x, i


def _ec_point(curve, point):
    """elliptic.Unmarshal: an uncompressed point, coordinates below p, on the
    curve y^2 = x^3 - 3x + b."""
    p, b, size = _CURVES[curve]
    if len(point) != 1 + 2 * size or point[0] != 4:
        raise KnownHostsError("ssh: invalid curve point")
    x = int.from_bytes(point[1:1 + size], "big")
    y = int.from_bytes(point[1 + size:], "big")
    if x >= p or y >= p or (y * y - (x * x * x - 3 * x + b)) % p:
        raise KnownHostsError("ssh: invalid curve point")


def parse_public_key(raw):
    """``ssh.ParsePublicKey`` (golang.org/x/crypto/ssh keys.go) of the wire
    form of an RSA, DSA, ECDSA, Ed25519 or security-key public key, with its
    error texts.  Certificate types are not parsed here (``unknown key
    algorithm``; parity unpinned for them)."""
    algo, i = _ssh_string(raw, 0)
    algo = algo.decode("utf-8", errors="surrogateescape")
    if algo == "ssh-rsa":
        e, i = _ssh_mpint(raw, i)
        _, i = _ssh_mpint(raw, i)
        if e.bit_length() > 24:
            raise KnownHostsError("ssh: exponent too large")
        if e < 3 or e & 1 == 0:
            raise KnownHostsError("ssh: incorrect exponent")
    elif algo == "ssh-dss":
        for _ in range(4):
            _, i = _ssh_mpint(raw, i)
    elif algo in ("ecdsa-sha2-nistp256", "ecdsa-sha2-nistp384", "ecdsa-sha2-nistp521",
                  "sk-ecdsa-sha2-nistp256@openssh.com"):
        curve, i = _ssh_string(raw, i)
        point, i = _ssh_string(raw, i)
        if algo.startswith("sk-"):
            _, i = _ssh_string(raw, i)             # application
            if curve != b"nistp256":
                raise KnownHostsError("ssh: unsupported curve")
        curve = curve.decode("latin-1")
        if curve not in _CURVES:
            raise KnownHostsError("ssh: unsupported curve")
        _ec_point(curve, point)
    elif algo in ("ssh-ed25519", "sk-ssh-ed25519@openssh.com"):
        key, i = _ssh_string(raw, i)
        if algo.startswith("sk-"):
            _, i = _ssh_string(raw, i)
        if len(key) != 32:
            raise KnownHostsError("invalid size %d for Ed25519 public key" % len(key))
    else:
        raise KnownHostsError("ssh: unknown key algorithm: %s" % algo)
    if i < len(raw):
        raise KnownHostsError("ssh: trailing junk in public key")


def _next_word(line):
    """``nextWord``: up to the first space or tab, and the trimmed rest."""
    cut = [k for k in (line.find(" "), line.find("\t")) if k >= 0]
    if not cut:
        return line, ""
    k = min(cut)
    return line[:k], go_trim_space(line[k:])


def parse_known_hosts_line(line):
    """(should_ignore, host, line) - ``parseKnownHostsLine`` (knownhosts.go:48-80)."""
    ignore = False
    w, rest = _next_word(line)
    if w in (MARKER_CERT, MARKER_REVOKED):
        ignore = True
    else:
        rest = line
    host, rest = _next_word(rest)
    if not rest:
        raise KnownHostsError("knownhosts: missing host pattern")
    _, rest = _next_word(rest)
    if not rest:
        raise KnownHostsError("knownhosts: missing key type pattern")
    blob, _ = _next_word(rest)
    parse_public_key(go_std_b64decode(blob))
    return ignore, host, line


def parse_known_hosts(path):
    """``ParseKnownHosts`` (knownhosts.go:84-121): host -> key lines.  Lines
    are split as ``bufio.Scanner`` splits them (LF; a CR before it dropped; a
    line of 64 KiB or more ends the scan with ``token too long``)."""
    with open(path, "rb") as f:
        data = f.read()
    out = {}
    lines, too_long = go_scan_lines(data)
    for n, raw in enumerate(lines, 1):
        line = go_trim_space(raw.decode("utf-8", errors="surrogateescape"))
        if not line or line.startswith("#"):
            continue
        try:
            ignore, host, text = parse_known_hosts_line(line)
        except KnownHostsError as e:
            raise KnownHostsError("Error occurred parsing known_hosts file at path %s on line no. %d Error: %s"
                                  % (log.go_quote(path), n, log.go_quote(str(e))))
        if ignore or host.startswith("|"):
            continue
        for h in host.split(","):
            if h:
                out.setdefault(h, []).append(text)
    if too_long:
        raise KnownHostsError("bufio.Scanner: token too long")
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
