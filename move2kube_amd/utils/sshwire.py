"""In-process SSH host-key fetch (reference ``internal/common/knownhosts/knownhosts.go:137-155``).

``GetKey`` there dials ``host:22`` with golang.org/x/crypto/ssh as user ``git``
and no auth methods; the host-key callback records the key the server proved
it holds, and the handshake then fails at authentication.  This module does
the same with the standard library only: the SSH transport (RFC 4253) up to
the server's key-exchange reply, the exchange hash, and the host key's
signature over it, then a disconnect.  Nothing after the key exchange (no
NEWKEYS, no cipher) is needed, so no symmetric crypto is implemented.

Key exchange: ``curve25519-sha256`` (RFC 8731, X25519 per RFC 7748) and
``diffie-hellman-group14-sha256`` / ``-sha1`` (RFC 8268, 4253; ``pow`` over
the 2048-bit MODP group).  Host keys, offered in x/crypto/ssh's order
(``supportedHostKeyAlgos``: ECDSA P-256/384/521, ssh-rsa, ssh-dss, ed25519;
``rsa-sha2-512/256`` follow ssh-rsa so a server that no longer signs with
SHA-1 still answers), are verified: RSA PKCS#1 v1.5, DSA, ECDSA and Ed25519
(RFC 8032) in pure Python.  A server whose signature does not verify gives no
key, as in the reference.
"""

import hashlib
import os
import socket
import struct
import time

CLIENT_VERSION = b"SSH-2.0-Go"  # what x/crypto/ssh sends
KEX_ALGOS = ("curve25519-sha256", "curve25519-sha256@libssh.org", "diffie-hellman-group14-sha256",
             "diffie-hellman-group14-sha1")
HOST_KEY_ALGOS = ("ecdsa-sha2-nistp256", "ecdsa-sha2-nistp384", "ecdsa-sha2-nistp521", "ssh-rsa",
                  "rsa-sha2-512", "rsa-sha2-256", "ssh-dss", "ssh-ed25519")
CIPHERS = ("aes128-gcm@openssh.com", "chacha20-poly1305@openssh.com", "aes128-ctr", "aes192-ctr", "aes256-ctr")
MACS = ("hmac-sha2-256-etm@openssh.com", "hmac-sha2-256", "hmac-sha1")

MSG_DISCONNECT, MSG_IGNORE, MSG_DEBUG = 1, 2, 4
MSG_KEXINIT, MSG_KEXDH_INIT, MSG_KEXDH_REPLY = 20, 30, 31
MAX_PACKET = 256 * 1024
MAX_BANNER_LINES = 1024  # lines before the version line
MAX_SKIPPED = 1024  # IGNORE/DEBUG messages in a row

# RFC 3526 group 14 (2048-bit MODP), generator 2
GROUP14_P = int(
    "FFFFFFFFFFFFFFFFC90FDAA22168C234C4C6628B80DC1CD129024E088A67CC74020BBEA63B139B22514A08798E3404DD"
    "EF9519B3CD3A431B302B0A6DF25F14374FE1356D6D51C245E485B576625E7EC6F44C42E9A637ED6B0BFF5CB6F406B7ED"
    "EE386BFB5A899FA5AE9F24117C4B1FE649286651ECE45B3DC2007CB8A163BF0598DA48361C55D39A69163FA8FD24CF5F"
    "83655D23DCA3AD961C62F356208552BB9ED529077096966D670C354E4ABC9804F1746C08CA18217C32905E462E36CE3B"
    "E39E772C180E86039B2783A2EC07A28FB5C55DF06F4C52C9DE2BCBF6955817183995497CEA956AE515D2261898FA0510"
    "15728E5A8AACAA68FFFFFFFFFFFFFFFF", 16)


class SSHError(Exception):
    pass


# ---------------------------------------------------------------------------
# wire encoding (RFC 4251 §5)
# ---------------------------------------------------------------------------

def ssh_string(b):
    return struct.pack(">I", len(b)) + b


def ssh_mpint(n):
    if n == 0:
        return ssh_string(b"")
    raw = n.to_bytes((n.bit_length() + 8) // 8, "big")  # the extra byte keeps the sign bit clear
    return ssh_string(raw)


def name_list(names):
    return ssh_string(",".join(names).encode())


class Reader:
    def __init__(self, data):
        self.data = data
        self.pos = 0

    def byte(self):
        if self.pos >= len(self.data):
            raise SSHError("short message")
        self.pos += 1
        return self.data[self.pos - 1]

    def raw(self, n):
        if self.pos + n > len(self.data):
            raise SSHError("short message")
        self.pos += n
        return self.data[self.pos - n:self.pos]

    def uint32(self):
        return struct.unpack(">I", self.raw(4))[0]

    def string(self):
        return self.raw(self.uint32())

    def mpint(self):
        b = self.string()
        return int.from_bytes(b, "big", signed=True) if b else 0

    def names(self):
        s = self.string()
        return s.decode("ascii", "replace").split(",") if s else []


# ---------------------------------------------------------------------------
# X25519 (RFC 7748 §5)
# ---------------------------------------------------------------------------

_P25519 = 2 ** 255 - 19


def x25519(scalar, u_bytes):
    k = bytearray(scalar)
    k[0] &= 248
    k[31] &= 127
    k[31] |= 64
    k = int.from_bytes(k, "little")
    u = int.from_bytes(u_bytes, "little") & ((1 << 255) - 1)
    p = _P25519
    x1, x2, z2, x3, z3, swap = u, 1, 0, u, 1, 0
    for t in range(254, -1, -1):
        kt = (k >> t) & 1
        if swap ^ kt:
            x2, x3, z2, z3 = x3, x2, z3, z2
        swap = kt
        a, b = x2 + z2, x2 - z2
        aa, bb = a * a % p, b * b % p
        e = aa - bb
        c, d = x3 + z3, x3 - z3
        da, cb = d * a % p, c * b % p
        x3, z3 = (da + cb) ** 2 % p, x1 * (da - cb) ** 2 % p
        x2, z2 = aa * bb % p, e * (aa + 121665 * e) % p
    if swap:
        x2, z2 = x3, z3
    return (x2 * pow(z2, p - 2, p) % p).to_bytes(32, "little")


X25519_BASE = (9).to_bytes(32, "little")


# ---------------------------------------------------------------------------
# Ed25519 verification (RFC 8032 §5.1.7)
# ---------------------------------------------------------------------------

_ED_L = 2 ** 252 + 27742317777372353535851937790883648493
_ED_D = -121665 * pow(121666, _P25519 - 2, _P25519) % _P25519
_ED_I = pow(2, (_P25519 - 1) // 4, _P25519)


def _ed_recover_x(y, sign):
    p = _P25519
    if y >= p:
        return None
    x2 = (y * y - 1) * pow(_ED_D * y * y + 1, p - 2, p) % p
    if x2 == 0:
        return None if sign else 0
    x = pow(x2, (p + 3) // 8, p)
    if (x * x - x2) % p:
        x = x * _ED_I % p
    if (x * x - x2) % p:
        return None
    if (x & 1) != sign:
        x = p - x
    return x


def _ed_add(P, Q):
    p = _P25519
    x1, y1, z1, t1 = P
    x2, y2, z2, t2 = Q
    a = (y1 - x1) * (y2 - x2) % p
    b = (y1 + x1) * (y2 + x2) % p
    c = 2 * t1 * t2 * _ED_D % p
    d = 2 * z1 * z2 % p
    e, f, g, h = b - a, d - c, d + c, b + a
    return e * f % p, g * h % p, f * g % p, e * h % p


def ed_mul(s, P):
    Q = (0, 1, 1, 0)
    while s:
        if s & 1:
            Q = _ed_add(Q, P)
        P = _ed_add(P, P)
        s >>= 1
    return Q


def _ed_point(x, y):
    return x, y, 1, x * y % _P25519


_ED_BY = 4 * pow(5, _P25519 - 2, _P25519) % _P25519
ED_B = _ed_point(_ed_recover_x(_ED_BY, 0), _ED_BY)


def ed_decompress(b):
    if len(b) != 32:
        return None
    y = int.from_bytes(b, "little")
    sign = y >> 255
    y &= (1 << 255) - 1
    x = _ed_recover_x(y, sign)
    return None if x is None else _ed_point(x, y)


def ed_compress(P):
    p = _P25519
    zi = pow(P[2], p - 2, p)
    x, y = P[0] * zi % p, P[1] * zi % p
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def _ed_equal(P, Q):
    p = _P25519
    return (P[0] * Q[2] - Q[0] * P[2]) % p == 0 and (P[1] * Q[2] - Q[1] * P[2]) % p == 0


def ed25519_verify(pub, msg, sig):
    if len(pub) != 32 or len(sig) != 64:
        return False
    A = ed_decompress(pub)
    R = ed_decompress(sig[:32])
    if A is None or R is None:
        return False
    s = int.from_bytes(sig[32:], "little")
    if s >= _ED_L:
        return False
    h = int.from_bytes(hashlib.sha512(sig[:32] + pub + msg).digest(), "little") % _ED_L
    return _ed_equal(ed_mul(s, ED_B), _ed_add(R, ed_mul(h, A)))


# ---------------------------------------------------------------------------
# ECDSA over the NIST prime curves (a = -3), verification (FIPS 186-4 §6.4.2)
# ---------------------------------------------------------------------------

class Curve:
    def __init__(self, name, p, n, b, gx, gy, hash_fn):
        self.name, self.p, self.n, self.b, self.g, self.hash = name, p, n, b, (gx, gy), hash_fn
        self.size = (p.bit_length() + 7) // 8

    def on_curve(self, P):
        x, y = P
        return 0 <= x < self.p and 0 <= y < self.p and (y * y - (x * x * x - 3 * x + self.b)) % self.p == 0

    # Jacobian coordinates; None is the point at infinity
    def _dbl(self, P):
        if P is None:
            return None
        p = self.p
        X, Y, Z = P
        if Y == 0:
            return None
        zz = Z * Z % p
        m = 3 * (X - zz) * (X + zz) % p
        yy = Y * Y % p
        s = 4 * X * yy % p
        x3 = (m * m - 2 * s) % p
        return x3, (m * (s - x3) - 8 * yy * yy) % p, 2 * Y * Z % p

    def _add(self, P, Q):
        if P is None:
            return Q
        if Q is None:
            return P
        p = self.p
        X1, Y1, Z1 = P
        X2, Y2, Z2 = Q
        z1z1, z2z2 = Z1 * Z1 % p, Z2 * Z2 % p
        u1, u2 = X1 * z2z2 % p, X2 * z1z1 % p
        s1, s2 = Y1 * Z2 * z2z2 % p, Y2 * Z1 * z1z1 % p
        if u1 == u2:
            return self._dbl(P) if s1 == s2 else None
        h, r = (u2 - u1) % p, (s2 - s1) % p
        hh = h * h % p
        hhh = h * hh % p
        v = u1 * hh % p
        x3 = (r * r - hhh - 2 * v) % p
        return x3, (r * (v - x3) - s1 * hhh) % p, Z1 * Z2 * h % p

    def mul_add(self, k1, P1, k2, P2):
        """k1*P1 + k2*P2 in affine coordinates (None at infinity)."""
        J1, J2 = (P1[0], P1[1], 1), (P2[0], P2[1], 1)
        J12 = self._add(J1, J2)
        R = None
        for i in range(max(k1.bit_length(), k2.bit_length()) - 1, -1, -1):
            R = self._dbl(R)
            b1, b2 = (k1 >> i) & 1, (k2 >> i) & 1
            if b1 or b2:
                R = self._add(R, J12 if b1 and b2 else (J1 if b1 else J2))
        if R is None or R[2] % self.p == 0:
            return None
        zi = pow(R[2], self.p - 2, self.p)
        return R[0] * zi * zi % self.p, R[1] * zi * zi * zi % self.p

    def verify(self, Q, digest, r, s):
        n = self.n
        if not (0 < r < n and 0 < s < n) or not self.on_curve(Q):
            return False
        e = int.from_bytes(digest, "big")
        excess = len(digest) * 8 - n.bit_length()
        if excess > 0:
            e >>= excess
        w = pow(s, n - 2, n)
        X = self.mul_add(e * w % n, self.g, r * w % n, Q)
        return X is not None and X[0] % n == r

    def decode_point(self, b):
        if len(b) != 1 + 2 * self.size or b[0] != 4:
            return None
        return int.from_bytes(b[1:1 + self.size], "big"), int.from_bytes(b[1 + self.size:], "big")


CURVES = {
    "nistp256": Curve(
        "nistp256", 2 ** 256 - 2 ** 224 + 2 ** 192 + 2 ** 96 - 1,
        0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551,
        0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b,
        0x6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296,
        0x4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5, hashlib.sha256),
    "nistp384": Curve(
        "nistp384", 2 ** 384 - 2 ** 128 - 2 ** 96 + 2 ** 32 - 1,
        0xffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973,
        0xb3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef,
        0xaa87ca22be8b05378eb1c71ef320ad746e1d3b628ba79b9859f741e082542a385502f25dbf55296c3a545e3872760ab7,
        0x3617de4a96262c6f5d9e98bf9292dc29f8f41dbd289a147ce9da3113b5f0b8c00a60b1ce1d7e819d7a431d7c90ea0e5f,
        hashlib.sha384),
    "nistp521": Curve(
        "nistp521", 2 ** 521 - 1,
        0x01fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffa51868783bf2f966b7fcc0148f709a5d03bb5c9b8899c47aebb6fb71e91386409,
        0x0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1bf073573df883d2c34f1ef451fd46b503f00,
        0x00c6858e06b70404e9cd9e3ecb662395b4429c648139053fb521f828af606b4d3dbaa14b5e77efe75928fe1dc127a2ffa8de3348b3c1856a429bf97e7e31c2e5bd66,
        0x011839296a789a3bc0045c8a5fb42c7d1bd998f54449579b446817afbd17273e662c97ee72995ef42640c550b9013fad0761353c7086a272c24088be94769fd16650,
        hashlib.sha512),
}


# ---------------------------------------------------------------------------
# host-key signatures (RFC 4253 §6.6, RFC 8332, RFC 5656, RFC 8709)
# ---------------------------------------------------------------------------

_DIGEST_INFO = {  # DER DigestInfo prefixes (RFC 8017 §9.2 note 1)
    "sha1": bytes.fromhex("3021300906052b0e03021a05000414"),
    "sha256": bytes.fromhex("3031300d060960864801650304020105000420"),
    "sha512": bytes.fromhex("3051300d060960864801650304020305000440"),
}
_RSA_HASH = {"ssh-rsa": "sha1", "rsa-sha2-256": "sha256", "rsa-sha2-512": "sha512"}


def key_type(key_blob):
    return Reader(key_blob).string().decode("ascii", "replace")


def verify_signature(key_blob, sig_blob, data, sig_algo_expected):
    """True when ``sig_blob`` is a valid signature of ``data`` by ``key_blob``."""
    try:
        kr, sr = Reader(key_blob), Reader(sig_blob)
        ktype = kr.string().decode("ascii", "replace")
        salgo = sr.string().decode("ascii", "replace")
        sig = sr.string()
        if salgo != sig_algo_expected:
            return False
        if ktype == "ssh-rsa" and salgo in _RSA_HASH:
            e, n = kr.mpint(), kr.mpint()
            if n <= 0 or e <= 0:
                return False
            k = (n.bit_length() + 7) // 8
            if len(sig) > k:
                return False
            h = _RSA_HASH[salgo]
            t = _DIGEST_INFO[h] + hashlib.new(h, data).digest()
            if k < len(t) + 11:
                return False
            em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
            return pow(int.from_bytes(sig, "big"), e, n) == int.from_bytes(em, "big")
        if ktype == "ssh-dss" and salgo == "ssh-dss":
            p, q, g, y = kr.mpint(), kr.mpint(), kr.mpint(), kr.mpint()
            if len(sig) != 40:
                return False
            r, s = int.from_bytes(sig[:20], "big"), int.from_bytes(sig[20:], "big")
            if not (0 < r < q and 0 < s < q):
                return False
            w = pow(s, q - 2, q)
            z = int.from_bytes(hashlib.sha1(data).digest(), "big")
            v = pow(g, z * w % q, p) * pow(y, r * w % q, p) % p % q
            return v == r
        if ktype.startswith("ecdsa-sha2-") and salgo == ktype:
            curve = CURVES.get(kr.string().decode("ascii", "replace"))
            if curve is None or "ecdsa-sha2-" + curve.name != ktype:
                return False
            Q = curve.decode_point(kr.string())
            if Q is None:
                return False
            rs = Reader(sig)
            r, s = rs.mpint(), rs.mpint()
            return curve.verify(Q, curve.hash(data).digest(), r, s)
        if ktype == "ssh-ed25519" and salgo == "ssh-ed25519":
            return ed25519_verify(kr.string(), data, sig)
    except SSHError:
        return False
    return False


# ---------------------------------------------------------------------------
# the transport, client side, up to the key-exchange reply
# ---------------------------------------------------------------------------

class _Conn:
    """Reads bounded by one deadline for the whole exchange, so a server that
    drips bytes or chatters (banner lines, IGNORE packets) cannot hold the
    caller longer than its timeout."""

    def __init__(self, sock, deadline=None):
        self.sock = sock
        self.buf = b""
        self.deadline = deadline  # None: only the socket's own timeout

    def _recv(self, n):
        if self.deadline is not None:
            left = self.deadline - time.monotonic()
            if left <= 0:
                raise socket.timeout("timed out")
            self.sock.settimeout(left)
        chunk = self.sock.recv(n)
        if not chunk:
            raise SSHError("connection closed by the server")
        return chunk

    def _fill(self, n):
        while len(self.buf) < n:
            self.buf += self._recv(65536)

    def read_line(self):
        while b"\n" not in self.buf:
            if len(self.buf) > 8192:
                raise SSHError("no SSH version line")
            self.buf += self._recv(4096)
        line, self.buf = self.buf.split(b"\n", 1)
        return line.rstrip(b"\r")

    def read_message(self):
        """The next packet that is not IGNORE or DEBUG."""
        for _ in range(MAX_SKIPPED):
            payload = self.read_packet()
            if not payload or payload[0] not in (MSG_IGNORE, MSG_DEBUG):
                return payload
        raise SSHError("too many IGNORE/DEBUG messages")

    def read_packet(self):
        self._fill(5)
        length, pad = struct.unpack(">IB", self.buf[:5])
        if length > MAX_PACKET or length < pad + 1:
            raise SSHError("bad packet length %d" % length)
        self._fill(4 + length)
        payload = self.buf[5:4 + length - pad]
        self.buf = self.buf[4 + length:]
        return payload

    def send_packet(self, payload):
        pad = 8 - (5 + len(payload)) % 8
        if pad < 4:
            pad += 8
        self.sock.sendall(struct.pack(">IB", 1 + len(payload) + pad, pad) + payload + os.urandom(pad))


def _kexinit(kex, hostkeys):
    return (bytes([MSG_KEXINIT]) + os.urandom(16) + name_list(kex) + name_list(hostkeys)
            + name_list(CIPHERS) * 2 + name_list(MACS) * 2 + name_list(("none",)) * 2
            + name_list(()) * 2 + b"\x00" + struct.pack(">I", 0))


def _negotiate(ours, theirs, what):
    for a in ours:
        if a in theirs:
            return a
    raise SSHError("no common algorithm for %s; we offered: %s; peer offered: %s" % (what, list(ours), theirs))


def fetch_host_key(host, port=22, timeout=5.0, kex_algos=KEX_ALGOS, host_key_algos=HOST_KEY_ALGOS):
    """(key type, key blob) of the host key that ``host`` proves it holds in a
    key exchange, negotiated from ``host_key_algos`` in order.  Raises
    :class:`SSHError` or ``OSError``."""
    deadline = time.monotonic() + timeout
    sock = socket.create_connection((host, port), timeout=timeout)
    try:
        sock.settimeout(timeout)
        conn = _Conn(sock, deadline)
        sock.sendall(CLIENT_VERSION + b"\r\n")
        for _ in range(MAX_BANNER_LINES):  # RFC 4253 §4.2: the server may send other lines first
            v_s = conn.read_line()
            if v_s.startswith(b"SSH-"):
                break
        else:
            raise SSHError("no SSH version line in the first %d lines" % MAX_BANNER_LINES)
        if not (v_s.startswith(b"SSH-2.0-") or v_s.startswith(b"SSH-1.99-")):
            raise SSHError("unsupported server version %r" % v_s)
        i_c = _kexinit(kex_algos, host_key_algos)
        conn.send_packet(i_c)
        i_s = conn.read_message()
        if not i_s or i_s[0] != MSG_KEXINIT:
            raise SSHError("expected KEXINIT, got message %d" % (i_s[0] if i_s else -1))
        r = Reader(i_s)
        r.raw(17)
        kex = _negotiate(kex_algos, r.names(), "key exchange")
        hk = _negotiate(host_key_algos, r.names(), "host key")
        if kex.startswith("curve25519"):
            priv = os.urandom(32)
            q_c = x25519(priv, X25519_BASE)
            conn.send_packet(bytes([MSG_KEXDH_INIT]) + ssh_string(q_c))
        else:
            x = int.from_bytes(os.urandom(32), "big") | (1 << 255)
            e = pow(2, x, GROUP14_P)
            conn.send_packet(bytes([MSG_KEXDH_INIT]) + ssh_mpint(e))
        reply = conn.read_message()
        if not reply or reply[0] != MSG_KEXDH_REPLY:
            if reply and reply[0] == MSG_DISCONNECT:
                rr = Reader(reply[1:])
                rr.uint32()
                raise SSHError("disconnected by the server: %s" % rr.string().decode("utf-8", "replace"))
            raise SSHError("expected KEXDH_REPLY, got message %d" % (reply[0] if reply else -1))
        rr = Reader(reply[1:])
        k_s = rr.string()
        if kex.startswith("curve25519"):
            q_s = rr.string()
            if len(q_s) != 32:
                raise SSHError("bad curve25519 public key")
            shared = x25519(priv, q_s)
            if shared == bytes(32):
                raise SSHError("degenerate curve25519 shared secret")
            k = int.from_bytes(shared, "big")
            kex_part = ssh_string(q_c) + ssh_string(q_s)
            hash_fn = hashlib.sha256
        else:
            f = rr.mpint()
            if not 1 < f < GROUP14_P - 1:
                raise SSHError("bad diffie-hellman reply")
            k = pow(f, x, GROUP14_P)
            kex_part = ssh_mpint(e) + ssh_mpint(f)
            hash_fn = hashlib.sha256 if kex.endswith("sha256") else hashlib.sha1
        sig = rr.string()
        h = hash_fn(ssh_string(CLIENT_VERSION) + ssh_string(v_s) + ssh_string(i_c) + ssh_string(i_s)
                    + ssh_string(k_s) + kex_part + ssh_mpint(k)).digest()
        ktype = key_type(k_s)
        expect_type = "ssh-rsa" if hk.startswith("rsa-sha2-") else hk
        if ktype != expect_type:
            raise SSHError("host key type %s does not match the negotiated %s" % (ktype, hk))
        if not verify_signature(k_s, sig, h, hk):
            raise SSHError("host key signature does not verify")
        try:  # SSH_DISCONNECT_BY_APPLICATION
            conn.send_packet(bytes([MSG_DISCONNECT]) + struct.pack(">I", 11) + ssh_string(b"") + ssh_string(b""))
        except OSError:
            pass
        return ktype, k_s
    finally:
        sock.close()
