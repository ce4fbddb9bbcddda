"""In-process SSH host-key fetch (utils/sshwire.py; reference
internal/common/knownhosts/knownhosts.go:137-155) against a local fake SSH
server that signs the exchange hash with keys made by ``ssh-keygen``.  The
fake server is itself checked with OpenSSH's ``ssh-keyscan``, so both ends
are held to a real implementation of the protocol."""

import base64
import hashlib
import os
import shutil
import socket
import struct
import subprocess
import threading
import time

import pytest

from move2kube_amd.utils import knownhosts, sshwire
from move2kube_amd.utils.sshwire import Reader, ssh_mpint, ssh_string

pytestmark = pytest.mark.skipif(shutil.which("ssh-keygen") is None, reason="ssh-keygen not installed")


# -- keys ---------------------------------------------------------------------

def _load_openssh_private(path):
    lines = open(path).read().strip().splitlines()
    raw = base64.b64decode("".join(lines[1:-1]))
    assert raw.startswith(b"openssh-key-v1\x00")
    r = Reader(raw[len(b"openssh-key-v1\x00"):])
    assert r.string() == b"none" and r.string() == b"none"
    r.string()
    assert r.uint32() == 1
    pub = r.string()
    pr = Reader(r.string())
    pr.uint32(), pr.uint32()
    ktype = pr.string().decode()
    if ktype == "ssh-ed25519":
        pr.string()
        priv = {"seed": pr.string()[:32]}
    elif ktype.startswith("ecdsa-sha2-"):
        curve = pr.string().decode()
        pr.string()
        priv = {"curve": curve, "d": pr.mpint()}
    elif ktype == "ssh-rsa":
        n, e, d = pr.mpint(), pr.mpint(), pr.mpint()
        priv = {"n": n, "d": d}
    elif ktype == "ssh-dss":
        p, q, g, y, x = pr.mpint(), pr.mpint(), pr.mpint(), pr.mpint(), pr.mpint()
        priv = {"p": p, "q": q, "g": g, "x": x}
    else:
        raise AssertionError(ktype)
    return ktype, pub, priv


_L = 2 ** 252 + 27742317777372353535851937790883648493


def _sign(ktype, priv, algo, data):
    if ktype == "ssh-ed25519":
        h = hashlib.sha512(priv["seed"]).digest()
        a = int.from_bytes(h[:32], "little")
        a &= (1 << 254) - 8
        a |= 1 << 254
        A = sshwire.ed_compress(sshwire.ed_mul(a, sshwire.ED_B))
        r = int.from_bytes(hashlib.sha512(h[32:] + data).digest(), "little") % _L
        R = sshwire.ed_compress(sshwire.ed_mul(r, sshwire.ED_B))
        k = int.from_bytes(hashlib.sha512(R + A + data).digest(), "little") % _L
        sig = R + ((r + k * a) % _L).to_bytes(32, "little")
    elif ktype.startswith("ecdsa-sha2-"):
        c = sshwire.CURVES[priv["curve"]]
        e = int.from_bytes(c.hash(data).digest(), "big")
        while True:
            k = int.from_bytes(os.urandom(c.size + 8), "big") % c.n
            if k == 0:
                continue
            x = c.mul_add(k, c.g, 0, c.g)[0] % c.n
            s = pow(k, c.n - 2, c.n) * (e + x * priv["d"]) % c.n
            if x and s:
                break
        sig = ssh_mpint(x) + ssh_mpint(s)
    elif ktype == "ssh-rsa":
        hname = {"ssh-rsa": "sha1", "rsa-sha2-256": "sha256", "rsa-sha2-512": "sha512"}[algo]
        t = sshwire._DIGEST_INFO[hname] + hashlib.new(hname, data).digest()
        n = priv["n"]
        k = (n.bit_length() + 7) // 8
        em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
        sig = pow(int.from_bytes(em, "big"), priv["d"], n).to_bytes(k, "big")
    elif ktype == "ssh-dss":
        p, q, g, x = priv["p"], priv["q"], priv["g"], priv["x"]
        z = int.from_bytes(hashlib.sha1(data).digest(), "big")
        while True:
            k = int.from_bytes(os.urandom(28), "big") % q
            if not k:
                continue
            r = pow(g, k, p) % q
            s = pow(k, q - 2, q) * (z + x * r) % q
            if r and s:
                break
        sig = r.to_bytes(20, "big") + s.to_bytes(20, "big")
    return ssh_string(algo.encode()) + ssh_string(sig)


@pytest.fixture(scope="module")
def keys(tmp_path_factory):
    d = tmp_path_factory.mktemp("hostkeys")
    out = {}
    for name, args in (("ed25519", ["-t", "ed25519"]), ("ecdsa256", ["-t", "ecdsa", "-b", "256"]),
                       ("ecdsa384", ["-t", "ecdsa", "-b", "384"]), ("ecdsa521", ["-t", "ecdsa", "-b", "521"]),
                       ("rsa", ["-t", "rsa", "-b", "2048"]), ("dsa", ["-t", "dsa"])):
        path = str(d / name)
        p = subprocess.run(["ssh-keygen", "-q", "-N", "", "-C", "", "-f", path] + args, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT)
        if p.returncode != 0:
            continue  # (a build of OpenSSH without DSA)
        ktype, pub, priv = _load_openssh_private(path)
        assert open(path + ".pub").read().split()[1] == base64.b64encode(pub).decode()
        out[name] = (ktype, pub, priv)
    return out


# -- the fake server ----------------------------------------------------------

class FakeServer:
    """Speaks the server side of RFC 4253 up to KEXDH_REPLY for every
    connection: ``hostkeys`` maps a host-key algorithm name to a loaded key."""

    def __init__(self, hostkeys, kex=("curve25519-sha256", "diffie-hellman-group14-sha256"), corrupt=False,
                 banner_lines=()):
        self.hostkeys, self.kex, self.corrupt, self.banner_lines = hostkeys, kex, corrupt, banner_lines
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(8)
        self.port = self.sock.getsockname()[1]
        self.seen = []  # (kex, host key algo) per handshake
        self.t = threading.Thread(target=self._serve, daemon=True)
        self.t.start()

    def close(self):
        self.sock.close()

    def _serve(self):
        while True:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._handle, args=(c,), daemon=True).start()

    def _handle(self, c):
        c.settimeout(10)
        try:
            conn = sshwire._Conn(c)
            v_s = b"SSH-2.0-FakeServer_1.0"
            c.sendall(b"".join(b + b"\r\n" for b in self.banner_lines) + v_s + b"\r\n")
            v_c = conn.read_line()
            i_s = sshwire._kexinit(self.kex, tuple(self.hostkeys))
            conn.send_packet(i_s)
            i_c = conn.read_packet()
            r = Reader(i_c)
            r.raw(17)
            kex = sshwire._negotiate(r.names(), self.kex, "kex")
            algo = sshwire._negotiate(r.names(), tuple(self.hostkeys), "host key")
            ktype, k_s, priv = self.hostkeys[algo]
            init = Reader(conn.read_packet())
            assert init.byte() == sshwire.MSG_KEXDH_INIT
            if kex.startswith("curve25519"):
                q_c = init.string()
                b = os.urandom(32)
                q_s = sshwire.x25519(b, sshwire.X25519_BASE)
                k = int.from_bytes(sshwire.x25519(b, q_c), "big")
                part, reply_mid, hf = ssh_string(q_c) + ssh_string(q_s), ssh_string(q_s), hashlib.sha256
            else:
                e = init.mpint()
                y = int.from_bytes(os.urandom(32), "big")
                f = pow(2, y, sshwire.GROUP14_P)
                k = pow(e, y, sshwire.GROUP14_P)
                part, reply_mid = ssh_mpint(e) + ssh_mpint(f), ssh_mpint(f)
                hf = hashlib.sha256 if kex.endswith("sha256") else hashlib.sha1
            h = hf(ssh_string(v_c) + ssh_string(v_s) + ssh_string(i_c) + ssh_string(i_s) + ssh_string(k_s)
                   + part + ssh_mpint(k)).digest()
            sig = _sign(ktype, priv, algo, h + (b"x" if self.corrupt else b""))
            self.seen.append((kex, algo))
            conn.send_packet(bytes([sshwire.MSG_IGNORE]) + ssh_string(b"padding"))
            conn.send_packet(bytes([sshwire.MSG_KEXDH_REPLY]) + ssh_string(k_s) + reply_mid + ssh_string(sig))
            while c.recv(4096):
                pass
        except (OSError, sshwire.SSHError, AssertionError):
            pass
        finally:
            c.close()


@pytest.fixture
def server(keys):
    made = []

    def make(names, **kw):
        hostkeys = {}
        for algo, key in names:
            if key not in keys:
                pytest.skip("%s keys not available" % key)
            hostkeys[algo] = keys[key]
        s = FakeServer(hostkeys, **kw)
        made.append(s)
        return s
    yield make
    for s in made:
        s.close()


CASES = [("ssh-ed25519", "ed25519"), ("ecdsa-sha2-nistp256", "ecdsa256"), ("ecdsa-sha2-nistp384", "ecdsa384"),
         ("ecdsa-sha2-nistp521", "ecdsa521"), ("ssh-rsa", "rsa"), ("rsa-sha2-512", "rsa"), ("rsa-sha2-256", "rsa"),
         ("ssh-dss", "dsa")]


@pytest.mark.parametrize("algo,key", CASES)
@pytest.mark.parametrize("kex", ["curve25519-sha256", "curve25519-sha256@libssh.org",
                                 "diffie-hellman-group14-sha256", "diffie-hellman-group14-sha1"])
def test_fetch_host_key_every_algorithm(server, keys, algo, key, kex):
    s = server([(algo, key)], kex=(kex,))
    ktype, blob = sshwire.fetch_host_key("127.0.0.1", port=s.port, timeout=10)
    assert (ktype, blob) == (keys[key][0], keys[key][1])
    assert s.seen == [(kex, algo)]


@pytest.mark.parametrize("algo,key", [c for c in CASES if c[0] in ("ssh-ed25519", "ecdsa-sha2-nistp256",
                                                                   "ecdsa-sha2-nistp521", "rsa-sha2-512")])
def test_fake_server_is_accepted_by_openssh(server, keys, algo, key):
    """OpenSSH's ssh-keyscan completes the key exchange with the fake server
    (it checks the signature) and reports the same key."""
    if shutil.which("ssh-keyscan") is None:
        pytest.skip("ssh-keyscan not installed")
    s = server([(algo, key)])
    kt = {"ssh-ed25519": "ed25519", "ecdsa-sha2-nistp256": "ecdsa", "ecdsa-sha2-nistp521": "ecdsa",
          "rsa-sha2-512": "rsa"}[algo]
    p = subprocess.run(["ssh-keyscan", "-T", "10", "-p", str(s.port), "-t", kt, "127.0.0.1"],
                       stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=30)
    lines = [ln.split() for ln in p.stdout.decode().splitlines() if ln and not ln.startswith("#")]
    assert lines == [["[127.0.0.1]:%d" % s.port, keys[key][0], base64.b64encode(keys[key][1]).decode()]]


def test_negotiates_the_key_a_go_client_would(server, keys):
    s = server([("ssh-ed25519", "ed25519"), ("ssh-rsa", "rsa"), ("ecdsa-sha2-nistp384", "ecdsa384"),
                ("ecdsa-sha2-nistp256", "ecdsa256")], banner_lines=(b"welcome", b"to the fake"))
    line = knownhosts.fetch_line_in_process("127.0.0.1", port=s.port, timeout=10)
    assert line == "127.0.0.1 ecdsa-sha2-nistp256 " + base64.b64encode(keys["ecdsa256"][1]).decode()
    s2 = server([("ssh-ed25519", "ed25519"), ("rsa-sha2-256", "rsa")])
    assert knownhosts.fetch_line_in_process("127.0.0.1", port=s2.port, timeout=10).split()[1] == "ssh-rsa"


def test_bad_signature_gives_no_key(server):
    s = server([("ssh-ed25519", "ed25519")], corrupt=True)
    with pytest.raises(sshwire.SSHError, match="does not verify"):
        sshwire.fetch_host_key("127.0.0.1", port=s.port, timeout=10)
    assert knownhosts.fetch_line_in_process("127.0.0.1", port=s.port, timeout=10) == ""


def test_no_common_algorithm_and_closed_port(server):
    s = server([("ssh-ed25519", "ed25519")], kex=("sntrup761x25519-sha512@openssh.com",))
    with pytest.raises(sshwire.SSHError, match="key exchange"):
        sshwire.fetch_host_key("127.0.0.1", port=s.port, timeout=10)
    probe = socket.socket()
    probe.bind(("127.0.0.1", 0))
    port = probe.getsockname()[1]
    probe.close()
    assert knownhosts.fetch_line_in_process("127.0.0.1", port=port, timeout=2) == ""


def test_not_an_ssh_server():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)

    def serve():
        c, _ = srv.accept()
        c.sendall(b"HTTP/1.1 400 Bad Request\r\n\r\n")
        c.close()
    t = threading.Thread(target=serve, daemon=True)
    t.start()
    try:
        # (a reset when the peer closes before reading our version line is an OSError)
        with pytest.raises((sshwire.SSHError, OSError)):
            sshwire.fetch_host_key("127.0.0.1", port=srv.getsockname()[1], timeout=5)
    finally:
        srv.close()


def test_primitives_match_published_vectors():
    # RFC 7748 §5.2 and RFC 8032 §7.1 test 1
    assert sshwire.x25519(
        bytes.fromhex("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4"),
        bytes.fromhex("e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c")).hex() == \
        "c3da55379de9c6908e94ea4df28d084f32eccf03491c71f754b4075577a28552"
    pub = bytes.fromhex("d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a")
    sig = bytes.fromhex("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b4"
                        "6bd25bf5f0595bbe24655141438e7a100b")
    assert sshwire.ed25519_verify(pub, b"", sig) and not sshwire.ed25519_verify(pub, b"\x00", sig)
    for c in sshwire.CURVES.values():  # generator on the curve, of order n
        assert c.on_curve(c.g) and c.mul_add(c.n, c.g, 0, c.g) is None
    assert ssh_mpint(0) == b"\x00\x00\x00\x00" and ssh_mpint(0x80) == b"\x00\x00\x00\x02\x00\x80"
    assert struct.unpack(">I", ssh_mpint(0x7f)[:4])[0] == 1


def _serve_bytes(chunks):
    """A one-shot server that sends ``chunks`` (after reading the client's
    version line) and closes."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)

    def serve():
        try:
            c, _ = srv.accept()
        except OSError:
            return
        try:
            c.settimeout(5)
            c.recv(256)
            for ch in chunks:
                c.sendall(ch)
        except OSError:
            pass
        finally:
            c.close()
    threading.Thread(target=serve, daemon=True).start()
    return srv


def _pkt(payload, pad=4):
    return struct.pack(">IB", 1 + len(payload) + pad, pad) + payload + b"\x00" * pad


@pytest.mark.parametrize("chunks", [
    [b"SSH-2.0-x\r\n", struct.pack(">IB", 1 << 30, 4)],                      # absurd packet length
    [b"SSH-2.0-x\r\n", struct.pack(">IB", 3, 10)],                           # padding longer than the packet
    [b"SSH-2.0-x\r\n", _pkt(b"\x14" + b"\x00" * 16)],                        # KEXINIT cut short
    [b"SSH-2.0-x\r\n", _pkt(bytes([20]) + bytes(16) + ssh_string(b"\xff\xfe") * 10 + b"\x00" + bytes(4))],
    [b"SSH-1.5-old\r\n"],                                                    # SSH 1 only
    [b"SSH-2.0-x\r\n", _pkt(sshwire._kexinit(("curve25519-sha256",), ("ssh-ed25519",))),
     _pkt(bytes([31]) + ssh_string(b"\x00\x00\x00\x0bssh-ed25519" + ssh_string(b"k" * 32)) + ssh_string(b"short"))],
    [b"SSH-2.0-x\r\n", _pkt(sshwire._kexinit(("curve25519-sha256",), ("ssh-ed25519",))),
     _pkt(bytes([1]) + struct.pack(">I", 2) + ssh_string(b"go away") + ssh_string(b""))],
    [b"x" * 9000],                                                           # no version line at all
])
def test_hostile_servers_fail_cleanly(chunks):
    srv = _serve_bytes(chunks)
    try:
        with pytest.raises((sshwire.SSHError, OSError)):
            sshwire.fetch_host_key("127.0.0.1", port=srv.getsockname()[1], timeout=5)
    finally:
        srv.close()


def test_chatty_servers_are_cut_off():
    # banner lines and IGNORE packets are allowed, but not without end
    srv = _serve_bytes([b"hello\r\n" * (sshwire.MAX_BANNER_LINES + 5)])
    try:
        with pytest.raises(sshwire.SSHError, match="version line"):
            sshwire.fetch_host_key("127.0.0.1", port=srv.getsockname()[1], timeout=5)
    finally:
        srv.close()
    ignore = _pkt(bytes([sshwire.MSG_IGNORE]) + ssh_string(b""))
    srv = _serve_bytes([b"SSH-2.0-x\r\n", ignore * (sshwire.MAX_SKIPPED + 5)])
    try:
        with pytest.raises(sshwire.SSHError, match="IGNORE"):
            sshwire.fetch_host_key("127.0.0.1", port=srv.getsockname()[1], timeout=5)
    finally:
        srv.close()


def test_dripping_server_is_bounded_by_the_timeout():
    # one byte every 0.2 s never trips a per-recv timeout of 1 s; the deadline
    # for the whole exchange does
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    stop = threading.Event()

    def serve():
        try:
            c, _ = srv.accept()
        except OSError:
            return
        try:
            while not stop.is_set():
                c.sendall(b"x")
                stop.wait(0.2)
        except OSError:
            pass
        finally:
            c.close()
    threading.Thread(target=serve, daemon=True).start()
    t0 = time.monotonic()
    try:
        with pytest.raises((sshwire.SSHError, OSError)):
            sshwire.fetch_host_key("127.0.0.1", port=srv.getsockname()[1], timeout=1.0)
        assert time.monotonic() - t0 < 3
    finally:
        stop.set()
        srv.close()
