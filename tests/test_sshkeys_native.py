"""Private SSH keys parsed, decrypted and re-encoded in process
(``ops/csrc/sshkey.cpp`` through ``utils/sshkeys.py``), as the reference's
``loadSSHKey`` does with x/crypto/ssh and crypto/x509
(``internal/common/sshkeys/sshkeys.go:170-232``).

The fixtures under ``tests/fixtures/sshkeys`` were generated once with this
container's OpenSSH 8.9 / OpenSSL 3.0 (``make_fixtures.sh``); each
``*.expected.pem`` is what ``ssh-keygen -p -m PEM -N ''`` wrote for its key,
so the in-process output is checked byte for byte against the ssh-keygen path
-- with ssh-keygen removed from PATH.
"""

import glob
import os
import shutil
import stat

import pytest

from move2kube_amd import qaengine
from move2kube_amd.qaengine.engine import Engine
from move2kube_amd.utils import sshkeys

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "fixtures", "sshkeys")
PASS = "m2k-pass"

native = pytest.importorskip("move2kube_amd.ops._m2k_sshkey")

CONVERTIBLE = sorted(os.path.basename(p)[:-len(".expected.pem")] for p in glob.glob(os.path.join(FIX, "*.expected.pem")))
ENCRYPTED = {"rsa_openssh_ctr", "rsa_openssh_cbc", "ec521_openssh_ctr", "rsa_pkcs1_aes128", "rsa_pkcs1_aes256",
             "rsa_pkcs1_des3", "ec384_sec1_aes128", "ec256_sec1_aes192"}


def _read(name):
    with open(os.path.join(FIX, name), "rb") as f:
        return f.read()


def test_fixture_set_covers_the_formats():
    assert len(CONVERTIBLE) == 15
    assert ENCRYPTED < set(CONVERTIBLE)


@pytest.mark.parametrize("name", CONVERTIBLE)
def test_native_pem_equals_ssh_keygen_output(name):
    data = _read(name + ".key")
    status, text = native.private_key_pem(data, None)
    if name in ENCRYPTED:
        # detected by parsing (an OpenSSH key carries no "ENCRYPTED" marker)
        assert (status, text) == (1, "ssh: this private key is passphrase protected")
        status, text = native.private_key_pem(data, PASS.encode())
    assert status == 0, text
    assert text == _read(name + ".expected.pem").decode()


@pytest.mark.parametrize("name,go_type", [("ed25519_openssh", "*ed25519.PrivateKey"),
                                          ("ed25519_pkcs8", "ed25519.PrivateKey"),
                                          ("dsa_pem", "*dsa.PrivateKey")])
def test_other_key_types_are_reported_with_their_go_type(name, go_type):
    assert native.private_key_pem(_read(name + ".key"), None) == (3, go_type)


@pytest.mark.parametrize("name,passphrase,err", [
    ("rsa_openssh_ctr", b"wrong", "x509: decryption password incorrect"),        # check-int mismatch
    ("rsa_pkcs1_des3", b"wrong", "x509: decryption password incorrect"),         # RFC 1423 padding
    ("rsa_openssh", b"m2k-pass", "ssh: key is not password protected"),
    ("rsa_pkcs1", b"m2k-pass", "ssh: not an encrypted key"),
    ("rsa_openssh_ctr", b"", "bcrypt_pbkdf: empty password"),
    ("dsa_openssh", None, "ssh: unhandled key type"),                             # x/crypto: no ssh-dss
])
def test_errors_are_go_texts(name, passphrase, err):
    status, text = native.private_key_pem(_read(name + ".key"), passphrase)
    assert (status, text) == (2, err)


@pytest.mark.parametrize("data,err", [
    (b"", "ssh: no key found"),
    (b"-----BEGIN FOO KEY-----\nAAAA\n-----END FOO KEY-----\n", 'ssh: unsupported key type "FOO KEY"'),
    (b"-----BEGIN RSA PRIVATE KEY-----\nMAA=\n-----END RSA PRIVATE KEY-----\n", None),
    (b"-----BEGIN OPENSSH PRIVATE KEY-----\nAAAA\n-----END OPENSSH PRIVATE KEY-----\n",
     "ssh: invalid openssh private key format"),
])
def test_malformed_input(data, err):
    status, text = native.private_key_pem(data, None)
    assert status == 2
    if err is not None:
        assert text == err


def test_pem_decode_follows_encoding_pem():
    # leading text, headers, CRLF lines, a malformed first block skipped
    data = (b"junk\r\n-----BEGIN X-----\r\nbroken\n-----BEGIN K-----\r\nProc-Type: 4,ENCRYPTED\r\n"
            b"DEK-Info: AES-128-CBC,00\r\n\r\naGVs\r\nbG8=\r\n-----END K-----  \r\ntrailer")
    assert native.pem_decode(data) == ("K", [("Proc-Type", "4,ENCRYPTED"), ("DEK-Info", "AES-128-CBC,00")], b"hello")
    assert native.pem_decode(b"no pem here") is None


def test_bcrypt_pbkdf_parameter_errors():
    with pytest.raises(ValueError, match="number of rounds is too small"):
        native.bcrypt_pbkdf(b"p", b"s", 0, 48)
    with pytest.raises(ValueError, match="bad salt length"):
        native.bcrypt_pbkdf(b"p", b"", 1, 48)
    k1 = native.bcrypt_pbkdf(b"password", b"salt", 4, 48)
    assert len(k1) == 48 and k1 == native.bcrypt_pbkdf(b"password", b"salt", 4, 48)
    assert k1 != native.bcrypt_pbkdf(b"password", b"salt", 5, 48)
    assert native.bcrypt_pbkdf(b"password", b"salt", 4, 64)[:1] == k1[:1]   # blocks interleave


# -- through sshkeys.get_ssh_key, without ssh-keygen ----------------------------

class _Answers(Engine):
    def __init__(self, answers):
        self.answers = answers
        self.asked = []

    def fetch_answer(self, prob):
        self.asked.append((prob.type, prob.desc))
        for prefix, ans in self.answers.items():
            if prob.desc.startswith(prefix):
                prob.set_answer(ans)
                return prob
        prob.set_answer(prob.default)
        return prob


@pytest.fixture
def home_without_keygen(tmp_path, monkeypatch):
    home = tmp_path / "home"
    (home / ".ssh").mkdir(parents=True)
    monkeypatch.setenv("HOME", str(home))
    empty = tmp_path / "bin"
    empty.mkdir()
    monkeypatch.setenv("PATH", str(empty))
    assert shutil.which("ssh-keygen") is None
    sshkeys.reset()
    qaengine.reset()
    yield home
    qaengine.reset()
    sshkeys.reset()


def _install(home, name, as_name="id_key"):
    dst = home / ".ssh" / as_name
    shutil.copyfile(os.path.join(FIX, name + ".key"), str(dst))
    dst.chmod(stat.S_IRUSR | stat.S_IWUSR)


@pytest.mark.parametrize("name", ["rsa_openssh_ctr", "ec256_sec1_aes192", "rsa_pkcs8"])
def test_get_ssh_key_without_ssh_keygen(home_without_keygen, name):
    _install(home_without_keygen, name)
    eng = _Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["id_key"],
                    "Select the key": ["id_key"], "Enter the password": [PASS]})
    qaengine.add_engine(eng)
    key, ok = sshkeys.get_ssh_key("git.corp.example")
    assert ok and key == _read(name + ".expected.pem").decode()
    asked_password = ("Password", 'Enter the password to decrypt the private key "id_key" : ') in eng.asked
    assert asked_password == (name in ENCRYPTED)


def test_a_key_mentioning_encrypted_is_not_taken_for_an_encrypted_one(home_without_keygen):
    # the old substring test asked for a password here; parsing does not
    data = _read("rsa_pkcs1.key").decode()
    (home_without_keygen / ".ssh" / "id_key").write_text("ENCRYPTED? no.\n" + data)
    eng = _Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["id_key"],
                    "Select the key": ["id_key"]})
    qaengine.add_engine(eng)
    key, ok = sshkeys.get_ssh_key("git.corp.example")
    assert ok and key == _read("rsa_pkcs1.expected.pem").decode()
    assert all(t != "Password" for t, _ in eng.asked)


def test_wrong_password_and_ed25519_keep_the_placeholder(home_without_keygen, capsys):
    _install(home_without_keygen, "rsa_openssh_ctr", "enc")
    _install(home_without_keygen, "ed25519_openssh", "ed")
    qaengine.add_engine(_Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["enc", "ed"],
                                  "Select the key to use to for the git domain a": ["enc"],
                                  "Select the key to use to for the git domain b": ["ed"],
                                  "Enter the password": ["nope"]}))
    assert sshkeys.get_ssh_key("a.example") == ("", False)
    assert sshkeys.get_ssh_key("b.example") == ("", False)
    err = capsys.readouterr().err
    assert "x509: decryption password incorrect" in err
    assert "Unknown key type [*ed25519.PrivateKey]" in err


def _rearmour(name, mutate):
    """An OpenSSH key file with its binary body changed by ``mutate``."""
    import base64
    lines = _read(name + ".key").decode().strip().splitlines()
    body = bytearray(base64.b64decode("".join(lines[1:-1])))
    mutate(body)
    t = base64.b64encode(bytes(body)).decode()
    return ("\n".join([lines[0]] + [t[i:i + 70] for i in range(0, len(t), 70)] + [lines[-1]]) + "\n").encode()


def _kdf_rounds_offset(body):
    """Offset of the bcrypt rounds field: magic, cipher, kdf, then kdfoptions
    (string salt, uint32 rounds)."""
    import struct
    off = len(b"openssh-key-v1\0")
    for _ in range(2):                       # ciphername, kdfname
        off += 4 + struct.unpack(">I", bytes(body[off:off + 4]))[0]
    off += 4                                 # kdfoptions length
    salt_len = struct.unpack(">I", bytes(body[off:off + 4]))[0]
    return off + 4 + salt_len


def test_hostile_bcrypt_rounds_are_refused():
    """A key asking for 2^32-1 bcrypt rounds would make x/crypto (and
    ssh-keygen) spin for days; it is refused (DEVIATIONS.md 6)."""
    def huge(body):
        o = _kdf_rounds_offset(body)
        body[o:o + 4] = b"\xff\xff\xff\xff"
    status, text = native.private_key_pem(_rearmour("rsa_openssh_ctr", huge), PASS.encode())
    assert (status, text) == (2, "ssh: bcrypt_pbkdf rounds 4294967295 exceed the limit of 4096")


def test_error_text_with_bytes_that_are_not_utf8():
    """Error texts can carry bytes of the file: Go's %q escapes them where it
    quotes; raw bytes elsewhere come back as surrogate escapes instead of
    failing the call (a fuzz run under ASan found one)."""
    data = b"-----BEGIN \xf4\x90 KEY-----\nAAAA\n-----END \xf4\x90 KEY-----\n"
    assert native.private_key_pem(data, None) == (2, 'ssh: unsupported key type "\\xf4\\x90 KEY"')
    block = native.pem_decode(b"-----BEGIN K-----\nX-\xff: \xfe\n\naGVs\n-----END K-----\n")
    assert block == ("K", [("X-\udcff", "\udcfe")], b"hel")
