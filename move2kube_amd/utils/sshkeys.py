"""SSH keys for the CI/CD git secrets (reference ``internal/common/sshkeys/sshkeys.go``).

Public host keys for github.com, gitlab.com and bitbucket.org are built in;
the user's ``~/.ssh/known_hosts`` and private keys are only read after a QA
confirmation.  Private keys are parsed, decrypted and re-encoded to PEM
(PKCS#1 RSA / SEC1 EC, what ``x509.MarshalPKCS1PrivateKey`` /
``MarshalECPrivateKey`` write and Tekton's git-init accepts) in process by the
native ``_m2k_sshkey`` extension (``ops/csrc/sshkey.cpp``: OpenSSH, legacy
encrypted PEM, PKCS#1/#8, SEC1), as ``ssh.ParseRawPrivateKey`` does in the
reference; a key is encrypted when parsing says so, and its passphrase is
asked through a Password problem (never cached).  Where the extension is not
built, ``ssh-keygen`` does the re-encoding instead.
"""

import os
import shutil
import subprocess
import tempfile

from . import common, log
from .knownhosts import KnownHostsError, parse_known_hosts

DOMAIN_TO_PUBLIC_KEYS = {
    "github.com": ["github.com ssh-rsa AAAAB3NzaC1yc2EAAAABIwAAAQEAq2A7hRGmdnm9tUDbO9IDSwBK6TbQa+PXYPCPy6rbTrTtw7PHkccKrpp0yVhp5HdEIcKr6pLlVDBfOLX9QUsyCOV0wzfjIJNlGEYsdlLJizHhbn2mUjvSAHQqZETYP81eFzLQNnPHt4EVVUh7VfDESU84KezmD5QlWpXLmvU31/yMf+Se8xhHTvKSCZIFImWwoG6mbUoWf9nzpIoaSjB+weqqUUmpaaasXVal72J+UX2B+2RPW3RcT0eOzQgqlJL3RKrTJvdsjE3JEAvGq3lGHSZXy28G3skua2SmVi/w4yCE6gbODqnTWlg7+wC604ydGXA8VJiS5ap43JXiUFFAaQ=="],  # noqa: E501
    "gitlab.com": ["gitlab.com ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIAfuCHKVTjquxvt6CM6tdG4SLp1Btn/nOeHHE5UOzRdf",
                   "gitlab.com ssh-rsa AAAAB3NzaC1yc2EAAAADAQABAAABAQCsj2bNKTBSpIYDEGk9KxsGh3mySTRgMtXL583qmBpzeQ+jqCMRgBqB98u3z++J1sKlXHWfM9dyhSevkMwSbhoR8XIq/U0tCNyokEi/ueaBMCvbcTHhO7FcwzY92WK4Yt0aGROY5qX2UKSeOvuP4D6TPqKF1onrSzH9bx9XUf2lEdWT/ia1NEKjunUqu1xOB/StKDHMoX4/OKyIzuS0q/T1zOATthvasJFoPrAjkohTyaDUz2LN5JoH839hViyEG82yB+MjcFV5MU3N1l1QL3cVUCh93xSaua1N85qivl+siMkPGbO5xR/En4iEY6K2XPASUEMaieWVNTRCtJ4S8H+9",  # noqa: E501
                   "gitlab.com ecdsa-sha2-nistp256 AAAAE2VjZHNhLXNoYTItbmlzdHAyNTYAAAAIbmlzdHAyNTYAAABBBFSMqzJeV9rUzU4kWitGjeR4PWSa29SPqJ1fVkhtj3Hw9xjLVXVYrU9QlYWrOLXBpQ6KWjbjTDTdDkoohFzgbEY="],  # noqa: E501
    "bitbucket.org": ["bitbucket.org ssh-rsa AAAAB3NzaC1yc2EAAAABIwAAAQEAubiN81eDcafrgMeLzaFPsw2kNvEcqTKl/VqLat/MaB33pZy0y3rJZtnqwR2qOOvbwKZYKiEO1O6VqNEBxKvJJelCq0dTXWT5pbO2gDXC6h6QDXCaHo6pOHGPUy+YBaGQRGuSusMEASYiWunYN0vCAI8QaXnWMXNMdFP3jHAJH0eDsoiGnLPBlBp4TNm6rYI74nMzgz3B9IikW4WVK+dc8KZJZWYjAuORU3jc1c/NPskD2ASinf8v3xnfXeukU0sJ5N6m5E8VLjObPEO+mN2t/FZTMZLiFqPWc/ALSqnMnnhwrNi2rbfg/rd/IpL8Le3pSBne8+seeFVBoGqzHM9yXw=="],  # noqa: E501
}

_state = {"known_hosts_loaded": False, "keys_loaded": False, "key_dir": "", "keys": []}


def reset():
    _state.update({"known_hosts_loaded": False, "keys_loaded": False, "key_dir": "", "keys": []})


def _home():
    return os.path.expanduser("~")


def load_known_hosts_of_current_user():
    from ..models import qa
    from ..qaengine import fetch_answer
    if _state["known_hosts_loaded"]:
        return
    _state["known_hosts_loaded"] = True
    home = _home()
    log.debug("Home directory: %r", home)
    path = os.path.join(home, ".ssh", "known_hosts")
    log.debug("Looking in the known_hosts at path %r for public keys.", path)
    msg = ("The CI/CD pipeline needs access to the git repos in order to clone, build and push.\n"
           "Move2Kube has public keys for github.com, gitlab.com, and bitbucket.org by default.\n"
           "If any of the repos use ssh authentication we will need public keys in order to verify.\n"
           "Do you want to load the public keys from your [%s]?:" % path)
    prob = qa.new_confirm_problem(msg, ["No, I will add them later if necessary."], False)
    if not fetch_answer(prob).get_bool_answer():
        log.debug("Don't read public keys from known_hosts. They will be added later if necessary.")
        return
    try:
        keys = parse_known_hosts(path)
    except (OSError, KnownHostsError) as e:
        log.warning("Failed to get public keys from the known_hosts file at path %r Error: %r", path,
                    common.go_error_text(e))
        return
    for domain, lines in keys.items():
        DOMAIN_TO_PUBLIC_KEYS.setdefault(domain, lines)
    if log.debug_enabled():   # log.Debug("DomainToPublicKeys:", m): fmt.Sprint, no space after a string
        from .gotemplate import go_sprint
        log.debug("%s", "DomainToPublicKeys:" + go_sprint(DOMAIN_TO_PUBLIC_KEYS))


def _load_ssh_keys_of_current_user():
    from ..models import qa
    from ..qaengine import fetch_answer
    if _state["keys_loaded"]:
        return
    _state["keys_loaded"] = True
    home = _home()
    log.debug("Home directory: %r", home)
    d = os.path.join(home, ".ssh")
    _state["key_dir"] = d
    log.debug("Looking in ssh directory at path %r for keys.", d)
    msg = ("The CI/CD pipeline needs access to the git repos in order to clone, build and push.\n"
           "If any of the repos require ssh keys you will need to provide them.\n"
           "Do you want to load the private ssh keys from [%s]?:" % d)
    prob = qa.new_confirm_problem(msg, ["No, I will add them later if necessary."], False)
    if not fetch_answer(prob).get_bool_answer():
        log.debug("Don't read private keys. They will be added later if necessary.")
        return
    try:
        names = sorted(os.listdir(d))
    except OSError as e:
        log.error("Failed to read the ssh directory at path %r Error: %r", d, common.go_path_error(e, "open"))
        return
    if not names:
        log.warning("No key files where found in %s", d)
        return
    prob = qa.new_multiselect_problem("These are the files we found in %r . Which keys should we consider?" % d,
                                      ["Select all the keys that give acess to git repos."], names, names)
    names = fetch_answer(prob).get_slice_answer()
    if not names:
        log.info("All key files ignored.")
        return
    _state["keys"] = names


class KeyError_(ValueError):
    pass


_PEM_TYPES = ("-----BEGIN RSA PRIVATE KEY-----", "-----BEGIN EC PRIVATE KEY-----")

# SSH_ASKPASS helper: prints what the parent writes into the FIFO named by
# M2K_ASKPASS_FIFO.  Neither the passphrase nor anything derived from it is
# on a command line or in an environment variable.
_ASKPASS = '#!/bin/sh\nexec cat "$M2K_ASKPASS_FIFO"\n'


def _feed_fifo(fifo, secret, done):
    import threading

    def run():
        try:
            with open(fifo, "w") as f:   # blocks until ssh-keygen's askpass opens it
                f.write(secret + "\n")
        except OSError:
            pass
        done.set()
    t = threading.Thread(target=run, daemon=True)
    t.start()
    return t


def _to_pem(path, passphrase=None):
    """Re-encode a private key file as PEM, like ``marshalRSAIntoPEM`` /
    ``marshalECDSAIntoPEM`` (``sshkeys.go:170-232``): PKCS#1 RSA or SEC1 EC.
    Other key types (ed25519, DSA) are an error, as in the reference.

    ``ssh-keygen -p -m PEM -N ''`` does the re-encoding on a private copy.  The
    old passphrase of an encrypted key reaches it through ``SSH_ASKPASS``
    (``SSH_ASKPASS_REQUIRE=force``) and a FIFO in a private directory, never
    through argv or the environment.  Without ``ssh-keygen`` this raises; the
    caller warns and the secret keeps its placeholder."""
    import threading
    exe = shutil.which("ssh-keygen")
    if exe is None:
        raise KeyError_("ssh-keygen is not available to re-encode the private key as PEM")
    with tempfile.TemporaryDirectory(prefix="m2k-key-") as td:
        os.chmod(td, 0o700)
        tmp = os.path.join(td, "key")
        shutil.copyfile(path, tmp)
        os.chmod(tmp, 0o600)
        env = {k: v for k, v in os.environ.items() if not k.startswith("SSH_")}
        done = threading.Event()
        feeder = None
        argv = [exe, "-p", "-m", "PEM", "-N", "", "-f", tmp]
        if passphrase is None:
            argv[2:2] = ["-P", ""]       # not encrypted: an empty old passphrase is no secret
        else:
            helper = os.path.join(td, "askpass")
            with open(helper, "w") as f:
                f.write(_ASKPASS)
            os.chmod(helper, 0o700)
            fifo = os.path.join(td, "pass")
            os.mkfifo(fifo, 0o600)
            env.update({"SSH_ASKPASS": helper, "SSH_ASKPASS_REQUIRE": "force", "DISPLAY": ":0",
                        "M2K_ASKPASS_FIFO": fifo})
            feeder = _feed_fifo(fifo, passphrase, done)
        try:
            p = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, stdin=subprocess.DEVNULL,
                               env=env, timeout=30, start_new_session=True)
        finally:
            if feeder is not None and not done.is_set():
                # askpass never ran: open the reading end so the writer returns
                try:
                    fd = os.open(fifo, os.O_RDONLY | os.O_NONBLOCK)
                    feeder.join(1)
                    os.close(fd)
                except OSError:
                    pass
        if p.returncode != 0:
            raise KeyError_(p.stderr.decode("utf-8", "replace").strip() or "ssh-keygen failed")
        with open(tmp) as f:
            pem = f.read()
        first = pem.lstrip().split("\n", 1)[0].strip()
        if first not in _PEM_TYPES:
            raise KeyError_("Unknown key type [%s]" % _go_key_type(exe, tmp, env))
    return pem


_GO_KEY_TYPES = {"ED25519": "*ed25519.PrivateKey", "DSA": "*dsa.PrivateKey"}


def _go_key_type(exe, path, env):
    """The Go type ``ssh.ParseRawPrivateKey`` would return (for the error text)."""
    try:
        p = subprocess.run([exe, "-l", "-f", path], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                           stdin=subprocess.DEVNULL, env=env, timeout=30)
        kind = p.stdout.decode("ascii", "replace").strip().rsplit("(", 1)[-1].rstrip(")")
    except (OSError, subprocess.SubprocessError):
        kind = ""
    return _GO_KEY_TYPES.get(kind, "*%s.PrivateKey" % (kind.lower() or "unknown"))


def _is_encrypted(path):
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return False
    if b"ENCRYPTED" in data:
        return True
    if shutil.which("ssh-keygen") is None:
        return False
    p = subprocess.run(["ssh-keygen", "-y", "-P", "", "-f", path], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, stdin=subprocess.DEVNULL, timeout=30)
    return p.returncode != 0 and b"incorrect passphrase" in p.stderr


def _native():
    """The in-process converter (``ops/csrc/sshkey.cpp``), or None."""
    if os.environ.get("M2K_DISABLE_NATIVE"):
        return None
    try:
        from ..ops import _m2k_sshkey as m
    except ImportError:
        if os.environ.get("M2K_REQUIRE_NATIVE"):
            raise
        return None
    return m


_PEM_OK, _NEEDS_PASSPHRASE, _PARSE_ERROR, _UNKNOWN_TYPE = 0, 1, 2, 3


def load_ssh_key(filename):
    """``loadSSHKey`` (sshkeys.go:191-232): the key file as PKCS#1 RSA or SEC1
    EC PEM; an encrypted key (``PassphraseMissingError``) asks for its
    passphrase; other key types are ``Unknown key type [%T]``."""
    from ..models import qa
    from ..qaengine import fetch_answer
    path = os.path.join(_state["key_dir"], filename)
    m = _native()
    if m is None:
        return _load_with_ssh_keygen(path, filename)
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError as e:
        err = common.go_path_error(e, "open")
        log.error("Failed to read the private key file at path %s Error: %s", _q(path), _q(str(err)))
        raise
    status, text = m.private_key_pem(data, None)
    if status == _PARSE_ERROR:
        log.error("Failed to parse the private key file at path %s Error %s", _q(path), _q(text))
        raise KeyError_(text)
    if status == _NEEDS_PASSPHRASE:
        prob = qa.new_password_problem("Enter the password to decrypt the private key %s : " % _q(filename),
                                       ["Password:"])
        password = fetch_answer(prob).get_string_answer()
        status, text = m.private_key_pem(data, password.encode("utf-8", "surrogateescape"))
        if status == _PARSE_ERROR:
            log.error("Failed to parse the encrypted private key file at path %s Error %s", _q(path), _q(text))
            raise KeyError_(text)
    if status == _UNKNOWN_TYPE:
        log.error("Unknown key type [%s]", text)
        raise KeyError_("Unknown key type [%s]" % text)
    return text


def _load_with_ssh_keygen(path, filename):
    """The fallback without the extension: ``ssh-keygen`` re-encodes the key."""
    from ..models import qa
    from ..qaengine import fetch_answer
    passphrase = None
    if _is_encrypted(path):
        prob = qa.new_password_problem("Enter the password to decrypt the private key %s : " % _q(filename),
                                       ["Password:"])
        passphrase = fetch_answer(prob).get_string_answer()
    return _to_pem(path, passphrase)


def get_ssh_key(domain):
    """(pem, True) for the key the user picks for ``domain``; ('', False) otherwise."""
    from ..models import qa
    from ..qaengine import fetch_answer
    _load_ssh_keys_of_current_user()
    if not _state["keys"]:
        return "", False
    names = list(_state["keys"]) + ["NONE"]
    prob = qa.new_select_problem("Select the key to use to for the git domain %s :" % domain,
                                 ["If none of the keys are correct, select None."], "NONE", names)
    name = fetch_answer(prob).get_string_answer()
    if name == "NONE":
        log.debug("No key selected for domain %s", domain)
        return "", False
    log.debug("%s", "Loading the key" + name)   # log.Debug("Loading the key", filename): fmt.Sprint
    try:
        return load_ssh_key(name), True
    except (OSError, ValueError, subprocess.SubprocessError) as e:
        log.warning("Failed to load the key %s Error %s", _q(name), _q(str(e)))
        return "", False


def _q(s):
    return log.go_quote(s)
