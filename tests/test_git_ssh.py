"""The git / SSH subsystem behind the Tekton git secrets:

* ``utils/git.py``: ``GetGitRemoteNames`` / ``GetGitRepoDetails`` /
  ``GetGitRepoName`` (``internal/common/utils.go:636-718``), including Go's
  ``filepath.Base``/``Ext`` and ``url.Parse`` edge cases;
* ``utils/knownhosts.py``: ``ParseKnownHosts`` and ``GetKnownHostsLine``
  (``internal/common/knownhosts/knownhosts.go:50-166``);
* ``utils/sshkeys.py``: the known_hosts / private-key QA and the PEM
  re-encoding of ``sshkeys.go:36-270``.
"""

import base64
import os
import shutil
import stat
import subprocess

import pytest

import logparse

from move2kube_amd import qaengine
from move2kube_amd.qaengine.engine import Engine
from move2kube_amd.utils import git, knownhosts, log, sshkeys

HAVE_KEYGEN = shutil.which("ssh-keygen") is not None


# -- git ---------------------------------------------------------------------

def _repo(root, config, head="ref: refs/heads/main\n", refs=("refs/heads/main",)):
    d = root / ".git"
    d.mkdir(parents=True)
    (d / "HEAD").write_text(head)
    (d / "config").write_text(config)
    for r in refs:
        p = d / r
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("3f786850e387550fdab836ed7e6dc881de23001b\n")
    return root


def _remote(url, name="origin"):
    return '[core]\n\tbare = false\n[remote "%s"]\n\turl = %s\n' % (name, url)


@pytest.mark.parametrize("path,base", [("", "."), ("/", "/"), ("a/b/", "b"), ("//", "/"), ("x", "x"),
                                       ("/a/b.git", "b.git")])
def test_go_base(path, base):
    assert git.go_base(path) == base


@pytest.mark.parametrize("path,ext", [(".cfg", ".cfg"), ("a.b.git", ".git"), ("a/b", ""), ("a.d/b", ""),
                                      ("/", ""), (".", ".")])
def test_go_ext(path, ext):
    assert git.go_ext(path) == ext


@pytest.mark.parametrize("url,name", [
    ("git@github.com:konveyor/move2kube-demos.git", "move2kube-demos"),
    ("https://github.com/konveyor/move2kube.git", "move2kube"),
    ("https://github.com/konveyor/move2kube", "move2kube"),
    ("https://github.com/konveyor/move2kube/", "move2kube"),
    ("https://example.com/a/b.tar.gz", "b.tar"),
    ("ssh://git@example.com:2222/team/tool.git", "tool"),
    ("https://example.com/team/.cfg", ""),        # filepath.Ext(".cfg") is the whole name
    ("https://example.com", ""),                  # Path "" -> Base "." -> Ext "." -> ""
    ("https://example.com/", "/"),                # Base("/") is "/", which has no extension
    ("https://example.com/my%20repo.git", "my repo"),   # url.Path is unescaped
    ("https://example.com/bad%zzescape.git", None),     # invalid escape: url.Parse error
    ("https://example.com:port/x.git", None),            # invalid port
    ("mailto:someone", ""),                       # opaque URL: empty Path
    ("git@host:a:b", None),                       # scp form with two colons
    ("gitlab:group/sub", "sub"),                  # starts with "git": split at ':'
])
def test_repo_name_follows_go(tmp_path, url, name):
    _repo(tmp_path, _remote(url))
    got, root = git.repo_name(str(tmp_path))
    if name is None:
        assert (got, root) == ("", "")
    else:
        assert (got, root) == (name, str(tmp_path))


def test_repo_name_without_origin_or_repo(tmp_path):
    _repo(tmp_path / "r", _remote("https://x/y.git", name="upstream"))
    assert git.repo_name(str(tmp_path / "r")) == ("", "")
    (tmp_path / "plain").mkdir()
    assert git.repo_name(str(tmp_path / "plain")) == ("", "")


def test_repo_details_branch_resolution(tmp_path):
    # loose ref
    _repo(tmp_path / "a", _remote("git@github.com:o/a.git"))
    urls, branch, root = git.repo_details(str(tmp_path / "a"), "origin")
    assert (urls, branch, root) == (["git@github.com:o/a.git"], "main", str(tmp_path / "a"))
    # packed ref
    b = _repo(tmp_path / "b", _remote("u"), head="ref: refs/heads/feature/x\n", refs=())
    (b / ".git" / "packed-refs").write_text("# pack-refs with: peeled\n"
                                            "89e6c98d92887913cadf06b2adb97f26cde4849b refs/heads/feature/x\n")
    assert git.repo_details(str(b), "origin")[1] == "x"     # filepath.Base of the ref name
    # unborn branch: go-git's Head() fails, so the branch stays empty
    _repo(tmp_path / "c", _remote("u"), refs=())
    assert git.repo_details(str(tmp_path / "c"), "origin")[1] == ""
    # detached HEAD
    _repo(tmp_path / "d", _remote("u"), head="3f786850e387550fdab836ed7e6dc881de23001b\n")
    assert git.repo_details(str(tmp_path / "d"), "origin")[1] == "HEAD"
    # a subdirectory finds the repo above it (DetectDotGit)
    sub = tmp_path / "a" / "x" / "y"
    sub.mkdir(parents=True)
    assert git.repo_details(str(sub), "origin")[2] == str(tmp_path / "a")


def test_remote_names_and_gitdir_file(tmp_path):
    cfg = _remote("https://a/u.git", "upstream") + '[remote "origin"]\n\turl = https://a/o.git\n'
    real = _repo(tmp_path / "real", cfg)
    wt = tmp_path / "wt"
    wt.mkdir()
    (wt / ".git").write_text("gitdir: %s\n" % (real / ".git"))
    assert git.remote_names(str(wt)) == ["upstream", "origin"]
    assert git.repo_details(str(wt), "upstream")[0] == ["https://a/u.git"]


def test_gather_git_info_prefers_upstream_then_origin(tmp_path):
    from move2kube_amd.models import plan as plantypes
    cfg = _remote("https://a/o.git") + '[remote "upstream"]\n\turl = https://a/u.git\n'
    _repo(tmp_path / "r", cfg)
    s = plantypes.Service.new("svc", plantypes.ANY2KUBE)
    assert s.gather_git_info(str(tmp_path / "r"))[0]
    assert s.repo_info.git_repo_url == "https://a/u.git"
    _repo(tmp_path / "o", _remote("https://a/o.git") + '[remote "fork"]\n\turl = https://a/f.git\n')
    s2 = plantypes.Service.new("svc2", plantypes.ANY2KUBE)
    s2.gather_git_info(str(tmp_path / "o"))
    assert s2.repo_info.git_repo_url == "https://a/o.git"


def test_config_is_read_as_git_config(tmp_path):
    """go-git's config decoder: section names case-insensitive, quotes and
    escapes removed, comments dropped, every ``url`` kept in order (the first
    is the one GetGitRepoDetails' callers use)."""
    cfg = ('[Remote "origin"]\n\tURL = "https://a/o.git" ; the fork\n\turl = https://b/o.git # mirror\n'
           '[remote.Upstream]\n\turl = git@u:x/y.git\n')
    _repo(tmp_path / "r", cfg)
    assert git.remote_names(str(tmp_path / "r")) == ["origin", "upstream"]
    assert git.repo_details(str(tmp_path / "r"), "origin")[0] == ["https://a/o.git", "https://b/o.git"]
    assert git.parse_config('[a "s\\"q"]\n x = "p q" r\\\n  s\n y\n') == [("a", 's"q', "x", "p q r  s"), ("a", 's"q', "y", None)]


def test_unparsable_config_has_no_remotes(tmp_path, capsys):
    from move2kube_amd.utils import log
    _repo(tmp_path / "r", '[remote "origin"]\n\turl = "https://a/o.git\n')
    with pytest.raises(git.GitConfigError):
        git.remote_names(str(tmp_path / "r"))
    log.set_verbose(True)
    try:
        assert git.repo_details(str(tmp_path / "r"), "origin") == ([], "main", str(tmp_path / "r"))
    finally:
        log.set_verbose(False)
    assert "Unable to get remote named origin Error: " in capsys.readouterr().err


def test_dot_git_discovery_stops_at_the_first_entry(tmp_path):
    """dotGitToOSFilesystems: the walk up stops at the first ``.git``, file or
    directory; a ``.git`` file needs the ``gitdir: `` prefix, and a ``.git``
    directory without HEAD is no repository (the walk does not go on)."""
    _repo(tmp_path, _remote("https://a/top.git"))
    bad_file = tmp_path / "sub1"
    bad_file.mkdir()
    (bad_file / ".git").write_text("nonsense\n")
    with pytest.raises(git.GitError, match="^.git file has no gitdir:  prefix$"):
        git.remote_names(str(bad_file))
    empty = tmp_path / "sub2"
    (empty / ".git").mkdir(parents=True)
    with pytest.raises(git.GitError, match="^repository does not exist$"):
        git.repo_details(str(empty), "origin")
    (tmp_path / "sub3").mkdir()
    assert git.repo_details(str(tmp_path / "sub3"), "origin")[2] == str(tmp_path)


# -- known_hosts ---------------------------------------------------------------

def _keys():
    """Public keys made with ssh-keygen (tests/fixtures/sshkeys/public_keys.txt)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "sshkeys", "public_keys.txt")
    with open(path) as f:
        return dict(ln.split()[0:2] for ln in f if ln.strip())


def _wire(*fields):
    return b"".join(len(f).to_bytes(4, "big") + f for f in fields)


def _b64(raw):
    return base64.b64encode(raw).decode()


def test_parse_known_hosts(tmp_path):
    k = _keys()
    kh = tmp_path / "known_hosts"
    kh.write_bytes(("\n".join([
        "# comment",
        "",
        "github.com,140.82.121.3 ssh-rsa %s" % k["ssh-rsa"],
        "gitlab.example.com\tssh-ed25519   %s comment here\r" % k["ssh-ed25519"],
        "@cert-authority *.example.com ssh-rsa %s" % k["ssh-rsa"],
        "@revoked old.example.com ssh-dss %s" % k["ssh-dss"],
        "|1|abc=|def= ecdsa-sha2-nistp256 %s" % k["ecdsa-sha2-nistp256"],
        "github.com ecdsa-sha2-nistp384 %s" % k["ecdsa-sha2-nistp384"],
        "  p521.example.com ecdsa-sha2-nistp521 %s  " % k["ecdsa-sha2-nistp521"],
    ]) + "\n# caf\xe9\n").encode("latin-1"))   # a byte that is not UTF-8, in a comment
    got = knownhosts.parse_known_hosts(str(kh))
    assert sorted(got) == ["140.82.121.3", "github.com", "gitlab.example.com", "p521.example.com"]
    assert len(got["github.com"]) == 2 and got["github.com"][0].startswith("github.com,140.82.121.3 ssh-rsa ")
    assert got["gitlab.example.com"] == ["gitlab.example.com\tssh-ed25519   %s comment here" % k["ssh-ed25519"]]


@pytest.mark.parametrize("blob,err", [
    # ssh.ParsePublicKey (x/crypto/ssh keys.go) and base64.StdEncoding texts
    ("!!notbase64!!", "illegal base64 data at input byte 0"),
    ("AAAAB3NzaC1yc2E=x", "illegal base64 data at input byte 16"),
    (_b64(_wire(b"ssh-foo")), "ssh: unknown key algorithm: ssh-foo"),
    (_b64(b"\x00\x00\x00\x07ssh-rsa\x00\x00\x00\x01\x23"), "ssh: short read"),
    (_b64(_wire(b"ssh-rsa", b"\x01\x00\x00\x01", b"\x00\xc3")), "ssh: exponent too large"),
    (_b64(_wire(b"ssh-rsa", b"\x01\x00", b"\x00\xc3")), "ssh: incorrect exponent"),
    (_b64(_wire(b"ssh-rsa", b"\x01\x00\x01", b"\x00\xc3", b"x")), "ssh: trailing junk in public key"),
    (_b64(_wire(b"ssh-ed25519", b"\x01" * 31)), "invalid size 31 for Ed25519 public key"),
    (_b64(_wire(b"ecdsa-sha2-nistp256", b"nistp999", b"\x04")), "ssh: unsupported curve"),
    (_b64(_wire(b"ecdsa-sha2-nistp256", b"nistp256", b"\x04" + b"\x01" * 64)), "ssh: invalid curve point"),
])
def test_key_blob_errors_read_like_x_crypto_ssh(tmp_path, blob, err):
    kh = tmp_path / "known_hosts"
    kh.write_text("# first\nok ssh-rsa %s\nhost ssh-rsa %s\n" % (_keys()["ssh-rsa"], blob))
    with pytest.raises(knownhosts.KnownHostsError) as ei:
        knownhosts.parse_known_hosts(str(kh))
    assert str(ei.value) == 'Error occurred parsing known_hosts file at path "%s" on line no. 3 Error: "%s"' % (kh, err)


@pytest.mark.parametrize("line,err", [
    ("lonelyhost", "missing host pattern"),
    ("@revoked", "missing host pattern"),
    ("host ssh-rsa", "missing key type pattern"),
])
def test_parse_known_hosts_errors_name_the_line(tmp_path, line, err):
    kh = tmp_path / "known_hosts"
    kh.write_text("# first\nok ssh-rsa %s\n%s\n" % (_keys()["ssh-rsa"], line))
    with pytest.raises(knownhosts.KnownHostsError, match="on line no. 3 .*%s" % err):
        knownhosts.parse_known_hosts(str(kh))


def test_known_hosts_lines_split_like_bufio_scanner(tmp_path):
    """A line of 64 KiB or more ends bufio.Scanner's scan: ParseKnownHosts
    returns scanner.Err()."""
    kh = tmp_path / "known_hosts"
    kh.write_text("ok ssh-rsa %s\n# %s\n" % (_keys()["ssh-rsa"], "x" * 70000))
    with pytest.raises(knownhosts.KnownHostsError, match="^bufio.Scanner: token too long$"):
        knownhosts.parse_known_hosts(str(kh))
    from move2kube_amd.utils.common import go_scan_lines
    assert go_scan_lines(b"a\r\nb\rc\n\nd") == ([b"a", b"b\rc", b"", b"d"], False)


def test_host_key_line_follows_go_client_preference():
    scan = ["# host:22 SSH-2.0-OpenSSH_8.9",
            "host ssh-ed25519 AAAAed", "host ssh-rsa AAAArsa", "host ecdsa-sha2-nistp256 AAAAec"]
    assert knownhosts.pick_host_key_line(scan, "host") == "host ecdsa-sha2-nistp256 AAAAec"
    assert knownhosts.pick_host_key_line(scan[:3], "host") == "host ssh-rsa AAAArsa"
    assert knownhosts.pick_host_key_line(scan[:2], "host") == "host ssh-ed25519 AAAAed"
    assert knownhosts.pick_host_key_line([], "host") == ""


def test_get_known_hosts_line_uses_every_key_type(tmp_path, monkeypatch):
    stub = tmp_path / "bin" / "ssh-keyscan"
    stub.parent.mkdir()
    log = tmp_path / "argv"
    stub.write_text('#!/bin/sh\necho "$@" > %s\n'
                    'echo "# $3 SSH-2.0"\necho "$5 ssh-ed25519 AAAAed"\necho "$5 ssh-rsa AAAArsa"\n' % log)
    stub.chmod(0o755)
    monkeypatch.setenv("PATH", str(stub.parent) + os.pathsep + os.environ["PATH"])
    monkeypatch.delenv("M2K_NO_NETWORK", raising=False)
    # the in-process handshake (tests/test_sshwire.py) fails: ssh-keyscan is the fallback
    monkeypatch.setattr(knownhosts, "fetch_line_in_process", lambda host, timeout=5, port=22: "")
    assert knownhosts.get_known_hosts_line("git.example.org") == "git.example.org ssh-rsa AAAArsa"
    assert "rsa,ecdsa,ed25519" in log.read_text()
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    assert knownhosts.get_known_hosts_line("git.example.org") == ""


# -- sshkeys -------------------------------------------------------------------

class _Answers(Engine):
    """Answers problems by description prefix; records what was asked."""

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
def qa_home(tmp_path, monkeypatch):
    home = tmp_path / "home"
    (home / ".ssh").mkdir(parents=True)
    monkeypatch.setenv("HOME", str(home))
    sshkeys.reset()
    saved = dict(sshkeys.DOMAIN_TO_PUBLIC_KEYS)
    qaengine.reset()
    yield home
    qaengine.reset()
    sshkeys.reset()
    sshkeys.DOMAIN_TO_PUBLIC_KEYS.clear()
    sshkeys.DOMAIN_TO_PUBLIC_KEYS.update(saved)


def _keygen(path, kind, passphrase="", fmt=None):
    argv = ["ssh-keygen", "-q", "-t", kind, "-N", passphrase, "-f", str(path)]
    if kind == "rsa":
        argv[4:4] = ["-b", "2048"]
    if fmt:
        argv += ["-m", fmt]
    subprocess.run(argv, check=True, stdin=subprocess.DEVNULL)


def test_known_hosts_of_user_are_added_after_confirm(qa_home):
    (qa_home / ".ssh" / "known_hosts").write_text("git.corp.example ssh-rsa %s\n" % _keys()["ssh-rsa"])
    eng = _Answers({"The CI/CD pipeline needs access": ["true"]})
    qaengine.add_engine(eng)
    sshkeys.load_known_hosts_of_current_user()
    assert sshkeys.DOMAIN_TO_PUBLIC_KEYS["git.corp.example"][0].startswith("git.corp.example ssh-rsa")
    assert eng.asked[0][0] == "Confirm" and str(qa_home / ".ssh" / "known_hosts") in eng.asked[0][1]
    sshkeys.load_known_hosts_of_current_user()          # asked once per run
    assert len(eng.asked) == 1


def test_known_hosts_not_read_when_declined(qa_home):
    (qa_home / ".ssh" / "known_hosts").write_text("declined.example ssh-rsa %s\n" % _keys()["ssh-rsa"])
    qaengine.add_engine(_Answers({}))                    # the default is "no"
    sshkeys.load_known_hosts_of_current_user()
    assert "declined.example" not in sshkeys.DOMAIN_TO_PUBLIC_KEYS


@pytest.mark.skipif(not HAVE_KEYGEN, reason="ssh-keygen not installed")
def test_select_key_through_qa_cache(qa_home, tmp_path):
    _keygen(qa_home / ".ssh" / "id_ecdsa", "ecdsa")
    _keygen(qa_home / ".ssh" / "id_ed25519", "ed25519")
    cache = tmp_path / "qa.yaml"
    cache.write_text(
        "apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
        "    - description: |-\n"
        "        The CI/CD pipeline needs access to the git repos in order to clone, build and push.\n"
        "        If any of the repos require ssh keys you will need to provide them.\n"
        "        Do you want to load the private ssh keys from [%s]?:\n"
        "      solution:\n        type: Confirm\n        answer:\n          - \"true\"\n      resolved: true\n"
        "    - description: These are the files we found in \"%s\" . Which keys should we consider?\n"
        "      solution:\n        type: MultiSelect\n        answer:\n          - id_ecdsa\n          - id_ed25519\n"
        "      resolved: true\n"
        "    - description: 'Select the key to use to for the git domain git.corp.example :'\n"
        "      solution:\n        type: Select\n        answer:\n          - id_ecdsa\n      resolved: true\n"
        "    - description: 'Select the key to use to for the git domain other.example :'\n"
        "      solution:\n        type: Select\n        answer:\n          - id_ed25519\n      resolved: true\n"
        % (qa_home / ".ssh", qa_home / ".ssh"))
    qaengine.start_engine(qaskip=True)
    qaengine.add_caches([str(cache)])
    key, ok = sshkeys.get_ssh_key("git.corp.example")
    assert ok and key.startswith("-----BEGIN EC PRIVATE KEY-----")
    # ed25519 has no PEM form in the reference (ParseRawPrivateKey -> *ed25519.PrivateKey): not used
    assert sshkeys.get_ssh_key("other.example") == ("", False)


@pytest.fixture
def keygen_fallback(monkeypatch):
    """The path without the native key converter: ssh-keygen re-encodes."""
    monkeypatch.setattr(sshkeys, "_native", lambda: None)


@pytest.mark.skipif(not HAVE_KEYGEN, reason="ssh-keygen not installed")
@pytest.mark.parametrize("fmt", [None, "PEM"])
def test_encrypted_key_through_password_problem(qa_home, monkeypatch, fmt, keygen_fallback):
    secret = "correct horse battery"
    _keygen(qa_home / ".ssh" / "id_rsa", "rsa", passphrase=secret, fmt=fmt)
    eng = _Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["id_rsa"],
                    "Select the key": ["id_rsa"], "Enter the password": [secret]})
    qaengine.add_engine(eng)
    seen = []
    real_popen = subprocess.Popen

    class SpyPopen(real_popen):
        def __init__(self, args, *a, **kw):
            seen.append((list(args), dict(kw.get("env") or os.environ)))
            super().__init__(args, *a, **kw)
    monkeypatch.setattr(subprocess, "Popen", SpyPopen)
    key, ok = sshkeys.get_ssh_key("git.corp.example")
    assert ok and key.startswith("-----BEGIN RSA PRIVATE KEY-----") and "ENCRYPTED" not in key
    assert ("Password", 'Enter the password to decrypt the private key "id_rsa" : ') in [
        (t, d.replace("'", '"')) for t, d in eng.asked]
    assert seen, "ssh-keygen was not run"
    for argv, env in seen:
        assert not any(secret in a for a in argv), argv
        assert not any(secret in v for v in env.values())


@pytest.mark.skipif(not HAVE_KEYGEN, reason="ssh-keygen not installed")
@pytest.mark.parametrize("fallback", [False, True])
def test_wrong_password_keeps_placeholder(qa_home, monkeypatch, fallback):
    if fallback:
        monkeypatch.setattr(sshkeys, "_native", lambda: None)
    _keygen(qa_home / ".ssh" / "id_rsa", "rsa", passphrase="right-one")
    qaengine.add_engine(_Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["id_rsa"],
                                  "Select the key": ["id_rsa"], "Enter the password": ["wrong-one"]}))
    assert sshkeys.get_ssh_key("git.corp.example") == ("", False)


def test_missing_ssh_keygen_is_a_warning_not_an_openssh_key(qa_home, monkeypatch, capsys, keygen_fallback):
    k = qa_home / ".ssh" / "id_rsa"
    k.write_text("-----BEGIN OPENSSH PRIVATE KEY-----\nAAAA\n-----END OPENSSH PRIVATE KEY-----\n")
    k.chmod(stat.S_IRUSR | stat.S_IWUSR)
    qaengine.add_engine(_Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["id_rsa"],
                                  "Select the key": ["id_rsa"]}))
    monkeypatch.setattr(shutil, "which", lambda name, *a, **kw: None)
    assert sshkeys.get_ssh_key("git.corp.example") == ("", False)
    assert "ssh-keygen is not available" in capsys.readouterr().err


def test_no_keys_selected_when_declined(qa_home):
    (qa_home / ".ssh" / "id_rsa").write_text("x")
    eng = _Answers({})
    qaengine.add_engine(eng)
    assert sshkeys.get_ssh_key("github.com") == ("", False)
    assert [t for t, _ in eng.asked] == ["Confirm"]


def test_unreadable_known_hosts_is_a_warning(qa_home, capsys):
    (qa_home / ".ssh" / "known_hosts").mkdir()            # a directory: the read fails
    qaengine.add_engine(_Answers({"The CI/CD pipeline needs access": ["true"]}))
    sshkeys.load_known_hosts_of_current_user()
    assert logparse.logged_containing(capsys.readouterr().err, "Failed to get public keys from the known_hosts file "
                                      "at path", "warning")


@pytest.mark.parametrize("case", ["no-dir", "empty", "none-selected", "key-none"])
def test_private_key_selection_edges(qa_home, capsys, case):
    """sshkeys.go:105-160: no ~/.ssh (an error line), an empty one (a warning),
    every key unselected (an info line), and NONE for the domain."""
    import shutil as _sh
    log.set_verbose(True)
    answers = {"The CI/CD pipeline needs access": ["true"]}
    if case == "no-dir":
        _sh.rmtree(str(qa_home / ".ssh"))
    elif case != "empty":
        (qa_home / ".ssh" / "id_rsa").write_text("x")
        answers["These are the files"] = [] if case == "none-selected" else ["id_rsa"]
        answers["Select the key"] = ["NONE"]
    qaengine.add_engine(_Answers(answers))
    try:
        assert sshkeys.get_ssh_key("git.corp.example") == ("", False)
    finally:
        log.set_verbose(False)
    err = capsys.readouterr().err
    want = {"no-dir": ("error", "Failed to read the ssh directory at path"),
            "empty": ("warning", "No key files where found in"),
            "none-selected": ("info", "All key files ignored."),
            "key-none": ("debug", "No key selected for domain git.corp.example")}[case]
    assert logparse.logged_containing(err, want[1], want[0])


@pytest.mark.skipif(not HAVE_KEYGEN, reason="ssh-keygen not installed")
def test_keygen_fallback_names_the_go_key_type(qa_home, capsys, keygen_fallback):
    """Without the extension, an Ed25519 key fails as ``ParseRawPrivateKey``'s
    type does in the reference's error text."""
    _keygen(qa_home / ".ssh" / "id_ed25519", "ed25519")
    qaengine.add_engine(_Answers({"The CI/CD pipeline needs access": ["true"], "These are the files": ["id_ed25519"],
                                  "Select the key": ["id_ed25519"]}))
    assert sshkeys.get_ssh_key("git.corp.example") == ("", False)
    assert 'Unknown key type [*ed25519.PrivateKey]' in capsys.readouterr().err


def test_native_converter_switches(monkeypatch):
    monkeypatch.setenv("M2K_DISABLE_NATIVE", "1")
    assert sshkeys._native() is None
    monkeypatch.delenv("M2K_DISABLE_NATIVE")
    import builtins
    real = builtins.__import__

    def no_ext(name, *a, **k):
        if a and a[2] and "_m2k_sshkey" in a[2]:
            raise ImportError("not built")
        return real(name, *a, **k)
    monkeypatch.setattr(builtins, "__import__", no_ext)
    assert sshkeys._native() is None
    monkeypatch.setenv("M2K_REQUIRE_NATIVE", "1")
    with pytest.raises(ImportError):
        sshkeys._native()


def test_user_key_loading_debug_lines(qa_home, capsys):
    """sshkeys.go:60-63,97,111-113: the home and the paths looked in, and the
    merged host keys as log.Debug's fmt.Sprint prints a Go map."""
    (qa_home / ".ssh" / "known_hosts").write_text("git.corp.example ssh-rsa %s\n" % _keys()["ssh-rsa"])
    qaengine.add_engine(_Answers({"The CI/CD pipeline needs access": ["true"]}))
    log.set_verbose(True)
    try:
        sshkeys.load_known_hosts_of_current_user()
        sshkeys._load_ssh_keys_of_current_user()
    finally:
        log.set_verbose(False)
    msgs = [m for lv, m in logparse.messages(capsys.readouterr().err) if lv == "debug"]
    assert msgs.count('Home directory: "%s"' % qa_home) == 2
    assert 'Looking in the known_hosts at path "%s" for public keys.' % (qa_home / ".ssh" / "known_hosts") in msgs
    assert 'Looking in ssh directory at path "%s" for keys.' % (qa_home / ".ssh") in msgs
    (dump,) = [m for m in msgs if m.startswith("DomainToPublicKeys:")]
    assert dump.startswith("DomainToPublicKeys:map[") and "git.corp.example:[git.corp.example ssh-rsa " in dump
