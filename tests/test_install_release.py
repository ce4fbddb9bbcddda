"""``scripts/install.sh``: the reference's release flow (scripts/install.sh:27-235)
against a mirror served by stub ``curl`` / ``wget`` on PATH.  The archive is
a real ``scripts/builddist.py`` build with its ``.sha256sum``; the other tools
(tar, awk, sha256sum, openssl, python3) are the system's, each present or
absent per test."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "install.sh")
BASE = "https://mirror.example/m2k/releases"
TAG = "v0.3.1"
ARCHIVE = "move2kube-amd-%s-linux-amd64.tar.gz" % TAG
SYSTOOLS = ("bash", "sh", "uname", "tr", "mkdir", "tar", "gzip", "mktemp", "grep", "head", "sed", "awk", "rm", "mv",
            "ln", "id", "cat", "chmod", "dirname", "cp", "env", "printf", "readlink", "basename")

STUB_GET = r"""#!/bin/sh
# stub %(tool)s: serves %(base)s/... from $STUB_ROOT; records every URL
out=""; url=""
while [ $# -gt 0 ]; do
  case "$1" in
    -o|-O) out="$2"; shift ;;
    -*) ;;
    *) url="$1" ;;
  esac
  shift
done
echo "%(tool)s $url" >> "$STUB_LOG"
rel="${url#%(base)s}"
[ "$rel" = "" ] && rel="/index.html"
f="$STUB_ROOT$rel"
if [ ! -f "$f" ]; then echo "%(tool)s: 404 $url" >&2; exit %(code)s; fi
if [ -n "$out" ] && [ "$out" != "-" ]; then cat "$f" > "$out"; else cat "$f"; fi
"""


@pytest.fixture(scope="module")
def archive(tmp_path_factory):
    if os.uname().machine != "x86_64":
        pytest.skip("archives are named for linux-amd64")
    out = tmp_path_factory.mktemp("dist")
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "builddist.py"), "--version", TAG,
                    "--commit", "abc", "--tree", "clean", "--out", str(out)], check=True, stdout=subprocess.PIPE)
    assert (out / ARCHIVE).exists() and (out / (ARCHIVE + ".sha256sum")).exists()
    return out


def _mirror(tmp_path, archive, tags=(TAG,)):
    root = tmp_path / "mirror"
    root.mkdir()
    links = "".join('<a href="/m2k/releases/tag/%s">%s</a>\n' % (t, t) for t in tags)
    (root / "index.html").write_text("<html><body>\n%s</body></html>\n" % links)
    for t in tags:
        d = root / "download" / t
        d.mkdir(parents=True)
        name = "move2kube-amd-%s-linux-amd64.tar.gz" % t
        shutil.copyfile(str(archive / ARCHIVE), str(d / name))
        digest = (archive / (ARCHIVE + ".sha256sum")).read_text().split()[0]
        (d / (name + ".sha256sum")).write_text("%s  %s\n" % (digest, name))
    return root


def _env(tmp_path, mirror, tools=("curl", "sha256sum", "openssl")):
    sysbin = tmp_path / "sysbin"
    sysbin.mkdir()
    for t in SYSTOOLS + tuple(x for x in ("sha256sum", "openssl") if x in tools):
        p = shutil.which(t)
        if p is None:
            pytest.skip("%s not installed" % t)
        os.symlink(p, str(sysbin / t))
    os.symlink(sys.executable, str(sysbin / "python3"))
    for tool, code in (("curl", 22), ("wget", 8)):
        if tool in tools:
            (sysbin / tool).write_text(STUB_GET % {"tool": tool, "base": BASE, "code": code})
            (sysbin / tool).chmod(0o755)
    (sysbin / "sudo").write_text('#!/bin/sh\necho "sudo $*" >> "$STUB_LOG"\nexit 1\n')
    (sysbin / "sudo").chmod(0o755)
    home = tmp_path / "home"
    home.mkdir(exist_ok=True)
    return {"PATH": str(sysbin), "HOME": str(home), "STUB_ROOT": str(mirror), "STUB_LOG": str(tmp_path / "urls.log"),
            "MOVE2KUBE_RELEASE_URL": BASE, "TMPDIR": str(tmp_path)}


def _run(env, *args, **kw):
    return subprocess.run(["bash", SCRIPT] + list(args), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          stdin=subprocess.DEVNULL, timeout=300, **kw)


def _log(tmp_path):
    p = tmp_path / "urls.log"
    return p.read_text().splitlines() if p.exists() else []


def test_latest_install_then_reinstall(tmp_path, archive):
    env = _env(tmp_path, _mirror(tmp_path, archive))
    prefix = tmp_path / "prefix"
    p = _run(env, "latest", str(prefix))
    out = p.stdout.decode()
    assert p.returncode == 0, out
    assert "Downloading %s/download/%s/%s" % (BASE, TAG, ARCHIVE) in out
    assert "Verifying checksum... Done." in out
    lines = out.splitlines()
    assert TAG in lines and lines[-1] == "Done!"     # testVersion runs the installed launcher
    assert "move2kube not found. Is %s/bin on your $PATH?" % prefix in lines
    assert _log(tmp_path) == ["curl " + BASE, "curl %s/download/%s/%s.sha256sum" % (BASE, TAG, ARCHIVE),
                              "curl %s/download/%s/%s" % (BASE, TAG, ARCHIVE)]
    assert subprocess.run([str(prefix / "bin" / "move2kube"), "version"], stdout=subprocess.PIPE,
                          env={"PATH": env["PATH"], "HOME": env["HOME"]}).stdout.decode().strip() == TAG
    # again: already the latest, nothing downloaded
    os.unlink(str(tmp_path / "urls.log"))
    p = _run(env, "latest", str(prefix))
    assert p.returncode == 0 and "Move2Kube %s is already the latest" % TAG in p.stdout.decode()
    assert _log(tmp_path) == ["curl " + BASE]
    assert not any(l.startswith("sudo") for l in _log(tmp_path))   # the prefix is writable


def test_pinned_tag_changes_version(tmp_path, archive):
    env = _env(tmp_path, _mirror(tmp_path, archive, tags=(TAG, "v0.3.2")))
    prefix = tmp_path / "prefix"
    assert _run(env, TAG, str(prefix)).returncode == 0
    p = _run(env, "v0.3.2", str(prefix))
    out = p.stdout.decode()
    assert p.returncode == 0, out
    assert "Move2Kube v0.3.2 is available. Changing from version %s." % TAG in out
    assert "curl %s/download/v0.3.2/move2kube-amd-v0.3.2-linux-amd64.tar.gz" % BASE in _log(tmp_path)


def test_checksum_mismatch_installs_nothing(tmp_path, archive):
    mirror = _mirror(tmp_path, archive)
    (mirror / "download" / TAG / (ARCHIVE + ".sha256sum")).write_text("0" * 64 + "  " + ARCHIVE + "\n")
    env = _env(tmp_path, mirror)
    prefix = tmp_path / "prefix"
    p = _run(env, "latest", str(prefix))
    out = p.stdout.decode()
    assert p.returncode != 0
    assert "does not match. Aborting." in out and "Failed to install move2kube" in out
    assert not prefix.exists()
    assert not list(tmp_path.glob("move2kube-installer-*"))        # the download directory is cleaned up


def test_wget_and_openssl_fallbacks(tmp_path, archive):
    env = _env(tmp_path, _mirror(tmp_path, archive), tools=("wget", "openssl"))
    p = _run(env, "latest", str(tmp_path / "prefix"))
    out = p.stdout.decode()
    assert p.returncode == 0, out
    assert "Verifying checksum... Done." in out
    assert all(l.startswith("wget ") for l in _log(tmp_path))


def test_missing_tools_and_missing_release(tmp_path, archive):
    mirror = _mirror(tmp_path, archive)
    p = _run(_env(tmp_path, mirror, tools=("sha256sum",)), "latest", str(tmp_path / "p1"))
    assert p.returncode != 0 and "Either curl or wget is required" in p.stdout.decode()
    (tmp_path / "sysbin").rename(tmp_path / "sysbin.1")
    p = _run(_env(tmp_path, mirror, tools=("curl",)), "latest", str(tmp_path / "p2"))
    assert p.returncode != 0 and "sha256sum or openssl must first be installed" in p.stdout.decode()
    (tmp_path / "sysbin").rename(tmp_path / "sysbin.2")
    p = _run(_env(tmp_path, mirror), "v9.9.9", str(tmp_path / "p3"))
    out = p.stdout.decode()
    assert p.returncode != 0 and "Unable to download %s/download/v9.9.9/" % BASE in out
    assert not (tmp_path / "p3").exists()


def test_local_archive_still_installs(tmp_path, archive):
    env = _env(tmp_path, _mirror(tmp_path, archive))
    p = _run(env, str(archive / ARCHIVE), str(tmp_path / "prefix"))
    assert p.returncode == 0, p.stdout.decode()
    assert "Verifying checksum... Done." in p.stdout.decode() and _log(tmp_path) == []


@pytest.mark.skipif(os.geteuid() != 0, reason="needs root to run the installer as another user")
def test_sudo_only_for_an_unwritable_prefix(archive):
    import tempfile
    shared = tempfile.mkdtemp(prefix="m2k-install-", dir="/tmp")   # traversable by nobody
    try:
        base = __import__("pathlib").Path(shared)
        os.chmod(shared, 0o755)
        env = _env(base, _mirror(base, archive))
        script = base / "install.sh"
        shutil.copyfile(SCRIPT, str(script))
        prefix = base / "rootonly"
        prefix.mkdir()
        subprocess.run(["chmod", "-R", "a+rX", shared], check=True)
        log = base / "urls.log"
        log.write_text("")
        os.chmod(str(log), 0o666)
        work = base / "work"
        work.mkdir()
        os.chmod(str(work), 0o777)
        env["TMPDIR"] = str(work)
        p = subprocess.run(["bash", str(script), "latest", str(prefix)], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, timeout=300, user=65534, group=65534,
                           cwd=str(work))
        out = p.stdout.decode()
        # the stub sudo refuses, so the install fails -- after it was asked for
        assert p.returncode != 0, out
        lines = log.read_text().splitlines()
        assert any(l.startswith("sudo mkdir -p %s/lib" % prefix) for l in lines), (lines, out)
    finally:
        shutil.rmtree(shared, ignore_errors=True)
