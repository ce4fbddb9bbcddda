"""scripts/installdeps.sh installs pack, kubectl and a v1 operator-sdk into the
install directory (reference scripts/installdeps.sh:40-160), driven here by a
stub ``curl`` on PATH that serves fake release artifacts; ``tar``, ``install``
and the other tools are the system's."""

import os
import shutil
import subprocess
import tarfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "installdeps.sh")
SYSTOOLS = ("bash", "sh", "uname", "tr", "mkdir", "tar", "gzip", "install", "mktemp", "grep", "cut", "rm", "id",
            "cat", "chmod", "dirname", "cp", "env", "printf")

STUB_CURL = r"""#!/bin/sh
# stub curl: -fsSL [-o FILE] URL ; records every URL
out=""; url=""
while [ $# -gt 0 ]; do
  case "$1" in
    -o) out="$2"; shift ;;
    -*) ;;
    *) url="$1" ;;
  esac
  shift
done
echo "$url" >> "$STUB_LOG"
body() {
  case "$url" in
    */stable.txt) printf 'v1.19.4' ;;
    *pack-v*.tgz) cat "$STUB_DIR/pack.tgz" ;;
    */kubectl) printf '#!/bin/sh\necho "kubectl stub"\n' ;;
    *operator-sdk-v1*) printf '#!/bin/sh\necho '"'"'operator-sdk version: "v1.0.0", commit: "stub"'"'"'\n' ;;
    *) echo "curl: (22) The requested URL returned error: 404" >&2; return 22 ;;
  esac
}
if [ -n "$out" ]; then body > "$out"; else body; fi
"""


@pytest.fixture
def env(tmp_path):
    stub = tmp_path / "stub"
    sysbin = tmp_path / "sysbin"
    stub.mkdir()
    sysbin.mkdir()
    for t in SYSTOOLS:
        p = shutil.which(t)
        if p is None:
            pytest.skip("%s not installed" % t)
        os.symlink(p, str(sysbin / t))
    (stub / "curl").write_text(STUB_CURL)
    (stub / "curl").chmod(0o755)
    pack = tmp_path / "pack"
    pack.write_text("#!/bin/sh\necho pack stub\n")
    pack.chmod(0o755)
    with tarfile.open(str(stub / "pack.tgz"), "w:gz") as tf:
        tf.add(str(pack), arcname="pack")
    home = tmp_path / "home"
    home.mkdir()
    return {"PATH": "%s:%s" % (stub, sysbin), "HOME": str(home), "STUB_DIR": str(stub),
            "STUB_LOG": str(tmp_path / "urls.log"), "INSTALL_DOCKER": "0",
            "MOVE2KUBE_DEP_INSTALL_PATH": str(tmp_path / "deps")}


def _run(env, *args, cwd=None):
    return subprocess.run(["bash", SCRIPT] + list(args), env=env, cwd=cwd, stdout=subprocess.PIPE,
                          stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, timeout=60)


def test_installs_missing_tools_into_prefix(env, tmp_path):
    p = _run(env, "-y")
    out = p.stdout.decode()
    assert p.returncode == 0, out
    deps = tmp_path / "deps"
    for tool in ("pack", "kubectl", "operator-sdk"):
        assert os.access(str(deps / tool), os.X_OK), tool
    assert subprocess.run([str(deps / "operator-sdk"), "version"], stdout=subprocess.PIPE).stdout.startswith(
        b'operator-sdk version: "v1')
    urls = (tmp_path / "urls.log").read_text().split()
    assert urls == [
        "https://github.com/buildpacks/pack/releases/download/v0.12.0/pack-v0.12.0-linux.tgz",
        "https://storage.googleapis.com/kubernetes-release/release/stable.txt",
        "https://storage.googleapis.com/kubernetes-release/release/v1.19.4/bin/linux/amd64/kubectl",
        "https://github.com/operator-framework/operator-sdk/releases/download/v1.0.0/"
        "operator-sdk-v1.0.0-x86_64-linux-gnu",
    ] if os.uname().machine == "x86_64" else urls
    assert ('PATH="%s:$PATH"' % deps) in (tmp_path / "home" / ".bash_profile").read_text()
    # a second run finds everything on PATH and downloads nothing
    env2 = dict(env, PATH="%s:%s" % (deps, env["PATH"]))
    os.remove(str(tmp_path / "urls.log"))
    p = _run(env2, "-y")
    assert p.returncode == 0, p.stdout.decode()
    assert not (tmp_path / "urls.log").exists()
    assert "already on $PATH" in p.stdout.decode()


def test_old_operator_sdk_is_replaced_and_versions_pin(env, tmp_path):
    old = tmp_path / "stub" / "operator-sdk"
    old.write_text('#!/bin/sh\necho \'operator-sdk version: "v0.19.2", commit: "old"\'\n')
    old.chmod(0o755)
    env = dict(env, PACK_VERSION="v0.13.1", KUBECTL_VERSION="v1.20.0",
               OPERATOR_SDK_URL="https://mirror.example/operator-sdk-v1.3.0")
    p = _run(env, "-y")
    out = p.stdout.decode()
    assert p.returncode == 0, out
    assert "is not v1" in out
    urls = (tmp_path / "urls.log").read_text().split()
    assert urls[0].endswith("/v0.13.1/pack-v0.13.1-linux.tgz")
    assert "stable.txt" not in " ".join(urls) and urls[1].endswith("/v1.20.0/bin/linux/%s/kubectl" % (
        "amd64" if os.uname().machine == "x86_64" else "arm64"))
    assert urls[2] == "https://mirror.example/operator-sdk-v1.3.0"
    assert os.access(str(tmp_path / "deps" / "operator-sdk"), os.X_OK)


def test_failed_download_fails_the_install(env, tmp_path):
    env = dict(env, OPERATOR_SDK_URL="https://mirror.example/nothing-here")
    p = _run(env, "-y")
    assert p.returncode != 0
    assert "Failed to install the dependencies" in p.stdout.decode()
    assert not (tmp_path / "deps" / "operator-sdk").exists()


def test_check_mode_and_bad_args(env, tmp_path):
    p = _run(env, "--check")
    out = p.stdout.decode()
    assert p.returncode == 0 and "pack          MISSING" in out and "operator-sdk  MISSING" in out
    assert not (tmp_path / "deps").exists()
    p = _run(env, "-x")
    assert p.returncode == 1 and "Usage: installdeps.sh [-y] [--check]" in p.stdout.decode()


def test_prompt_declined_installs_nothing(env, tmp_path):
    p = subprocess.run(["bash", SCRIPT], env=env, input=b"n\n", stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       timeout=60)
    assert p.returncode == 1 and "nothing installed" in p.stdout.decode()
    assert not (tmp_path / "deps").exists()


def test_force_install_ignores_tools_already_on_path(env, tmp_path):
    # FORCE_INSTALL=1 (the image build): every tool goes to the install
    # directory even when PATH has a good one
    for t, body in (("pack", "echo pack"), ("kubectl", "echo kubectl"),
                    ("operator-sdk", 'echo \'operator-sdk version: "v1.2.0", commit: "x"\'')):
        p = tmp_path / "stub" / t
        p.write_text("#!/bin/sh\n%s\n" % body)
        p.chmod(0o755)
    p = _run(env, "-y")
    assert p.returncode == 0 and not (tmp_path / "deps" / "pack").exists()   # present: nothing to do
    p = _run(dict(env, FORCE_INSTALL="1"), "-y")
    out = p.stdout.decode()
    assert p.returncode == 0, out
    for t in ("pack", "kubectl", "operator-sdk"):
        assert os.access(str(tmp_path / "deps" / t), os.X_OK), t
    assert "is not v1" not in out
