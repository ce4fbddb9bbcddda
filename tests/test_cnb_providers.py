"""CNB provider chain against fakes: a Docker Engine API served on a unix
socket, and stub podman / pack executables."""

import itertools
import json
import os
import socketserver
import sys
import threading
from http.server import BaseHTTPRequestHandler

import pytest

from move2kube_amd.containerizer.cnb import providers

STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "stubbin")
LABEL = json.dumps([{"group": [{"id": "google.nodejs.runtime"}, {"id": "google.go.runtime"}]}])


_FAKE_LOCK = threading.Lock()
_FAKE_IDS = itertools.count()


class _FakeDockerd(BaseHTTPRequestHandler):
    state = {}

    def log_message(self, *a):
        pass

    def _json(self, code, obj):
        data = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_POST(self):  # noqa: N802
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n else b""
        if self.path.startswith("/images/create"):
            self.state.setdefault("pulls", []).append(self.path)
            if "doesnotexist" in self.path:   # what dockerd answers for an image no registry has
                return self._json(404, {"message": "pull access denied for this/doesnotexist"})
            return self._json(200, {"status": "pulled"})
        if self.path == "/containers/create":
            cfg = json.loads(body or b"{}")
            with _FAKE_LOCK:
                cid = "c%d" % next(_FAKE_IDS)
            mounts = (cfg.get("HostConfig") or {}).get("Mounts") or []
            src = mounts[0]["Source"] if mounts else ""
            self.state[cid] = 0 if (cfg.get("Image") == "hello-world" or os.path.exists(os.path.join(src, "package.json"))) else 1
            return self._json(201, {"Id": cid})
        if self.path.endswith("/start"):
            return self._json(204, {})
        if "/wait" in self.path:
            cid = self.path.split("/")[2]
            return self._json(200, {"StatusCode": self.state.get(cid, 1)})
        return self._json(404, {"message": "no"})

    def do_GET(self):  # noqa: N802
        if "/logs" in self.path:
            return self._json(200, "detected")
        if self.path.startswith("/images/") and self.path.endswith("/json"):
            return self._json(200, {"Config": {"Labels": {providers.ORDER_LABEL: LABEL}}})
        return self._json(404, {"message": "no"})

    def do_DELETE(self):  # noqa: N802
        return self._json(204, {})


class _UnixServer(socketserver.ThreadingMixIn, socketserver.UnixStreamServer):
    daemon_threads = True

    def get_request(self):
        req, _ = super().get_request()
        return req, ("local", 0)


@pytest.fixture
def fake_dockerd(tmp_path, monkeypatch):
    sock = str(tmp_path / "docker.sock")
    srv = _UnixServer(sock, _FakeDockerd)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    monkeypatch.setenv("DOCKER_HOST", "unix://" + sock)
    yield sock
    srv.shutdown()
    srv.server_close()


# --- internal/containerizer/cnb/dockerapiprovider_test.go: TestIsBuilderAvailable ---------
# The Go test needs a Docker daemon that can pull cloudfoundry/cnb:cflinuxfs3;
# the fake dockerd above answers the same Engine API calls.

CF_BUILDER = "cloudfoundry/cnb:cflinuxfs3"


def _pulls(builder):
    return [p for p in _FakeDockerd.state.get("pulls", []) if "cloudfoundry%2Fcnb" in p]


def test_is_builder_available_normal_use_case(fake_dockerd):
    _FakeDockerd.state.clear()
    assert providers.DockerAPIProvider().is_builder_available(CF_BUILDER)


def test_is_builder_available_result_from_cache(fake_dockerd):
    _FakeDockerd.state.clear()
    p = providers.DockerAPIProvider()
    assert p.is_builder_available(CF_BUILDER)
    assert sorted(p.available_images) == [CF_BUILDER]
    assert p.is_builder_available(CF_BUILDER)
    assert len(_pulls(CF_BUILDER)) == 1   # the second answer came from the cache


def test_is_builder_available_non_existent_image(fake_dockerd):
    _FakeDockerd.state.clear()
    assert not providers.DockerAPIProvider().is_builder_available("this/doesnotexist:foobar")


def test_docker_api_provider(fake_dockerd, tmp_path):
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    other = tmp_path / "other"
    other.mkdir()
    p = providers.DockerAPIProvider()
    assert p.is_sock_accessible()
    assert p.is_builder_supported(str(app), "gcr.io/buildpacks/builder") is True
    assert p.is_builder_supported(str(other), "gcr.io/buildpacks/builder") is False
    assert p.get_all_buildpacks(["gcr.io/buildpacks/builder"]) == {
        "gcr.io/buildpacks/builder": ["google.nodejs.runtime", "google.go.runtime"]}


def test_podman_provider(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", STUBS + os.pathsep + "/usr/bin:/bin")
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    p = providers.ContainerRuntimeProvider()
    assert p.get_runtime() == "podman"
    assert p.is_builder_supported(str(app), "b") is True
    assert p.is_builder_supported(str(tmp_path), "b") is False
    assert p.get_all_buildpacks(["b"]) == {"b": ["org.cloudfoundry.nodejs", "org.cloudfoundry.go"]}


def test_pack_provider(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", STUBS + os.pathsep + "/usr/bin:/bin")
    monkeypatch.setattr(providers, "DOCKER_SOCK", str(tmp_path / "sock"))
    (tmp_path / "sock").write_text("")
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    p = providers.PackProvider()
    assert p.is_builder_supported(str(app), "b") is True
    assert p.is_builder_supported(str(tmp_path), "b") is False
    assert p.get_all_buildpacks(["b"]) == {"b": ["paketo-buildpacks/nodejs", "paketo-buildpacks/java"]}


def test_chain_falls_through_to_first_working_provider(monkeypatch, tmp_path):
    monkeypatch.delenv("M2K_DISABLE_CNB", raising=False)
    monkeypatch.setenv("DOCKER_HOST", "unix://" + str(tmp_path / "missing.sock"))
    monkeypatch.setenv("PATH", STUBS + os.pathsep + "/usr/bin:/bin")
    providers.reset_providers()
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    try:
        assert providers.is_builder_supported(str(app), "b") is True  # docker API fails -> podman answers
    finally:
        providers.reset_providers()


_SLOW_PODMAN = """#!/bin/sh
case "$*" in
  "run --storage-driver=vfs --rm hello-world") exit 0 ;;
  "--storage-driver=vfs images -q "*) [ "$4" = missing ] || echo 5f1b ;;
  "pull --storage-driver=vfs "*) exit 1 ;;
  "run --rm --storage-driver=vfs -v "*" /cnb/lifecycle/detector")
    src="${5%:/workspace}"
    touch "$LOGDIR/running.$$"
    sleep 0.3
    ls "$LOGDIR" | grep -c '^running' > "$LOGDIR/seen.$$"
    rm -f "$LOGDIR/running.$$"
    [ -f "$src/package.json" ] ;;
  *) exit 1 ;;
esac
"""


def test_batched_probes_run_concurrently_and_match_sequential(monkeypatch, tmp_path):
    """``is_builder_supported_batch`` gives the per-pair answers of the
    sequential chain, with the detector containers running at the same time;
    a builder that cannot be pulled falls through the chain to False."""
    bindir, logdir = tmp_path / "bin", tmp_path / "log"
    bindir.mkdir()
    logdir.mkdir()
    (bindir / "podman").write_text(_SLOW_PODMAN)
    os.chmod(str(bindir / "podman"), 0o755)
    monkeypatch.setenv("PATH", str(bindir) + os.pathsep + "/usr/bin:/bin")
    monkeypatch.setenv("LOGDIR", str(logdir))
    monkeypatch.setenv("M2K_DISABLE_CNB", "0")
    monkeypatch.setattr(providers, "DOCKER_SOCK", str(tmp_path / "nosock"))
    monkeypatch.setattr(providers, "providers", lambda: [providers.ContainerRuntimeProvider()])
    apps = []
    for i in range(3):
        a = tmp_path / ("app%d" % i)
        a.mkdir()
        if i != 1:
            (a / "package.json").write_text("{}")
        apps.append(str(a))
    pairs = [(a, b) for a in apps for b in ("b1", "b2", "missing")]
    got = providers.is_builder_supported_batch(pairs)
    assert got == [True, True, False, False, False, False, True, True, False]
    seen = [int((logdir / f).read_text()) for f in os.listdir(str(logdir)) if f.startswith("seen.")]
    assert len(seen) == 6 and max(seen) >= 2
    assert [providers.is_builder_supported(a, b) for a, b in pairs] == got


def test_batched_probe_errors(monkeypatch):
    """A probe that fails with a chain error (here ValueError) is not taken as
    'supported': it goes on down the chain, ending unsupported; any other
    exception propagates, as from the sequential chain."""
    p = providers.ContainerRuntimeProvider()
    p.runtime = "podman"
    monkeypatch.setattr(providers.ContainerRuntimeProvider, "is_builder_available", lambda self, b: True)
    monkeypatch.setattr(providers, "providers", lambda: [p])

    def bad(cmds, parallel=None, timeout=600):
        return [ValueError("bad mount") for _ in cmds]
    monkeypatch.setattr(providers, "_run_many", bad)
    assert providers.is_builder_supported_batch([("/a", "b1"), ("/b", "b2")]) == [False, False]

    def worse(cmds, parallel=None, timeout=600):
        return [RuntimeError("bug") for _ in cmds]
    monkeypatch.setattr(providers, "_run_many", worse)
    with pytest.raises(RuntimeError):
        providers.is_builder_supported_batch([("/a", "b1")])


def test_docker_api_batched_probes_match_sequential(fake_dockerd, tmp_path):
    """The Docker API provider's batch answers equal its one-at-a-time
    answers (the fake daemon's detector passes where a package.json is)."""
    dirs = []
    for i in range(6):
        d = tmp_path / ("app%d" % i)
        d.mkdir()
        if i % 2 == 0:
            (d / "package.json").write_text("{}")
        dirs.append(str(d))
    pairs = [(d, b) for d in dirs for b in ("gcr.io/buildpacks/builder", "cloudfoundry/cnb:cflinuxfs3")]
    p = providers.DockerAPIProvider()
    assert p.is_builder_supported_batch(pairs) == [p.is_builder_supported(d, b) for d, b in pairs]
    assert p.is_builder_supported_batch(pairs) == [i // 2 % 2 == 0 for i in range(len(pairs))]


# -- runc + skopeo + umoci (runcprovider.go:45-208) ------------------------------

RUNC_STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "stubbin_runc")


@pytest.fixture
def runc_env(monkeypatch, tmp_path):
    log = tmp_path / "stub.log"
    log.write_text("")
    monkeypatch.setenv("M2K_STUB_LOG", str(log))
    monkeypatch.setenv("PATH", RUNC_STUBS + os.pathsep + "/usr/bin:/bin")
    base = tmp_path / "cnb"
    monkeypatch.setattr(providers.RuncProvider, "_paths",
                        staticmethod(lambda: (str(base / "images"), str(base / "bundles"))))
    return log, base


def test_runc_provider_rewrites_bundle_and_parses_detection(runc_env, tmp_path):
    log, base = runc_env
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    other = tmp_path / "other"
    other.mkdir()
    p = providers.RuncProvider()
    assert p.is_available()
    builder = "gcr.io/buildpacks/builder:v1"    # GetImageNameAndTag: image "builder", tag "v1"
    assert p.is_builder_supported(str(app), builder) is True
    assert p.is_builder_supported(str(other), builder) is False   # "No buildpack groups passed detection."
    cfg = json.loads((base / "bundles" / "builder" / "config.json").read_text())
    ws = [m for m in cfg["mounts"] if m["destination"] == "/workspace"]
    assert ws == [{"destination": "/workspace", "type": "bind", "source": str(other), "options": ["rbind", "ro"]}]
    assert [m["destination"] for m in cfg["mounts"]] == ["/proc", "/workspace"]   # replaced in place
    assert cfg["process"]["args"] == ["/cnb/lifecycle/detector"] and cfg["process"]["terminal"] is False
    calls = log.read_text().splitlines()
    copies = [c for c in calls if c.startswith("skopeo copy")]
    assert copies == ["skopeo copy docker://%s oci:builder:v1 @%s" % (builder, base / "images")]
    unpacks = [c for c in calls if c.startswith("umoci")]
    assert unpacks == ["umoci unpack --image builder:v1 %s @%s"
                       % (base / "bundles" / "builder", base / "images")]
    runs = [c for c in calls if c.startswith("runc")]
    assert runs == ["runc run cnbbuilder @%s" % (base / "bundles" / "builder")] * 2


def test_runc_provider_appends_workspace_mount_when_missing(runc_env, tmp_path):
    _log, base = runc_env
    p = providers.RuncProvider()
    p._init(["b:latest"])
    cfgp = base / "bundles" / "b" / "config.json"
    cfg = json.loads(cfgp.read_text())
    cfg["mounts"] = [m for m in cfg["mounts"] if m["destination"] != "/workspace"]
    cfgp.write_text(json.dumps(cfg))
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    assert p.is_builder_supported(str(app), "b:latest") is True
    cfg = json.loads(cfgp.read_text())
    assert cfg["mounts"][-1] == {"destination": "/workspace", "type": "bind", "source": str(app),
                                 "options": ["rbind", "ro"]}


def test_runc_provider_errors_send_the_probe_on(runc_env, tmp_path):
    p = providers.RuncProvider()
    crash = tmp_path / "crash-app"
    crash.mkdir()
    (crash / "crash").write_text("")
    with pytest.raises(providers.ProviderError):       # runc exits non-zero: error, not "unsupported"
        p.is_builder_supported(str(crash), "b:latest")
    with pytest.raises(providers.ProviderError, match="Runc Builder image not available"):
        p.is_builder_supported(str(tmp_path), "missing/image:1")   # skopeo copy failed: no bundle


def test_runc_provider_buildpacks_from_skopeo_label(runc_env):
    p = providers.RuncProvider()
    assert p.get_all_buildpacks(["b:latest", "missing/image:1"]) == {
        "b:latest": ["paketo-buildpacks/nodejs", "paketo-buildpacks/go"]}


def test_runc_provider_unavailable_without_all_three_tools(monkeypatch, tmp_path):
    only = tmp_path / "bin"
    only.mkdir()
    os.symlink(os.path.join(RUNC_STUBS, "runc"), only / "runc")
    monkeypatch.setenv("PATH", str(only))
    p = providers.RuncProvider()
    assert not p.is_available()
    with pytest.raises(providers.ProviderError):
        p.get_all_buildpacks(["b"])


# -- docker API: create without the bind mount, then copy a tar in ------------------
# (dockerapiprovider.go:176-194, 232-340)

class _NoBindDockerd(_FakeDockerd):
    """Refuses bind mounts (a remote daemon, or a rootless one without access to
    the path); the source must arrive through PUT /containers/<id>/archive."""
    archives = {}

    def do_POST(self):  # noqa: N802
        if self.path == "/containers/create":
            n = int(self.headers.get("Content-Length") or 0)
            cfg = json.loads(self.rfile.read(n) or b"{}")
            if (cfg.get("HostConfig") or {}).get("Mounts"):
                return self._json(500, {"message": "invalid mount config: bind source path does not exist"})
            with _FAKE_LOCK:
                cid = "n%d" % next(_FAKE_IDS)
            self.state[cid] = 0 if cfg.get("Image") == "hello-world" else None
            return self._json(201, {"Id": cid})
        if "/wait" in self.path:
            cid = self.path.split("/")[2]
            code = self.state.get(cid)
            if code is None:
                names = self.archives.get(cid, [])
                code = 0 if "workspace/package.json" in names else 1
            return self._json(200, {"StatusCode": code})
        return super().do_POST()

    def do_PUT(self):  # noqa: N802
        import io
        import tarfile
        cid = self.path.split("/")[2]
        assert self.path.endswith("/archive?path=/"), self.path
        assert self.headers.get("Content-Type") == "application/x-tar"
        data = self.rfile.read(int(self.headers.get("Content-Length") or 0))
        with tarfile.open(fileobj=io.BytesIO(data)) as tf:
            self.archives[cid] = [m.name.lstrip("/") for m in tf.getmembers()]
        return self._json(200, {})


@pytest.fixture
def nobind_dockerd(tmp_path, monkeypatch):
    sock = str(tmp_path / "docker.sock")
    srv = _UnixServer(sock, _NoBindDockerd)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    monkeypatch.setenv("DOCKER_HOST", "unix://" + sock)
    yield _NoBindDockerd.archives
    srv.shutdown()
    srv.server_close()


def test_docker_api_copies_source_as_tar_when_bind_mount_fails(nobind_dockerd, tmp_path):
    app = tmp_path / "app"
    (app / "src" / "lib").mkdir(parents=True)
    (app / "package.json").write_text("{}")
    (app / "src" / "lib" / "index.js").write_text("x")
    os.symlink("src/lib/index.js", app / "main.js")
    other = tmp_path / "other"
    other.mkdir()
    (other / "README").write_text("")
    p = providers.DockerAPIProvider()
    assert p.is_builder_supported(str(app), "gcr.io/buildpacks/builder") is True
    assert p.is_builder_supported(str(other), "gcr.io/buildpacks/builder") is False
    copied = [names for names in nobind_dockerd.values() if "workspace/package.json" in names]
    assert copied and set(copied[0]) == {"workspace/package.json", "workspace/src", "workspace/src/lib",
                                         "workspace/src/lib/index.js", "workspace/main.js"}


def test_runtime_probes_start_in_the_background(monkeypatch, tmp_path):
    """start_runtime_prefetch starts `podman run hello-world` and the image
    checks without waiting; the chain later takes their results (same answers
    as probing on demand), and reset_providers reaps probes nobody used."""
    log = tmp_path / "calls"
    wrapper = tmp_path / "bin" / "podman"
    wrapper.parent.mkdir()
    wrapper.write_text('#!/bin/sh\necho "$*" >> %s\nexec %s "$@"\n' % (log, os.path.join(STUBS, "podman")))
    wrapper.chmod(0o755)
    monkeypatch.setenv("PATH", str(wrapper.parent) + os.pathsep + "/usr/bin:/bin")
    monkeypatch.setenv("M2K_DISABLE_CNB", "0")
    monkeypatch.setattr(providers, "DOCKER_SOCK", str(tmp_path / "no-docker.sock"))
    providers.reset_providers()
    providers.start_runtime_prefetch(["b"])
    rt = [p for p in providers.providers() if isinstance(p, providers.ContainerRuntimeProvider)][0]
    assert rt._pending is not None          # started, not collected
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    assert providers.is_builder_supported_batch([(str(app), "b"), (str(tmp_path), "b")]) == [True, False]
    assert rt._pending is None and rt.runtime == "podman"
    calls = log.read_text().splitlines()
    assert calls[0].startswith("run --storage-driver=vfs --rm hello-world") or calls[1].startswith("run ")
    assert sum(c.startswith("--storage-driver=vfs images -q b") for c in calls) == 1   # not probed twice
    # started and never used: reaped by the reset
    providers.start_runtime_prefetch(["c"])
    pids = [c.pid for c in providers.providers()[1]._pending[2] if not isinstance(c, Exception)]
    providers.reset_providers()
    for pid in pids:
        with pytest.raises(ChildProcessError):
            os.waitpid(pid, os.WNOHANG)
    providers.reset_providers()


def test_unused_runtime_probes_are_killed_at_exit(tmp_path):
    """A process that started the podman probes and ended before the planner
    used them kills and reaps them in its atexit handlers (the CLI runs them
    before its os._exit): no probe outlives the command."""
    import subprocess
    import sys
    import time
    podman = tmp_path / "bin" / "podman"
    podman.parent.mkdir()
    pidfile = tmp_path / "pids"
    podman.write_text('#!/bin/sh\necho $$ >> %s\nexec sleep 30\n' % pidfile)
    podman.chmod(0o755)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from move2kube_amd.containerizer.cnb import providers\n"
            "providers.DOCKER_SOCK = %r\n"
            "providers.start_runtime_prefetch(['b1', 'b2'])\n"
            "import time; time.sleep(0.5)\n"
            "from move2kube_amd import _cli_exit\n"
            "_cli_exit(0)\n") % (root, str(tmp_path / "no.sock"))
    env = dict(os.environ, PATH=str(podman.parent) + os.pathsep + "/usr/bin:/bin", M2K_DISABLE_CNB="0")
    t = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], env=env, timeout=60)
    assert r.returncode == 0 and time.monotonic() - t < 20
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 3   # hello-world and two image checks
    for pid in pids:
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


def test_no_background_probes_when_the_docker_socket_exists(monkeypatch, tmp_path):
    sock = tmp_path / "docker.sock"
    sock.write_text("")
    monkeypatch.setattr(providers, "DOCKER_SOCK", str(sock))
    monkeypatch.setenv("M2K_DISABLE_CNB", "0")
    providers.reset_providers()
    providers.start_runtime_prefetch(["b"])
    assert all(getattr(p, "_pending", None) is None for p in providers.providers())
    providers.reset_providers()


def test_error_tuples_tolerate_a_partly_imported_subprocess(monkeypatch):
    """Another thread importing ``subprocess`` leaves a partly initialised
    module in sys.modules for a moment (a collector thread did, and the
    container-types collector failed with "partially initialized module
    'subprocess' has no attribute 'SubprocessError'" once in ~30 runs)."""
    import types
    monkeypatch.setitem(sys.modules, "subprocess", types.ModuleType("subprocess"))
    assert providers._chain_errors() == (providers.ProviderError, OSError, ValueError, KeyError)
    assert providers._start_errors() == (OSError,)


def test_docker_api_run_container_debug_lines(nobind_dockerd, tmp_path, capsys):
    """dockerapiprovider.go:152-225: the bind-mounted create fails, the plain
    one succeeds and the source is copied in, then the container's id, exit
    status and removal."""
    import logparse
    from move2kube_amd.utils import log
    app = tmp_path / "app"
    app.mkdir()
    (app / "package.json").write_text("{}")
    p = providers.DockerAPIProvider()
    log.set_verbose(True)
    try:
        assert p.is_builder_supported(str(app), "gcr.io/buildpacks/builder") is True
    finally:
        log.set_verbose(False)
    msgs = [m for lv, m in logparse.messages(capsys.readouterr().err) if lv == "debug"]
    assert any(m.startswith("Error during container creation : docker API POST /containers/create") for m in msgs)
    (created,) = [m for m in msgs if m.endswith("with image gcr.io/buildpacks/builder with no volumes")]
    cid = created.split()[1]
    assert "Data copied from %s to /workspace in container %s with image gcr.io/buildpacks/builder" % (app, cid) in msgs
    assert "Container %s created with image gcr.io/buildpacks/builder" % cid in msgs
    assert "Container exited with status code: 0" in msgs


def test_docker_api_without_a_daemon(monkeypatch, tmp_path):
    monkeypatch.setenv("DOCKER_HOST", "unix://" + str(tmp_path / "none.sock"))
    p = providers.DockerAPIProvider()
    with pytest.raises(providers.ProviderError, match=r"^Cannot connect to the Docker daemon at unix://.*none\.sock\. "
                                                      r"Is the docker daemon running\?$"):
        p.run_container("hello-world")


def test_runc_provider_log_lines(runc_env, monkeypatch, tmp_path, capsys):
    """runcprovider.go:45-99: the builders' data, a failed inspect, a missing
    order label (logged with the nil error), and the tools looked for."""
    import logparse
    from move2kube_amd.utils import log
    p = providers.RuncProvider()
    log.set_verbose(True)
    try:
        p.get_all_buildpacks(["b:latest", "missing/image:1"])
        monkeypatch.setattr(providers, "_run", lambda cmd, timeout=600: __import__("subprocess").CompletedProcess(
            cmd, 0, b'{"Name": "x", "Labels": {"other": "y"}}'))
        assert p.get_all_buildpacks(["nolabel:1"]) == {}
        monkeypatch.setattr(providers, "_run", lambda cmd, timeout=600: __import__("subprocess").CompletedProcess(
            cmd, 0, b'{"Labels": {"a": 1}}'))
        assert p.get_all_buildpacks(["badlabels:1"]) == {}
        monkeypatch.setenv("PATH", str(tmp_path))
        assert not p.is_available()
    finally:
        log.set_verbose(False)
    err = capsys.readouterr().err
    assert logparse.logged(err, "Getting data of all builders [b:latest missing/image:1]", "debug")
    assert logparse.logged(err, "Error while getting supported buildpacks for builder missing/image:1 : exit status 1",
                           "warning")
    assert logparse.logged(err, "%s missing in builder nolabel:1 : %%!s(<nil>)" % providers.ORDER_LABEL, "warning")
    assert logparse.logged(err, "Unable to seriablize inspect output for builder badlabels:1 : json: cannot unmarshal "
                                "number into Go struct field Output.Labels of type string", "warning")
    assert logparse.logged(err, 'Unable to find runc, ignoring runc based cnb check : exec: "runc": executable file '
                                'not found in $PATH', "debug")
