"""Cloud Native Buildpack detection providers (reference ``internal/containerizer/cnb/``).

Fallback chain ``[docker Engine API, podman, pack, runc+skopeo+umoci]``: the
first provider that does not error decides whether a builder image supports
a source directory (``/cnb/lifecycle/detector`` exit status).  Buildpack lists
come from the builder image label ``io.buildpacks.buildpack.order``.

Every provider degrades gracefully when its runtime is absent (the common case
on build hosts and on this framework's CI), and availability probes are cached
per process so that a missing runtime costs one probe, not one per directory.
"""

import io
import os
import shutil
import sys
import threading

from ...utils import common, fastjson, gojson, log, proc
from ...utils.constants import settings
from ...utils.lazyre import LazyModule
from ...utils.lazyre import lazy as _lazy_re

subprocess = LazyModule("subprocess")

ORDER_LABEL = "io.buildpacks.buildpack.order"
# bounds for external tools (the reference waits forever; a hung pull or
# detector must not hang `plan`)
PULL_TIMEOUT_S = 1800
RUN_TIMEOUT_S = 600
DOCKER_SOCK = "/var/run/docker.sock"
# detector containers started at once (each is a builder image with its own
# memory footprint; the reference runs one at a time)
CONTAINER_PARALLEL = int(os.environ.get("M2K_CNB_PARALLEL", "4") or 4)

_lock = threading.Lock()


# cnb.order (provider.go:33-48): buildpackRef embeds buildpackInfo
_ORDER = ("slice", "cnb.order", ("struct", "cnb.orderEntry", (
    ("group", ("slice", "[]cnb.buildpackRef", ("struct", "cnb.buildpackRef", (
        ("id", gojson.STRING), ("version", gojson.STRING), ("homepage", gojson.STRING),
        ("optional", gojson.BOOL))))),)))


def get_builders_from_label(label):
    """``getBuildersFromLabel``: the buildpack ids of the builder's order
    label, decoded into ``cnb.order`` as json.Unmarshal does."""
    try:
        order = gojson.unmarshal(label, _ORDER)
    except ValueError as e:
        log.warning("Unable to read order : %s", e)
        return []
    log.debug("Builder data :%s", label)
    out = []
    for og in order or []:
        for bp in (og or {}).get("group") or []:
            out.append((bp or {}).get("id", ""))
    return out


_PACK_GROUP_RE = _lazy_re(r"(?s)Group\s#\d+:[\r\n\s]+[^\s]+")


class ProviderError(RuntimeError):
    pass


# ---------------------------------------------------------------------------
# Docker Engine API over the unix socket
# ---------------------------------------------------------------------------

_unix_conn_cls = None


def _UnixHTTPConnection(path, timeout=60):
    """http.client connection over a unix socket.  The class is built on first
    use: http.client (with its email parser) costs ~20 ms of CLI start-up that
    runs without a docker daemon never need."""
    global _unix_conn_cls
    if _unix_conn_cls is None:
        import http.client

        class UnixHTTPConnection(http.client.HTTPConnection):
            def __init__(self, path, timeout=60):
                super().__init__("localhost", timeout=timeout)
                self._path = path

            def connect(self):
                import socket
                s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                s.settimeout(self.timeout)
                s.connect(self._path)
                self.sock = s
        _unix_conn_cls = UnixHTTPConnection
    return _unix_conn_cls(path, timeout=timeout)


class DockerAPIProvider:
    """Talks to dockerd through ``DOCKER_HOST`` (unix socket) like docker's Go client."""

    def __init__(self):
        self.sock_state = None  # None unknown / True / False
        self.available_images = set()
        host = os.environ.get("DOCKER_HOST", "unix://" + DOCKER_SOCK)
        self.sock_path = host[len("unix://"):] if host.startswith("unix://") else None

    def _request(self, method, path, body=None, headers=None, timeout=600, raw=False):
        if not self.sock_path or not os.path.exists(self.sock_path):
            # docker/client's errConnectionFailed
            raise ProviderError("Cannot connect to the Docker daemon at unix://%s. Is the docker daemon running?"
                                % (self.sock_path or DOCKER_SOCK))
        conn = _UnixHTTPConnection(self.sock_path, timeout=timeout)
        try:
            hdrs = dict(headers or {})
            if body is not None and not isinstance(body, (bytes, bytearray)) and not hasattr(body, "read"):
                import json
                body = json.dumps(body).encode()
                hdrs.setdefault("Content-Type", "application/json")
            conn.request(method, path, body=body, headers=hdrs)
            resp = conn.getresponse()
            data = resp.read()
        except OSError as e:
            raise ProviderError(str(e))
        finally:
            conn.close()
        if resp.status >= 400:
            raise ProviderError("docker API %s %s: %d %s" % (method, path, resp.status, data[:200]))
        if raw:
            return data
        return fastjson.loads(data) if data else None

    def pull_image(self, image):
        name, tag = (image.rsplit(":", 1) + ["latest"])[:2] if ":" in image.rsplit("/", 1)[-1] else (image, "latest")
        import urllib.parse
        self._request("POST", "/images/create?" + urllib.parse.urlencode({"fromImage": name, "tag": tag}), raw=True)

    def inspect_image(self, image):
        import urllib.parse
        return self._request("GET", "/images/%s/json" % urllib.parse.quote(image, safe=""))

    def _copy_dir(self, cid, src, dst):
        buf = io.BytesIO()
        import tarfile
        with tarfile.open(fileobj=buf, mode="w") as tw:
            for root, dirs, files in os.walk(src):
                dirs.sort()
                for name in sorted(dirs) + sorted(files):
                    full = os.path.join(root, name)
                    rel = os.path.relpath(full, src)
                    try:
                        tw.add(full, arcname=os.path.join(dst.lstrip("/"), rel), recursive=False)
                    except OSError:
                        continue
        self._request("PUT", "/containers/%s/archive?path=/" % cid, body=buf.getvalue(),
                      headers={"Content-Type": "application/x-tar"}, raw=True)

    def run_container(self, image, cmd="", volsrc="", voldest=""):
        cfg = {"Image": image}
        if cmd:
            cfg["Cmd"] = [cmd]
        host = {}
        if volsrc and voldest:
            host["Mounts"] = [{"Type": "bind", "Source": volsrc, "Target": voldest, "ReadOnly": True}]
        # the debug lines of runContainer (dockerapiprovider.go:152-225)
        try:
            resp = self._request("POST", "/containers/create", body=dict(cfg, HostConfig=host))
        except ProviderError as e:
            log.debug("Error during container creation : %s", e)
            try:
                resp = self._request("POST", "/containers/create", body=cfg)
            except ProviderError:
                log.debug("Container creation failed with image %s with no volumes", image)
                raise
            log.debug("Container %s created with image %s with no volumes", resp["Id"], image)
            if volsrc and voldest:
                try:
                    self._copy_dir(resp["Id"], volsrc, voldest)
                except ProviderError as e:
                    log.debug("Container data copy failed for image %s with volume %s:%s : %s", image, volsrc,
                              voldest, e)
                    self._remove(resp["Id"])
                    raise
                log.debug("Data copied from %s to %s in container %s with image %s", volsrc, voldest, resp["Id"],
                          image)
        cid = resp["Id"]
        log.debug("Container %s created with image %s", cid, image)
        try:
            try:
                self._request("POST", "/containers/%s/start" % cid, raw=True)
            except ProviderError as e:
                log.debug("Error during container startup of container %s : %s", cid, e)
                raise
            try:
                st = self._request("POST", "/containers/%s/wait?condition=not-running" % cid)
            except ProviderError as e:
                log.debug("Error during waiting for container : %s", e)
                raise
            code = (st or {}).get("StatusCode", 0)
            log.debug("Container exited with status code: %d", code)
            try:
                logs = self._request("GET", "/containers/%s/logs?stdout=1" % cid, raw=True).decode("utf-8", "replace")
            except ProviderError as e:
                log.debug("Error while getting container logs : %s", e)
                raise
            if code != 0:
                raise ProviderError("Container execution terminated with error code : %d" % code)
            return logs
        finally:
            self._remove(cid)

    def _remove(self, cid):
        try:
            self._request("DELETE", "/containers/%s?force=1" % cid, raw=True)
        except ProviderError:
            pass

    def is_sock_accessible(self):
        if self.sock_state is None:
            try:
                self.pull_image("hello-world")
                self.run_container("hello-world")
                self.sock_state = True
            except (ProviderError, KeyError, ValueError):
                self.sock_state = False
        return self.sock_state

    def is_builder_available(self, builder):
        if not self.is_sock_accessible():
            return False
        if builder in self.available_images:
            return True
        try:
            self.pull_image(builder)
        except ProviderError as e:
            log.warning("Error while pulling builder %s : %s", builder, e)
            return False
        self.available_images.add(builder)
        return True

    def is_builder_supported(self, path, builder):
        if not self.is_builder_available(builder):
            raise ProviderError("Builder image not available : %s" % builder)
        try:
            out = self.run_container(builder, "/cnb/lifecycle/detector", os.path.abspath(path), "/workspace")
            log.debug(out)
            return True
        except ProviderError as e:
            log.debug("Detect failed %s : %s", builder, e)
            return False

    def is_builder_supported_batch(self, pairs):
        """[(path, builder)] -> [True/False, or None where this provider cannot
        answer]: builder images are settled once each, then the detector
        containers run up to ``CONTAINER_PARALLEL`` at a time on the daemon
        (the reference creates, runs and removes one container per probe, in
        sequence)."""
        out = [None] * len(pairs)
        runnable = [i for i, (_, builder) in enumerate(pairs) if self.is_builder_available(builder)]

        def probe(i):
            path, builder = pairs[i]
            try:
                log.debug(self.run_container(builder, "/cnb/lifecycle/detector", os.path.abspath(path), "/workspace"))
                return True
            except ProviderError as e:
                log.debug("Detect failed %s : %s", builder, e)
                return False
        results = parallel_map(probe, runnable, min(settings.workers, CONTAINER_PARALLEL))
        for i, r in zip(runnable, results):
            if isinstance(r, Exception):
                if not isinstance(r, _chain_errors()):
                    raise r
                r = None
            out[i] = r
        return out

    def get_all_buildpacks(self, builders):
        if not self.is_sock_accessible():
            raise ProviderError("Container runtime not supported in this instance")
        out = {}
        for b in builders:
            try:
                info = self.inspect_image(b)
            except ProviderError as e:
                log.debug("Unable to inspect image %s : %s", b, e)
                continue
            labels = ((info or {}).get("Config") or {}).get("Labels") or {}
            out[b] = get_builders_from_label(labels.get(ORDER_LABEL, ""))
        return out


# ---------------------------------------------------------------------------
# podman CLI
# ---------------------------------------------------------------------------

def _subprocess_errors(name):
    """``subprocess.<name>`` once that module is loaded, else nothing: until
    then no such error can have been raised (the tools run through
    ``utils.proc``, which loads it only to raise a timeout), and naming it in
    an ``except`` would import it into a cold CLI process."""
    # another thread may be importing it right now: a partly initialised
    # module lacks the name, and nothing it has not defined can be raised yet
    err = getattr(sys.modules.get("subprocess"), name, None)
    return (err,) if err is not None else ()


def _chain_errors():
    """Errors that send a probe on to the next provider of the chain."""
    return (ProviderError, OSError, ValueError, KeyError) + _subprocess_errors("SubprocessError")


def _start_errors():
    """A tool that could not start or overran its time limit."""
    return (OSError,) + _subprocess_errors("TimeoutExpired")


def parallel_map(fn, items, workers=None):
    """[fn(x) for x in items] on up to ``workers`` threads (child processes
    run concurrently; the GIL is free while they are waited for).  An
    exception from fn is returned in its slot, not raised."""
    items = list(items)
    if workers is None:
        workers = settings.workers
    out = [None] * len(items)
    if len(items) <= 1 or workers <= 1:
        for k, x in enumerate(items):
            try:
                out[k] = fn(x)
            except Exception as e:  # noqa: BLE001
                out[k] = e
        return out
    it = iter(range(len(items)))
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                k = next(it, None)
            if k is None:
                return
            try:
                out[k] = fn(items[k])
            except Exception as e:  # noqa: BLE001
                out[k] = e
    threads = [threading.Thread(target=worker, daemon=True) for _ in range(min(workers, len(items)))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    return out


def _run(cmd, timeout=600):
    return common.run_tool(cmd, stdout=proc.PIPE, stderr=proc.STDOUT, timeout=timeout)


def _run_many(cmds, parallel=None, timeout=RUN_TIMEOUT_S):
    """:func:`_run` of every command, up to ``parallel`` at once; an error is
    returned in its slot."""
    return common.run_tools(cmds, parallel=parallel, stdout=proc.PIPE, stderr=proc.STDOUT, timeout=timeout)


def _collect(children, timeout):
    """Results of started children (or their start errors), in order."""
    out = []
    for c in children:
        if isinstance(c, BaseException):
            out.append(c)
            continue
        r = c.wait(timeout)
        out.append(proc._timeout_error(r, timeout) if r.timed_out else r)
    return out


def _go_err(proc_or_exc, argv0):
    """The Go error text of a finished command or of its failed start."""
    if isinstance(proc_or_exc, BaseException):
        if isinstance(proc_or_exc, OSError):
            return str(common.go_exec_error(proc_or_exc, argv0))
        return str(proc_or_exc)
    return common.go_exit_status(proc_or_exc.returncode)


def _out(p):
    return p.stdout.decode("utf-8", "replace") if isinstance(getattr(p, "stdout", None), bytes) else ""


class ContainerRuntimeProvider:
    """``containerRuntimeProvider`` (containerruntimeprovider.go): podman with
    the vfs storage driver."""

    HELLO = ["podman", "run", "--storage-driver=vfs", "--rm", "hello-world"]

    def __init__(self):
        self.runtime = None  # "podman" | "none"
        self.available = set()
        self._hello = None   # prefetched runtime probe (a result or its exception)
        self._images = {}    # builder -> prefetched `images -q` (a result or its exception)
        self._pending = None  # probes started by start_prefetch, not collected yet

    @staticmethod
    def _images_cmd(rt, builder):
        return [rt, "--storage-driver=vfs", "images", "-q", builder]

    @staticmethod
    def _images_run(rt, builder):
        return proc.run(ContainerRuntimeProvider._images_cmd(rt, builder), stdout=proc.PIPE, stderr=proc.DEVNULL,
                        timeout=600)

    def prefetch(self, builders):
        """Start the runtime probe and the local-image checks of ``builders``
        at once.  The reference runs them one after another
        (containerruntimeprovider.go:45-95); both are read-only, so their
        results are taken in that order later by :meth:`get_runtime` and
        :meth:`is_builder_available`, with the same logs and decisions.  The
        image checks of a runtime that then fails its probe are discarded."""
        self.start_prefetch(builders)
        self._finish_prefetch()

    def start_prefetch(self, builders):
        """:meth:`prefetch` without waiting: the probes run while the caller
        goes on (the planner starts them before it walks the tree)."""
        self._finish_prefetch()
        if self.runtime == "none":
            return
        todo = [b for b in dict.fromkeys(builders) if b not in self.available and b not in self._images]
        hello = self.runtime is None and self._hello is None
        if not todo and not hello:
            return
        children = []
        for b in ([None] if hello else []) + todo:
            try:
                if b is None:
                    children.append(proc.spawn(self.HELLO, stdout=proc.PIPE, stderr=proc.STDOUT))
                else:
                    children.append(proc.spawn(self._images_cmd("podman", b), stdout=proc.PIPE, stderr=proc.DEVNULL))
            except OSError as e:
                children.append(e)
        self._pending = (hello, todo, children)
        _register_prefetch_reaper()

    def abandon_prefetch(self):
        """Kill and reap probes started by :meth:`start_prefetch` that nobody
        collected (the command ended before the planner needed them)."""
        pending, self._pending = self._pending, None
        if pending is None:
            return
        import signal
        for c in pending[2]:
            if isinstance(c, BaseException):
                continue
            try:
                os.kill(c.pid, signal.SIGKILL)
            except OSError:
                pass
            c.wait()

    def _finish_prefetch(self):
        pending, self._pending = self._pending, None
        if pending is None:
            return
        hello, todo, children = pending
        res = _collect(children, 600)
        if hello:
            self._hello = (res.pop(0),)
        for b, r in zip(todo, res):
            self._images[b] = r

    def get_runtime(self):
        self._finish_prefetch()
        if self.runtime is None:
            try:
                if self._hello is not None:
                    p, self._hello = self._hello[0], None
                    if isinstance(p, BaseException):
                        raise p
                else:
                    p = _run(self.HELLO)
            except _start_errors() as e:
                log.debug("Podman not supported : %s : %s", _go_err(e, "podman"), "")
                self.runtime = "none"
            else:
                if p.returncode == 0:
                    self.runtime = "podman"
                else:
                    log.debug("Podman not supported : %s : %s", _go_err(p, "podman"), _out(p))
                    self.runtime = "none"
        return self.runtime if self.runtime != "none" else None

    def is_builder_available(self, builder):
        rt = self.get_runtime()
        if rt is None:
            return False
        if builder in self.available:
            return True
        self._finish_prefetch()
        log.debug("Checking if the image %s exists locally", builder)
        try:
            p = self._images.pop(builder, None)
            if p is None:
                p = self._images_run(rt, builder)
            elif isinstance(p, BaseException):
                raise p
        except _start_errors() as e:
            log.warning("Error while checking if the builder %s exists locally. Error: %r Output: %r", builder,
                        _go_err(e, rt), "")
            return False
        if p.returncode != 0:
            log.warning("Error while checking if the builder %s exists locally. Error: %r Output: %r", builder,
                        _go_err(p, rt), _out(p))
            return False
        if p.stdout:
            self.available.add(builder)
            return True
        log.debug("Pulling image %s", builder)
        try:
            p = _run([rt, "pull", "--storage-driver=vfs", builder])
        except _start_errors() as e:
            log.warning("Error while pulling builder %s : %s : %s", builder, _go_err(e, rt), "")
            return False
        if p.returncode != 0:
            log.warning("Error while pulling builder %s : %s : %s", builder, _go_err(p, rt), _out(p))
            return False
        self.available.add(builder)
        return True

    def _detect_cmd(self, path, builder):
        try:
            p = common.go_abs(path)
        except OSError as e:
            # filepath.Abs fails only when the working directory is gone;
            # the reference warns and mounts "" (containerruntimeprovider.go:113-116)
            log.warning("Unable to resolve to absolute path : getwd: %s", (e.strerror or str(e)).lower())
            p = ""
        return [self.runtime, "run", "--rm", "--storage-driver=vfs", "-v", p + ":/workspace",
                builder, "/cnb/lifecycle/detector"]

    def _detect_result(self, builder, p):
        if p.returncode != 0:
            log.debug("Detect failed %s : %s : %s", builder, _go_err(p, self.runtime), _out(p))
            return False
        return True

    def is_builder_supported(self, path, builder):
        if not self.is_builder_available(builder):
            raise ProviderError("Builder image not available : %s" % builder)
        log.debug("Running detect on image %s", builder)
        return self._detect_result(builder, _run(self._detect_cmd(path, builder)))

    def is_builder_supported_batch(self, pairs):
        """[(path, builder)] -> [True/False, or None where this provider cannot
        answer].  Builder availability is settled once per builder (it may
        pull); the detector containers then run concurrently - the reference
        runs one at a time, each a container start.  The log lines come out in
        the order of the pairs."""
        out = [None] * len(pairs)
        runnable = []
        self.prefetch([b for _, b in pairs])
        for i, (path, builder) in enumerate(pairs):
            if self.is_builder_available(builder):
                runnable.append(i)
        for i in runnable:
            log.debug("Running detect on image %s", pairs[i][1])
        results = _run_many([self._detect_cmd(*pairs[i]) for i in runnable],
                            min(settings.workers, CONTAINER_PARALLEL))
        for i, r in zip(runnable, results):
            if isinstance(r, Exception):
                if not isinstance(r, _chain_errors()):
                    raise r
                r = None  # this pair goes on down the chain, as in is_builder_supported
            else:
                r = self._detect_result(pairs[i][1], r)
            out[i] = r
        return out

    @staticmethod
    def _inspect_cmd(rt, builder):
        return [rt, "inspect", "--storage-driver=vfs", "--format", '{{ index .Config.Labels "' + ORDER_LABEL + '"}}',
                builder]

    def get_all_buildpacks(self, builders):
        procs = None
        self._finish_prefetch()
        if self.runtime is None and self._hello is None and builders:
            # the runtime probe and the (read-only) inspects start together;
            # the inspects of a runtime that then fails its probe are discarded
            children = []
            for cmd in [self.HELLO] + [self._inspect_cmd("podman", b) for b in builders]:
                try:
                    children.append(proc.spawn(cmd, stdout=proc.PIPE, stderr=proc.STDOUT))
                except OSError as e:
                    children.append(e)
            res = _collect(children, RUN_TIMEOUT_S)
            self._hello = (res[0],)
            procs = res[1:]
        rt = self.get_runtime()
        if rt is None:
            raise ProviderError("Container runtime not supported in this instance")
        out = {}
        log.debug("Getting data of all builders %s", "[" + " ".join(builders) + "]")
        for b in builders:
            log.debug("Inspecting image %s", b)
        if procs is None:  # one `inspect` per builder, concurrently
            procs = _run_many([self._inspect_cmd(rt, b) for b in builders])
        else:
            procs = [common.go_exec_error(p, rt) if isinstance(p, FileNotFoundError) else p for p in procs]
        for b, p in zip(builders, procs):
            if isinstance(p, Exception):
                raise p
            if p.returncode != 0:
                log.debug("Unable to inspect image %s : %s, %s", b, _go_err(p, rt), _out(p))
                continue
            out[b] = get_builders_from_label(p.stdout.decode("utf-8", "replace"))
        return out


# ---------------------------------------------------------------------------
# pack CLI
# ---------------------------------------------------------------------------

class PackProvider:
    def is_available(self):
        if shutil.which("pack") is None:
            log.debug("Unable to find pack : %s", 'exec: "pack": executable file not found in $PATH')
            return False
        if not os.path.exists(DOCKER_SOCK):
            log.debug("Unable to find pack docker socket, ignoring CNB based containerization approach : %s",
                      "stat %s: no such file or directory" % DOCKER_SOCK)
            return False
        return True

    def is_builder_supported(self, path, builder):
        if not self.is_available():
            raise ProviderError("Pack not supported in this instance")
        child = subprocess.Popen(["pack", "build", "m2ktestcflinuxf2selector:1", "-B", builder, "-p", path],
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL)
        try:
            for raw in child.stdout:
                t = raw.decode("utf-8", "replace").rstrip("\r\n")
                if t.strip() == "":
                    continue
                log.debug("%s", t)
                if "===> ANALYZING" in t:
                    log.debug("Found compatible cnb for %s", path)
                    child.kill()
                    return True
                if "No buildpack groups passed detection." in t:
                    log.debug("No compatible cnb for %s", path)
                    child.kill()
                    return False
        finally:
            try:
                child.kill()
            except OSError:
                pass
            child.wait()
        raise ProviderError("Error while using pack")

    def get_all_buildpacks(self, builders):
        out = {}
        rx = _PACK_GROUP_RE
        for b in builders:
            try:
                p = _run(["pack", "inspect-builder", b])
            except _start_errors() as e:
                log.warning("Error while getting supported buildpacks for builder %s : %s", b, e)
                continue
            if p.returncode != 0:  # cmd.Output() returns an *ExitError (packprovider.go:131-136)
                log.warning("Error while getting supported buildpacks for builder %s : %s", b,
                            common.go_exit_status(p.returncode))
                continue
            for m in rx.findall(p.stdout.decode("utf-8", "replace")):
                out.setdefault(b, []).append(m.split()[-1])
        return out


# ---------------------------------------------------------------------------
# runc + skopeo + umoci
# ---------------------------------------------------------------------------

# skopeo's inspect.Output (Created is a *time.Time, decoded by its own
# UnmarshalJSON: not checked here)
_SKOPEO_INSPECT = ("struct", "inspect.Output", (
    ("Name", gojson.STRING), ("Tag", gojson.STRING), ("Digest", gojson.STRING),
    ("RepoTags", ("slice", "[]string", gojson.STRING)), ("DockerVersion", gojson.STRING),
    ("Labels", ("map", "map[string]string", gojson.STRING)), ("Architecture", gojson.STRING),
    ("Os", gojson.STRING), ("Layers", ("slice", "[]string", gojson.STRING)),
    ("Env", ("slice", "[]string", gojson.STRING))))


class RuncProvider:
    @staticmethod
    def _paths():
        # resolved at call time (the reference captured AssetsPath at package init -
        # SURVEY 2.13 #11); a writable scratch dir, the asset tree is used read-only
        from ... import assets
        base = os.path.join(assets.scratch_dir(), "cnb")
        return os.path.join(base, "images"), os.path.join(base, "bundles")

    def is_available(self):
        for tool in ("runc", "skopeo", "umoci"):
            if shutil.which(tool) is None:
                log.debug("Unable to find %s, ignoring runc based cnb check : %s", tool,
                          'exec: "%s": executable file not found in $PATH' % tool)
                return False
        return True

    def _init(self, builders):
        images, bundles = self._paths()
        os.makedirs(images, exist_ok=True)
        os.makedirs(bundles, exist_ok=True)
        for b in builders:
            image, tag = common.get_image_name_and_tag(b)
            if os.path.exists(os.path.join(images, image)):
                continue
            p = subprocess.run(["skopeo", "copy", "docker://" + b, "oci:" + image + ":" + tag], cwd=images,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                               timeout=PULL_TIMEOUT_S)
            if p.returncode != 0:
                continue
            subprocess.run(["umoci", "unpack", "--image", image + ":" + tag, os.path.abspath(os.path.join(bundles, image))],
                           cwd=images, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                           timeout=RUN_TIMEOUT_S)

    def is_builder_supported(self, path, builder):
        if not self.is_available():
            raise ProviderError("Runc Builder image not available : %s" % builder)
        self._init([builder])
        _, bundles = self._paths()
        image, _ = common.get_image_name_and_tag(builder)
        cfg_path = os.path.join(bundles, image, "config.json")
        if not os.path.exists(os.path.dirname(cfg_path)):
            log.debug("Unable to find pack builder oci bundle, ignoring builder : %s",
                      "stat %s: no such file or directory" % os.path.dirname(cfg_path))
            raise ProviderError("Runc Builder image not available : %s" % builder)
        spec = common.read_json(cfg_path)
        mount = {"destination": "/workspace", "type": "bind", "source": os.path.abspath(path), "options": ["rbind", "ro"]}
        mounts = spec.get("mounts") or []
        for i, m in enumerate(mounts):
            if m.get("destination") == "/workspace":
                mounts[i] = mount
                break
        else:
            mounts.append(mount)
        spec["mounts"] = mounts
        spec.setdefault("process", {})["args"] = ["/cnb/lifecycle/detector"]
        spec["process"]["terminal"] = False
        common.write_json(cfg_path, spec)
        p = subprocess.run(["runc", "run", "cnbbuilder"], cwd=os.path.dirname(cfg_path),
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                           timeout=RUN_TIMEOUT_S)
        if p.returncode != 0:
            raise ProviderError("Error while executing runc")
        return b"ERROR: No buildpack groups passed detection." not in p.stdout

    def get_all_buildpacks(self, builders):
        if not self.is_available():
            raise ProviderError("Runc not supported in this instance")
        out = {}
        log.debug("Getting data of all builders %s", "[" + " ".join(builders) + "]")
        for b in builders:
            p = _run(["skopeo", "inspect", "docker://" + b])     # CombinedOutput
            log.debug("Builder %s data :%s", b, p.stdout.decode("utf-8", "replace"))
            if p.returncode != 0:
                log.warning("Error while getting supported buildpacks for builder %s : %s", b,
                            common.go_exit_status(p.returncode))
                continue
            try:
                labels = (gojson.unmarshal(p.stdout, _SKOPEO_INSPECT) or {}).get("Labels") or {}
            except ValueError as e:
                log.warning("Unable to seriablize inspect output for builder %s : %s", b, e)
                continue
            if ORDER_LABEL not in labels:
                log.warning("%s missing in builder %s : %s", ORDER_LABEL, b, "%!s(<nil>)")
                continue
            out[b] = get_builders_from_label(labels[ORDER_LABEL])
        return out


_providers = None
_providers_switch = None


def providers():
    """Provider chain dockerAPI -> podman/docker CLI -> pack -> runc.  ``M2K_DISABLE_CNB=1``
    empties it (deterministic offline runs: benches, golden tests); the chain
    is rebuilt when the switch changes within a process."""
    global _providers, _providers_switch
    switch = os.environ.get("M2K_DISABLE_CNB", "") not in ("", "0")
    with _lock:
        if _providers is None or _providers_switch != switch:
            _providers_switch = switch
            _providers = [] if switch else [DockerAPIProvider(), ContainerRuntimeProvider(), PackProvider(), RuncProvider()]
        return _providers


def reset_providers():
    global _providers
    with _lock:
        old, _providers = _providers, None
    for p in old or ():
        if isinstance(p, ContainerRuntimeProvider):
            p._finish_prefetch()  # reap probes nobody asked for


_reaper_registered = []


def _register_prefetch_reaper():
    """At interpreter exit (the CLI runs the atexit handlers before its
    ``os._exit``), kill the prefetch probes still running: the reference
    starts none of them unless the planner reaches the provider."""
    if _reaper_registered:
        return
    _reaper_registered.append(True)
    import atexit
    atexit.register(_reap_prefetch)


def _reap_prefetch():
    for p in _providers or ():
        if isinstance(p, ContainerRuntimeProvider):
            p.abandon_prefetch()


def start_runtime_prefetch(builders):
    """Start the container runtime's probes for ``builders`` in the
    background, when that provider is the one the chain will reach (no Docker
    socket: the Docker Engine API provider comes first)."""
    if os.path.exists(DOCKER_SOCK):
        return
    for p in providers():
        if isinstance(p, ContainerRuntimeProvider):
            p.start_prefetch(builders)
            return


def _log_not_supported():
    from . import log_not_supported
    log_not_supported()


def _log_long_wait():
    from . import log_long_wait
    log_long_wait()


def is_builder_supported(path, builder):
    _log_long_wait()
    for p in providers():
        try:
            return p.is_builder_supported(path, builder)
        except _chain_errors() as e:
            log.debug("CNB provider %s: %s", type(p).__name__, e)
            continue
    _log_not_supported()
    return False


def is_builder_supported_batch(pairs):
    """``[is_builder_supported(path, builder) for path, builder in pairs]``:
    each pair goes down the provider chain until a provider answers; a
    provider with a batch method answers its pairs concurrently."""
    _log_long_wait()
    results = [False] * len(pairs)
    todo = list(range(len(pairs)))
    for p in providers():
        if not todo:
            break
        batch = getattr(p, "is_builder_supported_batch", None)
        if batch is not None:
            try:
                got = batch([pairs[i] for i in todo])
            except _chain_errors() as e:
                log.debug("CNB provider %s: %s", type(p).__name__, e)
                continue
            rest = []
            for i, r in zip(todo, got):
                if r is None:
                    rest.append(i)
                else:
                    results[i] = r
            todo = rest
            continue
        rest = []
        for i in todo:
            try:
                results[i] = p.is_builder_supported(*pairs[i])
            except _chain_errors() as e:
                log.debug("CNB provider %s: %s", type(p).__name__, e)
                rest.append(i)
        todo = rest
    if todo:
        _log_not_supported()
    return results


def get_all_buildpacks(builders):
    for p in providers():
        try:
            bps = p.get_all_buildpacks(builders)
        except _chain_errors() as e:
            log.debug("CNB provider %s: %s", type(p).__name__, e)
            continue
        if bps:
            return bps
    _log_not_supported()
    return {}
