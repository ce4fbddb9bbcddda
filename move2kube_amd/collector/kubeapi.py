"""Kubernetes discovery without a process per request.

The reference builds a client-go discovery client from the default kubeconfig
loading rules and calls ``ServerGroups`` / ``ServerGroupsAndResources``
(``internal/collector/clustercollector.go:178-260``): one in-process pass
over ``/api``, ``/apis`` and every group/version document.  This module does
the same with the standard library:

* :class:`KubeconfigClient` reads the kubeconfig (``$KUBECONFIG`` list, merged
  first-wins as client-go does, else ``~/.kube/config``), picks the current
  context and talks HTTP(S) to the API server itself: bearer token / token
  file, basic auth, client certificate + key (inline ``*-data`` or files),
  cluster CA (inline or file), ``insecure-skip-tls-verify``,
  ``tls-server-name``.  Zero processes are spawned.
* :class:`ProxyClient` covers what it cannot (``exec`` / ``auth-provider``
  credential plugins, ``proxy-url``, in-cluster configs): one
  ``kubectl proxy --port=0`` process authenticates every request; it is
  stopped when discovery ends.

Group/version documents are fetched concurrently on a small thread pool
(client-go's ``ServerGroupsAndResources`` also fetches them in parallel).
"""

import base64
import concurrent.futures
import http.client
import json
import os
import re
import select
import shutil
import ssl
import subprocess
import tempfile
import threading
import time
import urllib.parse

from ..utils import common, log, yamlio

DISCOVERY_TIMEOUT = 32.0  # client-go's default discovery timeout
MAX_PARALLEL = 8


class DiscoveryError(RuntimeError):
    pass


class UnsupportedConfig(DiscoveryError):
    """The kubeconfig needs something only the cluster CLI can do."""


class NoKubeconfig(UnsupportedConfig):
    """No kubeconfig file exists."""


class ClientConfigError(DiscoveryError):
    """client-go's ``ClientConfig()`` error: no configuration at all."""


# clientcmd ErrEmptyConfig inside errConfigurationInvalid (client-go v0.19)
EMPTY_CONFIG = ("invalid configuration: no configuration has been provided, try setting KUBERNETES_MASTER "
                "environment variable")
IN_CLUSTER_TOKEN = "/var/run/secrets/kubernetes.io/serviceaccount/token"


def in_cluster_possible():
    """``inClusterClientConfig.Possible``: the service env vars and a token file."""
    return (os.environ.get("KUBERNETES_SERVICE_HOST", "") != "" and os.environ.get("KUBERNETES_SERVICE_PORT", "") != ""
            and os.path.isfile(IN_CLUSTER_TOKEN))


# ---------------------------------------------------------------------------
# kubeconfig loading (client-go NewDefaultClientConfigLoadingRules)
# ---------------------------------------------------------------------------

def kubeconfig_paths():
    env = os.environ.get("KUBECONFIG", "")
    if env:
        return [p for p in env.split(os.pathsep) if p]
    return [os.path.join(os.path.expanduser("~"), ".kube", "config")]


def _named(items, key):
    out = {}
    for it in items or []:
        if isinstance(it, dict) and isinstance(it.get("name"), str) and it["name"] not in out:
            out[it["name"]] = (it.get(key) or {})
    return out


def load_kubeconfig(paths=None):
    """Merge the kubeconfig files: the first file that sets a value wins.
    Returns {"current-context", "contexts", "clusters", "users"}; relative file
    references are made absolute against the file that declared them."""
    merged = {"current-context": "", "contexts": {}, "clusters": {}, "users": {}}
    found = False
    for path in paths or kubeconfig_paths():
        try:
            with open(path) as f:
                doc = yamlio.load(f.read()) or {}
        except (OSError, yamlio.YAMLError):
            continue
        if not isinstance(doc, dict):
            continue
        found = True
        base = os.path.dirname(os.path.abspath(path))
        if not merged["current-context"] and isinstance(doc.get("current-context"), str):
            merged["current-context"] = doc["current-context"]
        for section, key in (("contexts", "context"), ("clusters", "cluster"), ("users", "user")):
            for name, val in _named(doc.get(section), key).items():
                if name in merged[section] or not isinstance(val, dict):
                    continue
                val = dict(val)
                for fk in ("certificate-authority", "client-certificate", "client-key", "tokenFile"):
                    if isinstance(val.get(fk), str) and val[fk] and not os.path.isabs(val[fk]):
                        val[fk] = os.path.join(base, val[fk])
                merged[section][name] = val
    if not found:
        raise NoKubeconfig("no kubeconfig file found (%s)" % os.pathsep.join(paths or kubeconfig_paths()))
    return merged


def resolve_context(cfg):
    name = cfg.get("current-context") or ""
    ctx = cfg["contexts"].get(name)
    if ctx is None:
        raise UnsupportedConfig("current context %r not found in kubeconfig" % name)
    cluster = cfg["clusters"].get(ctx.get("cluster", ""))
    if cluster is None:
        raise UnsupportedConfig("cluster %r of context %r not found" % (ctx.get("cluster"), name))
    user = cfg["users"].get(ctx.get("user", ""), {})
    return cluster, user


# ---------------------------------------------------------------------------
# clients
# ---------------------------------------------------------------------------

class _HTTPSConnection(http.client.HTTPSConnection):
    """HTTPS with SNI / certificate check against ``tls-server-name`` when set."""

    def __init__(self, host, port, server_hostname, **kw):
        super().__init__(host, port, **kw)
        self._sni = server_hostname or host

    def connect(self):
        http.client.HTTPConnection.connect(self)
        self.sock = self._context.wrap_socket(self.sock, server_hostname=self._sni)


class _HTTPClient:
    """GET JSON documents from one API server; one keep-alive connection per thread."""

    def __init__(self, scheme, host, port, prefix="", headers=None, ssl_context=None, server_hostname=None):
        self.scheme, self.host, self.port = scheme, host, port
        self.prefix = prefix.rstrip("/")
        self.headers = dict(headers or {})
        self.headers.setdefault("Accept", "application/json")
        self.headers.setdefault("User-Agent", "move2kube/collect")
        self.ssl_context = ssl_context
        self.server_hostname = server_hostname
        self._local = threading.local()
        self._all = []
        self._lock = threading.Lock()

    def _conn(self):
        c = getattr(self._local, "conn", None)
        if c is None:
            if self.scheme == "https":
                c = _HTTPSConnection(self.host, self.port, self.server_hostname, timeout=DISCOVERY_TIMEOUT,
                                     context=self.ssl_context)
            else:
                c = http.client.HTTPConnection(self.host, self.port, timeout=DISCOVERY_TIMEOUT)
            self._local.conn = c
            with self._lock:
                self._all.append(c)
        return c

    def get_json(self, path):
        for attempt in (0, 1):
            c = self._conn()
            try:
                c.request("GET", self.prefix + path, headers=self.headers)
                r = c.getresponse()
                body = r.read()
            except (OSError, http.client.HTTPException) as e:
                c.close()
                self._local.conn = None
                if attempt == 0 and isinstance(e, (http.client.RemoteDisconnected, ConnectionResetError,
                                                   BrokenPipeError)):
                    continue  # stale keep-alive connection
                raise DiscoveryError("GET %s: %s" % (path, e))
            if r.status != 200:
                raise DiscoveryError("GET %s: HTTP %d %s" % (path, r.status, body[:200].decode("utf-8", "replace")))
            try:
                return json.loads(body)
            except ValueError as e:
                raise DiscoveryError("GET %s: invalid JSON: %s" % (path, e))
        raise DiscoveryError("GET %s: connection failed" % path)

    def get_many(self, paths):
        """{path: document or DiscoveryError}, fetched concurrently."""
        out = {}
        if not paths:
            return out
        with concurrent.futures.ThreadPoolExecutor(max_workers=min(MAX_PARALLEL, len(paths))) as ex:
            futs = {ex.submit(self.get_json, p): p for p in paths}
            for f in concurrent.futures.as_completed(futs):
                p = futs[f]
                try:
                    out[p] = f.result()
                except DiscoveryError as e:
                    out[p] = e
        return out

    def close(self):
        with self._lock:
            conns, self._all = self._all, []
        for c in conns:
            c.close()


class KubeconfigClient(_HTTPClient):
    """Direct client for the kubeconfig's current context."""

    def __init__(self, paths=None):
        cluster, user = resolve_context(load_kubeconfig(paths))
        for unsupported in ("exec", "auth-provider"):
            if user.get(unsupported):
                raise UnsupportedConfig("kubeconfig user uses %s credentials" % unsupported)
        if cluster.get("proxy-url"):
            raise UnsupportedConfig("kubeconfig cluster uses proxy-url")
        server = cluster.get("server") or ""
        u = urllib.parse.urlsplit(server)
        if u.scheme not in ("http", "https") or not u.hostname:
            raise UnsupportedConfig("unsupported server URL %r" % server)
        headers = {}
        token = user.get("token") or ""
        if not token and user.get("tokenFile"):
            try:
                with open(user["tokenFile"]) as f:
                    token = f.read().strip()
            except OSError as e:
                raise UnsupportedConfig("cannot read tokenFile: %s" % e)
        if token:
            headers["Authorization"] = "Bearer " + token
        elif user.get("username") or user.get("password"):
            cred = "%s:%s" % (user.get("username", ""), user.get("password", ""))
            headers["Authorization"] = "Basic " + base64.b64encode(common.go_bytes(cred)).decode()
        ctx = None
        if u.scheme == "https":
            ctx = self._ssl_context(cluster, user)
        port = u.port or (443 if u.scheme == "https" else 80)
        super().__init__(u.scheme, u.hostname, port, u.path, headers, ctx, cluster.get("tls-server-name") or None)

    @staticmethod
    def _ssl_context(cluster, user):
        # client-go trusts only the cluster CA when one is given (tls.Config
        # RootCAs), the system roots otherwise
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
        if cluster.get("insecure-skip-tls-verify"):
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        elif cluster.get("certificate-authority-data"):
            ctx.load_verify_locations(cadata=base64.b64decode(cluster["certificate-authority-data"]).decode("utf-8", "replace"))
        elif cluster.get("certificate-authority"):
            ctx.load_verify_locations(cafile=cluster["certificate-authority"])
        else:
            ctx.load_default_certs()
        cert, key = user.get("client-certificate-data"), user.get("client-key-data")
        if cert and key:
            with tempfile.TemporaryDirectory(prefix="m2k-kc-") as d:
                cp, kp = os.path.join(d, "c.pem"), os.path.join(d, "k.pem")
                for p, data in ((cp, cert), (kp, key)):
                    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
                    with os.fdopen(fd, "wb") as f:
                        f.write(base64.b64decode(data))
                ctx.load_cert_chain(cp, kp)
        elif user.get("client-certificate") and user.get("client-key"):
            ctx.load_cert_chain(user["client-certificate"], user["client-key"])
        return ctx


class ProxyClient(_HTTPClient):
    """``<kubectl|oc> proxy --port=0``: one process authenticates every request."""

    _ANNOUNCE = re.compile(rb"Starting to serve on ([0-9.]+|\[[0-9a-fA-F:]+\]|localhost):(\d+)")

    def __init__(self, cmd, timeout=20.0):
        if not cmd or shutil.which(cmd) is None:
            raise DiscoveryError("no cluster CLI for a proxy")
        self.proc = subprocess.Popen([cmd, "proxy", "--port=0", "--address=127.0.0.1", "--accept-hosts=^127\\.0\\.0\\.1$"],
                                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL)
        buf, deadline = b"", time.monotonic() + timeout
        port = None
        while time.monotonic() < deadline:
            r, _, _ = select.select([self.proc.stdout], [], [], max(0.0, deadline - time.monotonic()))
            if not r:
                break
            chunk = os.read(self.proc.stdout.fileno(), 4096)
            if not chunk:
                break
            buf += chunk
            m = self._ANNOUNCE.search(buf)
            if m:
                port = int(m.group(2))
                break
        if port is None:
            self.close()
            raise DiscoveryError("%s proxy did not start: %s" % (cmd, buf[-300:].decode("utf-8", "replace")))
        super().__init__("http", "127.0.0.1", port)

    def close(self):
        if hasattr(self, "_lock"):      # not yet set when the proxy failed to start
            super().close()
        p = getattr(self, "proc", None)
        if p is not None and p.poll() is None:
            p.terminate()
            try:
                p.wait(timeout=5)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if p is not None and p.stdout is not None:
            p.stdout.close()


def open_client(cluster_cmd):
    """Direct kubeconfig client, else a proxy through the cluster CLI.  With
    no kubeconfig at all and no in-cluster service account, client-go's
    ``ClientConfig()`` fails and so does this (ClientConfigError)."""
    try:
        return KubeconfigClient()
    except NoKubeconfig as e:
        if not in_cluster_possible():
            raise ClientConfigError(EMPTY_CONFIG) from None
        log.debug("Direct discovery not possible (%s); using %s proxy", e, cluster_cmd)
    except (UnsupportedConfig, ssl.SSLError, OSError, ValueError) as e:
        log.debug("Direct discovery not possible (%s); using %s proxy", e, cluster_cmd)
    return ProxyClient(cluster_cmd)
