"""The discovery transport off the happy path (our stand-in for client-go's
discovery client, reference ``internal/collector/clustercollector.go:178-260``):
kubeconfig merging and context resolution, each credential form, the
configurations handed to the CLI proxy instead, and the HTTP errors a
discovery pass can meet.  Servers are in-process ``http.server`` instances on
127.0.0.1."""

import base64
import json
import os
import shutil
import ssl
import subprocess
import sys
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from move2kube_amd.collector import kubeapi


class _Server:
    """Answers every GET with ``reply(handler) -> (status, body bytes)`` and
    records (path, Authorization)."""

    def __init__(self, reply):
        seen = self.seen = []

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def do_GET(self):
                seen.append((self.path, self.headers.get("Authorization")))
                code, body = reply(self)
                if code is None:       # drop the connection without an answer
                    self.close_connection = True
                    return
                self.send_response(code)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.srv.server_address[1]
        self.t = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.t.start()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


@pytest.fixture
def server():
    made = []

    def make(reply):
        s = _Server(reply)
        made.append(s)
        return s
    yield make
    for s in made:
        s.close()


def _client(port, prefix=""):
    return kubeapi._HTTPClient("http", "127.0.0.1", port, prefix)


def test_get_json_errors(server):
    s = server(lambda h: {"/pre/bad": (500, b"boom " * 100), "/pre/notjson": (200, b"{nope")}.get(h.path, (200, b"[1]")))
    c = _client(s.port, "/pre/")
    try:
        with pytest.raises(kubeapi.DiscoveryError, match=r"^GET /bad: HTTP 500 boom boom"):
            c.get_json("/bad")
        with pytest.raises(kubeapi.DiscoveryError, match="^GET /notjson: invalid JSON: "):
            c.get_json("/notjson")
        assert c.get_json("/ok") == [1]
        assert [p for p, _ in s.seen] == ["/pre/bad", "/pre/notjson", "/pre/ok"]
        assert c.get_many([]) == {}
        got = c.get_many(["/bad", "/ok"])
        assert got["/ok"] == [1] and isinstance(got["/bad"], kubeapi.DiscoveryError)
    finally:
        c.close()


def test_stale_keepalive_is_retried_once(server):
    """A connection the server closed between requests is reopened once; a
    server that drops every request is an error on the second attempt."""
    drops = {"n": 1}

    def reply(h):
        if h.path == "/always-drop" or (h.path == "/drop-once" and drops["n"]):
            if h.path == "/drop-once":
                drops["n"] -= 1
            return None, b""
        return 200, b'{"ok": true}'
    s = server(reply)
    c = _client(s.port)
    try:
        assert c.get_json("/x") == {"ok": True}
        assert c.get_json("/drop-once") == {"ok": True}
        with pytest.raises(kubeapi.DiscoveryError, match="^GET /always-drop: "):
            c.get_json("/always-drop")
    finally:
        c.close()


def test_connection_refused():
    import socket
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    with pytest.raises(kubeapi.DiscoveryError, match="^GET /api: "):
        _client(port).get_json("/api")


def _write(path, doc):
    path.write_text(json.dumps(doc))
    return str(path)


def _kc(path, cluster, user=None, ctx="c", extra=None):
    doc = {"current-context": ctx, "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}],
           "clusters": [{"name": "k", "cluster": cluster}], "users": [{"name": "u", "user": user or {}}]}
    doc.update(extra or {})
    return _write(path, doc)


def test_kubeconfig_merge_first_wins_and_relative_paths(tmp_path):
    (tmp_path / "a").mkdir()
    first = _kc(tmp_path / "a" / "cfg", {"server": "https://one", "certificate-authority": "ca.pem"},
                {"tokenFile": "tok", "client-key": "/abs/key"})
    second = _kc(tmp_path / "second", {"server": "https://two"}, ctx="other",
                 extra={"contexts": [{"name": "other", "context": {"cluster": "k2"}}, "junk", {"name": 3}],
                        "clusters": [{"name": "k", "cluster": {"server": "https://ignored"}},
                                     {"name": "k2", "cluster": "not a map"}]})
    bad_yaml = tmp_path / "bad"
    bad_yaml.write_text("a: [unclosed\n")
    scalar = tmp_path / "scalar"
    scalar.write_text("just a string\n")
    cfg = kubeapi.load_kubeconfig([str(tmp_path / "missing"), str(bad_yaml), str(scalar), first, second])
    assert cfg["current-context"] == "c"
    assert sorted(cfg["contexts"]) == ["c", "other"] and "k2" not in cfg["clusters"]
    assert cfg["clusters"]["k"] == {"server": "https://one", "certificate-authority": str(tmp_path / "a" / "ca.pem")}
    assert cfg["users"]["u"] == {"tokenFile": str(tmp_path / "a" / "tok"), "client-key": "/abs/key"}


def test_kubeconfig_paths_and_no_file(tmp_path, monkeypatch):
    monkeypatch.setenv("KUBECONFIG", os.pathsep.join(["", "/x/one", "/x/two", ""]))
    assert kubeapi.kubeconfig_paths() == ["/x/one", "/x/two"]
    monkeypatch.delenv("KUBECONFIG")
    monkeypatch.setenv("HOME", str(tmp_path))
    assert kubeapi.kubeconfig_paths() == [str(tmp_path / ".kube" / "config")]
    with pytest.raises(kubeapi.UnsupportedConfig, match="no kubeconfig file found"):
        kubeapi.load_kubeconfig()


def test_resolve_context_errors(tmp_path):
    cfg = kubeapi.load_kubeconfig([_kc(tmp_path / "a", {"server": "http://h"}, ctx="nope")])
    with pytest.raises(kubeapi.UnsupportedConfig, match="current context 'nope' not found"):
        kubeapi.resolve_context(cfg)
    cfg["current-context"] = "c"
    cfg["clusters"] = {}
    with pytest.raises(kubeapi.UnsupportedConfig, match="cluster 'k' of context 'c' not found"):
        kubeapi.resolve_context(cfg)


@pytest.mark.parametrize("cluster,user,msg", [
    ({"server": "http://h"}, {"exec": {"command": "x"}}, "uses exec credentials"),
    ({"server": "http://h"}, {"auth-provider": {"name": "gcp"}}, "uses auth-provider credentials"),
    ({"server": "http://h", "proxy-url": "http://proxy:3128"}, {}, "uses proxy-url"),
    ({"server": "unix:///var/run/k8s.sock"}, {}, "unsupported server URL 'unix:///var/run/k8s.sock'"),
    ({}, {}, "unsupported server URL ''"),
    ({"server": "https://h"}, {"tokenFile": "/nonexistent/token"}, "cannot read tokenFile: "),
])
def test_configs_left_to_the_proxy(tmp_path, cluster, user, msg):
    with pytest.raises(kubeapi.UnsupportedConfig, match=msg):
        kubeapi.KubeconfigClient([_kc(tmp_path / "kc", cluster, user)])


def test_token_file_and_basic_auth(tmp_path, server):
    s = server(lambda h: (200, b"{}"))
    url = {"server": "http://127.0.0.1:%d/prefix" % s.port}
    (tmp_path / "tok").write_text("  from-file\n")
    c = kubeapi.KubeconfigClient([_kc(tmp_path / "kc1", url, {"tokenFile": "tok"})])
    assert c.get_json("/api") == {} and (c.host, c.port, c.prefix) == ("127.0.0.1", s.port, "/prefix")
    c.close()
    c = kubeapi.KubeconfigClient([_kc(tmp_path / "kc2", url, {"username": "bob", "password": "pä:ss"})])
    c.get_json("/api")
    c.close()
    c = kubeapi.KubeconfigClient([_kc(tmp_path / "kc3", url, {"token": "inline", "tokenFile": "/ignored"})])
    c.get_json("/api")
    c.close()
    assert s.seen == [("/prefix/api", "Bearer from-file"),
                      ("/prefix/api", "Basic " + base64.b64encode("bob:pä:ss".encode()).decode()),
                      ("/prefix/api", "Bearer inline")]


def test_default_ports(tmp_path):
    c = kubeapi.KubeconfigClient([_kc(tmp_path / "a", {"server": "http://h"})])
    assert (c.scheme, c.port, c.ssl_context) == ("http", 80, None)
    c = kubeapi.KubeconfigClient([_kc(tmp_path / "b", {"server": "https://h", "tls-server-name": "api.internal"})])
    assert (c.scheme, c.port, c.server_hostname) == ("https", 443, "api.internal")
    assert c.ssl_context.verify_mode == ssl.CERT_REQUIRED and c.ssl_context.check_hostname


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    d = tmp_path_factory.mktemp("pki")
    key, crt = str(d / "k.pem"), str(d / "c.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", crt,
                    "-days", "1", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return crt, key


def test_ssl_context_forms(cert):
    crt, key = cert
    insecure = kubeapi.KubeconfigClient._ssl_context({"insecure-skip-tls-verify": True,
                                                      "certificate-authority": "/never/read"}, {})
    assert insecure.verify_mode == ssl.CERT_NONE and not insecure.check_hostname
    from_file = kubeapi.KubeconfigClient._ssl_context({"certificate-authority": crt},
                                                      {"client-certificate": crt, "client-key": key})
    assert len(from_file.get_ca_certs()) == 1
    with pytest.raises(OSError):
        kubeapi.KubeconfigClient._ssl_context({"certificate-authority": crt + ".missing"}, {})
    with pytest.raises(ssl.SSLError):
        kubeapi.KubeconfigClient._ssl_context({}, {"client-certificate-data": base64.b64encode(b"junk").decode(),
                                                   "client-key-data": base64.b64encode(b"junk").decode()})


FAKE_API = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "fake_apiserver.py")


def test_insecure_skip_verify_and_ca_file_against_tls_server(tmp_path, cert):
    crt, key = cert
    p = subprocess.Popen([sys.executable, FAKE_API, "--tls", crt, key], stdout=subprocess.PIPE)
    try:
        port = int(p.stdout.readline().decode().rsplit(":", 1)[1])
        for i, cluster in enumerate(({"insecure-skip-tls-verify": True}, {"certificate-authority": crt})):
            cluster["server"] = "https://127.0.0.1:%d" % port
            c = kubeapi.KubeconfigClient([_kc(tmp_path / ("kc%d" % i), cluster)])
            try:
                assert c.get_json("/api")["versions"] == ["v1"]
            finally:
                c.close()
        c = kubeapi.KubeconfigClient([_kc(tmp_path / "kc-untrusted", {"server": "https://127.0.0.1:%d" % port})])
        with pytest.raises(kubeapi.DiscoveryError, match="CERTIFICATE_VERIFY_FAILED"):
            c.get_json("/api")
        c.close()
    finally:
        p.terminate()
        p.wait(timeout=10)
        p.stdout.close()


def _script(tmp_path, name, body):
    s = tmp_path / name
    s.write_text("#!/bin/sh\n" + body)
    s.chmod(0o755)
    return str(s)


def test_proxy_without_cli_or_announcement(tmp_path, monkeypatch):
    """A proxy that never announces its port is stopped before the error."""
    started = []
    real_popen = subprocess.Popen

    def popen(*a, **kw):
        started.append(real_popen(*a, **kw))
        return started[-1]
    monkeypatch.setattr(kubeapi.subprocess, "Popen", popen)
    with pytest.raises(kubeapi.DiscoveryError, match="no cluster CLI for a proxy"):
        kubeapi.ProxyClient("")
    with pytest.raises(kubeapi.DiscoveryError, match="no cluster CLI for a proxy"):
        kubeapi.ProxyClient(str(tmp_path / "absent"))
    cli = _script(tmp_path, "kubectl", "echo 'error: no configuration has been provided'\nexit 1\n")
    with pytest.raises(kubeapi.DiscoveryError, match=r"proxy did not start: error: no configuration has been provided"):
        kubeapi.ProxyClient(cli)
    silent = _script(tmp_path, "oc", "exec sleep 30\n")
    with pytest.raises(kubeapi.DiscoveryError, match=r"oc proxy did not start: $"):
        kubeapi.ProxyClient(silent, timeout=0.3)
    assert len(started) == 2 and all(p.returncode is not None and p.stdout.closed for p in started)


def test_proxy_that_ignores_sigterm_is_killed(tmp_path, monkeypatch):
    cli = _script(tmp_path, "kubectl", "trap '' TERM\necho 'Starting to serve on 127.0.0.1:1'\n"
                                       "while :; do sleep 0.05; done\n")
    c = kubeapi.ProxyClient(cli)
    assert c.port == 1
    real_wait = c.proc.wait

    def short_wait(timeout=None):
        return real_wait(timeout=0.2 if timeout else None)
    monkeypatch.setattr(c.proc, "wait", short_wait)
    c.close()
    assert c.proc.returncode == -9


def test_open_client_falls_back_to_proxy(tmp_path, monkeypatch):
    monkeypatch.setenv("KUBECONFIG", _kc(tmp_path / "kc", {"server": "http://h", "proxy-url": "http://p"}))
    cli = _script(tmp_path, "kubectl", "echo 'Starting to serve on 127.0.0.1:7'\nexec sleep 30\n")
    c = kubeapi.open_client(cli)
    try:
        assert isinstance(c, kubeapi.ProxyClient) and c.port == 7
    finally:
        c.close()
