#!/usr/bin/env python3
"""Canned Kubernetes discovery API for the cluster-collector tests.

``fake_apiserver.py --announce [--tls CERT KEY] [--token T]`` serves
``/api``, ``/apis`` and the group/version documents on 127.0.0.1 (port 0),
prints kubectl proxy's ``Starting to serve on 127.0.0.1:<port>`` line and runs
until killed.  Every request path is appended to ``$M2K_FAKE_API_LOG`` (if
set) so tests can count requests."""

import json
import os
import ssl
import sys
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

GROUPS = [
    ("apps", ["apps/v1"], "apps/v1"),
    ("networking.k8s.io", ["networking.k8s.io/v1", "networking.k8s.io/v1beta1"], "networking.k8s.io/v1"),
    ("extensions", ["extensions/v1beta1"], "extensions/v1beta1"),
    ("route.openshift.io", ["route.openshift.io/v1"], "route.openshift.io/v1"),
]
RESOURCES = {
    "/api/v1": [("pods", "Pod"), ("pods/log", "Pod"), ("services", "Service")],
    "/apis/apps/v1": [("deployments", "Deployment"), ("deployments/scale", "Scale")],
    "/apis/networking.k8s.io/v1": [("ingresses", "Ingress")],
    "/apis/networking.k8s.io/v1beta1": [("ingresses", "Ingress")],
    "/apis/extensions/v1beta1": [("ingresses", "Ingress"), ("deployments", "Deployment")],
    "/apis/route.openshift.io/v1": [("routes", "Route")],
}


def document(path):
    if path == "/api":
        return {"kind": "APIVersions", "versions": ["v1"]}
    if path == "/apis":
        return {"kind": "APIGroupList", "groups": [
            {"name": n, "versions": [{"groupVersion": gv, "version": gv.split("/")[1]} for gv in gvs],
             "preferredVersion": {"groupVersion": pref}} for n, gvs, pref in GROUPS]}
    if path in RESOURCES:
        gv = path.split("/", 2)[2] if path.startswith("/apis/") else "v1"
        return {"kind": "APIResourceList", "groupVersion": gv,
                "resources": [{"name": n, "kind": k, "namespaced": True} for n, k in RESOURCES[path]]}
    return None


def main(argv):
    token = None
    tls = None
    fail = set()
    i = 0
    while i < len(argv):
        if argv[i] == "--token":
            token = argv[i + 1]
            i += 2
        elif argv[i] == "--tls":
            tls = (argv[i + 1], argv[i + 2])
            i += 3
        elif argv[i] == "--fail":
            fail.add(argv[i + 1])
            i += 2
        else:
            i += 1
    log_path = os.environ.get("M2K_FAKE_API_LOG")

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def do_GET(self):
            if log_path:
                with open(log_path, "a") as f:
                    f.write("%s %s\n" % (self.path, self.headers.get("Authorization", "")))
            doc = None
            if token is not None and self.headers.get("Authorization") != "Bearer " + token:
                code, doc = 401, {"kind": "Status", "reason": "Unauthorized"}
            elif self.path in fail:
                code, doc = 503, {"kind": "Status", "reason": "ServiceUnavailable"}
            else:
                doc = document(self.path)
                code = 200 if doc is not None else 404
                doc = doc if doc is not None else {"kind": "Status", "reason": "NotFound"}
            body = json.dumps(doc).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    if tls:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(*tls)
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    sys.stdout.write("Starting to serve on 127.0.0.1:%d\n" % srv.server_address[1])
    sys.stdout.flush()
    srv.serve_forever()


if __name__ == "__main__":
    main(sys.argv[1:])
