"""HTTP REST QA engine - the protocol the move2kube UI drives.

Reference: ``internal/qaengine/httprestengine.go:33-143``.

* ``GET  /problems/current``           -> current problem as JSON; blocks until
  the translator produces one.
* ``POST /problems/current/solution``  -> body is a JSON ``[]string`` answer.

The translator thread publishes the open problem under a condition variable
that GET handlers wait on (every concurrent GET sees the same problem) and
takes the answer off a queue; the reference shares ``currentProblem`` across
handler goroutines unsynchronised and hands each waiting GET its own problem
off a channel.
"""

import json
import queue
import socket
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ..models import qa
from ..utils import fastjson, log
from .engine import Engine

PROBLEMS_URL = "/problems"
CURRENT_PROBLEM_URL = PROBLEMS_URL + "/current"
CURRENT_SOLUTION_URL = CURRENT_PROBLEM_URL + "/solution"


def free_port():
    s = socket.socket()
    s.bind(("", 0))
    port = s.getsockname()[1]
    s.close()
    return port



def _json_kind(v):
    """UnmarshalTypeError's name for a decoded JSON value."""
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    return "array" if isinstance(v, list) else "object"


def _string_slice(v):
    """``json.Unmarshal(body, &sol)`` into a ``[]string``: null is an empty
    answer; another type is Go's UnmarshalTypeError (null elements stay "")."""
    if v is None:
        return None
    if not isinstance(v, list):
        raise ValueError("json: cannot unmarshal %s into Go value of type []string" % _json_kind(v))
    for x in v:
        if x is not None and not isinstance(x, str):
            raise ValueError("json: cannot unmarshal %s into Go value of type string" % _json_kind(x))
    return ["" if x is None else x for x in v]

class HTTPRESTEngine(Engine):
    go_type = "*qaengine.HTTPRESTEngine"
    interactive = True  # may block on a person: the write cache is flushed first

    def __init__(self, port=0, host=""):
        self.port = port
        self.host = host
        self.current = qa.Problem(id=0, resolved=True)
        # guards ``current``; GET handlers wait on it for an open problem, so
        # any number of concurrent GETs see the same problem (the reference
        # hands each waiting handler its own problem off a channel)
        self._cond = threading.Condition()
        self.answers = queue.Queue()
        self.server = None
        self.thread = None

    def go_s(self):
        """``%s`` of ``*HTTPRESTEngine`` (the two channel fields print as
        addresses in the reference; these are placeholders)."""
        chan = "%!s(chan qaengine.Problem=0xc000000000)"
        return "&{%%!s(int=%d) %s %s %s}" % (self.port, self.current.go_s(), chan, chan)

    def start_engine(self):
        if self.port == 0:
            self.port = free_port()
        engine = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, fmt, *args):
                log.debug("qa-http: " + fmt, *args)

            def _send(self, code, body, ctype="application/json"):
                data = body.encode() if isinstance(body, str) else body
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):  # noqa: N802
                if self.path.split("?")[0] != CURRENT_PROBLEM_URL:
                    self._send(404, "404 page not found\n", "text/plain")
                    return
                log.debug("Looking for a problem fron HTTP REST service")  # sic (httprestengine.go:106)
                prob = engine.next_problem()
                log.debug("QA Engine serves problem id: %d, desc: %s", prob.id, prob.desc)
                self._send(200, json.dumps(prob.to_json()) + "\n")

            def do_POST(self):  # noqa: N802
                if self.path.split("?")[0] != CURRENT_SOLUTION_URL:
                    self._send(404, "404 page not found\n", "text/plain")
                    return
                try:
                    n = int(self.headers.get("Content-Length") or 0)
                    body = self.rfile.read(max(0, n))
                    sol = _string_slice(fastjson.loads(body))
                except ValueError as e:
                    errstr = "Error in un-marshalling solution in QA engine: %s" % e
                    self._send(500, errstr + "\n", "text/plain")
                    log.error("%s", errstr)
                    return
                log.debug("QA Engine receives solution: %s", "[" + " ".join(sol or []) + "]")
                err = engine.submit_solution(sol or [])
                if err:
                    errstr = "Unsuitable answer : %s" % err
                    self._send(500, errstr + "\n", "text/plain")
                    log.error("%s", errstr)
                else:
                    self._send(200, "")

        try:
            self.server = ThreadingHTTPServer((self.host, self.port), Handler)
        except OSError as e:
            raise RuntimeError("Unable to listen on port %d : %s" % (self.port, e))
        self.server.daemon_threads = True
        self.thread = threading.Thread(target=self.server.serve_forever, name="m2k-qa-http", daemon=True)
        self.thread.start()
        log.info("Started QA engine on: localhost:%d", self.port)

    def stop(self):
        if self.server is not None:
            self.server.shutdown()
            self.server.server_close()

    # called from HTTP handler threads
    def next_problem(self, timeout=None):
        """The open problem; blocks until the translator asks one."""
        with self._cond:
            self._cond.wait_for(lambda: self.current.id != 0 and not self.current.resolved, timeout)
            return self.current.copy()

    def submit_solution(self, sol):
        with self._cond:
            if self.current.id == 0 or self.current.resolved:
                return "no open problem"
            p = self.current.copy()
            try:
                p.set_answer(sol)
            except qa.ProblemError as e:
                return str(e)
            self.current = p
        self.answers.put(p.copy())
        return None

    # called from the translator thread
    def fetch_answer(self, prob):
        if prob.id == 0:
            prob.resolved = True
        if not prob.resolved:
            log.debug("Passing problem to HTTP REST QA Engine ID: %d, desc: %s", prob.id, prob.desc)
            with self._cond:
                self.current = prob.copy()
                self._cond.notify_all()
            prob = self.answers.get()
            if not prob.resolved:
                raise qa.ProblemError("Unable to resolve question %s" % prob.desc)
        return prob
