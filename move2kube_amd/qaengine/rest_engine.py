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

import queue
import socket
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import unquote

from ..models import qa
from ..utils import fastjson, log
from ..utils.constants import settings
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


class _PartialSlice(ValueError):
    """UnmarshalTypeError; ``partial`` is what Unmarshal still stored."""

    def __init__(self, msg, partial):
        ValueError.__init__(self, msg)
        self.partial = partial


def _string_slice(v):
    """``json.Unmarshal(body, &sol)`` into a ``[]string``: null is an empty
    answer; another type is Go's UnmarshalTypeError for the first mismatch,
    and Unmarshal still fills the slice, mismatched and null elements as ""."""
    if v is None:
        return None
    if not isinstance(v, list):
        raise _PartialSlice("json: cannot unmarshal %s into Go value of type []string" % _json_kind(v), None)
    out = ["" if not isinstance(x, str) else x for x in v]
    for x in v:
        if x is not None and not isinstance(x, str):
            raise _PartialSlice("json: cannot unmarshal %s into Go value of type string" % _json_kind(x), out)
    return out


_ROUTES = {CURRENT_PROBLEM_URL: "GET", CURRENT_SOLUTION_URL: "POST"}
_STATUS_TEXT = {200: "OK", 301: "Moved Permanently", 404: "Not Found", 405: "Method Not Allowed",
                500: "Internal Server Error"}


def _clean_path(p):
    """net/http's ``cleanPath``: ``path.Clean`` of the rooted path, keeping a
    trailing slash."""
    if p == "":
        return "/"
    if p[0] != "/":
        p = "/" + p
    parts = []
    for seg in p.split("/"):
        if seg in ("", "."):
            continue
        if seg == "..":
            if parts:
                parts.pop()
            continue
        parts.append(seg)
    np = "/" + "/".join(parts)
    if p.endswith("/") and np != "/":
        np += "/"
    return np


def _html_escape(s):
    """``htmlEscape`` of net/http (``htmlReplacer``)."""
    return (s.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")
            .replace('"', "&#34;").replace("'", "&#39;"))


MAX_POST_HANDLER_READ_BYTES = 256 << 10   # net/http server.go: maxPostHandlerReadBytes
_ERROR_HEADERS = "\r\nContent-Type: text/plain; charset=utf-8\r\nConnection: close\r\n\r\n"


class _BadBody(Exception):
    """A request body net/http cannot read (corrupt chunked encoding, EOF)."""


def _parse_content_length(values):
    """net/http transfer.go fixLength / parseContentLength: the length, or
    None when Go answers 400 (differing duplicates, not a non-negative int)."""
    first = values[0].strip(" \t")
    if any(v.strip(" \t") != first for v in values[1:]):
        return None
    if first == "":
        return 0
    digits = first[1:] if first[:1] in "+-" else first
    if not digits.isdigit() or not digits.isascii():
        return None
    n = int(first)
    return n if 0 <= n < 1 << 63 else None

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
            protocol_version = "HTTP/1.1"  # keep-alive like net/http

            def log_message(self, fmt, *args):
                log.debug("qa-http: " + fmt, *args)

            # -- the request body, as net/http reads and discards it ------------
            def _body_setup(self):
                """transfer.go readTransfer: chunked (one Transfer-Encoding,
                "chunked", HTTP/1.1 only) or a Content-Length; False after
                answering a request net/http refuses before any handler runs."""
                self._chunked = False
                self._remaining = 0
                self._body_done = False
                te = self.headers.get_all("Transfer-Encoding") or []
                if te and self.request_version != "HTTP/1.0":
                    if len(te) != 1 or te[0].strip(" \t").lower() != "chunked":
                        self._refuse("501 Not Implemented", "Unsupported transfer encoding")
                        return False
                    self._chunked = True
                    return True
                cls = self.headers.get_all("Content-Length") or []
                if cls:
                    n = _parse_content_length(cls)
                    if n is None:
                        self._refuse("400 Bad Request", "400 Bad Request")
                        return False
                    self._remaining = n
                self._body_done = self._remaining == 0
                return True

            def _refuse(self, status, body):
                """server.go: the reply to a request readRequest rejected."""
                self.close_connection = True
                self.wfile.write(("HTTP/1.1 " + status + _ERROR_HEADERS + body).encode("latin-1"))
                self.wfile.flush()

            def _read_chunk_line(self):
                line = self.rfile.readline(4097)
                if not line.endswith(b"\n"):
                    raise _BadBody("unexpected EOF" if not line else "header line too long")
                return line.rstrip(b"\r\n")

            def _read_body(self, limit=None):
                """The body's bytes (at most ``limit``+1 of them when a limit
                is given); raises _BadBody when it cannot be read."""
                out = bytearray()
                if not self._chunked:
                    n = self._remaining if limit is None else min(self._remaining, limit + 1)
                    data = self.rfile.read(n) if n else b""
                    self._remaining -= len(data)
                    if len(data) < n:
                        raise _BadBody("unexpected EOF")
                    self._body_done = self._remaining == 0
                    return bytes(data)
                while True:
                    if limit is not None and len(out) > limit:
                        return bytes(out)
                    size_line = self._read_chunk_line().split(b";", 1)[0].strip()
                    try:
                        size = int(size_line, 16)
                    except ValueError:
                        raise _BadBody("invalid byte in chunk length")
                    if size == 0:
                        while self._read_chunk_line():
                            pass   # trailers
                        self._body_done = True
                        return bytes(out)
                    chunk = self.rfile.read(size)
                    if len(chunk) < size or self.rfile.read(2) != b"\r\n":
                        raise _BadBody("malformed chunked encoding")
                    out += chunk

            def _discard_body(self):
                """server.go chunkWriter.writeHeader: an unread body is read
                and thrown away (up to maxPostHandlerReadBytes) so the
                connection can be reused; a bigger or unreadable one closes it."""
                if self._body_done:
                    return
                if not self._chunked and self._remaining >= MAX_POST_HANDLER_READ_BYTES:
                    self.close_connection = True
                    return
                try:
                    self._read_body(MAX_POST_HANDLER_READ_BYTES)
                except (_BadBody, OSError):
                    self.close_connection = True
                    return
                if not self._body_done:
                    self.close_connection = True

            def _go_reply(self, code, body=b"", headers=()):
                """A response laid out as net/http's chunkWriter writes it:
                the handler's own headers sorted by name, then Date,
                Content-Length, a sniffed Content-Type (only for a non-empty
                body without one) and Connection."""
                self._discard_body()
                http11 = self.request_version != "HTTP/1.0"
                lines = ["%s %d %s\r\n" % ("HTTP/1.1" if http11 else "HTTP/1.0", code, _STATUS_TEXT[code])]
                for k, v in sorted(headers):
                    lines.append("%s: %s\r\n" % (k, v))
                lines.append("Date: %s\r\n" % self.date_time_string())
                if self.command != "HEAD" or body:
                    lines.append("Content-Length: %d\r\n" % len(body))
                if body and not any(k == "Content-Type" for k, _ in headers):
                    lines.append("Content-Type: text/plain; charset=utf-8\r\n")
                if self.close_connection and http11:
                    lines.append("Connection: close\r\n")
                elif not self.close_connection and not http11:
                    lines.append("Connection: keep-alive\r\n")
                lines.append("\r\n")
                self.wfile.write("".join(lines).encode("latin-1") + (b"" if self.command == "HEAD" else body))
                self.wfile.flush()

            def _go_error(self, code, msgs):
                """``http.Error`` (once per message: a second call only
                appends its line, net/http ignores the superfluous header)."""
                self._go_reply(code, "".join(m + "\n" for m in msgs).encode("utf-8"),
                               [("Content-Type", "text/plain; charset=utf-8"), ("X-Content-Type-Options", "nosniff")])

            def _dispatch(self):
                """http.DefaultServeMux (clean-path redirect) in front of the
                gorilla/mux router: a known path with another method is 405
                with an empty body, an unknown path 404."""
                if not self._body_setup():
                    return
                raw_path, _, query = self.path.partition("?")
                path = unquote(raw_path)
                clean = _clean_path(path)
                if clean != path and self.command != "CONNECT":
                    url = clean + ("?" + query if query else "")
                    hdrs = [("Location", url)]
                    body = b""
                    if self.command in ("GET", "HEAD"):
                        hdrs.append(("Content-Type", "text/html; charset=utf-8"))
                        if self.command == "GET":
                            body = ('<a href="%s">Moved Permanently</a>.\n\n' % _html_escape(url)).encode("utf-8")
                    self._go_reply(301, body, hdrs)
                    return
                route = _ROUTES.get(path)
                if route is None:
                    self._go_error(404, ["404 page not found"])
                elif route != self.command:
                    self._go_reply(405)
                elif route == "GET":
                    self._problem()
                else:
                    self._solution()

            do_GET = do_POST = do_PUT = do_DELETE = do_PATCH = do_OPTIONS = do_HEAD = _dispatch

            def _problem(self):
                log.debug("Looking for a problem fron HTTP REST service")  # sic (httprestengine.go:106)
                prob = engine.next_problem()
                log.debug("QA Engine serves problem id: %d, desc: %s", prob.id, prob.desc)
                self._go_reply(200, fastjson.go_encode(prob.to_json()))

            def _solution(self):
                errs = []
                try:
                    body = self._read_body()   # ioutil.ReadAll(r.Body)
                except (_BadBody, OSError) as e:
                    self.close_connection = True
                    body = b""
                    log.debug("qa-http: reading the request body: %s", e)
                try:
                    sol = _string_slice(fastjson.loads(body))
                except _PartialSlice as e:
                    errs.append("Error in un-marshalling solution in QA engine: %s" % e)
                    log.error("%s", errs[-1])
                    sol = e.partial
                except ValueError as e:
                    errs.append("Error in un-marshalling solution in QA engine: %s" % e)
                    log.error("%s", errs[-1])
                    sol = None
                if errs and settings.fixed:
                    self._go_error(500, errs)
                    return
                # the reference goes on with what Unmarshal left in the slice
                # (httprestengine.go:127-140: no return after http.Error)
                log.debug("QA Engine receives solution: %s", "[" + " ".join(sol or []) + "]")
                err = engine.submit_solution(sol or [])
                if err:
                    errs.append("Unsuitable answer : %s" % err)
                    log.error("%s", errs[-1])
                if errs:
                    self._go_error(500, errs)
                else:
                    self._go_reply(200)

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
        """``h.currentProblem.SetAnswer(sol)``: applied to the open problem
        itself, so a rejected answer leaves what SetAnswer already changed
        (a select's answer becomes ``[]``) for the next GET to show.  With no
        open problem the reference's handler blocks forever on the answer
        channel; here it is an error."""
        with self._cond:
            if self.current.id == 0 or self.current.resolved:
                return "no open problem"
            try:
                self.current.set_answer(sol)
            except qa.ProblemError as e:
                return str(e)
            p = self.current.copy()
        self.answers.put(p)
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
