"""Interactive engines: the HTTP REST protocol the UI uses and the terminal engine."""

import io

import pytest
import json
import re
import socket
import threading
import urllib.error
import urllib.request

from move2kube_amd import qaengine
from move2kube_amd.models import qa
from move2kube_amd.qaengine.cli_engine import CliEngine
from move2kube_amd.qaengine.rest_engine import HTTPRESTEngine


def _get(port, path):
    with urllib.request.urlopen("http://127.0.0.1:%d%s" % (port, path), timeout=20) as r:
        return r.status, r.read().decode()


def _post(port, path, body):
    req = urllib.request.Request("http://127.0.0.1:%d%s" % (port, path), data=body.encode(), method="POST")
    try:
        with urllib.request.urlopen(req, timeout=20) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


def test_rest_engine_round_trip():
    e = HTTPRESTEngine(0, "127.0.0.1")
    qaengine.reset()
    qaengine.add_engine(e)
    results = {}

    def ask():
        p = qa.new_select_problem("Pick one", ["ctx"], "a", ["a", "b", "c"])
        results["ans"] = qaengine.fetch_answer(p).get_string_answer()

    t = threading.Thread(target=ask)
    t.start()
    try:
        code, body = _get(e.port, "/problems/current")
        assert code == 200
        prob = json.loads(body)
        assert prob["description"] == "Pick one" and prob["solution"]["options"] == ["a", "b", "c"]
        code, body = _post(e.port, "/problems/current/solution", '["zzz"]')
        assert code == 500  # not an option; the problem stays current
        code, body = _get(e.port, "/problems/current")
        assert json.loads(body)["description"] == "Pick one"
        code, _ = _post(e.port, "/problems/current/solution", '["b"]')
        assert code == 200
        t.join(20)
        assert results["ans"] == "b"
        try:
            _get(e.port, "/nope")
            raise AssertionError("expected 404")
        except urllib.error.HTTPError as err:
            assert err.code == 404
    finally:
        e.stop()


def test_rest_engine_concurrent_gets_and_bad_requests():
    """GETs that wait at the same time all receive the same open problem, and
    two problems asked in a row are served in order; malformed solution
    bodies get a 500 without disturbing the open problem."""
    e = HTTPRESTEngine(0, "127.0.0.1")
    qaengine.reset()
    qaengine.add_engine(e)
    answers = []

    def ask():
        for desc in ("first", "second"):
            p = qa.new_input_problem(desc, [], "d")
            answers.append(qaengine.fetch_answer(p).get_string_answer())

    seen = []

    def get():
        seen.append(json.loads(_get(e.port, "/problems/current")[1])["description"])

    getters = [threading.Thread(target=get) for _ in range(4)]
    for g in getters:
        g.start()
    t = threading.Thread(target=ask)
    t.start()
    try:
        for g in getters:
            g.join(20)
        assert seen == ["first"] * 4
        # json.Unmarshal(body, &sol []string) errors, http.Error text; the
        # handler does not return after it (httprestengine.go:127-140), so
        # SetAnswer runs on what Unmarshal left and adds its own error line
        pre = "Error in un-marshalling solution in QA engine: "
        assert _post(e.port, "/problems/current/solution", "{not json") == \
            (500, pre + "invalid character 'n' looking for beginning of object key string\n"
             "Unsuitable answer : The answer slice is empty\n")
        assert _post(e.port, "/problems/current/solution", '[1, 2]') == \
            (500, pre + "json: cannot unmarshal number into Go value of type string\n"
             "Unsuitable answer : The question type is not multiselect, but there are multiple answers\n")
        assert _post(e.port, "/problems/current/solution", '{"a": "b"}') == \
            (500, pre + "json: cannot unmarshal object into Go value of type []string\n"
             "Unsuitable answer : The answer slice is empty\n")
        assert _post(e.port, "/problems/current/solution", '["one"]')[0] == 200
        assert json.loads(_get(e.port, "/problems/current")[1])["description"] == "second"
        assert _post(e.port, "/problems/current/solution", '["two"]')[0] == 200
        t.join(20)
        assert answers == ["one", "two"]
    finally:
        e.stop()


def _raw(port, request):
    """One request on a fresh socket; the response bytes with the Date value
    blanked (Content-Length framing, the connection stays open)."""
    import re
    import socket
    with socket.create_connection(("127.0.0.1", port), timeout=20) as c:
        c.sendall(request)
        data = b""
        while b"\r\n\r\n" not in data:
            data += c.recv(65536)
        head, _, body = data.partition(b"\r\n\r\n")
        m = re.search(rb"Content-Length: (\d+)", head)
        n = int(m.group(1)) if m else 0
        while len(body) < n:
            body += c.recv(65536)
    return re.sub(rb"Date: [^\r]+", b"Date: X", head) + b"\r\n\r\n" + body


def test_rest_engine_wire_bytes_follow_net_http():
    """What ``json.NewEncoder(w).Encode`` and net/http put on the wire
    (httprestengine.go:67-69,113): compact JSON, raw UTF-8, ``<``/``>``/``&``
    as ``\\u003c``/``\\u003e``/``\\u0026``, a trailing newline, a sniffed
    ``text/plain`` type after Date and Content-Length; gorilla/mux answers a
    known path with the wrong method 405 with an empty body, an unknown path
    ``http.Error``'s 404; DefaultServeMux redirects an unclean path."""
    e = HTTPRESTEngine(0, "127.0.0.1")
    qaengine.reset()
    qaengine.add_engine(e)
    got = {}

    def ask():
        p = qa.new_select_problem("Expose <svc> & café?", ["a\tb"], "é", ["é", "<none>"])
        got["ans"] = qaengine.fetch_answer(p).get_string_answer()

    t = threading.Thread(target=ask, daemon=True)
    t.start()
    try:
        body = ('{"id":%d,"description":"Expose \\u003csvc\\u003e \\u0026 café?","context":["a\\tb"],'
                '"solution":{"type":"Select","default":["é"],"options":["é","\\u003cnone\\u003e"],"answer":[]}}\n')
        resp = _raw(e.port, b"GET /problems/current HTTP/1.1\r\nHost: x\r\n\r\n")
        pid = json.loads(resp.partition(b"\r\n\r\n")[2])["id"]
        want = body % pid
        assert resp == (b"HTTP/1.1 200 OK\r\nDate: X\r\nContent-Length: %d\r\n"
                        b"Content-Type: text/plain; charset=utf-8\r\n\r\n" % len(want.encode()) + want.encode())
        assert _raw(e.port, b"POST /problems/current HTTP/1.1\r\nHost: x\r\nContent-Length: 0\r\n\r\n") == \
            b"HTTP/1.1 405 Method Not Allowed\r\nDate: X\r\nContent-Length: 0\r\n\r\n"
        assert _raw(e.port, b"GET /problems/current/solution HTTP/1.1\r\nHost: x\r\n\r\n") == \
            b"HTTP/1.1 405 Method Not Allowed\r\nDate: X\r\nContent-Length: 0\r\n\r\n"
        assert _raw(e.port, b"GET /nope HTTP/1.1\r\nHost: x\r\n\r\n") == (
            b"HTTP/1.1 404 Not Found\r\nContent-Type: text/plain; charset=utf-8\r\n"
            b"X-Content-Type-Options: nosniff\r\nDate: X\r\nContent-Length: 19\r\n\r\n404 page not found\n")
        assert _raw(e.port, b"GET /problems//current?a=1 HTTP/1.1\r\nHost: x\r\n\r\n") == (
            b"HTTP/1.1 301 Moved Permanently\r\nContent-Type: text/html; charset=utf-8\r\n"
            b"Location: /problems/current?a=1\r\nDate: X\r\nContent-Length: 56\r\n\r\n"
            b'<a href="/problems/current?a=1">Moved Permanently</a>.\n\n')
        # a rejected option, then an accepted one
        sol = b'["<x>"]'
        assert _raw(e.port, b"POST /problems/current/solution HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s"
                    % (len(sol), sol)) == (
            b"HTTP/1.1 500 Internal Server Error\r\nContent-Type: text/plain; charset=utf-8\r\n"
            b"X-Content-Type-Options: nosniff\r\nDate: X\r\nContent-Length: 45\r\n\r\n"
            b"Unsuitable answer : Unknown options selected\n")
        sol = '["é"]'.encode()
        assert _raw(e.port, b"POST /problems/current/solution HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s"
                    % (len(sol), sol)) == b"HTTP/1.1 200 OK\r\nDate: X\r\nContent-Length: 0\r\n\r\n"
        t.join(20)
        assert got["ans"] == "é"
    finally:
        e.stop()


def _read_response(c):
    """One response off a keep-alive connection: (head, body)."""
    data = b""
    while b"\r\n\r\n" not in data:
        chunk = c.recv(65536)
        if not chunk:
            break
        data += chunk
    head, _, body = data.partition(b"\r\n\r\n")
    m = re.search(rb"Content-Length: (\d+)", head)
    n = int(m.group(1)) if m else 0
    while len(body) < n:
        body += c.recv(65536)
    return re.sub(rb"Date: [^\r]+", b"Date: X", head), body


def test_rest_engine_keep_alive_drains_unread_bodies():
    """net/http reads and discards a body the handler left unread before it
    answers (server.go chunkWriter.writeHeader, up to maxPostHandlerReadBytes),
    so the next request on the connection parses; a chunked solution body is
    read as ioutil.ReadAll reads it; a bad Content-Length or an unsupported
    Transfer-Encoding is refused before any handler (server.go readRequest)."""
    e = HTTPRESTEngine(0, "127.0.0.1")
    qaengine.reset()
    qaengine.add_engine(e)
    got = {}

    def ask():
        p = qa.new_input_problem("Name?", [], "d")
        got["ans"] = qaengine.fetch_answer(p).get_string_answer()

    t = threading.Thread(target=ask, daemon=True)
    t.start()
    try:
        with socket.create_connection(("127.0.0.1", e.port), timeout=20) as c:
            # a POST with a body to an unknown route, a chunked POST to the
            # GET route, then a GET: all on one connection
            c.sendall(b"POST /nope HTTP/1.1\r\nHost: x\r\nContent-Length: 5\r\n\r\nhello")
            head, body = _read_response(c)
            assert head.startswith(b"HTTP/1.1 404 Not Found") and body == b"404 page not found\n"
            assert b"Connection: close" not in head
            c.sendall(b"POST /problems/current HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n"
                      b"3\r\nabc\r\n0\r\n\r\n")
            head, body = _read_response(c)
            assert head.startswith(b"HTTP/1.1 405 Method Not Allowed") and b"Connection: close" not in head
            c.sendall(b"GET /problems/current HTTP/1.1\r\nHost: x\r\n\r\n")
            head, body = _read_response(c)
            assert head.startswith(b"HTTP/1.1 200 OK") and json.loads(body)["description"] == "Name?"
            # the answer as a chunked body, on the same connection
            c.sendall(b"POST /problems/current/solution HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n"
                      b"\r\n4\r\n[\"na\r\n4;ext=1\r\nme\"]\r\n0\r\nX-Trailer: 1\r\n\r\n")
            head, body = _read_response(c)
            assert head == b"HTTP/1.1 200 OK\r\nDate: X\r\nContent-Length: 0"
        t.join(20)
        assert got["ans"] == "name"
        for bad, want in ((b"Content-Length: x1", b"400 Bad Request"),
                          (b"Content-Length: -1", b"400 Bad Request"),
                          (b"Content-Length: 1\r\nContent-Length: 2", b"400 Bad Request"),
                          (b"Transfer-Encoding: gzip", b"501 Not Implemented")):
            with socket.create_connection(("127.0.0.1", e.port), timeout=20) as c:
                c.sendall(b"POST /problems/current/solution HTTP/1.1\r\nHost: x\r\n" + bad + b"\r\n\r\n")
                data = b""
                while True:
                    chunk = c.recv(65536)
                    if not chunk:
                        break
                    data += chunk
            text = b"400 Bad Request" if want.startswith(b"400") else b"Unsupported transfer encoding"
            assert data == (b"HTTP/1.1 " + want + b"\r\nContent-Type: text/plain; charset=utf-8\r\n"
                            b"Connection: close\r\n\r\n" + text)
        # a body too big to discard closes the connection after the reply
        with socket.create_connection(("127.0.0.1", e.port), timeout=20) as c:
            c.sendall(b"POST /nope HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % (1 << 20))
            head, body = _read_response(c)
            assert head.startswith(b"HTTP/1.1 404") and b"Connection: close" in head
    finally:
        e.stop()


def test_rest_engine_bad_body_still_answers_a_multiselect():
    """The reference's fall-through after an unmarshal error: for a
    multi-select, SetAnswer(nil) succeeds, so the translator goes on with no
    selection while the client gets the 500.  ``M2K_COMPAT=fixed`` stops at the
    error instead."""
    from move2kube_amd.utils.constants import settings
    for fixed in (False, True):
        e = HTTPRESTEngine(0, "127.0.0.1")
        qaengine.reset()
        qaengine.add_engine(e)
        got = {}

        def ask():
            p = qa.new_multiselect_problem("Pick", [], ["a"], ["a", "b"])
            got["ans"] = qaengine.fetch_answer(p).get_slice_answer()

        saved = settings.compat
        settings.compat = "fixed" if fixed else "reference"
        t = threading.Thread(target=ask, daemon=True)
        t.start()
        try:
            _get(e.port, "/problems/current")
            code, body = _post(e.port, "/problems/current/solution", "{bad")
            assert code == 500
            assert body == "Error in un-marshalling solution in QA engine: invalid character 'b' looking for " \
                           "beginning of object key string\n"
            t.join(2 if not fixed else 0.3)
            if fixed:
                assert t.is_alive()
                assert _post(e.port, "/problems/current/solution", '["b"]')[0] == 200
                t.join(20)
                assert got["ans"] == ["b"]
            else:
                assert got["ans"] == []
        finally:
            settings.compat = saved
            e.stop()


def test_cli_engine_select_confirm_input_multiselect():
    out = io.StringIO()
    inp = io.StringIO("2\ny\nhello\n1,3\n\n")
    e = CliEngine(stdin=inp, stdout=out)
    p = e.fetch_answer(qa.new_select_problem("s", [], "a", ["a", "b"]))
    assert p.get_string_answer() == "b"
    assert e.fetch_answer(qa.new_confirm_problem("c", [], False)).get_bool_answer() is True
    assert e.fetch_answer(qa.new_input_problem("i", [], "d")).get_string_answer() == "hello"
    ms = e.fetch_answer(qa.new_multiselect_problem("m", [], [], ["x", "y", "z"]))
    assert ms.get_slice_answer() == ["x", "z"]
    assert e.fetch_answer(qa.new_input_problem("i2", [], "dflt")).get_string_answer() == "dflt"
    assert "Hints:" in out.getvalue()


def test_cli_engine_plain_multiline_password_and_eof():
    out = io.StringIO()
    inp = io.StringIO("line 1\nline 2\n\n\ns3cret\n")
    e = CliEngine(stdin=inp, stdout=out)
    ml = e.fetch_answer(qa.new_multiline_input_problem("ml", [], "dflt"))
    assert ml.get_string_answer() == "line 1\nline 2"
    assert e.fetch_answer(qa.new_multiline_input_problem("ml2", [], "dflt")).get_string_answer() == "dflt"
    assert e.fetch_answer(qa.new_password_problem("pw", [])).get_string_answer() == "s3cret"
    # end of input while a question waits: Fatalf like the reference's survey error
    from move2kube_amd.utils import log
    with pytest.raises(log.FatalError):
        e.fetch_answer(qa.new_input_problem("late", [], ""))


def _cache_answers(path):
    from move2kube_amd.utils import yamlio
    with open(path) as f:
        d = yamlio.load(f.read())
    return [s["description"] for s in (d.get("spec") or {}).get("solutions") or []]


def test_write_cache_is_flushed_before_an_interactive_prompt(tmp_path):
    """Answers from non-interactive engines are written behind; the file is
    complete before any engine that may block on a person is consulted."""
    from move2kube_amd.qaengine.default_engine import DefaultEngine
    cache = str(tmp_path / "m2kqacache.yaml")
    qaengine.add_engine(DefaultEngine())
    qaengine.set_write_cache(cache)
    qaengine.fetch_answer(qa.new_input_problem("first", [], "a"))
    assert _cache_answers(cache) == []          # written behind

    seen = {}

    class Prompt(CliEngine):
        def fetch_answer(self, prob):
            seen["on_disk"] = _cache_answers(cache)
            prob.set_answer(["typed"])
            return prob
    qaengine.reset()
    qaengine.add_engine(Prompt())
    qaengine.set_write_cache(cache)
    qaengine.fetch_answer(qa.new_input_problem("first", [], "a"))  # pending
    qaengine.fetch_answer(qa.new_input_problem("second", [], "b"))
    assert seen["on_disk"] == ["first"]
    qaengine.flush_write_cache()
    assert _cache_answers(cache) == ["first", "second"]


def test_pending_answers_dropped_when_output_is_removed(tmp_path):
    from move2kube_amd.qaengine.default_engine import DefaultEngine
    out = tmp_path / "out"
    cache = str(out / "m2kqacache.yaml")
    qaengine.add_engine(DefaultEngine())
    qaengine.set_write_cache(cache)
    qaengine.fetch_answer(qa.new_input_problem("q1", [], "a"))
    qaengine.before_remove(str(out))
    import shutil
    shutil.rmtree(str(out))
    qaengine.flush_write_cache()
    assert not out.exists()           # like the reference: nothing rewrites it
    out.mkdir()
    qaengine.fetch_answer(qa.new_input_problem("q2", [], "b"))
    qaengine.flush_write_cache()
    assert _cache_answers(cache) == ["q1", "q2"]


def test_engines_print_like_go_values(tmp_path, capsys):
    """engine.go logs an engine with %T ("Ignoring engine") and %s ("Error
    while fetching answer using engine &{...}": the Cache struct with every
    problem, ints and bools as %!s(...))."""
    import logparse
    from move2kube_amd.models import qa
    from move2kube_amd.qaengine import engine as eng
    from move2kube_amd.qaengine.cache_engine import CacheEngine
    from move2kube_amd.qaengine.default_engine import DefaultEngine
    from move2kube_amd.utils import log
    log.set_verbose(False)
    cf = tmp_path / "c.yaml"
    cf.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
                  "    - description: Pick one\n      solution:\n        type: Select\n        default:\n          - a\n"
                  "        options:\n          - a\n          - b\n        answer:\n          - b\n")
    ce = CacheEngine(str(cf))
    ce.start_engine()
    assert ce.go_s() == ("&{{{move2kube.konveyor.io/v1alpha1 QACache} {} {%s [{%%!s(int=0) Pick one [] {Select [a] "
                         "[a b] [b]} %%!s(bool=true)}]}}}" % cf)
    assert DefaultEngine().go_s() == "&{}"
    eng.add_engine(CacheEngine(str(tmp_path / "missing.yaml")))
    err = capsys.readouterr().err
    msgs = logparse.messages(err)
    assert msgs[0][0] == "error" and msgs[0][1].startswith("Unable to load cache : ")
    assert msgs[1][0] == "error" and msgs[1][1].startswith("Ignoring engine *qaengine.CacheEngine due to error : ")
    assert qa.Problem(id=3, desc="d", type="Input", answer=None).go_s() == "{%!s(int=3) d [] {Input [] [] []} %!s(bool=false)}"
