"""Interactive engines: the HTTP REST protocol the UI uses and the terminal engine."""

import io
import json
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
