"""The QA engine chain (``qaengine/engine.py``; reference
``internal/qaengine/engine.go:29-123``) off the happy path: engines that fail
to start are skipped with the reference's error line, an engine that fails is
logged and the next one asked, the last engine is retried a bounded number of
times (the reference loops forever) before the default is
taken, a problem with no default then stops the run, and an interactive
engine sees the write cache flushed before it may block on a person."""

import pytest

import logparse
from move2kube_amd import qaengine
from move2kube_amd.models import qa
from move2kube_amd.qaengine import engine
from move2kube_amd.utils import log


@pytest.fixture(autouse=True)
def fresh_chain():
    log.set_verbose(False)
    engine.reset()
    yield
    engine.reset()


class Fake(engine.Engine):
    go_type = "*qaengine.Fake"

    def __init__(self, answers=(), fail_start=False, interactive=False):
        self.answers = list(answers)   # each: an answer list, None (unresolved) or an Exception
        self.fail_start = fail_start
        self.interactive = interactive
        self.asked = 0

    def start_engine(self):
        if self.fail_start:
            raise RuntimeError("no terminal")

    def fetch_answer(self, prob):
        self.asked += 1
        a = self.answers.pop(0) if self.answers else None
        if isinstance(a, Exception):
            raise a
        if a is not None:
            prob.set_answer(a)
        return prob


def _select(default="b"):
    return qa.new_select_problem("Pick one:", [], default, ["a", "b", "c"])


def test_an_engine_that_cannot_start_is_ignored(capsys):
    engine.add_engine(Fake(fail_start=True))
    assert engine.engines() == []
    assert logparse.logged(capsys.readouterr().err, "Ignoring engine *qaengine.Fake due to error : no terminal",
                           "error")


def test_a_cache_file_that_cannot_be_read_is_ignored(tmp_path, capsys):
    bad = tmp_path / "cache.yaml"
    bad.write_text("kind: [\n")
    engine.add_caches([str(bad)])
    assert engine.engines() == []
    assert logparse.logged_containing(capsys.readouterr().err, "Ignoring engine *qaengine.CacheEngine due to error :",
                                      "error")


def test_the_first_engine_that_resolves_wins(capsys):
    first, second = Fake([RuntimeError("down")]), Fake([["c"]])
    engine.add_engine(first)
    engine.add_engine(second)
    assert engine.fetch_answer(_select()).get_string_answer() == "c"
    assert logparse.logged(capsys.readouterr().err, "Error while fetching answer using engine &{} : down", "warning")


def test_the_last_engine_is_retried_then_the_default_is_taken():
    last = Fake([None] * 3 + [["a"]])
    engine.add_engine(last)
    assert engine.fetch_answer(_select()).get_string_answer() == "a"
    assert last.asked == 4
    stubborn = Fake()
    engine.reset()
    engine.add_engine(stubborn)
    assert engine.fetch_answer(_select("b")).get_string_answer() == "b"
    assert stubborn.asked == 1 + engine.MAX_LAST_ENGINE_RETRIES


def test_no_answer_and_no_default_is_fatal():
    engine.add_engine(Fake([RuntimeError("x")] * 20))
    prob = qa.new_select_problem("Name?", [], "a", ["a", "b"])
    prob.default = []
    with pytest.raises(log.FatalError, match="Unable to get answer to Name\\? : x"):
        engine.fetch_answer(prob)


def test_an_empty_chain_takes_defaults():
    assert engine.fetch_answer(_select("c")).get_string_answer() == "c"


def test_interactive_engines_see_the_cache_flushed(tmp_path):
    cache = engine.set_write_cache(str(tmp_path / "out" / "m2kqacache.yaml"))
    auto = Fake([["a"], ["a"]])
    engine.add_engine(auto)
    engine.fetch_answer(_select())
    with open(cache.file) as f:
        before = f.read()
    assert "Pick one:" not in before          # write-behind: pending
    person = Fake([["b"]], interactive=True)
    engine.reset()
    cache = engine.set_write_cache(str(tmp_path / "out2" / "m2kqacache.yaml"))
    engine.add_engine(Fake([None]))
    engine.add_engine(person)
    engine.fetch_answer(qa.new_select_problem("First:", [], "a", ["a", "b"]))
    engine.fetch_answer(qa.new_select_problem("Second:", [], "a", ["a", "b"]))
    with open(cache.file) as f:
        text = f.read()
    assert "First:" in text                   # flushed before the person was asked the second question
    assert engine.get_write_cache() is cache


def test_before_remove_keeps_or_drops_pending_answers(tmp_path):
    cache = engine.set_write_cache(str(tmp_path / "out" / "m2kqacache.yaml"))
    engine.add_engine(Fake([["a"], ["a"]]))
    engine.fetch_answer(qa.new_select_problem("Kept:", [], "a", ["a"]))
    engine.before_remove(str(tmp_path / "elsewhere"))   # not under the output: persisted
    assert "Kept:" in open(cache.file).read()
    engine.fetch_answer(qa.new_select_problem("Dropped:", [], "a", ["a"]))
    engine.before_remove(str(tmp_path / "out"))         # the output goes: pending dropped
    engine.flush_write_cache()
    assert "Dropped:" not in open(cache.file).read()
    engine.reset()
    engine.before_remove(str(tmp_path))                 # no cache: nothing to do


def test_start_engine_picks_by_flags():
    assert type(qaengine.start_engine(qaskip=True)).__name__ == "DefaultEngine"
    engine.reset()
    assert type(qaengine.start_engine()).__name__ == "CliEngine"
    engine.reset()
    e = qaengine.start_engine(qadisablecli=True)
    try:
        assert type(e).__name__ == "HTTPRESTEngine" and e.port > 0
    finally:
        e.stop()


def test_engine_base_prints_like_go():
    e = engine.Engine()
    assert e.go_s() == "&{}" and repr(e) == "Engine"
    e.start_engine()
    with pytest.raises(NotImplementedError):
        e.fetch_answer(None)


def test_cache_miss_error_prints_the_problem_like_go(tmp_path):
    """``GetSolution`` (types/qaengine/cache.go:125) reports a miss with
    ``%+v`` of the Problem struct: field names, nil slices as ``[]``."""
    c = qa.Cache(str(tmp_path / "c.yaml"))
    prob = qa.new_select_problem("Pick one:", ["ctx a", "ctx b"], "b", ["a", "b"])
    with pytest.raises(qa.ProblemError) as ei:
        c.get_solution(prob)
    assert str(ei.value) == ("The problem {ID:%d Desc:Pick one: Context:[ctx a ctx b] Solution:{Type:Select "
                             "Default:[b] Options:[a b] Answer:[]} Resolved:false} was not found in the cache"
                             % prob.id)
