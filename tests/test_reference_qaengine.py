"""QA engine parity (``internal/qaengine/{cache,default,}engine_test.go``)."""

import pytest

from conftest import ref_path
from move2kube_amd import qaengine
from move2kube_amd.models import qa
from move2kube_amd.qaengine.cache_engine import CacheEngine
from move2kube_amd.qaengine.default_engine import DefaultEngine
from move2kube_amd.utils import yamlio

CACHE = ref_path("internal", "qaengine", "testdata", "qaenginetest.yaml")


@pytest.fixture
def cache_engine(tmp_path):
    qaengine.reset()
    qaengine.add_engine(CacheEngine(CACHE))
    qaengine.set_write_cache(str(tmp_path / "qatest.yaml"))
    yield tmp_path / "qatest.yaml"
    qaengine.reset()


@pytest.mark.reference
def test_cache_input(cache_engine):
    p = qa.new_input_problem("Enter the container registry username : ", ["Enter username for container registry login"], "")
    assert qaengine.fetch_answer(p).get_string_answer() == "testuser"


@pytest.mark.reference
def test_cache_select(cache_engine):
    p = qa.new_select_problem("What type of container registry login do you want to use?",
                              ["Docker login from config mode, will use the default config from your local machine."],
                              "No authentication", ["Use existing pull secret", "No authentication", "UserName/Password"])
    assert qaengine.fetch_answer(p).get_string_answer() == "UserName/Password"


@pytest.mark.reference
def test_cache_multiline(cache_engine):
    p = qa.new_multiline_input_problem("Multiline input problem test description : ",
                                       ["Multiline input problem test context."], "")
    assert qaengine.fetch_answer(p).get_string_answer() == "line1 \nline2 \nline3 \n"


@pytest.mark.reference
def test_cache_confirm(cache_engine):
    p = qa.new_confirm_problem("Confirm problem test description : ", ["Confirm input problem test context."], True)
    assert qaengine.fetch_answer(p).get_bool_answer() is True


@pytest.mark.reference
def test_cache_multiselect_and_write_cache(cache_engine):
    d = ["Option A", "Option C"]
    p = qa.new_multiselect_problem("MultiSelect input problem test description : ",
                                   ["MultiSelect input problem test context"], d,
                                   ["Option A", "Option B", "Option C", "Option D"])
    assert qaengine.fetch_answer(p).get_slice_answer() == d
    qaengine.flush_write_cache()
    written = yamlio.load(cache_engine.read_text())
    assert written["kind"] == "QACache"
    sol = written["spec"]["solutions"][0]
    assert sol["solution"]["answer"] == d and sol["resolved"] is True


@pytest.mark.reference
def test_cache_regex_description_match(tmp_path):
    f = tmp_path / "c.yaml"
    f.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
                 "    - description: '\\[.*\\] Enter the name of the registry'\n      solution:\n        type: Input\n"
                 "        answer:\n          - quay.io\n      resolved: true\n")
    qaengine.reset()
    qaengine.add_engine(CacheEngine(str(f)))
    p = qa.new_input_problem("[svc] Enter the name of the registry : ", [], "docker.io")
    assert qaengine.fetch_answer(p).get_string_answer() == "quay.io"


def test_default_engine_answers():
    qaengine.reset()
    qaengine.add_engine(DefaultEngine())
    assert qaengine.fetch_answer(qa.new_input_problem("in", [], "def")).get_string_answer() == "def"
    assert qaengine.fetch_answer(qa.new_select_problem("sel", [], "b", ["a", "b"])).get_string_answer() == "b"
    assert qaengine.fetch_answer(qa.new_multiselect_problem("ms", [], ["a"], ["a", "b"])).get_slice_answer() == ["a"]
    assert qaengine.fetch_answer(qa.new_confirm_problem("c", [], True)).get_bool_answer() is True
    assert qaengine.fetch_answer(qa.new_multiline_input_problem("ml", [], "x\ny")).get_string_answer() == "x\ny"


def test_caches_are_prepended_and_last_added_wins(tmp_path):
    def cache(path, ans):
        path.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
                        "    - description: q\n      solution:\n        type: Input\n        answer:\n          - %s\n"
                        "      resolved: true\n" % ans)
        return str(path)
    qaengine.reset()
    qaengine.add_engine(DefaultEngine())
    qaengine.add_caches([cache(tmp_path / "a.yaml", "A"), cache(tmp_path / "b.yaml", "B")])
    assert [type(e).__name__ for e in qaengine.engines()] == ["CacheEngine", "CacheEngine", "DefaultEngine"]
    assert qaengine.fetch_answer(qa.new_input_problem("q", [], "d")).get_string_answer() == "A"


def test_passwords_not_cached(tmp_path):
    qaengine.reset()
    qaengine.add_engine(DefaultEngine())
    qaengine.set_write_cache(str(tmp_path / "w.yaml"))
    qaengine.fetch_answer(qa.new_password_problem("pw", []))
    qaengine.fetch_answer(qa.new_input_problem("user", [], "u"))
    qaengine.flush_write_cache()
    data = yamlio.load((tmp_path / "w.yaml").read_text())
    assert [s["description"] for s in data["spec"]["solutions"]] == ["user"]
