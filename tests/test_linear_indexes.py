"""The indexes that make ``translate`` linear in the number of services give
the same answers as the reference's linear scans:

* QA cache lookups (``types/qaengine/cache.go:84-111``): first cached problem
  whose description equals the new one case-insensitively or matches it as a
  regex, with the same type;
* IR container merge (``internal/types/ir.go:369-380``): first container of
  the same build type sharing a (case-folded) image name;
* IR storage merge (``ir.go:387-395``): first storage with the same name.
"""

import random

from hypothesis import given, settings
from hypothesis import strategies as st

from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import qa

WORDS = ["What", "URL/path", "should", "we", "expose", "the", "service", "web", "api", "db", "on?", "Select",
         "all", "services", "[quay.io]", "type", "of", "registry", "login", "(x)", "a.b", "v*", "é", "ß", "SS",
         "Enter", "name", ":", "0001", "0002", "x+", "^start", "end$", "\\d+", "{2}"]


def _desc(rng):
    return " ".join(rng.choice(WORDS) for _ in range(rng.randint(1, 9)))


def _linear_first(problems, p, pred=None):
    for i, cp in enumerate(problems):
        if cp.matches(p) and (pred is None or pred(cp)):
            return i
    return -1


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=0, max_value=10 ** 9))
def test_desc_index_agrees_with_linear_scan(seed):
    rng = random.Random(seed)
    problems = [qa.Problem(0, _desc(rng), type=rng.choice([qa.SELECT, qa.INPUT])) for _ in range(rng.randint(0, 40))]
    idx = qa._DescIndex(problems)
    for _ in range(30):
        p = qa.Problem(0, rng.choice([_desc(rng), rng.choice(problems).desc if problems else "x"]),
                       type=rng.choice([qa.SELECT, qa.INPUT]))
        assert idx.first_match(p) == _linear_first(problems, p)
        # replacement at the matched position keeps the index in step
        i = idx.first_match(p)
        if i >= 0 and rng.random() < 0.5:
            problems[i] = p.copy()
            idx.remove(i)
            idx.add(i, p.desc)


def test_cache_add_and_lookup_match_reference_order(tmp_path):
    c = qa.Cache(str(tmp_path / "c.yaml"))
    c.write_behind = True
    mk = qa.new_input_problem
    for i in range(200):
        p = mk("What URL/path should we expose the service app-%04d on?" % i, [], "/app-%04d" % i)
        p.set_answer(["/x%d" % i])
        assert c.add_problem_solution(p)
    assert len(c.problems) == 200
    # a regex-shaped cached description matches a later, longer question
    rx = mk("Select the key to use .* domain github.com :", [], "")
    rx.set_answer(["NONE"])
    c.add_problem_solution(rx)
    q = mk("Select the key to use to for the git domain github.com :", [], "")
    assert c.get_solution(q).answer == ["NONE"]
    # the same question again rewrites its entry in place
    again = mk("what url/path should we expose the service APP-0042 on?", [], "")
    again.set_answer(["/new"])
    c.add_problem_solution(again)
    assert len(c.problems) == 201 and c.problems[42].answer == ["/new"]
    q = mk("What URL/path should we expose the service app-0042 on?", [], "")
    assert c.get_solution(q).answer == ["/new"]


def test_cache_index_follows_a_replaced_list(tmp_path):
    c = qa.Cache(str(tmp_path / "c.yaml"))
    c.write_behind = True
    p = qa.new_input_problem("one", [], "")
    p.set_answer(["1"])
    c.add_problem_solution(p)
    c.problems = [qa.Problem(0, "two", type=qa.INPUT, answer=["2"], resolved=True)]
    assert c.get_solution(qa.new_input_problem("two", [], "")).answer == ["2"]


def _linear_add(containers, new):
    for c in containers:
        if c.merge(new):
            return
    containers.append(new)


def _container(rng):
    c = irtypes.Container(rng.choice(["NewDockerfile", "Reuse", "S2I"]),
                          rng.choice(["web", "WEB", "api", "db", "cache", "x"]) + rng.choice(["", ":1", ":2"]),
                          rng.random() < 0.5)
    for _ in range(rng.randint(0, 2)):
        c.image_names.append(rng.choice(["web", "api:1", "Db", "z"]))
    c.exposed_ports = [rng.choice([80, 8080])]
    return c


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=0, max_value=10 ** 9))
def test_container_index_agrees_with_linear_merge(seed):
    rng = random.Random(seed)
    news = [_container(rng) for _ in range(rng.randint(0, 30))]
    ir = irtypes.IR()
    ref = []
    for c in news:
        ir.add_container(c.copy())
        _linear_add(ref, c.copy())
    assert [(c.container_build_type, c.image_names, c.exposed_ports) for c in ir.containers] == \
           [(c.container_build_type, c.image_names, c.exposed_ports) for c in ref]


def test_container_index_survives_list_replacement():
    ir = irtypes.IR()
    ir.add_container(irtypes.Container("Reuse", "a", False))
    ir.containers = [irtypes.Container("Reuse", "b", False)]
    ir.add_container(irtypes.Container("Reuse", "B", False))
    assert len(ir.containers) == 1
    ir.add_container(irtypes.Container("Reuse", "a", False))
    assert [c.image_names for c in ir.containers] == [["b"], ["a"]]


def test_storage_index_agrees_with_linear_merge():
    rng = random.Random(7)
    ir = irtypes.IR()
    ref = []
    for _ in range(300):
        st_ = irtypes.Storage(name=rng.choice("abcdefg"), storage_type=rng.choice(["PVC", "Secret"]),
                              content={"k": str(rng.random())})
        ir.add_storage(st_.copy())
        for s in ref:
            if s.merge(st_.copy()):
                break
        else:
            ref.append(st_.copy())
    assert [(s.name, s.storage_type, s.content) for s in ir.storages] == \
           [(s.name, s.storage_type, s.content) for s in ref]


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=0, max_value=10 ** 9))
def test_container_finder_agrees_with_get_container(seed):
    """``IR.container_finder`` (the port-merge optimizer's lookup) returns the
    same container as the linear ``GetContainer`` scan (``ir.go:398-409``),
    including the ``<registry>/<ns>/<name>`` form for new images."""
    rng = random.Random(seed)
    names = ["web", "WEB", "api", "db", "Straße", "STRASSE", "quay.io/x/web", "docker.io/ns/api"]
    ir = irtypes.IR()
    ir.kubernetes.registry_url = rng.choice(["quay.io", "docker.io", ""])
    for _ in range(rng.randint(0, 12)):
        c = irtypes.Container(rng.choice(["Reuse", "NewDockerfile", "CNB"]), rng.choice(names), rng.random() < 0.5)
        for _ in range(rng.randint(0, 2)):
            c.add_image_name(rng.choice(names))
        ir.containers.append(c)
    find = ir.container_finder()
    for _ in range(20):
        q = rng.choice(names + ["%s/%s/%s" % (ir.kubernetes.registry_url, "ns", rng.choice(names)), "nope"])
        want, ok = ir.get_container(q)
        got, ok2 = find(q)
        assert ok == ok2 and got is want, q
