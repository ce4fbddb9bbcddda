"""The QA cache matcher skips compiling a cached description as a regex when a
literal it requires is missing from the new description
(``models/qa.py:required_literals``).  The result must always equal the
reference rule, ``strings.EqualFold(s1, s2) || regexp.MatchString(s1, s2)``
(``internal/types/qaengine/problem.go``)."""

import glob
import os
import re
import warnings

from hypothesis import given, settings, strategies as st

from move2kube_amd.models import qa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reference(s1, s2):
    if s1.casefold() == s2.casefold():
        return True
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            return re.search(qa._go_regex(s1), s2) is not None
    except re.error:
        return False


def _fresh(s1, s2):
    qa._matcher.cache_clear()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return qa._match_string(s1, s2)


_ATOMS = st.sampled_from(list("abcAB .?*+{}[]()^$|\\-,:0123") + ["\\.", "\\d", "\\s", "[a-c]", "(ab)", "x{2}", "a{1,", "(?i)",
                                                                  "[^]a]", "\\?", "Select", " service", "\\000",
                                                                  "\\x41", "\\x{42}", "\\pL", "\\u0041"])


@settings(max_examples=600, deadline=None)
@given(st.lists(_ATOMS, max_size=8).map("".join), st.lists(_ATOMS, max_size=8).map("".join))
def test_filter_agrees_with_regex_on_random_patterns(s1, s2):
    assert _fresh(s1, s2) == _reference(s1, s2)


@settings(max_examples=300, deadline=None)
@given(st.lists(_ATOMS, max_size=8).map("".join), st.text(alphabet="abcAB .?-:0123xSelctvi", max_size=20))
def test_required_literals_are_required(pattern, text):
    lits = qa.required_literals(pattern)
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            found = re.search(pattern, text) is not None
    except re.error:
        return
    if found and lits is not None:
        assert all(lit in text for lit in lits)


def test_required_literals_examples():
    assert qa.required_literals("Select all services that are needed:") == ["Select all services that are needed:"]
    assert qa.required_literals("What URL/path should we expose the service web's 8080 port on?") == [
        "What URL/path should we expose the service web's 8080 port o"]
    assert qa.required_literals("ab{2}cd") == ["a", "cd"]
    assert qa.required_literals("a.b\\.c[xy]d(e)f") == ["a", "b.c", "d", "f"]
    assert qa.required_literals("a|b") is None
    assert qa.required_literals("(?i)abc") is None
    # numeric escapes: the digits belong to the escape, not to the text
    assert qa.required_literals("\\000?") == []
    assert qa.required_literals("a\\x41?b") == ["a", "b"]
    assert qa.required_literals("a\\x{41}b") == ["a", "b"]


def test_cached_descriptions_of_the_fixtures_match_as_before():
    """Every pair of descriptions from the QA caches in the tree."""
    from move2kube_amd.utils import yamlio
    descs = []
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "**", "*qacache*.yaml"), recursive=True)):
        with open(f) as fh:
            doc = yamlio.load(fh.read()) or {}
        for p in ((doc.get("spec") or {}).get("solutions") or []):
            if isinstance(p, dict) and isinstance(p.get("description"), str):
                descs.append(p["description"])
    assert descs
    for a in descs:
        for b in descs:
            assert _fresh(a, b) == _reference(a, b), (a, b)


_DESCS = st.lists(st.sampled_from(["Select ", "service ", "api", "web", "[a-z]+", ".*", "port", " for ",
                                   "Choose", "the ", "(x|y)", "registry", ":", "?"]), max_size=9).map("".join)


@settings(max_examples=300, deadline=None)
@given(st.lists(_DESCS, max_size=40), _DESCS)
def test_desc_index_lookup_strategies_agree(listed, desc):
    """_DescIndex.candidates finds the filed pieces of a description either
    by probing every window of it or, for a small index, by substring tests of
    the pieces; both give the windows' set, and the first match equals a linear
    scan of the list (the reference's loop)."""
    problems = [qa.Problem(0, d, [], qa.INPUT, [], [], None, True) for d in listed]
    idx = qa._DescIndex(problems)
    windows = set(idx.fold.get(qa.common.go_fold(desc), ())) | idx.always
    for i in range(len(desc) - idx.Q + 1):
        windows |= idx.grams.get(desc[i:i + idx.Q], set())
    assert idx.candidates(desc) == sorted(windows)
    p = qa.Problem(0, desc, [], qa.INPUT, [], [], None, False)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        linear = next((i for i, cp in enumerate(problems) if cp.matches(p)), -1)
        assert idx.first_match(p) == linear


@settings(max_examples=500, deadline=None)
@given(st.text(alphabet="ab .^$+*?:é\n", max_size=20))
def test_simple_pattern_fast_path_equals_the_scan(pattern):
    """Patterns of literals, "." "^" "$" "+" and "*" / "?" take the str-method
    split; it gives what the character scan gives."""
    assert qa._simple_required_literals(pattern) == qa._required_literals_scan(pattern)
    assert qa.required_literals(pattern) == qa._required_literals_scan(pattern)
