"""The ledger of ported reference tests (``tests/reference_ledger.json``): every
Go test of the reference maps to a pytest node id that exists, and no entry is
stale.  The Go names come from ``tests/goreftests.py``, which reads the
reference's ``*_test.go`` files as ``go test`` would name their tests."""

import json
import os
import subprocess
import sys

import pytest

import goreftests
from conftest import REFERENCE

pytestmark = pytest.mark.reference

HERE = os.path.dirname(os.path.abspath(__file__))
LEDGER = os.path.join(HERE, "reference_ledger.json")


@pytest.fixture(scope="module")
def ledger():
    with open(LEDGER, encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def go_tests():
    return goreftests.all_test_names(REFERENCE)


def test_every_go_test_is_mapped(ledger, go_tests):
    unmapped = [(f, n) for f, names in go_tests.items() for n in names if n not in ledger["tests"].get(f, {})]
    assert unmapped == []


def test_no_stale_entries(ledger, go_tests):
    stale = [(f, n) for f, m in ledger["tests"].items() for n in m if n not in go_tests.get(f, [])]
    assert stale == []


def test_files_without_tests_are_explained(ledger, go_tests):
    empty = sorted(f for f, names in go_tests.items() if not names)
    assert empty == sorted(ledger["not_compiled"])
    for f in empty:   # all of it commented out: nothing but comments and the package clause
        with open(os.path.join(REFERENCE, f), encoding="utf-8") as fh:
            code = goreftests._strip_comments(fh.read())
        assert [ln for ln in code.split("\n") if ln.strip()] == ["package optimize"], f


def test_each_pytest_ports_one_go_test(ledger):
    ids = [n for m in ledger["tests"].values() for n in m.values()]
    assert len(ids) == len(set(ids))
    assert len(ids) >= 300


def test_every_node_id_is_collected(ledger):
    ids = sorted({n for m in ledger["tests"].values() for n in m.values()})
    files = sorted({i.split("::")[0] for i in ids})
    root = os.path.dirname(HERE)
    out = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-p", "no:cacheprovider"] + files,
                         cwd=root, capture_output=True, text=True, timeout=300)
    collected = {ln.strip() for ln in out.stdout.splitlines() if "::" in ln}
    assert [i for i in ids if i not in collected] == [], out.stdout[-2000:] + out.stderr[-2000:]


def test_extractor_reads_the_go_test_forms():
    """goreftests on the shapes the reference uses: literal t.Run, positional
    and keyed tables, a repeated name, a testify suite, a commented-out test."""
    src = '''package p

func TestPlain(t *testing.T) {}

func TestRuns(t *testing.T) {
	t.Run("first \\"one\\"", func(t *testing.T) {})
	tcs := []struct{ name, in string }{
		{"row a", "x"},
		{"row a", "y"},
	}
	for _, tc := range tcs {
		t.Run(tc.name, func(t *testing.T) {})
	}
	t.Run("last", func(t *testing.T) { s := "}"; _ = s })
}

func TestKeyed(t *testing.T) {
	tcs := []struct {
		in   int
		name string
	}{
		{in: 1, name: "k1"},
		{name: "k2", in: 2},
	}
	for _, tc := range tcs {
		t.Run(tc.name, func(t *testing.T) {})
	}
}

type S struct{ suite.Suite }

func (s *S) TestB() {}
func (s *S) TestA() {}

func TestSuite(t *testing.T) {
	suite.Run(t, new(S))
}

/*
func TestCommented(t *testing.T) {}
*/
'''
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix="_test.go", delete=False) as f:
        f.write(src)
    try:
        assert goreftests.test_names(f.name) == [
            "TestPlain", 'TestRuns/first "one"', "TestRuns/row a", "TestRuns/row a#01", "TestRuns/last",
            "TestKeyed/k1", "TestKeyed/k2", "TestSuite/TestA", "TestSuite/TestB"]
    finally:
        os.remove(f.name)
