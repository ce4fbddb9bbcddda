"""Differential tests of the native YAML loader (``ops/csrc/yaml_parse.cpp``)
against the PyYAML loader classes it replaces (``utils/yamlio.py:_Loaders``).

For every input and every mode (go-yaml v3 typed, go-yaml v2 typed, raw) and
both single- and multi-document decoding, the native parser must either decline
(return the ``unsupported`` sentinel, after which yamlio uses PyYAML) or return
exactly what PyYAML returns - same values, same Python types, same key order.
It must never accept a document PyYAML rejects.
"""

import math
import os

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from move2kube_amd.ops import native
from move2kube_amd.utils import yamlio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from conftest import REFERENCE  # noqa: E402
SENTINEL = object()
MODES = (yamlio._TYPED, yamlio._V2, yamlio._RAW)

pytestmark = pytest.mark.skipif(native.module() is None or not hasattr(native.module(), "yaml_load"),
                                reason="native extension not built")


def _native(text, mode, multi):
    return native.module().yaml_load(text, mode, multi, yamlio.go_resolve_number, SENTINEL)


def _pyyaml(text, mode, multi):
    lz = yamlio._lz()
    loader = (lz.typed, lz.v2, lz.raw)[mode]
    try:
        if multi:
            return True, list(lz.yaml.load_all(text, Loader=loader))
        return True, lz.yaml.load(text, Loader=loader)
    except lz.yaml.YAMLError as e:
        return False, e


def same(a, b):
    """Equal values with equal types (True != 1 here) and equal key order."""
    if type(a) is not type(b):
        return False
    if isinstance(a, dict):
        return list(a.keys()) == list(b.keys()) and all(same(k1, k2) and same(a[k1], b[k2])
                                                         for k1, k2 in zip(a.keys(), b.keys()))
    if isinstance(a, list):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    if isinstance(a, float) and math.isnan(a):
        return math.isnan(b)
    return a == b


def check(text):
    """Compare native and PyYAML on `text` in every mode; True if native decoded it."""
    decoded = False
    for mode in MODES:
        for multi in (False, True):
            got = _native(text, mode, multi)
            if got is SENTINEL:
                continue
            ok, want = _pyyaml(text, mode, multi)
            assert ok, "native accepted a document PyYAML rejects (mode %d, multi %s): %r\n%s" % (
                mode, multi, text, want)
            assert same(got, want), "mode %d multi %s\n%r\nnative: %r\npyyaml: %r" % (mode, multi, text, got, want)
            decoded = True
    return decoded


def _corpus():
    roots = [os.path.join(ROOT, d) for d in ("samples", "tests/fixtures", "tests/golden", "move2kube_amd/assets")]
    if os.path.isdir(REFERENCE):
        roots.append(REFERENCE)
    files = []
    for r in roots:
        for dp, _dn, fns in os.walk(r):
            if "/.git" in dp:
                continue
            for fn in fns:
                if fn.endswith((".yaml", ".yml")) or fn == "m2k.plan":
                    files.append(os.path.join(dp, fn))
    return sorted(files)


def test_corpus_files_decode_identically():
    files = _corpus()
    assert len(files) > 100
    native_ok = 0
    for f in files:
        with open(f, encoding="utf-8", errors="surrogateescape") as fh:
            text = fh.read()
        try:
            text.encode("utf-8")
        except UnicodeEncodeError:
            continue
        if check(text):
            native_ok += 1
    # the subset has to cover the files move2kube actually reads
    assert native_ok >= 0.85 * len(files), (native_ok, len(files))


EDGE_CASES = [
    "", "\n", "# only a comment\n", "---\n", "---\n...\n", "a\n---\nb\n", "a\n---\n", "---\na\n---\n",
    "a\n...\n", "a\n...\n---\nb\n", "a\n...\nb\n", "--- # c\na: 1\n", "--- a\n", "...\n",
    "key: value\n", "key: value # comment\n", "key: a#b\n", "key: 'it''s'\n", 'key: "a\\tb\\u00e9\\x41"\n',
    "key:\n", "key: ~\n", "key: null\nother: Null\n", "k: ''\n", 'k: ""\n',
    "a: true\nb: True\nc: yes\nd: no\ne: on\nf: off\ng: y\nh: n\ni: FALSE\n",
    "a: 1\nb: -2\nc: 0x1F\nd: 0o17\ne: 017\nf: 1e3\ng: .5\nh: 1_000\ni: +3\nj: 12:30\nk: .inf\nl: -.Inf\nm: .nan\n",
    "a: 9223372036854775807\nb: 9223372036854775808\nc: 18446744073709551616\nd: -9223372036854775809\n",
    "1: a\n2.5: b\ntrue: c\nnull: d\n~: e\n",
    "- a\n- b\n-\n- - c\n  - d\n- e: f\n  g: h\n",
    "key:\n- a\n- b\nother: c\n", "key:\n  - a\n  - b\n", "a:\n  b:\n    c: d\n  e: f\ng: h\n",
    "- a: 1\n  b:\n  - x\n  - y\n- c\n",
    "a: [1, two, \"three\", 'four', [5], {six: 6}]\n", "a: {}\nb: []\nc: { }\nd: [ ]\n",
    "a: [x, y,]\n", "a: [x: y]\n", "a: {x}\n", "a: [x,\n  y]\n", "[a, b]\n", "{a: b}\n", "[a]: b\n",
    "a: |\n  line1\n  line2\n", "a: |-\n  line1\n\n", "a: |+\n  line1\n\n\nb: 1\n", "a: |\n  x", "a: |-\n  x",
    "a: >\n  folded\n  text\n\n  para\n", "a: >-\n  one\n    more\n  two\n", "a: >+\n  x\n\n",
    "a: |2\n   leading\n  x\n", "a: |\n\n  after blank\n", "a: |\n  # not a comment\n# a comment\nb: 1\n",
    "- |\n  in seq\n- >\n  folded\n  seq\n", "a: |\n  x\n   \n  y\n", "a: |4\n    x\n",
    "a: b: c\n", "a: - b\n", "a:\n  b\n  c\n", "a: b\n  c\n", "key: 'multi\n  line'\n", "a: \"x\n  y\"\n",
    "&anchor a: 1\n", "a: &x 1\nb: *x\n", "a: !!str 1\n", "<<: {a: 1}\n", "? a\n: b\n", "%YAML 1.1\n---\na\n",
    "a:\tb\n", "a: 1\na: 2\n", "  a: 1\n  b: 2\n", "  a: 1\nb: 2\n", "a: 1\n b: 2\n",
    "a: http://x:80/y\n", "a: x:y\n", "a:b\n", "a :b\n", "'q': 1\n\"d\": 2\n", "'q' : 1\n", "a: '#x'\n",
    "a: -\n", "a: -1\n", "a: ?x\n", "a: :x\n", "a: @x\n", "a: `x`\n", "a: %x\n", "- - - x\n",
    "a:\r\n  b: c\r\n", "a: é\nü: ñ\n", "a: \u00a0x\n", "emoji: \U0001F600\n", "a: x\u2028y\n",
    "a: 'x' y\n", "a: \"x\"#y\n", "a: 'x' # c\n", "- 'x' #c\n", "a: [x] # c\n", "a: [x]#c\n",
    "a: #c\n  b: 1\n", "a: # c\n- x\n", "#c\na: 1 # c\n# c\n", "a:\n  # c\n  b: 1\n",
    "image: nginx:1.19\nports:\n  - \"80:80\"\n  - 443:443\n", "command: [\"sh\", \"-c\", \"echo $$HOME\"]\n",
    "x: <<\n", "- <<\n", "a: <none>\n", "a: =\n", "a: ---\n", "a: ...\n", "---a\n", "--- \n", "----\n",
    # implicit keys: libyaml and go-yaml refuse more than 1024 characters
    "k" * 1024 + ": v\n", "k" * 1025 + ": v\n", "k" * 1100 + ": v\n", "'" + "k" * 1100 + "': v\n",
    "a: {" + "k" * 1100 + ": v}\n", "- " + "k" * 1100 + ": v\n", "\u00e9" * 600 + ": v\n",
]


@pytest.mark.parametrize("text", EDGE_CASES)
def test_edge_cases(text):
    check(text)


def test_edge_cases_mostly_native():
    # sanity: the well-formed core of the list is decoded natively, not deferred
    for text in ["key: value\n", "- a\n- b: c\n", "a: [1, x]\n", "a: |\n  x\n", "a: >\n  x\n  y\n",
                 "---\na\n---\nb\n", "a:\n- x\nb: 1\n", "k: 'it''s'\n"]:
        assert check(text), text


def test_loader_entry_points_use_native(monkeypatch):
    """yamlio.load/load_all/load_v2/load_raw go through the native loader and
    fall back to PyYAML for what it declines."""
    assert yamlio.load("a: 1\nb: [x]\n") == {"a": 1, "b": ["x"]}
    assert yamlio.load_raw("a: 1\n") == {"a": "1"}
    assert yamlio.load_v2("a: yes\n") == {"a": True}
    assert yamlio.load_all("a\n---\nb\n") == ["a", "b"]
    assert yamlio.load("a: &x 1\nb: *x\n") == {"a": 1, "b": 1}  # anchors: PyYAML path
    with pytest.raises(yamlio.YAMLError):
        yamlio.load("a: b: c\n")
    # go-yaml's Unmarshal decodes the first document of a stream
    assert yamlio.load("a\n---\nb\n") == "a"
    assert yamlio.load("---\nk: v\n---\n: bad\n") == {"k": "v"}


# ---- generated documents ----------------------------------------------------

_TEXT = st.text(alphabet=st.sampled_from(list("abcXYZ019 -_:#'\"./\\!&*?|>{}[],%@`~=+<\n") + ["é", "ß", "\u00a0"]),
                max_size=12)
_SCALAR = st.one_of(st.none(), st.booleans(), st.integers(min_value=-2**70, max_value=2**70),
                    st.floats(allow_nan=False, width=64), _TEXT,
                    st.sampled_from(["yes", "no", "on", "off", "y", "n", "true", "null", "~", "0x1f", "017", "1e3",
                                     ".5", "12:30", "1_000", "-", "- x", "a: b", "#x", " lead", "trail ", "", "<<"]))
_KEY = st.one_of(_TEXT.filter(lambda s: s != "<<"), st.integers(min_value=-100, max_value=100), st.booleans())
_TREE = st.recursive(_SCALAR, lambda ch: st.one_of(st.lists(ch, max_size=4),
                                                   st.dictionaries(_KEY, ch, max_size=4)), max_leaves=25)


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_TREE)
def test_generated_go_yaml_style(data):
    # documents as go-yaml v3 writes them (our emitter), i.e. plans and caches
    try:
        text = yamlio.dump(data)
    except Exception:  # noqa: BLE001 - unencodable (e.g. non-string keys mix); not a parser concern
        return
    check(text)


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_TREE, st.sampled_from([False, None]), st.sampled_from([2, 4]), st.booleans())
def test_generated_pyyaml_styles(data, flow, indent, explicit):
    # documents in other writers' styles (flow collections, 4-space indents, markers)
    yaml = yamlio._lz().yaml
    try:
        text = yaml.safe_dump(data, default_flow_style=flow, indent=indent, explicit_start=explicit,
                              allow_unicode=True, sort_keys=False, width=60)
    except yaml.YAMLError:
        return
    check(text)
    check(text + "---\n" + text)


def test_nesting_past_go_yaml_limit_is_a_parse_error():
    """go-yaml refuses nesting past 10000 levels ("exceeded max depth"); the
    native parser raises that as YAMLError instead of recursing on, and the
    document is never handed to PyYAML, whose C composer overflows the stack."""
    import subprocess
    import sys
    code = ("from move2kube_amd.utils import yamlio\n"
            "import sys\n"
            "for t in [sys.argv[1] * 200000, '- ' * 200000 + 'x', 'a: x\\'\\n' + '[' * 200000]:\n"
            "    try:\n"
            "        yamlio.load(t)\n"
            "        print('accepted')\n"
            "    except yamlio.YAMLError as e:\n"
            "        print(str(e).splitlines()[0])\n")
    for native in ("1", "0"):
        p = subprocess.run([sys.executable, "-c", code, "["], cwd=ROOT, capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, M2K_NATIVE_YAML=native))
        assert p.returncode == 0, p.stderr[-2000:]
        assert p.stdout.splitlines() == ["yaml: exceeded max depth of 10000"] * 3, (native, p.stdout)
    assert yamlio.load("a: " + "[" * 9000 + "]" * 9000) is not None


def test_mutated_documents_decode_like_the_pyyaml_path(monkeypatch):
    """Differential fuzzing: the YAML files of samples/ and the fixtures with
    bytes dropped, inserted or replaced (indicators, quotes, tabs, anchors,
    tags, BOM, NUL, number-like words) decode to the same value, or fail with
    the same error, through the native loader and through PyYAML.  (A longer
    run of this loop, 12,900 documents, found no difference either.)"""
    import glob
    import random
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.setattr(yamlio, "_memo", None)
    nat = yamlio._native_loader()
    if not nat:
        pytest.skip("native extension not built")
    rnd = random.Random(11)
    corpus = []
    for p in sorted(glob.glob(os.path.join(root, "samples", "**", "*.y*ml"), recursive=True))[:25]:
        with open(p, encoding="utf-8", errors="replace") as f:
            corpus.append(f.read()[:3000])
    alphabet = list(":-[]{}\"'|>#&*!%@`?,\t\n ") + ["é", "﻿", "\x00", "\\u00", "0x", "1e9", ".inf", "~",
                                                   "null", "yes", "0o7", "+1", "<<", "!!str ", "&a ", "*a"]

    def outcome(fn, text):
        try:
            return ("ok", fn(text))
        except Exception as e:  # noqa: BLE001 - compared, not handled
            return ("err", type(e).__name__, str(e))
    for doc in corpus:
        for _ in range(20):
            t = list(doc)
            for _ in range(rnd.randint(1, 4)):
                op, i = rnd.randint(0, 2), rnd.randrange(len(t) + 1)
                if op == 0 and i < len(t):
                    del t[i]
                elif op == 1:
                    t.insert(i, rnd.choice(alphabet))
                elif i < len(t):
                    t[i] = rnd.choice(alphabet)
            text = "".join(t)
            for fn in (yamlio.load, yamlio.load_v2, yamlio.load_all):
                monkeypatch.setattr(yamlio, "_native_load", nat)
                native_says = outcome(fn, text)
                monkeypatch.setattr(yamlio, "_native_load", False)
                assert outcome(fn, text) == native_says, (fn.__name__, text)
