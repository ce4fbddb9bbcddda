"""Repeated mapping keys: go-yaml v3 (the reference's ``yaml.Unmarshal`` for
plans, QA caches, collect outputs, cluster metadata, CF manifests and kubectl
output) fails the decode with ``yaml: unmarshal errors`` naming every repeated
key and the line of its first occurrence; go-yaml v2 (compose files, and the
Kubernetes objects client-go decodes through sigs.k8s.io/yaml) keeps the last
value.  The native block parser never decodes such a document itself."""

import pytest

from move2kube_amd.ops import native
from move2kube_amd.utils import yamlio


@pytest.mark.parametrize("text,errors", [
    ("a: 1\na: 2\n", ['line 2: mapping key "a" already defined at line 1']),
    ("a: 1\nb: 2\na: 3\na: 4\n", ['line 3: mapping key "a" already defined at line 1',
                                   'line 4: mapping key "a" already defined at line 1',
                                   'line 4: mapping key "a" already defined at line 3']),
    ('1: x\n"1": y\n', ['line 2: mapping key "1" already defined at line 1']),   # same node value
    ("x:\n  c: {d: 1, d: 2}\ny:\n  - k: 1\n    k: 2\n", ['line 2: mapping key "d" already defined at line 2',
                                                           'line 5: mapping key "k" already defined at line 4']),
    # a mapping with repeated keys is not descended into
    ("a: {b: 1, b: 2}\na: 2\n", ['line 2: mapping key "a" already defined at line 1']),
])
def test_v3_decoders_refuse_repeated_keys(text, errors):
    want = "yaml: unmarshal errors:\n  " + "\n  ".join(errors)
    for load in (yamlio.load, yamlio.load_raw):
        with pytest.raises(yamlio.YAMLError) as ei:
            load(text)
        assert str(ei.value) == want
    with pytest.raises(yamlio.YAMLError):
        yamlio.load_all(text)


def test_v2_decoders_keep_the_last_value():
    assert yamlio.load_v2("a: 1\na: 2\n") == {"a": 2}
    assert yamlio.load_v2("a: yes\na: no\n") == {"a": False}
    assert yamlio.load_all_v2("a: 1\na: 2\n---\nb: 1\n") == [{"a": 2}, {"b": 1}]
    with yamlio.parse_cache():  # the shared typed parse answers both flavours
        assert yamlio.load_v2("k: 1\nk: 2\n") == {"k": 2}
        with pytest.raises(yamlio.YAMLError):
            yamlio.load("k: 1\nk: 2\n")


def test_distinct_node_values_are_not_repeated_keys():
    # 1 and 01 are different node values (go-yaml compares the source text)
    yamlio.load("1: a\n01: b\n")


@pytest.mark.skipif(not native.available(), reason="native extension not built")
def test_native_parser_defers_repeated_keys():
    m = native.module()
    sentinel = object()
    for text in ("a: 1\na: 2\n", "x: {a: 1, a: 2}\n", "'a': 1\na: 2\n", "1: a\n'1': b\n"):
        assert m.yaml_load(text, 0, False, yamlio.go_resolve_number, sentinel) is sentinel
    assert m.yaml_load("a: 1\nb: 2\n", 0, False, yamlio.go_resolve_number, sentinel) == {"a": 1, "b": 2}


def test_plan_with_a_repeated_key_is_refused(tmp_path):
    from move2kube_amd.models import plan as plantypes
    p = tmp_path / "m2k.plan"
    p.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: Plan\nmetadata:\n  name: a\n  name: b\n"
                 "spec:\n  inputs:\n    rootDir: .\n")
    with pytest.raises(Exception) as ei:
        plantypes.read_plan(str(p))
    assert 'mapping key "name" already defined at line 4' in str(ei.value)


def test_repeated_key_checks_are_linear():
    import time
    n = 50000
    text = "".join("k%d: %d\n" % (i, i) for i in range(n))
    t0 = time.perf_counter()
    assert len(yamlio.load(text)) == n
    with pytest.raises(yamlio.YAMLError):
        yamlio.load(text + "k7: again\n")
    assert time.perf_counter() - t0 < 20
