"""The native struct marshaller (``ops/csrc/k8s_marshal.cpp``) against its
specification, ``k8s/schema.py::_marshal_struct``: every object the expected
trees are written from, plus randomly shaped objects of every struct type
(right and wrong value types), give equal trees with equal key order - or the
same exception."""

import os
import random
import sys
import tempfile

import pytest

from move2kube_amd.k8s import schema
from move2kube_amd.ops import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")


def _fn():
    fn = schema._native_marshal()
    assert fn, "native schema_marshal not available"
    return fn


def _shape(o):
    """Value plus key order, recursively (== on dicts ignores order)."""
    if isinstance(o, dict):
        return ("d", [(k, _shape(v)) for k, v in o.items()])
    if isinstance(o, list):
        return ("l", [_shape(v) for v in o])
    return ("v", type(o).__name__, o)


def _both(obj, typ):
    fn = _fn()
    try:
        want = ("ok", _shape(schema._marshal_struct(obj, typ)))
    except Exception as e:  # noqa: BLE001
        want = ("err", type(e).__name__, str(e))
    try:
        got = ("ok", _shape(fn(obj, typ)))
    except Exception as e:  # noqa: BLE001
        got = ("err", type(e).__name__, str(e))
    return want, got


def _collect_objects():
    import refconfigs
    from move2kube_amd import transformer
    from move2kube_amd.utils import log
    seen = []
    orig = transformer.serialize_object

    def spy(obj):
        seen.append({k: v for k, v in obj.items() if k != transformer.GOTYPE})
        return orig(obj)
    log.set_quiet()
    transformer.serialize_object = spy
    try:
        names = list(refconfigs.CONFIGS) + sorted(refconfigs.COVERAGE_CONFIGS)
        for name in names:
            work = tempfile.mkdtemp(prefix="m2k-marshal-")
            run = refconfigs.Run(name, work).prepare()
            undo = run.apply_env()
            try:
                with run.session() as s:
                    run.step(s)
            finally:
                undo()
    finally:
        transformer.serialize_object = orig
    return seen


def test_objects_of_every_expected_tree():
    objs = _collect_objects()
    assert len(objs) > 300
    typed = 0
    for obj in objs:
        typ = schema.type_for(obj)
        if typ is None:
            continue
        typed += 1
        want, got = _both(obj, typ)
        assert got == want, (obj.get("kind"), obj.get("apiVersion"))
    assert typed > 300


_SCALARS = [None, "", "x", 0, 1, -3, 2.5, 0.0, True, False, [], {}, [1, "a"], {"k": "v"}, {"k": None}]


def _random_value(rng, ftype, depth):
    if depth > 4 or rng.random() < 0.15:
        return rng.choice(_SCALARS)
    if ftype.startswith("*"):
        return _random_value(rng, ftype[1:], depth)
    if ftype.startswith("[]"):
        return [_random_value(rng, ftype[2:], depth + 1) for _ in range(rng.randint(0, 3))]
    if ftype.startswith("map:"):
        return {"k%d" % i: _random_value(rng, ftype[4:], depth + 1) for i in range(rng.randint(0, 3))}
    if ftype == "map":
        return {"a": "b", "c": rng.choice(_SCALARS)}
    if ftype in schema._STRUCTS:
        return _random_struct(rng, ftype, depth + 1)
    if ftype == "bytes":
        return rng.choice(["aGk=", b"hi", bytearray(b"x"), ""])
    return rng.choice(_SCALARS)


def _random_struct(rng, typ, depth=0):
    d = {}
    for jname, ftype, _omit in schema._fields(typ):
        if jname == "inline":
            d.update(_random_struct(rng, ftype, depth))
            continue
        if rng.random() < 0.5:
            d[jname] = _random_value(rng, ftype, depth)
    if rng.random() < 0.2:
        d["unknownField"] = "dropped"
    return d


@pytest.mark.parametrize("seed", range(6))
def test_random_objects_of_every_struct_type(seed):
    rng = random.Random(seed)
    for typ in sorted(schema._STRUCTS):
        for _ in range(8):
            obj = _random_struct(rng, typ)
            want, got = _both(obj, typ)
            assert got == want, (typ, obj)


def test_empty_and_shared_empty_structs():
    fn = _fn()
    for typ in schema._STRUCTS:
        assert _shape(fn({}, typ)) == _shape(schema._marshal_struct({}, typ))
    # an absent non-pointer struct is emitted as its empty form (``resources: {}``)
    out = fn({"name": "c"}, "Container")
    assert out == {"name": "c", "resources": {}}


def test_wrong_shapes_raise_like_python():
    for obj, typ in (([1], "Pod"), ({"spec": [1, 2]}, "Deployment"), ({"metadata": {"labels": 5}}, "Service"),
                     ({"spec": {"ports": 7}}, "Service"), ({"data": ["x"]}, "Secret")):
        want, got = _both(obj, typ)
        assert got == want


def test_failed_schema_init_leaves_no_half_built_table():
    """A table that fails part-way (an inline field naming no struct) raises and
    leaves nothing behind: marshal reports the missing init, and a later init
    with the real table compiles from scratch (fresh process: the table of
    this one is already published)."""
    import subprocess
    probe = ("from move2kube_amd.ops import native\n"
             "from move2kube_amd.k8s import schema\n"
             "m = native.module()\n"
             "bad = {'A': [('x', 'string', False)], 'B': [('inline', 'Missing', False)]}\n"
             "try:\n    m.schema_init(bad, schema._marshal_value)\nexcept ValueError as e:\n    print('init', e)\n"
             "try:\n    m.schema_marshal({}, 'A')\nexcept RuntimeError as e:\n    print('marshal', e)\n"
             "m.schema_init(schema._STRUCTS, schema._marshal_value)\n"
             "print(m.schema_marshal({'name': 'c'}, 'Container'))\n")
    p = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=60)
    assert p.returncode == 0, p.stderr.decode()
    assert p.stdout.decode().splitlines() == ["init inline type Missing is not a struct",
                                              "marshal schema_init was not called",
                                              "{'name': 'c', 'resources': {}}"]


def test_field_strings_and_tuples_compile_alike():
    """schema_init takes each struct's field DSL string (what a CLI run hands
    over) or its parsed tuples; both give the same marshalling, and a field
    without a type is refused (fresh processes: a published table is kept)."""
    import subprocess
    probe = ("from move2kube_amd.ops import native\n"
             "from move2kube_amd.k8s import schema\n"
             "import sys\n"
             "m = native.module()\n"
             "if sys.argv[1] == 'bad':\n"
             "    try:\n        m.schema_init({'A': 'name:string,o oops'}, schema._marshal_value)\n"
             "    except ValueError as e:\n        print(e)\n"
             "    raise SystemExit\n"
             "table = {k: (v if sys.argv[1] == 'str' else schema._fields(k)) for k, v in schema._STRUCTS.items()}\n"
             "m.schema_init(table, schema._marshal_value)\n"
             "obj = {'metadata': {'name': 'x', 'labels': {'a': 'b'}}, 'spec': {'replicas': 2, 'template': {'spec': "
             "{'containers': [{'name': 'c', 'ports': [{'containerPort': 80}]}]}}}}\n"
             "print(sorted(m.schema_marshal(obj, 'Deployment').items()))\n")
    outs = []
    for form in ("str", "tuple", "bad"):
        p = subprocess.run([sys.executable, "-c", probe, form], cwd=ROOT, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, timeout=60)
        assert p.returncode == 0, p.stderr.decode()
        outs.append(p.stdout.decode())
    assert outs[0] == outs[1] and "'replicas': 2" in outs[0]
    assert outs[2].strip() == "field oops has no type"
