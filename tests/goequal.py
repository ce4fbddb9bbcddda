"""``reflect.DeepEqual`` / ``cmp.Equal`` for the model objects: the reference's
unit tests compare whole structs, so the ported tests do too.

Two values are equal when they have the same type and, recursively, equal
contents: dicts by keys and values, lists/tuples element by element, other
objects field by field over their instance attributes.  Attributes starting
with ``_`` are caches of this implementation (index tables), not Go fields,
and are left out."""


def _fields(o):
    d = getattr(o, "__dict__", None)
    if d is None:
        slots = [n for c in type(o).__mro__ for n in getattr(c, "__slots__", ())]
        if not slots:
            return None
        d = {n: getattr(o, n) for n in slots if hasattr(o, n)}
    return {k: v for k, v in d.items() if not k.startswith("_")}


def diff(got, want, path="$"):
    """None when equal, else a description of the first difference."""
    if type(got) is not type(want):
        return "%s: type %s != %s (%r vs %r)" % (path, type(got).__name__, type(want).__name__, got, want)
    if isinstance(got, dict):
        if set(got) != set(want):
            return "%s: keys %r != %r" % (path, sorted(map(str, got)), sorted(map(str, want)))
        for k in got:
            d = diff(got[k], want[k], "%s[%r]" % (path, k))
            if d:
                return d
        return None
    if isinstance(got, (list, tuple)):
        if len(got) != len(want):
            return "%s: length %d != %d (%r vs %r)" % (path, len(got), len(want), got, want)
        for i, (x, y) in enumerate(zip(got, want)):
            d = diff(x, y, "%s[%d]" % (path, i))
            if d:
                return d
        return None
    fg, fw = _fields(got), _fields(want)
    if fg is None or fw is None:
        return None if got == want else "%s: %r != %r" % (path, got, want)
    return diff(fg, fw, path)


def assert_deep_equal(got, want):
    d = diff(got, want)
    assert d is None, d


def subtests(*cases):
    """One ``pytest.param`` per row of a Go table test: the first item of each
    case is the subtest name, used as the pytest id; a repeated name gets
    ``#01``, ``#02``, ... as testing.T names it."""
    import pytest
    seen, out = {}, []
    for c in cases:
        n = seen.get(c[0], 0)
        seen[c[0]] = n + 1
        out.append(pytest.param(*c[1:], id=c[0] + ("#%02d" % n if n else "")))
    return out
