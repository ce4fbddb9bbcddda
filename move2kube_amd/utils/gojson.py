"""``json.Unmarshal`` into a typed Go value (Go 1.15 ``encoding/json``), for
the places the reference decodes a tool's JSON output into its own structs:
``cf curl /v2/apps`` (``sourcetypes.CfInstanceApps``), ``skopeo inspect``
(``inspect.Output``) and a CNB builder's
``io.buildpacks.builder.metadata`` order label (``cnb.order``).

The syntax check and the scanning are :mod:`fastjson`'s; this module walks
the decoded value against a type spec the way ``decodeState`` walks a
``reflect.Value``: object keys match a field's JSON name exactly or
case-insensitively, unknown keys are ignored, ``null`` leaves a value as it
is (a slice or map becomes nil), and a type mismatch is an
``UnmarshalTypeError`` - ``json: cannot unmarshal <value> into Go struct field
<Struct>.<field path> of type <type>`` inside a struct, ``... into Go value of
type <type>`` outside one - the first of which is raised once the whole
document has been decoded.

Type specs (tuples): ``("string",)``, ``("bool",)``, ``("int", gotype, bits)``,
``("slice", gotype, elem)``, ``("map", gotype, elem)`` (string keys),
``("struct", gotype, fields)`` with ``fields`` a tuple of ``(json name,
spec)`` - an embedded struct's fields listed as the outer struct's, as Go
promotes them.  The decoded value is plain dicts (present fields only), lists,
str, int and bool.
"""

from . import fastjson

STRING = ("string",)
BOOL = ("bool",)


class Number(str):
    """A JSON number kept as its literal text (Go reports ``number 1.5``)."""


def _kind(v):
    if isinstance(v, Number):
        return "number"
    if isinstance(v, bool):
        return "bool"
    return {str: "string", list: "array", dict: "object"}[type(v)]


def _short(gotype):
    """The struct name an UnmarshalTypeError shows: ``reflect.Type.Name()``."""
    return gotype.rsplit(".", 1)[-1]


class _Decoder:
    def __init__(self):
        self.err = None

    def mismatch(self, value, gotype, ctx):
        if self.err is None:
            if ctx[0]:
                self.err = "json: cannot unmarshal %s into Go struct field %s.%s of type %s" % (
                    value, ctx[0], ".".join(ctx[1]), gotype)
            else:
                self.err = "json: cannot unmarshal %s into Go value of type %s" % (value, gotype)

    def value(self, v, spec, ctx):
        kind = spec[0]
        if v is None:
            return None
        if kind == "string":
            if isinstance(v, str) and not isinstance(v, Number):
                return str(v)
            return self.mismatch(_kind(v), "string", ctx)
        if kind == "bool":
            if isinstance(v, bool):
                return v
            return self.mismatch(_kind(v), "bool", ctx)
        if kind == "int":
            _, gotype, bits = spec
            if isinstance(v, Number):
                digits = v[1:] if v[:1] == "-" else v
                if digits.isascii() and digits.isdigit() and -(1 << (bits - 1)) <= int(v) < (1 << (bits - 1)):
                    return int(v)
                return self.mismatch("number " + v, gotype, ctx)
            return self.mismatch(_kind(v), gotype, ctx)
        if kind == "slice":
            if not isinstance(v, list):
                return self.mismatch(_kind(v), spec[1], ctx)
            return [self.value(x, spec[2], ctx) for x in v]
        if kind == "map":
            if not isinstance(v, dict):
                return self.mismatch(_kind(v), spec[1], ctx)
            elem = spec[2]
            # a null element is the element type's zero value
            return {k: (_zero(elem) if x is None else self.value(x, elem, ctx)) for k, x in v.items()}
        # struct
        _, gotype, fields = spec
        if not isinstance(v, dict):
            return self.mismatch(_kind(v), gotype, ctx)
        out = {}
        for key, x in v.items():
            f = next((f for f in fields if f[0] == key), None)
            if f is None:
                folded = key.casefold()
                f = next((f for f in fields if f[0].casefold() == folded), None)
            if f is None:
                continue
            got = self.value(x, f[1], (_short(gotype), ctx[1] + [f[0]]))
            if x is not None:
                out[f[0]] = got
        return out


def _zero(spec):
    return {"string": "", "bool": False, "int": 0}.get(spec[0])


def unmarshal(data, spec):
    """The decoded value, or ValueError with the syntax error or the first
    UnmarshalTypeError as encoding/json words it."""
    doc = fastjson.loads(data, parse_int=Number, parse_float=Number)
    d = _Decoder()
    out = d.value(doc, spec, ("", []))
    if d.err is not None:
        raise ValueError(d.err)
    return out
