"""Helpers for decoding go-yaml-typed documents and encoding Go structs.

Documents are loaded with :func:`move2kube_amd.utils.yamlio.load_raw` (scalars
kept as text, the way go-yaml hands a scalar to a typed Go field) and then
coerced field by field with these helpers.  Encoding builds ordered dicts in
Go struct-field order and wraps Go maps in :class:`GoMap` so the emitter sorts
them like go-yaml.
"""

from ..utils.yamlio import GoMap

__all__ = ["GoMap", "as_str", "as_bool", "as_int", "as_str_list", "as_str_map",
           "as_str_list_map", "as_list", "as_map", "DecodeError"]


class DecodeError(ValueError):
    pass


def as_str(v, default=""):
    if v is None:
        return default
    if isinstance(v, (dict, list)):
        raise DecodeError("cannot unmarshal collection into string")
    return str(v)


_TRUE = {"true", "True", "TRUE", "y", "Y", "yes", "Yes", "YES", "on", "On", "ON"}
_FALSE = {"false", "False", "FALSE", "n", "N", "no", "No", "NO", "off", "Off", "OFF"}


def as_bool(v, default=False):
    if v is None:
        return default
    if isinstance(v, bool):
        return v
    s = str(v)
    if s in _TRUE:
        return True
    if s in _FALSE:
        return False
    raise DecodeError("cannot unmarshal %r into bool" % (v,))


def as_int(v, default=0):
    if v is None:
        return default
    if isinstance(v, bool):
        raise DecodeError("cannot unmarshal bool into int")
    if isinstance(v, int):
        return v
    s = str(v).replace("_", "")
    try:
        return int(s, 0)
    except ValueError:
        try:
            f = float(s)
            if f == int(f):
                return int(f)
        except ValueError:
            pass
        raise DecodeError("cannot unmarshal %r into int" % (v,))


def as_list(v):
    if v is None:
        return []
    if not isinstance(v, list):
        raise DecodeError("cannot unmarshal %r into a sequence" % (v,))
    return v


def as_map(v):
    if v is None:
        return {}
    if not isinstance(v, dict):
        raise DecodeError("cannot unmarshal %r into a mapping" % (v,))
    return v


def as_str_list(v):
    return [as_str(x) for x in as_list(v)]


def as_str_map(v):
    return {as_str(k): as_str(x) for k, x in as_map(v).items()}


def as_str_list_map(v):
    return {as_str(k): as_str_list(x) for k, x in as_map(v).items()}
