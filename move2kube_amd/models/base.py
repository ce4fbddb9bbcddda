"""Helpers for decoding go-yaml-typed documents and encoding Go structs.

Documents are loaded with :func:`move2kube_amd.utils.yamlio.load_raw` (scalars
kept as text, the way go-yaml hands a scalar to a typed Go field) and then
coerced field by field with these helpers.  Encoding builds ordered dicts in
Go struct-field order and wraps Go maps in :class:`GoMap` so the emitter sorts
them like go-yaml.
"""

import math

from ..utils.yamlio import GoMap, go_resolve_number

__all__ = ["GoMap", "as_str", "as_bool", "as_int", "as_str_list", "as_str_map",
           "as_str_list_map", "as_list", "as_map", "DecodeError", "read_document", "decode_loaded"]


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
    """A scalar into a Go int field: decode.go ``scalar()`` takes a resolved
    int, or a float64 truncated toward zero (resolve.go numbers: ``0x``,
    ``0o``, ``0b``, a leading-zero octal, underscores)."""
    if v is None:
        return default
    if isinstance(v, bool):
        raise DecodeError("cannot unmarshal bool into int")
    if isinstance(v, int):
        return v
    r = v if isinstance(v, float) else go_resolve_number(str(v))
    if isinstance(r, int) and not isinstance(r, bool):
        return r
    if isinstance(r, float) and not math.isnan(r) and -2.0 ** 63 <= r <= 2 ** 63 - 1:
        return int(r)
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


def read_document(path, decode, gotype):
    """``common.ReadMove2KubeYaml(path, &out)`` (utils.go:210-251) for the Go
    type named ``gotype`` in :mod:`.gotypes`: the move2kube group checks of
    ``common.read_move2kube_yaml``, then ``decode`` of the loaded document."""
    from ..utils import common
    text, data = common.read_move2kube_yaml_text(path)
    return decode_loaded(path, text, data, decode, gotype)


def decode_loaded(path, text, data, decode, gotype):
    """The typed half of :func:`read_document` for a document already read: a
    shape ``decode`` rejects fails with go-yaml's full list of type errors
    (:func:`.gotypes.error_text`), logged at debug level as utils.go:246-248
    does.  The Go types are only loaded on that path."""
    try:
        return decode(data)
    except DecodeError as e:
        from ..utils import log
        from . import gotypes
        msg = gotypes.error_text(text, getattr(gotypes, gotype)) or str(e)
        log.debug("Error occurred while unmarshalling yaml file at path %s Error: %r", path, msg)
        raise DecodeError(msg) from None
