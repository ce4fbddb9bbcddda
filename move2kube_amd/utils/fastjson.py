"""JSON decoding straight on the C scanner (``_json.make_scanner``), the one
the stdlib ``json`` package wraps, so the read paths of a command (cluster
profiles, detector output, ``~/.docker/config.json``) do not import the
four-module ``json`` package.  Same results and errors class as
``json.loads`` (``ValueError``); encoding still goes through ``json``.
"""

import _json

_CONSTANTS = {"-Infinity": float("-inf"), "Infinity": float("inf"), "NaN": float("nan")}


class _Context:
    """The attributes ``_json.make_scanner`` reads from a ``JSONDecoder``."""

    def __init__(self, parse_int=int):
        self.strict = True
        self.object_hook = None
        self.object_pairs_hook = None
        self.parse_float = float
        self.parse_int = parse_int
        self.parse_constant = _CONSTANTS.__getitem__
        self.memo = {}


_scanners = {}
_WS = " \t\n\r"


def loads(s, parse_int=int):
    if isinstance(s, (bytes, bytearray)):
        s = s.decode("utf-8-sig" if s[:3] == b"\xef\xbb\xbf" else "utf-8")
    scan = _scanners.get(parse_int)
    if scan is None:
        scan = _scanners[parse_int] = _json.make_scanner(_Context(parse_int))
    i, n = 0, len(s)
    while i < n and s[i] in _WS:
        i += 1
    try:
        obj, end = scan(s, i)
    except StopIteration as e:
        raise ValueError("Expecting value: char %d" % e.value) from None
    while end < n and s[end] in _WS:
        end += 1
    if end != n:
        raise ValueError("Extra data: char %d" % end)
    return obj


def load(f, parse_int=int):
    return loads(f.read(), parse_int)
