"""Compose helpers (reference ``internal/source/compose/utils.go``) plus the
value parsers the Go compose libraries provide (durations, byte sizes, port
specs, volume specs, Kubernetes quantity formatting)."""

import functools
import os

from ...utils import common, fsindex, log
from ...utils.constants import settings
from ...utils.lazyre import lazy as _lazy_re

MODE_READ_ONLY = "ro"
TMPFS_PATH = "tmpfs"
DEFAULT_SECRET_BASE_PATH = "/var/secrets"
ENV_FILE = "env_file"


def get_environment_variables():
    """OS environment as the v3 interpolation source (empty with --ignoreenv)."""
    if settings.ignore_environment:
        return {}
    return dict(os.environ)


def make_volumes_from_tmpfs(service_name, tfs_list):
    vms, vols = [], []
    for i, t in enumerate(tfs_list or []):
        name = "%s-%s-%d" % (service_name, TMPFS_PATH, i)
        vms.append({"name": name, "mountPath": t.split(":")[0]})
        vols.append({"name": name, "emptyDir": {"medium": "Memory"}})
    return vms, vols


def is_path(s):
    return "/" in s or s == "."


def get_hash(data):
    return common.fnv64a(data)


# ---------------------------------------------------------------------------
# Go value parsers
# ---------------------------------------------------------------------------

_DUR_UNITS = {"ns": 1, "us": 1000, "\u00b5s": 1000, "\u03bcs": 1000, "ms": 10 ** 6, "s": 10 ** 9,
              "m": 60 * 10 ** 9, "h": 3600 * 10 ** 9}
_INT64_MAX = (1 << 63) - 1


def parse_duration(s):
    """Go 1.15 ``time.ParseDuration`` -> nanoseconds: ``[-+]?([0-9]*(\\.[0-9]*)?[a-z]+)+``
    with its integer arithmetic, overflow checks and error texts
    (``time: invalid duration "x"``, ``time: missing unit in duration "1"``,
    ``time: unknown unit "d" in duration "1d"``)."""
    from ...utils.log import go_quote
    if s is None:
        raise ValueError("time: invalid duration " + go_quote(""))
    orig = s = str(s)

    def invalid():
        return ValueError("time: invalid duration " + go_quote(orig))
    neg = False
    if s and s[0] in "+-":
        neg = s[0] == "-"
        s = s[1:]
    if s == "0":
        return 0
    if not s:
        raise invalid()
    d = 0
    while s:
        if not (s[0] == "." or "0" <= s[0] <= "9"):
            raise invalid()
        i = 0
        while i < len(s) and "0" <= s[i] <= "9":
            i += 1
        pre = i > 0
        v = int(s[:i]) if pre else 0
        if v > _INT64_MAX:                      # leadingInt overflow
            raise invalid()
        s = s[i:]
        f, scale, post = 0, 1.0, False
        if s and s[0] == ".":
            s = s[1:]
            i = 0
            overflow = False
            while i < len(s) and "0" <= s[i] <= "9":
                if not overflow:
                    y = f * 10 + int(s[i])
                    if f > _INT64_MAX // 10 or y > _INT64_MAX:   # leadingFraction stops accumulating
                        overflow = True
                    else:
                        f = y
                        scale *= 10
                i += 1
            post = i > 0
            s = s[i:]
        if not pre and not post:
            raise invalid()
        i = 0
        while i < len(s) and not (s[i] == "." or "0" <= s[i] <= "9"):
            i += 1
        if i == 0:
            raise ValueError("time: missing unit in duration " + go_quote(orig))
        u, s = s[:i], s[i:]
        unit = _DUR_UNITS.get(u)
        if unit is None:
            raise ValueError("time: unknown unit " + go_quote(u) + " in duration " + go_quote(orig))
        if v > _INT64_MAX // unit:
            raise invalid()
        v *= unit
        if f > 0:
            v += int(float(f) * (float(unit) / scale))
            if v > _INT64_MAX:
                raise invalid()
        d += v
        if d > _INT64_MAX:
            raise invalid()
    return -d if neg else d


_BRACKETED_HOST_RE = _lazy_re(r"^\[([^\]]+)\]:(.*)$")
_RAM_RE = _lazy_re(r"^(\d+(?:\.\d+)*) ?([kKmMgGtTpP])?[iI]?[bB]?$")
_RAM_MULT = {"k": 1024, "m": 1024 ** 2, "g": 1024 ** 3, "t": 1024 ** 4, "p": 1024 ** 5}


def ram_in_bytes(v):
    """docker/go-units ``RAMInBytes`` (binary multipliers); ints pass through."""
    if isinstance(v, bool):
        raise ValueError("invalid size")
    if isinstance(v, (int, float)):
        return int(v)
    m = _RAM_RE.match(str(v).strip())
    if not m:
        raise ValueError("invalid size: %r" % v)
    num = float(m.group(1))
    unit = (m.group(2) or "").lower()
    return int(num * _RAM_MULT.get(unit, 1))


def format_quantity_decimal_exponent(value):
    """apimachinery Quantity.String() for an int with an unknown format
    (falls back to DecimalExponent)."""
    if value == 0:
        return "0"
    neg = value < 0
    v = abs(int(value))
    exp = 0
    while v % 1000 == 0 and v != 0:
        v //= 1000
        exp += 3
    s = str(v) + ("e%d" % exp if exp else "")
    return ("-" if neg else "") + s


def format_milli_quantity(milli):
    """Quantity.String() of NewMilliQuantity(milli, DecimalSI)."""
    if milli == 0:
        return "0"
    neg = milli < 0
    m = abs(int(milli))
    if m % 1000 == 0:
        v = m // 1000
        suffixes = [(10 ** 18, "E"), (10 ** 15, "P"), (10 ** 12, "T"), (10 ** 9, "G"), (10 ** 6, "M"), (10 ** 3, "k")]
        out = str(v)
        for mult, suf in suffixes:
            if v % mult == 0:
                out = str(v // mult) + suf
                break
    else:
        out = str(m) + "m"
    return ("-" if neg else "") + out


def shell_split(s):
    """docker/cli ``ShellCommand`` (mattn/go-shellwords) for string commands."""
    try:
        import shlex  # its module regex compiles at import: only for string commands
        return shlex.split(s)
    except ValueError:
        return s.split()


# ---------------------------------------------------------------------------
# port specs (docker/go-connections nat.ParsePortSpec)
# ---------------------------------------------------------------------------

def _port_range(s):
    if "-" in s:
        a, b = s.split("-", 1)
        a, b = int(a), int(b)
        if b < a:
            raise ValueError("invalid range")
        return list(range(a, b + 1))
    return [int(s)]


def parse_port_spec(raw):
    """Returns [(host_ip, published, target, proto)]; published 0 when unset."""
    spec = str(raw)
    proto = "tcp"
    if "/" in spec:
        spec, proto = spec.rsplit("/", 1)
        proto = proto.lower() or "tcp"
    parts = spec.rsplit(":", 2) if spec.count(":") <= 2 else None
    if parts is None:
        # IPv6 host ip in brackets
        m = _BRACKETED_HOST_RE.match(spec)
        if not m:
            raise ValueError("Invalid port spec %r" % raw)
        rest = m.group(2).split(":")
        parts = [m.group(1)] + rest
    host_ip, host_port, cont = "", "", ""
    if len(parts) == 1:
        cont = parts[0]
    elif len(parts) == 2:
        host_port, cont = parts
    else:
        host_ip, host_port, cont = parts
    if not cont:
        raise ValueError("No port specified: %r" % raw)
    cports = _port_range(cont)
    hports = _port_range(host_port) if host_port else []
    out = []
    if hports and len(hports) != len(cports):
        if len(hports) > 1:
            raise ValueError("Invalid ranges specified for container and host Ports: %r" % raw)
        # single host port range start for a container range -> docker picks a port
        hports = hports * len(cports)
    for i, c in enumerate(cports):
        out.append((host_ip, hports[i] if hports else 0, c, proto))
    return out


# ---------------------------------------------------------------------------
# volume specs
# ---------------------------------------------------------------------------

def parse_volume_v3(spec):
    """docker/cli ``loader.ParseVolume`` for Linux hosts.

    Returns dict(type, source, target, read_only)."""
    spec = str(spec)
    parts = spec.split(":")
    vol = {"type": "volume", "source": "", "target": "", "read_only": False}
    if len(parts) == 1:
        vol["target"] = parts[0]
    else:
        vol["source"] = parts[0]
        vol["target"] = parts[1]
        if len(parts) >= 3:
            for opt in parts[2].split(","):
                if opt == "ro":
                    vol["read_only"] = True
                elif opt == "rw":
                    vol["read_only"] = False
    src = vol["source"]
    if src and (src[0] in "./~"):
        vol["type"] = "bind"
    return vol


def resolve_bind_source(src, working_dir):
    if src.startswith("~"):
        home = os.path.expanduser("~")
        src = home + src[1:]
    if not os.path.isabs(src):
        src = os.path.normpath(os.path.join(working_dir, src))
    return src


def duration_seconds(d):
    """``int64(time.Duration(d).Seconds())``: whole seconds, truncated toward
    zero (a negative "-1.5s" is -1)."""
    q = abs(d) // 10 ** 9
    return -q if d < 0 else q


def command_memo(name, error_type, wrap, state=None):
    """Memoise a compose-file parser for the enclosing ``fsindex.scope()``
    (one command): the planner tries every YAML file as compose and the
    translator parses the same files again for each of their services.  The
    result depends only on the file, the ``.env``/OS environment and
    ``--ignoreenv``, none of which change within a command.  A parse error
    (``error_type``) is worded with ``wrap % (path, %q of the cause)``,
    remembered, and logged at debug level on every call as the reference's
    parser does.  ``state`` (snapshot/restore) is command-wide state the
    parse reads and writes: the memo keys on it and replays its effect."""
    from ...utils.log import go_quote

    def deco(fn):
        def checked(path):
            try:
                return fn(path)
            except RecursionError:  # nested too deeply for the recursive walks: this file only
                raise error_type(wrap % (path, go_quote("document nested too deeply"))) from None
            except error_type as e:
                raise error_type(wrap % (path, go_quote(str(e)))) from None

        @functools.wraps(fn)
        def parse(path):
            cache = fsindex.scoped_cache(name)
            if cache is None:
                try:
                    return checked(path)
                except error_type as e:
                    log.debug(str(e))
                    raise
            key = (path, settings.ignore_environment, state.snapshot() if state is not None else None)
            hit = cache.get(key)
            if hit is None:
                try:
                    hit = (True, checked(path))
                except error_type as e:
                    hit = (False, e)
                hit += (state.snapshot() if state is not None else None,)
                cache[key] = hit
            elif state is not None:
                state.restore(hit[2])
            if hit[0]:
                return hit[1]
            log.debug(str(hit[1]))
            raise hit[1]
        return parse
    return deco
