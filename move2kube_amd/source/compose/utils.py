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
_RAM_RE = _lazy_re(r"^([0-9]+(?:\.[0-9]+)*) ?([kKmMgGtTpP])?[iI]?[bB]?\Z")
_RAM_MULT = {"k": 1024, "m": 1024 ** 2, "g": 1024 ** 3, "t": 1024 ** 4, "p": 1024 ** 5}


def ram_in_bytes(v):
    """docker/go-units v0.4.0 ``RAMInBytes`` (binary multipliers; RE2's
    ``\\d`` and ``$``: ASCII digits, end of text); ints pass through.  Errors
    are ``invalid size: '<s>'`` and ParseFloat's for ``1.2.3``."""
    if isinstance(v, bool):
        raise ValueError("invalid size")
    if isinstance(v, (int, float)):
        return int(v)
    v = str(v)
    m = _RAM_RE.match(v)
    if not m:
        raise ValueError("invalid size: '%s'" % v)
    if m.group(1).count(".") > 1:
        raise ValueError('strconv.ParseFloat: parsing "%s": invalid syntax' % m.group(1))
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
# port specs: docker/cli ``toServicePortConfigs`` over go-connections'
# ``nat.ParsePortSpecs`` and ``opts.ConvertPortToPortConfig``
# ---------------------------------------------------------------------------

def _parse_uint16(s):
    """``strconv.ParseUint(s, 10, 16)``; None when it fails."""
    if not s or not s.isascii() or not s.isdigit():
        return None
    v = int(s)
    return v if v <= 0xFFFF else None


def _parse_port_range(ports):
    """``nat.ParsePortRange``: (start, end), or None on any error (the
    callers replace the error with their own text)."""
    if not ports:
        return None
    if "-" not in ports:
        v = _parse_uint16(ports)
        return None if v is None else (v, v)
    parts = ports.split("-")
    a, b = _parse_uint16(parts[0]), _parse_uint16(parts[1])
    if a is None or b is None or b < a:
        return None
    return a, b


def _split_host_port(hostport):
    """``net.SplitHostPort`` (Go 1.15): (host, port), or raises ValueError
    with the ``*net.AddrError`` text."""
    def err(why):
        return ValueError("address %s: %s" % (hostport, why) if hostport else why)
    i = hostport.rfind(":")
    if i < 0:
        raise err("missing port in address")
    j = k = 0
    if hostport[:1] == "[":
        end = hostport.find("]")
        if end < 0:
            raise err("missing ']' in address")
        if end + 1 == len(hostport):
            raise err("missing port in address")
        if end + 1 != i:
            raise err("too many colons in address" if hostport[end + 1] == ":" else "missing port in address")
        host = hostport[1:end]
        j, k = 1, end + 1
    else:
        host = hostport[:i]
        if ":" in host:
            raise err("too many colons in address")
    if "[" in hostport[j:]:
        raise err("unexpected '[' in address")
    if "]" in hostport[k:]:
        raise err("unexpected ']' in address")
    return host, hostport[i + 1:]


def _go_parse_ipv4(s):
    for i in range(4):
        if not s:
            return False
        if i:
            if s[0] != ".":
                return False
            s = s[1:]
        n = 0
        c = 0
        while c < len(s) and "0" <= s[c] <= "9":
            n = min(n * 10 + ord(s[c]) - 48, 0xFFFFFF)
            c += 1
        if c == 0 or n > 0xFF:
            return False
        s = s[c:]
    return not s


def go_parse_ip_ok(s):
    """Is ``net.ParseIP(s)`` (Go 1.15) non-nil: dotted IPv4 (leading zeros
    allowed) or IPv6 without a zone."""
    for ch in s:
        if ch == ".":
            return _go_parse_ipv4(s)
        if ch == ":":
            if "%" in s:
                return False
            import ipaddress
            try:
                ipaddress.IPv6Address(s)
            except ValueError:
                return False
            return True
    return False


def parse_port_spec(raw):
    """``nat.ParsePortSpec``: [(host_ip, host_port, container_port, proto)]
    with the host port a string ("", a number, or a range when one container
    port takes a host range); ValueError with go-connections' text."""
    parts = raw.split(":")
    n = len(parts)
    if n == 1:
        raw_ip, host_port, cport = "", "", parts[0]
    elif n == 2:
        raw_ip, host_port, cport = "", parts[0], parts[1]
    elif n == 3:
        raw_ip, host_port, cport = parts
    else:
        raw_ip, host_port, cport = ":".join(parts[:n - 2]), parts[n - 2], parts[n - 1]
    # SplitProtoPort
    pp = cport.split("/")
    if not cport or not pp[0]:
        proto, cport = "", ""
    elif len(pp) == 1:
        proto = "tcp"
    elif not pp[1]:
        proto, cport = "tcp", pp[0]
    else:
        proto, cport = pp[1], pp[0]
    try:
        ip, _ = _split_host_port(raw_ip + ":")
    except ValueError as e:
        raise ValueError("Invalid ip address %s: %s" % (raw_ip, e))
    if ip and not go_parse_ip_ok(ip):
        raise ValueError("Invalid ip address: %s" % ip)
    if cport == "":
        raise ValueError("No port specified: %s<empty>" % raw)
    cr = _parse_port_range(cport)
    if cr is None:
        raise ValueError("Invalid containerPort: %s" % cport)
    start, end = cr
    hstart = hend = 0
    if host_port:
        hr = _parse_port_range(host_port)
        if hr is None:
            raise ValueError("Invalid hostPort: %s" % host_port)
        hstart, hend = hr
    if host_port and end - start != hend - hstart and end != start:
        raise ValueError("Invalid ranges specified for container and host Ports: %s and %s" % (cport, host_port))
    if proto.lower() not in ("tcp", "udp", "sctp"):
        raise ValueError("Invalid proto: %s" % proto)
    out = []
    for i in range(end - start + 1):
        if host_port:
            host_port = str(hstart + i)
        if start == end and hstart != hend:
            host_port = "%s-%d" % (host_port, hend)
        out.append((ip, host_port, start + i, proto.lower()))
    return out


def to_service_port_configs(value):
    """docker/cli ``toServicePortConfigs``: one short-syntax entry ->
    [(target, published, protocol, mode)], its ports in the string order of
    their ``nat.Port`` keys ("10/tcp" before "9/tcp"), a host port range
    expanded into one config per host port, and the warning
    ``ConvertPortToPortConfig`` logs for a host IP other than 0.0.0.0."""
    bindings = {}
    for ip, host_port, cport, proto in parse_port_spec(value):
        bindings.setdefault("%d/%s" % (cport, proto), []).append((ip, host_port))
    out = []
    for key in sorted(bindings):
        cport, proto = key.split("/")
        for ip, host_port in bindings[key]:
            if ip and ip != "0.0.0.0":
                log.warning("ignoring IP-address (%s:%s:%s) service will listen on '0.0.0.0'", ip, host_port, key)
            r = _parse_port_range(host_port) or (0, 0)
            for published in range(r[0], r[1] + 1):
                out.append((int(cport), published, proto, "ingress"))
    return out


# ---------------------------------------------------------------------------
# volume specs: docker/cli ``loader.ParseVolume`` (cli/compose/loader/volume.go)
# ---------------------------------------------------------------------------

def _is_windows_drive(buf, ch):
    return ch == ":" and len(buf) == 1 and buf[0].isalpha()


def _is_file_path(source):
    if source[0] in "./~" or source.startswith("\\\\"):
        return True
    return len(source) > 1 and _is_windows_drive(source[0], source[1])


def parse_volume_v3(spec):
    """Short volume syntax -> dict(type, source, target, read_only); ValueError
    with docker/cli's text.  A one-letter first section followed by ``:`` is
    a Windows drive (``c:/data:/data``), so ``v:/data`` is an anonymous
    volume whose target is ``v:/data``; a section after ``source:target`` is
    the options (``ro``/``rw``; others ignored) and one more is too many."""
    spec = str(spec)
    vol = {"type": "volume", "source": "", "target": "", "read_only": False}
    if not spec:
        raise ValueError("invalid empty volume spec")
    if len(spec) <= 2:
        vol["target"] = spec
        return vol
    buf = ""
    for ch in spec + "\0":
        if _is_windows_drive(buf, ch):
            buf += ch
        elif ch in (":", "\0"):
            err = None
            if not buf:
                err = "empty section between colons"
            elif vol["source"] == "" and ch == "\0":
                vol["target"] = buf
            elif vol["source"] == "":
                vol["source"] = buf
            elif vol["target"] == "":
                vol["target"] = buf
            elif ch == ":":
                err = "too many colons"
            else:
                for opt in buf.split(","):
                    if opt == "ro":
                        vol["read_only"] = True
                    elif opt == "rw":
                        vol["read_only"] = False
            if err:
                raise ValueError("invalid spec: %s: %s" % (spec, err))
            buf = ""
        else:
            buf += ch
    src = vol["source"]
    vol["type"] = "bind" if src and _is_file_path(src) else "volume"
    return vol


def go_abs_path(working_dir, p):
    """docker/cli loader ``absPath``: ``filepath.Join`` unless already absolute."""
    if os.path.isabs(p):
        return p
    return os.path.normpath(os.path.join(working_dir, p)) if (working_dir or p) else ""


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
    parser does; so are the lines the parse itself logs.  ``state``
    (snapshot/restore) is command-wide state the parse reads and writes: the
    memo keys on it and replays its effect."""
    from ...utils.log import go_quote

    def deco(fn):
        def checked(path):
            """(ok, result or error, log lines the parse wrote)."""
            with log.hold() as held:
                try:
                    return True, fn(path), held.lines
                except RecursionError:  # nested too deeply for the recursive walks: this file only
                    err = error_type(wrap % (path, go_quote("document nested too deeply")))
                except error_type as e:
                    err = error_type(wrap % (path, go_quote(str(e))))
            return False, err, held.lines

        @functools.wraps(fn)
        def parse(path):
            cache = fsindex.scoped_cache(name)
            if cache is None:
                hit = checked(path)
            else:
                key = (path, settings.ignore_environment, state.snapshot() if state is not None else None)
                hit = cache.get(key)
                if hit is None:
                    hit = checked(path) + (state.snapshot() if state is not None else None,)
                    cache[key] = hit
                elif state is not None:
                    state.restore(hit[3])
            # the parse's own log lines (a loader warning) come again with every call
            if hit[2]:
                log.emit(hit[2])
            if hit[0]:
                return hit[1]
            log.debug(str(hit[1]))
            raise hit[1]
        return parse
    return deco
