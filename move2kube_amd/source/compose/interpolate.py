"""Compose variable interpolation.

* v3 follows docker/cli ``template.Substitute``: ``$$`` escapes, ``$VAR``,
  ``${VAR}``, ``${VAR:-default}``, ``${VAR-default}``, ``${VAR:?err}``,
  ``${VAR?err}``; an unset variable becomes the empty string; a malformed
  ``$`` is an error.
* v1/v2 follows libcompose: the same substitution syntax, unset variables are
  replaced by "" with a warning.
Only values are interpolated (not keys), recursively through maps and lists.
"""

import os
import re

from ...utils import log
from ...utils.lazyre import lazy as _lazy_re

_PATTERN = _lazy_re(
    r"\$(?:(?P<escaped>\$)|(?P<named>[_a-zA-Z][_a-zA-Z0-9]*)|\{(?P<braced>[_a-zA-Z][_a-zA-Z0-9]*(?::?[-?][^}]*)?)\}|(?P<invalid>))")
_BRACED_RE = _lazy_re(r"^([_a-zA-Z][_a-zA-Z0-9]*)(?:(:?)([-?])(.*))?$", re.S)


class InterpolationError(ValueError):
    pass


def substitute(s, mapping, warn_missing=False):
    def repl(m):
        if m.group("escaped") is not None:
            return "$"
        name = m.group("named") or m.group("braced")
        if name is None:
            raise InterpolationError("Invalid template: %r" % s)
        if m.group("braced") is not None:
            mm = _BRACED_RE.match(name)
            var, colon, op, arg = mm.group(1), mm.group(2), mm.group(3), mm.group(4)
            val = mapping(var)
            if op == "-":
                if val is None or (colon and val == ""):
                    return arg
                return val
            if op == "?":
                if val is None or (colon and val == ""):
                    raise InterpolationError("required variable %s is missing a value: %s" % (var, arg))
                return val
            name = var
        val = mapping(name)
        if val is None:
            if warn_missing:
                log.warning("The %s variable is not set. Substituting a blank string.", name)
            return ""
        return val
    if "$" not in s:
        return s
    return _PATTERN.sub(repl, s)


def interpolate(obj, mapping, warn_missing=False):
    if isinstance(obj, str):
        return substitute(obj, mapping, warn_missing)
    if isinstance(obj, dict):
        return {k: interpolate(v, mapping, warn_missing) for k, v in obj.items()}
    if isinstance(obj, list):
        return [interpolate(v, mapping, warn_missing) for v in obj]
    return obj


def os_env_mapping(env=None):
    env = dict(os.environ) if env is None else env
    return env.get


class EnvFileError(ValueError):
    """A line docker/cli's ``opts.ParseEnvFile`` refuses."""


def parse_env_file(path):
    """docker/cli ``opts.ParseEnvFile`` (``parseKeyValueFile``): lines as
    ``bufio.Scanner`` splits them, a UTF-8 BOM dropped from the first,
    leading white space trimmed, ``#`` comments; ``KEY=VAL`` keeps the value
    as written (trailing blanks too), a bare ``KEY`` takes the OS
    environment's value when there is one.  A key with blanks, an empty key,
    bytes that are not UTF-8 or a 64 KiB line raise :class:`EnvFileError`
    with docker/cli's text; an unreadable file raises OSError."""
    from ...utils import common
    data = common.read_bytes(path)
    lines, too_long = common.go_scan_lines(data)
    out = {}
    for n, raw in enumerate(lines):
        try:
            text = raw.decode("utf-8")
        except UnicodeDecodeError:
            raise EnvFileError("env file %s contains invalid utf8 bytes at line %d: [%s]"
                               % (path, n + 1, " ".join(str(b) for b in raw))) from None
        if n == 0 and text.startswith("\ufeff"):
            text = text[1:]
        line = text.lstrip(common._GO_SPACE)
        if not line or line.startswith("#"):
            continue
        key, eq, value = line.partition("=")
        variable = key.lstrip(" \t")
        if " " in variable or "\t" in variable:
            raise EnvFileError("poorly formatted environment: variable '%s' contains whitespaces" % variable)
        if not variable:
            raise EnvFileError("poorly formatted environment: no variable name on line '%s'" % line)
        if eq:
            out[variable] = value
        else:
            v = os.environ.get(line)
            if v is not None:
                out[common.go_trim_space(line)] = v
    if too_long:
        raise EnvFileError("bufio.Scanner: token too long")
    return out
