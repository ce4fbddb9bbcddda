"""Compose variable interpolation, each version as its reference library does it.

* v3: docker/cli ``compose/template.Substitute`` (``$$``, ``$VAR``,
  ``${VAR}``, ``${VAR:-d}``, ``${VAR-d}``, ``${VAR:?e}``, ``${VAR?e}``) and
  ``compose/interpolation.Interpolate`` with the loader's type casts.
* v1/v2: libcompose's hand-written scanner (``$$``, ``$VAR``, ``${VAR}``,
  ``${VAR:-d}``/``${VAR-d}``, no ``?`` forms) with its package-level
  defaults.
Only values are interpolated (not keys), recursively through maps and lists.
Also ``parse_env_file``: docker/cli's ``opts.ParseEnvFile``.
"""

import os

from ...utils import log
from ...utils.lazyre import lazy as _lazy_re


class InterpolationError(ValueError):
    pass


# -- v3: docker/cli compose/template + compose/interpolation ------------------

_V3_PATTERN = _lazy_re(r"\$(?i:(?P<escaped>\$)|(?P<named>[_a-z][_a-z0-9]*)|"
                       r"\{(?P<braced>[_a-z][_a-z0-9]*(?::?[-?][^}]*)?)\}|(?P<invalid>))")


class InvalidTemplateError(InterpolationError):
    """docker/cli ``template.InvalidTemplateError``; ``template`` is what
    ``newPathError`` quotes."""

    def __init__(self, template):
        super().__init__("Invalid template: " + log.go_quote(template))
        self.template = template


def _v3_funcs(sub, mapping):
    """``DefaultSubstituteFuncs`` in order - softDefault ``:-``, hardDefault
    ``-``, requiredNonEmpty ``:?``, required ``?`` - each applied when its
    separator occurs anywhere in the substitution (``strings.Contains``) and
    splitting at the first occurrence, so ``${A:?no-value}`` is a hard
    default ``value`` for the variable ``A:?no``.  Returns (value, applied);
    raises InvalidTemplateError for a required variable."""
    for sep, empty_too, required in ((":-", True, False), ("-", False, False), (":?", True, True),
                                     ("?", False, True)):
        if sep not in sub:
            continue
        name, arg = sub.split(sep, 1)
        value = mapping(name)
        missing = value is None or (empty_too and value == "")
        if required:
            if missing:
                raise InvalidTemplateError("required variable %s is missing a value: %s" % (name, arg))
            return value
        return arg if missing else value
    value = mapping(sub)
    return "" if value is None else value


def substitute_v3(template, mapping):
    """``template.Substitute``: (result, error or None).  As in docker/cli the
    error is a variable that every later substitution overwrites - with
    nothing when it succeeds - so a malformed ``$`` or a missing required
    variable only fails the value when no substitution follows it; its own
    place becomes ""."""
    err = [None]

    def repl(m):
        if m.group("escaped") is not None:
            return "$"
        sub = m.group("named") or m.group("braced")
        if not sub:
            err[0] = InvalidTemplateError(template)
            return ""
        try:
            value = _v3_funcs(sub, mapping)
        except InvalidTemplateError as e:
            err[0] = e
            return ""
        err[0] = None
        return value
    if "$" not in template:
        return template, None
    return _V3_PATTERN.sub(repl, template), err[0]


def _to_int(v):
    t = v[1:] if v[:1] in "+-" else v
    if not t or not t.isascii() or not t.isdigit():
        raise ValueError("strconv.Atoi: parsing %s: invalid syntax" % log.go_quote(v))
    n = -int(t) if v[:1] == "-" else int(t)
    if not -(1 << 63) <= n < (1 << 63):
        raise ValueError("strconv.Atoi: parsing %s: value out of range" % log.go_quote(v))
    return n


def _to_float(v):
    from ...utils.common import go_parse_float
    return go_parse_float(v)


def _to_bool(v):
    low = v.lower()
    if low in ("y", "yes", "true", "on"):
        return True
    if low in ("n", "no", "false", "off"):
        return False
    raise ValueError("invalid boolean: %s" % v)


# loader/interpolate.go interpolateTypeCastMapping: an interpolated string at
# one of these paths becomes the type the schema expects ("*" any key, "[]" a
# list element)
_V3_CASTS = tuple((tuple(pattern.split(".")), cast) for pattern, cast in (
    ("services.*.configs.[].mode", _to_int), ("services.*.secrets.[].mode", _to_int),
    ("services.*.healthcheck.retries", _to_int), ("services.*.healthcheck.disable", _to_bool),
    ("services.*.deploy.replicas", _to_int), ("services.*.deploy.update_config.parallelism", _to_int),
    ("services.*.deploy.update_config.max_failure_ratio", _to_float),
    ("services.*.deploy.rollback_config.parallelism", _to_int),
    ("services.*.deploy.rollback_config.max_failure_ratio", _to_float),
    ("services.*.deploy.restart_policy.max_attempts", _to_int),
    ("services.*.deploy.placement.max_replicas_per_node", _to_int),
    ("services.*.ports.[].target", _to_int), ("services.*.ports.[].published", _to_int),
    ("services.*.ulimits.*", _to_int), ("services.*.ulimits.*.hard", _to_int), ("services.*.ulimits.*.soft", _to_int),
    ("services.*.privileged", _to_bool), ("services.*.read_only", _to_bool), ("services.*.stdin_open", _to_bool),
    ("services.*.tty", _to_bool), ("volumes.*.external", _to_bool), ("networks.*.external", _to_bool),
    ("networks.*.internal", _to_bool), ("networks.*.attachable", _to_bool)))


def _caster(path):
    parts = path.split(".")
    for pattern, cast in _V3_CASTS:
        if len(pattern) == len(parts) and all(p in ("*", x) for p, x in zip(pattern, parts)):
            return cast
    return None


def _interpolate_v3(value, path, mapping):
    if isinstance(value, str):
        new, err = substitute_v3(value, mapping)
        if err is not None:
            raise InterpolationError("invalid interpolation format for %s: %s. You may need to escape any $ with "
                                     "another $." % (path, log.go_quote(err.template)))
        if new == value:
            return value
        cast = _caster(path)
        if cast is None:
            return new
        try:
            return cast(new)
        except ValueError as e:
            raise InterpolationError("error while interpolating %s: failed to cast to expected type: %s"
                                     % (path, e)) from None
    if isinstance(value, dict):
        return {k: _interpolate_v3(v, path + "." + str(k), mapping) for k, v in value.items()}
    if isinstance(value, list):
        return [_interpolate_v3(v, path + ".[]", mapping) for v in value]
    return value


def interpolate_v3(config, mapping):
    """``interpolation.Interpolate`` with the loader's type casts over a v3
    config dict; the first error in document order (Go walks its maps in
    random order) as InterpolationError with docker/cli's text."""
    return {k: _interpolate_v3(v, str(k), mapping) for k, v in config.items()}


# -- v1/v2: libcompose config/interpolation.go (57bd716502dc) -----------------

def _lc_name_char(c):
    return c == "_" or "A" <= c <= "Z" or "a" <= c <= "z" or "0" <= c <= "9"


class _LcFailed(Exception):
    """parseLine's ``success == false`` - or an input on which libcompose
    indexes past the end of the line (a trailing ``$`` or ``${NAME:``: a
    panic) or rescans forever (a default without its ``}`` that a later
    ``}`` appears to close)."""


def _lc_default(line, pos):
    """parseDefaultValue: every leading ``:`` and ``-`` is skipped, the rest up
    to ``}`` is the default; (default, index before the ``}``)."""
    n = len(line)
    while pos < n and line[pos] in ":-":
        pos += 1
    start = pos
    while pos < n:
        if line[pos] == "}":
            return line[start:pos], pos - 1
        pos += 1
    raise _LcFailed()


def _lc_braces(line, pos, mapping, defaults):
    """parseVariableWithBraces: a default (``:-`` or ``-``) is recorded in the
    package-level ``defaultValues`` under the name read so far, then the
    closing ``}`` returns the mapping of the name."""
    n = len(line)
    name = []
    while pos < n:
        c = line[pos]
        if c == "}":
            if not name:
                raise _LcFailed()
            return mapping("".join(name)), pos
        if _lc_name_char(c):
            name.append(c)
        elif c == "-" or c == ":":
            if c == ":" and (pos + 1 >= n or line[pos + 1] != "-"):
                raise _LcFailed()
            defaults["".join(name)], pos = _lc_default(line, pos)
        else:
            raise _LcFailed()
        pos += 1
    raise _LcFailed()


def _lc_parse_line(line, mapping, defaults):
    out = []
    pos, n = 0, len(line)
    while pos < n:
        c = line[pos]
        if c != "$":
            out.append(c)
            pos += 1
            continue
        pos += 1
        if pos >= n:
            raise _LcFailed()
        c = line[pos]
        if c == "$":
            out.append("$")
        elif c == "{":
            val, pos = _lc_braces(line, pos + 1, mapping, defaults)
            out.append(val)
        elif _lc_name_char(c) and not ("0" <= c <= "9"):
            start = pos
            while pos < n and _lc_name_char(line[pos]):
                pos += 1
            out.append(mapping(line[start:pos]))
            pos -= 1
        else:
            raise _LcFailed()
        pos += 1
    return "".join(out)


def _lc_value(key, value, mapping, defaults):
    if isinstance(value, str):
        try:
            return _lc_parse_line(value, mapping, defaults)
        except _LcFailed:
            raise InterpolationError('Invalid interpolation format for key "%s": "%s"' % (key, value)) from None
    if isinstance(value, list):
        return [_lc_value(key, v, mapping, defaults) for v in value]
    if isinstance(value, dict):
        return {k: _lc_value(key, v, mapping, defaults) for k, v in value.items()}
    return value


def interpolate_v1v2(raw_services, lookup, defaults):
    """``InterpolateRawServiceMap``: every field of every service, the error
    naming the field's key.  ``lookup(name)`` is libcompose's environment
    lookup (None when it finds nothing; the OS lookup finds nothing for an
    empty variable).  An unset variable takes a default recorded by any
    ``${NAME:-x}`` or ``${NAME-x}`` read before it in this command (libcompose
    keeps them in a package-level map, so they outlive the value and the file
    that set them); so does a variable set to "" - both forms mean "unset or
    empty" here.  Otherwise unset is "" with a warning, which the reference
    never shows: it parses at logrus FatalLevel (v1v2.go:118-121)."""
    def mapping(name):
        value = lookup(name)
        if value is None:
            if name in defaults:
                return defaults[name]
            log.warning("The %s variable is not set. Substituting a blank string.", name)
            return ""
        if value == "" and name in defaults:
            return defaults[name]
        return value
    return {name: ({k: _lc_value(k, v, mapping, defaults) for k, v in svc.items()} if isinstance(svc, dict) else svc)
            for name, svc in raw_services.items()}


class EnvFileError(ValueError):
    """A line docker/cli's ``opts.ParseEnvFile`` refuses."""


def parse_env_file(path, first_wins=False):
    """docker/cli ``opts.ParseEnvFile`` (``parseKeyValueFile``): lines as
    ``bufio.Scanner`` splits them, a UTF-8 BOM dropped from the first,
    leading white space trimmed, ``#`` comments; ``KEY=VAL`` keeps the value
    as written (trailing blanks too), a bare ``KEY`` takes the OS
    environment's value when there is one.  A key with blanks, an empty key,
    bytes that are not UTF-8 or a 64 KiB line raise :class:`EnvFileError`
    with docker/cli's text; an unreadable file raises OSError.  A key given
    twice keeps its last value, or its first with ``first_wins`` (libcompose's
    ``EnvfileLookup`` returns the first line that names the key)."""
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
            if not (first_wins and variable in out):
                out[variable] = value
        else:
            v = os.environ.get(line)
            if v is not None and not (first_wins and common.go_trim_space(line) in out):
                out[common.go_trim_space(line)] = v
    if too_long:
        raise EnvFileError("bufio.Scanner: token too long")
    return out
