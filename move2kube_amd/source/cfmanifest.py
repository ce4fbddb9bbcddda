"""Cloud Foundry application manifest reading (reference
``internal/source/cfmanifest2kube.go:422-489`` on top of the CF CLI
``util/manifest`` package and bosh ``((var))`` templates).

Both the CF CLI (``ReadAndInterpolateManifest``) and the reference's own
reader first run the file through the bosh template, which decodes it with
go-yaml v2 (YAML 1.1 scalars: ``yes``/``on`` are booleans, ``010`` is octal;
a repeated key keeps its last value) and marshals it again; the decode here
is the same v2 one.

``((var))`` placeholders without a value are reported as missing variables;
:func:`read_application_manifest` replaces them with ``{{ $var }}`` (Yamls/
Knative) or ``{{ index  .Values "globalvariables" "var"}}`` (Helm) so the
generated manifests stay parameterised.
"""

import re

from ..models import plan as plantypes
from ..utils import common, log, yamlio
from ..utils.lazyre import lazy as _lazy_re

_VAR_RE = _lazy_re(r"\(\((!?[-/\.\w]+)\)\)", re.UNICODE)


class ManifestError(ValueError):
    pass


class NullInt:
    __slots__ = ("is_set", "value")

    def __init__(self, is_set=False, value=0):
        self.is_set = is_set
        self.value = value


class FilteredString:
    __slots__ = ("is_set", "value")

    def __init__(self, is_set=False, value=""):
        self.is_set = is_set
        self.value = value


class Application:
    def __init__(self):
        self.name = ""
        self.buildpack = FilteredString()
        self.buildpacks = []
        self.command = FilteredString()
        self.docker_image = ""
        self.docker_username = ""
        self.environment_variables = {}
        self.instances = NullInt()
        self.memory = ""
        self.path = ""
        self.routes = []
        self.services = []
        self.stack_name = ""
        self.no_route = False
        self.health_check_type = ""
        self.raw = {}


def _var_names(obj, out):
    if isinstance(obj, str):
        if "((" not in obj:
            return
        for m in _VAR_RE.finditer(obj):
            out.add(m.group(1).lstrip("!").split(".")[0])
    elif isinstance(obj, dict):
        for k, v in obj.items():
            _var_names(k, out)
            _var_names(v, out)
    elif isinstance(obj, list):
        for v in obj:
            _var_names(v, out)


def _evaluate(obj, values):
    """bosh template evaluation: a scalar that is exactly ((var)) is replaced by the
    value; embedded placeholders are string-interpolated."""
    if isinstance(obj, str):
        if "((" not in obj:
            return obj
        m = _VAR_RE.fullmatch(obj)
        if m:
            name = m.group(1).lstrip("!")
            if name in values:
                return values[name]
            return obj

        def repl(mm):
            name = mm.group(1).lstrip("!")
            if name in values:
                return go_sprint(values[name])
            return mm.group(0)
        return _VAR_RE.sub(repl, obj)
    if isinstance(obj, dict):
        return {_evaluate(k, values): _evaluate(v, values) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_evaluate(v, values) for v in obj]
    return obj


def _load(path):
    try:
        text = common.read_text(path)
    except OSError as e:
        raise ManifestError(common.go_path_error(e, "open"))
    try:
        return yamlio.load_v2(text)
    except yamlio.YAMLError as e:
        raise ManifestError(str(e))


def get_missing_variables(path):
    """Names of ``((vars))`` used by the manifest (all are missing: no vars
    files), ``getMissingVariables`` (cfmanifest2kube.go:472-489)."""
    try:
        doc = _load(path)
        names = set()
        _var_names(doc, names)
        if not names:
            # interpolation succeeded, so the manifest itself must decode
            _decode_manifest(doc)
    except ManifestError as e:
        log.debug("Error %s", e)
        raise
    return sorted(names)


def go_sprint(v):
    """``fmt.Sprint`` (``utils/gotemplate.py``, loaded on first use: ``collect``
    reads manifests without the template engine)."""
    from ..utils.gotemplate import go_sprint as sprint
    return sprint(v)


def _str(v):
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (dict, list)):
        raise ManifestError("cannot unmarshal collection into string")
    if isinstance(v, float):
        return yamlio.go_format_float(v)
    return str(v)


def _decode_application(d):
    if not isinstance(d, dict):
        raise ManifestError("cannot unmarshal application")
    a = Application()
    a.raw = d
    a.name = _str(d.get("name"))
    if "buildpack" in d:
        a.buildpack = FilteredString(True, _str(d.get("buildpack")))
        if a.buildpack.value in ("default", "null") or d.get("buildpack") is None:
            a.buildpack = FilteredString(True, "")
    bps = d.get("buildpacks")
    if bps is not None:
        if not isinstance(bps, list):
            raise ManifestError("buildpacks must be a list")
        a.buildpacks = [_str(x) for x in bps]
    if "command" in d:
        a.command = FilteredString(True, _str(d.get("command")))
    docker = d.get("docker")
    if docker is not None:
        if not isinstance(docker, dict):
            raise ManifestError("docker must be a mapping")
        a.docker_image = _str(docker.get("image"))
        a.docker_username = _str(docker.get("username"))
    env = d.get("env")
    if env is not None:
        if not isinstance(env, dict):
            raise ManifestError("env must be a mapping")
        a.environment_variables = {}
        for k, v in env.items():
            if isinstance(v, dict):
                raise ManifestError("env var %s cannot be a map" % k)
            a.environment_variables[_str(k)] = go_sprint(v) if v is not None else "<nil>"
    if "instances" in d and d.get("instances") is not None:
        try:
            a.instances = NullInt(True, int(str(d.get("instances"))))
        except ValueError:
            raise ManifestError("invalid instances value %r" % (d.get("instances"),))
    a.memory = _str(d.get("memory"))
    a.path = _str(d.get("path"))
    routes = d.get("routes")
    if isinstance(routes, list):
        a.routes = [_str((r or {}).get("route")) if isinstance(r, dict) else _str(r) for r in routes]
    svcs = d.get("services")
    if isinstance(svcs, list):
        a.services = [_str(s) if not isinstance(s, dict) else _str(s.get("name")) for s in svcs]
    a.stack_name = _str(d.get("stack"))
    a.no_route = bool(d.get("no-route"))
    a.health_check_type = _str(d.get("health-check-type"))
    return a


def _type_error(value, into):
    tag = {bool: "!!bool", int: "!!int", float: "!!float", str: "!!str", list: "!!seq", dict: "!!map"}.get(type(value), "!!str")
    shown = ""
    if tag not in ("!!seq", "!!map"):
        raw = _str(value)
        shown = " `" + (raw[:7] + "..." if len(raw) > 10 else raw) + "`"
    # the line is the node's in the bosh template's re-marshalled text, which
    # sorts the top-level keys: "applications" (or the whole document) comes
    # first there unless a key sorting before it exists (parity unpinned then)
    return "yaml: unmarshal errors:\n  line 1: cannot unmarshal %s%s into %s" % (tag, shown, into)


def _decode_manifest(doc):
    if doc is None:
        return []
    if not isinstance(doc, dict):
        raise ManifestError(_type_error(doc, "manifest.Manifest"))
    apps = doc.get("applications")
    if apps is None:
        return []
    if not isinstance(apps, list):
        raise ManifestError(_type_error(apps, "[]manifest.Application"))
    return [_decode_application(x) for x in apps]


def read_application_manifest(path, service_name="", artifact_type=plantypes.YAMLS):
    """(applications, variables) of a CF manifest (cfmanifest2kube.go:422-470).
    A document nested too deeply for the recursive walks is a ManifestError
    of this file (Go's growable stacks never hit that limit)."""
    try:
        return _read_application_manifest(path, service_name, artifact_type)
    except RecursionError:
        raise ManifestError("%s: document nested too deeply" % path) from None


def _read_application_manifest(path, service_name, artifact_type):
    try:
        variables = get_missing_variables(path)
    except ManifestError as e:
        log.debug("Unable to read as cf manifest %s : %s", path, e)
        raise
    try:
        doc = _load(path)
    except ManifestError as e:
        log.error("Unable to read manifest file at path %r Error: %r", path, str(e))
        raise
    values = {}
    for v in variables:
        if artifact_type == plantypes.HELM:
            values[v] = '{{ index  .Values "globalvariables" "' + v + '"}}'
        else:
            values[v] = "{{ $" + v + " }}"
    try:
        apps = _decode_manifest(_evaluate(doc, values))
    except ManifestError as e:
        log.debug("UnMarshalling error %s", e)
        raise
    if len(apps) == 1:
        return apps, variables
    if service_name:
        return [a for a in apps if a.name == service_name], variables
    return apps, variables
