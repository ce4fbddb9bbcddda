"""Compose file format v3 loader (reference ``internal/source/compose/v3.go``).

Parsing mirrors docker/cli's loader as the reference uses it: YAML parse,
pruning of env_files that do not exist, version/forbidden-key/schema checks,
interpolation from the OS environment (skipped with ``--ignoreenv``), service
transformation (short/long port and volume syntax, environment list/map,
healthcheck, deploy, secrets, configs) and bind-volume path resolution
relative to the compose file's directory.
"""

import os
import stat

from ...containerizer.reusedockerfile import ReuseDockerfileContainerizer
from ...models import ir as irtypes
from ...utils import common, log, yamlio
from ...utils.constants import VOLUME_PREFIX
from ...utils.lazyre import lazy as _lazy_re
from ...utils.log import go_quote
from . import schema as cschema
from . import utils as cu
from .interpolate import EnvFileError, InterpolationError, interpolate_v3, parse_env_file

SUPPORTED_V3 = {"3", "3.0", "3.1", "3.2", "3.3", "3.4", "3.5", "3.6", "3.7", "3.8", "3.9"}

TOP_KEYS = {"version", "services", "networks", "volumes", "secrets", "configs"}
SERVICE_KEYS = {
    "build", "cap_add", "cap_drop", "cgroup_parent", "command", "configs", "container_name", "credential_spec",
    "depends_on", "deploy", "devices", "dns", "dns_search", "domainname", "entrypoint", "env_file", "environment",
    "expose", "external_links", "extra_hosts", "healthcheck", "hostname", "image", "init", "ipc", "isolation",
    "labels", "links", "logging", "mac_address", "network_mode", "networks", "pid", "ports", "privileged",
    "read_only", "restart", "secrets", "security_opt", "shm_size", "stdin_open", "stop_grace_period",
    "stop_signal", "sysctls", "tmpfs", "tty", "ulimits", "user", "userns_mode", "volumes", "working_dir",
}
# docker/cli types.ForbiddenProperties
FORBIDDEN = ("extends", "volume_driver", "volumes_from", "cpu_quota", "cpu_shares", "cpuset", "mem_limit",
             "memswap_limit")


class ComposeError(ValueError):
    pass


def _version(d):
    if "version" not in d:
        return "1.0"
    v = d["version"]
    if isinstance(v, bool):
        v = "true" if v else "false"
    elif isinstance(v, float):
        v = yamlio.go_format_float(v)
    v = str(v)
    if v == "3":
        return "3.0"
    return v


def _env_file_missing(p):
    """``os.IsNotExist(err) || finfo.IsDir()`` of ``removeNonExistentEnvFilesV3``
    (v3.go:61-65): only a path that does not exist, or a directory, is dropped.
    Any other stat error (permission denied on a parent, ENOTDIR, a loop)
    panics there on the nil FileInfo; here the file is kept, and reading it
    fails the load (:func:`_read_env_file`)."""
    import stat
    try:
        return stat.S_ISDIR(os.stat(p).st_mode)
    except FileNotFoundError:
        return True
    except OSError:
        return False


def remove_non_existent_env_files(path, parsed):
    base = os.path.dirname(path)
    services = parsed.get("services") if isinstance(parsed, dict) else None
    if not isinstance(services, dict):
        return parsed
    for sname, vals in services.items():
        if not isinstance(vals, dict) or cu.ENV_FILE not in vals:
            continue
        ef = vals[cu.ENV_FILE]
        if isinstance(ef, str):
            p = ef if os.path.isabs(ef) else os.path.join(base, ef)
            if _env_file_missing(p):
                log.warning("Unable to find env config file %s referred in service %s in file %s. Ignoring it.", p, sname, path)
                del vals[cu.ENV_FILE]
        elif isinstance(ef, list):
            kept = []
            for e in ef:
                if isinstance(e, str):
                    p = e if os.path.isabs(e) else os.path.join(base, e)
                    if _env_file_missing(p):
                        log.warning("Unable to find env config file %s referred in service %s in file %s. Ignoring it.", p, sname, path)
                        continue
                    kept.append(e)
            vals[cu.ENV_FILE] = kept
    return parsed


def _read_env_file(p):
    """docker/cli ``opts.ParseEnvFile`` on an env file the removal kept: an
    error opening or reading it is the load's error as it is
    (``open <path>: permission denied``).  A FIFO, socket or device is an
    error too, where ``os.Open`` in the reference would block on it forever."""
    try:
        return parse_env_file(p)
    except FileNotFoundError:   # removed between the removal pass and here
        return {}
    except OSError as e:
        from ...utils import common
        raise EnvFileError(common.go_path_error(e, getattr(e, "go_op", "open"))) from None


def _as_list_of_str(v):
    if v is None:
        return []
    if isinstance(v, (str, int, float)):
        return [str(v)]
    return [str(x) if not isinstance(x, bool) else ("true" if x else "false") for x in v]


def _scalar_str(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return yamlio.go_format_float(v)
    return "" if v is None else str(v)


def _mapping_with_equals(v):
    """list 'K=V' / 'K' or map -> ordered {K: V or None}."""
    out = {}
    if isinstance(v, dict):
        for k, x in v.items():
            out[str(k)] = None if x is None else _scalar_str(x)
    elif isinstance(v, list):
        for item in v:
            s = _scalar_str(item)
            if "=" in s:
                k, x = s.split("=", 1)
                out[k] = x
            else:
                out[s] = None
    return out


def _labels(v):
    m = _mapping_with_equals(v)
    return {k: (x if x is not None else "") for k, x in m.items()}


_SERVICE_NAME_RE = _lazy_re(r"^[a-zA-Z0-9._-]+\Z")


def _validate(d):
    if not isinstance(d, dict):
        raise ComposeError("Top-level object must be a mapping")
    for k in d:
        if not isinstance(k, str):
            raise ComposeError("Non-string key at top level: %r" % (k,))
        if k not in TOP_KEYS and not k.startswith("x-"):
            # gojsonschema names the root context "(root)"
            raise ComposeError("(root) Additional property %s is not allowed" % k)
    services = d.get("services")
    if not isinstance(services, dict):
        if "services" in d and services is None:
            services = {}
        elif "services" in d:
            raise ComposeError("services must be a mapping")
        else:
            services = {}
    for sname, svc in services.items():
        # "services": patternProperties ^[a-zA-Z0-9._-]+$, additionalProperties false;
        # a service is "type": "object" (null included: LoadServices would not survive it)
        if not _SERVICE_NAME_RE.match(str(sname)):
            raise ComposeError("services Additional property %s is not allowed" % sname)
        if not isinstance(svc, dict):
            raise ComposeError("services.%s must be a mapping" % sname)
        for k in svc:
            if k not in SERVICE_KEYS and not str(k).startswith("x-"):
                raise ComposeError("services.%s Additional property %s is not allowed" % (sname, k))
    for key in ("networks", "volumes", "secrets", "configs"):
        v = d.get(key)
        if v is not None and not isinstance(v, dict):
            raise ComposeError("%s must be a mapping" % key)
    return services


def _check_forbidden(d):
    """docker/cli ``validateForbidden``, before interpolation: a service using
    one of ``types.ForbiddenProperties`` fails the load."""
    services = d.get("services")
    if isinstance(services, dict) and any(isinstance(svc, dict) and any(k in FORBIDDEN for k in svc)
                                          for svc in services.values()):
        raise ComposeError("Configuration contains forbidden properties")


def _go_repr(k):
    """Go ``%#v`` of a YAML key go-yaml v2 decoded into interface{}."""
    if k is None:
        return "<nil>"
    if isinstance(k, bool):
        return "true" if k else "false"
    if isinstance(k, float):
        return yamlio.go_format_float(k)
    return str(k)


def _check_string_keys(v, prefix):
    """docker/cli ``ParseYAML``: every mapping key in the document must be a
    string (go-yaml v2 turns ``y:``, ``on:``, ``1:`` keys into bools/ints),
    otherwise the whole file fails to load (``convertToStringKeysRecursive``)."""
    if isinstance(v, dict):
        for k, x in v.items():
            if not isinstance(k, str):
                where = "at top level" if not prefix else "in " + prefix
                raise ComposeError("Non-string key %s: %s" % (where, _go_repr(k)))
            _check_string_keys(x, k if not prefix else prefix + "." + k)
    elif isinstance(v, list):
        for i, x in enumerate(v):
            _check_string_keys(x, "%s[%d]" % (prefix, i))


def _external(spec):
    ext = spec.get("external")
    return isinstance(ext, dict) or bool(ext)


def _version_ge(v, other):
    """docker ``versions.GreaterThanOrEqualTo``: dotted fields compared as
    integers (a non-number is 0)."""
    def ints(x):
        out = []
        for f in x.split("."):
            f = f.strip()
            out.append(int(f) if f.isascii() and f.isdigit() else 0)
        return out
    a, b = ints(v), ints(other)
    n = max(len(a), len(b))
    return a + [0] * (n - len(a)) >= b + [0] * (n - len(b))


def _external_name(kind, name, spec, version, deprecated_from):
    """The ``external.name`` rules of ``LoadNetworks`` / ``LoadVolumes`` /
    ``loadFileObjectConfig``: it conflicts with ``name``, is deprecated (a
    warning) from ``deprecated_from`` on, and becomes the name; an external
    object without either is named after its key."""
    external = _external(spec)
    out = {"name": _scalar_str(spec.get("name") or ""), "external": external}
    if not external:
        return out
    ext = spec.get("external")
    ext_name = _scalar_str(ext.get("name") or "") if isinstance(ext, dict) else ""
    if ext_name:
        if out["name"]:
            raise ComposeError("%s %s: %s.external.name and %s.name conflict; only use %s.name"
                               % (kind, name, kind, kind, kind))
        if _version_ge(version, deprecated_from):
            log.warning("%s %s: %s.external.name is deprecated in favor of %s.name", kind, name, kind, kind)
        out["name"] = ext_name
    elif not out["name"]:
        out["name"] = name
    return out


@cu.command_memo("compose-v3", ComposeError, "Unable to load Compose file at path %s Error: %s")
def parse_v3(path):
    """Parse and load a v3 compose file -> normalized config dict (``ParseV3``,
    v3.go:93-121: every failure is ``Unable to load Compose file at path <p>
    Error: <%q of the cause>``, logged at debug level)."""
    try:
        text = common.read_text(path)
    except OSError as e:
        raise ComposeError(common.go_path_error(e, "open"))
    try:
        parsed = yamlio.load_v2(text)
    except yamlio.YAMLError as e:
        raise ComposeError(str(e))
    if not isinstance(parsed, dict):
        raise ComposeError("Top-level object must be a mapping")
    _check_string_keys(parsed, "")
    parsed = remove_non_existent_env_files(path, parsed)
    version = _version(parsed)      # schema.Version: read before interpolation
    _check_forbidden(parsed)
    env = cu.get_environment_variables()
    try:
        parsed = interpolate_v3(parsed, env.get)
    except InterpolationError as e:
        raise ComposeError(str(e))
    if version not in SUPPORTED_V3:   # schema.Validate: no schema for the version
        raise ComposeError("unsupported Compose file version: %s" % version)
    services = _validate(parsed)
    try:
        cschema.validate_v3(parsed)
    except cschema.SchemaError as e:
        raise ComposeError(str(e))
    wd = os.path.dirname(path)
    cfg = {"version": version, "services": [], "networks": {}, "volumes": parsed.get("volumes") or {},
           "secrets": {}, "configs": {}}
    # loadSections: services, networks, volumes, secrets, configs; the first error ends the load
    for sname in services:
        try:
            cfg["services"].append(_load_service(sname, services[sname] or {}, wd, env))
        except (ValueError, TypeError) as e:  # Transform / resolveEnvironment / resolveVolumePaths
            raise ComposeError(str(e)) from None
    for name, spec in (parsed.get("networks") or {}).items():
        cfg["networks"][name] = _external_name("network", name, spec or {}, version, "3.5")
    for name, spec in (parsed.get("volumes") or {}).items():
        spec = spec or {}
        if _external(spec):
            for key, present in (("driver", spec.get("driver")), ("driver_opts", spec.get("driver_opts")),
                                 ("labels", spec.get("labels"))):
                if present:
                    raise ComposeError('conflicting parameters "external" and %s specified for volume %s'
                                       % (go_quote(key), go_quote(name)))
        _external_name("volume", name, spec, version, "3.4")
    for kind in ("secrets", "configs"):
        for name, spec in (parsed.get(kind) or {}).items():
            spec = spec or {}
            obj = _external_name(kind[:-1], name, spec, version, "3.5")
            f = _scalar_str(spec.get("file") or "")
            cfg[kind][name] = {"file": f if obj["external"] else cu.go_abs_path(wd, f), "external": obj["external"],
                               "name": obj["name"]}
    cfg["services"].sort(key=lambda s: s["name"])
    return cfg


def _go_type_name(v):
    """``%T`` of a value go-yaml v2 decoded into interface{}."""
    if isinstance(v, bool):
        return "bool"
    return {int: "int", float: "float64", str: "string", list: "[]interface {}"}.get(
        type(v), "map[string]interface {}" if isinstance(v, dict) else "<nil>")


def _transform_ports(entries):
    """``transformServicePort`` over the list: the first bad entry's error."""
    out = []
    for p in entries:
        if isinstance(p, dict):
            out.append({"target": int(p.get("target") or 0), "published": int(p.get("published") or 0),
                        "protocol": _scalar_str(p.get("protocol") or ""), "mode": _scalar_str(p.get("mode") or "")})
        elif isinstance(p, (int, str)) and not isinstance(p, bool):
            for tgt, pub, proto, mode in cu.to_service_port_configs(str(p)):
                out.append({"target": tgt, "published": pub, "protocol": proto, "mode": mode})
        else:
            raise ValueError("invalid type %s for port" % _go_type_name(p))
    return out


def _transform(name, d):
    """The values docker/cli's ``Transform`` (mapstructure with the loader's
    transform hooks) can fail on, each under its field path; every failure is
    collected and the lot is one ``mapstructure.Error`` (``N error(s)
    decoding:`` and the sorted ``* error decoding '<path>': <cause>``
    lines)."""
    errs = []
    out = {"ports": [], "memory": {}, "volumes": []}
    if d.get("ports") is not None:
        try:
            out["ports"] = _transform_ports(d["ports"])
        except ValueError as e:
            errs.append("error decoding 'Ports': %s" % e)
    res = (d.get("deploy") or {}).get("resources") or {}
    for key in ("limits", "reservations"):
        r = res.get(key)
        if isinstance(r, dict) and r.get("memory") is not None:
            try:
                out["memory"][key] = cu.ram_in_bytes(r["memory"])
            except ValueError as e:
                errs.append("error decoding 'Deploy.Resources.%s.memory': %s" % (key.capitalize(), e))
    for i, v in enumerate(d.get("volumes") or []):
        if isinstance(v, dict):
            out["volumes"].append({"type": _scalar_str(v.get("type") or "volume"),
                                   "source": _scalar_str(v.get("source") or ""),
                                   "target": _scalar_str(v.get("target") or ""), "read_only": bool(v.get("read_only"))})
            continue
        try:
            if not isinstance(v, str):
                raise ValueError("invalid type %s for service volume" % _go_type_name(v))
            out["volumes"].append(cu.parse_volume_v3(v))
        except ValueError as e:
            errs.append("error decoding 'Volumes[%d]': %s" % (i, e))
    if errs:
        raise ComposeError("%d error(s) decoding:\n\n%s" % (len(errs), "\n".join(sorted("* " + e for e in errs))))
    return out


def _is_windows_abs(p):
    """docker/cli loader ``isAbs`` (windows_path.go): ``C:\\x`` / ``C:/x``, or a UNC path."""
    if len(p) >= 3 and p[0].isascii() and p[0].isalpha() and p[1] == ":" and p[2] in "\\/":
        return True
    return p.startswith("\\\\") or p.startswith("//")


def _resolve_volume_paths(vols, wd, env):
    """``resolveVolumePaths``: a bind mount needs a source; ``~`` is the
    environment's HOME (a warning when it has none); a relative source is
    joined to the compose file's directory."""
    for vol in vols:
        if vol["type"] != "bind":
            continue
        src = vol["source"]
        if src == "":
            raise ComposeError('invalid mount config for type "bind": field Source must not be empty')
        if src.startswith("~"):
            if "HOME" in env:
                src = src.replace("~", env["HOME"], 1)
            else:
                log.warning("cannot expand '~', because the environment lacks HOME")
        if not src.startswith("/") and not _is_windows_abs(src):
            src = cu.go_abs_path(wd, src)
        vol["source"] = src


def _load_service(name, d, wd, env):
    t = _transform(name, d)
    s = {"name": name}
    b = d.get("build")
    if isinstance(b, str):
        s["build_context"], s["build_dockerfile"] = b, ""
    elif isinstance(b, dict):
        s["build_context"] = _scalar_str(b.get("context") or "")
        s["build_dockerfile"] = _scalar_str(b.get("dockerfile") or "")
    else:
        s["build_context"], s["build_dockerfile"] = "", ""
    s["image"] = _scalar_str(d.get("image") or "")
    s["container_name"] = _scalar_str(d.get("container_name") or "")
    for key in ("command", "entrypoint"):
        v = d.get(key)
        s[key] = cu.shell_split(v) if isinstance(v, str) else (_as_list_of_str(v) if v is not None else None)
    s["working_dir"] = _scalar_str(d.get("working_dir") or "")
    s["stdin_open"] = bool(d.get("stdin_open"))
    s["tty"] = bool(d.get("tty"))
    s["hostname"] = _scalar_str(d.get("hostname") or "")
    s["domainname"] = _scalar_str(d.get("domainname") or "")
    s["pid"] = _scalar_str(d.get("pid") or "")
    s["privileged"] = bool(d.get("privileged"))
    s["user"] = _scalar_str(d.get("user") or "")
    s["cap_add"] = _as_list_of_str(d.get("cap_add"))
    s["cap_drop"] = _as_list_of_str(d.get("cap_drop"))
    s["labels"] = _labels(d.get("labels"))
    s["restart"] = _scalar_str(d.get("restart") or "")
    s["tmpfs"] = _as_list_of_str(d.get("tmpfs"))
    s["expose"] = _as_list_of_str(d.get("expose"))
    # ports
    s["ports"] = t["ports"]
    # environment: env_file contents first, then environment entries; bare keys from env
    environment = {}
    for ef in _as_list_of_str(d.get(cu.ENV_FILE)):
        p = ef if os.path.isabs(ef) else os.path.join(wd, ef)
        for k, v in _read_env_file(p).items():
            environment[k] = v
    for k, v in _mapping_with_equals(d.get("environment")).items():
        environment[k] = v
    # updateEnvironment: a key with no value or an empty one takes the loader's environment
    # ("lookupEnv is prioritized over the file content")
    for k, v in list(environment.items()):
        if (v is None or v == "") and k in env:
            environment[k] = env[k]
    s["environment"] = environment
    # networks
    nets = d.get("networks")
    s["networks"] = list(nets.keys()) if isinstance(nets, dict) else _as_list_of_str(nets)
    # deploy
    dep = d.get("deploy") or {}
    deploy = {"mode": _scalar_str(dep.get("mode") or ""), "replicas": dep.get("replicas"),
              "labels": _labels(dep.get("labels")), "limits": None, "reservations": None, "restart_condition": None}
    res = dep.get("resources") or {}
    for key in ("limits", "reservations"):
        r = res.get(key)
        if isinstance(r, dict):
            deploy[key] = {"cpus": _scalar_str(r.get("cpus")) if r.get("cpus") is not None else "",
                           "memory": t["memory"].get(key, 0)}
    rp = dep.get("restart_policy")
    if isinstance(rp, dict):
        deploy["restart_condition"] = _scalar_str(rp.get("condition") or "")
    s["deploy"] = deploy
    # healthcheck
    hc = d.get("healthcheck")
    if isinstance(hc, dict):
        test = hc.get("test")
        if isinstance(test, str):
            test = ["CMD-SHELL", test]
        s["healthcheck"] = {"test": _as_list_of_str(test), "disable": bool(hc.get("disable")),
                            "interval": hc.get("interval"), "timeout": hc.get("timeout"),
                            "retries": hc.get("retries"), "start_period": hc.get("start_period")}
    else:
        s["healthcheck"] = None
    # secrets / configs (short or long syntax)
    for key in ("secrets", "configs"):
        items = []
        for it in d.get(key) or []:
            if isinstance(it, dict):
                mode = it.get("mode")
                items.append({"source": _scalar_str(it.get("source") or ""), "target": _scalar_str(it.get("target") or ""),
                              "mode": int(mode) if mode is not None else None})
            else:
                items.append({"source": _scalar_str(it), "target": "", "mode": None})
        s[key] = items
    # volumes
    _resolve_volume_paths(t["volumes"], wd, env)
    s["volumes"] = t["volumes"]
    return s


class V3Loader:
    def convert_to_ir(self, composefilepath, plan, service):
        log.debug("About to load configuration from docker compose file at path %s", composefilepath)
        try:
            cfg = parse_v3(composefilepath)
        except ComposeError as e:
            log.warning("Error while loading docker compose config : %s", e)
            raise
        log.debug("About to start loading docker compose to intermediate rep")
        return self._convert(os.path.dirname(composefilepath), cfg, plan, service)

    def _convert(self, filedir, cfg, plan, service):
        from ...utils.constants import settings
        ir = irtypes.empty_ir()
        ir.storages = self.get_secret_storages(cfg["secrets"]) + self.get_config_storages(cfg["configs"])
        if not settings.fixed:
            # make([]Storage, len(n)) followed by append leaves n zero-value storages in front
            zeros = [irtypes.Storage() for _ in range(len(cfg["secrets"]))]
            zeros2 = [irtypes.Storage() for _ in range(len(cfg["configs"]))]
            secrets = ir.storages[:len(cfg["secrets"])]
            configs = ir.storages[len(cfg["secrets"]):]
            ir.storages = zeros + secrets + zeros2 + configs
        for cs in cfg["services"]:
            if cs["name"] != service.service_name:
                continue
            name = common.normalize_for_service_name(cs["name"])
            sc = irtypes.new_service_with_name(name)
            cont = {}
            cont["image"] = cs["image"] or name + ":latest"
            if cs["build_dockerfile"] or cs["build_context"]:
                try:
                    ir.add_container(ReuseDockerfileContainerizer().get_container(plan, service))
                except Exception as e:  # noqa: BLE001
                    log.warning("Unable to get containization script even though build parameters are present : %s", e)
            if cs["working_dir"]:
                cont["workingDir"] = cs["working_dir"]
            if cs["entrypoint"] is not None:
                cont["command"] = cs["entrypoint"]
            if cs["command"] is not None:
                cont["args"] = cs["command"]
            if cs["stdin_open"]:
                cont["stdin"] = True
            cont["name"] = common.go_lower(cs["container_name"]) or common.go_lower(sc.name)
            if cs["tty"]:
                cont["tty"] = True
            cont["ports"] = self.get_ports(cs["ports"], cs["expose"])
            self.add_ports(cs["ports"], cs["expose"], sc)
            sc.annotations = dict(cs["labels"]) if cs["labels"] else None
            merged = common.merge_string_maps(cs["labels"], cs["deploy"]["labels"])
            sc.labels = merged
            if cs["hostname"]:
                sc.pod_spec["hostname"] = cs["hostname"]
            if cs["domainname"]:
                sc.pod_spec["subdomain"] = cs["domainname"]
            if cs["pid"]:
                if cs["pid"] == "host":
                    sc.pod_spec["hostPID"] = True
                else:
                    log.warning("Ignoring PID key for service \"%s\". Invalid value \"%s\".", name, cs["pid"])
            secctx = {}
            if cs["privileged"]:
                secctx["privileged"] = True
            if cs["user"]:
                try:
                    secctx["runAsUser"] = common.cast_to_int(cs["user"])
                except ValueError:
                    log.warning("Ignoring user directive. User to be specified as a UID (numeric).")
            if cs["cap_add"] or cs["cap_drop"]:
                secctx["capabilities"] = {"add": list(cs["cap_add"]), "drop": list(cs["cap_drop"])}
            if secctx:
                cont["securityContext"] = secctx
            if cs["deploy"]["mode"] == "global":
                sc.daemon = True
            sc.networks = self.get_networks(cs, cfg)
            self._resources(cs["deploy"], cont)
            hc = cs["healthcheck"]
            if hc is not None and not hc["disable"]:
                try:
                    cont["livenessProbe"] = self.get_health_check(hc)
                except ValueError as e:
                    log.warning("Unable to parse health check : %s", e)
            restart = cs["restart"]
            if cs["deploy"]["restart_condition"] is not None:
                restart = cs["deploy"]["restart_condition"]
            if restart == "unless-stopped":
                log.warning("Restart policy 'unless-stopped' in service %s is not supported, convert it to 'always'", name)
                sc.restart_policy = "Always"
            if cs["deploy"]["replicas"] is not None:
                sc.replicas = int(cs["deploy"]["replicas"])
            env = self.get_envs(cs)
            if env:
                cont["env"] = env
            vms, vols = cu.make_volumes_from_tmpfs(name, cs["tmpfs"])
            for v in vols:
                sc.add_volume(v)
            mounts = list(vms)
            for sec in cs["secrets"]:
                target = common.go_join(cu.DEFAULT_SECRET_BASE_PATH, sec["source"])
                src = sec["source"]
                if sec["target"]:
                    tokens = sec["source"].split("/")
                    prefix = "" if sec["target"].startswith("/") else cu.DEFAULT_SECRET_BASE_PATH + "/"
                    if tokens[-1] == sec["target"]:
                        target = prefix + sec["source"]
                    else:
                        t = sec["target"]
                        suffix = "/" + tokens[-1]
                        target = prefix + (t[:-len(suffix)] if t.endswith(suffix) else t)
                    src = tokens[-1]
                vsrc = {"secretName": sec["source"], "items": [{"key": sec["source"], "path": src}]}
                if sec["mode"] is not None:
                    vsrc["defaultMode"] = int(sec["mode"])
                sc.add_volume({"name": sec["source"], "secret": vsrc})
                mounts.append({"name": sec["source"], "mountPath": target})
            for c in cs["configs"]:
                target = c["target"] or "/" + c["source"]
                vname = common.make_file_name_compliant(c["source"])
                vsrc = {"name": vname}
                o = cfg["configs"].get(c["source"])
                if o is not None:
                    if o["external"]:
                        log.error("Config metadata %s has an external source", c["source"])
                    else:
                        vsrc["items"] = [{"key": os.path.basename(o["file"]), "path": os.path.basename(target)}]
                        if c["mode"] is not None:
                            vsrc["defaultMode"] = int(c["mode"])
                else:
                    log.error("Unable to find configmap object for %s", vname)
                sc.add_volume({"name": vname, "configMap": vsrc})
                mounts.append({"name": vname, "mountPath": target, "subPath": os.path.basename(target)})
            for vol in cs["volumes"]:
                if cu.is_path(vol["source"]):
                    vname = "%s%d" % (VOLUME_PREFIX, cu.get_hash(vol["source"]))
                    mounts.append({"name": vname, "mountPath": vol["target"]})
                    sc.add_volume({"name": vname, "hostPath": {"path": vol["source"]}})
                else:
                    mounts.append({"name": vol["source"], "mountPath": vol["target"]})
                    sc.add_volume({"name": vol["source"], "persistentVolumeClaim": {"claimName": vol["source"]}})
                    ir.add_storage(irtypes.Storage(name=vol["source"], storage_type=irtypes.PVC_KIND))
            if mounts:
                cont["volumeMounts"] = mounts
            sc.containers = [cont]
            ir.services[name] = sc
        return ir

    @staticmethod
    def _resources(deploy, cont):
        res = {}
        for key, out in (("limits", "limits"), ("reservations", "requests")):
            r = deploy.get(key)
            if r is None:
                continue
            rl = {}
            if r["memory"]:
                rl["memory"] = cu.format_quantity_decimal_exponent(r["memory"])
            if r["cpus"] != "":
                try:
                    cpu = common.cast_to_float(r["cpus"])
                except ValueError as e:
                    log.warning("Unable to convert cpu limits %s value : %s",
                                "resources" if key == "limits" else "reservation", e)
                    cpu = 0.0
                milli = common.go_float_to_int64(cpu * 1000)
                if milli != 0:
                    rl["cpu"] = cu.format_milli_quantity(milli)
            res[out] = rl
        if res:
            cont["resources"] = res

    def get_secret_storages(self, secrets):
        out = []
        for name in sorted(secrets):
            obj = secrets[name]
            st = irtypes.Storage(name=name, storage_type=irtypes.SECRET_KIND)
            if not obj["external"]:
                try:
                    with open(obj["file"], "rb") as f:
                        st.content = {name: f.read()}
                except OSError:
                    log.warning("Could not read the secret file [%s]", obj["file"])
            out.append(st)
        return out

    def get_config_storages(self, configs):
        out = []
        for name in sorted(configs):
            obj = configs[name]
            st = irtypes.Storage(name=name, storage_type=irtypes.CONFIGMAP_KIND)
            if not obj["external"]:
                f = obj["file"]
                try:
                    is_dir = stat.S_ISDIR(os.stat(f).st_mode)
                except OSError as e:
                    log.warning("Could not identify the type of secret artifact [%s]. Encountered [%s]", f,
                                common.go_path_error(e, "stat"))
                else:
                    if not is_dir:
                        try:
                            with open(f, "rb") as fh:
                                st.content = {name: fh.read()}
                        except OSError as e:
                            log.warning("Could not read the secret file [%s]. Encountered [%s]", f,
                                        common.go_path_error(e, "open"))
                    else:
                        try:
                            st.content = self._dir_content_as_map(f)
                        except OSError as e:
                            log.warning("Could not read the secret directory [%s]. Encountered [%s]", f,
                                        common.go_path_error(e, "open"))
            out.append(st)
        return out

    @staticmethod
    def _dir_content_as_map(directory):
        """``getAllDirContentAsMap`` (v3.go:625-651): the directory's files by
        name (ioutil.ReadDir: sorted, lstat, so a symlink is read as a file)."""
        data = {}
        count = 0
        for entry in sorted(os.listdir(directory)):
            p = os.path.join(directory, entry)
            try:
                if stat.S_ISDIR(os.lstat(p).st_mode):
                    continue
            except OSError:
                continue
            log.debug("Reading file into the data map: [%s]", entry)
            try:
                with open(p, "rb") as fh:
                    data[entry] = fh.read()
            except OSError:
                log.debug("Unable to read file data : %s", entry)
                continue
            count += 1
        log.debug("Read %d files into the data map", count)
        return data

    @staticmethod
    def get_ports(ports, expose):
        out = []
        exist = set()
        for p in ports:
            proto = "UDP" if p["protocol"].lower() == "udp" else "TCP"
            out.append({"containerPort": p["target"], "protocol": proto})
            exist.add(str(p["target"]))
        for e in expose:
            val, proto = e, "TCP"
            if "/" in e:
                val, pr = e.split("/", 1)
                proto = pr.upper()
            if val in exist:
                continue
            try:
                n = common.cast_to_int(val)
            except ValueError:
                n = 0
            out.append({"containerPort": n, "protocol": proto})
        return out

    @staticmethod
    def add_ports(ports, expose, service):
        exist = set()
        for p in ports:
            service.add_port_forwarding(irtypes.Port(p["published"]), irtypes.Port(p["target"]))
            exist.add(str(p["target"]))
        for e in expose:
            val = e.split("/", 1)[0]
            if val in exist:
                continue
            try:
                n = common.cast_to_int(val)
            except ValueError:
                n = 0
            service.add_port_forwarding(irtypes.Port(n), irtypes.Port(n))

    @staticmethod
    def get_networks(cs, cfg):
        out = []
        for key in cs["networks"]:
            n = cfg["networks"].get(key, {}).get("name") or key
            out.append(n)
        return out

    @staticmethod
    def get_health_check(hc):
        probe = {}
        if len(hc["test"]) > 1:
            probe["exec"] = {"command": list(hc["test"][1:])}
        else:
            log.warning("Could not find command to execute in probe : %s", hc["test"])
        if hc["timeout"] is not None:
            probe["timeoutSeconds"] = cu.duration_seconds(cu.parse_duration(hc["timeout"]))
        if hc["interval"] is not None:
            probe["periodSeconds"] = cu.duration_seconds(cu.parse_duration(hc["interval"]))
        if hc["retries"] is not None:
            probe["failureThreshold"] = int(hc["retries"])
        if hc["start_period"] is not None:
            probe["initialDelaySeconds"] = cu.duration_seconds(cu.parse_duration(hc["start_period"]))
        return probe

    @staticmethod
    def get_envs(cs):
        out = []
        for name in sorted(cs["environment"]):
            v = cs["environment"][name]
            out.append({"name": name, "value": v if v is not None else "unknown"})
        return out
