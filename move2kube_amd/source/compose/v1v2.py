"""Compose file format v1/v2 loader (reference ``internal/source/compose/v1v2.go``).

Parsing mirrors libcompose's ``project.Parse()`` as the reference configures
it (``v1v2.go:93-129``): interpolation with ``.env`` (current directory) then
OS environment lookups, pruning of missing env_files (the Preprocess hook,
``v1v2.go:49-90``), schema validation (v1: every top-level key is a service;
v2: ``services``/``networks``/``volumes``), then per service libcompose's
``readEnvFile`` (env_file lines folded into ``environment``) and ``extends``
(same file or ``file:``, chained; lists appended, maps merged, scalars
replaced; ``links``/``volumes_from`` cannot be extended), and resolution of
build contexts and bind-volume sources relative to the file that declared
them.
"""

import os

from ...containerizer.reusedockerfile import ReuseDockerfileContainerizer
from ...models import ir as irtypes
from ...utils import common, log, yamlio
from ...utils.constants import VOLUME_PREFIX, settings
from ...utils.lazyre import lazy as _lazy_re
from . import schema as cschema
from . import utils as cu
from .interpolate import EnvFileError, InterpolationError, interpolate_v1v2, parse_env_file
from .v3 import ComposeError, _as_list_of_str, _labels, _scalar_str

V1_SERVICE_KEYS = {
    "build", "cap_add", "cap_drop", "cgroup_parent", "command", "container_name", "cpu_shares", "cpu_quota",
    "cpuset", "devices", "dns", "dns_search", "dockerfile", "domainname", "entrypoint", "env_file", "environment",
    "expose", "extends", "external_links", "extra_hosts", "hostname", "image", "ipc", "labels", "links",
    "log_driver", "log_opt", "mac_address", "mem_limit", "memswap_limit", "mem_swappiness", "net", "pid", "ports",
    "privileged", "read_only", "restart", "security_opt", "shm_size", "stdin_open", "stop_signal", "tty",
    "ulimits", "user", "volumes", "volume_driver", "volumes_from", "working_dir", "group_add", "tmpfs",
    "stop_grace_period", "oom_score_adj", "cpus",
}
V2_SERVICE_KEYS = V1_SERVICE_KEYS - {"dockerfile", "log_driver", "log_opt", "net"} | {
    "depends_on", "logging", "network_mode", "networks", "isolation", "healthcheck", "init", "sysctls",
    "userns_mode", "pids_limit", "runtime", "storage_opt", "mem_reservation", "blkio_config", "cpu_count",
    "cpu_percent", "cpu_period", "cpu_rt_period", "cpu_rt_runtime", "device_cgroup_rules", "scale"}
V2_TOP_KEYS = {"version", "services", "networks", "volumes"}
SUPPORTED_V2 = {"2", "2.0", "2.1"}


def _normalize_project_name(s):
    # re.sub(r"[^a-z0-9]", "", strings.ToLower(s))
    return "".join(c for c in common.go_lower(s) if "a" <= c <= "z" or "0" <= c <= "9")


def _read_raw(path):
    """``CreateConfig``: the raw document -> (version, raw services, parsed)."""
    try:
        text = common.read_text(path)
    except OSError as e:
        raise ComposeError(common.go_path_error(e, "open"))
    try:
        parsed = yamlio.load_v2(text)
    except yamlio.YAMLError as e:
        raise ComposeError(str(e))
    if parsed is None:
        raise ComposeError("empty file %s" % path)
    if not isinstance(parsed, dict):
        raise ComposeError("top-level object of %s must be a mapping" % path)
    version = parsed.get("version")
    if version is not None:
        if isinstance(version, float):
            version = yamlio.go_format_float(version)
        version = str(version)
        if version not in SUPPORTED_V2:
            raise ComposeError("Unsupported config version %s" % version)
        unknown = [k for k in parsed if k not in V2_TOP_KEYS]
        if unknown:
            raise ComposeError("Additional property %s is not allowed" % unknown[0])
        raw_services = parsed.get("services") or {}
        if not isinstance(raw_services, dict):
            raise ComposeError("services must be a mapping")
    else:
        version = ""
        raw_services = parsed
    return version, raw_services, parsed


def _env_lookup():
    """libcompose ``ComposableEnvLookup``: ``.env`` of the working directory,
    then the OS environment (``v1v2.go:98-112``)."""
    env_path = ".env" if settings.ignore_environment else os.path.abspath(".env")
    dotenv = {}
    if os.path.isfile(env_path):
        try:
            dotenv = parse_env_file(env_path, first_wins=True)
        except (OSError, EnvFileError):   # libcompose EnvfileLookup: an unparsable .env is empty
            dotenv = {}

    def lookup(k):
        if k in dotenv:
            return dotenv[k]
        return os.environ.get(k) or None    # OsEnvLookup: an empty variable is not found
    return lookup


def _lc_defaults():
    """libcompose's package-level ``defaultValues``: one map for the whole
    command (the reference's process), shared by every file it parses."""
    from ...utils import fsindex
    d = fsindex.scoped_cache("libcompose-defaults")
    return d if d is not None else {}


class _DefaultsState:
    """What the compose-file memo keys on and replays: a file parsed again
    with other defaults in force parses differently, and its parse records
    its own defaults."""

    @staticmethod
    def snapshot():
        return tuple(sorted(_lc_defaults().items()))

    @staticmethod
    def restore(snap):
        d = _lc_defaults()
        d.clear()
        d.update(snap)


def _prune_env_files(raw_services, compose_path):
    """``removeNonExistentEnvFilesV2`` (``v1v2.go:49-90``), the Preprocess hook.
    Paths are checked against the directory of the compose file the reference
    passed in - also for services of a file pulled in through ``extends``."""
    base = os.path.dirname(os.path.abspath(compose_path))
    for name, svc in raw_services.items():
        if not isinstance(svc, dict) or cu.ENV_FILE not in svc:
            continue
        ef = svc[cu.ENV_FILE]
        if isinstance(ef, str):
            p = ef if os.path.isabs(ef) else os.path.join(base, ef)
            if not os.path.isfile(p):
                log.warning("Unable to find env config file %s referred in service %s in file %s. Ignoring it.",
                            p, name, compose_path)
                del svc[cu.ENV_FILE]
        elif isinstance(ef, list):
            kept = []
            for e in ef:
                if not isinstance(e, str):
                    continue
                p = e if os.path.isabs(e) else os.path.join(base, e)
                if os.path.isfile(p):
                    kept.append(e)
                else:
                    log.warning("Unable to find env config file %s referred in service %s in file %s. Ignoring it.",
                                p, name, compose_path)
            svc[cu.ENV_FILE] = kept


# libcompose's dockerConfigHints (config/validation.go), after docker-compose's
_CONFIG_HINTS = {"cpu_share": "cpu_shares", "add_host": "extra_hosts", "hosts": "extra_hosts",
                 "extra_host": "extra_hosts", "device": "devices", "link": "links", "memory_swap": "memswap_limit",
                 "port": "ports", "privilege": "privileged", "priviliged": "privileged", "privilige": "privileged",
                 "volume": "volumes", "workdir": "working_dir"}
_SERVICE_NAME_RE = _lazy_re(r"^[a-zA-Z0-9._-]+\Z")


def _validate(raw_services, version):
    allowed = V2_SERVICE_KEYS if version else V1_SERVICE_KEYS
    for name, svc in raw_services.items():
        if not isinstance(name, str):
            raise ComposeError("Non-string service name %r" % (name,))
        # the services schema: patternProperties ^[a-zA-Z0-9._-]+$, additionalProperties
        # false; libcompose words it as an unsupported option of the "(root)" service
        if not _SERVICE_NAME_RE.match(name):
            raise ComposeError("Unsupported config option for (root) service: '%s'" % name)
        if not isinstance(svc, dict):
            raise ComposeError("Service %s has neither an image nor a build context specified" % name
                               if svc is None else "Invalid type for service %s" % name)
        for k in svc:
            if k not in allowed:
                hint = _CONFIG_HINTS.get(k)
                raise ComposeError("Unsupported config option for %s service: '%s'" % (name, k)
                                   + (" (did you mean '%s'?)" % hint if hint else ""))
        try:
            cschema.validate_v2_service(name, svc)
        except cschema.SchemaError as e:
            raise ComposeError("Service %s configuration is invalid: %s" % (name, e))
        if version == "" and "extends" not in svc:
            has_build = "build" in svc or "dockerfile" in svc
            if ("image" in svc) == ("build" in svc) or ("image" in svc and has_build):
                raise ComposeError("Service %s has neither an image nor a build context specified. "
                                   "At least one must be provided." % name)


def _load_file(path, lookup, compose_path):
    """Interpolate -> Preprocess -> Validate, as libcompose's ``Merge`` /
    ``parseV2`` does for the main file and for every ``extends: {file: ...}``."""
    version, raw_services, parsed = _read_raw(path)
    try:
        raw_services = interpolate_v1v2(raw_services, lookup, _lc_defaults())
    except InterpolationError as e:
        raise ComposeError(str(e))
    _prune_env_files(raw_services, compose_path)
    _validate(raw_services, version)
    return version, raw_services, parsed


class _EnvSlice(tuple):
    """libcompose ``MaporEqualSlice``: ``environment`` after ``readEnvFile``.
    A typed slice, so ``merge`` (which only appends ``[]interface{}``) replaces it."""


def _environment_slice(env):
    if isinstance(env, dict):
        return ["%s=%s" % (k, _scalar_str(v)) if v is not None else str(k) for k, v in env.items()]
    return _as_list_of_str(env)


def _read_env_file(svc, in_file):
    """libcompose ``readEnvFile``: fold ``env_file`` into ``environment``.
    Files are read last to first; a line is added unless an existing entry
    starts with its key (the text up to and including the first ``=``), so
    explicit ``environment`` entries win, then later files over earlier ones.
    Lines are taken verbatim (trimmed; blank and ``#`` lines skipped)."""
    if cu.ENV_FILE not in svc:
        return svc
    ef = svc[cu.ENV_FILE]
    files = [ef] if isinstance(ef, str) else [e for e in (ef or []) if isinstance(e, str)]
    if not files:
        return svc
    env = _environment_slice(svc.get("environment")) if "environment" in svc else []
    for f in reversed(files):
        p = f
        if p.startswith("~/"):
            p = os.environ.get("HOME", "") + p[1:]
        if not os.path.isabs(p):
            p = os.path.join(os.path.dirname(in_file), p)
        try:
            with open(p, encoding="utf-8", errors="replace") as fh:
                lines = fh.read().splitlines()
        except OSError as e:
            raise ComposeError("Failed to read env file %s: %s" % (p, e))
        for raw in lines:
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            key = line[:line.index("=") + 1] if "=" in line else line
            if not any(v.startswith(key) for v in env):
                env.append(line)
    svc["environment"] = _EnvSlice(env)
    del svc[cu.ENV_FILE]
    return svc


def _merge_value(existing, value):
    """libcompose ``merge``: raw lists append, raw maps merge, anything else is replaced."""
    if type(existing) is list and type(value) is list:
        return existing + value
    if isinstance(existing, dict) and isinstance(value, dict):
        out = dict(existing)
        out.update(value)
        return out
    return value


_NO_MERGE = ("links", "volumes_from")


def _parse_service(svc, in_file, datas, lookup, compose_path, depth=0):
    """libcompose ``parseV1``/``parseV2``: env files, then ``extends``.
    Returns the raw service with ``_file`` naming the file each path-like value
    is relative to (the extended service's own file for inherited keys)."""
    if depth > 32:
        raise ComposeError("extends: circular or too deep reference in %s" % in_file)
    svc = _read_env_file(dict(svc), in_file)
    svc.setdefault("_file", {})
    svc["_file"] = dict(svc["_file"])
    for k in svc:
        if k != "_file" and k not in svc["_file"]:
            svc["_file"][k] = in_file
    ext = svc.get("extends")
    if not isinstance(ext, dict):
        return svc
    file = _scalar_str(ext.get("file") or "")
    service = _scalar_str(ext.get("service") or "")
    if not service:
        return svc
    if not file:
        if service not in datas:
            raise ComposeError("Failed to find service %s to extend" % service)
        base = _parse_service(datas[service], in_file, datas, lookup, compose_path, depth + 1)
    else:
        if file.startswith("~/"):
            file = os.environ.get("HOME", "") + file[1:]
        resolved = file if os.path.isabs(file) else os.path.join(os.path.dirname(in_file), file)
        _v, base_services, _p = _load_file(resolved, lookup, compose_path)
        if service not in base_services:
            raise ComposeError("Failed to find service %s in file %s" % (service, file))
        base = _parse_service(base_services[service], resolved, base_services, lookup, compose_path, depth + 1)
    for k in _NO_MERGE:
        if k in base:
            raise ComposeError("Cannot extend service '%s' in %s: services with '%s' cannot be extended"
                               % (service, file or in_file, k))
    merged = dict(base)
    files = dict(base["_file"])
    for k, v in svc.items():
        if k == "_file":
            continue
        merged[k] = _merge_value(merged[k], v) if k in merged else v
        if not (k in base and type(base[k]) is list and type(v) is list):
            files[k] = svc["_file"].get(k, in_file)
    merged["_file"] = files
    return merged


@cu.command_memo("compose-v1v2", ComposeError, "Failed to load docker compose file at path %s Error: %s",
                  state=_DefaultsState)
def parse_v2(path):
    """Parse a v1/v2 compose file the way the reference's libcompose
    ``project.Parse()`` does (``v1v2.go:93-129``): interpolation (``.env`` then
    OS env), env-file pruning, validation, then per service ``env_file``
    folding and ``extends`` resolution (same file or ``file:``, chained).
    The reference sets logrus to FatalLevel around ``Parse`` (v1v2.go:118-121),
    so nothing logged in here - libcompose's warnings, the env-file pruning's
    own - is shown.
    Returns {"version", "project", "services": [...], "networks": {...}}."""
    with log.hold():        # dropped: FatalLevel
        return _parse_v2(path)


def _parse_v2(path):
    lookup = _env_lookup()
    version, raw_services, parsed = _load_file(path, lookup, path)
    base = os.path.dirname(os.path.abspath(path))
    services = []
    for name, svc in raw_services.items():
        merged = _parse_service(svc, os.path.abspath(path), raw_services, lookup, path)
        try:
            services.append(_load_service(name, merged, base, version))
        except (ValueError, TypeError) as e:  # utils.Convert's yaml decode: MemStringorInt's RAMInBytes
            raise ComposeError(str(e)) from None
    services.sort(key=lambda s: s["name"])
    networks = {}
    project = _project_name(base)
    if version:
        nets = parsed.get("networks") or {}
        if not isinstance(nets, dict):
            raise ComposeError("networks must be a mapping")
        for nname, spec in nets.items():
            spec = spec if isinstance(spec, dict) else {}
            ext = spec.get("external")
            external = bool(ext) if not isinstance(ext, dict) else True
            real = nname
            if external and isinstance(ext, dict) and ext.get("name"):
                real = ext["name"]
            networks[nname] = {"external": external, "real": real}
        _consolidate_volume_names(parsed.get("volumes"), services, project)
    return {"version": version, "project": project, "services": services, "networks": networks}


def _project_name(base):
    """libcompose ``lookupProjectName`` + ``normalizeName``: ``COMPOSE_PROJECT_NAME``,
    else the compose file's directory name; lower-cased, ``[^a-z0-9]`` dropped."""
    return _normalize_project_name(os.environ.get("COMPOSE_PROJECT_NAME") or os.path.basename(base))


def _consolidate_volume_names(vols, services, project):
    """libcompose ``Project.handleVolumeConfig``: a named volume declared in the
    top-level ``volumes:`` becomes ``<project>_<name>``, or its ``external.name``
    when external; a declaration without a body (``name:``) is left alone.
    Parity unpinned: this follows libcompose's project loader, which is not in
    the reference tree (tests/golden/reference/DEVIATIONS.md §4)."""
    if not isinstance(vols, dict):
        return
    renames = {}
    for vname, spec in vols.items():
        if not isinstance(spec, dict):
            continue
        ext = spec.get("external")
        if ext:
            if isinstance(ext, dict) and ext.get("name"):
                renames[vname] = _scalar_str(ext["name"])
        else:
            renames[vname] = "%s_%s" % (project, vname)
    for s in services:
        for v in s["volumes"]:
            src = v["source"]
            if src and src[0] not in "./~" and src in renames:
                v["source"] = renames[src]


def _resolve(p, base):
    if p.startswith("~"):
        p = os.path.expanduser("~") + p[1:]
    if os.path.isabs(p):
        return p
    return os.path.normpath(os.path.join(base, p))


def _is_url(s):
    # ^(https?://|git://|github\.com/|git@)
    return s.startswith(("http://", "https://", "git://", "github.com/", "git@"))


def _load_service(name, d, base, version):
    files = d.get("_file") or {}

    def base_of(key):
        f = files.get(key)
        return os.path.dirname(f) if f else base
    s = {"name": name}
    b = d.get("build")
    ctx, dockerfile = "", ""
    if isinstance(b, str):
        ctx = b
    elif isinstance(b, dict):
        ctx = _scalar_str(b.get("context") or "")
        dockerfile = _scalar_str(b.get("dockerfile") or "")
    if version == "" and d.get("dockerfile"):
        dockerfile = _scalar_str(d.get("dockerfile"))
    if ctx and not _is_url(ctx):
        ctx = _resolve(ctx, base_of("build"))
    s["build_context"], s["build_dockerfile"] = ctx, dockerfile
    s["image"] = _scalar_str(d.get("image") or "")
    s["container_name"] = _scalar_str(d.get("container_name") or "")
    for key in ("command", "entrypoint"):
        v = d.get(key)
        s[key] = cu.shell_split(v) if isinstance(v, str) else (_as_list_of_str(v) if v is not None else None)
    env = d.get("environment")
    if isinstance(env, dict):
        s["environment"] = ["%s=%s" % (k, _scalar_str(v)) if v is not None else str(k) for k, v in env.items()]
    else:
        s["environment"] = _as_list_of_str(env)
    s["working_dir"] = _scalar_str(d.get("working_dir") or "")
    s["stdin_open"] = bool(d.get("stdin_open"))
    s["tty"] = bool(d.get("tty"))
    s["ports"] = _as_list_of_str(d.get("ports"))
    s["expose"] = _as_list_of_str(d.get("expose"))
    s["privileged"] = bool(d.get("privileged"))
    s["user"] = _scalar_str(d.get("user") or "")
    s["cap_add"] = _as_list_of_str(d.get("cap_add"))
    s["cap_drop"] = _as_list_of_str(d.get("cap_drop"))
    s["group_add"] = _as_list_of_str(d.get("group_add"))
    s["stop_grace_period"] = _scalar_str(d.get("stop_grace_period") or "")
    mem = d.get("mem_limit")
    # MemStringorInt: an int, else the scalar's text through RAMInBytes ("" fails)
    s["mem_limit"] = cu.ram_in_bytes(mem) if mem is not None else 0
    s["restart"] = _scalar_str(d.get("restart") or "")
    s["labels"] = _labels(d.get("labels"))
    s["hostname"] = _scalar_str(d.get("hostname") or "")
    s["domainname"] = _scalar_str(d.get("domainname") or "")
    nets = d.get("networks")
    s["networks"] = list(nets.keys()) if isinstance(nets, dict) else _as_list_of_str(nets)
    s["tmpfs"] = _as_list_of_str(d.get("tmpfs"))
    s["volumes_from"] = _as_list_of_str(d.get("volumes_from"))
    vols = []
    for v in d.get("volumes") or []:
        spec = _scalar_str(v) if not isinstance(v, dict) else ""
        parts = spec.split(":")
        vol = {"source": "", "destination": "", "access_mode": ""}
        if len(parts) == 1:
            vol["destination"] = parts[0]
        else:
            vol["source"], vol["destination"] = parts[0], parts[1]
            if len(parts) > 2:
                vol["access_mode"] = parts[2]
        src = vol["source"]
        if src and src[0] in "./~":
            vol["source"] = _resolve(src, base_of("volumes"))
        vols.append(vol)
    s["volumes"] = vols
    return s


class V1V2Loader:
    def convert_to_ir(self, composefilepath, plan, service):
        proj = parse_v2(composefilepath)
        return self._convert(os.path.dirname(composefilepath), proj, plan, service)

    def _convert(self, filedir, proj, plan, service):
        ir = irtypes.empty_ir()
        for cs in proj["services"]:
            name = cs["name"]
            if name != service.service_name:
                continue
            sc = irtypes.new_service_with_name(common.normalize_for_service_name(name))
            sc.annotations = dict(cs["labels"]) if cs["labels"] else None
            if cs["hostname"]:
                sc.pod_spec["hostname"] = cs["hostname"]
            if cs["domainname"]:
                sc.pod_spec["subdomain"] = cs["domainname"]
            cont = {"image": cs["image"] or name + ":latest"}
            if cs["build_dockerfile"] or cs["build_context"]:
                try:
                    ir.add_container(ReuseDockerfileContainerizer().get_container(plan, service))
                except Exception as e:  # noqa: BLE001
                    log.warning("Unable to get containization script even though build parameters are present : %s", e)
            cname = common.go_lower(cs["container_name"])
            if cname != cs["container_name"]:
                log.debug("Container name in service %r has been changed from %r to %r", name, cs["container_name"], cname)
            cont["name"] = cname or sc.name
            if cs["entrypoint"] is not None:
                cont["command"] = cs["entrypoint"]
            if cs["command"] is not None:
                cont["args"] = cs["command"]
            env = self.get_envs(cs["environment"])
            if env:
                cont["env"] = env
            if cs["working_dir"]:
                cont["workingDir"] = cs["working_dir"]
            if cs["stdin_open"]:
                cont["stdin"] = True
            if cs["tty"]:
                cont["tty"] = True
            cont["ports"] = self.get_ports(cs["ports"], cs["expose"])
            self.add_ports(cs["ports"], cs["expose"], sc)
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
            # group_add goes to a pod security context the reference never attaches (kept for parity)
            try:    # getGroupAdd (v1v2.go:448-459)
                for g in cs["group_add"]:
                    common.cast_to_int(g)
            except ValueError as e:
                log.warning("GroupAdd should be in gid format, not as group name : unable to get group_add: %s", e)
            if cs["stop_grace_period"]:
                try:
                    sc.pod_spec["terminationGracePeriodSeconds"] = cu.duration_seconds(cu.parse_duration(cs["stop_grace_period"]))
                except ValueError:
                    log.warning("Failed to parse duration %s for service %s", cs["stop_grace_period"], name)
            if cs["mem_limit"]:
                cont["resources"] = {"limits": {"memory": cu.format_quantity_decimal_exponent(cs["mem_limit"])}}
            if cs["restart"] == "unless-stopped":
                log.warning("Restart policy 'unless-stopped' in service %s is not supported, convert it to 'always'", name)
                sc.restart_policy = "Always"
            for n in cs["networks"]:
                if n != "default":
                    net = proj["networks"].get(n)
                    if net is None:
                        real = proj["project"] + "_" + n
                    elif net["external"]:
                        real = net["real"]
                    else:
                        real = proj["project"] + "_" + n
                    sc.networks.append(real)
            vms, vols = cu.make_volumes_from_tmpfs(name, cs["tmpfs"])
            for v in vols:
                sc.add_volume(v)
            mounts = list(vms)
            if cs["volumes_from"]:
                log.warning("Ignoring VolumeFrom in compose for service %s : %s", service.service_name, cs["volumes_from"])
            for vol in cs["volumes"]:
                ro = vol["access_mode"] == cu.MODE_READ_ONLY
                if cu.is_path(vol["source"]):
                    vname = "%s%d" % (VOLUME_PREFIX, cu.get_hash(vol["source"]))
                    m = {"name": vname, "mountPath": vol["destination"]}
                    if ro:
                        m["readOnly"] = True
                    mounts.append(m)
                    sc.add_volume({"name": vname, "hostPath": {"path": vol["source"]}})
                else:
                    m = {"name": vol["source"], "mountPath": vol["destination"]}
                    if ro:
                        m["readOnly"] = True
                    mounts.append(m)
                    pvc = {"claimName": vol["source"]}
                    if ro:
                        pvc["readOnly"] = True
                    sc.add_volume({"name": vol["source"], "persistentVolumeClaim": pvc})
                    mode = "ReadOnlyMany" if ro else "ReadWriteMany"
                    ir.add_storage(irtypes.Storage(name=vol["source"], storage_type=irtypes.PVC_KIND,
                                                   pvc_spec={"accessModes": [mode]}))
            if mounts:
                cont["volumeMounts"] = mounts
            sc.containers = [cont]
            ir.services[name] = sc
        return ir

    @staticmethod
    def get_envs(envars):
        out = []
        for e in envars:
            i = min((j for j in (e.find("="), e.find(":")) if j >= 0), default=-1)  # [=:]
            if i < 0:
                out.append({"name": e, "value": "unknown"})
            else:
                out.append({"name": e[:i], "value": e[i + 1:]})
        return out

    @staticmethod
    def parse_container_port(value):
        proto = "TCP"
        if "/" in value:
            parts = value.split("/")
            value = parts[0]
            if parts[1].upper() == "UDP":
                proto = "UDP"
        if ":" not in value:
            p = common.cast_to_int(value)
            return p, p, proto
        parts = value.split(":")
        if len(parts) > 3:
            raise ValueError("Failed to parse the port %s properly" % value)
        sp, pp = parts[0], parts[1]
        if len(parts) == 3:
            sp, pp = parts[1], parts[2]
        return common.cast_to_int(sp), common.cast_to_int(pp), proto

    def get_ports(self, ports, expose):
        out, exist = [], set()
        for p in list(ports) + list(expose):
            try:
                _, pod, proto = self.parse_container_port(p)
            except ValueError:
                continue
            if pod not in exist:
                out.append({"containerPort": pod, "protocol": proto})
                exist.add(pod)
        return out

    def add_ports(self, ports, expose, service):
        exist = set()
        for p in list(ports) + list(expose):
            try:
                sp, pp, _ = self.parse_container_port(p)
            except ValueError:
                continue
            if sp not in exist:
                service.add_port_forwarding(irtypes.Port(sp), irtypes.Port(pp))
                exist.add(sp)
