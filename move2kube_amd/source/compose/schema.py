"""Type validation of compose files before loading.

The reference's loaders validate a compose document against the compose JSON
schema before converting it: docker/cli's v3 loader
(``cli/compose/schema/data/config_schema_v3.x.json`` via gojsonschema, called
from ``loader.Load`` after interpolation - ``internal/source/compose/v3.go:78-90``)
and libcompose for v1/v2 (``config_schema_v1.json`` / ``config_schema_v2.0.json``,
``internal/source/compose/v1v2.go:96-130``).  A document with a wrongly typed
value (``ports: 80``, ``environment: 5``, ``healthcheck: []``) is rejected as a
whole and Compose2Kube skips the file.

This module checks the value *types* of every key the loaders read, with
docker/cli's error wording (``services.web.ports must be a list``).  Where
the schema is stricter than what the loaders need (formats, patterns,
``uniqueItems``, additionalProperties below the service level) it is not
enforced: the check only guarantees that the loaders never see a value of a
type they cannot convert.
"""


class SchemaError(ValueError):
    pass


# -- type spec DSL --------------------------------------------------------------
#  "string" "integer" "number" "boolean" "null"   JSON scalar types
#  ("or", a, b, ...)                                one of the alternatives
#  ("list", item)                                   array of item
#  ("map", value)                                   mapping with any keys
#  ("obj", {key: spec})                             mapping, known keys typed
#  ("format", "duration")                           a string time.ParseDuration takes

STR, INT, NUM, BOOL, NULL = "string", "integer", "number", "boolean", "null"


def _or(*specs):
    return ("or",) + specs


def _list(item):
    return ("list", item)


def _map(value):
    return ("map", value)


def _obj(**props):
    return ("obj", props)


LIST_OF_STR = _list(STR)
STR_OR_LIST = _or(STR, LIST_OF_STR)
LIST_OR_DICT = _or(_map(_or(STR, NUM, BOOL, NULL)), LIST_OF_STR)
STR_OR_NUM = _or(STR, NUM)
EXTERNAL = _or(BOOL, _obj(name=STR))
# docker/cli schema.go registers a "duration" format checker (time.ParseDuration);
# the 3.x schemas put it on every duration-typed string
DURATION = ("format", "duration")

_BUILD = _or(STR, _obj(context=STR, dockerfile=STR, args=LIST_OR_DICT, labels=LIST_OR_DICT,
                       cache_from=LIST_OF_STR, network=STR, target=STR, shm_size=STR_OR_NUM,
                       extra_hosts=LIST_OR_DICT, isolation=STR))
_FILE_REF = _list(_or(STR, _obj(source=STR, target=STR, uid=STR, gid=STR, mode=NUM)))
_RESOURCE = _obj(cpus=STR_OR_NUM, memory=STR_OR_NUM, generic_resources=_list(_map(_or(STR, NUM, _map(_or(STR, NUM))))))
_UPDATE = _obj(parallelism=INT, delay=DURATION, failure_action=STR, monitor=DURATION, max_failure_ratio=NUM, order=STR)
_DEPLOY = _obj(
    mode=STR, endpoint_mode=STR, replicas=INT, labels=LIST_OR_DICT, rollback_config=_UPDATE, update_config=_UPDATE,
    resources=_obj(limits=_RESOURCE, reservations=_RESOURCE),
    restart_policy=_obj(condition=STR, delay=DURATION, max_attempts=INT, window=DURATION),
    placement=_obj(constraints=LIST_OF_STR, preferences=_list(_obj(spread=STR)), max_replicas_per_node=INT))
_HEALTHCHECK = _obj(disable=BOOL, interval=STR, retries=NUM, test=STR_OR_LIST, timeout=STR, start_period=STR)
_V3_HEALTHCHECK = _obj(disable=BOOL, interval=DURATION, retries=NUM, test=STR_OR_LIST, timeout=DURATION,
                       start_period=DURATION)
_PORTS = _list(_or(NUM, STR, _obj(mode=STR, host_ip=STR, target=INT, published=_or(STR, INT), protocol=STR)))
_VOLUMES = _list(_or(STR, _obj(type=STR, source=STR, target=STR, read_only=BOOL, consistency=STR,
                              bind=_obj(propagation=STR), volume=_obj(nocopy=BOOL),
                              tmpfs=_obj(size=_or(INT, STR)))))
_NETWORKS = _or(LIST_OF_STR, _map(_or(NULL, _obj(aliases=LIST_OF_STR, ipv4_address=STR, ipv6_address=STR,
                                                  priority=NUM))))
_ULIMITS = _map(_or(INT, _obj(hard=INT, soft=INT)))
_LOGGING = _obj(driver=STR, options=_map(_or(STR, NUM, NULL)))

_COMMON_SERVICE = dict(
    build=_BUILD, cap_add=LIST_OF_STR, cap_drop=LIST_OF_STR, cgroup_parent=STR, command=STR_OR_LIST,
    container_name=STR, devices=LIST_OF_STR, dns=STR_OR_LIST, dns_search=STR_OR_LIST, domainname=STR,
    entrypoint=STR_OR_LIST, env_file=STR_OR_LIST, environment=LIST_OR_DICT, expose=_list(_or(STR, NUM)),
    external_links=LIST_OF_STR, extra_hosts=LIST_OR_DICT, hostname=STR, image=STR, ipc=STR, labels=LIST_OR_DICT,
    links=LIST_OF_STR, mac_address=STR, network_mode=STR, networks=_NETWORKS, pid=_or(STR, NULL),
    ports=_PORTS, privileged=BOOL, read_only=BOOL, restart=STR, security_opt=LIST_OF_STR, shm_size=STR_OR_NUM,
    stdin_open=BOOL, stop_signal=STR, tmpfs=STR_OR_LIST, tty=BOOL, ulimits=_ULIMITS, user=STR, working_dir=STR,
    volumes=_VOLUMES, logging=_LOGGING, healthcheck=_HEALTHCHECK)

V3_SERVICE = _obj(**dict(
    _COMMON_SERVICE, configs=_FILE_REF, secrets=_FILE_REF, credential_spec=_obj(file=STR, registry=STR, config=STR),
    depends_on=LIST_OF_STR, deploy=_DEPLOY, init=BOOL, isolation=STR, stop_grace_period=DURATION,
    sysctls=LIST_OR_DICT, userns_mode=STR, healthcheck=_V3_HEALTHCHECK))

_TOP_VOLUME = _or(NULL, _obj(name=STR, driver=STR, driver_opts=_map(STR_OR_NUM), external=EXTERNAL,
                             labels=LIST_OR_DICT))
_TOP_NETWORK = _or(NULL, _obj(name=STR, driver=STR, driver_opts=_map(STR_OR_NUM), external=EXTERNAL,
                              internal=BOOL, attachable=BOOL, labels=LIST_OR_DICT,
                              ipam=_obj(driver=STR, config=_list(_map(_or(STR, NUM, NULL))))))
_TOP_FILE = _or(NULL, _obj(name=STR, file=STR, external=EXTERNAL, labels=LIST_OR_DICT, template_driver=STR))

V3_TOP = _obj(version=_or(STR, NUM), services=_or(NULL, _map(V3_SERVICE)),
              volumes=_or(NULL, _map(_TOP_VOLUME)), networks=_or(NULL, _map(_TOP_NETWORK)),
              secrets=_or(NULL, _map(_TOP_FILE)), configs=_or(NULL, _map(_TOP_FILE)))

# libcompose v1/v2 service keys (config_schema_v1.json / config_schema_v2.0.json)
V2_SERVICE = _obj(**dict(
    _COMMON_SERVICE, cpu_shares=STR_OR_NUM, cpu_quota=STR_OR_NUM, cpuset=STR, cpu_period=STR_OR_NUM,
    depends_on=LIST_OF_STR, dockerfile=STR, extends=_or(STR, _obj(service=STR, file=STR)), log_driver=STR,
    log_opt=_map(_or(STR, NUM, NULL)), mem_limit=STR_OR_NUM, memswap_limit=STR_OR_NUM, mem_reservation=STR_OR_NUM,
    mem_swappiness=INT, net=STR, oom_score_adj=INT, group_add=_list(STR_OR_NUM), stop_grace_period=STR,
    volume_driver=STR, volumes_from=LIST_OF_STR, oom_kill_disable=BOOL, userns_mode=STR, isolation=STR))


# -- validation ---------------------------------------------------------------

def _human(t):
    return {"obj": "mapping", "map": "mapping", "list": "list"}.get(t, t)


def _type_name(spec):
    if isinstance(spec, str):
        return spec
    if spec[0] == "or":
        names = []
        for s in spec[1:]:
            n = _human(_type_name(s))
            if n not in names:
                names.append(n)
        return names[0] if len(names) == 1 else ", ".join(names[:-1]) + " or " + names[-1]
    return _human(spec[0])


def _matches_scalar(v, t):
    if t == STR:
        return isinstance(v, str)
    if t == BOOL:
        return isinstance(v, bool)
    if t == NULL:
        return v is None
    if isinstance(v, bool):
        return False
    if t == NUM:
        return isinstance(v, (int, float))
    if t == INT:
        return isinstance(v, int) or (isinstance(v, float) and v.is_integer())
    return False


def _shape_ok(v, spec):
    """Does ``v`` have the outer shape of ``spec`` (used to pick an alternative;
    DURATION is never one)."""
    if isinstance(spec, str):
        return _matches_scalar(v, spec)
    kind = spec[0]
    if kind == "or":
        return any(_shape_ok(v, s) for s in spec[1:])
    if kind == "list":
        return isinstance(v, list)
    return isinstance(v, dict)


def check(v, spec, path):
    """Raise SchemaError naming the first value whose type does not fit ``spec``."""
    if spec == DURATION:
        if not isinstance(v, str):
            raise SchemaError("%s must be a string" % path)
        from .utils import parse_duration
        try:
            parse_duration(v)
        except ValueError:
            raise SchemaError("%s Does not match format 'duration'" % path) from None
        return
    if isinstance(spec, str):
        if not _matches_scalar(v, spec):
            raise SchemaError("%s must be a %s" % (path, _human(spec)))
        return
    kind = spec[0]
    if kind == "or":
        alts = [s for s in spec[1:] if _shape_ok(v, s)]
        if not alts:
            raise SchemaError("%s must be a %s" % (path, _type_name(spec)))
        errors = []
        for s in alts:
            try:
                check(v, s, path)
                return
            except SchemaError as e:
                errors.append(e)
        raise errors[0]
    if kind == "list":
        if not isinstance(v, list):
            raise SchemaError("%s must be a list" % path)
        for i, x in enumerate(v):
            check(x, spec[1], "%s.%d" % (path, i) if path else str(i))
        return
    if not isinstance(v, dict):
        raise SchemaError("%s must be a mapping" % path)
    if kind == "map":
        for k, x in v.items():
            check(x, spec[1], "%s.%s" % (path, k) if path else str(k))
        return
    props = spec[1]
    for k, x in v.items():
        sub = props.get(k)
        if sub is not None:
            check(x, sub, "%s.%s" % (path, k) if path else str(k))


def validate_v3(doc):
    check(doc, V3_TOP, "")


def validate_v2_service(name, svc):
    check(svc, V2_SERVICE, name)
    # libcompose registers a "ports" format checker that runs nat.ParsePortSpecs on
    # each string entry (numbers are not format-checked)
    from .utils import parse_port_spec
    for i, p in enumerate(svc.get("ports") or []):
        if isinstance(p, str):
            try:
                parse_port_spec(p)
            except ValueError:
                raise SchemaError("%s.ports.%d Does not match format 'ports'" % (name, i)) from None
