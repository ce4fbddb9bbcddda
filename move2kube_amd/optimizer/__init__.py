"""IR optimizers, applied in a fixed order (reference ``internal/optimizer/``):
normalize characters -> ingress exposure (QA) -> minimum replicas ->
imagePullPolicy Always -> port merge (QA)."""

from .. import qaengine
from ..models import ir as irtypes
from ..models import qa
from ..utils import common, log, trace
from ..utils.constants import ANNOTATION_LABEL_VALUE, DEFAULT_SERVICE_PORT, EXPOSE_SELECTOR

MIN_REPLICAS = 2
_QUOTE_CHARS = "',\""


def strip_quotation(s):
    """``regexp.MustCompile(`^[',"](.*)[',"]$`).ReplaceAllString(s, "$1")``
    (normalizecharactersoptimizer.go:48-52) without a regex.  RE2's ``.`` does
    not match a newline and its ``$`` is the end of the text, so a value with a
    line break inside keeps its quotes."""
    if len(s) >= 2 and s[0] in _QUOTE_CHARS and s[-1] in _QUOTE_CHARS and "\n" not in s:
        return s[1:-1]
    return s


class NormalizeCharacterOptimizer:
    def optimize(self, ir):
        for service in ir.services.values():
            for c in service.containers:
                if "env" not in c:
                    continue
                out = []
                for env in c.get("env") or []:
                    if "affinity" in env.get("name", ""):
                        continue
                    env = dict(env)
                    env["name"] = strip_quotation(env.get("name", "").strip())
                    if "value" in env:
                        env["value"] = strip_quotation((env.get("value") or "").strip())
                    out.append(env)
                c["env"] = out if out else None
                if c["env"] is None:
                    del c["env"]
        return ir


class IngressOptimizer:
    def optimize(self, ir):
        if not ir.services:
            log.debug("No services to optimize")
            return ir
        names = sorted(ir.services)
        exposed = [n for n in names if ir.services[n].service_rel_path != ""]
        prob = qa.new_multiselect_problem("Select all services that should be exposed:",
                                          ["Exposed services will be reachable from outside the cluster."], exposed, names)
        exposed = qaengine.fetch_answer(prob).get_slice_answer()
        if not exposed:
            log.debug("User deselected all services. Not exposing anything.")
            return ir
        for name in exposed:
            msg = "What URL/path should we expose the service %s on?" % name
            hints = ["By default we expose the service on /<service name>:"]
            path = "/" + name
            if len(exposed) == 1:
                hints = ["Since there's only one exposed service, the default path is /"]
                path = "/"
            prob = qa.new_input_problem(msg, hints, path)
            path = qaengine.fetch_answer(prob).get_string_answer()
            log.debug("Exposing service %s on path %s", name, path)
            path = self.normalize(path)
            svc = ir.services[name]
            svc.service_rel_path = path
            if svc.annotations is None:
                svc.annotations = {}
            svc.annotations[EXPOSE_SELECTOR] = ANNOTATION_LABEL_VALUE
        return ir

    @staticmethod
    def normalize(path):
        path = path.strip()
        if not path:
            log.warning("User gave an empty service path. Assuming it should be exposed on /")
        if not path.startswith("/"):
            path = "/" + path
        return path


class ReplicaOptimizer:
    def optimize(self, ir):
        for s in ir.services.values():
            if s.replicas < MIN_REPLICAS:
                s.replicas = MIN_REPLICAS
        return ir


class ImagePullPolicyOptimizer:
    def optimize(self, ir):
        for s in ir.services.values():
            for c in s.containers:
                c["imagePullPolicy"] = "Always"
        return ir


class PortMergeOptimizer:
    def optimize(self, ir):
        find = None
        for name in sorted(ir.services):
            service = ir.services[name]
            if any(c.get("ports") for c in service.containers):
                continue
            log.debug("The service %s has no ports", service.name)
            if find is None:
                find = ir.container_finder()  # containers do not change in this pass
            p2c = self.gather_ports(ir, service, find)
            if not p2c:
                continue
            selected = self.ask(service, p2c)
            if not selected:
                log.info("User deselected all ports. Not adding any ports to the service %s", service.name)
                continue
            for port in sorted(selected):
                idx = selected[port]
                service.containers[idx].setdefault("ports", []).append({"containerPort": port})
                service.add_port_forwarding(irtypes.Port(port), irtypes.Port(port))
        return ir

    @staticmethod
    def gather_ports(ir, service, find=None):
        p2c = {}
        find = find or ir.get_container
        for idx, c in enumerate(service.containers):
            irc, ok = find(c.get("image", ""))
            if ok:
                for port in irc.exposed_ports:
                    if port in p2c:
                        log.debug("The port %d is eligible to be exposed by both container %s and container %s of service %s",
                                  port, service.containers[p2c[port]].get("name"), c.get("name"), service.name)
                        continue
                    p2c[port] = idx
        if not p2c:
            if not service.containers:
                log.info("The service %s has no ports because it has no containers.", service.name)
            else:
                log.info("Could not find any eligibile ports for the service %s . Adding default port %d",
                         service.name, DEFAULT_SERVICE_PORT)
                p2c[DEFAULT_SERVICE_PORT] = 0
        return p2c

    @staticmethod
    def ask(service, p2c):
        eligible = [str(p) for p in sorted(p2c)]
        prob = qa.new_multiselect_problem(
            "Service %s has no ports. Please select the ports that should be added to it:" % service.name,
            ["If this is a headless service deselect all the ports."], eligible, eligible)
        ans = qaengine.fetch_answer(prob).get_slice_answer()
        out = {}
        for a in ans:
            try:
                p = common.cast_to_int(a)
            except ValueError as e:
                log.debug("Failed to parse %r as an integer port. Error: %r", a, str(e))
                continue
            out[p] = p2c.get(p, 0)
        return out


def _go_type(x):
    """``%T`` of the reference's value: ``*optimize.<type>``, the Go type name being
    the class name with its first letter lowered."""
    n = type(x).__name__
    return "*optimize." + n[:1].lower() + n[1:]


def get_optimizers():
    return [NormalizeCharacterOptimizer(), IngressOptimizer(), ReplicaOptimizer(), ImagePullPolicyOptimizer(),
            PortMergeOptimizer()]


def optimize(ir):
    log.info("Begin Optimization")
    for o in get_optimizers():
        log.debug("[%s] Begin Optimization", _go_type(o))
        try:
            with trace.span(type(o).__name__, "optimizer"):
                ir = o.optimize(ir)
        except Exception as e:  # noqa: BLE001
            if isinstance(e, log.FatalError):
                raise
            log.warning("[%s] Failed : %s", _go_type(o), e)
        else:
            log.debug("[%s] Done", _go_type(o))
    log.info("Optimization done")
    return ir
