"""Services, Ingress and Routes (reference ``internal/apiresource/service.go``).

Exposed services get a Route per port when the cluster supports Routes,
otherwise one fan-out Ingress for all exposed services (pathType Prefix, TLS
when a secret is configured); every non ingress-only service also gets a
ClusterIP Service (headless when it has no ports).  Existing Routes, Ingresses
and NodePort/LoadBalancer Services are converted to what the cluster supports.
"""

from ..utils import common, log
from ..utils.constants import EXPOSE_SELECTOR
from .base import IAPIResource, get_annotations, get_service_labels, is_type, object_meta_copy

SERVICE = "Service"
INGRESS = "Ingress"
ROUTE = "Route"


def _int_or_string(name, number):
    return name if name else number


class Service(IAPIResource):
    def __init__(self, cluster=None):
        self.cluster = cluster

    def get_supported_kinds(self):
        return [SERVICE, INGRESS, ROUTE]

    def create_new_resources(self, ir, supported):
        objs = []
        ingress_enabled = False
        for service in ir.sorted_services():
            created = False
            if service.has_valid_annotation(EXPOSE_SELECTOR) or service.only_ingress:
                if common.is_string_present(supported, ROUTE):
                    objs.extend(self.create_routes(service, ir))
                    created = True
                elif common.is_string_present(supported, INGRESS):
                    created = True
                    ingress_enabled = True
            if service.only_ingress:
                if not created:
                    log.error("Failed to create the ingress for service %r . Probable cause: The cluster doesn't support ingress resources.", service.name)
                continue
            if not common.is_string_present(supported, SERVICE):
                log.error("Could not find a valid resource type in cluster to create a Service")
                continue
            if created or not service.has_valid_annotation(EXPOSE_SELECTOR):
                objs.append(self.create_service(service, "ClusterIP"))
            else:
                objs.append(self.create_service(service, "NodePort"))
        if ingress_enabled:
            objs.append(self.create_ingress(ir))
        return objs

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        if common.is_string_present(supported, ROUTE):
            if is_type(obj, "route.openshift.io/v1", ROUTE):
                return [obj], True
            if is_type(obj, "networking.k8s.io/v1", INGRESS):
                return self.ingress_to_route(obj), True
            if is_type(obj, "v1", SERVICE):
                if (obj.get("spec") or {}).get("type") in ("LoadBalancer", "NodePort"):
                    return self.service_to_routes(obj, ir), True
                return [obj], True
        elif common.is_string_present(supported, INGRESS):
            if is_type(obj, "route.openshift.io/v1", ROUTE):
                return self.route_to_ingress(obj, ir), True
            if is_type(obj, "networking.k8s.io/v1", INGRESS):
                return [obj], True
            if is_type(obj, "v1", SERVICE):
                if (obj.get("spec") or {}).get("type") in ("LoadBalancer", "NodePort"):
                    return self.service_to_ingress(obj, ir), True
                return [obj], True
        elif common.is_string_present(supported, SERVICE):
            if is_type(obj, "route.openshift.io/v1", ROUTE):
                return self.route_to_service(obj), True
            if is_type(obj, "networking.k8s.io/v1", INGRESS):
                return self.ingress_to_service(obj), True
            if is_type(obj, "v1", SERVICE):
                return [obj], True
        return None, False

    # -- conversions -----------------------------------------------------------
    @staticmethod
    def _route(meta, host, path, to_name, target_port):
        return {"kind": ROUTE, "apiVersion": "route.openshift.io/v1", "metadata": meta,
                "spec": {"host": host, "path": path, "to": {"kind": SERVICE, "name": to_name, "weight": 1},
                         "port": {"targetPort": target_port}},
                "status": {"ingress": [{"host": ""}]}}

    def ingress_to_route(self, ingress):
        objs = []
        for rule in (ingress.get("spec") or {}).get("rules") or []:
            for path in (rule.get("http") or {}).get("paths") or []:
                svc = (path.get("backend") or {}).get("service") or {}
                port = svc.get("port") or {}
                tp = _int_or_string(port.get("name", ""), port.get("number", 0))
                objs.append(self._route(object_meta_copy(ingress.get("metadata")), rule.get("host", ""),
                                        path.get("path", ""), svc.get("name", ""), tp))
        return objs

    def service_to_routes(self, service, ir):
        objs = []
        ports = (service.get("spec") or {}).get("ports") or []
        name = (service.get("metadata") or {}).get("name", "")
        prefix = "/" + name
        for sp in ports:
            path = prefix
            if len(ports) > 1:
                path = prefix + "/" + (sp.get("name") or str(sp.get("port", 0)))
            tp = _int_or_string(sp.get("name", ""), sp.get("port", 0))
            objs.append(self._route(object_meta_copy(service.get("metadata")), ir.target_cluster_spec.host,
                                    path, name, tp))
        svc = common.deep_copy(service)
        svc.setdefault("spec", {})["type"] = "ClusterIP"
        objs.append(svc)
        return objs

    def route_to_ingress(self, route, ir):
        spec = route.get("spec") or {}
        tp = (spec.get("port") or {}).get("targetPort", 0)
        port = {"name": tp} if isinstance(tp, str) else {"number": tp}
        host = spec.get("host", "")
        ing = {"kind": INGRESS, "apiVersion": "networking.k8s.io/v1", "metadata": object_meta_copy(route.get("metadata")),
               "spec": {"rules": [{"host": host, "http": {"paths": [{
                   "path": spec.get("path", ""),
                   "backend": {"service": {"name": (spec.get("to") or {}).get("name", ""), "port": port}}}]}}]}}
        if ir.is_ingress_tls_enabled():
            tls = {"hosts": [host], "secretName": "<TODO: fill the tls secret for this domain>"}
            if host == ir.target_cluster_spec.host:
                tls["secretName"] = ir.ingress_tls_secret_name
            ing["spec"]["tls"] = [tls]
        return [ing]

    def service_to_ingress(self, service, ir):
        rules = []
        ports = (service.get("spec") or {}).get("ports") or []
        name = (service.get("metadata") or {}).get("name", "")
        prefix = "/" + name
        for sp in ports:
            path = prefix
            if len(ports) > 1:
                path = prefix + "/" + (sp.get("name") or str(sp.get("port", 0)))
            rules.append({"host": ir.target_cluster_spec.host, "http": {"paths": [{
                "path": path, "backend": {"service": {"name": name, "port": {"number": sp.get("port", 0)}}}}]}})
        ing = {"kind": INGRESS, "apiVersion": "networking.k8s.io/v1",
               "metadata": object_meta_copy(service.get("metadata")), "spec": {"rules": rules}}
        if ir.is_ingress_tls_enabled():
            ing["spec"]["tls"] = [{"hosts": [ir.target_cluster_spec.host], "secretName": ir.ingress_tls_secret_name}]
        svc = common.deep_copy(service)
        svc.setdefault("spec", {})["type"] = "ClusterIP"
        return [ing, svc]

    def route_to_service(self, route):
        spec = route.get("spec") or {}
        tp = (spec.get("port") or {}).get("targetPort", 0)
        port = {"name": tp if isinstance(tp, str) else "", "port": tp if isinstance(tp, int) else 0}
        m = object_meta_copy(route.get("metadata"))
        m["name"] = (spec.get("to") or {}).get("name", "")
        return [{"kind": SERVICE, "apiVersion": "v1", "metadata": m,
                 "spec": {"type": "NodePort", "ports": [port]}}]

    def ingress_to_service(self, ingress):
        objs = []
        for rule in (ingress.get("spec") or {}).get("rules") or []:
            for path in (rule.get("http") or {}).get("paths") or []:
                svc = (path.get("backend") or {}).get("service") or {}
                port = svc.get("port") or {}
                m = object_meta_copy(ingress.get("metadata"))
                m["name"] = svc.get("name", "")
                objs.append({"kind": SERVICE, "apiVersion": "v1", "metadata": m,
                             "spec": {"type": "NodePort", "ports": [{"name": port.get("name", ""),
                                                                     "port": port.get("number", 0)}]}})
        return objs

    # -- creation -----------------------------------------------------------------
    def create_routes(self, service, ir):
        routes = []
        ports = self.get_service_ports(service)
        prefix = service.service_rel_path
        for sp in ports:
            path = prefix
            if len(ports) > 1:
                path = prefix + "/" + (sp["name"] or str(sp["port"]))
            meta = {"name": service.name, "labels": get_service_labels(service.name)}
            routes.append(self._route(meta, ir.target_cluster_spec.host, path, service.name, sp["name"]))
        return routes

    def create_ingress(self, ir):
        paths = []
        for service in ir.sorted_services():
            if not service.has_valid_annotation(EXPOSE_SELECTOR):
                continue
            backend = service.backend_service_name or service.name
            ports = self.get_service_ports(service)
            prefix = service.service_rel_path
            for sp in ports:
                path = prefix
                if len(ports) > 1:
                    path = prefix + "/" + (sp["name"] or str(sp["port"]))
                bport = {"name": sp["name"]} if sp["name"] else {"number": sp["port"]}
                paths.append({"path": path, "pathType": "Prefix",
                              "backend": {"service": {"name": backend, "port": bport}}})
        name = ir.name
        if len(ir.services) == 1:
            name = next(iter(ir.services.values())).name
        ing = {"kind": INGRESS, "apiVersion": "networking.k8s.io/v1",
               "metadata": {"name": name, "labels": get_service_labels(name)},
               "spec": {"rules": [{"host": ir.target_cluster_spec.host, "http": {"paths": paths}}]}}
        if ir.is_ingress_tls_enabled():
            ing["spec"]["tls"] = [{"hosts": [ir.target_cluster_spec.host], "secretName": ir.ingress_tls_secret_name}]
        return ing

    def create_service(self, service, stype):
        ports = self.get_service_ports(service)
        m = {"name": service.name, "labels": get_service_labels(service.name)}
        ann = get_annotations(service)
        if ann:
            m["annotations"] = ann
        svc = {"kind": SERVICE, "apiVersion": "v1", "metadata": m,
               "spec": {"type": stype, "selector": get_service_labels(service.name), "ports": ports}}
        if not ports:
            svc["spec"]["clusterIP"] = "None"
        return svc

    @staticmethod
    def get_service_ports(service):
        out = []
        for f in service.port_forwardings:
            name = f.service_port.name or "port-%d" % f.service_port.number
            tp = f.pod_port.name if f.pod_port.name else f.pod_port.number
            out.append({"name": name, "port": f.service_port.number, "targetPort": tp})
        return out
