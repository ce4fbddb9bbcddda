"""Helm ``values.yaml`` model (reference ``types/output/helmvaluesoutput.go``)."""

from .base import GoMap

PARAMETER_REGISTRY_PREFIX = "{{.Values.registryurl}}/{{.Values.registrynamespace}}/"
SERVICES_TAG = "services"
IMAGE_TAG_TAG = "imagetag"
CONTAINERS_TAG = "containers"


class HelmValues:
    def __init__(self):
        self.ingress_host = ""
        self.registry_url = ""
        self.registry_namespace = ""
        # services[svc][container] = imagetag
        self.services = {}
        self.storage_class = ""
        self.global_variables = {}

    def to_yaml(self):
        d = {}
        if self.ingress_host:
            d["ingresshost"] = self.ingress_host
        d["registryurl"] = self.registry_url
        d["registrynamespace"] = self.registry_namespace
        d["services"] = GoMap({svc: {"containers": GoMap({c: {"imagetag": tag} for c, tag in conts.items()})}
                               for svc, conts in self.services.items()})
        if self.storage_class:
            d["storageclass"] = self.storage_class
        if self.global_variables:
            d["globalvariables"] = GoMap(self.global_variables)
        return d

    def merge(self, new):
        """``HelmValues.Merge``."""
        if new.registry_namespace:
            self.registry_namespace = new.registry_namespace
        if new.registry_url:
            self.registry_url = new.registry_url
        if new.storage_class:
            self.storage_class = new.storage_class
        for k, v in new.global_variables.items():
            self.global_variables[k] = v
        for svc, conts in new.services.items():
            if svc not in self.services:
                self.services[svc] = dict(conts)
            else:
                for c, tag in conts.items():
                    self.services[svc][c] = tag

    def copy(self):
        h = HelmValues()
        h.ingress_host = self.ingress_host
        h.registry_url = self.registry_url
        h.registry_namespace = self.registry_namespace
        h.services = {k: dict(v) for k, v in self.services.items()}
        h.storage_class = self.storage_class
        h.global_variables = dict(self.global_variables)
        return h
