"""ImageStream, NetworkPolicy and Knative Service handlers (reference
``internal/apiresource/imagestream.go``, ``networkpolicy.go``,
``knativeservice.go``)."""

from ..utils import common, log
from ..utils.constants import ANNOTATION_LABEL_VALUE, GROUP_NAME
from .base import IAPIResource, get_annotations, get_service_labels, is_type

IMAGESTREAM = "ImageStream"
NETWORK_POLICY = "NetworkPolicy"
NETWORK_SELECTOR = GROUP_NAME + "/network"
KNATIVE_SERVICE = "Service"


class ImageStream(IAPIResource):
    def __init__(self, cluster=None):
        self.cluster = cluster

    def get_supported_kinds(self):
        return [IMAGESTREAM]

    def create_new_resources(self, ir, supported):
        objs = []
        for service in ir.sorted_services():
            if common.is_string_present(supported, IMAGESTREAM):
                objs.extend(self.create_image_stream(service.name, service))
            else:
                log.debug("Could not find a valid resource type in cluster to create a ImageStream")
        return objs

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        if common.is_string_present(supported, IMAGESTREAM) and is_type(obj, "image.openshift.io/v1", IMAGESTREAM):
            return [obj], True
        return None, False

    @staticmethod
    def create_image_stream(name, service):
        out = []
        for c in service.containers:
            image = c.get("image") or name
            _, tag = common.get_image_name_and_tag(image)
            out.append({"kind": IMAGESTREAM, "apiVersion": "image.openshift.io/v1",
                        "metadata": {"name": name, "labels": get_service_labels(name)},
                        "spec": {"tags": [{"from": {"kind": "DockerImage", "name": image}, "name": tag}]}})
        return out


def get_network_policy_labels(networks):
    return {NETWORK_SELECTOR + "/" + n: ANNOTATION_LABEL_VALUE for n in networks or []}


class NetworkPolicy(IAPIResource):
    def __init__(self, cluster=None):
        self.cluster = cluster

    def get_supported_kinds(self):
        return [NETWORK_POLICY]

    def create_new_resources(self, ir, supported):
        if not common.is_string_present(supported, NETWORK_POLICY):
            log.error("Could not find a valid resource type in cluster to create a NetworkPolicy")
            return None   # nil in the reference; an empty list when the kind is supported
        objs = []
        for service in ir.sorted_services():
            for net in service.networks:
                log.debug("Network %s is detected at Source, shall be converted to equivalent NetworkPolicy at Destination", net)
                objs.append(self.create_network_policy(net))
        return objs

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        if common.is_string_present(supported, NETWORK_POLICY) and is_type(obj, "networking.k8s.io/v1", NETWORK_POLICY):
            return [obj], True
        return None, False

    @staticmethod
    def create_network_policy(name):
        return {"kind": NETWORK_POLICY, "apiVersion": "networking.k8s.io/v1", "metadata": {"name": name},
                "spec": {"podSelector": {"matchLabels": {NETWORK_SELECTOR + "/" + name: ANNOTATION_LABEL_VALUE}},
                         "ingress": [{"from": [{"podSelector": {"matchLabels": get_network_policy_labels([name])}}]}]}}


class KnativeService(IAPIResource):
    def __init__(self, cluster=None):
        self.cluster = cluster

    def get_supported_kinds(self):
        return [KNATIVE_SERVICE]

    def create_new_resources(self, ir, supported):
        objs = []
        for service in ir.sorted_services():
            ps = common.deep_copy(service.pod_spec)
            ps["restartPolicy"] = "Always"
            m = {"name": service.name, "labels": get_service_labels(service.name)}
            ann = get_annotations(service)
            if ann:
                m["annotations"] = ann
            objs.append({"kind": KNATIVE_SERVICE, "apiVersion": "serving.knative.dev/v1", "metadata": m,
                         "spec": {"template": {"spec": ps}}})
        return objs

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        if is_type(obj, "serving.knative.dev/v1", KNATIVE_SERVICE):
            return [obj], True
        return None, False
