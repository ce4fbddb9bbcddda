"""Kubernetes YAMLs -> IR (reference ``internal/source/kube2kube.go``); a thin
adapter over :class:`~move2kube_amd.apiresourceset.K8sAPIResourceSet`."""

from ..apiresourceset import K8sAPIResourceSet
from ..models import plan as plantypes
from .translator import Translator


class KubeTranslator(Translator):
    translation_type = plantypes.KUBE2KUBE

    def get_service_options(self, input_path, plan):
        return K8sAPIResourceSet().get_service_options(input_path, plan)

    def translate(self, services, plan):
        return K8sAPIResourceSet().translate(services, plan)
