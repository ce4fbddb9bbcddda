"""Knative Service YAMLs -> IR (reference ``internal/source/knative2kube.go``);
a thin adapter over :class:`~move2kube_amd.apiresourceset.KnativeAPIResourceSet`."""

from ..apiresourceset import KnativeAPIResourceSet
from ..models import plan as plantypes
from .translator import Translator


class KnativeTranslator(Translator):
    translation_type = plantypes.KNATIVE2KUBE

    def get_service_options(self, input_path, plan):
        return KnativeAPIResourceSet().get_service_options(input_path, plan)

    def translate(self, services, plan):
        return KnativeAPIResourceSet().translate(services, plan)
