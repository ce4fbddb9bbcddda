"""Reuse containerizer: the image already exists; nothing to build
(reference ``internal/containerizer/reusecontainerizer.go``)."""

from ..models import ir as irtypes
from ..models import plan as plantypes
from .base import Containerizer, ContainerizerError


class ReuseContainerizer(Containerizer):
    build_type = plantypes.REUSE

    def get_container(self, plan, service):
        if service.container_build_type == self.build_type:
            return irtypes.new_container(self.build_type, service.image, False)
        raise ContainerizerError("Unsupported service type for Containerization or insufficient information in service")
