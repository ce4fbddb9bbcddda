"""Manual containerizer: a new image the user has to build by hand; it ends up
in ``Manualimages.md`` (reference ``internal/containerizer/manualcontainerizer.go``)."""

from ..models import ir as irtypes
from ..models import plan as plantypes
from .base import Containerizer, ContainerizerError


class ManualContainerizer(Containerizer):
    build_type = plantypes.MANUAL

    def get_container(self, plan, service):
        if service.container_build_type == self.build_type:
            return irtypes.new_container(self.build_type, service.image, True)
        raise ContainerizerError("Unsupported service type for Containerization or insufficient information in service")
