"""Per-kind Kubernetes API resource handlers: creation from the IR and
conversion of objects to kinds the target cluster supports."""

from .base import APIResource  # noqa: F401
from .deployment import Deployment  # noqa: F401
from .others import ImageStream, KnativeService, NetworkPolicy  # noqa: F401
from .service import Service  # noqa: F401
from .storage import Storage  # noqa: F401
from .tekton import (EventListener, Pipeline, Role, RoleBinding, ServiceAccount, TriggerBinding,  # noqa: F401
                     TriggerTemplate)
