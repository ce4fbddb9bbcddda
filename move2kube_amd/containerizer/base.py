"""Containerizer framework (reference ``internal/containerizer/containerizer.go``).

The registry is ``[Dockerfile, S2I, CNB, Reuse]``; each is initialised on the
user's source tree *and* on the assets dir, so users can drop their own
detector directories into their sources.  ``Manual`` and ``ReuseDockerfile``
are not in the registry - the translators call them directly, exactly like the
reference.

Batch API: :meth:`Containerizers.get_containerization_options_batch` evaluates
many directories at once; all (detector x directory) detect scripts of the
batch run concurrently in the native process pool.
"""

from ..models import plan as plantypes
from ..utils import log
from ..utils.constants import settings

CONTAINERIZER_JSON_PORT = "port"
CONTAINERIZER_JSON_BUILDER = "builder"
CONTAINERIZER_JSON_IMAGE_NAME = "image_name"


class ContainerizationOption:
    __slots__ = ("containerization_type", "target_options")

    def __init__(self, ctype, target_options):
        self.containerization_type = ctype
        self.target_options = list(target_options)

    def __repr__(self):
        return "ContainerizationOption(%s, %r)" % (self.containerization_type, self.target_options)

    def __eq__(self, o):
        return (isinstance(o, ContainerizationOption) and o.containerization_type == self.containerization_type
                and o.target_options == self.target_options)


class Containerizer:
    build_type = ""

    def init(self, path):
        pass

    def get_target_options(self, plan, path):
        return []

    def get_target_options_batch(self, plan, paths):
        return [self.get_target_options(plan, p) for p in paths]

    def get_container(self, plan, service):
        raise NotImplementedError

    def get_container_build_strategy(self):
        return self.build_type


class ContainerizerError(RuntimeError):
    pass


class Containerizers:
    def __init__(self):
        self.containerizers = []

    def init_containerizers(self, path):
        from .cnb import CNBContainerizer
        from .dockerfile import DockerfileContainerizer
        from .reuse import ReuseContainerizer
        from .s2i import S2IContainerizer
        self.containerizers = [DockerfileContainerizer(), S2IContainerizer(), CNBContainerizer(), ReuseContainerizer()]
        for c in self.containerizers:
            c.init(path)
            c.init(settings.assets_path)
        return self

    def get_containerization_options(self, plan, sourcepath):
        return self.get_containerization_options_batch(plan, [sourcepath])[0]

    def get_containerization_options_batch(self, plan, paths):
        per = [c.get_target_options_batch(plan, paths) for c in self.containerizers]
        out = []
        for j in range(len(paths)):
            cops = []
            for c, opts in zip(self.containerizers, per):
                if opts[j]:
                    cops.append(ContainerizationOption(c.get_container_build_strategy(), opts[j]))
            out.append(cops)
        return out

    def get_container(self, plan, service):
        for c in self.containerizers:
            if c.get_container_build_strategy() != service.container_build_type:
                continue
            log.debug("Containerizing %s using %s", service.service_name, service.container_build_type)
            try:
                return c.get_container(plan, service)
            except Exception as e:  # noqa: BLE001
                log.error("Error during containerization : %s", e)
                raise
        if settings.fixed and service.container_build_type == plantypes.MANUAL:
            # Manual is not in the registry in the reference, so a
            # manual CF app is dropped there; "fixed" compat containerizes it.
            from .manual import ManualContainerizer
            return ManualContainerizer().get_container(plan, service)
        raise ContainerizerError("service %s has an invalid containerization strategy %s"
                                 % (service.service_name, service.container_build_type))
