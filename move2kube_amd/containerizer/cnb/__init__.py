"""CNB containerizer (reference ``internal/containerizer/cnbcontainerizer.go``)."""

import os
import sys
import threading

from ... import assets
from ...models import plan as plantypes
from ...utils import common
from ...utils.constants import DEFAULT_SERVICE_PORT
from ..base import Containerizer, ContainerizerError

DEFAULT_BUILDERS = ["cloudfoundry/cnb:cflinuxfs3", "gcr.io/buildpacks/builder"]

_cache = {}
_cache_lock = threading.Lock()


def reset_cache():
    with _cache_lock:
        _cache.clear()


# once-per-process warnings of the provider chain (cnb/provider.go)
_warned = {"not_supported": False, "long_wait": False}


def log_not_supported():
    if not _warned["not_supported"]:
        from ...utils import log
        log.warning("No CNB containerizer method accessible")
        _warned["not_supported"] = True


def log_long_wait():
    # the reference initialises its flag to true so the warning never fires
    # (SURVEY 2.13 #14); "fixed" compat warns once.
    from ...utils.constants import settings
    if settings.fixed and not _warned["long_wait"]:
        from ...utils import log
        log.warning("This could take a few minutes to complete.")
        _warned["long_wait"] = True


def prefetch_builder_probes(builders=None):
    """Start the container runtime's read-only probes of the default builders
    (runtime check, local images) now, so that they have run by the time the
    planner reaches CNB containerization."""
    if _chain_off():
        return
    from . import providers
    providers.start_runtime_prefetch(list(builders or DEFAULT_BUILDERS))


def _chain_off():
    """``M2K_DISABLE_CNB`` empties the provider chain: answered here without
    loading the providers (what they would say: every probe unsupported)."""
    return (os.environ.get("M2K_DISABLE_CNB", "") not in ("", "0")
            and __name__ + ".providers" not in sys.modules)


class CNBContainerizer(Containerizer):
    build_type = plantypes.CNB

    def __init__(self):
        self.builders = list(DEFAULT_BUILDERS)

    def init(self, path):
        self.builders = list(DEFAULT_BUILDERS)

    def get_target_options(self, plan, path):
        with _cache_lock:
            if path in _cache:
                return list(_cache[path])
        if _chain_off():
            supported = []
            for _ in self.builders:
                log_long_wait()
                log_not_supported()
        else:
            from . import providers  # docker API / podman / pack / runc: only when CNB is probed
            supported = [b for b in self.builders if providers.is_builder_supported(path, b)]
        with _cache_lock:
            _cache[path] = supported
        return list(supported)

    def get_container(self, plan, service):
        from ...models import ir as irtypes
        container = irtypes.new_container(self.build_type, service.image, True)
        if service.container_build_type != self.build_type:
            raise ContainerizerError("Service %s has container build type %s . Expected %s"
                                     % (service.service_name, service.container_build_type, self.build_type))
        if not service.target_options:
            raise ContainerizerError("Service %s has no containerization target options" % service.service_name)
        builder = service.target_options[0]
        script = common.get_string_from_template(assets.template("cnbbuild.sh.tpl"),
                                                 {"ImageName": service.image, "Builder": builder})
        srcs = service.source_artifacts.get(plantypes.SOURCE_DIRECTORY_ARTIFACT) or []
        if not srcs:
            raise ContainerizerError("Service %s has no source code directory specified" % service.service_name)
        rel = common.go_rel(plan.root_dir, srcs[0])
        container.add_file(common.go_join(rel, service.service_name + "-cnb-build.sh"), script)
        container.add_exposed_port(DEFAULT_SERVICE_PORT)
        return container

    def get_target_options_batch(self, plan, paths):
        """Builders whose detector accepts each path; the uncached (path,
        builder) probes of the whole batch go to the providers at once."""
        out = [None] * len(paths)
        todo = {}  # insertion-ordered set: a level of a large tree has thousands of paths
        with _cache_lock:
            for k, p in enumerate(paths):
                if p in _cache:
                    out[k] = list(_cache[p])
                else:
                    todo[p] = None
        todo = list(todo)
        if todo:
            pairs = [(p, b) for p in todo for b in self.builders]
            if _chain_off():
                log_long_wait()
                if pairs:
                    log_not_supported()
                ok = [False] * len(pairs)
            else:
                from . import providers
                ok = providers.is_builder_supported_batch(pairs)
            nb = len(self.builders)
            with _cache_lock:
                for j, p in enumerate(todo):
                    _cache[p] = [b for b, good in zip(self.builders, ok[j * nb:(j + 1) * nb]) if good]
            with _cache_lock:
                for k, p in enumerate(paths):
                    if out[k] is None:
                        out[k] = list(_cache[p])
        return out

    def get_all_buildpacks(self):
        if _chain_off():
            log_not_supported()
            return {}
        from . import providers
        return providers.get_all_buildpacks(self.builders)
