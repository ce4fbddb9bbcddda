"""Reuse-Dockerfile containerizer: writes ``<svc>-docker-build.sh`` next to an
existing Dockerfile (reference ``internal/containerizer/reusedockerfilecontainerizer.go``)."""

import os

from .. import assets
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..utils import common, log
from .base import Containerizer, ContainerizerError


class ReuseDockerfileContainerizer(Containerizer):
    build_type = plantypes.REUSE_DOCKERFILE

    def get_container(self, plan, service):
        container = irtypes.new_container(self.build_type, service.image, True)
        if not service.target_options:
            raise ContainerizerError("Failed to reuse the Dockerfile. The service %s doesn't have any containerization "
                                     "target options" % service.service_name)
        df_path = service.target_options[0]
        try:
            os.stat(df_path)
        except FileNotFoundError as e:      # os.IsNotExist: other stat errors pass silently
            log.error("Unable to find the Dockerfile at path %r Error: %r", df_path, common.go_path_error(e, "stat"))
            log.error("Will assume the dockerfile will be copied and will proceed.")
        except (OSError, ValueError):
            pass
        df_dir = common.go_dir(df_path)
        script_path = common.go_join(df_dir, service.service_name + "-docker-build.sh")
        rel_ctx = "."
        srcs = service.build_artifacts.get(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT)
        if srcs:
            rel_ctx = common.go_rel(df_dir, srcs[0])
        script = common.get_string_from_template(assets.template("dockerbuild.sh.tpl"), {
            "Dockerfilename": common.go_base(df_path), "ImageName": service.image, "Context": rel_ctx})
        rel_script = plan.get_relative_path(script_path)
        container.add_file(rel_script, script)
        return container
