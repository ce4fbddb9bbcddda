"""Compose2Kube (reference ``internal/source/compose2kube.go``).

Every ``.yml``/``.yaml`` file is tried as compose v3 first and v1/v2 second.
For each compose service a ReuseDockerfile option (when ``build.context`` is
set) and a Reuse option are planned; image-info YAMLs (``ImageMetadata`` from
``collect``) are attached by image tag.  The compose loaders are imported on
the first YAML file, so a tree without one never loads them.
"""

import os

from ..models import collection
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..utils import common, log
from .translator import Translator


def _read_image_info(path):
    from ..models.base import read_document
    return read_document(path, collection.ImageInfo.from_yaml, "IMAGE_INFO")


class ComposeTranslator(Translator):
    translation_type = plantypes.COMPOSE2KUBE

    def new_service(self, name):
        s = plantypes.Service.new(name, self.translation_type)
        s.add_source_type(plantypes.COMPOSE_SOURCE)
        s.container_build_type = plantypes.REUSE
        return s

    def _reuse_service(self, compose_path, name, image, image_meta):
        s = self.new_service(name)
        s.image = image or name + ":latest"
        s.update_container_build_pipeline = False
        s.update_deploy_pipeline = True
        s.add_source_artifact(plantypes.COMPOSE_FILE_ARTIFACT, compose_path)
        if image in image_meta:
            s.add_source_artifact(plantypes.IMAGE_INFO_ARTIFACT, image_meta[image])
        return s

    def _services_for(self, compose_path, name, image, rel_ctx, rel_df, image_meta):
        out = []
        name = common.normalize_for_service_name(name)
        log.debug("Found a docker compose service : %s", name)
        if rel_ctx:
            s = self._reuse_service(compose_path, name, image, image_meta)
            s.container_build_type = plantypes.REUSE_DOCKERFILE
            s.update_container_build_pipeline = True
            s.update_deploy_pipeline = True
            ctx = rel_ctx if os.path.isabs(rel_ctx) else common.go_join(os.path.dirname(compose_path), rel_ctx)
            s.add_source_type(plantypes.DIRECTORY_SOURCE)
            s.add_build_artifact(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT, ctx)
            df = common.go_join(ctx, "Dockerfile")
            if rel_df:
                df = rel_df if os.path.isabs(rel_df) else common.go_join(ctx, rel_df)
            s.add_source_artifact(plantypes.DOCKERFILE_ARTIFACT, df)
            s.target_options.append(df)
            out.append(s)
        out.append(self._reuse_service(compose_path, name, image, image_meta))
        return out

    def services_from_compose_file(self, path, image_meta):
        from .compose.v1v2 import parse_v2
        from .compose.v3 import ComposeError, parse_v3
        try:
            cfg = parse_v3(path)
        except ComposeError as e3:
            try:
                proj = parse_v2(path)
            except ComposeError as e2:
                log.debug("Failed to parse file at path %s as a docker compose file. Error V3: %r Error V1V2: %r",
                          path, str(e3), str(e2))
                return []
            log.debug("Found a docker compose file at path %s", path)
            out = []
            for s in proj["services"]:
                out.extend(self._services_for(path, s["name"], s["image"], s["build_context"], s["build_dockerfile"], image_meta))
            return out
        log.debug("Found a docker compose file at path %s", path)
        out = []
        for s in cfg["services"]:
            out.extend(self._services_for(path, s["name"], s["image"], s["build_context"], s["build_dockerfile"], image_meta))
        return out

    def get_service_options(self, input_path, plan):
        try:
            yamls = common.get_files_by_ext(input_path, [".yaml", ".yml"])
        except (OSError, ValueError) as e:
            log.error("Unable to fetch yaml files at path %s Error: %r", input_path, common.go_error_text(e))
            raise
        image_meta = {}
        for p in yamls:
            try:
                im = _read_image_info(p)
            except Exception:  # noqa: BLE001
                continue
            if im.kind != collection.IMAGE_METADATA_KIND:
                continue
            for tag in im.tags:
                image_meta[tag] = p
        services = []
        for p in yamls:
            services.extend(self.services_from_compose_file(p, image_meta))
        return services

    def translate(self, services, plan):
        ir = irtypes.new_ir(plan)
        for service in services:
            if service.translation_type != self.translation_type:
                log.debug("Expected service to have compose2kube translation type. Got %s . Skipping.",
                          service.translation_type)
                continue
            for path in service.source_artifacts.get(plantypes.COMPOSE_FILE_ARTIFACT) or []:
                log.debug("File %s being loaded from compose service : %s", path, service.service_name)
                from .compose.v1v2 import V1V2Loader
                from .compose.v3 import ComposeError, V3Loader
                try:
                    cir = V3Loader().convert_to_ir(path, plan, service)
                    version = "v3"
                except ComposeError as e3:
                    try:
                        cir = V1V2Loader().convert_to_ir(path, plan, service)
                        version = "v1v2"
                    except ComposeError as e2:
                        log.error("Unable to parse the docker compose file at path %s Error V3: %r Error V1V2: %r",
                                  path, str(e3), str(e2))
                        continue
                ir.merge(cir)
                log.debug("compose %s translator returned %d services", version, len(ir.services))
            for path in service.source_artifacts.get(plantypes.IMAGE_INFO_ARTIFACT) or []:
                try:
                    im = _read_image_info(path)
                except Exception as e:  # noqa: BLE001
                    log.error("Failed to read image info yaml at path %s Error: %r", path, common.go_error_text(e))
                    continue
                ir.add_container(irtypes.new_container_from_image_info(im))
        return ir
