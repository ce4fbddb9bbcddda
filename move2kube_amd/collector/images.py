"""Image metadata via ``docker inspect`` (reference ``internal/collector/imagescollector.go``)."""

import os

from ..models.collection import ImageInfo
from ..utils import common, fastjson, log
from ..utils.constants import DEFAULT_DIRECTORY_PERMISSION, settings
from . import Collector, CommandError, concurrently, run
from ..utils.lazyre import lazy as _lazy_re

_NUM = _lazy_re(r"[0-9]+")


def get_image_info(data):
    info = ImageInfo()
    try:
        images = fastjson.loads(data)
    except ValueError as e:
        log.error("Unable to unmarshal image info : %s", e)
        images = []
    for image in images or []:
        cfg = image.get("ContainerConfig") or {}
        info.tags = list(image.get("RepoTags") or [])
        try:
            info.user_id = common.cast_to_int(cfg.get("User", ""))
        except (ValueError, TypeError):
            log.debug("UserID not available in image metadata for [%s]", (info.tags or [""])[0])
            info.user_id = -1
        info.accessed_dirs.append(cfg.get("WorkingDir", ""))
        for key in sorted(cfg.get("ExposedPorts") or {}):
            m = _NUM.search(key)
            try:
                if m is None:
                    raise ValueError(key)
                info.ports.append(common.cast_to_int(m.group(0)))   # "0123" is octal, "080" an error
            except ValueError:
                log.debug("PortNumber not available in image metadata for [%s]", (info.tags or [""])[0])
    return info


def get_docker_inspect_result(image):
    try:
        return run(["docker", "inspect", image], combined=True)
    except FileNotFoundError as e:
        log.warning("Error while running docker-inspect: %s", e)
        raise
    except CommandError as e:
        out = e.output.decode("utf-8", "replace")
        if "permission denied" in out:
            log.warning("Error while running docker-inspect due to lack of permissions")
            log.warning("Please refer to [https://docs.docker.com/engine/install/linux-postinstall/] to fix this issue")
        elif "No such object" in out:
            log.warning('Image [%s] not available in local image repo. Run "docker pull %s"', image, image)
            return None
        else:
            log.warning("Error while running docker-inspect: %s", e)
        raise


def get_all_image_names():
    try:
        out = run(["docker", "image", "list", "--format", "{{.Repository}}:{{.Tag}}"])
    except CommandError as e:
        log.warning("Error while running docker image list : %s", e)
        raise
    except OSError:
        # the reference runs it through `bash -c`: a missing docker is bash's 127
        log.warning("Error while running docker image list : %s", common.go_exit_status(127))
        raise
    images = []
    for image in out.decode("utf-8", "replace").split("\n"):
        if image.startswith("<none>") or image.endswith("<none>"):
            log.debug("Ignore image with <none> : %s", image)
            continue
        if image:
            images.append(image)
    # the reference filters the list but never appends to its result
    return images if settings.fixed else []


def get_dc_image_names(directory):
    """``getDCImageNames`` (imagescollector.go:156-170): every YAML file read
    with ``common.ReadYaml`` into ``sourcetypes.DockerCompose`` - a file whose
    ``services`` is not a mapping of mappings (null services and fields
    allowed) fails that typed decode and is skipped; a listing error is a
    warning and no file is read."""
    names = []
    try:
        files = common.get_files_by_ext(directory, [".yml", ".yaml"])
    except (OSError, ValueError) as e:
        log.warning("Unable to fetch yaml files and recognize Docker image yamls : %s", common.go_error_text(e, "lstat"))
        files = []
    for path in files:
        try:
            doc = common.read_yaml(path)
        except Exception:  # noqa: BLE001
            continue
        if doc is None:
            continue
        if not isinstance(doc, dict):
            continue
        services = doc.get("services")
        if services is None:
            continue
        if not isinstance(services, dict) or not all(
                v is None or (isinstance(v, dict) and not isinstance(v.get("image"), (dict, list)))
                for v in services.values()):
            continue
        for name in sorted(services):
            svc = services[name] or {}
            image = svc.get("image")
            names.append("" if image is None else common.go_bool_str(image) if isinstance(image, bool) else str(image))
    return names


class ImagesCollector(Collector):
    annotations = ("k8s", "dockerswarm", "dockercompose")

    def collect(self, input_path, output_path):
        output_path = os.path.join(output_path, "images")
        try:
            os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        except OSError as e:
            err = common.go_path_error(e, "mkdir")
            log.error("Unable to create output directory %s : %s", output_path, err)
            raise RuntimeError(err) from e
        names = get_all_image_names() if input_path == "" else get_dc_image_names(input_path)
        log.debug("Images : %s", names)
        # one `docker inspect` per image, up to 8 at a time (the reference runs
        # them one after another); results are handled in list order
        inspected = concurrently(*[(lambda n=name: get_docker_inspect_result(n)) for name in names])
        for name, data in zip(names, inspected):
            if isinstance(data, (OSError, CommandError)):
                continue
            if isinstance(data, Exception):
                raise data
            if data is None:
                continue
            info = get_image_info(data)
            shortest = ""
            for tag in info.tags:
                if shortest == "" or len(shortest) > len(tag):
                    shortest = tag
            path = os.path.join(output_path, common.normalize_for_filename(shortest) + ".yaml")
            try:
                common.write_yaml(path, info)
            except OSError as e:
                log.error("Unable to write file %s : %s", path, common.go_path_error(e, "open"))
            else:
                if not settings.fixed:
                    # imagescollector.go:75-76 logs the write's error unconditionally: %s of a nil error
                    log.error("Unable to write file %s : %s", path, "%!s(<nil>)")
