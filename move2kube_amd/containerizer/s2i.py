"""S2I containerizer (reference ``internal/containerizer/s2icontainerizer.go``).

Same detect protocol as the Dockerfile containerizer with ``m2ks2idetect.sh``;
the JSON must carry ``builder``.  Writes ``<svc>-s2i-build.sh`` and renders
*every* file of the detector directory (sub-directories such as
``.s2i/environment`` included) as a Go template with the detect JSON plus
``image_name``.
"""

import os

from .. import assets
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..parallel.detect_pool import run_detect
from ..utils import common, log
from ..utils.fsindex import get_index
from ..utils.gotemplate import TemplateError
from .base import CONTAINERIZER_JSON_BUILDER, CONTAINERIZER_JSON_IMAGE_NAME, ContainerizerError
from .dockerfile import DockerfileContainerizer, _port_from, parse_detect_output

S2I_DETECT_SCRIPT = "m2ks2idetect.sh"


class S2IContainerizer(DockerfileContainerizer):
    build_type = plantypes.S2I
    script = S2I_DETECT_SCRIPT
    # s2icontainerizer.go:51-80 (the trailing space is the reference's)
    kind_name = "S2I"
    fetch_warning = "Unable to fetch files to recognize s2i detect files : %s"
    detected_debug = "Detected S2I containerization options : %s "

    def get_container(self, plan, service):
        if service.container_build_type != self.build_type or not service.target_options:
            raise ContainerizerError("Unsupported service type for Containerization or insufficient information in service")
        container = irtypes.new_container(self.build_type, service.image, True)
        container.repo_info = service.repo_info.copy()
        cdir = service.target_options[0]
        srcs = service.source_artifacts.get(plantypes.SOURCE_DIRECTORY_ARTIFACT) or []
        if not srcs:
            raise ContainerizerError("Service %s has no source code directory specified" % service.service_name)
        src_dir = srcs[0]
        r = run_detect(cdir, self.script, src_dir)
        if not r.ok:
            log.error("Detect using S2I containerizer at path %r on the source code at path %r failed. Error: %r",
                      cdir, src_dir, r.stdout)
            raise ContainerizerError(common.go_exit_status(r.code))
        output = r.stdout.strip()
        try:
            m = parse_detect_output(output)
        except ValueError as e:
            log.error("Unable to unmarshal the output of the detect script at path %r Output: %r Error: %r",
                      cdir, output, str(e))
            raise ContainerizerError(str(e)) from e
        port = _port_from(m)
        if port is not None:
            container.add_exposed_port(port)
        m[CONTAINERIZER_JSON_IMAGE_NAME] = service.image
        builder = m.get(CONTAINERIZER_JSON_BUILDER)
        if not isinstance(builder, str):
            raise ContainerizerError("the S2I detect output of %s has no builder" % cdir)
        script = common.get_string_from_template(assets.template("s2ibuild.sh.tpl"),
                                                 {"Builder": builder, "ImageName": service.image})
        rel = common.go_rel(plan.root_dir, src_dir)
        container.add_file(common.go_join(rel, service.service_name + "-s2i-build.sh"), script)
        try:
            files = get_index(cdir).files()
        except OSError:
            files = []
        for f in files:
            if os.path.basename(f) == self.script:
                continue
            relf = common.go_rel(cdir, f)
            try:
                tpl = common.read_text(f)
            except OSError as e:
                log.error("Skipping path %r . Failed to read the template. Error: %r", f, common.go_path_error(e, "open"))
                continue
            try:
                contents = common.get_string_from_template(tpl, m)
            except TemplateError as e:
                log.error("Skipping path %r . Unable to translate the template to string. Error %r", f, str(e))
                continue
            container.add_file(common.go_join(rel, relf), contents)
        return container
