"""New-Dockerfile containerizer (reference ``internal/containerizer/dockerfilecontainerizer.go``).

Detector protocol (the extension ABI): every directory containing an
``m2kdfdetect.sh`` is a detector.  ``/bin/sh m2kdfdetect.sh <dir>`` is run
with the detector directory as cwd; exit status 0 means "can containerize",
stdout is a JSON object whose keys feed the detector's ``Dockerfile`` Go
template.  All other files of the detector directory are copied next to the
generated ``Dockerfile.<service>``.
"""

import os

from .. import assets
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..parallel.detect_pool import run_detect, run_detect_jobs
from ..utils import common, fastjson, log
from ..utils.fsindex import get_index
from ..utils.gotemplate import TemplateError
from .base import CONTAINERIZER_JSON_PORT, Containerizer, ContainerizerError

DOCKERFILE_DETECT_SCRIPT = "m2kdfdetect.sh"


_GO_JSON_KIND = {list: "array", str: "string", float: "number", bool: "bool"}


def parse_detect_output(output):
    """The detect script's JSON as ``json.Unmarshal`` into a
    ``map[string]interface{}`` leaves it: numbers are float64, ``null`` is the
    nil (empty) map, any other non-object is Go's UnmarshalTypeError."""
    v = fastjson.loads(output, parse_int=float)
    if v is None:
        return {}
    if not isinstance(v, dict):
        raise ValueError("json: cannot unmarshal %s into Go value of type map[string]interface {}"
                         % _GO_JSON_KIND[type(v)])
    return v


def _port_from(m):
    v = m.get(CONTAINERIZER_JSON_PORT)
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return int(v)
    return None


def _go_list(items):
    """fmt ``%v`` / ``%s`` of a ``[]string``."""
    return "[" + " ".join(items) + "]"


class DockerfileContainerizer(Containerizer):
    build_type = plantypes.NEW_DOCKERFILE
    script = DOCKERFILE_DETECT_SCRIPT
    # log texts of dockerfilecontainerizer.go:49-81 (s2icontainerizer.go has its own)
    kind_name = "Dockerfile"
    fetch_warning = "Unable to fetch files to recognize docker detect scripts : %s"
    detected_debug = "Detected Dockerfile containerization options : %s"

    def __init__(self):
        self.detectors = []

    def init(self, path):
        try:
            files = common.get_files_by_name(path, [self.script])
        except (OSError, ValueError) as e:
            log.warning(self.fetch_warning, e)
            files = []
        for f in files:
            self.detectors.append(os.path.dirname(f))
        log.debug(self.detected_debug, _go_list(self.detectors))

    def get_target_options_batch(self, plan, paths):
        jobs = [(d, self.script, p) for p in paths for d in self.detectors]
        res = run_detect_jobs(jobs)
        out = []
        k = 0
        verbose = log.debug_enabled()
        for p in paths:
            opts = []
            for d in self.detectors:
                r = res[k]
                k += 1
                if verbose:
                    self._log_detect(d, p, r)
                if r.ok:
                    opts.append(d)
            out.append(opts)
        return out

    def _log_detect(self, d, p, r):
        """The per-detector debug lines of ``GetTargetOptions``/``detect``
        (``cmd`` prints as exec.Cmd's String(): path and arguments)."""
        log.debug("Executing detect script %s on %s : %s", d, p, "/bin/sh %s %s" % (self.script, p))
        if r.ok:
            log.debug("Output of %s containerizer detect script %s : %s", self.kind_name, d, r.stdout)
        else:
            log.debug("%s detector cannot containerize %s Error: %s", d, p,
                      log.go_quote(common.go_exit_status(r.code)))

    def get_target_options(self, plan, path):
        return self.get_target_options_batch(plan, [path])[0]

    def get_container(self, plan, service):
        if service.container_build_type != self.build_type or not service.target_options:
            raise ContainerizerError("Unsupported service type for containerization or insufficient information in service")
        container = irtypes.new_container(self.build_type, service.image, True)
        container.repo_info = service.repo_info.copy()
        cdir = service.target_options[0]
        tpl_path = os.path.join(cdir, "Dockerfile")
        try:
            template = common.read_text(tpl_path)
        except OSError as e:
            log.error("Unable to read the Dockerfile template at path %r Error: %r", tpl_path,
                      common.go_path_error(e, "open"))
            raise ContainerizerError(str(e)) from e
        srcs = service.source_artifacts.get(plantypes.SOURCE_DIRECTORY_ARTIFACT) or []
        if not srcs:
            raise ContainerizerError("Service %s has no source code directory specified" % service.service_name)
        src_dir = srcs[0]
        r = run_detect(cdir, self.script, src_dir)
        if not r.ok:
            err = common.go_exit_status(r.code)
            log.error("Detect using Dockerfile containerizer at path %r on the source code at path %r failed. "
                      "Error: %r", cdir, src_dir, err)
            raise ContainerizerError(err)
        contents = template
        if r.stdout != "":
            try:
                m = parse_detect_output(r.stdout)
            except ValueError as e:
                log.error("Unable to unmarshal the output of the detect script at path %r Output: %r Error: %r",
                          cdir, r.stdout, str(e))
                raise ContainerizerError(str(e)) from e
            port = _port_from(m)
            if port is not None:
                container.add_exposed_port(port)
            try:
                contents = common.get_string_from_template(template, m)
            except TemplateError as e:
                log.warning("Template conversion failed : %s", e)
                contents = ""
        rel = common.go_rel(plan.root_dir, src_dir)
        df_name = "Dockerfile." + service.service_name
        df_path = common.go_join(rel, df_name)
        container.add_file(df_path, contents)
        try:
            script = common.get_string_from_template(assets.template("dockerbuild.sh.tpl"), {
                "Dockerfilename": df_name, "ImageName": service.image, "Context": "."})
            container.add_file(common.go_join(rel, service.service_name + "-docker-build.sh"), script)
            container.repo_info.target_path = df_path
        except TemplateError as e:
            log.error("Unable to translate Dockerfile build template to string Error: %r", str(e))
        # copy every other file of the detector directory next to the Dockerfile
        try:
            files = get_index(cdir).files()
        except OSError:
            files = []
        for f in files:
            name = os.path.basename(f)
            if name in ("Dockerfile", self.script):
                continue
            try:
                container.add_file(common.go_join(rel, name), common.read_text(f))
            except OSError as e:
                log.error("Failed to read the file at path %r Error: %r", f, common.go_path_error(e, "open"))
                raise ContainerizerError(str(e)) from e
        return container
