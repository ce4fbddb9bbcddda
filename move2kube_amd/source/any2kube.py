"""Any2Kube: containerize plain source directories (reference ``internal/source/any2kube.go``).

Discovery semantics follow the reference's ``filepath.Walk``: the first
directory on a root-to-leaf path that any containerizer can handle becomes a
service named after the directory, and its sub-tree is skipped; directories
already claimed as ``SourceCode`` by earlier translators are skipped;
``.m2kignore`` files mark directories (``foo/``) or their contents (``foo/*``)
as ignored.

Execution is level-synchronous instead of serial DFS: every candidate directory
of one depth is evaluated in a single batch, so all (detector x directory)
detect scripts of the level run concurrently in the native process pool.  The
set of directories evaluated is exactly the set the serial walk would visit
(a directory is only a candidate if no ancestor matched), and results are
emitted in the walk's lexical DFS order, so the plan is identical.
"""

import os

from ..containerizer import Containerizers
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..utils import common, log
from ..utils.constants import IGNORE_FILENAME
from ..utils.fsindex import DIR, get_index
from .translator import Translator


class Any2KubeTranslator(Translator):
    translation_type = plantypes.ANY2KUBE

    def new_service(self, name):
        s = plantypes.Service.new(name, self.translation_type)
        s.add_source_type(plantypes.DIRECTORY_SOURCE)
        s.update_container_build_pipeline = True
        s.update_deploy_pipeline = True
        return s

    def get_service_options(self, input_path, plan):
        services = []
        cz = Containerizers().init_containerizers(input_path)
        pre = []
        for name in sorted(plan.services):
            for es in plan.services[name]:
                sc = es.source_artifacts.get(plantypes.SOURCE_DIRECTORY_ARTIFACT) or []
                if sc:
                    pre.append(sc[0])
        ignore_dirs, ignore_contents = self.get_ignore_paths(input_path)
        try:
            idx = get_index(input_path)
        except OSError as e:
            log.warning("Skipping path %r due to error. Error: %r", input_path, str(e))
            return services
        children = {}
        for p, k in zip(idx.paths, idx.kinds):
            if k == DIR and p != idx.root:
                children.setdefault(os.path.dirname(p), []).append(p)
        root = idx.root
        if not os.path.isdir(root) or os.path.islink(root):
            return services
        matched = {}
        frontier = [root]
        while frontier:
            candidates = []
            nxt = []
            for d in frontier:
                if common.is_string_present(pre, d):
                    continue
                if common.is_string_present(ignore_dirs, d):
                    if common.is_string_present(ignore_contents, d):
                        continue
                    nxt.extend(children.get(d, []))
                    continue
                candidates.append(d)
            if candidates:
                opts = cz.get_containerization_options_batch(plan, candidates)
                for d, o in zip(candidates, opts):
                    if o:
                        matched[d] = o
                        continue
                    log.debug("No known containerization approach is supported for directory %r", d)
                    if not common.is_string_present(ignore_contents, d):
                        nxt.extend(children.get(d, []))
            frontier = nxt
        for path in sorted(matched, key=lambda p: os.fsencode(p).split(b"/")):   # the walk's order: bytes
            for cop in matched[path]:
                s = self.new_service(os.path.basename(path))
                s.container_build_type = cop.containerization_type
                s.target_options = list(cop.target_options)
                if not common.is_string_present(s.build_artifacts.get(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT), path):
                    s.source_artifacts.setdefault(plantypes.SOURCE_DIRECTORY_ARTIFACT, []).append(path)
                    s.build_artifacts.setdefault(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT, []).append(path)
                found, err = s.gather_git_info(path, plan)
                if found and err is not None:
                    log.warning("Error while parsing the git repo at path %r Error: %r", path, str(err))
                services.append(s)
        return services

    def translate(self, services, plan):
        ir = irtypes.new_ir(plan)
        cz = Containerizers().init_containerizers(plan.root_dir)
        for service in services:
            if service.translation_type != self.translation_type:
                continue
            log.debug("Translating %s", service.service_name)
            try:
                container = cz.get_container(plan, service)
            except Exception as e:  # noqa: BLE001
                log.error("Unable to translate service %s Error: %r", service.service_name, str(e))
                continue
            ir.add_container(container)
            irs = irtypes.new_service_from_plan_service(service)
            sc = {"name": service.service_name, "image": service.image}
            ports = []
            for port in container.exposed_ports:
                ports.append({"containerPort": port})
                irs.add_port_forwarding(irtypes.Port(port), irtypes.Port(port))
            sc["ports"] = ports
            irs.containers = [sc]
            ir.services[service.service_name] = irs
        return ir

    @staticmethod
    def get_ignore_paths(input_path):
        ignore_dirs, ignore_contents = [], []
        try:
            files = common.get_files_by_name(input_path, [IGNORE_FILENAME])
        except OSError as e:
            log.warning("Unable to fetch .m2kignore files at path %r Error: %r", input_path, str(e))
            return ignore_dirs, ignore_contents
        for fp in files:
            try:
                data = common.read_bytes(fp)
            except OSError as e:
                log.warning("Failed to open the .m2kignore file at path %r Error: %r", fp, common.go_path_error(e, "open"))
                continue
            base = os.path.dirname(fp)
            # bufio.Scanner lines: LF only, a CR before it dropped, the scan
            # silently ending at a line of 64 KiB or more (any2kube.go:165-178)
            for raw in common.go_scan_lines(data)[0]:
                line = common.go_trim_space(raw.decode("utf-8", errors="surrogateescape"))
                if line.endswith("*"):
                    ignore_contents.append(common.go_join(base, line[:-1]))
                else:
                    ignore_dirs.append(common.go_join(base, line))
        return ignore_dirs, ignore_contents
