"""Dockerfile2Kube: reuse existing Dockerfiles (reference ``internal/source/dockerfile2kube.go``).

Every file of the tree is sniffed (natively, in parallel) for "first non-ARG
instruction is a FROM matching the reference regex".  Dockerfiles are grouped
by git repository (origin remote name; the project name when not in a repo)
and split into services by common path prefix (``bucketDFs``).
"""

import os

from ..containerizer.reusedockerfile import ReuseDockerfileContainerizer
from ..models import ir as irtypes
from ..models import plan as plantypes
from ..ops import native
from ..utils import common, git, log
from ..utils.constants import settings
from ..utils.fsindex import get_index
from .dockerfile_parser import is_dockerfile_line
from .translator import Translator


class _DF:
    __slots__ = ("path", "pathsuffix", "context")

    def __init__(self, path, pathsuffix, context):
        self.path = path
        self.pathsuffix = pathsuffix
        self.context = context

    def copy(self):
        return _DF(self.path, self.pathsuffix, self.context)


class DockerfileTranslator(Translator):
    translation_type = plantypes.DOCKERFILE2KUBE

    def new_service(self, name):
        s = plantypes.Service.new(name, self.translation_type)
        s.container_build_type = plantypes.REUSE_DOCKERFILE
        s.add_source_type(plantypes.DIRECTORY_SOURCE)
        s.update_container_build_pipeline = True
        s.update_deploy_pipeline = True
        return s

    def get_service_options(self, input_path, plan):
        services = []
        try:
            sdfs = get_dockerfile_services(input_path, plan.name)
        except OSError as e:
            err = common.go_path_error(e, "stat")
            log.error("Unable to get Dockerfiles : %s", err)
            raise RuntimeError(err) from e
        for sn in sorted(sdfs):
            dfs = sdfs[sn]
            ns = self.new_service(sn)
            ns.image = sn + ":latest"
            ns.add_build_artifact(plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT, dfs[0].context)
            for df in dfs:
                ns.add_source_artifact(plantypes.DOCKERFILE_ARTIFACT, df.path)
                ns.target_options.append(df.path)
            found, err = ns.gather_git_info(dfs[0].path, plan)
            if found and err is not None:
                log.warning("Error while parsing the git repo at path %r Error: %r", dfs[0].path, str(err))
            services.append(ns)
        return services

    def translate(self, services, plan):
        ir = irtypes.new_ir(plan)
        for service in services:
            if service.translation_type != self.translation_type:
                log.debug("The service %s has translation type %s . Expected %s . Skipping.", service.service_name,
                          service.translation_type, self.translation_type)
                continue
            if not service.target_options:
                log.debug("The service %s has no containerization target options. Skipping.", service.service_name)
                continue
            log.debug("Translating %s", service.service_name)
            try:
                c = ReuseDockerfileContainerizer().get_container(plan, service)
            except Exception as e:  # noqa: BLE001
                log.warning("Unable to get reuse the Dockerfile for service %s even though build parameters are present. Error: %r",
                            service.service_name, str(e))
                continue
            c.repo_info = service.repo_info.copy()
            c.repo_info.target_path = service.target_options[0]
            ir.add_container(c)
            irs = irtypes.new_service_from_plan_service(service)
            cont = {"name": service.service_name, "image": service.image}
            for port in c.exposed_ports:
                cont.setdefault("ports", []).append({"containerPort": port})
                irs.add_port_forwarding(irtypes.Port(port), irtypes.Port(port))
            irs.containers = [cont]
            ir.services[service.service_name] = irs
        return ir


def find_dockerfiles(input_path):
    """All files under ``input_path`` recognised as Dockerfiles (walk order)."""
    idx = get_index(input_path)
    files = idx.files()
    lines = native.sniff_dockerfiles(files, settings.workers)
    out = []
    for f, line in zip(files, lines):
        if is_dockerfile_line(line):
            log.debug("Identified a docker file : %s", f)
            out.append(f)
    return out


def get_dockerfile_services(input_path, proj_name):
    """``getDockerfileServices`` (dockerfile2kube.go:147-199): a missing input
    path is warned about (unquoted, unlike ``GetFilesByExt``) and raised as
    OSError; a file is walked as itself, with the walk's "is not a directory"
    warning."""
    try:
        os.stat(input_path)
    except FileNotFoundError as e:
        log.warning("Error in walking through files due to : %s", common.go_path_error(e, "stat"))
        raise
    files = find_dockerfiles(input_path)
    log.debug("No of dockerfiles identified : %d", len(files))
    repo_dfs = {}
    for f in files:
        repo, context = git.repo_name(os.path.dirname(f))
        if repo == "":
            repo = proj_name
            context = input_path
        repo_dfs.setdefault(repo, []).append(_DF(f, f, context))
    sdfs = {}
    for repo in sorted(repo_dfs):
        dfs = repo_dfs[repo]
        if len(dfs) == 1:
            sdfs[repo] = [dfs[0]]
            continue
        buckets = bucket_dfs(dfs)
        for k in sorted(buckets):
            v = buckets[k]
            sep = "" if (repo == "" or k == "") else "-"
            nk = repo + sep + k
            if nk in sdfs:
                sdfs[nk] = v + sdfs[nk]
            else:
                sdfs[nk] = v
    return sdfs


def bucket_dfs(dfs):
    dfs = [d.copy() for d in dfs]
    n = {}
    common_path = common.clean_and_find_common_directory([d.pathsuffix for d in dfs])
    if common_path != ".":
        for d in dfs:
            pre = common_path + "/"
            if d.pathsuffix.startswith(pre):
                d.pathsuffix = d.pathsuffix[len(pre):]
    for d in dfs:
        parts = d.pathsuffix.split("/")
        prefix = ""
        if len(parts) > 1:
            prefix = parts[0]
            if d.path.endswith(d.pathsuffix):
                d.context = d.path[:len(d.path) - len(d.pathsuffix)] + parts[0]
            else:
                d.context = d.path + parts[0]
        n.setdefault(prefix, []).append(d)
    out = {}
    for p in sorted(n):
        files = n[p]
        if len(files) == 1:
            out[p] = [files[0]]
        elif p == "":
            out.setdefault(p, []).extend(files)
        else:
            sub = bucket_dfs(files)
            for k in sorted(sub):
                v = sub[k]
                sep = "" if (p == "" or k == "") else "-"
                nk = p + sep + k
                if nk in out:
                    out[nk] = v + out[nk]
                else:
                    out[nk] = v
    return out
