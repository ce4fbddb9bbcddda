"""The plan file (``kind: Plan``) - the checkpoint between ``plan`` and ``translate``.

Schema and semantics follow the reference ``types/plan/plan.go:134-426`` and
``types/plan/planutils.go:38-268``:

* paths are stored relative to ``spec.inputs.rootDir`` (or to the temp dir for
  ``m2kassets/...``) and made absolute on read; which fields are converted is
  driven by the reference's ``m2kpath`` tags (``normal``, ``keys:...``,
  ``if:ContainerBuildType:in:...``), reproduced in :func:`_convert_paths`;
* ``rootDir`` itself is written relative to the current working directory;
* YAML field order/omitempty rules match the Go struct tags so that
  read -> write round-trips byte-for-byte.
"""

import os

from ..utils import common, log, yamlio
from ..utils.constants import (ASSETS_DIR, DEFAULT_CLUSTER_TYPE, DEFAULT_PROJECT_NAME,
                               SCHEME_GROUP_VERSION, settings)
from .base import (GoMap, as_bool, as_list, as_map, as_str, as_str_list, read_document,
                   as_str_list_map)

PLAN_KIND = "Plan"

# TranslationTypeValue
COMPOSE2KUBE = "Compose2Kube"
CFMANIFEST2KUBE = "Cfmanifest2Kube"
ANY2KUBE = "Any2Kube"
KUBE2KUBE = "Kube2Kube"
KNATIVE2KUBE = "Knative2Kube"
DOCKERFILE2KUBE = "Dockerfile2Kube"

# SourceTypeValue
COMPOSE_SOURCE = "DockerCompose"
DIRECTORY_SOURCE = "Directory"
CFMANIFEST_SOURCE = "CfManifest"
KNATIVE_SOURCE = "Knative"
K8S_SOURCE = "Kubernetes"

# ContainerBuildTypeValue
NEW_DOCKERFILE = "NewDockerfile"
REUSE_DOCKERFILE = "ReuseDockerfile"
REUSE = "Reuse"
CNB = "CNB"
MANUAL = "Manual"
S2I = "S2I"

# SourceArtifactTypeValue
K8S_FILE_ARTIFACT = "Kubernetes"
KNATIVE_FILE_ARTIFACT = "Knative"
COMPOSE_FILE_ARTIFACT = "DockerCompose"
IMAGE_INFO_ARTIFACT = "ImageInfo"
CFMANIFEST_ARTIFACT = "CfManifest"
CF_RUNNING_MANIFEST_ARTIFACT = "CfRunningManifest"
SOURCE_DIRECTORY_ARTIFACT = "SourceCode"
DOCKERFILE_ARTIFACT = "Dockerfile"

# BuildArtifactTypeValue
SOURCE_DIRECTORY_BUILD_ARTIFACT = "SourceCode"

# TargetInfoArtifactTypeValue
K8S_CLUSTER_ARTIFACT = "KubernetesCluster"

# TargetArtifactTypeValue
HELM = "Helm"
YAMLS = "Yamls"
KNATIVE = "Knative"

_CONVERTED_SOURCE_ARTIFACT_KEYS = ["Kubernetes", "Knative", "DockerCompose", "CfManifest",
                                   "CfRunningManifest", "SourceCode", "Dockerfile"]
_CONVERTED_TARGET_OPTION_TYPES = [NEW_DOCKERFILE, REUSE_DOCKERFILE, S2I]


class RepoInfo:
    __slots__ = ("git_repo_dir", "git_repo_url", "git_repo_branch", "target_path")

    def __init__(self, git_repo_dir="", git_repo_url="", git_repo_branch="", target_path=""):
        self.git_repo_dir = git_repo_dir
        self.git_repo_url = git_repo_url
        self.git_repo_branch = git_repo_branch
        self.target_path = target_path

    def is_zero(self):
        return not (self.git_repo_dir or self.git_repo_url or self.git_repo_branch or self.target_path)

    def to_yaml(self):
        return {"gitRepoDir": self.git_repo_dir, "gitRepoURL": self.git_repo_url,
                "gitRepoBranch": self.git_repo_branch, "targetPath": self.target_path}

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        return cls(as_str(d.get("gitRepoDir")), as_str(d.get("gitRepoURL")),
                   as_str(d.get("gitRepoBranch")), as_str(d.get("targetPath")))

    def __eq__(self, o):
        return isinstance(o, RepoInfo) and self.to_yaml() == o.to_yaml()

    def copy(self):
        return RepoInfo(self.git_repo_dir, self.git_repo_url, self.git_repo_branch, self.target_path)

    def __repr__(self):
        return "RepoInfo(%r)" % self.to_yaml()


class Service:
    """A plan service option (``types/plan/plan.go:190-215``)."""

    def __init__(self, service_name="", translation_type=""):
        self.service_name = service_name
        self.service_rel_path = ""
        self.image = ""
        self.translation_type = translation_type
        self.container_build_type = ""
        self.source_types = []
        self.target_options = []
        self.source_artifacts = {}
        self.build_artifacts = {}
        self.update_container_build_pipeline = False
        self.update_deploy_pipeline = False
        self.repo_info = RepoInfo()

    @classmethod
    def new(cls, service_name, translation_type):
        """``plantypes.NewService``."""
        s = cls(service_name, translation_type)
        s.service_rel_path = "/" + service_name
        s.image = service_name + ":latest"
        s.container_build_type = REUSE
        return s

    # -- encoding ------------------------------------------------------------
    def to_yaml(self):
        d = {"serviceName": self.service_name}
        if self.service_rel_path:
            d["serviceRelPath"] = self.service_rel_path
        d["image"] = self.image
        d["translationType"] = self.translation_type
        d["containerBuildType"] = self.container_build_type
        d["sourceType"] = list(self.source_types) if self.source_types is not None else None
        if self.target_options:
            d["targetOptions"] = list(self.target_options)
        d["sourceArtifacts"] = GoMap({k: list(v) if v is not None else None
                                      for k, v in self.source_artifacts.items()}) if self.source_artifacts is not None else None
        if self.build_artifacts:
            d["buildArtifacts"] = GoMap({k: list(v) if v is not None else None for k, v in self.build_artifacts.items()})
        d["updateContainerBuildPipeline"] = self.update_container_build_pipeline
        d["updateDeployPipeline"] = self.update_deploy_pipeline
        if not self.repo_info.is_zero():
            d["repoInfo"] = self.repo_info.to_yaml()
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        s = cls()
        s.service_name = as_str(d.get("serviceName"))
        s.service_rel_path = as_str(d.get("serviceRelPath"))
        s.image = as_str(d.get("image"))
        s.translation_type = as_str(d.get("translationType"))
        s.container_build_type = as_str(d.get("containerBuildType"))
        s.source_types = as_str_list(d.get("sourceType")) if d.get("sourceType") is not None else []
        s.target_options = as_str_list(d.get("targetOptions"))
        s.source_artifacts = as_str_list_map(d.get("sourceArtifacts"))
        s.build_artifacts = as_str_list_map(d.get("buildArtifacts"))
        s.update_container_build_pipeline = as_bool(d.get("updateContainerBuildPipeline"))
        s.update_deploy_pipeline = as_bool(d.get("updateDeployPipeline"))
        s.repo_info = RepoInfo.from_yaml(d.get("repoInfo"))
        return s

    def copy(self):
        s = common.shallow_copy(self)
        s.source_types = list(self.source_types)
        s.target_options = list(self.target_options)
        s.source_artifacts = {k: list(v) for k, v in self.source_artifacts.items()}
        s.build_artifacts = {k: list(v) for k, v in self.build_artifacts.items()}
        s.repo_info = self.repo_info.copy()
        return s

    def __eq__(self, o):
        return isinstance(o, Service) and self.to_yaml() == o.to_yaml()

    def __repr__(self):
        return "Service(%r)" % (self.to_yaml(),)

    # -- mutation (plan.go:249-370) -------------------------------------------
    def add_source_artifact(self, sat, value):
        self.source_artifacts.setdefault(sat, []).append(value)

    def add_build_artifact(self, bat, value):
        self.build_artifacts.setdefault(bat, []).append(value)

    def add_source_type(self, st):
        if st not in self.source_types:
            self.source_types.append(st)
        return True

    def _add_target_option(self, opt):
        if opt not in self.target_options:
            self.target_options.append(opt)

    def merge(self, new):
        if (self.service_name != new.service_name or self.image != new.image
                or self.translation_type != new.translation_type
                or self.container_build_type != new.container_build_type):
            return False
        a = self.build_artifacts.get(SOURCE_DIRECTORY_BUILD_ARTIFACT) or []
        b = new.build_artifacts.get(SOURCE_DIRECTORY_BUILD_ARTIFACT) or []
        if a and b and a[0] != b[0]:
            return False
        self.update_container_build_pipeline = self.update_container_build_pipeline or new.update_container_build_pipeline
        self.update_deploy_pipeline = self.update_deploy_pipeline or new.update_deploy_pipeline
        for st in new.source_types:
            self.add_source_type(st)
        for t in new.target_options:
            self._add_target_option(t)
        for k, v in new.source_artifacts.items():
            if k in self.source_artifacts:
                self.source_artifacts[k] = common.merge_string_slices(self.source_artifacts[k], v)
            else:
                self.source_artifacts[k] = list(v)
        for k, v in new.build_artifacts.items():
            if k in self.build_artifacts:
                self.build_artifacts[k] = common.merge_string_slices(self.build_artifacts[k], v)
            else:
                self.build_artifacts[k] = list(v)
        return True

    def gather_git_info(self, path, plan=None):
        """Fill ``repo_info`` from the git repo containing ``path`` (plan.go:218-247).

        Returns (found_repo, error)."""
        import stat
        from ..utils import git
        try:
            st = os.stat(path)
        except OSError as e:
            log.error("Failed to stat the path %r Error %r", path, common.go_path_error(e, "stat"))
            return False, e
        if not stat.S_ISDIR(st.st_mode):
            parent = common.go_dir(path)
            log.debug("The path %r is not a directory. Using %r instead.", path, parent)
            path = parent
        preferred = "upstream"
        err = None
        try:
            remotes = git.remote_names(path)
        except git.GitError as e:
            remotes, err = [], e
        if err is not None or not remotes:
            # %q of a nil error prints %!q(<nil>)
            log.debug("No remotes found at path %r Error: %s", path, log.go_quote(str(err)) if err else "%!q(<nil>)")
        elif not common.is_string_present(remotes, preferred):
            preferred = "origin" if common.is_string_present(remotes, "origin") else remotes[0]
        try:
            urls, branch, repo_dir = git.repo_details(path, preferred)
        except git.GitError as e:
            log.debug("Failed to get the git repo at path %r Error: %r", path, str(e))
            return False, e
        self.repo_info.git_repo_branch = branch
        if not urls:
            log.debug("The git repo at path %r has no remotes set.", path)
        else:
            self.repo_info.git_repo_url = urls[0]
        self.repo_info.git_repo_dir = repo_dir
        return True, None


class KubernetesOutput:
    def __init__(self):
        self.registry_url = ""
        self.registry_namespace = ""
        self.artifact_type = YAMLS
        self.target_cluster_type = DEFAULT_CLUSTER_TYPE
        self.target_cluster_path = ""
        self.ignore_unsupported_kinds = False

    def is_zero(self):
        return not (self.registry_url or self.registry_namespace or self.artifact_type
                    or self.target_cluster_type or self.target_cluster_path or self.ignore_unsupported_kinds)

    def to_yaml(self):
        d = {}
        if self.registry_url:
            d["registryURL"] = self.registry_url
        if self.registry_namespace:
            d["registryNamespace"] = self.registry_namespace
        d["artifactType"] = self.artifact_type
        tc = {}
        if self.target_cluster_type:
            tc["type"] = self.target_cluster_type
        if self.target_cluster_path:
            tc["path"] = self.target_cluster_path
        if tc:
            d["targetCluster"] = tc
        if self.ignore_unsupported_kinds:
            d["ignoreUnsupportedKinds"] = True
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        k = cls()
        k.registry_url = as_str(d.get("registryURL"))
        k.registry_namespace = as_str(d.get("registryNamespace"))
        k.artifact_type = as_str(d.get("artifactType"))
        tc = as_map(d.get("targetCluster"))
        k.target_cluster_type = as_str(tc.get("type"))
        k.target_cluster_path = as_str(tc.get("path"))
        k.ignore_unsupported_kinds = as_bool(d.get("ignoreUnsupportedKinds"))
        return k

    def merge(self, new):
        """``KubernetesOutput.Merge`` (plan.go:102-119)."""
        if new.is_zero():
            return
        if new.registry_url:
            self.registry_url = new.registry_url
        if new.registry_namespace:
            self.registry_namespace = new.registry_namespace
        self.artifact_type = new.artifact_type
        self.ignore_unsupported_kinds = new.ignore_unsupported_kinds
        if new.target_cluster_type:
            self.target_cluster_type = new.target_cluster_type
            self.target_cluster_path = new.target_cluster_path

    def copy(self):
        return common.shallow_copy(self)


class Plan:
    """``kind: Plan`` document."""

    def __init__(self):
        self.api_version = SCHEME_GROUP_VERSION
        self.kind = PLAN_KIND
        self.name = DEFAULT_PROJECT_NAME
        self.root_dir = ""
        self.k8s_files = []
        self.qa_caches = []
        self.services = {}
        self.target_info_artifacts = {}
        self.kubernetes = KubernetesOutput()

    # -- encoding ------------------------------------------------------------
    def to_yaml(self):
        d = {}
        if self.api_version:
            d["apiVersion"] = self.api_version
        d["kind"] = self.kind
        if self.name:
            d["metadata"] = {"name": self.name}
        inputs = {"rootDir": self.root_dir}
        if self.k8s_files:
            inputs["kubernetesYamls"] = list(self.k8s_files)
        if self.qa_caches:
            inputs["qaCaches"] = list(self.qa_caches)
        inputs["services"] = GoMap({k: [s.to_yaml() for s in v] for k, v in self.services.items()})
        if self.target_info_artifacts:
            inputs["targetInfoArtifacts"] = GoMap({k: list(v) for k, v in self.target_info_artifacts.items()})
        d["spec"] = {"inputs": inputs, "outputs": {"kubernetes": self.kubernetes.to_yaml()}}
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        p = cls()
        p.api_version = as_str(d.get("apiVersion"))
        p.kind = as_str(d.get("kind"))
        p.name = as_str(as_map(d.get("metadata")).get("name"))
        spec = as_map(d.get("spec"))
        inputs = as_map(spec.get("inputs"))
        p.root_dir = as_str(inputs.get("rootDir"))
        p.k8s_files = as_str_list(inputs.get("kubernetesYamls"))
        p.qa_caches = as_str_list(inputs.get("qaCaches"))
        p.services = {as_str(k): [Service.from_yaml(x) for x in as_list(v)]
                      for k, v in as_map(inputs.get("services")).items()}
        p.target_info_artifacts = as_str_list_map(inputs.get("targetInfoArtifacts"))
        p.kubernetes = KubernetesOutput.from_yaml(as_map(spec.get("outputs")).get("kubernetes"))
        return p

    def copy(self):
        """Deep copy (the reference round-trips through YAML)."""
        p = Plan.from_yaml(yamlio.load_raw(yamlio.dump(self.to_yaml())))
        return p

    def __eq__(self, o):
        return isinstance(o, Plan) and self.to_yaml() == o.to_yaml()

    # -- services --------------------------------------------------------------
    def add_services_to_plan(self, services):
        """``Plan.AddServicesToPlan`` (plan.go:373-396)."""
        for service in services:
            existing = self.services.get(service.service_name)
            if existing is None:
                existing = self.services[service.service_name] = []
                log.debug("Added new service to plan : %s", service.service_name)
            merged = False
            for es in existing:
                if es.merge(service):
                    merged = True
            if not merged:
                existing.append(service)

    # -- paths -------------------------------------------------------------------
    def get_relative_path(self, abs_path):
        if abs_path == "":
            return abs_path
        if not os.path.isabs(abs_path):
            log.debug("The input path %r is not an absolute path. Cannot make it relative to the root directory.",
                      abs_path)
            return abs_path
        if is_assets_path(abs_path):
            return common.go_rel(settings.temp_path, abs_path)
        return common.go_rel(self.root_dir, abs_path)

    def get_absolute_path(self, rel_path):
        if rel_path == "":
            return rel_path
        if os.path.isabs(rel_path):
            log.debug("The input path %r is not an relative path. Cannot make it absolute.", rel_path)
            return rel_path
        if is_assets_path(rel_path):
            return common.go_join(settings.temp_path, rel_path)
        return common.go_join(self.root_dir, rel_path)

    def set_root_dir(self, root_dir):
        """Re-root every non-asset absolute path (planutils.go:214-237)."""
        old = self.root_dir

        def conv(p):
            if p == "" or not os.path.isabs(p) or is_assets_path(p):
                return p
            return common.go_join(root_dir, common.go_rel(old, p))
        _convert_paths(self, conv)
        self.root_dir = root_dir


def is_assets_path(path):
    if os.path.isabs(path):
        return path.startswith(settings.temp_path)
    return path.split(os.sep)[0] == ASSETS_DIR


def _convert_paths(plan, conv):
    """Apply ``conv`` to every path field selected by the reference's m2kpath tags."""
    plan.k8s_files = [conv(p) for p in plan.k8s_files]
    plan.qa_caches = [conv(p) for p in plan.qa_caches]
    plan.target_info_artifacts = {k: [conv(p) for p in v] for k, v in plan.target_info_artifacts.items()}
    plan.kubernetes.target_cluster_path = conv(plan.kubernetes.target_cluster_path)
    for services in plan.services.values():
        for s in services:
            if common.is_string_present(_CONVERTED_TARGET_OPTION_TYPES, s.container_build_type):
                s.target_options = [conv(p) for p in s.target_options]
            s.source_artifacts = {k: ([conv(p) for p in v] if common.is_string_present(_CONVERTED_SOURCE_ARTIFACT_KEYS, k) else v)
                                  for k, v in s.source_artifacts.items()}
            s.build_artifacts = {k: [conv(p) for p in v] for k, v in s.build_artifacts.items()}
            s.repo_info.git_repo_dir = conv(s.repo_info.git_repo_dir)
            s.repo_info.target_path = conv(s.repo_info.target_path)


def new_plan():
    """``plantypes.NewPlan``."""
    return Plan()


def read_plan(path):
    """Read a plan converting relative paths to absolute (planutils.go:165-178)."""
    try:
        plan = read_document(path, Plan.from_yaml, "PLAN")
    except Exception as e:  # noqa: BLE001 - logged like ReadPlan, then returned to the caller
        log.error("Failed to load the plan file at path %r Error %r", path, common.go_error_text(e))
        raise
    plan.root_dir = common.go_abs(plan.root_dir) if plan.root_dir else os.getcwd()
    _convert_paths(plan, plan.get_absolute_path)
    return plan


def write_plan(path, plan):
    """Write a plan converting absolute paths to relative (planutils.go:191-202)."""
    cp = plan.copy()
    try:
        _convert_paths(cp, cp.get_relative_path)
    except ValueError as e:
        log.error("Error while converting absolute paths to relative. Error: %r", str(e))
    cp.root_dir = os.path.relpath(cp.root_dir, os.getcwd()) if cp.root_dir else cp.root_dir
    common.write_yaml(path, cp.to_yaml())
