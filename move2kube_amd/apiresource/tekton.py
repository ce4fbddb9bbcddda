"""Tekton CI/CD and RBAC handlers (reference ``internal/apiresource/pipeline.go``,
``eventlistener.go``, ``triggerbinding.go``, ``triggertemplate.go``, ``role.go``,
``rolebinding.go``, ``serviceaccount.go``).

The pipeline clones each repo with the ``git-clone`` task and builds/pushes
every new Dockerfile / reuse-Dockerfile image with ``kaniko``.
"""

from ..models import plan as plantypes
from ..utils import common, log
from ..utils.constants import DEFAULT_REGISTRY_URL
from .base import IAPIResource

PIPELINE = "Pipeline"
EVENT_LISTENER = "EventListener"
TRIGGER_BINDING = "TriggerBinding"
TRIGGER_TEMPLATE = "TriggerTemplate"
ROLE = "Role"
ROLE_BINDING = "RoleBinding"
SERVICE_ACCOUNT = "ServiceAccount"

TEKTON_GV = "tekton.dev/v1beta1"
TRIGGERS_GV = "triggers.tekton.dev/v1alpha1"
RBAC_GV = "rbac.authorization.k8s.io/v1"

DEFAULT_GIT_BRANCH = "master"
GIT_URL_PLACEHOLDER = "<TODO: insert git repo url>"
CONTEXT_PLACEHOLDER = "<TODO: insert path to the directory containing Dockerfile>"
DOCKERFILE_PLACEHOLDER = "<TODO: insert path to the Dockerfile>"
REGISTRY_NAMESPACE_PLACEHOLDER = "<TODO: insert your registry namespace>"


class _PassThrough(IAPIResource):
    kinds = []

    def get_supported_kinds(self):
        return list(self.kinds)

    def convert_to_cluster_supported_kinds(self, obj, supported, others, ir):
        for k in self.get_supported_kinds():
            if common.is_string_present(supported, k):
                return [obj], True
        return None, False


def _str_param(name, value):
    return {"name": name, "value": value}


class Pipeline(_PassThrough):
    kinds = [PIPELINE]

    def create_new_resources(self, ir, supported):
        return [self.create(p, ir) for p in ir.tekton_resources.pipelines]

    @staticmethod
    def create(irp, ir):
        tasks = []
        first = True
        prev = ""
        for i, c in enumerate(ir.containers):
            if c.container_build_type in (plantypes.MANUAL, plantypes.REUSE):
                log.debug("Manual or reuse containerization. We will skip this for CICD.")
                continue
            if c.container_build_type in (plantypes.NEW_DOCKERFILE, plantypes.REUSE_DOCKERFILE):
                clone = "clone-%d" % i
                url = c.repo_info.git_repo_url or GIT_URL_PLACEHOLDER
                branch = c.repo_info.git_repo_branch or DEFAULT_GIT_BRANCH
                clone_task = {"name": clone, "taskRef": {"name": "git-clone"},
                              "workspaces": [{"name": "output", "workspace": irp["workspace_name"]}],
                              "params": [_str_param("url", url), _str_param("revision", branch),
                                         _str_param("deleteExisting", "true")]}
                if not first:
                    clone_task["runAfter"] = [prev]
                image = c.image_names[0]
                df_path, ctx = DOCKERFILE_PLACEHOLDER, CONTEXT_PLACEHOLDER
                if c.repo_info.git_repo_dir:
                    try:
                        rel = common.go_rel(c.repo_info.git_repo_dir, c.repo_info.target_path)
                        df_path = rel
                        ctx = common.go_dir(rel)
                    except ValueError as e:
                        log.debug("ERROR: Failed to make the path %r relative to the path %r Error %r",
                                  c.repo_info.git_repo_dir, c.repo_info.target_path, str(e))
                build = "build-push-%d" % i
                build_task = {"runAfter": [clone], "name": build, "taskRef": {"name": "kaniko"},
                              "workspaces": [{"name": "source", "workspace": irp["workspace_name"]}],
                              "params": [_str_param("IMAGE", "$(params.image-registry-url)/" + image),
                                         _str_param("DOCKERFILE", df_path), _str_param("CONTEXT", ctx)]}
                tasks.extend([clone_task, build_task])
                first = False
                prev = build
            elif c.container_build_type == plantypes.S2I:
                log.debug("S2I not yet supported for Tekton")
            elif c.container_build_type == plantypes.CNB:
                log.debug("CNB not yet supported for Tekton")
            else:
                log.error("Unknown containerization method: %s", c.container_build_type)
        return {"kind": PIPELINE, "apiVersion": TEKTON_GV, "metadata": {"name": irp["name"]},
                "spec": {"params": [{"name": "image-registry-url",
                                     "description": "registry-domain/namespace where the output image should be pushed.",
                                     "type": "string"}],
                         "workspaces": [{"name": irp["workspace_name"],
                                         "description": ("This workspace will receive the cloned git repo and be passed "
                                                         "to the kaniko task for building the image.")}],
                         "tasks": tasks}}


class EventListener(_PassThrough):
    kinds = [EVENT_LISTENER]

    def create_new_resources(self, ir, supported):
        out = []
        for el in ir.tekton_resources.event_listeners:
            out.append({"kind": EVENT_LISTENER, "apiVersion": TRIGGERS_GV, "metadata": {"name": el["name"]},
                        "spec": {"serviceAccountName": el["service_account_name"],
                                 "triggers": [{"bindings": [{"ref": el["trigger_binding_name"]}],
                                               "template": {"name": el["trigger_template_name"]}}]}})
        return out


class TriggerBinding(_PassThrough):
    kinds = [TRIGGER_BINDING]

    def create_new_resources(self, ir, supported):
        return [{"kind": TRIGGER_BINDING, "apiVersion": TRIGGERS_GV, "metadata": {"name": tb["name"]}}
                for tb in ir.tekton_resources.trigger_bindings]


class TriggerTemplate(_PassThrough):
    kinds = [TRIGGER_TEMPLATE]

    def create_new_resources(self, ir, supported):
        return [self.create(tt, ir) for tt in ir.tekton_resources.trigger_templates]

    @staticmethod
    def create(tt, ir):
        url = ir.kubernetes.registry_url or DEFAULT_REGISTRY_URL
        ns = ir.kubernetes.registry_namespace or REGISTRY_NAMESPACE_PLACEHOLDER
        run = {"kind": "PipelineRun", "apiVersion": TEKTON_GV, "metadata": {"name": tt["pipeline_run_name"]},
               "spec": {"pipelineRef": {"name": tt["pipeline_name"]},
                        "serviceAccountName": tt["service_account_name"],
                        "workspaces": [{"name": tt["workspace_name"], "volumeClaimTemplate": {
                            "spec": {"storageClassName": tt["storage_class_name"], "accessModes": ["ReadWriteOnce"],
                                     "resources": {"requests": {"storage": "1Gi"}}}}}],
                        "params": [_str_param("image-registry-url", url + "/" + ns)]}}
        return {"kind": TRIGGER_TEMPLATE, "apiVersion": TRIGGERS_GV, "metadata": {"name": tt["name"]},
                "spec": {"resourcetemplates": [run]}}


class Role(_PassThrough):
    kinds = [ROLE]

    def create_new_resources(self, ir, supported):
        if not common.is_string_present(supported, ROLE):
            log.error("Could not find a valid resource type in cluster to create a role.")
            return []
        out = []
        for r in ir.roles:
            out.append({"kind": ROLE, "apiVersion": RBAC_GV, "metadata": {"name": r.name},
                        "rules": [{"apiGroups": p.api_groups, "resources": p.resources, "verbs": p.verbs}
                                  for p in r.policy_rules]})
        return out


class RoleBinding(_PassThrough):
    kinds = [ROLE_BINDING]

    def create_new_resources(self, ir, supported):
        if not common.is_string_present(supported, ROLE_BINDING):
            log.error("Could not find a valid resource type in cluster to create a role binding.")
            return []
        return [{"kind": ROLE_BINDING, "apiVersion": RBAC_GV, "metadata": {"name": rb.name},
                 "subjects": [{"kind": SERVICE_ACCOUNT, "name": rb.service_account_name}],
                 "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": ROLE, "name": rb.role_name}}
                for rb in ir.role_bindings]


class ServiceAccount(_PassThrough):
    kinds = [SERVICE_ACCOUNT]

    def create_new_resources(self, ir, supported):
        if not common.is_string_present(supported, SERVICE_ACCOUNT):
            log.error("Could not find a valid resource type in cluster to create a service account.")
            return []
        out = []
        for sa in ir.service_accounts:
            obj = {"kind": SERVICE_ACCOUNT, "apiVersion": "v1", "metadata": {"name": sa.name}}
            if sa.secret_names:
                obj["secrets"] = [{"name": s} for s in sa.secret_names]
            out.append(obj)
        return out

