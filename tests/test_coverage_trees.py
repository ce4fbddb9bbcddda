"""Expected trees for the capability surface beyond the five BASELINE
configurations (``benchmarks/refconfigs.py:COVERAGE_CONFIGS``):

* ``profiles/<P>``: ``samples/`` in Yamls mode on each of the seven built-in
  cluster profiles (``internal/metadata/clusters/*.yaml``);
* ``artifacts/*``: Knative on the Kubernetes and Openshift profiles, Helm on
  Kubernetes (``knativetransformer.go:46-101``, ``k8stransformer.go:44-293``);
* ``carried-over/<P>``: old-version Kubernetes/OpenShift YAMLs
  (``tests/fixtures/carried_over``) through the K8sFiles loader, the kind
  handlers and the GroupVersion conversion of ``k8stransformer.go:106-141``;
* ``git-repos``: source trees that are git repos with remotes
  (``dockerfile2kube.go:146-263``, ``types/plan/plan.go:232-272``,
  ``tektonapiresourceset.go:203-286``, ``pipeline.go:78-143``);
* ``storage-class``: two compose services with a named volume each
  (``v3.go:405-470``, ``storagecustomizer.go:40-80``);
* ``compat-fixed/*``: ``M2K_COMPAT=fixed`` where it changes bytes
  (``cf``, ``storage-class``; DEVIATIONS.md section 5).

The trees were written by ``python benchmarks/refconfigs.py --write`` and
audited file class by file class (``tests/golden/reference/PROVENANCE.md``);
a test run never rewrites them.
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402

from move2kube_amd.utils import yamlio  # noqa: E402


def _run(name, work):
    run = refconfigs.Run(name, str(work)).prepare()
    undo = run.apply_env()
    try:
        with run.session() as s:
            out = run.step(s)
    finally:
        undo()
    return run, out


@pytest.mark.parametrize("name", sorted(refconfigs.COVERAGE_CONFIGS))
def test_coverage_tree_matches_expected(name, tmp_path):
    run, out = _run(name, tmp_path)
    golden = refconfigs.golden_dir(name)
    assert os.path.isdir(golden), golden
    assert refconfigs.diff_files(out, golden, work=run.work) == []


# files in which a fixed-mode tree differs from its reference-mode counterpart
# (DEVIATIONS.md section 5)
COMPAT_FIXED = {
    "compat-fixed/cf": (os.path.join(refconfigs.GOLDEN_REF, "cf"), {
        "Manualimages.md", "NOTES.txt", "cicd/myproject-clone-build-push-pipeline.yaml", "docker-compose.yaml",
        "m2kqacache.yaml", "myproject/app2-deployment.yaml", "myproject/app2-service.yaml",
        "myproject/myproject-ingress.yaml"}),
    "compat-fixed/storage-class": (refconfigs.golden_dir("storage-class"), {
        "myproject/cachedata-persistentvolumeclaim.yaml", "myproject/dbdata-persistentvolumeclaim.yaml"}),
}
_WORKLOADS = {"myproject/db-statefulset.yaml", "myproject/legacy-beta1-deployment.yaml",
              "myproject/legacy-ext-deployment.yaml", "myproject/node-agent-daemonset.yaml",
              "myproject/old-agent-daemonset.yaml"}
for _p, _ing in (("Kubernetes", {"beta-ing", "old-ing"}), ("Openshift", {"beta-ing"}),
                 ("IBM-Openshift", {"beta-ing"}), ("AWS-EKS", {"new-ing", "old-ing", "web"})):
    COMPAT_FIXED["compat-fixed/carried-over/" + _p] = (
        refconfigs.golden_dir("carried-over/" + _p), _WORKLOADS | {"myproject/%s-ingress.yaml" % i for i in _ing})
for _p in ("AWS-EKS", "Azure-AKS", "GCP-GKE"):
    COMPAT_FIXED["compat-fixed/profiles/" + _p] = (refconfigs.golden_dir("profiles/" + _p),
                                                 {"myproject/myproject-ingress.yaml"})


@pytest.mark.parametrize("name", sorted(COMPAT_FIXED))
def test_compat_fixed_trees_differ_only_where_documented(name):
    counterpart, files = COMPAT_FIXED[name]
    assert refconfigs.diff_files(refconfigs.golden_dir(name), counterpart) == sorted(files)
    dev = open(os.path.join(refconfigs.GOLDEN_REF, "DEVIATIONS.md")).read()
    assert "`%s`" % name in dev.split("## 5.")[1].split("## 6.")[0]
    fixed = refconfigs.golden_dir(name)
    if name == "compat-fixed/cf":
        with open(os.path.join(fixed, "Manualimages.md")) as f:
            assert f.read().rstrip().endswith("app2:latest")
    elif name == "compat-fixed/storage-class":
        for f in files:
            with open(os.path.join(fixed, f)) as fh:
                assert yamlio.load(fh.read())["spec"]["storageClassName"] == "default"
    else:   # objects relabelled to a version the profile lists, workloads with a selector
        from move2kube_amd import metadata
        from move2kube_amd.models import plan as plantypes
        profile = name.rsplit("/", 1)[1]
        spec = metadata.ClusterMDLoader.get_clusters(plantypes.new_plan())[profile].spec
        for f in files:
            with open(os.path.join(fixed, f)) as fh:
                obj = yamlio.load(fh.read())
            assert obj["apiVersion"] in (spec.get_supported_versions(obj["kind"]) or []), (f, obj["apiVersion"])
            if obj["kind"] in ("Deployment", "DaemonSet", "StatefulSet"):
                assert obj["spec"]["selector"]["matchLabels"], f


def _objects(name, sub="myproject"):
    root = os.path.join(refconfigs.golden_dir(name), sub)
    return {f: yamlio.load(open(os.path.join(root, f)).read()) for f in sorted(os.listdir(root))
            if f.endswith(".yaml")}


def test_every_profile_and_artifact_type_has_a_tree_or_a_reason():
    """(artifact type x profile) combinations the curator can produce: each has
    an expected tree here or in the BASELINE set, or a named reason in
    DEVIATIONS.md §7."""
    have = set(refconfigs.COVERAGE_CONFIGS) | set(refconfigs.CONFIGS)
    for p in refconfigs.PROFILES:
        assert "profiles/" + p in have
    assert {"helm-openshift", "artifacts/helm-kubernetes", "artifacts/knative-kubernetes",
            "artifacts/knative-openshift"} <= have
    dev = open(os.path.join(refconfigs.GOLDEN_REF, "DEVIATIONS.md")).read()
    assert "Helm or Knative on the other five profiles" in dev


def test_no_tree_writes_an_invalid_selector():
    """``selector: null`` would make an apps/v1 workload invalid; the reference
    never relabels across groups, so no expected tree has one."""
    for dp, _dn, fns in os.walk(refconfigs.GOLDEN_COVERAGE):
        for fn in fns:
            if fn.endswith(".yaml"):
                assert b"selector: null" not in open(os.path.join(dp, fn), "rb").read(), os.path.join(dp, fn)


@pytest.mark.parametrize("profile", ["AWS-EKS", "Azure-AKS", "GCP-GKE"])
def test_generated_ingress_keeps_networking_v1_where_profile_prefers_v1beta1(profile):
    """networking.k8s.io/v1 -> v1beta1 has no conversion function between the
    two external packages ("unknown conversion" in apimachinery v0.19.4), so the
    original v1 object is written."""
    ing = _objects("profiles/" + profile)["myproject-ingress.yaml"]
    assert ing["apiVersion"] == "networking.k8s.io/v1"
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["backend"]["service"]["name"]


@pytest.mark.parametrize("profile", ["Kubernetes", "Openshift", "AWS-EKS", "IBM-Openshift"])
def test_carried_over_versions(profile):
    objs = _objects("carried-over/" + profile)
    gv = {f: o["apiVersion"] for f, o in objs.items()}
    # cross-group targets (extensions -> apps) are not-registered errors: original kept
    assert gv["legacy-ext-deployment.yaml"] == "extensions/v1beta1"
    assert "selector" not in objs["legacy-ext-deployment.yaml"]["spec"]
    assert gv["old-agent-daemonset.yaml"] == "extensions/v1beta1"
    assert objs["old-agent-daemonset.yaml"]["spec"]["templateGeneration"] == 3
    # same group, other version: no conversion function (apimachinery v0.19.4
    # has no reflection fallback), so every input object keeps its apiVersion
    assert gv["legacy-beta1-deployment.yaml"] == "apps/v1beta1"
    assert objs["legacy-beta1-deployment.yaml"]["spec"]["rollbackTo"] == {"revision": 1}
    assert gv["node-agent-daemonset.yaml"] == "apps/v1beta2"
    assert gv["nightly-cronjob.yaml"] == "batch/v2alpha1"
    assert gv["db-statefulset.yaml"] == "apps/v1beta1"
    assert gv["web-hpa-horizontalpodautoscaler.yaml"] == "autoscaling/v2beta2"
    assert gv["old-ing-ingress.yaml"] == "extensions/v1beta1"
    assert gv["beta-ing-ingress.yaml"] == "networking.k8s.io/v1beta1"
    # RBAC never crosses into authorization.openshift.io (or back)
    assert gv["reader-role.yaml"] == "rbac.authorization.k8s.io/v1"
    assert gv["oc-reader-role.yaml"] == "authorization.openshift.io/v1"
    openshift = profile.endswith("Openshift")
    assert gv["reader-binding-rolebinding.yaml"] == "rbac.authorization.k8s.io/v1beta1"
    if openshift:
        assert gv["new-ing-route.yaml"] == "route.openshift.io/v1"      # Ingress v1 -> Route
        assert objs["web-deploymentconfig.yaml"]["kind"] == "DeploymentConfig"
    else:
        assert gv["new-ing-ingress.yaml"] == "networking.k8s.io/v1"
        assert gv["web-deployment.yaml"] == "apps/v1"


def test_git_repos_tree():
    root = refconfigs.golden_dir("git-repos")
    objs = _objects("git-repos")
    # Dockerfile2Kube: one repo with two Dockerfiles -> <repo>-<bucket>; one with one -> <repo>
    for svc in ("move2kube-demos-frontend", "move2kube-demos-backend", "internal-tools"):
        assert "%s-deployment.yaml" % svc in objs
    cicd = os.path.join(root, "cicd")
    gh = yamlio.load(open(os.path.join(cicd, "myproject-git-repo-github-com-secret.yaml")).read())
    assert gh["stringData"]["known_hosts"].startswith("github.com ssh-rsa ")
    other = yamlio.load(open(os.path.join(cicd, "myproject-git-repo-git-corp-invalid-secret.yaml")).read())
    assert other["metadata"]["annotations"] == {"tekton.dev/git-0": "git.corp.invalid"}
    assert other["stringData"]["known_hosts"] == "<TODO: insert the known host keys for your git repo>"
    pipe = yamlio.load(open(os.path.join(cicd, "myproject-clone-build-push-pipeline.yaml")).read())
    params = {}
    for t in pipe["spec"]["tasks"]:
        params[t["name"]] = {p["name"]: p["value"] for p in t.get("params", [])}
    clones = [v for k, v in sorted(params.items()) if k.startswith("clone-")]
    builds = [v for k, v in sorted(params.items()) if k.startswith("build-push-")]
    # the upstream remote wins over origin; the branch comes from packed-refs
    assert {"url": "https://git.corp.invalid/tools/internal-tools.git", "revision": "develop",
            "deleteExisting": "true"} in clones
    assert {"url": "git@github.com:konveyor/move2kube-demos.git", "revision": "main",
            "deleteExisting": "true"} in clones
    dockerfiles = sorted(b["DOCKERFILE"] for b in builds)
    assert dockerfiles == ["<TODO: insert path to the Dockerfile>", "Dockerfile",
                           "backend/Dockerfile", "frontend/Dockerfile"]
    cache = open(os.path.join(root, "m2kqacache.yaml")).read()
    assert "Unable to find the public key for the domain git.corp.invalid" in cache
    assert "$WORK/home/.ssh" in cache


def test_plan_records_repo_info(tmp_path):
    run = refconfigs.Run("git-repos", str(tmp_path)).prepare()
    from move2kube_amd import api
    undo = run.apply_env()
    try:
        with api.Session(qaskip=True) as s:
            plan = s.plan(run.src, "myproject")
    finally:
        undo()
    by_name = {name: svcs[0] for name, svcs in plan.services.items()}
    fe = by_name["move2kube-demos-frontend"].repo_info
    assert fe.git_repo_url == "git@github.com:konveyor/move2kube-demos.git"
    assert fe.git_repo_branch == "main"
    assert fe.git_repo_dir == os.path.join(run.src, "move2kube-demos")
    tools = by_name["internal-tools"].repo_info
    assert (tools.git_repo_url, tools.git_repo_branch) == ("https://git.corp.invalid/tools/internal-tools.git",
                                                           "develop")
    node = by_name["nodeapp"].repo_info
    assert node.git_repo_dir == os.path.join(run.src, "move2kube-demos")


def test_kind_conversions_to_the_cluster():
    """coverage/carried-over-kinds: what a target that lacks a kind gets
    (service.go:104-388, storage.go:75-196, deployment.go:66-171)."""
    from move2kube_amd.utils import yamlio

    def obj(profile, name):
        path = os.path.join(refconfigs.golden_dir("carried-over-kinds/" + profile), "myproject", name)
        with open(path) as f:
            return yamlio.load(f.read())
    # Kubernetes: the Route becomes an Ingress, a LoadBalancer Service an
    # Ingress (one rule per port) plus the same Service as ClusterIP
    ing = obj("Kubernetes", "shop-ingress.yaml")
    assert ing["spec"]["rules"][0]["host"] == "shop.example.com"
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["backend"]["service"] == {"name": "shop",
                                                                               "port": {"name": "http"}}
    gw = obj("Kubernetes", "gateway-ingress.yaml")
    assert [r["http"]["paths"][0]["path"] for r in gw["spec"]["rules"]] == ["/gateway/web", "/gateway/admin"]
    assert obj("Kubernetes", "gateway-service.yaml")["spec"]["type"] == "ClusterIP"
    # Openshift: an Ingress with two paths -> two Routes of one name, the last kept
    front = obj("Openshift", "front-route.yaml")
    assert front["spec"]["path"] == "/api" and front["spec"]["to"]["name"] == "gateway"
    assert obj("Openshift", "gateway-route.yaml")["spec"]["port"]["targetPort"] == "admin"
    # minimal profile: no Secret -> ConfigMap with decoded data; no Deployment
    # -> ReplicationController; restart-on-failure workloads -> Pods; Ingress
    # paths -> NodePort Services that replace the carried-over ones
    assert obj("minimal-cluster", "app-secret-configmap.yaml")["data"] == {"password": "s3cr3t"}
    assert obj("minimal-cluster", "legacy-rc-replicationcontroller.yaml")["kind"] == "ReplicationController"
    assert obj("minimal-cluster", "migrate-pod.yaml")["spec"]["restartPolicy"] == "OnFailure"
    assert obj("minimal-cluster", "seed-pod.yaml")["spec"]["restartPolicy"] == "OnFailure"
    svc = obj("minimal-cluster", "gateway-service.yaml")["spec"]
    assert svc == {"ports": [{"name": "web", "port": 0}], "type": "NodePort"}


_FIXED_COUNTERPARTS = {n[len("compat-fixed/"):] for n in COMPAT_FIXED}


@pytest.mark.parametrize("name", sorted(n for n in list(refconfigs.CONFIGS) + list(refconfigs.COVERAGE_CONFIGS)
                                        if not n.startswith("compat-fixed/") and n not in _FIXED_COUNTERPARTS))
def test_fixed_mode_changes_no_other_tree(name, tmp_path):
    """DEVIATIONS section 5 lists every tree ``M2K_COMPAT=fixed`` changes: on
    every other configuration the fixed mode writes the same bytes."""
    run = refconfigs.Run(name, str(tmp_path)).prepare()
    run.extra_env["M2K_COMPAT"] = "fixed"
    undo = run.apply_env()
    try:
        with run.session() as s:
            out = run.step(s)
    finally:
        undo()
    assert refconfigs.diff_files(out, refconfigs.golden_dir(name), work=run.work) == []
