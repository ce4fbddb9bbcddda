"""Carried-over Kubernetes/OpenShift YAMLs converted to the kinds the target
cluster supports (reference ``internal/apiresource/deployment.go:105-168``,
``internal/apiresource/service.go`` and ``apiresource.go:58-153``):
DeploymentConfig / ReplicationController / Pod(Always) -> Deployment on
Kubernetes and -> DeploymentConfig on OpenShift, Pod(OnFailure) -> Job,
Ingress -> Route on OpenShift.  Re-created objects replace the loaded ones
wholesale (``merge`` = DeepCopyInto), so source replica counts do not
survive: the replica optimizer's 2 does."""

import os
import shutil

import pytest

from move2kube_amd import api
from move2kube_amd.utils import yamlio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "k8s_conversions")


def _run(tmp_path, monkeypatch, cluster):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = str(tmp_path / "src")
    shutil.copytree(FIXTURE, src)
    cache = tmp_path / "qa.yaml"
    cache.write_text(yamlio.dump({
        "apiVersion": "move2kube.konveyor.io/v1alpha1", "kind": "QACache",
        "spec": {"solutions": [{"description": "Choose the cluster type:",
                                "solution": {"type": "Select", "answer": [cluster]}, "resolved": True}]}}))
    out = os.path.join(api.translate(src, str(tmp_path / "out"), name="conv", qacaches=[str(cache)]), "conv")
    return {f: yamlio.load(open(os.path.join(out, f)).read()) for f in sorted(os.listdir(out))}


WORKLOADS = ("legacy-dc", "old-rc", "lone-pod", "plain-dep")


@pytest.mark.parametrize("cluster,kind,api_version", [("Kubernetes", "Deployment", "apps/v1"),
                                                     ("Openshift", "DeploymentConfig", "apps.openshift.io/v1")])
def test_workload_kinds(tmp_path, monkeypatch, cluster, kind, api_version):
    objs = _run(tmp_path, monkeypatch, cluster)
    for name in WORKLOADS:
        o = objs["%s-%s.yaml" % (name, kind.lower())]
        assert (o["apiVersion"], o["kind"]) == (api_version, kind)
        assert o["spec"]["replicas"] == 2
        assert o["spec"]["template"]["spec"]["restartPolicy"] == "Always"
        assert "%s-service.yaml" % name in objs
    job = objs["batch-pod-job.yaml"]
    assert (job["apiVersion"], job["kind"]) == ("batch/v1", "Job")
    assert job["spec"]["template"]["spec"]["restartPolicy"] == "OnFailure"


def test_ingress_and_openshift_extras(tmp_path, monkeypatch):
    k8s = _run(tmp_path / "k", monkeypatch, "Kubernetes")
    assert "web-ing-ingress.yaml" in k8s and "conv-ingress.yaml" in k8s
    assert not any(f.endswith("-route.yaml") or f.endswith("-imagestream.yaml") for f in k8s)
    ocp = _run(tmp_path / "o", monkeypatch, "Openshift")
    assert not any(f.endswith("-ingress.yaml") for f in ocp)
    route = ocp["web-ing-route.yaml"]
    assert route["spec"]["host"] == "web.example.com" and route["spec"]["to"]["name"] == "plain-dep"
    for name in WORKLOADS:
        assert "%s-imagestream.yaml" % name in ocp and "%s-route.yaml" % name in ocp
