"""The Kubernetes and Knative API resource sets as source translators, off the
happy path (reference ``internal/apiresourceset/k8sapiresourceset.go:80-150``
and ``knativeapiresourceset.go:65-130``): each plan service whose file cannot
be read, decoded or used is logged with the reference's line and skipped."""

import os

import pytest

import logparse
from move2kube_amd.apiresourceset import K8sAPIResourceSet, KnativeAPIResourceSet
from move2kube_amd.models import plan as plantypes
from move2kube_amd.utils import log

K8S_SCHEME = "github.com/konveyor/move2kube/internal/apiresourceset/k8sapiresourceset.go:46"

DEPLOYMENT = """apiVersion: apps/v1
kind: Deployment
metadata: {name: web}
spec:
  template:
    spec:
      containers:
      - name: web
        image: nginx
        ports: [{containerPort: 8080, name: http}, {containerPort: 9090}]
"""

KSVC = """apiVersion: serving.knative.dev/v1
kind: Service
metadata: {name: hello}
spec:
  template:
    spec:
      containerConcurrency: 4
      timeoutSeconds: 30
      containers: [{image: hello}]
"""


@pytest.fixture(autouse=True)
def _quiet():
    log.set_verbose(False)
    yield
    log.set_verbose(False)


def _svc(name, artifact, path):
    s = plantypes.Service(name)
    if path is not None:
        s.source_artifacts[artifact] = [str(path)]
    return s


def _plan(root):
    p = plantypes.new_plan()
    p.root_dir = str(root)
    return p


def test_k8s_translate(tmp_path, capsys):
    (tmp_path / "dep.yaml").write_text(DEPLOYMENT)
    (tmp_path / "cm.yaml").write_text("apiVersion: v1\nkind: ConfigMap\nmetadata: {name: c}\n")
    (tmp_path / "nope.yaml").write_text("apiVersion: v1\nkind: Nope\n")
    art = plantypes.K8S_FILE_ARTIFACT
    services = [_svc("web", art, tmp_path / "dep.yaml"), _svc("none", art, None),
                _svc("gone", art, tmp_path / "gone.yaml"), _svc("cm", art, tmp_path / "cm.yaml"),
                _svc("nope", art, tmp_path / "nope.yaml")]
    ir = K8sAPIResourceSet().translate(services, _plan(tmp_path))
    assert list(ir.services) == ["web"]
    web = ir.services["web"]
    assert [c["image"] for c in web.pod_spec["containers"]] == ["nginx"]
    assert [(f.service_port.name, f.service_port.number, f.pod_port.number) for f in web.port_forwardings] == [
        ("http", 8080, 8080), ("", 9090, 9090)]
    err = capsys.readouterr().err
    assert logparse.logged(err, "No k8s artifacts found in service none", "warning")
    gone = tmp_path / "gone.yaml"
    assert logparse.logged(err, 'Unable to read the k8s file at path "%s" Error: "open %s: no such file or directory"'
                           % (gone, gone), "error")
    assert logparse.logged(err, 'Failed to get the pod specification for the k8s file at path "%s" Error: '
                           '"Incompatible object type"' % (tmp_path / "cm.yaml"), "error")
    assert logparse.logged(err, 'Failed to decode the k8s file at path "%s" Error: "no kind \\"Nope\\" is registered '
                           'for version \\"v1\\" in scheme \\"%s\\""' % (tmp_path / "nope.yaml", K8S_SCHEME), "error")


def test_k8s_service_options_skip_what_is_not_a_workload(tmp_path, capsys):
    (tmp_path / "dep.yaml").write_text(DEPLOYMENT)
    (tmp_path / "cm.yml").write_text("apiVersion: v1\nkind: ConfigMap\nmetadata: {name: c}\n")
    (tmp_path / "bad.yaml").write_text("a: [\n")
    (tmp_path / "dir.yaml").mkdir()
    log.set_verbose(True)
    services = K8sAPIResourceSet().get_service_options(str(tmp_path), _plan(tmp_path))
    assert [(s.service_name, s.source_artifacts[plantypes.K8S_FILE_ARTIFACT]) for s in services] == [
        ("web", [str(tmp_path / "dep.yaml")])]
    assert services[0].translation_type == plantypes.KUBE2KUBE and services[0].update_deploy_pipeline
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, 'Failed to decode the file at path "%s" as a k8s file. Error: '
                                      % (tmp_path / "bad.yaml"), "debug")


def test_yaml_listing_failure_is_logged_and_raised(tmp_path, capsys, monkeypatch):
    from move2kube_amd.utils import common

    def boom(*a):
        raise OSError(13, "Permission denied", str(tmp_path))
    monkeypatch.setattr(common, "get_files_by_ext", boom)
    with pytest.raises(OSError):
        K8sAPIResourceSet().get_service_options(str(tmp_path), _plan(tmp_path))
    assert logparse.logged_containing(capsys.readouterr().err, 'Unable to fetch yaml files at path "%s" Error: '
                                      % tmp_path, "error")


def test_knative_translate(tmp_path, capsys):
    (tmp_path / "ksvc.yaml").write_text(KSVC)
    (tmp_path / "conf.yaml").write_text("apiVersion: serving.knative.dev/v1\nkind: Configuration\n"
                                        "metadata: {name: c}\n")
    (tmp_path / "dep.yaml").write_text(DEPLOYMENT)
    art = plantypes.KNATIVE_FILE_ARTIFACT
    services = [_svc("hello", art, tmp_path / "ksvc.yaml"), _svc("none", art, None),
                _svc("gone", art, tmp_path / "gone.yaml"), _svc("conf", art, tmp_path / "conf.yaml"),
                _svc("dep", art, tmp_path / "dep.yaml")]
    ir = KnativeAPIResourceSet().translate(services, _plan(tmp_path))
    assert list(ir.services) == ["hello"]
    # the Knative-only fields of the revision spec are not pod-spec fields
    assert ir.services["hello"].pod_spec == {"containers": [{"image": "hello"}]}
    err = capsys.readouterr().err
    assert logparse.logged(err, "No knative artifacts found in service none", "warning")
    assert logparse.logged_containing(err, 'Unable to read the knative file at path "%s" Error: "open '
                                      % (tmp_path / "gone.yaml"), "error")
    assert logparse.logged(err, 'The knative file at path "%s" does not contain the required type. Expected: '
                                "*v1.Service Actual: *v1.Configuration" % (tmp_path / "conf.yaml"), "error")
    assert logparse.logged_containing(err, 'Failed to decode the knative file at path "%s" Error: "no kind '
                                      % (tmp_path / "dep.yaml"), "error")


def test_knative_service_options_follow_the_compat_mode(tmp_path, monkeypatch):
    """the reference's inverted check finds no Knative
    service; "fixed" finds them."""
    from move2kube_amd.utils.constants import settings
    (tmp_path / "ksvc.yaml").write_text(KSVC)
    (tmp_path / "dep.yaml").write_text(DEPLOYMENT)
    assert KnativeAPIResourceSet().get_service_options(str(tmp_path), _plan(tmp_path)) == []
    monkeypatch.setattr(settings, "compat", "fixed")
    (s,) = KnativeAPIResourceSet().get_service_options(str(tmp_path), _plan(tmp_path))
    assert s.service_name == "hello" and s.source_types == [plantypes.KNATIVE_SOURCE]
    assert s.source_artifacts[plantypes.KNATIVE_FILE_ARTIFACT] == [os.path.join(str(tmp_path), "ksvc.yaml")]
