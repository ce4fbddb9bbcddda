"""CfManifest2Kube planning of applications only a collected foundation knows
(reference ``internal/source/cfmanifest2kube.go:187-256``): an app of a
``CfInstanceApps`` file that no manifest covers is planned as Reuse for a
docker image, with the buildpack-matched containerizers of ``CfContainerizers``
files, or as Manual with the reference's warning.  That loop runs once per
file that reads as a manifest - any YAML without ``applications`` does, the
collect outputs included - and never marks its apps covered, so each such
app is planned once per such file, as in the reference.  Translation takes
the replicas, env and ports of the running instance."""

import pytest

import logparse
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source.cfmanifest2kube import CfManifestTranslator
from move2kube_amd.utils import log

HDR = "apiVersion: move2kube.konveyor.io/v1alpha1\n"

INSTANCE_APPS = HDR + """kind: CfInstanceApps
spec:
  applications:
  - name: web
    buildpack: nodejs_buildpack
    instances: 3
    memory: 256
    ports: [9000]
    env: {FROM_INSTANCE: "yes"}
  - name: img
    dockerImage: repo/img:2
  - name: mystery
    detectedBuildpack: cobol_buildpack
  - name: ""
"""

CONTAINERIZERS = HDR + """kind: CfContainerizers
spec:
  buildpackContainerizers:
  - buildpackName: nodejs_buildpack
    containerBuildType: CNB
    targetOptions: [cloudfoundry/cnb:cflinuxfs3]
"""


@pytest.fixture
def tree(tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    (tmp_path / "m2k_collect").mkdir()
    (tmp_path / "m2k_collect" / "instanceapps.yaml").write_text(INSTANCE_APPS)
    (tmp_path / "m2k_collect" / "cfcontainertypes.yaml").write_text(CONTAINERIZERS)
    (tmp_path / "app").mkdir()
    (tmp_path / "app" / "manifest.yml").write_text("applications:\n- name: other\n  buildpack: ruby_buildpack\n")
    plan = plantypes.new_plan()
    plan.root_dir = str(tmp_path)
    log.set_verbose(False)
    return tmp_path, plan


def _by(services):
    out = {}
    for s in services:
        out.setdefault(s.service_name, []).append(s)
    return out


def test_instance_only_apps(tree, capsys):
    root, plan = tree
    got = _by(CfManifestTranslator().get_service_options(str(root), plan))
    assert sorted(got) == ["img", "mystery", "other", "web"]
    # three files read as manifests: app/manifest.yml and the two collect outputs
    assert [len(got[n]) for n in ("img", "mystery", "other", "web")] == [3, 3, 1, 3]
    img = got["img"][0]
    assert img.container_build_type == plantypes.REUSE and img.image == "repo/img:2"
    assert not img.update_container_build_pipeline
    web = got["web"][0]
    assert web.container_build_type == plantypes.CNB and web.target_options == ["cloudfoundry/cnb:cflinuxfs3"]
    collect = str(root / "m2k_collect")
    assert web.source_artifacts[plantypes.CF_RUNNING_MANIFEST_ARTIFACT] == [collect + "/instanceapps.yaml"]
    assert web.build_artifacts[plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT] == [collect]
    assert got["mystery"][0].container_build_type == plantypes.MANUAL
    err = capsys.readouterr().err
    assert logparse.logged(err, "No known containerization approach for %s even though it has a cf manifest "
                                "manifest.yml; Defaulting to manual" % collect, "warning")


def test_instance_only_apps_are_planned_once_per_manifest(tree):
    root, plan = tree
    (root / "app2").mkdir()
    (root / "app2" / "manifest.yml").write_text("applications:\n- name: another\n")
    got = _by(CfManifestTranslator().get_service_options(str(root), plan))
    assert len(got["img"]) == 4 and len(got["web"]) == 4 and len(got["mystery"]) == 4
    assert len(got["other"]) == 1 and len(got["another"]) == 1


def test_manifest_app_matched_through_its_running_instance(tree):
    """A manifest app without a buildpack of its own matches a containerizer
    through the buildpack its running instance reports."""
    root, plan = tree
    (root / "app" / "manifest.yml").write_text("applications:\n- name: web\n  instances: 2\n")
    got = _by(CfManifestTranslator().get_service_options(str(root), plan))
    (web,) = got["web"]
    assert web.container_build_type == plantypes.CNB
    assert web.source_artifacts[plantypes.CFMANIFEST_ARTIFACT] == [str(root / "app" / "manifest.yml")]
    assert web.source_artifacts[plantypes.CF_RUNNING_MANIFEST_ARTIFACT] == [
        str(root / "m2k_collect" / "instanceapps.yaml")]
    svc = plantypes.Service.new("web", plantypes.CFMANIFEST2KUBE)
    svc.container_build_type = plantypes.REUSE
    svc.source_artifacts = dict(web.source_artifacts)
    ir = CfManifestTranslator().translate([svc], plan)
    sc = ir.services["web"]
    assert sc.replicas == 2                                   # the manifest's instances win
    (c,) = sc.containers
    assert {"name": "FROM_INSTANCE", "value": "yes"} in c["env"]
    assert c["ports"] == [{"containerPort": 9000}] and {"name": "PORT", "value": "9000"} in c["env"]


def test_translate_an_instance_only_service(tree, capsys):
    root, plan = tree
    svc = plantypes.Service.new("web", plantypes.CFMANIFEST2KUBE)
    svc.container_build_type = plantypes.REUSE
    svc.source_artifacts[plantypes.CF_RUNNING_MANIFEST_ARTIFACT] = [str(root / "m2k_collect" / "instanceapps.yaml")]
    gone = plantypes.Service.new("gone", plantypes.CFMANIFEST2KUBE)
    gone.container_build_type = plantypes.REUSE
    gone.source_artifacts[plantypes.CF_RUNNING_MANIFEST_ARTIFACT] = [str(root / "m2k_collect" / "instanceapps.yaml")]
    log.set_verbose(True)
    try:
        ir = CfManifestTranslator().translate([svc, gone], plan)
    finally:
        log.set_verbose(False)
    assert ir.services["web"].replicas == 3
    assert ir.services["gone"].containers[0]["ports"] == [{"containerPort": 8080}]
    err = capsys.readouterr().err
    assert logparse.logged_containing(err, "is not a valid cf apps file. Error: \"Failed to find the app gone in the "
                                      "cf apps file at path", "debug")
    assert logparse.logged(err, "No cf manifest file found for service web", "debug")


def test_a_service_no_manifest_application_names_is_left_out(tree):
    """DEVIATIONS §6: the reference indexes applications[0] of an empty list."""
    root, plan = tree
    (root / "app" / "manifest.yml").write_text("applications:\n- name: a\n- name: b\n")
    svc = plantypes.Service.new("renamed", plantypes.CFMANIFEST2KUBE)
    svc.container_build_type = plantypes.REUSE
    svc.source_artifacts[plantypes.CFMANIFEST_ARTIFACT] = [str(root / "app" / "manifest.yml")]
    ir = CfManifestTranslator().translate([svc], plan)
    assert ir.services == {} and len(ir.containers) == 1
