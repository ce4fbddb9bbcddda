"""Compose2Kube off the happy path (reference
``internal/source/compose2kube.go:40-200``): image-info YAMLs attached by
image tag, Dockerfile paths a v1/v2 file gives as absolute, plan services of
another translation type, and compose or image-info files that no longer load
at translate time."""

import pytest

import logparse
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source.compose2kube import ComposeTranslator
from move2kube_amd.utils import log

IMAGE_INFO = ("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: ImageMetadata\nmetadata:\n  name: web\n"
              "spec:\n  tags: [\"web:1\"]\n  ports: [8080]\n  userID: 1001\n")


@pytest.fixture(autouse=True)
def _quiet():
    log.set_verbose(False)
    yield
    log.set_verbose(False)


def _plan(root):
    p = plantypes.new_plan()
    p.root_dir = str(root)
    return p


def test_image_info_is_attached_by_tag(tmp_path):
    (tmp_path / "docker-compose.yaml").write_text('version: "3"\nservices:\n  web:\n    image: web:1\n'
                                                  '  db:\n    image: redis\n')
    (tmp_path / "web-info.yaml").write_text(IMAGE_INFO)
    (tmp_path / "other.yaml").write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: ClusterMetadata\n")
    services = ComposeTranslator().get_service_options(str(tmp_path), _plan(tmp_path))
    by_name = {s.service_name: s for s in services}
    assert by_name["web"].source_artifacts[plantypes.IMAGE_INFO_ARTIFACT] == [str(tmp_path / "web-info.yaml")]
    assert plantypes.IMAGE_INFO_ARTIFACT not in by_name["db"].source_artifacts
    ir = ComposeTranslator().translate([by_name["web"]], _plan(tmp_path))
    (c,) = [c for c in ir.containers if "web:1" in c.image_names]
    assert c.exposed_ports == [8080] and c.user_id == 1001 and not c.new


def test_v1v2_absolute_context_and_dockerfile(tmp_path):
    ctx = tmp_path / "ctx"
    ctx.mkdir()
    (tmp_path / "docker-compose.yml").write_text(
        'version: "2"\nservices:\n  app:\n    build:\n      context: %s\n      dockerfile: %s\n' % (ctx, ctx / "Df"))
    services = ComposeTranslator().get_service_options(str(tmp_path), _plan(tmp_path))
    (reuse_df,) = [s for s in services if s.container_build_type == plantypes.REUSE_DOCKERFILE]
    assert reuse_df.target_options == [str(ctx / "Df")]
    assert reuse_df.build_artifacts[plantypes.SOURCE_DIRECTORY_BUILD_ARTIFACT] == [str(ctx)]


def test_files_that_are_not_compose_are_skipped_with_both_errors(tmp_path, capsys):
    (tmp_path / "list.yaml").write_text("- a\n")
    log.set_verbose(True)
    assert ComposeTranslator().get_service_options(str(tmp_path), _plan(tmp_path)) == []
    assert logparse.logged_containing(capsys.readouterr().err, "Failed to parse file at path %s as a docker compose "
                                      'file. Error V3: "' % (tmp_path / "list.yaml"), "debug")


def test_listing_failure(tmp_path, monkeypatch, capsys):
    from move2kube_amd.utils import common

    def boom(*a):
        raise OSError(2, "No such file or directory", str(tmp_path / "gone"))
    monkeypatch.setattr(common, "get_files_by_ext", boom)
    with pytest.raises(OSError):
        ComposeTranslator().get_service_options(str(tmp_path / "gone"), _plan(tmp_path))
    assert logparse.logged(capsys.readouterr().err, 'Unable to fetch yaml files at path %s Error: "open %s: no such '
                           'file or directory"' % (tmp_path / "gone", tmp_path / "gone"), "error")


def test_translate_skips_other_types_and_files_that_no_longer_load(tmp_path, capsys):
    (tmp_path / "docker-compose.yaml").write_text('version: "3"\nservices:\n  web:\n    image: nginx\n')
    (tmp_path / "info.yaml").write_text(IMAGE_INFO)
    (web,) = [s for s in ComposeTranslator().get_service_options(str(tmp_path), _plan(tmp_path))]
    other = plantypes.Service.new("x", plantypes.ANY2KUBE)
    web.add_source_artifact(plantypes.IMAGE_INFO_ARTIFACT, str(tmp_path / "missing-info.yaml"))
    (tmp_path / "docker-compose.yaml").write_text("services: [broken\n")      # edited after planning
    log.set_verbose(True)
    ir = ComposeTranslator().translate([other, web], _plan(tmp_path))
    assert ir.services == {}
    err = capsys.readouterr().err
    assert logparse.logged(err, "Expected service to have compose2kube translation type. Got %s . Skipping."
                           % plantypes.ANY2KUBE, "debug")
    assert logparse.logged_containing(err, "Unable to parse the docker compose file at path %s Error V3: "
                                      % (tmp_path / "docker-compose.yaml"), "error")
    assert logparse.logged(err, 'Failed to read image info yaml at path %s Error: "open %s: no such file or '
                                'directory"' % (tmp_path / "missing-info.yaml", tmp_path / "missing-info.yaml"),
                           "error")
