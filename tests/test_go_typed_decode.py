"""Typed decode errors of the move2kube documents worded as go-yaml v3 reports
them (``models/gotypes.py``): ``yaml.Unmarshal`` into the reference's Go
structs (``types/plan/plan.go``, ``types/qaengine``, ``types/collection``)
collects one ``line N: cannot unmarshal <tag> [`value`] into <type>`` per bad
node (``decode.go`` ``terror``: values longer than 10 bytes cut to 7 plus
``...``) and keeps decoding.  Parity is pinned by those sources only (no Go
toolchain here)."""

import pytest

import logparse
from move2kube_amd.models import gotypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.models.base import DecodeError, as_int
from move2kube_amd.utils import log

PLAN = """apiVersion: move2kube.konveyor.io/v1alpha1
kind: Plan
metadata:
  name: [x]
spec:
  inputs:
    rootDir: {a: 1}
    services:
      api:
        - serviceName: api
          updateDeployPipeline: false - Directory
          updateContainerBuildPipeline: yes
          sourceType: ~ - Directory
          sourceArtifacts: [a]
          buildArtifacts:
            SourceCode: x
        - 12
      web: abc
  outputs:
    kubernetes:
      ignoreUnsupportedKinds: !!int 1
"""

PLAN_ERRORS = """yaml: unmarshal errors:
  line 4: cannot unmarshal !!seq into string
  line 7: cannot unmarshal !!map into string
  line 11: cannot unmarshal !!str `false -...` into bool
  line 13: cannot unmarshal !!str `~ - Dir...` into []plan.SourceTypeValue
  line 14: cannot unmarshal !!seq into map[plan.SourceArtifactTypeValue][]string
  line 16: cannot unmarshal !!str `x` into []string
  line 17: cannot unmarshal !!int `12` into plan.Service
  line 18: cannot unmarshal !!str `abc` into []plan.Service
  line 21: cannot unmarshal !!int `1` into bool"""


def test_plan_type_errors_list_every_bad_node(tmp_path, capsys):
    p = tmp_path / "m2k.plan"
    p.write_text(PLAN)
    assert gotypes.error_text(PLAN, gotypes.PLAN) == PLAN_ERRORS
    log.set_verbose(False)
    with pytest.raises(DecodeError) as ei:
        plantypes.read_plan(str(p))
    assert str(ei.value) == PLAN_ERRORS
    assert ("error", "Failed to load the plan file at path %s Error %s" % (log.go_quote(str(p)), log.go_quote(PLAN_ERRORS))) \
        in logparse.messages(capsys.readouterr().err)


@pytest.mark.parametrize("value,ok", [
    ("true", True), ("yes", True), ("Off", True), ("~", True), ("'true'", False), ("1", False), ("[true]", False),
])
def test_bool_fields_take_yaml_1_1_words(value, ok):
    doc = "spec:\n  outputs:\n    kubernetes:\n      ignoreUnsupportedKinds: %s\n" % value
    errs = gotypes.unmarshal_errors(doc, gotypes.PLAN)
    assert (errs == []) is ok, errs


@pytest.mark.parametrize("value,err", [
    ("8080", None), ("1.9", None), ("0x1f", None), ("017", None),
    ("3000000000", "line 6: cannot unmarshal !!int `3000000000` into int32"),
    ("abc", "line 6: cannot unmarshal !!str `abc` into int32"),
    ("true", "line 6: cannot unmarshal !!bool `true` into int32"),
])
def test_int_fields_follow_resolve_and_range(value, err):
    doc = "spec:\n  applications:\n    - name: a\n      memory: 1\n      ports:\n        - %s\n" % value
    errs = gotypes.unmarshal_errors(doc, gotypes.CF_INSTANCE_APPS)
    assert errs == ([err] if err else [])


def test_as_int_truncates_floats_and_reads_go_numbers():
    assert [as_int(v) for v in ("017", "0x10", "0o17", "0b11", "1_000", "1e3", "1.9", "-1.9", 7)] == \
        [15, 16, 15, 3, 1000, 1000, 1, -1, 7]
    with pytest.raises(DecodeError):
        as_int("abc")


def test_qa_cache_type_error_is_logged_with_go_text(tmp_path, capsys):
    from move2kube_amd.models import qa
    f = tmp_path / "c.yaml"
    f.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
                 "    - description: d\n      solution:\n        answer: yes please\n")
    log.set_verbose(False)
    with pytest.raises(DecodeError):
        qa.Cache(str(f)).load()
    want = "yaml: unmarshal errors:\n  line 7: cannot unmarshal !!str `yes please` into []string"  # 10 bytes: not cut
    assert ("error", "Unable to load cache : " + want) in logparse.messages(capsys.readouterr().err)


def test_collection_documents_use_their_go_types(tmp_path):
    from move2kube_amd.metadata import _read_cluster_metadata
    from move2kube_amd.source.compose2kube import _read_image_info
    cm = tmp_path / "cm.yaml"
    cm.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: ClusterMetadata\nspec:\n"
                  "  storageClasses: default\n  apiKindVersionMap:\n    Deployment: apps/v1\n")
    with pytest.raises(DecodeError) as ei:
        _read_cluster_metadata(str(cm))
    assert str(ei.value) == ("yaml: unmarshal errors:\n  line 4: cannot unmarshal !!str `default` into []string\n"
                             "  line 6: cannot unmarshal !!str `apps/v1` into []string")
    im = tmp_path / "im.yaml"
    im.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: ImageMetadata\nspec:\n  userID: root\n")
    with pytest.raises(DecodeError) as ei:
        _read_image_info(str(im))
    assert str(ei.value) == "yaml: unmarshal errors:\n  line 4: cannot unmarshal !!str `root` into int"
