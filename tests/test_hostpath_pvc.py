"""Host-path volumes through the storage customizer (reference
``internal/customizer/storagecustomizer.go:96-136``): the confirm question is
asked once per host path; "yes" turns every volume of that path into a claim
on one PVC named after the first volume; "no" keeps the first service's
hostPath, and a later service mounting the same path gets a claim with an
empty name (``hostPathsVisited[path]`` stays "" after a declined answer and
the reference still takes its else branch)."""

import os

import pytest

from move2kube_amd import api
from move2kube_amd.utils import log, yamlio

COMPOSE = ('version: "3"\nservices:\n  a:\n    image: nginx\n    volumes:\n      - ./data:/data\n'
           '  b:\n    image: redis\n    volumes:\n      - ./data:/var/data\n')


def _translate(tmp_path, monkeypatch, answer):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    log.set_quiet()
    src = tmp_path / "src"
    src.mkdir()
    (src / "docker-compose.yaml").write_text(COMPOSE)
    cache = tmp_path / "answers.yaml"
    cache.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
                     "    - description: 'Do you want to create PVC for host path [%s]?:'\n"
                     "      solution:\n        type: Confirm\n        answer:\n          - \"%s\"\n"
                     "      resolved: true\n" % (src / "data", answer))
    with api.Session(qaskip=True, qacaches=[str(cache)]) as s:
        out = s.translate(str(src), str(tmp_path / "out"), name="q")
    log.set_verbose(False)
    d = os.path.join(out, "q")
    return {f: yamlio.load(open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d))}


def _volumes(objs, svc):
    return objs["%s-deployment.yaml" % svc]["spec"]["template"]["spec"]["volumes"]


def test_host_path_to_one_shared_pvc(tmp_path, monkeypatch):
    objs = _translate(tmp_path, monkeypatch, "true")
    (va,), (vb,) = _volumes(objs, "a"), _volumes(objs, "b")
    name = va["name"]
    assert va == {"name": name, "persistentVolumeClaim": {"claimName": name}}
    assert vb == {"name": vb["name"], "persistentVolumeClaim": {"claimName": name}}
    pvcs = [o for o in objs.values() if o.get("kind") == "PersistentVolumeClaim"]
    assert len(pvcs) == 1 and pvcs[0]["metadata"]["name"] == name
    assert pvcs[0]["spec"]["volumeName"] == name and pvcs[0]["spec"]["resources"]["requests"]["storage"] == "100Mi"


@pytest.mark.parametrize("answer", ["false"])
def test_declined_host_path_quirk(tmp_path, monkeypatch, answer):
    objs = _translate(tmp_path, monkeypatch, answer)
    (va,), (vb,) = _volumes(objs, "a"), _volumes(objs, "b")
    assert va["hostPath"] == {"path": str(tmp_path / "src" / "data")}
    assert vb["persistentVolumeClaim"] == {"claimName": ""}
    assert not any(o.get("kind") == "PersistentVolumeClaim" for o in objs.values())
