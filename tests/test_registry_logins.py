"""Registry login answers through the whole translate (reference
``internal/customizer/registrycustomizer.go:150-280``): "Use existing pull
secret" names the secret that the pods referencing that registry's images
get; "UserName/Password" writes a ``kubernetes.io/dockerconfigjson`` Secret
as docker/cli's ``SaveToWriter`` encodes it (tab-indented, ``auth`` =
base64 of ``user:password``, keyed by the target registry).  In the
reference that Secret's name comes from a map entry only the docker-config
branch fills, so it has no name and no pod refers to it;
``M2K_COMPAT=fixed`` names it after its registry and references it."""

import base64
import os
import shutil

import pytest

from move2kube_amd import api
from move2kube_amd.utils import log, yamlio
from move2kube_amd.utils.constants import settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sol(desc, typ, ans):
    return ("    - description: '%s'\n      solution:\n        type: %s\n        answer:\n          - %s\n"
            "      resolved: true\n" % (desc, typ, ans))


@pytest.fixture(params=["reference", "fixed"])
def translated(request, tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    monkeypatch.setattr(settings, "compat", request.param)
    log.set_quiet()
    src = tmp_path / "src"
    shutil.copytree(os.path.join(ROOT, "samples", "nodejs"), str(src / "nodejs"))
    (src / "docker-compose.yaml").write_text('version: "3"\nservices:\n  cache:\n    image: quay.io/org/redis:6\n')
    cache = tmp_path / "answers.yaml"
    cache.write_text("apiVersion: move2kube.konveyor.io/v1alpha1\nkind: QACache\nspec:\n  solutions:\n"
                     + _sol("[docker.io] What type of container registry login do you want to use?", "Select",
                            "UserName/Password")
                     + _sol("[docker.io] Enter the container registry username : ", "Input", "bob")
                     + _sol("[quay.io] What type of container registry login do you want to use?", "Select",
                            "Use existing pull secret")
                     + _sol("[quay.io] Enter the name of the pull secret : ", "Input", "quay-pull"))
    with api.Session(qaskip=True, qacaches=[str(cache)]) as s:
        out = s.translate(str(src), str(tmp_path / "out"), name="q")
    d = os.path.join(out, "q")
    objs = {f: yamlio.load(open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d))}
    log.set_verbose(False)
    return request.param, objs


def _pull_secrets(obj):
    return obj["spec"]["template"]["spec"].get("imagePullSecrets")


def test_existing_pull_secret_is_referenced(translated):
    _mode, objs = translated
    assert _pull_secrets(objs["cache-deployment.yaml"]) == [{"name": "quay-pull"}]
    assert not any(o.get("kind") == "Secret" and o["metadata"].get("name") == "quay-pull" for o in objs.values())


def test_username_password_secret(translated):
    mode, objs = translated
    secrets = [(f, o) for f, o in objs.items() if o.get("kind") == "Secret"]
    assert len(secrets) == 1
    fname, sec = secrets[0]
    assert sec["type"] == "kubernetes.io/dockerconfigjson"
    # the password problem is never cached; --qaskip answers it with ""
    assert base64.b64decode(sec["data"][".dockerconfigjson"]) == (
        b'{\n\t"auths": {\n\t\t"docker.io": {\n\t\t\t"auth": "' + base64.b64encode(b"bob:") + b'"\n\t\t}\n\t}\n}')
    if mode == "reference":
        assert fname == "-secret.yaml" and "name" not in sec["metadata"]
        assert _pull_secrets(objs["nodejs-deployment.yaml"]) is None
    else:
        assert sec["metadata"]["name"] == "imagepullsecretdocker.io"
        assert _pull_secrets(objs["nodejs-deployment.yaml"]) == [{"name": "imagepullsecretdocker.io"}]
