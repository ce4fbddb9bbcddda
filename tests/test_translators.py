"""Source translators on small inputs: compose v1/v2/v3, CF manifests (with
variables and collected instance apps), k8s/knative YAML carry-over."""

import os
import textwrap

import pytest

from move2kube_amd import api
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source.cfmanifest2kube import CfManifestTranslator
from move2kube_amd.source.compose2kube import ComposeTranslator
from move2kube_amd.source.kube2kube import KubeTranslator
from move2kube_amd.utils import yamlio


def _write(p, text):
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(textwrap.dedent(text))


def _plan(root):
    p = plantypes.new_plan()
    p.name = "t"
    p.root_dir = root
    return p


def _translate(translator, root):
    p = _plan(root)
    services = translator.get_service_options(root, p)
    p.add_services_to_plan(services)
    chosen = [opts[0] for _, opts in sorted(p.services.items())]
    return services, translator.translate(chosen, p)


def test_compose_v2(tmp_path, assets_dir):
    root = str(tmp_path)
    _write(os.path.join(root, "docker-compose.yml"), """\
        version: "2"
        services:
          db:
            image: postgres:12
            environment:
              - POSTGRES_PASSWORD=secret
              - BROKEN
            ports:
              - "5432"
            mem_limit: 1000000
            restart: unless-stopped
          web:
            image: acme/web:2
            ports:
              - "80:8080/tcp"
            command: ["run", "--fast"]
    """)
    services, ir = _translate(ComposeTranslator(), root)
    assert sorted(s.service_name for s in services) == ["db", "web"]
    db = ir.services["db"]
    c = db.containers[0]
    assert c["image"] == "postgres:12"
    assert {"name": "POSTGRES_PASSWORD", "value": "secret"} in c["env"]
    assert db.restart_policy == "Always"
    assert c["resources"]["limits"]["memory"] == "1e6"
    web = ir.services["web"].containers[0]
    assert web["args"] == ["run", "--fast"]
    assert web["ports"][0]["containerPort"] == 8080


def test_compose_v3_interpolation_uses_os_env(tmp_path, assets_dir, monkeypatch):
    # docker/cli's v3 loader interpolates from the OS environment only (.env is a v1/v2 feature)
    root = str(tmp_path)
    monkeypatch.setenv("TAG_FROM_ENV", "9.9")
    monkeypatch.setenv("TAG", "1.2")
    _write(os.path.join(root, ".env"), "TAG=from-dotenv\n")
    _write(os.path.join(root, "docker-compose.yaml"), """\
        version: "3.4"
        services:
          app:
            image: "acme/app:${TAG}"
            environment:
              OTHER: "${TAG_FROM_ENV:-none}"
              DEFAULTED: "${MISSING:-fallback}"
    """)
    _, ir = _translate(ComposeTranslator(), root)
    c = ir.services["app"].containers[0]
    assert c["image"] == "acme/app:1.2"
    envs = {e["name"]: e["value"] for e in c["env"]}
    assert envs == {"DEFAULTED": "fallback", "OTHER": "9.9"}


def test_compose_v1v2_reads_dotenv(tmp_path, assets_dir, monkeypatch):
    # libcompose looks up ".env" relative to the working directory, like the reference
    root = str(tmp_path)
    monkeypatch.delenv("TAG", raising=False)
    monkeypatch.chdir(root)
    _write(os.path.join(root, ".env"), "TAG=1.2\n")
    _write(os.path.join(root, "docker-compose.yaml"), """\
        version: "2"
        services:
          app:
            image: "acme/app:${TAG}"
    """)
    _, ir = _translate(ComposeTranslator(), root)
    assert ir.services["app"].containers[0]["image"] == "acme/app:1.2"


def test_compose_invalid_files_are_ignored(tmp_path, assets_dir):
    root = str(tmp_path)
    _write(os.path.join(root, "not-compose.yaml"), "foo: [bar\n")
    _write(os.path.join(root, "k8s.yaml"), "apiVersion: v1\nkind: Service\nmetadata:\n  name: x\n")
    services = ComposeTranslator().get_service_options(root, _plan(root))
    assert services == []


def test_cf_manifest_with_vars_and_docker_image(tmp_path, assets_dir):
    root = str(tmp_path)
    _write(os.path.join(root, "app1", "manifest.yml"), """\
        applications:
        - name: web
          instances: 2
          memory: ((mem))
          env:
            MODE: ((mode))
          buildpacks:
            - nodejs_buildpack
        - name: img
          docker:
            image: acme/img:3
    """)
    _write(os.path.join(root, "app1", "package.json"), "{}")
    services = CfManifestTranslator().get_service_options(root, _plan(root))
    names = sorted({s.service_name for s in services})
    assert names == ["img", "web"]
    img = [s for s in services if s.service_name == "img"]
    assert img[0].container_build_type == plantypes.REUSE and img[0].image == "acme/img:3"
    web_types = {s.container_build_type for s in services if s.service_name == "web"}
    assert plantypes.NEW_DOCKERFILE in web_types


def test_cf_translate_sets_env_and_replicas(tmp_path, assets_dir):
    root = str(tmp_path)
    _write(os.path.join(root, "app", "manifest.yml"), """\
        applications:
        - name: web
          instances: 3
          env:
            GREETING: hi
    """)
    _write(os.path.join(root, "app", "package.json"), "{}")
    _, ir = _translate(CfManifestTranslator(), root)
    svc = ir.services["web"]
    assert svc.replicas == 3
    assert {"name": "GREETING", "value": "hi"} in svc.containers[0]["env"]
    assert any(c.new for c in ir.containers)


def test_kube_yamls_carried_over(tmp_path, assets_dir):
    root = str(tmp_path)
    _write(os.path.join(root, "deploy.yaml"), """\
        apiVersion: apps/v1
        kind: Deployment
        metadata:
          name: legacy
        spec:
          replicas: 3
          selector:
            matchLabels: {app: legacy}
          template:
            metadata:
              labels: {app: legacy}
            spec:
              containers:
              - name: c
                image: nginx:1
    """)
    services, ir = _translate(KubeTranslator(), root)
    assert [s.service_name for s in services] == ["legacy"]
    assert services[0].container_build_type == plantypes.REUSE
    assert ir.services["legacy"].containers[0]["image"] == "nginx:1"


def test_end_to_end_openshift_target(tmp_path):
    src = tmp_path / "src"
    _write(str(src / "node" / "package.json"), "{}")
    cache = tmp_path / "qa.yaml"
    cache.write_text(textwrap.dedent("""\
        apiVersion: move2kube.konveyor.io/v1alpha1
        kind: QACache
        spec:
          solutions:
            - description: 'Choose the cluster type:'
              solution:
                type: Select
                answer:
                  - Openshift
              resolved: true
    """))
    out = api.translate(str(src), str(tmp_path / "out"), "os", qacaches=[str(cache)])
    files = sorted(os.listdir(os.path.join(out, "os")))
    assert "node-deploymentconfig.yaml" in files and "node-route.yaml" in files and "node-imagestream.yaml" in files
    dc = yamlio.load(open(os.path.join(out, "os", "node-deploymentconfig.yaml")).read())
    assert dc["apiVersion"] == "apps.openshift.io/v1"
    assert dc["spec"]["triggers"][1]["type"] == "ImageChange"


def test_cf_manifest_variables_become_template_placeholders(tmp_path, assets_dir):
    from move2kube_amd.source import cfmanifest
    root = str(tmp_path)
    path = os.path.join(root, "manifest.yml")
    _write(path, """\
        applications:
        - name: web
          env:
            MODE: ((mode))
            URL: https://((host))/api
    """)
    assert cfmanifest.get_missing_variables(path) == ["host", "mode"]
    apps, variables = cfmanifest.read_application_manifest(path, "", plantypes.YAMLS)
    assert variables == ["host", "mode"]
    assert apps[0].environment_variables == {"MODE": "{{ $mode }}", "URL": "https://{{ $host }}/api"}
    apps, _ = cfmanifest.read_application_manifest(path, "", plantypes.HELM)
    assert apps[0].environment_variables["MODE"] == '{{ index  .Values "globalvariables" "mode"}}'


def test_cf_manifest_scalars_follow_yaml_1_1(tmp_path):
    """The bosh template decodes a CF manifest with go-yaml v2 before anyone
    reads it: yes/on are booleans (env values print "true"), 010 is octal, a
    repeated key keeps its last value."""
    from move2kube_amd.source import cfmanifest
    p = tmp_path / "manifest.yml"
    p.write_text("applications:\n- name: a\n  name: app\n  instances: 010\n  env:\n    FLAG: yes\n    OTHER: off\n")
    (app,), variables = cfmanifest.read_application_manifest(str(p))
    assert variables == [] and app.name == "app" and app.instances.value == 8
    assert app.environment_variables == {"FLAG": "true", "OTHER": "false"}
