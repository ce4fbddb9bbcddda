"""Compose v1/v2 feature coverage (reference ``internal/source/compose/v1v2.go:140-470``):
container name lower-casing, entrypoint/command, ``k=v`` / ``k:v`` / bare env,
``[ip:]svc:pod[/proto]`` ports plus expose, privileged, non-numeric user
(ignored), capabilities, group_add (never attached in the reference),
stop_grace_period, mem_limit, unless-stopped, networks (libcompose real
names), tmpfs, bind volumes (hostPath ``vol<fnv64a>``, read-only) and named
volumes (PVC + RWX/ROX storage)."""

import os
import shutil

from move2kube_amd import api
from move2kube_amd.utils import common, yamlio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "compose_v2_full")


def test_compose_v2_full(tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    src = str(tmp_path / "proj")
    shutil.copytree(FIXTURE, src)
    out = os.path.join(api.translate(src, str(tmp_path / "out"), name="v2"), "v2")
    objs = {f: yamlio.load(open(os.path.join(out, f)).read()) for f in os.listdir(out)}
    dep = objs["app-deployment.yaml"]
    meta = dep["metadata"]
    assert meta["annotations"]["role"] == "main" and "role" not in meta["labels"]
    assert meta["labels"]["move2kube.konveyor.io/network/proj_backend"] == "true"
    pod = dep["spec"]["template"]["spec"]
    assert pod["hostname"] == "apphost" and pod["subdomain"] == "example.com"
    assert pod["terminationGracePeriodSeconds"] == 90
    assert pod["restartPolicy"] == "Always"
    assert "securityContext" not in pod            # group_add is dropped, as in the reference
    (c,) = pod["containers"]
    assert c["name"] == "app-main"
    assert c["command"] == ["/start.sh"] and c["args"] == ["serve", "--port", "80"]
    assert c["env"] == [{"name": "A", "value": "1"}, {"name": "B", "value": "2"},
                        {"name": "BROKEN", "value": "unknown"}]
    assert c["workingDir"] == "/work" and c["stdin"] is True and c["tty"] is True
    assert c["securityContext"] == {"capabilities": {"add": ["SYS_TIME"]}, "privileged": True}
    assert c["resources"] == {"limits": {"memory": "268435456"}}
    assert [(p["containerPort"], p["protocol"]) for p in c["ports"]] == [(8001, "TCP"), (90, "UDP"), (3000, "TCP"),
                                                                        (4000, "TCP")]
    logs = os.path.join(src, "logs")
    vol = "vol%d" % common.fnv64a(logs.encode())
    assert c["volumeMounts"] == [
        {"mountPath": "/scratch", "name": "app-tmpfs-0"},
        {"mountPath": "/var/log/app", "name": vol, "readOnly": True},
        {"mountPath": "/data", "name": "appdata"},
        {"mountPath": "/shared", "name": "shared", "readOnly": True},
    ]
    assert pod["volumes"] == [
        {"emptyDir": {"medium": "Memory"}, "name": "app-tmpfs-0"},
        {"hostPath": {"path": logs}, "name": vol},
        {"name": "appdata", "persistentVolumeClaim": {"claimName": "appdata"}},
        {"name": "shared", "persistentVolumeClaim": {"claimName": "shared", "readOnly": True}},
    ]
    svc = objs["app-service.yaml"]
    assert [(p["port"], p["targetPort"]) for p in svc["spec"]["ports"]] == [(8001, 8001), (9000, 90), (3000, 3000),
                                                                           (4000, 4000)]
    assert objs["appdata-persistentvolumeclaim.yaml"]["spec"]["accessModes"] == ["ReadWriteMany"]
    assert objs["shared-persistentvolumeclaim.yaml"]["spec"]["accessModes"] == ["ReadOnlyMany"]
    assert objs["proj_backend-networkpolicy.yaml"]["metadata"]["name"] == "proj_backend"


def test_compose_v2_unsupported_minor_version_is_skipped(tmp_path, monkeypatch):
    # libcompose accepts 2, 2.0 and 2.1 only; docker/cli's v3 loader rejects 2.x:
    # a 2.4 file yields no services
    from move2kube_amd.source.compose2kube import ComposeTranslator
    from move2kube_amd.models import plan as plantypes
    d = tmp_path / "x"
    d.mkdir()
    (d / "docker-compose.yml").write_text('version: "2.4"\nservices:\n  a:\n    image: busybox\n')
    p = plantypes.new_plan()
    p.root_dir = str(d)
    assert ComposeTranslator().get_service_options(str(d), p) == []
