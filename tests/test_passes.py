"""Optimizer and parameterizer passes (cases mirror ``internal/optimizer/*_test.go``
and ``internal/parameterizer/parameterizer_test.go``)."""

from move2kube_amd import optimizer, parameterizer, qaengine
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.qaengine.default_engine import DefaultEngine


def _ir(services=None):
    ir = irtypes.new_ir(plantypes.new_plan())
    for name, (replicas, containers) in (services or {}).items():
        s = irtypes.Service(name)
        s.replicas = replicas
        s.containers = containers
        ir.services[name] = s
    return ir


def test_strip_quotation():
    assert optimizer.strip_quotation("'testString'") == "testString"
    assert optimizer.strip_quotation('"testString"') == "testString"
    assert optimizer.strip_quotation("testString") == "testString"


def test_normalize_characters():
    ir = _ir({"svcname1": (2, [{"name": "container-1", "env": [
        {"name": "NAME\t", "value": "git-resource"}, {"name": "NO_PROXY", "value": "'no-proxy.git.com'"},
        {"name": "VALID_VARIABLE", "value": "valid-variable"}]}]),
        "svcname2": (4, [{"name": "container-2", "env": [
            {"name": "\nNAME", "value": "git-resource2"}, {"name": " PROXY", "value": "  proxy.git.com "},
            {"name": "affinity", "value": "with-pod-affinity "}]}])})
    optimizer.NormalizeCharacterOptimizer().optimize(ir)
    assert ir.services["svcname1"].containers[0]["env"] == [
        {"name": "NAME", "value": "git-resource"}, {"name": "NO_PROXY", "value": "no-proxy.git.com"},
        {"name": "VALID_VARIABLE", "value": "valid-variable"}]
    assert ir.services["svcname2"].containers[0]["env"] == [
        {"name": "NAME", "value": "git-resource2"}, {"name": "PROXY", "value": "proxy.git.com"}]


def test_normalize_no_env_untouched():
    ir = _ir({"s": (1, [{"name": "c"}])})
    optimizer.NormalizeCharacterOptimizer().optimize(ir)
    assert ir.services["s"].containers == [{"name": "c"}]


def test_replicas_and_pull_policy():
    ir = _ir({"a": (0, [{"name": "c1"}]), "b": (4, [{"name": "c2", "imagePullPolicy": "Always"}])})
    optimizer.ReplicaOptimizer().optimize(ir)
    optimizer.ImagePullPolicyOptimizer().optimize(ir)
    assert ir.services["a"].replicas == 2 and ir.services["b"].replicas == 4
    assert all(c["imagePullPolicy"] == "Always" for s in ir.services.values() for c in s.containers)


def test_port_merge_by_image_name_and_url():
    qaengine.add_engine(DefaultEngine())
    ir = _ir({"svcname1": (2, [{"name": "container-1", "image": "image1"}]),
              "svcname2": (4, [{"name": "container-2", "image": "reg.io/ns/image2"}])})
    ir.kubernetes.registry_url = "reg.io"
    c1 = irtypes.new_container(plantypes.NEW_DOCKERFILE, "image1", True)
    c1.exposed_ports = [8088]
    c2 = irtypes.new_container(plantypes.NEW_DOCKERFILE, "image2", True)
    c2.exposed_ports = [8000, 8080]
    ir.containers = [c1, c2]
    optimizer.PortMergeOptimizer().optimize(ir)
    assert ir.services["svcname1"].containers[0]["ports"] == [{"containerPort": 8088}]
    assert ir.services["svcname2"].containers[0]["ports"] == [{"containerPort": 8000}, {"containerPort": 8080}]
    assert [(f.service_port.number, f.pod_port.number) for f in ir.services["svcname2"].port_forwardings] == \
        [(8000, 8000), (8080, 8080)]


def test_port_merge_defaults_to_8080_without_image_info():
    qaengine.add_engine(DefaultEngine())
    ir = _ir({"s": (1, [{"name": "c", "image": "unknown"}]), "empty": (1, [])})
    optimizer.PortMergeOptimizer().optimize(ir)
    assert ir.services["s"].containers[0]["ports"] == [{"containerPort": 8080}]
    assert ir.services["empty"].containers == []


def test_parameterize_no_services():
    ir = _ir()
    parameterizer.parameterize(ir)
    assert ir.target_cluster_spec.host == "{{ .Release.Name }}-{{ .Values.ingresshost }}"
    assert ir.values.services == {}


def test_parameterize_services_without_containers():
    ir = _ir({"svcname1": (2, []), "svcname2": (4, [])})
    parameterizer.parameterize(ir)
    assert ir.values.services == {"svcname1": {}, "svcname2": {}}


def test_parameterize_image_names():
    ir = _ir({"svcname1": (2, [{"name": "container-1"}])})
    parameterizer.parameterize(ir)
    assert ir.services["svcname1"].containers[0]["image"] == \
        ':{{ index .Values.services "svcname1" "containers" "container-1" "imagetag"  }}'
    assert ir.values.services == {"svcname1": {"container-1": "latest"}}


def test_parameterize_storage_class():
    ir = _ir()
    ir.storages = [irtypes.Storage(name="s1", storage_type=irtypes.PVC_KIND, pvc_spec={"storageClassName": "storage-1cn"}),
                   irtypes.Storage(name="cm", storage_type=irtypes.CONFIGMAP_KIND)]
    parameterizer.parameterize(ir)
    assert ir.storages[0].pvc_spec["storageClassName"] == "{{ .Values.storageclass }}"
    assert ir.values.storage_class == "storage-1cn"


def test_parameterize_mixed_storage_classes_skipped():
    ir = _ir()
    ir.storages = [irtypes.Storage(name="a", storage_type=irtypes.PVC_KIND, pvc_spec={"storageClassName": "x"}),
                   irtypes.Storage(name="b", storage_type=irtypes.PVC_KIND, pvc_spec={"storageClassName": "y"})]
    parameterizer.parameterize(ir)
    assert [s.pvc_spec["storageClassName"] for s in ir.storages] == ["x", "y"] and ir.values.storage_class == ""
