"""Optimizer and parameterizer passes: one pytest per subtest of
``internal/optimizer/imagepullpolicyoptimizer_test.go``,
``normalizecharactersoptimizer_test.go``, ``replicaoptimizer_test.go`` and
``internal/parameterizer/parameterizer_test.go``, each comparing the whole IR
the pass returns with the IR the Go test builds as ``want`` (``cmp.Equal``;
``tests/goequal.py``).  The parameterizer tests use ``cmpopts.EquateEmpty``
in Go; the IR here holds no nil/empty distinction there, so plain equality is
at least as strict.

``portmergeoptimizer_test.go`` is commented out as a whole in the reference
(Go never compiles it); the port-merge tests at the end of this file follow
its cases anyway and are not ledger entries."""

import copy

from goequal import assert_deep_equal

from move2kube_amd import optimizer, parameterizer, qaengine
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes
from move2kube_amd.qaengine.default_engine import DefaultEngine
from move2kube_amd.utils.constants import DEFAULT_PVC_SIZE


def _svc(name, replicas, *containers):
    """``types.Service{Name: name, Replicas: replicas}`` with ``containers``
    appended (``svc.Containers = append(svc.Containers, c)``)."""
    s = irtypes.Service(name)
    s.replicas = replicas
    if containers:
        s.containers = list(containers)
    return s


def _ir(*services):
    ir = irtypes.new_ir(plantypes.new_plan())
    for s in services:
        ir.services[s.name] = s
    return ir


def _env(*pairs):
    return [{"name": n, "value": v} for n, v in pairs]


# --- fixtures of the Go files ------------------------------------------------

def get_ir_without_services():
    return _ir()


def get_ir_with_services_and_without_containers():
    return _ir(_svc("svcname1", 2), _svc("svcname2", 2))


def get_ir_with_image_pull_policy_set_as_always():
    return _ir(_svc("svcname1", 2, {"name": "container-1", "imagePullPolicy": "Always"}),
               _svc("svcname2", 4, {"name": "container-2", "imagePullPolicy": "Always"}))


def get_ir_with_services_and_containers_with_valid_env():
    return _ir(_svc("svcname1", 2, {"name": "container-1", "env": _env(("NAME", "git-resource"),
                                                                        ("NO_PROXY", "no-proxy.git.com"))}),
               _svc("svcname2", 4, {"name": "container-2", "env": _env(("NAME", "git-resource2"),
                                                                        ("PROXY", "proxy.git.com"))}))


def get_ir_with_services_and_containers_without_env():
    ir = _ir()
    ir.services["svcname1"] = _svc("svcname1", 2, {"name": "container-1"})
    ir.services["svcname1"] = _svc("svcname2", 4, {"name": "container-2"})   # sic: the Go fixture reuses the key
    return ir


def get_expected_ir():
    return _ir(_svc("svcname1", 2, {"name": "container-1", "env": _env(
                   ("NAME", "git-resource"), ("NO_PROXY", "no-proxy.git.com"), ("VALID_VARIABLE", "valid-variable"))}),
               _svc("svcname2", 4, {"name": "container-2", "env": _env(("NAME", "git-resource2"),
                                                                        ("PROXY", "proxy.git.com"))}))


def get_expected_ir_with_affinity_in_container():
    return _ir(_svc("svcname1", 2, {"name": "container-1", "env": _env(("NAME", "git-resource"))}),
               _svc("svcname2", 4, {"name": "container-2", "env": _env(("NAME", "git-resource2"),
                                                                        ("PROXY", "proxy.git.com"))}))


def get_services_with_more_replicas_than_default_minimum_replicas():
    return _ir(_svc("svcname1", 4), _svc("svcname2", 3))


def get_ir_with_services_with_default_minimum_replicas():
    return _ir(_svc("svcname1", 2), _svc("svcname2", 2))


def get_expected_ir_with_modified_replicas():
    return _ir(_svc("svcname1", 2), _svc("svcname2", 4))


def get_ir_with_services_and_containers():
    return _ir(_svc("svcname1", 2, {"name": "container-1"}))


def _storage_1(kind):
    return irtypes.Storage(name="storage-1", storage_type=kind, pvc_spec={
        "volumeName": "storage-1", "resources": {"requests": {"storage": DEFAULT_PVC_SIZE}},
        "storageClassName": "storage-1cn"})


def get_ir_with_storage_pvc_kind():
    ir = _ir()
    ir.storages.append(_storage_1(irtypes.PVC_KIND))
    return ir


def get_ir_with_storage_not_pvc_kind():
    ir = _ir()
    ir.storages.append(_storage_1(irtypes.SECRET_KIND))
    return ir


def _optimize(opt, ir):
    actual = opt.optimize(copy.deepcopy(ir))
    assert actual is not None
    return actual


# --- TestImagePullPolicyOptimizer ----------------------------------------------

def test_image_pull_policy_ir_with_no_services():
    assert_deep_equal(_optimize(optimizer.ImagePullPolicyOptimizer(), get_ir_without_services()),
                      get_ir_without_services())


def test_image_pull_policy_ir_containing_services_that_have_no_containers():
    assert_deep_equal(_optimize(optimizer.ImagePullPolicyOptimizer(), get_ir_with_services_and_without_containers()),
                      get_ir_with_services_and_without_containers())


def test_image_pull_policy_ir_containing_services_and_containers_without_image_pull_policy():
    ir = _ir(_svc("svcname1", 2, {"name": "container-1"}), _svc("svcname2", 4, {"name": "container-2"}))
    assert_deep_equal(_optimize(optimizer.ImagePullPolicyOptimizer(), ir),
                      get_ir_with_image_pull_policy_set_as_always())


def test_image_pull_policy_ir_containing_services_and_containers_with_image_pull_policy_already_set_as_always():
    assert_deep_equal(_optimize(optimizer.ImagePullPolicyOptimizer(), get_ir_with_image_pull_policy_set_as_always()),
                      get_ir_with_image_pull_policy_set_as_always())


# --- TestStripQuotation ----------------------------------------------------------

def test_strip_matching_single_quotation_marks_from_input_string():
    assert optimizer.strip_quotation("'testString'") == "testString"


def test_strip_matching_double_quotation_marks_from_input_string():
    assert optimizer.strip_quotation('"testString"') == "testString"


def test_expect_unmodified_string_for_input_string_without_any_quotation():
    assert optimizer.strip_quotation("testString") == "testString"


# --- TestOptimize (normalizeCharacterOptimizer) ------------------------------------

def test_normalize_ir_with_no_services():
    assert_deep_equal(_optimize(optimizer.NormalizeCharacterOptimizer(), get_ir_without_services()),
                      get_ir_without_services())


def test_normalize_ir_containing_services_that_have_no_containers():
    assert_deep_equal(_optimize(optimizer.NormalizeCharacterOptimizer(), get_ir_with_services_and_without_containers()),
                      get_ir_with_services_and_without_containers())


def test_normalize_ir_containing_services_and_containers_but_the_containers_have_no_environment_variables():
    assert_deep_equal(_optimize(optimizer.NormalizeCharacterOptimizer(),
                                get_ir_with_services_and_containers_without_env()),
                      get_ir_with_services_and_containers_without_env())


def test_normalize_an_ir_containing_services_and_containers_and_all_the_environment_variables_are_valid():
    assert_deep_equal(_optimize(optimizer.NormalizeCharacterOptimizer(),
                                get_ir_with_services_and_containers_with_valid_env()),
                      get_ir_with_services_and_containers_with_valid_env())


def test_normalize_an_ir_containing_services_and_containers_and_some_of_the_environment_variables_are_invalid():
    ir = _ir(_svc("svcname1", 2, {"name": "container-1", "env": _env(
                 ("NAME\t", "git-resource"), ("NO_PROXY", "'no-proxy.git.com'"), ("VALID_VARIABLE", "valid-variable"))}),
             _svc("svcname2", 4, {"name": "container-2", "env": _env(("\nNAME", "git-resource2"),
                                                                      (" PROXY", "  proxy.git.com "))}))
    assert_deep_equal(_optimize(optimizer.NormalizeCharacterOptimizer(), ir), get_expected_ir())


def test_normalize_some_environment_variables_invalid_but_their_names_contain_the_string_affinity():
    ir = _ir(_svc("svcname1", 2, {"name": "container-1", "env": _env(("NAME\t", "git-resource"),
                                                                      ("affinity", "with-pod-affinity "))}),
             _svc("svcname2", 4, {"name": "container-2", "env": _env(("\nNAME", "git-resource2"),
                                                                      (" PROXY", "  proxy.git.com "))}))
    assert_deep_equal(_optimize(optimizer.NormalizeCharacterOptimizer(), ir),
                      get_expected_ir_with_affinity_in_container())


# --- TestReplicaOptimizer ------------------------------------------------------------

def test_replica_ir_with_no_services():
    assert_deep_equal(_optimize(optimizer.ReplicaOptimizer(), get_ir_without_services()), get_ir_without_services())


def test_replica_ir_with_services_with_exact_default_minimum_replicas():
    assert_deep_equal(_optimize(optimizer.ReplicaOptimizer(), get_ir_with_services_with_default_minimum_replicas()),
                      get_ir_with_services_with_default_minimum_replicas())


def test_replica_ir_with_services_with_less_replicas_than_default_minimum_replicas():
    ir = _ir(_svc("svcname1", 1), _svc("svcname2", 1))
    assert_deep_equal(_optimize(optimizer.ReplicaOptimizer(), ir), get_ir_with_services_with_default_minimum_replicas())


def test_replica_ir_with_services_with_more_replicas_than_default_minimum_replicas():
    assert_deep_equal(_optimize(optimizer.ReplicaOptimizer(),
                                get_services_with_more_replicas_than_default_minimum_replicas()),
                      get_services_with_more_replicas_than_default_minimum_replicas())


def test_replica_ir_with_services_with_less_and_more_replicas_respectively_than_default_minimum_replicas():
    ir = _ir(_svc("svcname1", 1), _svc("svcname2", 4))
    assert_deep_equal(_optimize(optimizer.ReplicaOptimizer(), ir), get_expected_ir_with_modified_replicas())


# --- TestParameterizer ------------------------------------------------------------------

PARAM_HOST = "{{ .Release.Name }}-{{ .Values.ingresshost }}"


def _parameterize(ir):
    actual = parameterizer.parameterize(copy.deepcopy(ir))
    assert actual is not None
    return actual


def test_parameterizer_1_ir_with_no_services_no_storage():
    actual = _parameterize(get_ir_without_services())
    actual.target_cluster_spec.host = ""
    assert_deep_equal(actual, get_ir_without_services())


def test_parameterizer_2_ir_containing_services_that_have_no_containers():
    actual = _parameterize(get_ir_with_services_and_without_containers())
    want = get_ir_with_services_and_without_containers()
    want.values.services = {"svcname1": {}, "svcname2": {}}
    actual.target_cluster_spec.host = ""
    assert_deep_equal(actual, want)


def test_parameterizer_3_ir_containing_services_with_containers():
    actual = _parameterize(get_ir_with_services_and_containers())
    want = get_ir_with_services_and_containers()
    want.target_cluster_spec.host = PARAM_HOST
    want.services["svcname1"].containers[0]["image"] = \
        ':{{ index .Values.services "svcname1" "containers" "container-1" "imagetag"  }}'
    want.values.services = {"svcname1": {"container-1": "latest"}}
    assert_deep_equal(actual, want)


def test_parameterizer_4_ir_with_no_services_but_storage_storage_type_is_not_pvc_kind():
    actual = _parameterize(get_ir_with_storage_not_pvc_kind())
    actual.target_cluster_spec.host = ""
    assert_deep_equal(actual, get_ir_with_storage_not_pvc_kind())


def test_parameterizer_5_ir_with_no_services_but_storage_storage_type_is_pvc_kind():
    actual = _parameterize(get_ir_with_storage_pvc_kind())
    want = get_ir_with_storage_pvc_kind()
    want.storages[0].pvc_spec["storageClassName"] = "{{ .Values.storageclass }}"
    want.target_cluster_spec.host = PARAM_HOST
    want.values.services = {}
    want.values.storage_class = "storage-1cn"
    assert_deep_equal(actual, want)


def test_parameterizer_6_ir_with_no_services_check_ingress_parameterizer():
    actual = _parameterize(get_ir_without_services())
    want = get_ir_without_services()
    want.target_cluster_spec.host = PARAM_HOST
    assert_deep_equal(actual, want)


# --- beyond the ledger ------------------------------------------------------------------

def test_parameterize_mixed_storage_classes_skipped():
    ir = _ir()
    ir.storages = [irtypes.Storage(name="a", storage_type=irtypes.PVC_KIND, pvc_spec={"storageClassName": "x"}),
                   irtypes.Storage(name="b", storage_type=irtypes.PVC_KIND, pvc_spec={"storageClassName": "y"})]
    parameterizer.parameterize(ir)
    assert [s.pvc_spec["storageClassName"] for s in ir.storages] == ["x", "y"] and ir.values.storage_class == ""


def test_port_merge_by_image_name_and_url():
    qaengine.add_engine(DefaultEngine())
    ir = _ir(_svc("svcname1", 2, {"name": "container-1", "image": "image1"}),
             _svc("svcname2", 4, {"name": "container-2", "image": "reg.io/ns/image2"}))
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
    ir = _ir(_svc("s", 1, {"name": "c", "image": "unknown"}), _svc("empty", 1))
    optimizer.PortMergeOptimizer().optimize(ir)
    assert ir.services["s"].containers[0]["ports"] == [{"containerPort": 8080}]
    assert ir.services["empty"].containers == []
