"""Collectors against stub kubectl / docker / cf executables on PATH."""

import os

import pytest

import logparse

from move2kube_amd import collector
from move2kube_amd.collector import cf as cfc
from move2kube_amd.collector.cluster import ClusterCollector
from move2kube_amd.collector.images import ImagesCollector, get_image_info
from move2kube_amd.utils import yamlio
from move2kube_amd.utils.constants import settings

STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "stubbin")


@pytest.fixture
def stub_path(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", STUBS + os.pathsep + "/usr/bin:/bin")
    # never a real cluster: a kubeconfig whose exec credentials send discovery
    # through the stub `kubectl proxy`, unless a test writes another one
    kc = tmp_path / "stub-kubeconfig"
    kc.write_text('{"current-context": "c", "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}], '
                  '"clusters": [{"name": "k", "cluster": {"server": "https://stub.invalid"}}], '
                  '"users": [{"name": "u", "user": {"exec": {"command": "stub-token", "apiVersion": "x"}}}]}')
    monkeypatch.setenv("KUBECONFIG", str(kc))
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    monkeypatch.setenv("M2K_STUB_LOG", str(tmp_path / "stub.log"))
    return tmp_path


def _read(path):
    return yamlio.load(open(path).read())


def test_cluster_collector_via_discovery(stub_path):
    out = stub_path / "out"
    ClusterCollector().collect("", str(out))
    files = os.listdir(str(out / "clusters"))
    assert len(files) == 1
    d = _read(str(out / "clusters" / files[0]))
    assert d["kind"] == "ClusterMetadata"
    assert d["metadata"]["name"] == "test-ctx\n"  # the reference keeps kubectl's newline
    assert d["spec"]["storageClasses"] == ["gold", "silver"]
    m = d["spec"]["apiKindVersionMap"]
    assert m["Deployment"] == ["apps/v1", "extensions/v1beta1"]
    assert m["Ingress"] == ["networking.k8s.io/v1", "networking.k8s.io/v1beta1", "extensions/v1beta1"]
    assert m["Route"] == ["route.openshift.io/v1"]
    assert m["Pod"] == ["v1"] and m["Service"] == ["v1"]
    # subresources count as in client-go's ServerGroupsAndResources
    assert m["Scale"] == ["apps/v1"]


def test_cluster_collector_fixed_mode_strips_context(stub_path):
    settings.compat = "fixed"
    ClusterCollector().collect("", str(stub_path / "o"))
    assert os.listdir(str(stub_path / "o" / "clusters"))[0].startswith("test-ctx")


def test_cluster_collector_without_cli(monkeypatch, tmp_path):
    monkeypatch.setenv("PATH", str(tmp_path))
    with pytest.raises(RuntimeError):
        ClusterCollector().collect("", str(tmp_path / "o"))


def test_group_order_policy():
    kinds = {"K": ["v1", "zzz.example.com/v1", "apps/v1", "extensions/v1beta1", "x.k8s.io/v1", "a.openshift.io/v1"]}
    ClusterCollector().group_order_policy(kinds)
    assert kinds["K"] == ["a.openshift.io/v1", "x.k8s.io/v1", "apps/v1", "extensions/v1beta1", "zzz.example.com/v1", "v1"]


def test_image_info_parsing():
    info = get_image_info(b'[{"RepoTags":["a:1"],"ContainerConfig":{"ExposedPorts":{"80/tcp":{}},"User":"root","WorkingDir":"/w"}}]')
    assert info.tags == ["a:1"] and info.ports == [80] and info.user_id == -1 and info.accessed_dirs == ["/w"]


def test_images_collector_from_compose(stub_path):
    src = stub_path / "src"
    src.mkdir()
    (src / "docker-compose.yml").write_text("version: '3'\nservices:\n  web:\n    image: app/web:1.0\n  cache:\n    image: redis:6\n")
    ImagesCollector().collect(str(src), str(stub_path / "out"))
    files = os.listdir(str(stub_path / "out" / "images"))
    assert len(files) == 1 and files[0].startswith("web-latest")
    d = _read(str(stub_path / "out" / "images" / files[0]))
    assert d["kind"] == "ImageMetadata"
    assert d["spec"]["ports"] == [443, 8080] and d["spec"]["userID"] == 1001


def test_cf_apps_collector(stub_path):
    cfc.CfAppsCollector().collect("", str(stub_path / "out"))
    files = os.listdir(str(stub_path / "out" / "cf"))
    assert len(files) == 1 and files[0].startswith("instanceapps-ap")
    d = _read(str(stub_path / "out" / "cf" / files[0]))
    apps = d["spec"]["applications"]
    assert [a["name"] for a in apps] == ["app1", "app2"]
    assert apps[0]["buildpack"] == "nodejs_buildpack" and apps[0]["instances"] == 2 and apps[0]["env"] == {"K": "V"}


def test_cf_buildpack_names_from_instance(stub_path):
    # a literal "null" string is passed through like the reference does
    assert cfc.get_cf_buildpack_names("") == ["staticfile_buildpack", "nodejs_buildpack", "null", "python_buildpack"]


def test_cf_container_types_matching():
    options = {"cloudfoundry/cnb:cflinuxfs3": ["org.cloudfoundry.nodejs", "org.cloudfoundry.python"],
               "gcr.io/buildpacks/builder": ["google.nodejs.runtime", "google.go.runtime"]}
    got = cfc.get_buildpack_containerizers(["nodejs_buildpack", "go_buildpack"], options)
    assert [b.buildpack_name for b in got] == ["nodejs_buildpack", "go_buildpack"]
    assert got[1].target_options == ["gcr.io/buildpacks/builder"]


def test_collect_orchestrator_filters_by_annotation(stub_path):
    out = stub_path / "m2k_collect"
    collector.collect("", str(out), ["CF"])
    assert sorted(os.listdir(str(out))) == ["cf"]


# ---------------------------------------------------------------------------
# discovery transport: one pass, no process per group/version
# ---------------------------------------------------------------------------

FAKE_API = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "fake_apiserver.py")


class _FakeAPI:
    def __init__(self, tmp_path, *args):
        import subprocess
        import sys
        self.log = str(tmp_path / "api.log")
        env = dict(os.environ, M2K_FAKE_API_LOG=self.log)
        self.p = subprocess.Popen([sys.executable, FAKE_API] + list(args), stdout=subprocess.PIPE, env=env)
        line = self.p.stdout.readline().decode()
        self.port = int(line.rsplit(":", 1)[1])

    def requests(self):
        return open(self.log).read().splitlines() if os.path.exists(self.log) else []

    def stop(self):
        self.p.terminate()
        self.p.wait(timeout=10)
        self.p.stdout.close()


def _kubeconfig(path, server, user):
    import json
    path.write_text(json.dumps({
        "apiVersion": "v1", "kind": "Config", "current-context": "c",
        "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}],
        "clusters": [{"name": "k", "cluster": server}],
        "users": [{"name": "u", "user": user}]}))
    return str(path)


def _stub_calls(stub_path):
    p = stub_path / "stub.log"
    return p.read_text().splitlines() if p.exists() else []


def _collect_map(stub_path, out="out"):
    ClusterCollector().collect("", str(stub_path / out))
    (f,) = os.listdir(str(stub_path / out / "clusters"))
    return _read(str(stub_path / out / "clusters" / f))


def test_discovery_direct_from_kubeconfig_spawns_no_process(stub_path, monkeypatch):
    """Token auth straight to the API server: the only CLI calls are the context
    name and the storage classes; discovery itself forks nothing, and the
    result equals the proxy path's."""
    via_proxy = _collect_map(stub_path, "o1")
    api = _FakeAPI(stub_path, "--token", "s3cret")
    try:
        monkeypatch.setenv("KUBECONFIG", _kubeconfig(stub_path / "kc", {"server": "http://127.0.0.1:%d" % api.port},
                                                     {"token": "s3cret"}))
        (stub_path / "stub.log").write_text("")
        direct = _collect_map(stub_path, "o2")
    finally:
        api.stop()
    assert _stub_calls(stub_path) == ["kubectl config current-context", "kubectl get sc -o yaml"]
    reqs = api.requests()
    assert len(reqs) == 2 + 6 and all(r.endswith("Bearer s3cret") for r in reqs)
    assert direct == via_proxy


def test_discovery_over_tls_with_ca_and_client_cert(stub_path, monkeypatch):
    import base64
    import shutil
    import subprocess
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    key, crt = str(stub_path / "k.pem"), str(stub_path / "c.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", crt,
                    "-days", "1", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    api = _FakeAPI(stub_path, "--tls", crt, key)
    try:
        b64 = lambda p: base64.b64encode(open(p, "rb").read()).decode()  # noqa: E731
        monkeypatch.setenv("KUBECONFIG", _kubeconfig(
            stub_path / "kc", {"server": "https://127.0.0.1:%d" % api.port, "certificate-authority-data": b64(crt)},
            {"client-certificate-data": b64(crt), "client-key-data": b64(key)}))
        m = _collect_map(stub_path)["spec"]["apiKindVersionMap"]
    finally:
        api.stop()
    assert m["Deployment"] == ["apps/v1", "extensions/v1beta1"]
    assert not any("proxy" in c for c in _stub_calls(stub_path))


def test_discovery_exec_plugin_uses_one_proxy_process(stub_path, monkeypatch):
    monkeypatch.setenv("KUBECONFIG", _kubeconfig(stub_path / "kc", {"server": "https://example.invalid"},
                                                 {"exec": {"command": "get-token", "apiVersion": "x"}}))
    m = _collect_map(stub_path)["spec"]["apiKindVersionMap"]
    assert m["Route"] == ["route.openshift.io/v1"]
    calls = _stub_calls(stub_path)
    assert sum(1 for c in calls if c.startswith("kubectl proxy")) == 1
    assert not any("--raw" in c for c in calls)


def test_discovery_failed_group_falls_back_to_cli_in_reference_mode(stub_path, monkeypatch):
    """client-go's ServerGroupsAndResources errors when a group fails, so the
    reference falls back to the CLI; "fixed" keeps the groups that answered."""
    api = _FakeAPI(stub_path, "--fail", "/apis/route.openshift.io/v1")
    try:
        monkeypatch.setenv("KUBECONFIG", _kubeconfig(stub_path / "kc", {"server": "http://127.0.0.1:%d" % api.port}, {}))
        m = _collect_map(stub_path, "ref")["spec"]["apiKindVersionMap"]
        assert any(c.startswith("kubectl api-resources") for c in _stub_calls(stub_path))
        assert "Route" not in m and m["Deployment"] == ["apps/v1"]
        settings.compat = "fixed"
        (stub_path / "stub.log").write_text("")
        m = _collect_map(stub_path, "fixed")["spec"]["apiKindVersionMap"]
        assert not any(c.startswith("kubectl api-resources") for c in _stub_calls(stub_path))
        assert "Route" not in m and m["Ingress"][0] == "networking.k8s.io/v1"
    finally:
        api.stop()


def test_collectors_run_concurrently_with_ordered_logs(monkeypatch, tmp_path):
    """Selected collectors run at the same time; their log lines come out in
    collector order; a failing one is a warning; a fatal one is raised after
    the lines of the collectors before it."""
    import io
    import time
    import move2kube_amd.collector as coll
    from move2kube_amd.utils import log

    class Slow(coll.Collector):
        annotations = ("x",)

        def __init__(self, name, delay, fail=None):
            self.name, self.delay, self.fail = name, delay, fail

        def __repr__(self):
            return self.name

        def collect(self, input_path, output_path):
            time.sleep(self.delay)
            log.info("%s working", self.name)
            if self.fail == "error":
                raise ValueError("boom")
            if self.fail == "fatal":
                log.fatal("%s cannot go on", self.name)

    buf = io.StringIO()
    monkeypatch.setattr(log.logger, "stream", buf)
    monkeypatch.setattr(coll, "get_collectors", lambda annotations=(): [Slow("a", 0.3), Slow("b", 0.1, "error"), Slow("c", 0.2)])
    t0 = time.perf_counter()
    coll.collect("", str(tmp_path / "out"), ["x"])
    assert time.perf_counter() - t0 < 0.55
    msgs = [m for _lv, m in logparse.messages(buf.getvalue())]
    assert msgs == ["Begin collection", "[a] Begin collection", "a working", "[a] Done", "[b] Begin collection",
                    "b working", '[b] failed. Error: "boom"', "[c] Begin collection", "c working", "[c] Done",
                    "Collection done"]
    buf.truncate(0)
    buf.seek(0)
    monkeypatch.setattr(coll, "get_collectors", lambda annotations=(): [Slow("a", 0.1), Slow("f", 0.0, "fatal"), Slow("c", 0.0)])
    with pytest.raises(log.FatalError):
        coll.collect("", str(tmp_path / "out"), ["x"])
    msgs = [m for _lv, m in logparse.messages(buf.getvalue())]
    assert msgs[-1] == "f cannot go on" and "[a] Done" in msgs and "[c] Done" not in msgs


def test_held_log_lines_nest(monkeypatch):
    import io
    import threading
    from move2kube_amd.utils import log
    buf = io.StringIO()
    monkeypatch.setattr(log.logger, "stream", buf)
    with log.hold() as outer:
        log.info("one")
        inner_lines = []

        def work():
            with log.hold() as h:
                log.info("two")
            inner_lines.extend(h.lines)
        t = threading.Thread(target=work)
        t.start()
        t.join()
        log.emit(inner_lines)
        log.info("three")
    assert buf.getvalue() == ""
    log.emit(outer.lines)
    assert [m for _lv, m in logparse.messages(buf.getvalue())] == ["one", "two", "three"]


def test_images_collector_inspects_concurrently(tmp_path, monkeypatch):
    """`docker inspect` runs for several images at once; every image still
    gets its metadata file."""
    import time
    from move2kube_amd.collector.images import ImagesCollector
    bindir = tmp_path / "bin"
    bindir.mkdir()
    (bindir / "docker").write_text(
        '#!/bin/sh\n[ "$1" = inspect ] || exit 1\nsleep 0.3\n'
        'printf \'[{"RepoTags": ["%s"], "ContainerConfig": {"User": "1001", "WorkingDir": "/app", '
        '"ExposedPorts": {"8080/tcp": {}}}}]\' "$2"\n')
    os.chmod(str(bindir / "docker"), 0o755)
    monkeypatch.setenv("PATH", str(bindir) + os.pathsep + os.environ["PATH"])
    src = tmp_path / "src"
    src.mkdir()
    (src / "docker-compose.yml").write_text(
        "version: '3'\nservices:\n" + "".join("  s%d:\n    image: img%d:1\n" % (i, i) for i in range(4)))
    t0 = time.perf_counter()
    ImagesCollector().collect(str(src), str(tmp_path / "out"))
    assert time.perf_counter() - t0 < 1.0   # 4 x 0.3 s one after another would be 1.2 s
    files = sorted(os.listdir(str(tmp_path / "out" / "images")))
    assert [f.split("-")[0] for f in files] == ["img%d" % i for i in range(4)]


def test_cf_commands_never_overlap(tmp_path, monkeypatch):
    """Concurrent collectors still run one `cf` command at a time."""
    import threading
    import move2kube_amd.collector as coll
    bindir = tmp_path / "bin"
    bindir.mkdir()
    (bindir / "cf").write_text('#!/bin/sh\nif [ -e "$LOG/busy" ]; then echo overlap >> "$LOG/overlaps"; fi\n'
                               'touch "$LOG/busy"\nsleep 0.1\nrm -f "$LOG/busy"\necho ok\n')
    os.chmod(str(bindir / "cf"), 0o755)
    monkeypatch.setenv("PATH", str(bindir) + os.pathsep + os.environ["PATH"])
    monkeypatch.setenv("LOG", str(tmp_path))
    threads = [threading.Thread(target=coll.run, args=(["cf", "curl", "/v2/apps"],)) for _ in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not (tmp_path / "overlaps").exists()


def test_version_sort_is_semver_precedence():
    """sortVersionList (clustercollector.go:412-456) ranks versions by
    Masterminds semver after alpha/beta become prerelease tags: a newer major
    beta comes before the older GA version."""
    from move2kube_amd.collector.cluster import ClusterCollector
    assert ClusterCollector.sort_versions(["v1", "v2beta1", "v2beta2"]) == ["v2beta2", "v2beta1", "v1"]
    assert ClusterCollector.sort_versions(["v1beta1", "v1", "v1alpha1", "v1beta2", "v2alpha1", "v1beta10"]) == \
        ["v2alpha1", "v1", "v1beta10", "v1beta2", "v1beta1", "v1alpha1"]
    assert ClusterCollector().cluster_by_groups_and_sort_versions(
        ["autoscaling/v1", "autoscaling/v2beta1", "v1", "batch/v1beta1", "batch/v1"]) == \
        ["v1", "autoscaling/v2beta1", "autoscaling/v1", "batch/v1", "batch/v1beta1"]


def test_version_sort_keeps_unparsable_versions_last(capsys):
    from move2kube_amd.collector.cluster import ClusterCollector
    from move2kube_amd.utils import log
    log.set_verbose(False)
    assert ClusterCollector.sort_versions(["v1beta", "v1", "latest"]) == ["v1", "v1beta", "latest"]
    err = capsys.readouterr().err
    assert "Skipping Version: v1-beta." in err and "Skipping Version: latest" in err


@pytest.mark.parametrize("output,warning", [
    ("error: You must be logged in to the server (Unauthorized)",
     "Error while running kubectl. Please configure the cluster authentication with following instructions: "
     "[https://kubernetes.io/docs/reference/kubectl/cheatsheet/#kubectl-context-and-configuration]"),
    ("The connection to the server localhost:8080 was refused",
     "Error while fetching storage classes using command [%s get sc -o yaml]" % os.path.join(STUBS, "kubectl")),
])
def test_storage_class_errors_are_interpreted(stub_path, monkeypatch, capsys, output, warning):
    """getStorageClasses / interpretError (clustercollector.go:124-173)."""
    from move2kube_amd.collector import CommandError
    from move2kube_amd.utils import log
    log.set_verbose(False)
    monkeypatch.setenv("M2K_STUB_SC_ERROR", output)
    with pytest.raises(CommandError):
        ClusterCollector().get_storage_classes()
    assert logparse.logged(capsys.readouterr().err, warning, "warning")


def test_interpret_error_for_oc():
    c = ClusterCollector()
    c.cluster_cmd = "oc"
    assert c.interpret_error("error: Username or password wrong") == \
        "Please login to cluster before running collect. (e.g. oc login <cluster url> --token=<token string>)"
    assert c.interpret_error("no route to host") == ""


def test_collector_registry_matches_the_classes():
    """get_collectors selects by the registry's annotations without importing
    the other collectors; they must be each class's own."""
    got = collector.get_collectors()
    assert [type(c).__name__ for c in got] == [r[1] for r in collector.REGISTRY]
    for c, (_, _, ann) in zip(got, collector.REGISTRY):
        assert tuple(c.get_annotations()) == ann
    assert [type(c).__name__ for c in collector.get_collectors(["cf"])] == ["CFContainerTypesCollector", "CfAppsCollector"]


def test_no_kubeconfig_fails_the_api_path_as_client_go_does(stub_path, monkeypatch, capsys):
    """clustercollector.go:179-186,301-306 and collect: with no kubeconfig and
    no in-cluster service account, client-go's ClientConfig() fails with
    ErrEmptyConfig; the CLI fallback collects instead, and no proxy starts."""
    monkeypatch.setenv("KUBECONFIG", str(stub_path / "none"))
    m = _collect_map(stub_path)["spec"]["apiKindVersionMap"]
    assert m["Deployment"] == ["apps/v1"]
    calls = _stub_calls(stub_path)
    assert not any(c.startswith("kubectl proxy") for c in calls)
    assert any(c.startswith("kubectl api-resources") for c in calls)
    err = capsys.readouterr().err
    empty = ("invalid configuration: no configuration has been provided, try setting KUBERNETES_MASTER "
             "environment variable")
    assert logparse.logged(err, 'Failed to get the default config for the cluster API client. Error: "%s"' % empty,
                           "warning")
    assert logparse.logged(err, "Failed to api handle for cluster", "warning")
    assert logparse.logged(err, 'Failed to collect using the API. Error: "%s" . Falling back to using the CLI.'
                           % empty, "warning")


def test_server_groups_failure_lines(stub_path, monkeypatch, capsys):
    api = _FakeAPI(stub_path, "--fail", "/apis")
    try:
        monkeypatch.setenv("KUBECONFIG", _kubeconfig(stub_path / "kc", {"server": "http://127.0.0.1:%d" % api.port}, {}))
        _collect_map(stub_path)
    finally:
        api.stop()
    err = capsys.readouterr().err
    assert logparse.logged(err, "API request for server-group list failed", "error")
    assert logparse.logged(err, "Failed to retrieve preferred group information from cluster", "warning")


def test_kinds_failure_lines(stub_path, monkeypatch, capsys):
    api = _FakeAPI(stub_path, "--fail", "/apis/apps/v1")
    try:
        monkeypatch.setenv("KUBECONFIG", _kubeconfig(stub_path / "kc", {"server": "http://127.0.0.1:%d" % api.port}, {}))
        _collect_map(stub_path)
    finally:
        api.stop()
    assert logparse.logged(capsys.readouterr().err, "Failed to retrieve <kind, group-version> information from cluster",
                           "warning")


def _explain_cc(monkeypatch, outputs):
    """A ClusterCollector whose CLI answers from ``outputs`` (argv tuple ->
    bytes, or an Exception to raise)."""
    from move2kube_amd.collector import CommandError
    cc = ClusterCollector()
    monkeypatch.setattr(cc, "get_cluster_command", lambda: "kubectl")

    def run(*args, combined=False):
        out = outputs.get(args, CommandError(["kubectl"] + list(args), 1))
        if isinstance(out, Exception):
            raise out
        return out
    monkeypatch.setattr(cc, "_run", run)
    return cc


def test_cli_explain_without_a_kind_line_is_kind_empty_in_reference_mode(monkeypatch):
    """clustercollector.go:616-623: an explain whose first line is not KIND
    (newer kubectl prints GROUP first) returns the command's nil error, so
    the kind and version are "" and the map gets an entry for kind ""."""
    outputs = {("api-resources", "-o", "name"): b"deployments.apps\npods\n",
               ("explain", "deployments"): b"GROUP:      apps\nKIND:       Deployment\nVERSION:    v1\n",
               ("explain", "pods"): b"KIND:     Pod\nVERSION:  v1\n"}
    for gv in ("apps/v1", "apps/v1beta2", "apps/v1beta1"):
        outputs[("explain", "", "--api-version=" + gv, "--recursive")] = b"KIND: x\n"
    cc = _explain_cc(monkeypatch, outputs)
    assert cc.collect_using_cli() == {"": [], "Pod": ["v1"]}
    settings.compat = "fixed"
    assert cc.collect_using_cli() == {"Pod": ["v1"]}


def test_cli_unsupported_versions_are_debug_lines_with_the_reason(monkeypatch, capsys):
    from move2kube_amd.utils import log
    outputs = {("api-resources", "-o", "name"): b"deployments.apps\n",
               ("explain", "deployments"): b"KIND: Deployment\nVERSION: apps/v1\n",
               ("explain", "Deployment", "--api-version=apps/v1", "--recursive"): b"KIND: Deployment\nVERSION: v1\n",
               ("explain", "Deployment", "--api-version=apps/v1beta2", "--recursive"): b"short",
               ("explain", "Deployment", "--api-version=apps/v1beta1", "--recursive"): b"KIND: x\nFIELDS:\n"}
    cc = _explain_cc(monkeypatch, outputs)
    log.set_verbose(True)
    try:
        assert cc.collect_using_cli() == {"Deployment": ["apps/v1"]}
    finally:
        log.set_verbose(False)
    err = capsys.readouterr().err
    assert logparse.logged(err, "Group version not found by CLI for kind [Deployment] : Description incomplete",
                           "debug")
    assert logparse.logged(err, "Group version not found by CLI for kind [Deployment] : GV [apps/v1beta1] not found",
                           "debug")


def test_storage_class_output_the_decode_refuses_or_items_of_another_type(monkeypatch, capsys):
    """clustercollector.go:137-160: a yaml.v3 error is logged and no class is
    kept; an item that is not a mapping is warned about with %T of the failed
    assertion's zero value."""
    cc = _explain_cc(monkeypatch, {("get", "sc", "-o", "yaml"): b"items: [unclosed\n"})
    import pytest as _pytest
    with _pytest.raises(Exception):
        cc.get_storage_classes()
    assert logparse.logged_containing(capsys.readouterr().err, "Error in unmarshalling yaml: yaml: ", "error")
    cc = _explain_cc(monkeypatch, {("get", "sc", "-o", "yaml"):
                                   b"items:\n- metadata: {name: gold}\n- just-a-string\n"})
    assert cc.get_storage_classes() == ["gold"]
    assert logparse.logged(capsys.readouterr().err, "Unknown type detected in cluster metadata "
                           "[map[string]interface {}]", "warning")


def test_cluster_output_directory_that_cannot_be_made(tmp_path, capsys):
    (tmp_path / "clusters").write_text("a file")
    with pytest.raises(RuntimeError):
        ClusterCollector().collect("", str(tmp_path))
    assert logparse.logged(capsys.readouterr().err, 'Unable to create output directory at path "%s" Error: "mkdir %s: '
                           'not a directory"' % (tmp_path / "clusters", tmp_path / "clusters"), "error")
