"""Small off-path branches: the translator registry when a translator fails
(reference ``internal/source/translator.go:48-66``: the counts are logged
before the error is checked, then "[%T] Failed : %s"), the abstract
translator, and the lazy regular expressions / modules."""

import pytest

import logparse
from move2kube_amd.models import plan as plantypes
from move2kube_amd.source import translator
from move2kube_amd.utils import lazyre, log


def test_a_failing_translator_is_warned_about_and_skipped(monkeypatch, capsys):
    from move2kube_amd.source.compose2kube import ComposeTranslator

    def boom(self, services, plan):
        raise RuntimeError("compose exploded")
    monkeypatch.setattr(ComposeTranslator, "translate", boom)
    plan = plantypes.new_plan()
    log.set_verbose(True)
    try:
        ir = translator.translate(plan)
    finally:
        log.set_verbose(False)
    assert ir.services == {}
    err = capsys.readouterr().err
    assert logparse.logged(err, "[*source.ComposeTranslator] Failed : compose exploded", "warning")
    msgs = [m for _lv, m in logparse.messages(err)]
    i = msgs.index("[*source.ComposeTranslator] Failed : compose exploded")
    assert msgs[i - 2:i] == ["Services translated : 0", "Containers translated : 0"]
    assert "[*source.CfManifestTranslator] Done" in msgs[i:]


def test_abstract_translator():
    t = translator.Translator()
    assert repr(t) == "*source.Translator" and t.get_translator_type() == ""
    with pytest.raises(NotImplementedError):
        t.get_service_options("", None)
    with pytest.raises(NotImplementedError):
        t.translate([], None)


def test_lazy_pattern_and_module():
    p = lazyre.lazy(r"a(b)")
    assert repr(p) == "LazyPattern('a(b)')"
    assert p.compiled().pattern == "a(b)"
    with pytest.raises(AttributeError):
        p.__wrapped__
    assert p.match("ab").group(1) == "b" and p.groups == 1
    m = lazyre.LazyModule("colorsys")
    with pytest.raises(AttributeError):
        m.__wrapped__
    assert m.rgb_to_hsv(0, 0, 0) == (0.0, 0.0, 0.0)


def test_dockerfile_planner_on_a_missing_input_path(tmp_path, capsys):
    """dockerfile2kube.go:44-50,147-152: the walk warning (unquoted), the
    planner's error, then the registry's "[%T] Failed"."""
    from move2kube_amd.source.dockerfile2kube import DockerfileTranslator
    gone = tmp_path / "gone"
    plan = plantypes.new_plan()
    with pytest.raises(RuntimeError, match="^stat %s: no such file or directory$" % gone):
        DockerfileTranslator().get_service_options(str(gone), plan)
    err = capsys.readouterr().err
    assert logparse.logged(err, "Error in walking through files due to : stat %s: no such file or directory" % gone,
                           "warning")
    assert logparse.logged(err, "Unable to get Dockerfiles : stat %s: no such file or directory" % gone, "error")


def test_dockerfile_translate_debug_lines(tmp_path, capsys):
    from move2kube_amd.source.dockerfile2kube import DockerfileTranslator
    (tmp_path / "Dockerfile").write_text("FROM alpine\nEXPOSE 8080\n")
    plan = plantypes.new_plan()
    plan.root_dir = str(tmp_path)
    (svc,) = DockerfileTranslator().get_service_options(str(tmp_path), plan)
    other = plantypes.Service.new("x", plantypes.ANY2KUBE)
    log.set_verbose(True)
    try:
        ir = DockerfileTranslator().translate([other, svc], plan)
    finally:
        log.set_verbose(False)
    assert list(ir.services) == [svc.service_name]
    err = capsys.readouterr().err
    assert logparse.logged(err, "The service x has translation type %s . Expected %s . Skipping."
                           % (plantypes.ANY2KUBE, plantypes.DOCKERFILE2KUBE), "debug")
    assert logparse.logged(err, "Translating %s" % svc.service_name, "debug")


def test_plugin_type_names_in_log_lines(monkeypatch, capsys):
    """``[%T] Begin ...`` / ``[%T] Failed : %s`` name the Go types of the
    reference's plugin lists: optimizer.go:31-33 (package ``optimize``),
    customizer.go:30-32, parameterizer.go:30-32 (package ``parameterize``)."""
    from move2kube_amd import customizer, optimizer, parameterizer
    assert [optimizer._go_type(o) for o in optimizer.get_optimizers()] == [
        "*optimize.normalizeCharacterOptimizer", "*optimize.ingressOptimizer", "*optimize.replicaOptimizer",
        "*optimize.imagePullPolicyOptimizer", "*optimize.portMergeOptimizer"]
    assert [customizer._go_type(c) for c in customizer.get_customizers()] == [
        "*customizer.registryCustomizer", "*customizer.storageCustomizer", "*customizer.ingressCustomizer"]
    assert [parameterizer._go_type(p) for p in parameterizer.get_parameterizers()] == [
        "*parameterize.imageNameParameterizer", "*parameterize.storageClassParameterizer",
        "*parameterize.ingressParameterizer"]

    class StorageCustomizer:
        def customize(self, ir):
            raise ValueError("No storage classes available in the cluster")

    class ReplicaOptimizer:
        def optimize(self, ir):
            raise ValueError("x")

    monkeypatch.setattr(customizer, "get_customizers", lambda: [StorageCustomizer()])
    monkeypatch.setattr(optimizer, "get_optimizers", lambda: [ReplicaOptimizer()])
    log.set_verbose(True)
    try:
        customizer.customize(object())
        optimizer.optimize(object())
    finally:
        log.set_verbose(False)
    err = capsys.readouterr().err
    assert logparse.logged(err, "[*customizer.storageCustomizer] Begin Customization", "debug")
    assert logparse.logged(err, "[*customizer.storageCustomizer] Failed : No storage classes available in the "
                                "cluster", "warning")
    assert logparse.logged(err, "[*optimize.replicaOptimizer] Failed : x", "warning")
