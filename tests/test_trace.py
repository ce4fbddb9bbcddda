"""Phase tracing (``M2K_TRACE``): a translate records every pipeline phase as
Chrome trace events."""

import json
import os
import shutil

from move2kube_amd import api
from move2kube_amd.utils import trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_translate_records_phases(tmp_path, monkeypatch):
    src = tmp_path / "src"
    shutil.copytree(os.path.join(ROOT, "samples", "nodejs"), str(src / "nodejs"))
    (src / ".m2kignore").write_text(".\n")
    out_json = tmp_path / "trace.json"
    monkeypatch.setattr(trace, "_events", None)
    trace.enable(str(out_json))
    try:
        api.translate(str(src), str(tmp_path / "out"), name="t")
    finally:
        written = trace.flush()
        names = set(trace.summary())
        monkeypatch.setattr(trace, "_events", None)
    assert written == str(out_json)
    data = json.loads(out_json.read_text())
    evs = data["traceEvents"]
    assert evs and all(e["ph"] == "X" and e["dur"] >= 0 for e in evs)
    for want in ("plan", "translate", "Any2KubeTranslator", "detect-batch", "IngressOptimizer",
                 "RegistryCustomizer", "K8sTransformer.write_objects"):
        assert want in names, (want, sorted(names))
    cats = {e["cat"] for e in evs}
    assert {"command", "plan", "translate", "optimizer", "customizer", "transform", "detect"} <= cats


def test_span_is_free_when_disabled(monkeypatch):
    monkeypatch.setattr(trace, "_events", None)
    with trace.span("x"):
        pass
    assert trace.events() == [] and trace.flush() is None
