"""The five BASELINE.json configurations over the reference's own ``samples/``
corpus, checked byte for byte against the reference-derived expected trees in
``tests/golden/reference/<config>`` (``benchmarks/refconfigs.py`` defines the
commands).  These trees are never rewritten by a test run: a difference is a
failure, to be fixed in the code or argued in
``tests/golden/reference/DEVIATIONS.md``.

The second half pins parts of those trees to the reference itself, without
going through our transformer: the byte-exact fixtures of the reference's
tests (``internal/containerizer/testdata``), the reference's own detector
scripts, and the build-script/output templates of
``internal/containerizer/scripts/constants.go`` and
``internal/transformer/templates/constants.go`` filled in by plain string
substitution.
"""

import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402

from conftest import REFERENCE, ref_path  # noqa: E402
from move2kube_amd.utils import yamlio  # noqa: E402


def _run_inprocess(name, tmp_path, steps=2):
    run = refconfigs.Run(name, str(tmp_path)).prepare()
    undo = run.apply_env()
    try:
        with run.session() as s:
            outs = [run.step(s) for _ in range(steps)]   # warm re-runs must not drift
    finally:
        undo()
    assert set(outs) == {run.out}
    return run.out


@pytest.mark.parametrize("name", sorted(refconfigs.CONFIGS))
def test_config_matches_reference_tree(name, tmp_path):
    out = _run_inprocess(name, tmp_path)
    golden = os.path.join(refconfigs.GOLDEN_REF, name)
    assert os.path.isdir(golden)
    assert refconfigs.diff_files(out, golden) == []


def test_configs_back_to_back_in_one_process(tmp_path):
    """No state of one run leaks into the next: configurations with CNB probing
    off (golang, helm-openshift) alternate with ones that probe it through the
    podman stand-in (cf collects buildpacks in process, java-cnb plans CNB)."""
    for i, name in enumerate(["golang", "cf", "helm-openshift", "java-cnb", "docker-compose", "cf"]):
        out = _run_inprocess(name, tmp_path / str(i), steps=1)
        assert refconfigs.diff_files(out, os.path.join(refconfigs.GOLDEN_REF, name)) == [], name


@pytest.mark.parametrize("name", [refconfigs.HEADLINE, "cf"])
def test_config_as_cli_processes(name, tmp_path):
    """The same trees from separate ``python -m move2kube_amd`` processes
    (``collect`` then ``translate`` for cf)."""
    run = refconfigs.Run(name, str(tmp_path)).prepare()
    out = run.run_cli()
    assert refconfigs.diff_files(out, os.path.join(refconfigs.GOLDEN_REF, name)) == []


def test_samples_are_the_reference_corpus():
    """``samples/`` is the reference's ``samples/`` byte for byte (BASELINE's corpus)."""
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference checkout not available")
    assert refconfigs.diff_files(refconfigs.SAMPLES, ref_path("samples")) == []


def test_reference_goldens_are_not_regenerated(monkeypatch, tmp_path):
    """``M2K_REGEN_GOLDEN`` only ever touches the regression set."""
    monkeypatch.setenv("M2K_REGEN_GOLDEN", "1")
    files = refconfigs.tree_files(refconfigs.GOLDEN_REF).values()
    before = {p: os.stat(p).st_mtime_ns for p in files}
    _run_inprocess("golang", tmp_path, steps=1)
    assert {p: os.stat(p).st_mtime_ns for p in files} == before


# ---------------------------------------------------------------------------
# anchors in the reference itself
# ---------------------------------------------------------------------------

def _go_consts(path):
    with open(path) as f:
        return dict(re.findall(r"\n\t(\w+) = `(.*?)`", f.read(), re.S))


def _golden(*parts):
    return os.path.join(refconfigs.GOLDEN_REF, *parts)


def _read(p):
    with open(p) as f:
        return f.read()


def _fill(tpl, **values):
    """``{{ .Key }}`` / ``{{.Key}}`` substitution for the flat templates."""
    for k, v in values.items():
        tpl = re.sub(r"\{\{\s*\.%s\s*\}\}" % k, lambda _m, v=v: v, tpl)
    assert "{{" not in tpl, tpl
    return tpl


@pytest.mark.reference
def test_dockerfile_matches_reference_fixture():
    """``internal/containerizer/testdata/dockerfilecontainerizer/getcontainer/normal/container.yaml``
    is the reference's own Dockerfile-containerizer output for ``samples/dockerfile``
    (nodejs detector); the expected trees carry the same bytes."""
    want = yamlio.load(_read(ref_path("internal", "containerizer", "testdata", "dockerfilecontainerizer",
                                      "getcontainer", "normal", "container.yaml")))["newfiles"]
    cdir = _golden(refconfigs.HEADLINE, "containers")
    assert _read(os.path.join(cdir, "dockerfile", "Dockerfile.dockerfile")) == want["Dockerfile.dockerfile"]
    assert _read(os.path.join(cdir, "dockerfile", "dockerfile-docker-build.sh")) == want["dockerfile-docker-build.sh"]
    # the nodejs sample goes through the same detector template
    assert _read(os.path.join(cdir, "nodejs", "Dockerfile.nodejs")) == want["Dockerfile.dockerfile"]


def _first_reference_detector(src):
    """Default technique = first matching detector in directory order
    (``GetFilesByName`` walk order, ``dockerfilecontainerizer.go:50-59``)."""
    detectors = ref_path("internal", "assets", "dockerfiles")
    for det in sorted(os.listdir(detectors)):
        d = os.path.join(detectors, det)
        p = subprocess.run(["bash", "m2kdfdetect.sh", src], cwd=d, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)
        if p.returncode == 0:
            return d, json.loads(p.stdout.decode() or "{}")
    return None, None


@pytest.mark.reference
def test_detector_dockerfiles_are_reference_templates():
    """Every ``Dockerfile.<svc>`` is the reference's detector template filled
    with the JSON that the reference's own detect script prints (run with bash;
    DEVIATIONS.md "platform shell")."""
    checked = 0
    for cfg in sorted(refconfigs.CONFIGS):
        croot = _golden(cfg, "containers")
        for dp, _dn, fns in os.walk(croot):
            for fn in fns:
                if not fn.startswith("Dockerfile."):
                    continue
                rel = os.path.relpath(dp, croot)
                if cfg == "cf":
                    src = refconfigs.CF_APP
                elif cfg in ("golang", "docker-compose"):
                    src = os.path.join(refconfigs.SAMPLES, cfg, rel) if rel != "." else os.path.join(
                        refconfigs.SAMPLES, cfg)
                else:
                    src = os.path.join(refconfigs.SAMPLES, rel)
                d, values = _first_reference_detector(src)
                assert d is not None, src
                want = _read(os.path.join(d, "Dockerfile"))
                for k, v in values.items():
                    want = re.sub(r"\{\{\s*\.%s\s*\}\}" % k, lambda _m, v=str(v): v, want)
                assert _read(os.path.join(dp, fn)) == want, (cfg, rel, d)
                checked += 1
    assert checked >= 12


@pytest.mark.reference
def test_build_scripts_are_reference_templates():
    """``*-docker-build.sh`` / ``*-cnb-build.sh`` / ``*-s2i-build.sh`` are
    ``internal/containerizer/scripts/constants.go`` filled in."""
    consts = _go_consts(ref_path("internal", "containerizer", "scripts", "constants.go"))
    checked = 0
    for cfg in sorted(refconfigs.CONFIGS):
        for dp, _dn, fns in os.walk(_golden(cfg, "containers")):
            for fn in fns:
                text = _read(os.path.join(dp, fn))
                if fn.endswith("-docker-build.sh"):
                    m = re.search(r"^docker build -f (\S+) -t (\S+) (\S+)$", text, re.M)
                    want = _fill(consts["Dockerbuild_sh"], Dockerfilename=m.group(1), ImageName=m.group(2),
                                 Context=m.group(3))
                elif fn.endswith("-cnb-build.sh"):
                    m = re.search(r"^pack build (\S+) -B (\S+)$", text, re.M)
                    want = _fill(consts["CNBBuilder_sh"], ImageName=m.group(1), Builder=m.group(2))
                elif fn.endswith("-s2i-build.sh"):
                    m = re.search(r"^s2i build \. (\S+) (\S+)$", text, re.M)
                    want = _fill(consts["S2IBuilder_sh"], Builder=m.group(1), ImageName=m.group(2))
                else:
                    continue
                assert text == want, (cfg, fn)
                checked += 1
    assert checked >= 20


@pytest.mark.reference
def test_output_scripts_are_reference_templates():
    """``deploy.sh``, ``helminstall.sh``, ``copysources.sh``, ``Chart.yaml``,
    the chart ``README.md`` and the Helm ``NOTES.txt`` header come from
    ``internal/transformer/templates/constants.go`` / ``k8stransformer.go:159-244``."""
    consts = _go_consts(ref_path("internal", "transformer", "templates", "constants.go"))
    proj = refconfigs.PROJECT
    rel_roots = {"golang": "../../samples/golang", "docker-compose": "../../samples/docker-compose",
                 "java-cnb": "../../java", "cf": "../../cf", "helm-openshift": "../../samples"}
    for cfg in sorted(refconfigs.CONFIGS):
        g = _golden(cfg)
        if cfg == "helm-openshift":
            assert _read(os.path.join(g, "helminstall.sh")) == _fill(consts["Helminstall_sh"], Project=proj)
            assert _read(os.path.join(g, proj, "Chart.yaml")) == _fill(consts["Chart_tpl"], Name=proj)
            assert _read(os.path.join(g, proj, "templates", "NOTES.txt")).startswith(consts["HelmNotes_txt"])
            assert _read(os.path.join(g, proj, "README.md")) == "This chart was created by Move2Kube\n"
            assert not os.path.exists(os.path.join(g, "deploy.sh"))
        else:
            assert _read(os.path.join(g, "deploy.sh")) == _fill(consts["Deploy_sh"], Project=proj)
        assert _read(os.path.join(g, "copysources.sh")) == _fill(consts["CopySources_sh"], RelRootDir=rel_roots[cfg],
                                                                  Dst="containers")
        assert _read(os.path.join(g, "Readme.md")).startswith(consts["K8sReadme_md"].split("{{")[0])


@pytest.mark.reference
def test_buildimages_and_pushimages_follow_reference_templates():
    """``buildimages.sh`` ranges over a map: Go templates visit map keys in
    sorted order, so that file is deterministic in the reference too."""
    consts = _go_consts(ref_path("internal", "transformer", "templates", "constants.go"))
    head_b = consts["Buildimages_sh"].split("{{range")[0]
    head_p = consts["Pushimages_sh"].split("{{range")[0]
    for cfg in sorted(refconfigs.CONFIGS):
        g = _golden(cfg)
        b = _read(os.path.join(g, "buildimages.sh"))
        assert b.startswith(head_b)
        body = b[len(head_b):]
        entries = re.findall(r"\ncd (\S*)\n\./(\S+)\ncd -", body)
        assert entries and body == "".join("\ncd %s\n./%s\ncd -" % e for e in entries) + "\n"
        assert [e[1] for e in entries] == sorted(e[1] for e in entries)
        p = _read(os.path.join(g, "pushimages.sh"))
        assert p.startswith(_fill(head_p, RegistryURL="docker.io", RegistryNamespace=refconfigs.PROJECT))
