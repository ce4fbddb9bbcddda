"""The expected trees are implementation-independent: every BASELINE and
coverage configuration, the regression corpus, and the BASELINE
configurations as CLI processes, through each twin switch
(``scripts/twin_check.py``; DEVIATIONS.md section 8).  Each switch runs in a
process of its own, because some are read at start-up (the bytecode bundle
when the package is imported, the template interpreter when
``utils/gotemplate.py`` is)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = {
    "default": {},
    "no-native": {"M2K_DISABLE_NATIVE": "1"},            # every pure-Python twin of the extension
    "python-yaml": {"M2K_NATIVE_YAML": "0"},              # go-yaml port in Python (parse)
    "python-marshal": {"M2K_NATIVE_MARSHAL": "0"},        # k8s/schema.py marshaller
    "detector-scripts": {"M2K_NATIVE_DETECT": "0"},       # the detector shell scripts, not the built-ins
    "template-interpreter": {"M2K_TEMPLATE_INTERPRET": "1"},  # text/template tree walker, not closures
    "no-bytecode-bundle": {"M2K_BYTECODE_BUNDLE": "0"},   # the normal import system
    "no-startcache": {"M2K_STARTCACHE": "0"},             # templates and regexes parsed from source
    "all-python": {"M2K_DISABLE_NATIVE": "1", "M2K_NATIVE_DETECT": "0", "M2K_TEMPLATE_INTERPRET": "1",
                   "M2K_BYTECODE_BUNDLE": "0", "M2K_STARTCACHE": "0"},
}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_expected_trees_through_twin(variant):
    env = {k: v for k, v in os.environ.items() if not k.startswith("M2K_")}
    env.update(VARIANTS[variant])
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "twin_check.py")], cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=900)
    lines = [l for l in p.stdout.decode().splitlines() if l.startswith("{")]
    assert lines, p.stderr.decode()[-3000:]
    d = json.loads(lines[-1])
    bad = {k: v for k, v in d["diffs"].items() if v}
    assert not bad and p.returncode == 0, (bad, p.stderr.decode()[-2000:])
    assert d["configs"] >= 39
