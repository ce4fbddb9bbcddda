#!/usr/bin/env python3
"""Every expected tree through one implementation twin.

Each hot component has a native implementation and a pure-Python one that is
its executable specification (walk, Dockerfile sniffer, YAML emit and parse,
Kubernetes marshal, detectors, template compiler and interpreter, start-up
cache, bytecode bundle).  The switch that picks a twin is read from the
environment, some of them at start-up, so this script runs in a process whose
environment already holds the switch (``tests/test_twin_matrix.py`` starts it
once per switch):

* in process: the five BASELINE configurations, every coverage configuration
  of ``benchmarks/refconfigs.py`` and the builder's regression corpus
  (``tests/fixtures/extra_samples``), each diffed with its expected tree;
* as CLI processes (``python -m move2kube_amd``, start-up switches included):
  the five BASELINE configurations.

Prints one JSON object: ``{"variant": ..., "diffs": {config: [files]}}``
(empty lists when every tree is identical).  The reference has one
implementation per component (``internal/common/utils.go:47-120`` walks,
``internal/transformer/transformer.go:162-204`` writes); this keeps our twins
from drifting apart.
"""

import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "benchmarks")):
    if p not in sys.path:
        sys.path.insert(0, p)

import refconfigs  # noqa: E402

SWITCHES = ("M2K_DISABLE_NATIVE", "M2K_NATIVE_YAML", "M2K_NATIVE_MARSHAL", "M2K_NATIVE_DETECT",
            "M2K_TEMPLATE_INTERPRET", "M2K_BYTECODE_BUNDLE", "M2K_STARTCACHE")
EXTRA_CORPUS = os.path.join(ROOT, "tests", "fixtures", "extra_samples")
EXTRA_GOLDEN = os.path.join(ROOT, "tests", "golden", "regression", "extra_samples")


def _inprocess(name, work):
    run = refconfigs.Run(name, work).prepare()
    undo = run.apply_env()
    try:
        with run.session() as s:
            out = run.step(s)
    finally:
        undo()
    return refconfigs.diff_files(out, refconfigs.golden_dir(name), work=run.work)


def _extra_samples(work):
    from move2kube_amd import api
    src = os.path.join(work, "samples")
    shutil.copytree(EXTRA_CORPUS, src, symlinks=True)
    out = api.translate(src, os.path.join(work, "out"), name="samples")
    return refconfigs.diff_files(out, EXTRA_GOLDEN)


def main(argv):
    names = list(refconfigs.CONFIGS) + sorted(refconfigs.COVERAGE_CONFIGS)
    if argv and argv[0] == "--quick":   # BASELINE configurations only
        names = list(refconfigs.CONFIGS)
    from move2kube_amd.utils import log
    log.set_quiet()
    diffs = {}
    root = tempfile.mkdtemp(prefix="m2k-twins-")
    try:
        for i, name in enumerate(names):
            diffs[name] = _inprocess(name, os.path.join(root, "i%d" % i))
        diffs["regression/extra_samples"] = _extra_samples(os.path.join(root, "extra"))
        for i, name in enumerate(refconfigs.CONFIGS):
            run = refconfigs.Run(name, os.path.join(root, "c%d" % i)).prepare()
            out = run.run_cli()
            diffs["cli/" + name] = refconfigs.diff_files(out, refconfigs.golden_dir(name), work=run.work)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    variant = ",".join("%s=%s" % (k, os.environ[k]) for k in SWITCHES if k in os.environ) or "default"
    print(json.dumps({"variant": variant, "configs": len(diffs), "diffs": diffs}))
    return 1 if any(diffs.values()) else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
