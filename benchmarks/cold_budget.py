#!/usr/bin/env python3
"""Where a configuration's cold CLI time above the bare interpreter goes,
from the wall clock of whole processes only (no instrumentation inside them):

* ``floor``      - ``python -c pass`` (the interpreter, ``site``, teardown):
  the driver's floor;
* ``bare_exit``  - ``python -c "import os; os._exit(0)"``: the same without
  the interpreter's teardown, which the CLI skips too (``_cli_exit``);
* ``imports``    - ``python -c "import ...; os._exit(0)"`` of exactly the
  package modules the configuration's command imports (recorded beforehand);
* ``version_c``  - the same ``version`` command run from ``-c`` (what
  ``__main__`` does, without ``runpy``);
* ``version``    - ``python -m move2kube_amd version``: the ``-m`` entry
  (``runpy``), the package and CLI start-up and a command that does nothing;
* ``command``    - the configuration's last command (``translate ...``).

The variants run round-robin, ``--runs`` rounds, so a drifting host hits all
alike; medians are reported, and the differences: ``floor - bare_exit`` (the
teardown the CLI does not pay), ``imports - bare_exit`` (module loading),
``version - bare_exit`` (the entry and CLI start-up, which includes the CLI's
own imports), ``version - version_c`` (the ``-m`` entry: ``runpy``) and
``command - imports`` (the command's work plus the ``-m`` entry).  One JSON
line per configuration.

    python benchmarks/cold_budget.py helm-openshift,golang --runs 40
"""

import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import refconfigs  # noqa: E402

_RECORD = r'''
import runpy, sys
sys.argv = ["move2kube_amd"] + ARGV
try:
    runpy.run_module("move2kube_amd", run_name="__main__", alter_sys=True)
except SystemExit:
    pass
'''


def _package_modules(argv, env, cwd):
    """The package modules a run of ``argv`` imports (in a child process
    that runs the CLI in process and prints ``sys.modules`` at exit)."""
    out = os.path.join(cwd, "modules.json")
    code = ("import atexit, json, sys\n"
            "atexit.register(lambda: json.dump(sorted(m for m in sys.modules if m.startswith('move2kube_amd')), "
            "open(%r, 'w')))\n" % out) + _RECORD.replace("ARGV", repr(argv))
    subprocess.run([sys.executable, "-c", code], env=env, cwd=cwd, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL, timeout=300)
    with open(out) as f:
        return [m for m in json.load(f) if m != "move2kube_amd.__main__"]


def budget(cfg, runs):
    root, _ = refconfigs.workdir_root("auto")
    work = tempfile.mkdtemp(prefix="m2k-budget-", dir=root)
    run = refconfigs.Run(cfg, work).prepare()
    env = run.env()
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    argv = run.cli_commands()[-1]
    mods = _package_modules(argv, env, work)
    py = sys.executable
    variants = {
        "floor": [py, "-c", "pass"],
        "bare_exit": [py, "-c", "import os; os._exit(0)"],
        "imports": [py, "-c", "import os, " + ", ".join(mods) + "; os._exit(0)"],
        "version_c": [py, "-c", "from move2kube_amd import _cli_exit, _cli_process\n_cli_process()\n"
                      "from move2kube_amd.cli.main import main\nimport gc\ngc.freeze()\n_cli_exit(main(['version']))"],
        "version": [py, "-m", "move2kube_amd", "version"],
        "command": [py, "-m", "move2kube_amd"] + argv,
    }
    times = {k: [] for k in variants}
    for i in range(runs + 1):
        names = list(variants)
        names = names[i % len(names):] + names[:i % len(names)]  # rotate the order each round
        for k in names:
            t = time.perf_counter()
            # no timeout=: with one, Popen.wait polls with sleeps of up to 50 ms
            # and the measured walls come out in steps of that schedule
            subprocess.run(variants[k], env=env, cwd=work, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           check=True)
            if i:  # round 0 primes the caches
                times[k].append((time.perf_counter() - t) * 1e3)
    med = {k: round(statistics.median(v), 3) for k, v in times.items()}
    return {"config": cfg, "runs": runs, "modules": len(mods), "median_ms": med,
            "teardown_skipped_ms": round(med["floor"] - med["bare_exit"], 3),
            "imports_ms": round(med["imports"] - med["bare_exit"], 3),
            "entry_and_cli_ms": round(med["version"] - med["bare_exit"], 3),
            "runpy_entry_ms": round(med["version"] - med["version_c"], 3),
            "command_over_imports_ms": round(med["command"] - med["imports"], 3),
            "command_over_floor_ms": round(med["command"] - med["floor"], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs")
    ap.add_argument("--runs", type=int, default=30)
    a = ap.parse_args()
    for cfg in a.configs.split(","):
        print(json.dumps(budget(cfg, a.runs)), flush=True)


if __name__ == "__main__":
    main()
