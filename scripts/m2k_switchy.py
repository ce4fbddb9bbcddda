"""``python -m move2kube_amd`` with the interpreter's thread switch interval
cut to ``M2K_SWITCH_INTERVAL`` seconds (default 1e-6) before the package is
imported, so that every thread of the CLI (collector workers, CNB provider
probes, process waiters, the output remover, the QA REST server) is preempted
between almost every pair of bytecodes: the Python-level stand-in for
``go test -race`` (``/root/reference/Makefile:91-92``) that
``scripts/stress.py`` runs the configurations through.

With ``M2K_THREAD_JITTER_SEED`` set, every thread the command starts first
sleeps 0-``M2K_THREAD_JITTER_MS`` ms (default 2; drawn from a generator seeded
with the seed and the thread's start order), so which of two racing threads
reaches a shared initialisation first changes from seed to seed."""

import os
import runpy
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:   # run directly rather than through refconfigs' PYTHONPATH
    sys.path.insert(1, ROOT)


def _install_jitter(seed, max_ms):
    import random
    import time
    counter = [0]
    lock = threading.Lock()
    run = threading.Thread.run

    def jittered_run(self):
        with lock:
            counter[0] += 1
            k = counter[0]
        time.sleep(random.Random("%s/%d" % (seed, k)).uniform(0.0, max_ms) / 1e3)
        return run(self)
    threading.Thread.run = jittered_run


if os.environ.get("M2K_THREAD_JITTER_SEED"):
    _install_jitter(os.environ["M2K_THREAD_JITTER_SEED"], float(os.environ.get("M2K_THREAD_JITTER_MS", "2") or 2))
sys.setswitchinterval(float(os.environ.get("M2K_SWITCH_INTERVAL", "1e-6") or 1e-6))
runpy.run_module("move2kube_amd", run_name="__main__", alter_sys=True)
