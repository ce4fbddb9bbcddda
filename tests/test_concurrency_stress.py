"""Python-level race checks - what ``go test -race`` (``/root/reference/Makefile:91-92``)
gives the reference for its goroutines (``packprovider.go:59-107``,
``dockerapiprovider.go:241-283``, ``httprestengine.go:43-83``).

* Every lazy loader and module-level cache that a worker thread can reach is
  initialised once, and no thread is handed a provisional value while another
  is still initialising (the round-4 race: ``ops/native.py`` marked itself
  tried before its import finished, and a collector thread asking meanwhile
  fell back to the subprocess runner).  Each test widens the initialisation
  window with a sleep and releases 8 threads at it together.
* ``scripts/stress.py`` (seeded CLI runs under a 1 us switch interval, thread
  start jitter and stand-in delays, every output tree diffed with its expected
  tree) runs in its small form; ``make stress`` runs 20 seeds.
"""

import os
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import stress  # noqa: E402


def _together(fn, n=8):
    """Run ``fn`` on ``n`` threads released at once; returns their results."""
    gate = threading.Barrier(n)
    out = [None] * n
    errs = []

    def body(i):
        gate.wait()
        try:
            out[i] = fn()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=body, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    return out


def _slow_counter(result, delay=0.05):
    calls = []
    lock = threading.Lock()

    def fn(*_a, **_k):
        with lock:
            calls.append(1)
        time.sleep(delay)
        return result() if callable(result) else result
    return fn, calls


# ---------------------------------------------------------------------------
# lazy loaders
# ---------------------------------------------------------------------------

def test_startcache_is_read_once_and_never_provisional(monkeypatch):
    import marshal
    from move2kube_amd.utils import startcache
    state = ({"t.tpl": marshal.dumps(("tree", 1))}, {})
    fn, calls = _slow_counter(state)
    monkeypatch.setattr(startcache, "_read_file", fn)
    monkeypatch.setattr(startcache, "_state", None)
    got = _together(lambda: startcache.template("t.tpl"))
    assert calls == [1]
    assert got == [("tree", 1)] * 8   # none saw the cache as unusable meanwhile


def test_gpu_library_loader_never_hands_out_a_provisional_none(monkeypatch):
    from move2kube_amd.ops import gpu
    lib = object()

    def opened():
        gpu._lib = lib
        return True
    fn, calls = _slow_counter(opened)
    monkeypatch.setattr(gpu, "_open_library", fn)
    monkeypatch.setattr(gpu, "_state", None)
    monkeypatch.setattr(gpu, "_lib", None)
    assert _together(gpu._load) == [lib] * 8
    assert calls == [1]


def test_k8s_native_marshaller_initialises_once(monkeypatch):
    import types
    from move2kube_amd.k8s import schema
    from move2kube_amd.ops import native
    inits = []

    def schema_init(structs, marshal_value):
        inits.append(1)
        time.sleep(0.05)

    def schema_marshal(d, typ):
        return d
    fake = types.SimpleNamespace(schema_init=schema_init, schema_marshal=schema_marshal)
    monkeypatch.setattr(native, "module", lambda: fake)
    monkeypatch.setattr(schema, "_native_fn", None)
    monkeypatch.delenv("M2K_NATIVE_MARSHAL", raising=False)
    got = _together(schema._native_marshal)
    assert inits == [1] and got == [schema_marshal] * 8


def test_cnb_provider_registry_builds_one_chain(monkeypatch):
    from move2kube_amd.containerizer.cnb import providers
    built = []
    for cls in (providers.DockerAPIProvider, providers.ContainerRuntimeProvider, providers.PackProvider,
                providers.RuncProvider):
        def make(cls=cls):
            built.append(cls.__name__)
            time.sleep(0.01)
            return object.__new__(cls)
        monkeypatch.setattr(providers, cls.__name__, make)
    monkeypatch.setattr(providers, "_providers", None)
    monkeypatch.setenv("M2K_DISABLE_CNB", "0")
    got = _together(providers.providers)
    assert all(g is got[0] for g in got)
    assert built == ["DockerAPIProvider", "ContainerRuntimeProvider", "PackProvider", "RuncProvider"]
    monkeypatch.setattr(providers, "_providers", None)


def test_yaml_loader_classes_build_once(monkeypatch):
    from move2kube_amd.utils import yamlio
    fn, calls = _slow_counter(object)
    monkeypatch.setattr(yamlio, "_Loaders", fn)
    monkeypatch.setattr(yamlio, "_loaders", None)
    got = _together(yamlio._lz)
    assert calls == [1] and all(g is got[0] for g in got)


def test_native_extension_loader_is_locked(monkeypatch):
    """The round-4 fix itself, through the same harness: the extension module
    for every thread, not None for the ones that asked during the import."""
    from move2kube_amd.ops import native
    real = native.module()
    import builtins
    orig_import = builtins.__import__

    def slow_import(name, *a, **k):
        if name.endswith("_m2k_native") or (a and a[2] and "_m2k_native" in a[2]):
            time.sleep(0.05)
        return orig_import(name, *a, **k)
    monkeypatch.setattr(builtins, "__import__", slow_import)
    monkeypatch.setattr(native, "_tried", False)
    monkeypatch.setattr(native, "_mod", None)
    assert _together(native.module) == [real] * 8


def test_problem_ids_are_unique_across_threads():
    from move2kube_amd.models import qa
    got = _together(lambda: [qa._next_id() for _ in range(500)])
    ids = [i for chunk in got for i in chunk]
    assert len(set(ids)) == len(ids) == 4000


def test_parse_cache_survives_overlapping_commands():
    """Two commands in one process (``api.Session`` users on threads) nest the
    command-scoped YAML memo; it lives until the last one leaves."""
    from move2kube_amd.utils import yamlio

    def cmd():
        with yamlio.parse_cache():
            time.sleep(0.01)
            return yamlio.load("a: [1, 2]\n")
    assert _together(cmd) == [{"a": [1, 2]}] * 8
    assert yamlio._memo is None and yamlio._memo_depth == 0


# ---------------------------------------------------------------------------
# the CLI under scripts/stress.py
# ---------------------------------------------------------------------------

def test_knobs_reach_every_pool_combination():
    combos = {tuple(sorted((k, v) for k, v in stress.knobs(s).items() if "SEED" not in k)) for s in range(24)}
    assert len(combos) == (len(stress.WORKERS) * len(stress.CNB_PARALLEL) * len(stress.NATIVE_DETECT)
                           * len(stress.DISABLE_NATIVE))


def test_switch_interval_exposes_a_check_then_act_race(tmp_path):
    """Canary for the harness: a deliberately unlocked lazy initialisation
    started from 8 threads runs more than once under the stress runs' switch
    interval (``scripts/m2k_switchy.py``), so a clean stress result means
    something."""
    prog = tmp_path / "racy.py"
    prog.write_text(
        "import sys, threading\n"
        "sys.setswitchinterval(1e-6)\n"
        "inits = []\n_v = None\n"
        "gate = threading.Barrier(8)\n"
        "def get():\n"
        "    global _v\n"
        "    gate.wait()\n"
        "    if _v is None:\n"
        "        inits.append(1)\n"
        "        x = 0\n"
        "        for i in range(20000): x += i\n"
        "        _v = x\n"
        "    return _v\n"
        "ts = [threading.Thread(target=get) for _ in range(8)]\n"
        "[t.start() for t in ts]; [t.join() for t in ts]\n"
        "print(len(inits))\n")
    runs = []
    for _ in range(5):
        runs.append(int(subprocess.run([sys.executable, str(prog)], stdout=subprocess.PIPE, check=True).stdout))
        if runs[-1] > 1:
            break
    assert max(runs) > 1, runs


def test_stress_harness_small_form(tmp_path):
    """Two seeds of every stress configuration (the five BASELINE ones, git
    repos, carried-over objects, and the five answered over the QA REST
    engine): no diff against the expected trees."""
    rows = stress.stress(stress.DEFAULT_CONFIGS, seeds=2, jobs=4, keep_on_failure=str(tmp_path / "kept"))
    bad = [(r["config"], r["seed"], r.get("error") or r["diff"]) for r in rows if not r["ok"]]
    assert not bad, bad
    assert len(rows) == 2 * len(stress.DEFAULT_CONFIGS)
    rest = [r for r in rows if r["config"].startswith("rest:")]
    assert rest and all(r["rest"]["answers"] > 0 for r in rest)


@pytest.mark.parametrize("seed", [3, 22])
def test_one_seeded_run_reproduces(seed):
    """A seed names its whole environment, so a failing seed can be rerun."""
    a, b = stress.run_one("cf", seed), stress.run_one("cf", seed)
    assert a["knobs"] == b["knobs"] and a["ok"] and b["ok"]
