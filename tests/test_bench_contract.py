"""bench.py contract: one JSON line, weak-scaling aggregate over ranks; the
2-rank run goes through torch.distributed.run with the gloo backend on CPU."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

try:  # bench.py joins torch.distributed; the image's builder stage has no torch
    import torch  # noqa: F401
    _HAVE_TORCH = True
except ImportError:
    _HAVE_TORCH = False
needs_torch = pytest.mark.skipif(not _HAVE_TORCH, reason="bench.py needs torch")

def refconfigs_names():
    return ["cf", "docker-compose", "golang", "helm-openshift", "java-cnb"]


KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _env():
    env = dict(os.environ)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def _last_json(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@needs_torch
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="CPU-only contract test")
def test_single_rank():
    p = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--check-runs", "1",
                        "--large-tree", "20,60"], cwd=ROOT,
                       env=_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr.decode()
    d = _last_json(p.stdout.decode())
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["value"] > 0
    assert d["manifest_diff_vs_ref"] == 0 and d["manifest_diff_vs_ref_headline"] == 0, \
        (d["manifest_diff_vs_ref_headline"], {k: v.get("manifest_diff_vs_ref") for k, v in d["per_config"].items()})
    assert sorted(d["per_config"]) == ["cf", "docker-compose", "golang", "helm-openshift", "java-cnb", "large-tree"]
    lt = d["per_config"]["large-tree"]
    assert sorted(lt["large_tree_translate_ms_per_service"]) == ["20", "60"] and lt["ratio_largest_vs_smallest"] > 0
    assert all(v["manifest_diff_vs_ref"] == 0 for k, v in d["per_config"].items() if k != "large-tree")
    # p50 and interquartile range per configuration, and the ratio to the
    # previous round's driver line (benchmarks/prev_round_bench.json)
    for name in refconfigs_names():
        row = d["per_config"][name]
        assert row["runs"] == 1 and row["warm_iqr_ms"] == 0 and row["cold_iqr_ms"] == 0
        assert row["cold_over_floor_iqr_ms"] == 0
        vs = d["per_config_vs_prev"][name]
        assert vs["warm_ratio"] > 0 and vs["warm_prev_p50_ms"] > 0 and vs["cold_over_floor_prev_p50_ms"] > 0
    assert d["per_config_vs_prev"]["prev"] == os.path.join("benchmarks", "prev_round_bench.json")
    assert len(d["host"]["per_rank"]) == 1 and d["host"]["pinned"] is False
    # the headline names BASELINE.json configuration 5 verbatim
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert d["config"]["model"] in json.load(f)["configs"]


@needs_torch
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="CPU-only contract test")
def test_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--steps", "1",
           "--warmup", "1", "--check-runs", "0"]
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert d["n_gpus"] == 2
    assert d["config"]["parallelism"] == "dp2"
    assert d["scaling"] == "weak"
    # host accounting of the timed region: CPU summed over both ranks, the
    # slowest rank's median step
    h = d["host"]
    assert h["cpus"] >= 1 and h["cpu_ms_per_step_all_ranks"] > 0
    assert 0 <= h["cpu_sys_ms_per_step_all_ranks"] <= h["cpu_ms_per_step_all_ranks"]
    assert h["slowest_rank_step_p50_ms"] > 0
    # each rank's own accounting: user / sys CPU, step p50 / p90, context switches
    assert len(h["per_rank"]) == 2
    for r in h["per_rank"]:
        assert set(r) == {"user_ms", "sys_ms", "step_p50_ms", "step_p90_ms", "nvcsw", "nivcsw", "cpus"}
        assert r["user_ms"] > 0 and r["step_p50_ms"] > 0 and r["cpus"] >= 1
    assert set(h["ctx_switches_per_step_all_ranks"]) == {"voluntary", "involuntary"}
    # CPU over ranks is user + sys of every rank (not the switch counts)
    total = sum(r["user_ms"] + r["sys_ms"] for r in h["per_rank"])
    assert abs(h["cpu_ms_per_step_all_ranks"] - total) < 0.01 * max(1.0, total) + 0.01


@needs_torch
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="CPU-only contract test")
def test_one_rank_under_torchrun_joins_the_group():
    """Launched by torchrun with one rank, bench.py still initialises the
    process group (the collective path of the multi-GPU runs) and reports
    the work tree it used."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29534", "bench.py", "--steps", "1",
           "--warmup", "1", "--check-runs", "0", "--workdir", "disk"]
    p = subprocess.run(cmd, cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert d["n_gpus"] == 1 and d["workdir_fs"] == "disk" and "on disk" in d["data"]


def test_baseline_configs_bench_golang():
    """benchmarks/baseline_configs.py (BASELINE.md per-configuration wall clock):
    one warm, one fork-model emulation and one cold CLI run of the golang
    config, all identical to the reference-derived expected tree."""
    p = subprocess.run([sys.executable, os.path.join("benchmarks", "baseline_configs.py"), "--runs", "1",
                        "--emulation-runs", "1", "--configs", "golang"], cwd=ROOT, env=_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    rows = [json.loads(l) for l in p.stdout.decode().splitlines() if l.startswith("{")]
    cfg = [r for r in rows if r.get("config") == "golang"]
    assert len(cfg) == 1 and cfg[0]["manifest_diff_vs_ref"] == 0
    assert cfg[0]["warm_p50_ms"] > 0 and cfg[0]["cold_p50_ms"] > 0
    assert cfg[0]["python_emulation_of_reference_fork_model_p50_ms"] > 0


def test_cold_diagnostics_scripts_run():
    """scripts/cold_phases.py and benchmarks/cold_trace.py (the cold-start
    breakdowns kept under profiles/) still run and report their fields."""
    p = subprocess.run([sys.executable, os.path.join("scripts", "cold_phases.py"), "golang", "--runs", "1"],
                       cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert d["command"] == "translate" and d["first_main"] > 0 and d["second_main"] > 0
    p = subprocess.run([sys.executable, os.path.join("benchmarks", "cold_trace.py"), "helm-openshift", "--runs", "1"],
                       cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert d["wall_p50_ms"] > 0 and "operator-sdk wait" in d["span_p50_ms"] and "plan" in d["span_p50_ms"]
    p = subprocess.run([sys.executable, os.path.join("benchmarks", "cold_importtime.py"), "golang", "--runs", "1"],
                       cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert d["self_us_ours"] > 0 and "move2kube_amd.cli.main" in d["self_cum_us"]
    p = subprocess.run([sys.executable, os.path.join("benchmarks", "cold_budget.py"), "golang", "--runs", "1"],
                       cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert d["modules"] > 20 and set(d["median_ms"]) == {"floor", "bare_exit", "imports", "version_c", "version", "command"}
    p = subprocess.run([sys.executable, os.path.join("benchmarks", "switch_ab.py"), "M2K_STARTCACHE", "0", "1",
                        "golang", "--pairs", "1"],
                       cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    d = _last_json(p.stdout.decode())
    assert set(d["median_ms"]) == {"0", "1"}


def test_default_check_runs_can_see_a_shift():
    """The untimed per-configuration check takes 9 runs by default (3 could
    not tell a 30 % regression from box noise)."""
    import ast
    with open(os.path.join(ROOT, "bench.py")) as f:
        tree = ast.parse(f.read())
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "add_argument" and \
                node.args and getattr(node.args[0], "value", None) == "--check-runs":
            default = [k.value.value for k in node.keywords if k.arg == "default"][0]
            assert default >= 9
            return
    raise AssertionError("--check-runs not found")


def test_per_config_vs_prev_ratios(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    prev = tmp_path / "prev.json"
    prev.write_text(json.dumps({"ms_per_step": 7.0, "per_config": {
        "golang": {"warm_p50_ms": 2.0, "cold_over_floor_p50_ms": 8.0}}}))
    now = {"golang": {"warm_p50_ms": 3.0, "cold_over_floor_p50_ms": 6.0}, "cf": {"warm_p50_ms": 1.0},
           "large-tree": {"ratio_largest_vs_smallest": 1.0}}
    out = bench.per_config_vs_prev(now, str(prev))
    assert out["golang"] == {"warm_ratio": 1.5, "warm_prev_p50_ms": 2.0, "cold_over_floor_ratio": 0.75,
                             "cold_over_floor_prev_p50_ms": 8.0}
    assert "cf" not in out and "large-tree" not in out and out["prev_ms_per_step"] == 7.0
    assert bench.per_config_vs_prev(now, str(tmp_path / "missing.json")) is None


def test_pin_to_cores_deals_physical_cores(monkeypatch):
    """--pin-cores: the job's CPUs grouped by (package, core id), cores dealt
    round-robin to the local ranks, SMT siblings kept together."""
    sys.path.insert(0, ROOT)
    import bench
    topo = {0: ("0", "0"), 1: ("0", "1"), 2: ("0", "0"), 3: ("0", "1"), 4: ("0", "2"), 5: ("0", "2")}
    set_to = []
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(topo))
    monkeypatch.setattr(bench.os, "sched_setaffinity", lambda pid, cpus: set_to.append(sorted(cpus)))
    real_open = open

    def fake_open(path, *a, **k):
        if path.startswith("/sys/devices/system/cpu/cpu"):
            import io
            cpu = int(path.split("/cpu/cpu")[1].split("/")[0])
            return io.StringIO(topo[cpu][0] if path.endswith("physical_package_id") else topo[cpu][1])
        return real_open(path, *a, **k)
    monkeypatch.setattr("builtins.open", fake_open)
    assert bench.pin_to_cores(0, 2) == [0, 2, 4, 5]   # cores 0 and 2 with their siblings
    assert bench.pin_to_cores(1, 2) == [1, 3]
    assert bench.pin_to_cores(3, 8) == [0, 2]          # more ranks than cores: shared modulo
    assert set_to == [[0, 2, 4, 5], [1, 3], [0, 2]]


def test_host_contention_control_runs():
    """benchmarks/host_contention.py (the control experiment for the scaling
    rehearsal) reports per-process CPU of each phase and its ratio to N=1."""
    p = subprocess.run([sys.executable, os.path.join("benchmarks", "host_contention.py"), "--ranks", "1,2",
                        "--iters", "3"], cwd=ROOT, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    rows = [json.loads(l) for l in p.stdout.decode().splitlines() if l.startswith("{")]
    assert [r["n"] for r in rows] == [1, 2]
    for r in rows:
        assert set(r["per_process"]) == {"cpu", "fs", "spawn"}
        assert r["per_process"]["cpu"]["user_ms"] > 0 and r["per_process"]["fs"]["wall_ms"] > 0
    assert rows[0]["ratio_to_first"]["cpu"]["user_ms"] == 1.0
