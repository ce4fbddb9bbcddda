#!/usr/bin/env python3
"""Race and stress harness for the Python-level concurrency of the CLI - the
stand-in for the reference's ``go test -race`` (``/root/reference/Makefile:91-92``),
which instruments every goroutine: the CNB providers
(``internal/containerizer/cnb/packprovider.go:59-107``,
``dockerapiprovider.go:241-283``), the QA REST engine
(``internal/qaengine/httprestengine.go:43-83``) and the collectors.

Each run is one configuration of ``benchmarks/refconfigs.py`` as the user's
CLI commands (``collect`` then ``translate`` for cf; ``rest:<config>`` answers
every question over the QA REST engine from one client while three others
poll the current problem, instead of ``--qaskip``; ``collect:k8s`` collects
cluster metadata through the stand-in ``kubectl proxy`` and inspects 13
images concurrently, and must reproduce a plain sequential run's tree), each
command a fresh
``python scripts/m2k_switchy.py ...`` process whose thread switch interval is
1 us, so every thread is preempted between almost every pair of bytecodes.
Runs vary, by seed:

* ``M2K_WORKERS`` (detector / collector pools) over 1, 2, 16;
* ``M2K_CNB_PARALLEL`` (CNB detector probes in flight) over 1, 4;
* ``M2K_NATIVE_DETECT`` over 1, 0 (built-in detectors or the shell scripts
  through the native process pool);
* ``M2K_DISABLE_NATIVE`` over unset, 1 (the native extension, or every
  pure-Python twin: the Python walker, sniffer, YAML codec, marshaller and
  the ``subprocess`` runner, where the round-4 race was);
* ``M2K_STUB_DELAY_SEED``: the ``podman``, ``cf`` and ``operator-sdk``
  stand-ins (``tests/fixtures/configs/bin``) sleep 0-24 ms, a function of the
  seed and their arguments, so the order in which concurrent tool calls finish
  changes from seed to seed;
* ``M2K_THREAD_JITTER_SEED``: every thread the CLI starts sleeps 0-2 ms
  before it runs (``scripts/m2k_switchy.py``), so which of two racing threads
  reaches a shared initialisation first changes too.

Every output tree is compared byte for byte with the configuration's expected
tree; a failing command or a differing file is a finding.  Exit status 1 when
anything differs.

Usage: ``python scripts/stress.py [--seeds 20] [--configs a,b] [--jobs 4]
[--json out.jsonl]``; ``make stress`` runs the small CI form.
"""

import argparse
import concurrent.futures
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402

DEFAULT_CONFIGS = (sorted(refconfigs.CONFIGS) + ["coverage/git-repos", "coverage/carried-over/Openshift"]
                   + ["rest:" + c for c in sorted(refconfigs.CONFIGS)] + ["collect:k8s"])
WORKERS = ("1", "2", "16")
CNB_PARALLEL = ("1", "4")
NATIVE_DETECT = ("1", "0")
DISABLE_NATIVE = ("", "1")
ENTRY = os.path.join(HERE, "m2k_switchy.py")


def knobs(seed):
    """The environment one seed runs under: every combination of the four
    switches is reached by 24 consecutive seeds."""
    return {"M2K_WORKERS": WORKERS[seed % 3], "M2K_CNB_PARALLEL": CNB_PARALLEL[(seed // 3) % 2],
            "M2K_NATIVE_DETECT": NATIVE_DETECT[(seed // 6) % 2], "M2K_DISABLE_NATIVE": DISABLE_NATIVE[(seed // 12) % 2],
            "M2K_STUB_DELAY_SEED": str(seed), "M2K_THREAD_JITTER_SEED": str(seed)}


def _name(config):
    return config[len("coverage/"):] if config.startswith("coverage/") else config


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _http(port, method, path, body=None, timeout=30.0):
    import http.client
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request(method, path, body=body, headers={"Content-Type": "application/json"} if body else {})
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def _rest_clients(proc, port, seed, pollers=3):
    """Answer every question of the translate process ``proc`` over the QA
    REST engine (``httprestengine.go:43-83``) the way ``--qaskip`` would (the
    default; an empty password), from one answering client, while ``pollers``
    other clients keep asking for the current problem - all with seeded
    pauses.  Returns (answers posted, error statuses seen)."""
    import random
    import threading
    rng = random.Random("rest/%d" % seed)
    pauses = [rng.uniform(0.0, 0.003) for _ in range(256)]
    stats = {"answers": 0, "errors": []}

    def answerer():
        i = 0
        while proc.poll() is None:
            try:
                st, body = _http(port, "GET", "/problems/current")
            except OSError:
                time.sleep(0.002)
                continue
            if st != 200:
                stats["errors"].append(("GET", st))
                continue
            prob = json.loads(body)
            sol = prob.get("solution") or {}
            ans = sol.get("default") or ([""] if sol.get("type") == "Password" else [])
            time.sleep(pauses[i % len(pauses)])
            i += 1
            try:
                st, body = _http(port, "POST", "/problems/current/solution", json.dumps(ans).encode())
            except OSError:
                continue
            stats["answers"] += 1
            if st != 200:
                stats["errors"].append(("POST", st, body.decode(errors="replace")[:200]))

    def poller(k):
        j = k
        while proc.poll() is None:
            try:
                _http(port, "GET", "/problems/current", timeout=5.0)
            except OSError:
                pass
            time.sleep(pauses[j % len(pauses)])
            j += 7
    threads = [threading.Thread(target=answerer, daemon=True)]
    threads += [threading.Thread(target=poller, args=(k,), daemon=True) for k in range(pollers)]
    for t in threads:
        t.start()
    return threads, stats


def _run_rest(run, env, seed):
    """The configuration's commands with ``translate`` answered over HTTP
    (``--qadisablecli --qaport``) instead of ``--qaskip``."""
    import subprocess
    full = run.env()
    full["PYTHONPATH"] = ROOT + os.pathsep + full.get("PYTHONPATH", "")
    full.update(env)
    stats = None
    for argv in run.cli_commands():
        if argv[0] == "translate":
            port = _free_port()
            argv = [a for a in argv if a != "--qaskip"] + ["--qadisablecli", "--qaport", str(port)]
        proc = subprocess.Popen([sys.executable, ENTRY] + argv, env=full, cwd=run.work,
                                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        threads = []
        if argv[0] == "translate":
            threads, stats = _rest_clients(proc, port, seed)
        try:
            _out, err = proc.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            proc.kill()
            _out, err = proc.communicate()
            raise RuntimeError("%s timed out (QA REST run hung)" % argv[0])
        for t in threads:
            t.join(timeout=10)
        if proc.returncode != 0:
            raise RuntimeError("%s failed: %s" % (argv[0], err.decode(errors="replace")[-2000:]))
        if argv[0] == "collect":
            dst = os.path.join(run.src, "m2k_collect")
            shutil.rmtree(dst, ignore_errors=True)
            shutil.copytree(os.path.join(run.work, "collect", "m2k_collect"), dst)
    return run.out, stats


STUBBIN = os.path.join(ROOT, "tests", "fixtures", "stubbin")
_COLLECT_IMAGES = ["stress/app%d:1.%d" % (i, i) for i in range(12)] + ["redis:6"]
_DOCKER_STUB = """#!/bin/sh
# scripts/stress.py: docker for `collect -a k8s` (inspect of the compose images)
if [ -n "$M2K_STUB_DELAY_SEED" ]; then
  _d=$(printf '%s %s' "$M2K_STUB_DELAY_SEED" "$*" | cksum); _d=${_d%% *}
  sleep "$(printf '0.%03d' $((_d % 25)))"
fi
case "$1 $2" in
  "inspect stress/"*) printf '[{"RepoTags":["%s"],"ContainerConfig":{"ExposedPorts":{"80/tcp":{},"8443/tcp":{}},'\\
'"User":"1001","WorkingDir":"/srv/%s"}}]' "$2" "$2" ;;
  "inspect redis:6") echo "Error: No such object: redis:6"; exit 1 ;;
  *) echo "unexpected: $*" >&2; exit 1 ;;
esac
"""


def _collect_k8s(work, env, launcher):
    """``collect -a k8s`` of a compose tree: cluster discovery through the
    stand-in ``kubectl proxy`` (``tests/fixtures/fake_apiserver.py``) and the
    concurrent ``docker inspect`` of 13 images (one missing).  Returns the
    collect output directory."""
    import subprocess
    src = os.path.join(work, "src")
    os.makedirs(src)
    with open(os.path.join(src, "docker-compose.yaml"), "w") as f:
        f.write("version: '3'\nservices:\n" + "".join("  s%d:\n    image: %s\n" % (i, img)
                                                        for i, img in enumerate(_COLLECT_IMAGES)))
    bindir = os.path.join(work, "bin")
    os.makedirs(bindir)
    with open(os.path.join(bindir, "docker"), "w") as f:
        f.write(_DOCKER_STUB)
    os.chmod(os.path.join(bindir, "docker"), 0o755)
    full = dict(os.environ)
    full.update(env)
    full["PATH"] = os.pathsep.join([bindir, STUBBIN, "/usr/bin", "/bin"])
    # exec credentials: discovery goes through the stand-in `kubectl proxy`
    kc = os.path.join(work, "kubeconfig")
    with open(kc, "w") as f:
        f.write('{"current-context": "c", "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}], '
                '"clusters": [{"name": "k", "cluster": {"server": "https://stub.invalid"}}], '
                '"users": [{"name": "u", "user": {"exec": {"command": "stub-token", "apiVersion": "x"}}}]}')
    full["KUBECONFIG"] = kc
    full.pop("KUBERNETES_SERVICE_HOST", None)
    full["HOME"] = os.path.join(work, "home")
    full["PYTHONPATH"] = ROOT + os.pathsep + full.get("PYTHONPATH", "")
    out = os.path.join(work, "collect")
    p = subprocess.run(launcher + ["collect", "-a", "k8s", "-s", src, "-o", out], env=full, cwd=work,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=300)
    if p.returncode != 0:
        raise RuntimeError("collect failed: %s" % p.stderr.decode(errors="replace")[-2000:])
    return os.path.join(out, "m2k_collect")


_COLLECT_EXPECTED = {}


def _collect_expected():
    """The tree of one plain, sequential ``collect -a k8s`` (no switch
    interval, one worker): what every stressed run must reproduce."""
    if "tree" not in _COLLECT_EXPECTED:
        work = tempfile.mkdtemp(prefix="m2k-stress-ref-")
        out = _collect_k8s(work, {"M2K_WORKERS": "1"}, [sys.executable, "-m", "move2kube_amd"])
        tree = {}
        for rel, path in refconfigs.tree_files(out).items():
            with open(path, "rb") as f:
                tree[rel] = f.read()
        shutil.rmtree(work, ignore_errors=True)
        _COLLECT_EXPECTED["tree"] = tree
    return _COLLECT_EXPECTED["tree"]


def _diff_collect(out):
    want = _collect_expected()
    have = refconfigs.tree_files(out)
    bad = sorted(set(want) ^ set(have))
    for rel in sorted(set(want) & set(have)):
        with open(have[rel], "rb") as f:
            if f.read() != want[rel]:
                bad.append(rel)
    return sorted(bad)


UI_NOTE_HEAD = "\nIMPORTANT!!: If you used the UI for translation"
UI_NOTE_TAIL = "in order to get it right.\n"


def _readme_is_ui_form(out, name):
    """With the CLI engine off (``--qadisablecli``, the UI's mode) the
    reference's ``Readme.md`` carries the UI users' copysources warning of its
    K8sReadme template (``internal/transformer/templates/constants.go``);
    otherwise it is the expected file."""
    with open(os.path.join(out, "Readme.md")) as f:
        text = f.read()
    with open(os.path.join(refconfigs.golden_dir(name), "Readme.md")) as f:
        want = f.read()
    i = text.find(UI_NOTE_HEAD)
    j = text.find(UI_NOTE_TAIL, i)
    return i >= 0 and j >= 0 and text[:i] + text[j + len(UI_NOTE_TAIL):] == want


def run_one(config, seed, switch="1e-6", keep_on_failure=None):
    """One seeded run; returns a result row (``diff`` lists differing files).
    A ``rest:<config>`` name answers the questions over the QA REST engine."""
    rest = config.startswith("rest:")
    name = _name(config[len("rest:"):] if rest else config)
    work = tempfile.mkdtemp(prefix="m2k-stress-")
    row = {"config": config, "seed": seed, "knobs": knobs(seed)}
    t0 = time.perf_counter()
    if config == "collect:k8s":
        try:
            out = _collect_k8s(work, dict(row["knobs"], M2K_SWITCH_INTERVAL=switch), [sys.executable, ENTRY])
            row["diff"] = _diff_collect(out)
        except RuntimeError as e:
            row["error"] = str(e)[-1500:]
            row["diff"] = None
        finally:
            shutil.rmtree(work, ignore_errors=True)
        row["wall_s"] = round(time.perf_counter() - t0, 3)
        row["ok"] = not row.get("error") and row["diff"] == []
        return row
    try:
        run = refconfigs.Run(name, work).prepare()
        env = dict(row["knobs"], M2K_SWITCH_INTERVAL=switch)
        try:
            if rest:
                out, stats = _run_rest(run, env, seed)
                row["rest"] = {"answers": stats["answers"], "errors": stats["errors"][:5]}
                if stats["errors"]:
                    raise RuntimeError("QA REST errors: %r" % stats["errors"][:5])
            else:
                out = run.run_cli(extra_env=env, launcher=[sys.executable, ENTRY])
        except RuntimeError as e:
            row["error"] = str(e)[-1500:]
            row["diff"] = None
        else:
            row["diff"] = refconfigs.diff_files(out, refconfigs.golden_dir(name), work=run.work)
            if rest and "Readme.md" in row["diff"] and _readme_is_ui_form(out, name):
                row["diff"].remove("Readme.md")
        if keep_on_failure and (row.get("error") or row["diff"]):
            dst = os.path.join(keep_on_failure, "%s-%d" % (name.replace("/", "_"), seed))
            shutil.rmtree(dst, ignore_errors=True)
            shutil.copytree(work, dst, symlinks=True)
            row["kept"] = dst
    finally:
        shutil.rmtree(work, ignore_errors=True)
    row["wall_s"] = round(time.perf_counter() - t0, 3)
    row["ok"] = not row.get("error") and row["diff"] == []
    return row


def stress(configs, seeds, jobs, switch="1e-6", first_seed=0, keep_on_failure=None, sink=None):
    """Run ``seeds`` seeded runs of every configuration on ``jobs`` concurrent
    workers (each run is its own processes); returns the result rows."""
    tasks = [(c, s) for s in range(first_seed, first_seed + seeds) for c in configs]
    rows = []
    with concurrent.futures.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(run_one, c, s, switch, keep_on_failure) for c, s in tasks]
        for f in concurrent.futures.as_completed(futs):
            r = f.result()
            rows.append(r)
            if sink is not None:
                sink(r)
    return sorted(rows, key=lambda r: (r["config"], r["seed"]))


def summary(rows):
    out = {}
    for r in rows:
        s = out.setdefault(r["config"], {"runs": 0, "failures": 0, "wall_s": 0.0, "failed_seeds": []})
        s["runs"] += 1
        s["wall_s"] = round(s["wall_s"] + r["wall_s"], 3)
        if not r["ok"]:
            s["failures"] += 1
            s["failed_seeds"].append(r["seed"])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--seeds", type=int, default=20, help="seeded runs per configuration")
    ap.add_argument("--first-seed", type=int, default=0)
    ap.add_argument("--configs", default=",".join(DEFAULT_CONFIGS))
    ap.add_argument("--jobs", type=int, default=max(1, min(8, (os.cpu_count() or 2) // 2)))
    ap.add_argument("--switch", default="1e-6", help="sys.setswitchinterval of every CLI process")
    ap.add_argument("--json", default=None, help="append one JSON row per run here")
    ap.add_argument("--keep", default=None, help="copy the work tree of a failing run under this directory")
    args = ap.parse_args(argv)
    configs = [c for c in args.configs.split(",") if c]
    for c in configs:
        if c != "collect:k8s":
            refconfigs._lookup(_name(c[len("rest:"):] if c.startswith("rest:") else c))   # unknown names fail here
    sink_f = open(args.json, "a") if args.json else None

    def sink(r):
        if sink_f:
            sink_f.write(json.dumps(r) + "\n")
            sink_f.flush()
        if not r["ok"]:
            print("FAIL %s seed %d %s: %s" % (r["config"], r["seed"], r["knobs"], r.get("error") or r["diff"]),
                  file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    try:
        rows = stress(configs, args.seeds, args.jobs, args.switch, args.first_seed, args.keep, sink)
    finally:
        if sink_f:
            sink_f.close()
    res = {"seeds": args.seeds, "first_seed": args.first_seed, "switch_interval_s": float(args.switch),
           "jobs": args.jobs, "wall_s": round(time.perf_counter() - t0, 1),
           "failures": sum(not r["ok"] for r in rows), "runs": len(rows), "per_config": summary(rows)}
    print(json.dumps(res), flush=True)
    return 1 if res["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
