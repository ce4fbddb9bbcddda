"""Cold-start A/B of garbage-collector settings in the CLI process: the release
launcher's entry with the collector on throughout ("plain"), off for the whole
process, off until the CLI module is imported and then frozen and re-enabled
(what the entry does), and with a raised generation-0 threshold.  Interleaved runs, p25/p50 per variant, one
JSON line.

    python scripts/gc_ab.py golang [--runs 25]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import refconfigs  # noqa: E402

MAIN_IMPORT = "from move2kube_amd.cli.main import main  # noqa: E402\n"
ENTRY_GC = "import gc  # noqa: E402\n\ngc.freeze()\ngc.enable()\n"
VARIANTS = {
    "plain": ("", "gc.enable()\n"),
    "gc_off": ("", ""),
    "gc_off_until_main": ("", "gc.freeze()\ngc.enable()\n"),
    "gc_threshold_20k": ("gc.set_threshold(20000, 10, 10)\n", "gc.enable()\n"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--runs", type=int, default=25)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="m2k-gcab-")
    run = refconfigs.Run(a.config, work).prepare()
    env = run.env()
    entry = open(refconfigs.release_launcher(work)[2]).read()
    assert MAIN_IMPORT in entry and ENTRY_GC in entry
    entry = "import gc\n" + entry.replace(ENTRY_GC, "")
    cmds = {}
    for k, (pre, post) in VARIANTS.items():
        path = os.path.join(work, "entry_%s.py" % k)
        with open(path, "w") as f:
            f.write(entry.replace("import gc\n", "import gc\n" + pre, 1).replace(MAIN_IMPORT, MAIN_IMPORT + post))
        cmds[k] = [sys.executable, "-S", path] + run.cli_commands()[-1]
    times = {k: [] for k in cmds}
    for i in range(a.runs + 2):
        for k, cmd in cmds.items():
            t0 = time.perf_counter()
            p = subprocess.run(cmd, env=env, cwd=work, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            dt = (time.perf_counter() - t0) * 1e3
            if p.returncode != 0:
                raise SystemExit("%s failed: %s" % (k, p.stderr.decode(errors="replace")[-1000:]))
            if i >= 2:
                times[k].append(dt)
    out = {"config": a.config, "runs": a.runs}
    for k, v in times.items():
        v.sort()
        out[k] = {"p25": round(v[len(v) // 4], 2), "p50": round(v[len(v) // 2], 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
