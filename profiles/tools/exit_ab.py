"""Cold-start A/B of how the CLI process ends: the release launcher's entry as
is (``_cli_exit``: atexit handlers, stream flush, ``os._exit``) against
``sys.exit`` (the interpreter's full teardown).  Interleaved runs, p25/p50 per
variant, one JSON line.

    python scripts/exit_ab.py golang [--runs 25]
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

FAST = "_cli_exit(main())"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--runs", type=int, default=25)
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="m2k-exitab-")
    run = refconfigs.Run(a.config, work).prepare()
    env = run.env()
    entry = open(refconfigs.release_launcher(work)[2]).read()
    assert FAST in entry
    cmds = {}
    for k, text in (("cli_exit", entry), ("sys_exit", entry.replace(FAST, "sys.exit(main())"))):
        path = os.path.join(work, "entry_%s.py" % k)
        with open(path, "w") as f:
            f.write(text)
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
