#!/usr/bin/env python3
"""Line coverage of the product package over the CPU test suite, with no
coverage package (``pytest_cov`` is not importable here) - the counterpart of
the reference's ``go test -coverprofile`` on every release build
(``/root/reference/Makefile:105-106``, ``.github/workflows/release.yml:22-24``,
``codecov.yml``).

How it measures:

* a C trace function (``scripts/csrc/linecov.c``, compiled on first use into
  ``build/linecov/``; ``sys.settrace`` in Python when no compiler is there)
  records which lines of files under ``move2kube_amd/`` run;
* it starts in every Python process of the run through a ``sitecustomize``
  placed first on ``PYTHONPATH`` - pytest itself and the CLI processes the
  tests start (``python -m move2kube_amd``, the stress and twin scripts), in
  every thread (``threading.settrace``) - and each process writes its lines
  at exit (``atexit``, and ``os._exit``, which the CLI's fast exit and forked
  test helpers use, is wrapped to write them first);
  processes started with ``-S``/``-I`` or a scrubbed environment are not
  counted;
* the executable lines of a module are the line numbers its compiled code
  objects carry (``co_lines``), so a line counts when any bytecode of it ran.

Usage::

    python scripts/coverage.py run [--out DIR] [-- PYTEST ARGS]   # default: tests -m "not gpu"
    python scripts/coverage.py report --data DIR [--data DIR2 ...] [--out DIR] [--floor scripts/coverage_floor.json]

``run`` also reports.  The report is ``coverage.txt`` (a per-module table,
lowest first) and ``coverage.json`` (per-module statements, hits, percent and
missed line ranges).  With ``--floor`` it fails (exit 2) when the total or any
module listed there drops more than the file's tolerance below its recorded
percentage; ``--write-floor`` records the current numbers.
"""

import argparse
import json
import os
import shutil
import subprocess
import sys
import sysconfig
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "move2kube_amd")
BUILD = os.path.join(ROOT, "build", "linecov")
DEFAULT_OUT = os.path.join(ROOT, "profiles", "r06_coverage")
FLOOR = os.path.join(HERE, "coverage_floor.json")
ENV_DIR = "M2KCOV_DIR"   # not M2K_*: some tests scrub those from child environments

SITECUSTOMIZE = r'''
import os as _os
_d = _os.environ.get("M2KCOV_DIR")
if _d:
    import atexit as _atexit
    import sys as _sys
    import threading as _threading
    _prefix = _os.environ["M2KCOV_PREFIX"]
    _lines = None
    try:
        _sys.path.insert(0, _os.environ["M2KCOV_LIB"])
        import m2k_linecov as _lc
        del _sys.path[0]
        _lc.set_prefix(_prefix)

        def _thread_start(frame, event, arg):
            _lc.start()
            return None
        _threading.settrace(_thread_start)
        _lc.start()
        _data = _lc.data
    except ImportError:   # no compiler: the slow Python tracer
        _lines = {}
        _skip = set()

        def _local(frame, event, arg):
            if event == "line":
                _lines[frame.f_code.co_filename].add(frame.f_lineno)
            return _local

        def _global(frame, event, arg):
            fn = frame.f_code.co_filename
            if fn in _skip:
                return None
            if not fn.startswith(_prefix):
                _skip.add(fn)
                return None
            _lines.setdefault(fn, set())
            return _local
        _threading.settrace(_global)
        _sys.settrace(_global)

        def _data():
            return {k: sorted(v) for k, v in _lines.items()}

    def _dump(pid=_os.getpid):
        import json as _json
        path = _os.path.join(_d, "%d-%d.json" % (pid(), id(_dump)))
        with open(path + ".tmp", "w") as f:
            _json.dump(_data(), f)
        _os.replace(path + ".tmp", path)
    _atexit.register(_dump)
    # a forked child (the tests' unprivileged helpers) or the CLI's fast exit
    # leaves through os._exit, which skips atexit: write the lines first
    _real_exit = _os._exit

    def _exit_after_dump(code, _real=_real_exit):
        try:
            _dump()
        except Exception:  # noqa: BLE001
            pass
        _real(code)
    _os._exit = _exit_after_dump
'''


def build_tracer():
    """Compile the C tracer into build/linecov/ (once); None without a compiler."""
    os.makedirs(BUILD, exist_ok=True)
    so = os.path.join(BUILD, "m2k_linecov" + sysconfig.get_config_var("EXT_SUFFIX"))
    src = os.path.join(HERE, "csrc", "linecov.c")
    if os.path.exists(so) and os.path.getmtime(so) >= os.path.getmtime(src):
        return so
    cc = os.environ.get("CC", "gcc")
    cmd = [cc, "-O2", "-shared", "-fPIC", "-Wall", "-I" + sysconfig.get_paths()["include"], src, "-o", so + ".tmp"]
    try:
        subprocess.run(cmd, check=True)
    except (OSError, subprocess.CalledProcessError) as e:
        sys.stderr.write("coverage: no C tracer (%s); using sys.settrace\n" % e)
        return None
    os.replace(so + ".tmp", so)
    return so


def executable_lines(path):
    """Line numbers carrying bytecode in the module's code objects."""
    with open(path, "rb") as f:
        src = f.read()
    try:
        top = compile(src, path, "exec", dont_inherit=True)
    except SyntaxError:
        return set()
    lines, todo = set(), [top]
    while todo:
        co = todo.pop()
        for _s, _e, line in co.co_lines():
            if line:
                lines.add(line)
        todo.extend(c for c in co.co_consts if hasattr(c, "co_lines"))
    return lines


def product_modules():
    out = {}
    for dp, dns, fns in os.walk(PKG):
        dns[:] = sorted(d for d in dns if d != "__pycache__")
        for fn in sorted(fns):
            if fn.endswith(".py") and not fn.startswith("_embedded"):
                p = os.path.join(dp, fn)
                out[os.path.relpath(p, ROOT)] = p
    return out


def _data_files(data_dirs):
    for d in [data_dirs] if isinstance(data_dirs, str) else data_dirs:
        for fn in sorted(os.listdir(d)):
            if fn.endswith(".json"):
                yield os.path.join(d, fn)


def _package_path(path):
    """The file under this tree that ``path`` names: line files written on
    another machine (the GPU box runs the snapshot at another root) are
    matched by their path below the package directory."""
    marker = os.sep + "move2kube_amd" + os.sep
    i = path.rfind(marker)
    return os.path.realpath(os.path.join(ROOT, path[i + 1:]) if i >= 0 else path)


def merge(data_dirs):
    """{file: lines that ran} over every process's line file in ``data_dirs``
    (one directory or a list, e.g. the CPU suite's and the GPU tests')."""
    hits = {}
    for fn in _data_files(data_dirs):
        with open(fn) as f:
            try:
                d = json.load(f)
            except ValueError:
                continue
        for path, lines in d.items():
            hits.setdefault(_package_path(path), set()).update(lines)
    return hits


def _ranges(lines):
    out, start, prev = [], None, None
    for l in sorted(lines):
        if start is None:
            start = prev = l
        elif l == prev + 1:
            prev = l
        else:
            out.append("%d" % start if start == prev else "%d-%d" % (start, prev))
            start = prev = l
    if start is not None:
        out.append("%d" % start if start == prev else "%d-%d" % (start, prev))
    return out


def report(data_dir, out_dir):
    hits = merge(data_dir)
    nproc = sum(1 for _ in _data_files(data_dir))
    rows = {}
    tot_s = tot_h = 0
    for rel, path in product_modules().items():
        ex = executable_lines(path)
        if not ex:
            continue
        ran = hits.get(os.path.realpath(path), set()) & ex
        tot_s += len(ex)
        tot_h += len(ran)
        rows[rel] = {"statements": len(ex), "hit": len(ran), "percent": round(100.0 * len(ran) / len(ex), 1),
                     "missed": _ranges(ex - ran)}
    res = {"total": {"statements": tot_s, "hit": tot_h, "percent": round(100.0 * tot_h / max(1, tot_s), 1)},
           "processes": nproc, "modules": rows}
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "coverage.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    lines = ["%-58s %6s %6s %6s" % ("module", "stmts", "hit", "%")]
    for rel, r in sorted(rows.items(), key=lambda kv: (kv[1]["percent"], kv[0])):
        lines.append("%-58s %6d %6d %6.1f" % (rel, r["statements"], r["hit"], r["percent"]))
    lines.append("%-58s %6d %6d %6.1f" % ("TOTAL", tot_s, tot_h, res["total"]["percent"]))
    with open(os.path.join(out_dir, "coverage.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return res


def check_floor(res, floor_path):
    """Failures against the committed floor: the total and each listed module
    may not drop more than ``tolerance`` points below the recorded percent."""
    with open(floor_path) as f:
        floor = json.load(f)
    tol = floor.get("tolerance", 1.0)
    bad = []
    if res["total"]["percent"] + tol < floor["total"]:
        bad.append("TOTAL %.1f%% < floor %.1f%%" % (res["total"]["percent"], floor["total"]))
    for mod, pct in sorted(floor.get("modules", {}).items()):
        got = res["modules"].get(mod, {}).get("percent", 0.0)
        if got + tol < pct:
            bad.append("%s %.1f%% < floor %.1f%%" % (mod, got, pct))
    return bad


def write_floor(res, floor_path, tolerance=1.0):
    with open(floor_path, "w") as f:
        json.dump({"tolerance": tolerance, "total": res["total"]["percent"],
                   "modules": {m: r["percent"] for m, r in sorted(res["modules"].items())}}, f, indent=1)
        f.write("\n")


def run(pytest_args, out_dir, keep_data=None):
    so = build_tracer()
    data = keep_data or tempfile.mkdtemp(prefix="m2kcov-")
    os.makedirs(data, exist_ok=True)
    site = tempfile.mkdtemp(prefix="m2kcov-site-")
    try:
        with open(os.path.join(site, "sitecustomize.py"), "w") as f:
            f.write(SITECUSTOMIZE)
        env = dict(os.environ)
        env[ENV_DIR] = data
        env["M2KCOV_PREFIX"] = PKG + os.sep
        env["M2KCOV_LIB"] = os.path.dirname(so) if so else site
        env["PYTHONPATH"] = os.pathsep.join([site, ROOT] + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
        rc = subprocess.run([sys.executable, "-m", "pytest"] + pytest_args, cwd=ROOT, env=env).returncode
        res = report(data, out_dir)
        res["pytest_exit"] = rc
        return res
    finally:
        shutil.rmtree(site, ignore_errors=True)
        if keep_data is None:
            shutil.rmtree(data, ignore_errors=True)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--out", default=DEFAULT_OUT)
    r.add_argument("--data", default=None, help="keep the per-process line files here")
    r.add_argument("--floor", default=None)
    r.add_argument("--write-floor", default=None)
    r.add_argument("pytest_args", nargs="*")
    p = sub.add_parser("report")
    p.add_argument("--data", required=True, action="append",
                   help="a directory of per-process line files (repeat to merge, e.g. CPU and GPU runs)")
    p.add_argument("--out", default=DEFAULT_OUT)
    p.add_argument("--floor", default=None)
    p.add_argument("--write-floor", default=None)
    args = ap.parse_args(argv)
    if args.cmd == "run":
        res = run(args.pytest_args or ["tests", "-q", "-m", "not gpu", "-p", "no:cacheprovider"], args.out,
                  args.data)
    else:
        res = report(args.data, args.out)
    print(json.dumps({"total": res["total"], "processes": res["processes"], "out": args.out,
                      "pytest_exit": res.get("pytest_exit")}))
    if args.write_floor:
        write_floor(res, args.write_floor)
    if args.floor:
        bad = check_floor(res, args.floor)
        for b in bad:
            print("below floor:", b, file=sys.stderr)
        if bad:
            return 2
    return 1 if res.get("pytest_exit") else 0


if __name__ == "__main__":
    sys.exit(main())
