#!/usr/bin/env python3
"""Planning on a large synthetic source tree.

Generates ``--apps`` application directories (nodejs / python / golang / java /
ruby / php / plain Dockerfile / compose) each with ``--depth`` levels of nested
source directories and ``--files`` files per level, then times ``move2kube plan``
in-process: the native path (single indexed walk, in-process built-in
detectors, native Dockerfile sniffing) and, on a subset, the reference's
execution model (every detector forked as ``/bin/sh``, serially).  Prints one
JSON line.
"""

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("M2K_NO_NETWORK", "1")
os.environ.setdefault("M2K_DISABLE_CNB", "1")

KINDS = {
    "node": {"package.json": '{"name": "x"}', "index.js": "console.log(1)\n"},
    "py": {"requirements.txt": "flask\n", "app.py": "if __name__ == '__main__':\n    pass\n"},
    "go": {"go.mod": "module x\n", "main.go": "package main\n"},
    "java": {"pom.xml": "<project/>\n"},
    "ruby": {"Gemfile": "source 'x'\n"},
    "php": {"index.php": "<?php\n"},
    "df": {"Dockerfile": "FROM alpine:3\nRUN true\n"},
    "compose": {"docker-compose.yml": "version: '3'\nservices:\n  s:\n    image: redis:6\n"},
}


def make_tree(root, apps, depth, files):
    kinds = sorted(KINDS)
    n_files = n_dirs = 0
    os.makedirs(root, exist_ok=True)
    # like samples/: the root itself is not a service
    with open(os.path.join(root, ".m2kignore"), "w") as f:
        f.write(".\n")
    for i in range(apps):
        kind = kinds[i % len(kinds)]
        # go/php detectors match recursively, so those apps sit at the top level
        # (under a team dir the whole team would become one service)
        parent = root if kind in ("go", "php") else os.path.join(root, "team%02d" % (i % 17))
        app = os.path.join(parent, "%s-app-%04d" % (kind, i))
        os.makedirs(app, exist_ok=True)
        n_dirs += 1
        for name, content in KINDS[kind].items():
            with open(os.path.join(app, name), "w") as f:
                f.write(content)
            n_files += 1
        d = app
        for lvl in range(depth):
            d = os.path.join(d, "src%d" % lvl)
            os.makedirs(d, exist_ok=True)
            n_dirs += 1
            for j in range(files):
                with open(os.path.join(d, "f%03d.txt" % j), "w") as f:
                    f.write("data %d\n" % j)
                n_files += 1
    return n_dirs, n_files


def time_plan(src):
    from move2kube_amd import api
    with api.Session() as s:
        t0 = time.perf_counter()
        p = s.plan(src, "bigtree")
        return time.perf_counter() - t0, len(p.services)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--apps", type=int, default=400)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--files", type=int, default=20)
    ap.add_argument("--ref-apps", type=int, default=40, help="subset size for the serial-fork reference model")
    a = ap.parse_args()
    from move2kube_amd.utils import log
    from move2kube_amd.utils.constants import settings
    log.set_quiet()
    work = tempfile.mkdtemp(prefix="m2k-bigtree-")
    try:
        big = os.path.join(work, "big")
        n_dirs, n_files = make_tree(big, a.apps, a.depth, a.files)
        native_s, n_services = time_plan(big)
        res = {"bench": "plan_large_tree", "apps": a.apps, "dirs": n_dirs, "files": n_files,
               "services": n_services, "native_s": round(native_s, 3)}
        if a.ref_apps:
            small = os.path.join(work, "small")
            make_tree(small, a.ref_apps, a.depth, a.files)
            nat_small, _ = time_plan(small)
            os.environ["M2K_NATIVE_DETECT"] = "0"
            saved = settings.workers
            settings.workers = 1
            try:
                ref_small, _ = time_plan(small)
            finally:
                settings.workers = saved
                os.environ.pop("M2K_NATIVE_DETECT", None)
            res.update({"ref_apps": a.ref_apps, "native_small_s": round(nat_small, 3),
                        "reference_model_small_s": round(ref_small, 3),
                        "speedup_vs_reference_model": round(ref_small / nat_small, 2) if nat_small else None})
        print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
