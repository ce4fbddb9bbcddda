"""Cold-start hygiene: a CLI ``translate`` of the BASELINE configurations does
not import the stdlib modules whose system bytecode caches are stale on the
MI355X image (``profiles/r03_cold_diag/pyc_diag.json``: argparse, gettext,
locale, json, base64, copy are recompiled by every process there), and the
C-scanner JSON reader decodes like ``json.loads``."""

import json
import os
import subprocess
import sys

import pytest

from move2kube_amd.utils import fastjson

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

STALE_ON_BOX = ("argparse", "gettext", "locale", "json", "base64", "copy")

_CHILD = """
import sys
sys.path.insert(0, %r)
from move2kube_amd.cli.main import main
rc = main(%r)
print(" ".join(sorted(m for m in %r if m in sys.modules)))
sys.exit(rc)
"""


@pytest.mark.parametrize("config", ["golang", "docker-compose", "helm-openshift"])
def test_cold_translate_skips_stale_stdlib_modules(tmp_path, config):
    import refconfigs
    run = refconfigs.Run(config, str(tmp_path)).prepare()
    argv = run.cli_commands()[-1]
    env = run.env()
    p = subprocess.run([sys.executable, "-c", _CHILD % (ROOT, argv, STALE_ON_BOX)], env=env, cwd=str(tmp_path),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert p.stdout.decode().strip().splitlines()[-1:] in ([], [""]), p.stdout.decode()
    assert os.path.isdir(run.out) and refconfigs.manifest_diff_vs_ref(config, run.out) == 0


@pytest.mark.parametrize("text", ['{"a": [1, 2.5, -3e2, true, false, null, "x\\u00e9\\n"], "b": {}}', "  [ ] ",
                                  '"\\ud83d\\ude00"', "12", '{"k": NaN, "i": Infinity, "j": -Infinity}',
                                  '{"d": {"e": [[], [{}]]}}'])
def test_fastjson_matches_json(text):
    want = json.loads(text)
    got = fastjson.loads(text)
    assert json.dumps(got, sort_keys=True) == json.dumps(want, sort_keys=True)
    assert fastjson.loads(text.encode()) == want or text.find("NaN") >= 0


def test_fastjson_parse_int_hook_and_errors():
    assert fastjson.loads('{"port": 8080}', parse_int=float) == {"port": 8080.0}
    for bad in ("", "{", "[1,]", "{} x", "'a'", "[1 2]"):
        with pytest.raises(ValueError):
            fastjson.loads(bad)


def test_cli_entry_process_setup():
    """``python -m move2kube_amd`` (like the release launcher) imports the CLI
    with the cyclic collector off, then freezes those objects and turns it back
    on; shutil comes without bz2/lzma and msvcrt is recorded as absent; a
    library import of the package changes none of that."""
    probe = ("import atexit, gc, sys\n"
             "sys.argv = ['move2kube', 'version']\n"
             "atexit.register(lambda: print(gc.isenabled(), gc.get_freeze_count() > 1000, 'bz2' in sys.modules,"
             " sys.modules.get('msvcrt', 0) is None))\n"
             "import runpy\nrunpy.run_module('move2kube_amd', run_name='__main__', alter_sys=True)\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-S", "-c", probe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=60)
    assert p.stdout.decode().split() == ["v0.1.0", "True", "True", "False", "True"], p.stderr.decode()
    lib = ("import gc, sys\nimport move2kube_amd.cli.main\n"
           "print(gc.isenabled(), gc.get_freeze_count(), 'msvcrt' in sys.modules)\n")
    p = subprocess.run([sys.executable, "-S", "-c", lib], env=env, stdout=subprocess.PIPE, timeout=60)
    assert p.stdout.decode().split() == ["True", "0", "False"]
