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

STALE_ON_BOX = ("argparse", "gettext", "locale", "json", "base64", "copy",
                "queue", "heapq")  # queue + heapq: 1.9 ms per process there (profiles/r05_perf2/cold_importtime.jsonl)
# package modules only error paths need (Go type tables for decode errors, fmt's printer for printf)
ERROR_PATH_ONLY = ("move2kube_amd.models.gotypes", "move2kube_amd.utils.gofmt_printer")

_CHILD = """
import sys
sys.path.insert(0, %r)
from move2kube_amd.cli.main import main
rc = main(%r)
print(" ".join(sorted(m for m in %r if m in sys.modules)))
sys.exit(rc)
"""


@pytest.mark.parametrize("config", ["golang", "docker-compose", "java-cnb", "cf", "helm-openshift"])
def test_cold_translate_skips_stale_stdlib_modules(tmp_path, config):
    import refconfigs
    run = refconfigs.Run(config, str(tmp_path)).prepare()
    argv = run.cli_commands()[-1]
    env = run.env()
    if len(run.cli_commands()) > 1:   # cf: collect first, its output copied into the source tree
        env["PYTHONPATH"] = ROOT
        import shutil
        for argv0 in run.cli_commands()[:-1]:
            subprocess.run([sys.executable, "-m", "move2kube_amd"] + argv0, env=env, cwd=str(tmp_path),
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True, timeout=120)
        shutil.copytree(os.path.join(str(tmp_path), "collect", "m2k_collect"), os.path.join(run.src, "m2k_collect"))
    p = subprocess.run([sys.executable, "-c", _CHILD % (ROOT, argv, STALE_ON_BOX + ERROR_PATH_ONLY)], env=env, cwd=str(tmp_path),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert p.stdout.decode().strip().splitlines()[-1:] in ([], [""]), p.stdout.decode()
    assert os.path.isdir(run.out) and refconfigs.manifest_diff_vs_ref(config, run.out) == 0


@pytest.mark.parametrize("text", ['{"a": [1, 2.5, -3e2, true, false, null, "x\\u00e9\\n"], "b": {}}', "  [ ] ",
                                  '"\\ud83d\\ude00"', "12", '{"d": {"e": [[], [{}]]}}'])
def test_fastjson_matches_json(text):
    want = json.loads(text)
    got = fastjson.loads(text)
    assert json.dumps(got, sort_keys=True) == json.dumps(want, sort_keys=True)
    assert fastjson.loads(text.encode()) == want


def test_fastjson_parse_int_hook():
    assert fastjson.loads('{"port": 8080}', parse_int=float) == {"port": 8080.0}


@pytest.mark.parametrize("data,msg", [
    (b"", "unexpected end of JSON input"), (b"{", "unexpected end of JSON input"),
    (b'{"a" 1}', "invalid character '1' after object key"),
    (b'{"a":1 "b":2}', "invalid character '\"' after object key:value pair"),
    (b"[1 2]", "invalid character '2' after array element"),
    (b"[1,]", "invalid character ']' looking for beginning of value"),
    (b"{,}", "invalid character ',' looking for beginning of object key string"),
    (b"01", "invalid character '1' after top-level value"), (b"{} x", "invalid character 'x' after top-level value"),
    (b"-a", "invalid character 'a' in numeric literal"),
    (b"1.x", "invalid character 'x' after decimal point in numeric literal"),
    (b"1ex", "invalid character 'x' in exponent of numeric literal"),
    (b"trux", "invalid character 'x' in literal true (expecting 'e')"),
    (b'"a\\x"', "invalid character 'x' in string escape code"),
    (b'"\\u12g4"', "invalid character 'g' in \\u hexadecimal character escape"),
    (b'"a\x01"', "invalid character '\\x01' in string literal"),
    (b"NaN", "invalid character 'N' looking for beginning of value"),
    (b'{"i": -Infinity}', "invalid character 'I' in numeric literal"),
    (b"\xef\xbb\xbf{}", "invalid character '\u00ef' looking for beginning of value"),
    (b"'a'", "invalid character '\\'' looking for beginning of value"),
])
def test_fastjson_errors_read_like_encoding_json(data, msg):
    """Go's scanner decides what is valid and words the error; the reference
    logs that text for detector output, docker inspect and CLI JSON."""
    with pytest.raises(ValueError) as ei:
        fastjson.loads(data)
    assert str(ei.value) == msg
    if data.isascii():                     # a str is its UTF-8 bytes to Go
        with pytest.raises(ValueError) as ei:
            fastjson.loads(data.decode())
        assert str(ei.value) == msg


def test_fastjson_invalid_utf8_in_strings_becomes_replacement_chars():
    assert fastjson.loads(b'{"k": "v\xff\xe2\x82"}') == {"k": "v\ufffd\ufffd\ufffd"}


def test_cli_entry_process_setup():
    """``python -m move2kube_amd`` (like the release launcher) imports the CLI
    with the cyclic collector off, freezes those objects and leaves it off for
    the command (``api.gc_paused``); shutil comes without bz2/lzma and msvcrt is recorded as absent; a
    library import of the package changes none of that."""
    probe = ("import atexit, gc, sys\n"
             "sys.argv = ['move2kube', 'version']\n"
             "atexit.register(lambda: print(gc.isenabled(), gc.get_freeze_count() > 1000, 'bz2' in sys.modules,"
             " sys.modules.get('msvcrt', 0) is None))\n"
             "import runpy\nrunpy.run_module('move2kube_amd', run_name='__main__', alter_sys=True)\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-S", "-c", probe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=60)
    assert p.stdout.decode().split() == ["v0.1.0", "False", "True", "False", "True"], p.stderr.decode()
    lib = ("import gc, sys\nimport move2kube_amd.cli.main\n"
           "print(gc.isenabled(), gc.get_freeze_count(), 'msvcrt' in sys.modules)\n")
    p = subprocess.run([sys.executable, "-S", "-c", lib], env=env, stdout=subprocess.PIPE, timeout=60)
    assert p.stdout.decode().split() == ["True", "0", "False"]


@pytest.mark.parametrize("rc,code", [(None, 0), (0, 0), (3, 3), ("failed", 1)])
def test_cli_exit_behaves_like_sys_exit(tmp_path, rc, code):
    """``_cli_exit`` skips the interpreter teardown but keeps what ``sys.exit``
    guarantees: non-daemon threads finish, atexit handlers run after them,
    buffered stdout reaches the pipe, the status is the same."""
    log = tmp_path / "order.txt"
    probe = ("import atexit, sys, threading, time\n"
             "import move2kube_amd\n"
             "def note(s):\n    open(%r, 'a').write(s + '\\n')\n"
             "atexit.register(note, 'atexit')\n"
             "t = threading.Thread(target=lambda: (time.sleep(0.2), note('thread')))\nt.start()\n"
             "sys.stdout.write('buffered output')\n"
             "move2kube_amd._cli_exit(%r)\n" % (str(log), rc))
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-c", probe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=60)
    assert p.returncode == code
    assert p.stdout == b"buffered output"
    assert log.read_text().split() == ["thread", "atexit"]
    if isinstance(rc, str):
        assert p.stderr.decode().strip() == rc


def test_cli_runs_leave_no_unclosed_files(tmp_path):
    """The fast exit relies on every file being closed by the code that opened
    it: a translate under ``-X dev`` that ends through the full interpreter
    teardown (where a leaked file would be finalized and warn) reports no
    ResourceWarning."""
    import refconfigs
    run = refconfigs.Run("helm-openshift", str(tmp_path)).prepare()
    env = dict(run.env(), PYTHONPATH=ROOT, PYTHONWARNINGS="always::ResourceWarning")
    child = "import sys\nfrom move2kube_amd.cli.main import main\nsys.exit(main(%r))\n" % run.cli_commands()[-1]
    p = subprocess.run([sys.executable, "-X", "dev", "-c", child], env=env,
                       cwd=str(tmp_path), stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert "ResourceWarning" not in p.stderr.decode()


@pytest.mark.skipif(not os.path.exists("/dev/full"), reason="needs /dev/full")
def test_cli_exit_reports_a_failed_stdout_flush():
    """Output that cannot be written (ENOSPC on /dev/full) is an error, as with
    ``sys.exit``: CPython's message on stderr and status 120."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    with open("/dev/full", "w") as full:
        p = subprocess.run([sys.executable, "-m", "move2kube_amd", "version"], env=env, stdout=full,
                           stderr=subprocess.PIPE, timeout=60)
    assert p.returncode == 120
    assert "Exception ignored in: <_io.TextIOWrapper name='<stdout>'" in p.stderr.decode()
    assert "OSError: [Errno 28]" in p.stderr.decode()
