"""The logger writes logrus v1.7.0 TextFormatter lines (``utils/log.py``):
coloured and padded on a terminal, ``key=value`` otherwise."""

import os
import pty
import re
import subprocess
import sys
import time

import logparse

from move2kube_amd.utils import log

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plain_lines_are_key_value():
    now = time.time()
    stamp = log._rfc3339(now)
    assert re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d(Z|[+-]\d\d:\d\d)", stamp)
    assert log.format_line(log.INFO, "Planning Translation", now, False) == \
        'time="%s" level=info msg="Planning Translation"\n' % stamp
    assert log.format_line(log.WARNING, "done", now, False) == 'time="%s" level=warning msg=done\n' % stamp
    assert log.format_line(log.DEBUG, "a/b-c_d.e@f^g+h", now, False) == \
        'time="%s" level=debug msg=a/b-c_d.e@f^g+h\n' % stamp
    assert log.format_line(log.CRITICAL, 'Error: "x"\n', now, False) == \
        'time="%s" level=fatal msg="Error: \\"x\\"\\n"\n' % stamp
    assert log.format_line(log.ERROR, "", now, False) == 'time="%s" level=error\n' % stamp


def test_terminal_lines_are_coloured_and_padded():
    t = log._START + 12.5
    assert log.format_line(log.INFO, "Planning Translation", t, True) == \
        "\x1b[36mINFO\x1b[0m[0012] Planning Translation" + " " * 24 + " \n"
    assert log.format_line(log.WARNING, "x" * 50 + "\n", t, True) == "\x1b[33mWARN\x1b[0m[0012] " + "x" * 50 + " \n"
    assert log.format_line(log.DEBUG, "é", t, True).startswith("\x1b[37mDEBU\x1b[0m[0012] é" + " " * 43)
    assert log.format_line(log.ERROR, "e", t, True).startswith("\x1b[31mERRO")
    assert log.format_line(log.CRITICAL, "f", t, True).startswith("\x1b[31mFATA")


def _run_cli(args, stderr):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "move2kube_amd"] + args, env=env, stdout=subprocess.DEVNULL,
                          stderr=stderr, timeout=60)


def test_cli_picks_the_format_from_its_stderr(tmp_path):
    missing = str(tmp_path / "nope")
    p = _run_cli(["plan", "-s", missing], subprocess.PIPE)
    line = p.stderr.decode().splitlines()[-1]
    assert re.fullmatch(r'time="[^"]+" level=fatal msg="Unable to access source directory : stat %s: no such file '
                        r'or directory"' % re.escape(missing), line), line
    master, slave = pty.openpty()
    try:
        p = _run_cli(["plan", "-s", missing], slave)
        os.close(slave)
        slave = None
        out = b""
        while True:
            try:
                chunk = os.read(master, 4096)
            except OSError:
                break
            if not chunk:
                break
            out += chunk
    finally:
        if slave is not None:
            os.close(slave)
        os.close(master)
    text = out.decode().replace("\r\n", "\n")
    assert p.returncode == 1
    assert re.search(r"\x1b\[31mFATA\x1b\[0m\[\d{4}\] \S", text), text


def test_write_containers_debug_lines(tmp_path, capsys):
    """writeContainers (transformer.go:59-160) at debug level."""
    import logparse
    from move2kube_amd import transformer
    from move2kube_amd.models import ir as irtypes
    log.set_verbose(True)
    try:
        c = irtypes.new_container("NewDockerfile", "img:latest", True)
        c.new_files = {"svc/Dockerfile.svc": "FROM x\n", "svc/svc-docker-build.sh": "#!/bin/sh\n"}
        assert transformer.write_containers([c], str(tmp_path), str(tmp_path), "quay.io", "ns") is True
    finally:
        log.set_verbose(False)
    msgs = [m for lv, m in logparse.messages(capsys.readouterr().err) if lv == "debug"]
    cpath = str(tmp_path / "containers")
    assert msgs[:4] == ["containerspath %s" % cpath, "Total number of containers : 1", "Container : true",
                        "New Container : img:latest"]
    assert "Writing at %s/svc/Dockerfile.svc" % cpath in msgs
    assert "buildscripts [containers/svc/svc-docker-build.sh]" in msgs
    assert "buildScriptMap map[svc-docker-build.sh:containers/svc/]" in msgs


def test_unwritable_readme_is_logged_and_the_run_goes_on(tmp_path, capsys):
    import logparse
    from move2kube_amd.transformer import K8sTransformer
    (tmp_path / "Readme.md").mkdir()
    log.set_verbose(False)
    K8sTransformer.write_readme("p", False, False, False, str(tmp_path))
    msgs = logparse.messages(capsys.readouterr().err)
    assert msgs[-1] == ("error", "Unable to write readme : open %s: is a directory" % (tmp_path / "Readme.md"))


def test_failed_object_and_container_writes_print_go_path_errors(tmp_path, capsys):
    """transformer.go:96 and :197 print the *os.PathError of ioutil.WriteFile
    (``open <path>: <errno text>``), not Python's OSError text."""
    import logparse
    from move2kube_amd import transformer
    from move2kube_amd.models import ir as irtypes
    log.set_verbose(False)
    (tmp_path / "web-service.yaml").mkdir()
    obj = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web"}, "spec": {}}
    assert transformer.write_transformed_objects(str(tmp_path), [obj]) == []
    c = irtypes.new_container("NewDockerfile", "img:latest", True)
    c.new_files = {"svc/Dockerfile.svc": "FROM x\n"}
    (tmp_path / "containers" / "svc" / "Dockerfile.svc").mkdir(parents=True)
    transformer.write_containers([c], str(tmp_path), str(tmp_path), "quay.io", "ns")
    msgs = logparse.messages(capsys.readouterr().err)
    assert ("error", 'Failed to write "Service" Error: "open %s/web-service.yaml: is a directory"' % tmp_path) in msgs
    assert ("warning", "Error writing file at %s/containers/svc/Dockerfile.svc : open %s/containers/svc/Dockerfile.svc: "
            "is a directory" % (tmp_path, tmp_path)) in msgs


def test_slice_and_map_arguments_print_as_go(capsys):
    """A []string argument prints as fmt's %v ([a b]) under %s and as %q
    (["a b" "c"]) under %r; a map as map[k:v] with sorted keys."""
    from move2kube_amd.utils import log
    log.warning("a %s b %r c %s d %r", ["x y", "z"], ["x y", "z"], {"b": 1, "a": [2]}, "q")
    err = capsys.readouterr().err
    assert logparse.logged(err, 'a [x y z] b ["x y" "z"] c map[a:[2] b:1] d "q"', "warning")
