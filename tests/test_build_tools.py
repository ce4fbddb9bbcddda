"""The in-tree build (``ops/build.py``, ``make build``, ``__graft_entry__.build``)
and the generated Blowfish table: the compiler lines each target gets, the
incremental rule, the report the build check prints, and ``blowfish_pi.h``
regenerated from pi byte for byte.  The real compiles run in
``__graft_entry__.build()`` and ``tests/test_sanitizers.py``."""

import contextlib
import importlib.util
import io
import os

import pytest

from move2kube_amd.ops import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "move2kube_amd", "ops", "csrc")


def test_blowfish_table_is_pi():
    spec = importlib.util.spec_from_file_location("gen_blowfish_pi", os.path.join(CSRC, "gen_blowfish_pi.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        gen.main()
    with open(os.path.join(CSRC, "blowfish_pi.h")) as f:
        assert buf.getvalue() == f.read()


@pytest.fixture
def fake_toolchain(tmp_path, monkeypatch):
    """Targets under tmp_path; every compiler call recorded and its output
    written instead of compiled."""
    cmds = []

    def run(cmd):
        cmds.append(cmd)
        out = cmd[cmd.index("-o") + 1]
        with open(out, "wb") as f:
            f.write(" ".join(cmd).encode())
    monkeypatch.setattr(build, "_run", run)
    for name in ("native_target", "sshkey_target", "hip_target"):
        monkeypatch.setattr(build, name, lambda name=name: str(tmp_path / (name + ".so")))
    monkeypatch.setattr(build, "find_hipcc", lambda: "/opt/rocm/bin/hipcc")
    return cmds


def test_compiler_lines(fake_toolchain, tmp_path):
    build.build_native(force=True)
    build.build_sshkey(force=True)
    build.build_hip(force=True)
    native, sshkey, hip = fake_toolchain
    assert "-std=c++17" in native and "-shared" in native and "-O3" in native
    # the release build carries its own libstdc++ (one mapped object per CLI process)
    assert "-static-libstdc++" in native and native[-3:] == ["-o", str(tmp_path / "native_target.so") + ".tmp",
                                                              "-lpthread"]
    assert sshkey[-1] == "-lcrypto" and "-O2" in sshkey
    assert hip[0] == "/opt/rocm/bin/hipcc" and "--offload-arch=gfx950" in hip and "-O3" in hip
    for name in ("native_target", "sshkey_target", "hip_target"):
        assert (tmp_path / (name + ".so")).exists() and not (tmp_path / (name + ".so.tmp")).exists()


def test_sanitizer_builds(fake_toolchain, tmp_path):
    build.build_native(force=True, out=str(tmp_path / "asan.so"), sanitize="address")
    build.build_sshkey(force=True, out=str(tmp_path / "tsan.so"), sanitize="thread")
    asan, tsan = fake_toolchain
    assert "-fsanitize=address,undefined" in asan and "-O1" in asan and "-g" in asan
    assert "-fsanitize=thread" in tsan


def test_builds_are_incremental(fake_toolchain, tmp_path):
    build.build_hip(force=True)
    assert len(fake_toolchain) == 1
    build.build_hip()                       # newer than its source: nothing to do
    assert len(fake_toolchain) == 1
    os.utime(str(tmp_path / "hip_target.so"), (1, 1))
    build.build_hip()                       # older than ed_kernel.hip: rebuilt
    assert len(fake_toolchain) == 2


def test_hip_build_needs_hipcc(fake_toolchain, monkeypatch):
    monkeypatch.setattr(build, "find_hipcc", lambda: None)
    with pytest.raises(RuntimeError, match="hipcc not found"):
        build.build_hip(force=True)


def test_find_hipcc_honours_the_environment(monkeypatch, tmp_path):
    fake = tmp_path / "hipcc"
    fake.write_text("#!/bin/sh\nexit 0\n")
    fake.chmod(0o755)
    monkeypatch.setenv("HIPCC", str(fake))
    assert build.find_hipcc() == str(fake)
    broken = tmp_path / "broken"
    broken.write_text("#!/bin/sh\nexit 1\n")
    broken.chmod(0o755)
    monkeypatch.setenv("HIPCC", str(broken))
    monkeypatch.setenv("PATH", str(tmp_path / "empty"))
    monkeypatch.setattr(build.os.path, "exists", lambda p: False if p == "/opt/rocm/bin/hipcc" else os.path.lexists(p))
    assert build.find_hipcc() is None


def test_build_report(fake_toolchain, tmp_path, monkeypatch):
    for fn in ("build_bytecode", "build_startcache"):
        path = tmp_path / (fn + ".bin")
        path.write_bytes(b"x")
        monkeypatch.setattr(build, fn, lambda force=False, path=path: str(path))
    monkeypatch.setattr(build, "have_openssl_headers", lambda: True)
    rep = build.build_report(force=True)
    assert [r["target"].split()[0] for r in rep] == ["_m2k_native", "_m2k_sshkey", "libm2k_ed_hip", "_bytecode.bin",
                                                     "_startcache.bin"]
    assert all(len(r["sha256"]) == 64 and r["bytes"] > 0 for r in rep)
    assert [r["compiled"] for r in rep[:3]] == [True, True, True]
    monkeypatch.setattr(build, "have_openssl_headers", lambda: False)
    rep = build.build_report(force=False)
    assert rep[1] == {"target": "_m2k_sshkey (g++, C++17/pybind11, libcrypto)",
                      "skipped": "OpenSSL headers not found (libssl-dev)"}
    assert rep[0]["compiled"] is False


def test_openssl_probe_without_a_compiler(monkeypatch):
    monkeypatch.setenv("CXX", "/nonexistent/c++")
    assert build.have_openssl_headers() is False


def test_graft_build_report_tolerates_a_skipped_target(monkeypatch, capsys):
    """``__graft_entry__.build()`` (the driver's build check) prints its JSON
    report when ``_m2k_sshkey`` was skipped for missing OpenSSL headers."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    monkeypatch.setattr(build, "build_report", lambda force=True: [
        {"target": "_m2k_native", "compiled": True},
        {"target": "_m2k_sshkey", "skipped": "OpenSSL headers not found (libssl-dev)"}])
    g.build()
    d = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert d["build_mode"] == "full" and d["build_exercised"] == ["_m2k_native"]
