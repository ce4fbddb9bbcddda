"""The C++ host runtime (``_m2k_native``) against pure-Python references."""

import os
import random

import pytest

from move2kube_amd.ops import editdistance, native
from move2kube_amd.source import dockerfile_parser
from move2kube_amd.utils import common, fsindex

needs_native = pytest.mark.skipif(not native.available(), reason="native extension not built")


@needs_native
def test_walk_matches_python(tmp_path):
    (tmp_path / "a" / "b").mkdir(parents=True)
    (tmp_path / "a" / "f.txt").write_text("x")
    (tmp_path / "a" / "b" / "g.yaml").write_text("y")
    (tmp_path / "z.yml").write_text("z")
    os.symlink(str(tmp_path / "z.yml"), str(tmp_path / "link.yml"))
    paths, kinds, errors = native.module().walk(str(tmp_path))
    ppaths, pkinds, perrors = fsindex._walk_py(str(tmp_path))
    assert list(paths) == list(ppaths)
    assert list(kinds) == list(pkinds)
    assert list(errors) == list(perrors)


@needs_native
def test_hashes_match_python():
    rng = random.Random(0)
    for n in (0, 1, 7, 64, 1000):
        data = bytes(rng.randrange(256) for _ in range(n))
        assert native.module().crc64_ecma(data) == common.crc64_ecma_py(data)
        assert native.module().fnv64a(data) == common.fnv64a_py(data)


@needs_native
def test_edit_distance_batch_matches_python():
    rng = random.Random(1)
    words = ["".join(rng.choice("abcde") for _ in range(rng.randint(0, 12))) for _ in range(40)]
    mat = native.module().edit_distance_batch(words, words[:9], 1, 1, 2, 4)
    for i, a in enumerate(words):
        for j, b in enumerate(words[:9]):
            assert mat[i][j] == editdistance.wagner_fischer_py(a, b)


@needs_native
def test_sniff_dockerfiles(tmp_path):
    good = tmp_path / "Dockerfile"
    good.write_text("# comment\nARG X=1\nFROM alpine:3 AS base\nRUN true\n")
    bad = tmp_path / "notes.txt"
    bad.write_text("hello\nFROM nothing\n")
    arg_only = tmp_path / "args"
    arg_only.write_text("ARG A\nRUN x\nFROM y\n")
    got = native.module().sniff_dockerfiles([str(good), str(bad), str(arg_only)], 2)
    want = [dockerfile_parser.sniff_first_from(str(p)) for p in (good, bad, arg_only)]
    assert list(got) == want
    assert got[0] != "" and got[1] == "" and got[2] == ""


@needs_native
def test_run_commands_parallel(tmp_path):
    argvs = [["/bin/sh", "-c", "printf '%s' \"$(pwd)\""], ["/bin/sh", "-c", "exit 3"], ["/bin/sh", "-c", "echo hi"]]
    cwds = [str(tmp_path), "", ""]
    res = native.module().run_commands(argvs, cwds, 3, 0.0)
    assert res[0][0] == 0 and res[0][1].decode() == str(tmp_path)
    assert res[1][0] == 3
    assert res[2] == (0, b"hi\n") or list(res[2]) == [0, b"hi\n"]


def test_python_fallback_distance_is_weighted():
    # sub = 2 = ins + del, so "ab" -> "ac" costs 2
    assert editdistance.wagner_fischer_py("ab", "ac") == 2
    assert editdistance.wagner_fischer_py("", "abc") == 3
    assert editdistance.wagner_fischer_py("kitten", "sitting") == 5


def test_write_files_batch(tmp_path, monkeypatch):
    from move2kube_amd.ops import native as nat
    umask = os.umask(0o022)
    os.umask(umask)
    d = tmp_path / "o"
    d.mkdir()
    items = [(str(d / "a.yaml"), "x: 1\n", 0o644), (str(d / "b.sh"), b"#!/bin/sh\n", 0o744),
             (str(d / "a.yaml"), "x: 2\n", 0o600), (str(tmp_path / "missing" / "c"), "z", 0o644)]
    errs = nat.write_files(items)
    assert errs[:3] == [None, None, None]
    assert isinstance(errs[3], OSError) and errs[3].errno == 2 and str(tmp_path / "missing" / "c") in str(errs[3])
    assert (d / "a.yaml").read_text() == "x: 2\n"               # last write wins
    assert (d / "a.yaml").stat().st_mode & 0o777 == 0o600 & ~umask
    assert (d / "b.sh").stat().st_mode & 0o777 == 0o744 & ~umask
    # ioutil.WriteFile: an existing file is truncated and keeps its permissions
    os.chmod(str(d / "b.sh"), 0o700)
    assert nat.write_files([(str(d / "b.sh"), "echo\n", 0o644)]) == [None]
    assert (d / "b.sh").stat().st_mode & 0o777 == 0o700 and (d / "b.sh").read_text() == "echo\n"
    # the pure-Python fallback behaves the same
    monkeypatch.setattr(nat, "_load", lambda: None)
    errs2 = nat.write_files(items)
    assert [type(e) for e in errs2] == [type(e) for e in errs]
    assert (d / "a.yaml").read_text() == "x: 2\n"


def test_remove_tree(tmp_path):
    from move2kube_amd.ops import native as nat
    keep = tmp_path / "keep"
    keep.mkdir()
    (keep / "precious").write_text("x")
    root = tmp_path / "out"
    (root / "a" / "b").mkdir(parents=True)
    (root / "a" / "b" / "f.yaml").write_text("1")
    (root / "top.txt").write_text("2")
    os.symlink(str(keep), str(root / "link-to-dir"))      # unlinked, never followed
    os.symlink(str(tmp_path / "missing"), str(root / "dangling"))
    nat.remove_tree(str(root))
    assert not root.exists() and (keep / "precious").read_text() == "x"
    f = tmp_path / "file"
    f.write_text("z")
    nat.remove_tree(str(f))
    assert not f.exists()
    with pytest.raises(OSError):
        nat.remove_tree(str(tmp_path / "nope"))


@needs_native
def test_non_utf8_file_names_round_trip(tmp_path):
    """File names are bytes on Linux: a Latin-1 name walks, is written and is
    removed through the native runtime like os.fsencode/os.fsdecode would."""
    root = os.fsencode(str(tmp_path))
    os.makedirs(os.path.join(root, b"d\xe9"))
    with open(os.path.join(root, b"d\xe9", b"caf\xe9.yaml"), "wb") as f:
        f.write(b"a: 1\n")
    paths, kinds, errors = native.walk(str(tmp_path))
    ppaths, pkinds, perrors = fsindex._walk_py(str(tmp_path))
    assert list(paths) == list(ppaths) and list(kinds) == list(pkinds) and not errors
    assert any(os.fsencode(p).endswith(b"caf\xe9.yaml") for p in paths)
    out = os.path.join(os.fsdecode(root), os.fsdecode(b"out\xff.txt"))
    assert native.write_files([(out, b"x", 0o644)]) == [None]
    with open(os.fsencode(out), "rb") as f:
        assert f.read() == b"x"
    native.remove_tree(os.fsdecode(os.path.join(root, b"d\xe9")))
    assert not os.path.exists(os.path.join(root, b"d\xe9"))


@needs_native
def test_sniff_dockerfiles_undecodable_from_line(tmp_path):
    """A Latin-1 byte in a FROM line is kept as a surrogate, as the Python
    sniffer does, instead of failing the batch (threaded and serial paths)."""
    p = tmp_path / "Dockerfile"
    p.write_bytes(b"FROM caf\xe9:1\nRUN x\n")
    want = dockerfile_parser.sniff_first_from(str(p))
    assert native.sniff_dockerfiles([str(p)]) == [want]
    assert native.sniff_dockerfiles([str(p)] * 100) == [want] * 100


def test_native_module_load_waits_for_a_loading_thread(monkeypatch):
    """Threads asking for the extension while another thread is still loading
    it get the module, not None (a collector thread once fell back to the
    Python process runner this way and imported subprocess half-way under
    another thread's feet)."""
    import threading
    import time
    import types
    from move2kube_amd.ops import native
    real = native.module()

    class SlowEnviron(dict):
        def get(self, key, default=None):
            time.sleep(0.05)   # widen the loading window
            return os.environ.get(key, default)
    monkeypatch.setattr(native, "os", types.SimpleNamespace(environ=SlowEnviron()))
    monkeypatch.setattr(native, "_tried", False)
    monkeypatch.setattr(native, "_mod", None)
    got = []
    threads = [threading.Thread(target=lambda: got.append(native.module())) for _ in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert got == [real] * 8


def test_dockerfile_sniff_native_matches_python_on_mutated_dockerfiles(tmp_path):
    """Differential fuzz of ops/csrc/m2k_native.cpp:sniff_one against
    source/dockerfile_parser.py:sniff_first_from over mutated Dockerfiles
    (directives, continuations with either escape, comments, CRLF, BOMs, bytes
    that are not UTF-8).  It found a first line holding only a continuation:
    buildkit trims the joined line before reading the instruction, so
    '\\\\\\n  FROM x' is a FROM."""
    import glob
    import random
    from move2kube_amd.ops import native
    from move2kube_amd.source.dockerfile_parser import sniff_first_from
    m = native.module()
    if m is None:
        pytest.skip("native extension not built")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    seeds = [open(p, "rb").read() for p in sorted(glob.glob(os.path.join(root, "samples", "**", "Dockerfile*"),
                                                            recursive=True))]
    toks = [b"\n", b"\r\n", b"\\\n", b"`\n", b"# escape=`\n", b"# escape=\\\n", b"#syntax=x\n", b"ARG X=1\n",
            b"FROM ", b"from ", b" AS ", b"--platform=linux ", b"# c\n", b"\t", b"  ", b"\xff", b"\xef\xbb\xbf",
            b"\\", b"`", b"#", b"ARG\n", b"FROM\n", b"\r"]
    rnd = random.Random(7)
    path = str(tmp_path / "Dockerfile")
    assert seeds
    for _ in range(3000):
        s = bytearray(rnd.choice(seeds))
        for _ in range(rnd.randint(1, 6)):
            i = rnd.randrange(len(s) + 1)
            if rnd.random() < 0.3 and i < len(s):
                del s[i:i + rnd.randint(1, 8)]
            else:
                s[i:i] = rnd.choice(toks)
        if rnd.random() < 0.2:
            s[0:0] = rnd.choice(toks)
        with open(path, "wb") as f:
            f.write(bytes(s))
        assert m.sniff_dockerfiles([os.fsencode(path)], 1)[0] == sniff_first_from(path), bytes(s)[:200]
    with open(path, "wb") as f:
        f.write(b"\\\n  FROM node:14\n")
    assert m.sniff_dockerfiles([os.fsencode(path)], 1)[0] == sniff_first_from(path) == "  FROM node:14"


def test_walk_order_is_byte_order_in_both_walkers(tmp_path):
    """filepath.Walk visits names in byte order (sort.Strings); the Python
    walker sorted str, which puts a surrogate-escaped byte (0xf5 ->
    U+DCF5) before U+E000 (bytes ee 80 80)."""
    from move2kube_amd.utils import fsindex
    base = os.fsencode(str(tmp_path))
    for name in (b"\xf5x", b"\xee\x80\x80", b"\xf0\x9f\x98\x80", b"a", b"\xff"):
        os.makedirs(os.path.join(base, name, b"sub"))
    want = sorted(os.listdir(base))       # bytes sort
    ppaths, _, _ = fsindex._walk_py(str(tmp_path))
    top = [p for p in ppaths if os.path.dirname(p) == str(tmp_path)]
    assert [os.fsencode(os.path.basename(p)) for p in top] == want
    if native.available():
        npaths, _, _ = native.module().walk(base)
        assert list(npaths) == list(ppaths)
