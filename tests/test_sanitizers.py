"""Host-code sanitizers for the native runtime (the reference's ``go test -race``,
``Makefile:92``): ``_m2k_native`` is rebuilt with ASan+UBSan and with TSan and
every multi-threaded entry point (walk, Dockerfile sniffing, edit distance,
closest match, batched writes, the spawn pool, the YAML emitter and loader) is driven in
a child interpreter with the sanitizer runtime preloaded; any report fails the
test (``halt_on_error``).  GPU code is not involved (GPU sanitizers are not
available on the target pool)."""

import os
import subprocess
import sys
import sysconfig
import textwrap

import pytest

from move2kube_amd.ops import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = textwrap.dedent(r'''
    import os, sys, threading
    sys.path.insert(0, sys.argv[1])      # the instrumented module
    sys.path.insert(1, sys.argv[2])      # the repo (pure-Python helpers only)
    import _m2k_native as m
    from move2kube_amd.utils import yamlio
    work = sys.argv[3]
    # a tree to walk and sniff
    files = []
    for i in range(40):
        d = os.path.join(work, "t", "d%02d" % i, "sub")
        os.makedirs(d, exist_ok=True)
        for j in range(5):
            p = os.path.join(d, "Dockerfile.%d" % j)
            with open(p, "w") as f:
                f.write("ARG x\nFROM alpine:3\n" if j % 2 else "RUN true\n")
            files.append(p)
    paths, kinds, errs = m.walk(os.path.join(work, "t"))
    assert len(paths) == 40 * 7 + 1, len(paths)
    assert sum(1 for r in m.sniff_dockerfiles(files, 8) if r) == 80
    opts = ["buildpack-%d-%s" % (i, "x" * (i % 50)) for i in range(3000)]
    qs = ["buildpack-%d" % i for i in range(0, 3000, 7)]
    mat = m.edit_distance_batch(qs[:40], opts[:500], 1, 1, 2, 8)
    assert mat.shape == (40, 500)
    idx, dist = m.closest_batch(opts, qs, 8)
    assert len(idx) == len(qs)
    buf, offs, mx = m.pack_strings(opts)
    assert mx == max(len(o) for o in opts)
    assert len(offs) == len(opts) + 1
    out = os.path.join(work, "o")
    os.makedirs(out)
    items = [os.path.join(out, "f%03d.yaml" % (i % 150)) for i in range(300)]
    errs = m.write_files(items, [b"k: %d\n" % i for i in range(300)], [0o644] * 300, 8)
    assert not any(errs)
    os.makedirs(os.path.join(out, "d1", "d2"))
    os.symlink(work, os.path.join(out, "d1", "up"))
    err, where = m.remove_tree(out)
    assert err == 0 and not os.path.exists(out), (err, where)
    res = m.run_commands([["/bin/sh", "-c", "echo %d" % i] for i in range(24)], ["/"] * 24, 8, 30.0)
    assert len(res) == 24
    # proc_spawn / proc_wait (proc_spawn.cpp) from 4 threads: pipes, merged
    # stderr, a timeout kill, a missing executable
    failures = []
    def tools(k):
      try:
        for i in range(6):
            pid, o, e = m.proc_spawn([b"/bin/sh", b"-c", b"echo out%d; echo err >&2" % i], None, -1, -1)
            rc, out, err, to = m.proc_wait(pid, o, e, 10.0)
            assert (rc, out, err, to) == (0, b"out%d\n" % i, b"err\n", False)
            pid, o, e = m.proc_spawn([b"/bin/sh", b"-c", b"echo x >&2; exit 3"], b"/", -1, -4)
            assert m.proc_wait(pid, o, e, 10.0) == (3, b"x\n", b"", False)
        pid, o, e = m.proc_spawn([b"/bin/sh", b"-c", b"exec sleep 5"], None, -2, -2)
        assert m.proc_wait(pid, o, e, 0.05)[3] is True
        # procgroup_*: several children in one poll loop, one of them timing
        # out, a big output, and a group dropped with a live member
        g = m.procgroup_new()
        for key, cmd, to in ((0, b"echo a; echo b >&2", 10.0), (1, b"exec sleep 5", 0.05),
                             (2, b"head -c 300000 /dev/zero", 10.0)):
            pid, o, e = m.proc_spawn([b"/bin/sh", b"-c", cmd], None, -1, -1)
            m.procgroup_add(g, key, pid, o, e, to)
        got = {}
        while True:
            r = m.procgroup_wait_any(g)
            if r is None:
                break
            got[r[0]] = r
        assert got[0][1:] == (0, b"a\n", b"b\n", False) and got[1][4] is True and len(got[2][2]) == 300000
        g = m.procgroup_new()
        pid, o, e = m.proc_spawn([b"/bin/sh", b"-c", b"exec sleep 5"], None, -1, -1)
        m.procgroup_add(g, 0, pid, o, e, 0.0)
        del g   # kills and reaps the sleeper
        try:
            m.proc_spawn([b"m2k-no-such-tool"], None, -1, -2)
        except FileNotFoundError:
            pass
        else:
            raise AssertionError("spawned a missing tool")
      except BaseException as ex:
        failures.append(repr(ex))
    ts = [threading.Thread(target=tools, args=(k,)) for k in range(4)]
    for t in ts: t.start()
    for t in ts: t.join()
    assert not failures, failures
    doc = {"a": [1, {"b": "x: y", "c": "multi\nline\n"}], "n": None, "f": 1.5, "u": "hé",
           "m": yamlio.GoMap({"b10": 1, "b9": 2, "k": "007"})}
    def emit():
        for _ in range(200):
            s = m.yaml_dump(doc, True, yamlio.GoMap, yamlio._scalar_lines, yamlio._string_style,
                            yamlio.go_key_sorted)
            assert s == yamlio.dump_py(doc, True), s
    ts = [threading.Thread(target=emit) for _ in range(4)]
    for t in ts: t.start()
    for t in ts: t.join()
    # the YAML loader on well-formed, truncated and malformed inputs (every prefix
    # of a document exercises each end-of-input path of the line scanner)
    unsup = object()
    text = m.yaml_dump(doc, True, yamlio.GoMap, yamlio._scalar_lines, yamlio._string_style, yamlio.go_key_sorted)
    text += "---\nk: 'q''s'\nl: [1, \"x\\u00e9\", {a: b}]\nb: |+\n  x\n\n  y\nf: >-\n  p\n   q\n"
    for i in range(len(text) + 1):
        for mode in (0, 1, 2):
            m.yaml_load(text[:i], mode, True, yamlio.go_resolve_number, unsup)
            m.yaml_load(text[:i], mode, False, yamlio.go_resolve_number, unsup)
    assert m.yaml_load(text, 0, True, yamlio.go_resolve_number, unsup)[0] == doc
    # mutation fuzzing over the YAML files of samples/: flipped, dropped and
    # inserted bytes (YAML indicators, quotes, tabs, newlines, non-ASCII)
    import glob, random
    rnd = random.Random(5)
    corpus = []
    for pth in sorted(glob.glob(os.path.join(sys.argv[2], "samples", "**", "*.y*ml"), recursive=True))[:12]:
        with open(pth, encoding="utf-8", errors="replace") as fh:
            corpus.append(fh.read()[:4000])
    alphabet = list(":-[]{}\"'|>#&*!%@`?,\t\n ") + ["\u00e9", "\ufeff", "\x00", "\\u00", "0x", "1e9", ".inf"]
    for doc_text in corpus:
        for _ in range(150):
            t = list(doc_text)
            for _ in range(rnd.randint(1, 6)):
                op, i = rnd.randint(0, 2), rnd.randrange(len(t) + 1)
                if op == 0 and i < len(t):
                    del t[i]
                elif op == 1:
                    t.insert(i, rnd.choice(alphabet))
                elif i < len(t):
                    t[i] = rnd.choice(alphabet)
            mutated = "".join(t)
            for mode in (0, 1, 2):
                m.yaml_load(mutated, mode, True, yamlio.go_resolve_number, unsup)
    # repeated keys are left to PyYAML
    assert m.yaml_load("a: 1\nb: {c: 1, c: 2}\n", 0, False, yamlio.go_resolve_number, unsup) is unsup
    # the struct marshaller (k8s_marshal.cpp) against its Python specification
    from move2kube_amd.k8s import schema
    m.schema_init(schema._STRUCTS, schema._marshal_value)
    objs = [({"kind": "Deployment", "apiVersion": "apps/v1", "metadata": {"name": "d", "labels": {"a": "b"}},
              "spec": {"replicas": 2, "template": {"spec": {"containers": [{"name": "c", "image": "i",
              "ports": [{"containerPort": 80}], "env": [{"name": "X", "value": ""}]}]}}}}, "Deployment"),
            ({"kind": "Secret", "data": {"k": "dg=="}, "type": ""}, "Secret"),
            ({"spec": [1, 2]}, "Service"), ({}, "Route"), ([1], "Pod")]
    def marshal():
        for _ in range(100):
            for o, t in objs:
                try:
                    got = m.schema_marshal(o, t)
                except AttributeError:
                    got = "err"
                try:
                    want = schema._marshal_struct(o, t)
                except AttributeError:
                    want = "err"
                assert got == want, (t, got, want)
    ts = [threading.Thread(target=marshal) for _ in range(4)]
    for t in ts: t.start()
    for t in ts: t.join()
    print("SANITIZER-DRIVER-OK")
''')


def _runtime(lib):
    p = subprocess.run(["gcc", "-print-file-name=" + lib], stdout=subprocess.PIPE, text=True)
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


@pytest.mark.parametrize("kind,lib", [("address", "libasan.so"), ("thread", "libtsan.so")])
def test_native_runtime_under_sanitizer(kind, lib, tmp_path):
    rt = _runtime(lib)
    if rt is None:
        pytest.skip("%s runtime not installed" % lib)
    moddir = tmp_path / "mod"
    moddir.mkdir()
    so = str(moddir / ("_m2k_native" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")))
    build.build_native(force=True, out=so, sanitize=kind)
    env = dict(os.environ)
    # libstdc++ is preloaded too: python itself does not link it, and without it
    # the runtime's __cxa_throw interceptor has no real function to forward
    # to, so the first C++ exception (the YAML loader's bail-out) aborts
    cxx = _runtime("libstdc++.so.6")
    env.update({
        "LD_PRELOAD": rt + (" " + cxx if cxx else ""),
        "M2K_DISABLE_NATIVE": "1",  # the package itself must not load the uninstrumented build
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "TSAN_OPTIONS": "halt_on_error=1:report_signal_unsafe=0",
    })
    drv = tmp_path / "driver.py"
    drv.write_text(DRIVER)
    work = tmp_path / "work"
    work.mkdir()
    p = subprocess.run([sys.executable, str(drv), str(moddir), ROOT, str(work)], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert p.returncode == 0 and "SANITIZER-DRIVER-OK" in p.stdout, p.stdout[-4000:]
    assert "WARNING: ThreadSanitizer" not in p.stdout and "ERROR: AddressSanitizer" not in p.stdout, p.stdout[-4000:]


SSHKEY_DRIVER = textwrap.dedent(r'''
    import glob, os, sys, threading
    sys.path.insert(0, sys.argv[1])
    import _m2k_sshkey as m
    fix = sys.argv[2]
    keys = sorted(glob.glob(os.path.join(fix, "*.key")))
    assert len(keys) >= 15
    def run(k):
        data = open(k, "rb").read()
        st, txt = m.private_key_pem(data, None)
        if st == 1:
            st, txt = m.private_key_pem(data, b"m2k-pass")
        exp = k[:-4] + ".expected.pem"
        if os.path.exists(exp):
            assert (st, txt) == (0, open(exp).read()), (k, st, txt)
        # every truncation and a byte flip at each of a few hundred offsets:
        # errors, never a crash or an out-of-bounds access
        for i in range(0, len(data), max(1, len(data) // 150)):
            m.private_key_pem(data[:i], None)
            bad = bytearray(data)
            bad[i] ^= 0x5A
            m.private_key_pem(bytes(bad), None)
            m.private_key_pem(bytes(bad), b"m2k-pass")
        # the same on the decoded body, re-armoured: every length field of
        # openssh-key-v1 / DER reached with huge, zero and off-by-one values
        import base64
        lines = data.decode("ascii", "replace").strip().splitlines()
        head = [l for l in lines if l.startswith("-----BEGIN")]
        if not head or any(":" in l for l in lines[1:4]):
            return
        body = base64.b64decode("".join(l for l in lines if not l.startswith("-----")))
        tail = head[0].replace("BEGIN", "END")
        def armour(b):
            t = base64.b64encode(b).decode()
            return ("\n".join([head[0]] + [t[j:j + 70] for j in range(0, len(t), 70)] + [tail]) + "\n").encode()
        for i in range(0, len(body), max(1, len(body) // 120)):
            for patch in (b"\xff\xff\xff\xff", b"\x00\x00\x00\x00", b"\x7f\xff\xff\xfe", b"\x00\x00\x00\x11"):
                b2 = body[:i] + patch + body[i + 4:]
                m.private_key_pem(armour(b2), None)
                m.private_key_pem(armour(b2), b"m2k-pass")
            m.private_key_pem(armour(body[:i]), b"m2k-pass")
    ts = [threading.Thread(target=run, args=(k,)) for k in keys]
    for t in ts: t.start()
    for t in ts: t.join()
    print("SANITIZER-DRIVER-OK")
''')


def test_sshkey_converter_under_asan(tmp_path):
    rt = _runtime("libasan.so")
    if rt is None:
        pytest.skip("libasan.so runtime not installed")
    moddir = tmp_path / "mod"
    moddir.mkdir()
    so = str(moddir / ("_m2k_sshkey" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")))
    build.build_sshkey(force=True, out=so, sanitize="address")
    cxx = _runtime("libstdc++.so.6")
    env = dict(os.environ, LD_PRELOAD=rt + (" " + cxx if cxx else ""),
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    drv = tmp_path / "driver.py"
    drv.write_text(SSHKEY_DRIVER)
    p = subprocess.run([sys.executable, str(drv), str(moddir), os.path.join(ROOT, "tests", "fixtures", "sshkeys")],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert p.returncode == 0 and "SANITIZER-DRIVER-OK" in p.stdout, p.stdout[-4000:]
    assert "ERROR: AddressSanitizer" not in p.stdout and "runtime error" not in p.stdout, p.stdout[-4000:]
