"""In-tree build of the native extensions.

* ``_m2k_native*.so`` - C++17 pybind11 module (host runtime), built with g++.
* ``libm2k_ed_hip.so`` - HIP library for gfx950 (``hipcc --offload-arch=gfx950``).
* ``move2kube_amd/_bytecode.bin`` - compiled code of every package module in
  one file (``ops/bytecode.py``), read once per CLI process.
* ``move2kube_amd/_startcache.bin`` - the packaged Go templates parsed and the
  package's regular expressions compiled (``ops/startcache_build.py``,
  ``utils/startcache.py``).

Run ``python -m move2kube_amd.ops.build`` (or ``__graft_entry__.build()``).
Builds are incremental: a target is rebuilt only when its sources changed.
"""

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def native_target():
    return os.path.join(HERE, "_m2k_native" + _ext_suffix())


def sshkey_target():
    return os.path.join(HERE, "_m2k_sshkey" + _ext_suffix())


def hip_target():
    return os.path.join(HERE, "libm2k_ed_hip.so")


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    print("+ " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


NATIVE_SOURCES = [os.path.join(CSRC, "m2k_native.cpp"), os.path.join(CSRC, "yaml_emit.cpp"),
                  os.path.join(CSRC, "yaml_parse.cpp"), os.path.join(CSRC, "k8s_marshal.cpp"),
                  os.path.join(CSRC, "proc_spawn.cpp")]
SANITIZERS = {"address": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"],
              "thread": ["-fsanitize=thread"]}


def build_native(force=False, out=None, sanitize=None):
    """Build ``_m2k_native``.  ``sanitize`` ("address" = ASan+UBSan, "thread" =
    TSan) builds an instrumented copy at ``out`` for the sanitizer test
    (``tests/test_sanitizers.py``); run it with the runtime ``LD_PRELOAD``-ed."""
    import pybind11
    srcs = NATIVE_SOURCES
    out = out or native_target()
    if not force and not _stale(out, srcs):
        return out
    inc = sysconfig.get_paths()["include"]
    cxx = os.environ.get("CXX", "g++")
    # The release build links libstdc++/libgcc statically with unused sections
    # dropped and their symbols kept local: a CLI process then maps one 0.6 MB
    # object instead of also loading and relocating the 2 MB libstdc++ (the
    # extension's import went from 1.9 to 0.5 ms; every command imports it).
    opt = (["-O3", "-fvisibility-inlines-hidden", "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections",
            "-Wl,-O1", "-static-libstdc++", "-static-libgcc", "-Wl,--exclude-libs,ALL", "-s"]
           if not sanitize else ["-O1", "-g"] + SANITIZERS[sanitize])
    _run([cxx] + opt + ["-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall",
                        "-I" + pybind11.get_include(), "-I" + inc] + srcs + ["-o", out + ".tmp", "-lpthread"])
    os.replace(out + ".tmp", out)
    return out


SSHKEY_SOURCES = [os.path.join(CSRC, "sshkey.cpp"), os.path.join(CSRC, "blowfish_pi.h")]


def build_sshkey(force=False, out=None, sanitize=None):
    """Build ``_m2k_sshkey`` (private SSH keys parsed and re-encoded in
    process, ``csrc/sshkey.cpp``), linked against the system's libcrypto.  A
    separate extension so that only a command that reads a key maps it."""
    import pybind11
    out = out or sshkey_target()
    if not force and not _stale(out, SSHKEY_SOURCES):
        return out
    inc = sysconfig.get_paths()["include"]
    cxx = os.environ.get("CXX", "g++")
    opt = (["-O2", "-fvisibility-inlines-hidden", "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections",
            "-static-libstdc++", "-static-libgcc", "-Wl,--exclude-libs,ALL", "-s"]
           if not sanitize else ["-O1", "-g"] + SANITIZERS[sanitize])
    _run([cxx] + opt + ["-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall",
                        "-I" + pybind11.get_include(), "-I" + inc, SSHKEY_SOURCES[0], "-o", out + ".tmp", "-lcrypto"])
    os.replace(out + ".tmp", out)
    return out


def find_hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            try:
                subprocess.run([c, "--version"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
                return c
            except (OSError, subprocess.CalledProcessError):
                continue
    return None


def build_hip(force=False, arch="gfx950"):
    src = os.path.join(CSRC, "ed_kernel.hip")
    out = hip_target()
    if not force and not _stale(out, [src]):
        return out
    hipcc = find_hipcc()
    if hipcc is None:
        raise RuntimeError("hipcc not found; cannot build the gfx950 kernel library")
    _run([hipcc, "--offload-arch=" + arch, "-O3", "-std=c++17", "-shared", "-fPIC", src, "-o", out + ".tmp"])
    os.replace(out + ".tmp", out)
    return out


def build_bytecode(force=False):
    """The package's bytecode bundle (``ops/bytecode.py``)."""
    from . import bytecode
    if not force and not bytecode.stale():
        return bytecode.target()
    return bytecode.write()


def build_startcache(force=False):
    """The start-up cache of parsed templates and compiled regular expressions
    (``ops/startcache_build.py``)."""
    from . import startcache_build
    if not force and not startcache_build.stale():
        return startcache_build.target()
    return startcache_build.write()


def have_openssl_headers():
    """Whether ``<openssl/evp.h>`` is on the compiler's include path (the
    ``libssl-dev`` package): ``_m2k_sshkey`` needs it to build."""
    cxx = os.environ.get("CXX", "g++")
    try:
        p = subprocess.run([cxx, "-E", "-x", "c++", "-"], input=b"#include <openssl/evp.h>\n",
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    except OSError:
        return False
    return p.returncode == 0


def build_all(force=False):
    outs = [build_native(force)]
    if have_openssl_headers():
        outs.append(build_sshkey(force))
    else:   # utils/sshkeys.py then parses keys through ssh-keygen
        sys.stderr.write("warning: OpenSSL headers not found (install libssl-dev); _m2k_sshkey not built, "
                         "encrypted SSH keys go through ssh-keygen\n")
    outs.append(build_hip(force))
    outs.append(build_bytecode(force))
    outs.append(build_startcache(force))
    return outs


def build_report(force=True):
    """Build every native target and describe what happened: one JSON-able
    dict per target with whether it was compiled in this call, the wall time
    and the output's size and SHA-256 (``__graft_entry__.build`` prints it)."""
    import hashlib
    import time
    report = []
    for name, fn, target in (("_m2k_native (g++, C++17/pybind11)", build_native, native_target()),
                             ("_m2k_sshkey (g++, C++17/pybind11, libcrypto)", build_sshkey, sshkey_target()),
                             ("libm2k_ed_hip (hipcc --offload-arch=gfx950)", build_hip, hip_target()),
                             ("_bytecode.bin (package bytecode bundle)", build_bytecode,
                              os.path.join(os.path.dirname(HERE), "_bytecode.bin")),
                             ("_startcache.bin (parsed templates, compiled regexes)", build_startcache,
                              os.path.join(os.path.dirname(HERE), "_startcache.bin"))):
        if fn is build_sshkey and not have_openssl_headers():
            report.append({"target": name, "skipped": "OpenSSL headers not found (libssl-dev)"})
            continue
        before = os.path.getmtime(target) if os.path.exists(target) else None
        t0 = time.perf_counter()
        out = fn(force)
        dt = time.perf_counter() - t0
        with open(out, "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
        report.append({"target": name, "path": os.path.relpath(out, os.path.dirname(os.path.dirname(HERE))),
                       "compiled": before is None or os.path.getmtime(out) != before,
                       "seconds": round(dt, 2), "bytes": os.path.getsize(out), "sha256": digest})
    return report


if __name__ == "__main__":
    force = "--force" in sys.argv
    for o in build_all(force):
        print(o)
