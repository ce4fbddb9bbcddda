#!/usr/bin/env python3
"""Build distribution archives (reference ``scripts/builddist.go``): one
``move2kube-amd-<version>-linux-<arch>.tar.gz`` and ``.zip`` holding the
package (with its in-tree native/HIP libraries), ``bench.py``, the samples,
README and a ``bin/move2kube`` launcher, plus a ``.sha256sum`` per archive."""

import argparse
import hashlib
import os
import platform
import shutil
import stat
import sys
import tarfile
import zipfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = ["move2kube_amd", "samples", "bench.py", "__graft_entry__.py", "README.md", "pyproject.toml"]
SKIP_DIRS = {"__pycache__", ".pytest_cache"}

LAUNCHER = """#!/usr/bin/env sh
HERE="$(cd "$(dirname "$0")/.." && pwd)"
PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}" exec "${PYTHON:-python3}" -m move2kube_amd "$@"
"""


def files(root):
    for item in INCLUDE:
        p = os.path.join(root, item)
        if os.path.isfile(p):
            yield item
            continue
        for dp, dns, fns in os.walk(p):
            dns[:] = sorted(d for d in dns if d not in SKIP_DIRS)
            for fn in sorted(fns):
                if fn.endswith(".pyc") or fn.endswith(".tmp"):
                    continue
                yield os.path.relpath(os.path.join(dp, fn), root)


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--version", required=True)
    ap.add_argument("--commit", default="")
    ap.add_argument("--tree", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "dist"))
    a = ap.parse_args()
    arch = {"x86_64": "amd64", "aarch64": "arm64"}.get(platform.machine(), platform.machine())
    name = "move2kube-amd-%s-linux-%s" % (a.version, arch)
    os.makedirs(a.out, exist_ok=True)
    listing = list(files(ROOT))
    tgz = os.path.join(a.out, name + ".tar.gz")
    zp = os.path.join(a.out, name + ".zip")
    with tarfile.open(tgz, "w:gz") as t:
        for rel in listing:
            t.add(os.path.join(ROOT, rel), arcname=os.path.join(name, rel), recursive=False)
        info = tarfile.TarInfo(os.path.join(name, "bin", "move2kube"))
        data = LAUNCHER.encode()
        info.size = len(data)
        info.mode = 0o755
        import io
        t.addfile(info, io.BytesIO(data))
    with zipfile.ZipFile(zp, "w", zipfile.ZIP_DEFLATED) as z:
        for rel in listing:
            z.write(os.path.join(ROOT, rel), os.path.join(name, rel))
        zi = zipfile.ZipInfo(os.path.join(name, "bin", "move2kube"))
        zi.external_attr = (stat.S_IFREG | 0o755) << 16
        z.writestr(zi, LAUNCHER)
    for p in (tgz, zp):
        with open(p + ".sha256sum", "w") as f:
            f.write("%s  %s\n" % (sha256(p), os.path.basename(p)))
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
