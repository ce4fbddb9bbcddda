"""Directory <-> base64 tar string (reference ``internal/common/tar.go:32-116``).

``tar_as_string`` walks the directory in lexical order (``filepath.Walk``) and
stores entries relative to it (the root itself as ``.``); ``ignore_files``
holds relative names to leave out.  ``untar_string`` recreates the tree,
directories with 0755 and files with their archived permission bits.  Unlike
the reference, entries that would land outside the destination (absolute
names, ``..``) are rejected.
"""

import base64
import io
import os
import tarfile

from . import common, log
from .constants import DEFAULT_DIRECTORY_PERMISSION


class TarError(ValueError):
    pass


def tar_as_string(path, ignore_files=()):
    buf = io.BytesIO()
    ignore = set(ignore_files)
    err = None
    with tarfile.open(fileobj=buf, mode="w", format=tarfile.PAX_FORMAT) as tw:
        def add(cur):
            """Add one entry; True if it is a directory to descend into.  Like
            the reference's Walk callback, an ignored name is left out of the
            archive but an ignored directory's contents are still walked."""
            rel = os.path.relpath(cur, path)
            info = tw.gettarinfo(cur, arcname=rel)
            if rel not in ignore:
                if info.isreg():
                    with open(cur, "rb") as f:
                        tw.addfile(info, f)
                else:
                    tw.addfile(info)
            return info.isdir()

        def walk(d):
            # filepath.Walk order: lexical, depth first, parent before children
            for name in sorted(os.listdir(d)):
                p = os.path.join(d, name)
                if add(p):
                    walk(p)

        try:
            if not os.path.lexists(path):
                raise FileNotFoundError("lstat %s: no such file or directory" % path)
            if add(path):
                walk(path)
        except OSError as e:
            # the Walk callback's os.Open (a file's contents, a directory's
            # names) is what fails on a path without permissions
            err = common.go_path_error(e, "open")
            log.warning("Failed to create tar string: %s : %s", path, err)
    s = base64.b64encode(buf.getvalue()).decode()
    if err is not None:
        raise TarError(err)
    return s


def _members(tr):
    """Iterate members, treating a missing end-of-archive trailer as EOF (the
    reference encodes its tar before closing the writer, so its strings lack
    the trailer and the last entry's padding)."""
    while True:
        try:
            m = tr.next()
        except tarfile.ReadError:
            return
        if m is None:
            return
        yield m


def untar_string(tar_string, path):
    try:
        raw = base64.b64decode(tar_string, validate=True)
    except ValueError as e:
        log.error("Unable to decode tarstring : %s", e)
        raise TarError(str(e))
    root = os.path.abspath(path)
    with tarfile.open(fileobj=io.BytesIO(raw), mode="r:") as tr:
        for m in _members(tr):
            dst = os.path.abspath(os.path.join(root, m.name))
            if dst != root and not dst.startswith(root + os.sep):
                raise TarError("tar entry %r escapes the destination" % m.name)
            if m.isdir():
                os.makedirs(dst, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
                continue
            if not m.isreg():
                continue
            os.makedirs(os.path.dirname(dst), mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
            src = tr.extractfile(m)
            data = src.read() if src is not None else b""
            with open(dst, "wb") as f:
                f.write(data)
            os.chmod(dst, m.mode & 0o777)
            if len(data) != m.size:
                raise TarError("Size mismatch: Wrote %d, Expected %d" % (len(data), m.size))
