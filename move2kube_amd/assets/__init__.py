"""Packaged assets and their bootstrap.

* ``m2kassets/`` - containerizer detector directories (``dockerfiles/*`` with
  ``m2kdfdetect.sh`` + ``Dockerfile`` template, ``s2i/*`` with
  ``m2ks2idetect.sh`` + ``.s2i/environment``).  Copied at start-up into a fresh
  temp dir exactly like the reference unpacks its embedded tar
  (``internal/common/utils.go:550-582``), so plans keep the portable
  ``m2kassets/...`` relative paths.
* ``templates/`` - output/build-script Go templates.
* ``clusters.json`` - the 7 built-in target-cluster profiles.
* ``cfbuildpacks.json`` - built-in CF buildpack containerization map.
"""

import os
import shutil

from ..utils import fastjson, log
from ..utils.constants import ASSETS_DIR, TEMP_DIR_PREFIX, settings

HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS_SRC = os.path.join(HERE, "m2kassets")
TEMPLATES_DIR = os.path.join(HERE, "templates")

_templates = {}
_clusters = None


def template(name):
    t = _templates.get(name)
    if t is None:
        with open(os.path.join(TEMPLATES_DIR, name)) as f:
            t = f.read()
        _templates[name] = t
    return t


def builtin_clusters():
    """{name: {"storageClasses": [...], "apiKindVersionMap": {...}}}"""
    global _clusters
    if _clusters is None:
        with open(os.path.join(HERE, "clusters.json")) as f:
            _clusters = fastjson.load(f)
    return _clusters


def builtin_cf_buildpacks():
    with open(os.path.join(HERE, "cfbuildpacks.json")) as f:
        return fastjson.load(f)["buildpackContainerizers"]


def _copy_tree(src, dst):
    os.makedirs(dst, exist_ok=True)
    for entry in os.scandir(src):
        s = entry.path
        d = os.path.join(dst, entry.name)
        if entry.is_dir(follow_symlinks=False):
            _copy_tree(s, d)
        else:
            shutil.copyfile(s, d)
            shutil.copymode(s, d)


def create_assets_data():
    """Point at the detector assets.

    The reference unpacks its embedded asset tar into a fresh
    ``<tmp>/m2kassets`` on every run (``internal/common/utils.go:550-582``).
    The installed package already holds that tree, and nothing writes into it
    (the runc CNB provider gets its own :func:`scratch_dir`), so it is used in
    place: ``temp_path`` is this package directory and plans keep the same
    portable ``m2kassets/...`` paths.  Set ``M2K_UNPACK_ASSETS=1`` to copy into
    a temp dir like the reference; single-file distributions, which carry the
    assets as an embedded tar (``make generate``), always unpack.

    Returns (assets_path, temp_path)."""
    if os.path.isdir(ASSETS_SRC) and os.environ.get("M2K_UNPACK_ASSETS", "") in ("", "0"):
        return ASSETS_SRC, HERE
    import tempfile
    temp_path = os.path.abspath(settings.temp_path)
    assets_path = os.path.abspath(settings.assets_path)
    try:
        temp_path = tempfile.mkdtemp(prefix=TEMP_DIR_PREFIX)
        assets_path = os.path.join(temp_path, ASSETS_DIR)
    except OSError:
        log.error("Unable to create temp dir. Defaulting to local path.")
    if os.path.isdir(ASSETS_SRC):
        _copy_tree(ASSETS_SRC, assets_path)
    else:
        from ..utils import tarutil
        from . import _embedded_assets  # noqa: F401 - generated module
        tarutil.untar_string(_embedded_assets.TAR, assets_path)
    return assets_path, temp_path


_scratch = []


def scratch_dir():
    """A writable per-command temp dir (created on first use, removed by :func:`cleanup`)."""
    if not _scratch:
        import tempfile
        _scratch.append(tempfile.mkdtemp(prefix=TEMP_DIR_PREFIX + "scratch-"))
    return _scratch[0]


def setup():
    """Create the assets dir and point the global settings at it (cmd main)."""
    assets_path, temp_path = create_assets_data()
    settings.temp_path = temp_path
    settings.assets_path = assets_path
    return temp_path


def cleanup(temp_path=None):
    temp_path = temp_path or settings.temp_path
    # never the package's own asset tree (used in place, see create_assets_data)
    if temp_path and os.path.realpath(temp_path) != os.path.realpath(HERE):
        shutil.rmtree(temp_path, ignore_errors=True)
    while _scratch:
        shutil.rmtree(_scratch.pop(), ignore_errors=True)
