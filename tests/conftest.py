import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"

# deterministic offline runs everywhere
os.environ.setdefault("M2K_NO_NETWORK", "1")
os.environ.setdefault("M2K_DISABLE_CNB", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "reference: needs the read-only reference checkout for its fixtures")


def pytest_collection_modifyitems(config, items):
    if os.path.isdir(REFERENCE):
        return
    skip = pytest.mark.skip(reason="reference fixtures not available")
    for item in items:
        if "reference" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _fresh_state():
    """Every test starts with no QA engines, no caches and default settings."""
    from move2kube_amd import api
    from move2kube_amd.utils.constants import settings
    api.reset_state()
    saved = (settings.compat, settings.ignore_environment, settings.temp_path, settings.assets_path)
    yield
    api.reset_state()
    settings.compat, settings.ignore_environment, settings.temp_path, settings.assets_path = saved


@pytest.fixture
def assets_dir(monkeypatch):
    """A private unpacked copy of m2kassets (tests may edit detectors; the CLI
    itself uses the packaged tree read-only)."""
    from move2kube_amd import assets
    from move2kube_amd.utils.constants import settings
    monkeypatch.setenv("M2K_UNPACK_ASSETS", "1")
    tmp = assets.setup()
    yield settings.assets_path
    assets.cleanup(tmp)


def ref_path(*parts):
    return os.path.join(REFERENCE, *parts)
