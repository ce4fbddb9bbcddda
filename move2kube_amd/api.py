"""In-process programmatic API (what the CLI does, without argv parsing or
process-global leftovers between runs).  Used by tests, ``bench.py`` and
embedding applications."""

import contextlib
import gc
import os
import sys

from . import assets, move2kube, qaengine
from .containerizer import cnb
from .models import plan as plantypes
from .utils import common, fsindex, sshkeys, yamlio
from .utils.constants import QA_CACHE_FILE, settings


def reset_state():
    """Forget engines, caches and provider probes from a previous run."""
    qaengine.reset()
    fsindex.drop_kept()
    cnb.reset_cache()
    providers = sys.modules.get("move2kube_amd.containerizer.cnb.providers")
    if providers is not None:
        providers.reset_providers()
    sshkeys.reset()


@contextlib.contextmanager
def gc_paused():
    """No cyclic collection during one command.  A run's objects live until it
    ends, so the collector's full passes only re-walk a heap that keeps
    growing: on a 5,000-app tree that made translate 18 % slower per service
    than on 100 apps (``benchmarks/translate_large_tree.py``).  The run's
    garbage (about 10 KB per service) is left to the next collection after it."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


class Session:
    """Assets directory + QA engine setup for one or more runs."""

    def __init__(self, qaskip=True, qacaches=(), ignore_env=True):
        self.qaskip = qaskip
        self.qacaches = list(qacaches)
        self.ignore_env = ignore_env
        self._temp = None

    def __enter__(self):
        self._saved_ignore_env = settings.ignore_environment
        self._temp = assets.setup()
        return self

    def __exit__(self, *exc):
        assets.cleanup(self._temp)
        settings.ignore_environment = self._saved_ignore_env
        return False

    def _start(self):
        reset_state()
        settings.ignore_environment = self.ignore_env
        qaengine.start_engine(self.qaskip, 0, False)
        qaengine.add_caches(list(reversed(self.qacaches)))

    def collect(self, src, outdir, annotations=()):
        """``move2kube collect -s src -o outdir -a ...``: metadata under
        ``outdir/m2k_collect``; no provider probe of an earlier run is reused."""
        reset_state()
        move2kube.collect(common.go_abs(src) if src else "", os.path.join(outdir, "m2k_collect"), list(annotations))

    def plan(self, src, name="myproject"):
        self._start()
        with gc_paused(), yamlio.parse_cache():
            return move2kube.create_plan(common.go_abs(src), name)

    def translate(self, src, outdir, name="myproject", plan=None, curate=True):
        """``move2kube translate -s src -o outdir -n name`` (new plan unless one is
        given).  Returns the project output directory."""
        self._start()
        with gc_paused(), yamlio.parse_cache():
            return self._translate(src, outdir, name, plan, curate)

    def _translate(self, src, outdir, name, plan, curate):
        if plan is None:
            src = common.go_abs(src)
            p = move2kube.create_plan(src, name, keep_index=fsindex.handoff_allowed(
                src, os.path.join(common.go_abs(outdir), name)))
        else:
            p = plan if isinstance(plan, plantypes.Plan) else plantypes.read_plan(plan)
        out = os.path.join(common.go_abs(outdir), p.name)
        os.makedirs(out, exist_ok=True)
        qaengine.set_write_cache(os.path.join(out, QA_CACHE_FILE))
        if curate:
            p = move2kube.curate_plan(p)
        move2kube.translate(p, out, False)
        return out


def translate(src, outdir, name="myproject", qaskip=True, qacaches=()):
    with Session(qaskip=qaskip, qacaches=qacaches) as s:
        return s.translate(src, outdir, name)
