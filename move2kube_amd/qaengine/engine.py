"""QA engine chain (reference ``internal/qaengine/engine.go:29-123``).

Engines are consulted in order until one resolves a problem; cache engines
added with :func:`add_caches` are *prepended* (highest priority).  Every
resolved answer is appended to the write cache (``<out>/m2kqacache.yaml``),
the resumable checkpoint of an interactive session.  Passwords are never
cached.

The reference rewrites the whole cache file on every answer.  Here the cache
is write-behind: it is flushed before any interactive engine (CLI prompt,
REST UI) can block waiting for a person, when the command ends (also on
errors and at interpreter exit), and pending answers are dropped when the
output directory holding the file is about to be removed - so the file on
disk at every point a user could interrupt is the one the reference would
have written.

Difference from the reference: when no engine resolves a problem the
reference loops forever on the last engine; here the last
engine is retried a bounded number of times and then the problem's default is
used (or an error raised when it has none).
"""

import atexit
import os
import threading

from ..models import qa
from ..utils import log
from ..utils.constants import DEFAULT_DIRECTORY_PERMISSION

_lock = threading.RLock()
_engines = []
_write_cache = None
MAX_LAST_ENGINE_RETRIES = 8


class Engine:
    # how the reference's log lines print the engine: %T, and %s of the
    # pointer (``&{...}``: every field with the verb applied)
    go_type = "*qaengine.Engine"

    def go_s(self):
        return "&{}"

    def start_engine(self):
        pass

    def fetch_answer(self, prob):
        raise NotImplementedError

    def __repr__(self):
        return type(self).__name__


def reset():
    """Drop all engines and the write cache (tests / in-process reuse)."""
    global _engines, _write_cache
    flush_write_cache()
    with _lock:
        _engines = []
        _write_cache = None


def engines():
    return list(_engines)


def start_engine(qaskip=False, qaport=0, qadisablecli=False):
    # imported on demand: the REST engine pulls in http.server, which a
    # --qaskip or terminal run never needs (CLI start-up time)
    if qaskip:
        from .default_engine import DefaultEngine
        e = DefaultEngine()
    elif not qadisablecli:
        from .cli_engine import CliEngine
        e = CliEngine()
    else:
        from .rest_engine import HTTPRESTEngine
        e = HTTPRESTEngine(qaport)
    add_engine(e)
    return e


def add_engine(e):
    try:
        e.start_engine()
    except Exception as ex:  # noqa: BLE001
        log.error("Ignoring engine %s due to error : %s", e.go_type, ex)
        return
    with _lock:
        _engines.append(e)


def add_caches(cache_files):
    from .cache_engine import CacheEngine
    new = []
    for f in cache_files:
        e = CacheEngine(f)
        try:
            e.start_engine()
        except Exception as ex:  # noqa: BLE001
            log.error("Ignoring engine %s due to error : %s", e.go_type, ex)
            continue
        new.append(e)
    with _lock:
        _engines[:0] = new


def fetch_answer(prob):
    """Resolve ``prob`` through the engine chain and record the answer."""
    ans = prob
    err = None
    with _lock:
        chain = list(_engines)
    if not chain:
        from .default_engine import DefaultEngine
        chain = [DefaultEngine()]
    for e in chain:
        if getattr(e, "interactive", False):
            flush_write_cache()
        try:
            ans = e.fetch_answer(prob.copy())
            err = None
        except Exception as ex:  # noqa: BLE001
            err = ex
            if log.logger.isEnabledFor(log.WARNING):  # go_s() prints the engine's whole cache
                log.warning("Error while fetching answer using engine %s : %s", e.go_s(), ex)
            continue
        if ans.resolved:
            break
    if not ans.resolved:
        last = chain[-1]
        for _ in range(MAX_LAST_ENGINE_RETRIES):
            try:
                ans = last.fetch_answer(prob.copy())
                err = None
            except Exception as ex:  # noqa: BLE001
                err = ex
                continue
            if ans.resolved:
                break
        if not ans.resolved:
            ans = prob.copy()
            try:
                ans.set_answer(prob.default)
                err = None
            except qa.ProblemError as ex:
                log.fatal("Unable to get answer to %s : %s", prob.desc, err or ex)
    if err is None and ans.resolved and _write_cache is not None:
        _write_cache.add_problem_solution(ans)
    return ans


def set_write_cache(cache_file, write_behind=True):
    global _write_cache
    flush_write_cache()
    d = os.path.dirname(cache_file)
    if d:
        os.makedirs(d, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
    c = qa.Cache(cache_file)
    c.write()
    c.write_behind = write_behind
    _write_cache = c
    return c


def flush_write_cache():
    c = _write_cache
    if c is not None:
        c.flush()


def before_remove(path):
    """``path`` is about to be deleted: drop pending answers if the write cache
    lives under it, otherwise persist them."""
    c = _write_cache
    if c is None:
        return
    cf = os.path.abspath(c.file)
    root = os.path.abspath(path)
    if cf == root or cf.startswith(root.rstrip(os.sep) + os.sep):
        c.discard_pending()
    else:
        c.flush()


atexit.register(flush_write_cache)


def get_write_cache():
    return _write_cache
