"""Phase tracing: Chrome trace-event JSON of every pipeline phase.

The reference's only tracing is its ``[%T] Begin`` / ``Done`` log lines around
each plugin (``internal/move2kube/planner.go:38-44``,
``internal/source/translator.go:47-64``, ``internal/optimizer/optimizer.go:41-48``)
with no timing.  Set ``M2K_TRACE=<file.json>`` (or call
:func:`enable`) and every :func:`span` - planners, metadata loaders, the
translate stages, optimizers, customizers, detector batches, writers - is
recorded with wall-clock begin/end and thread id.  The file is written when
the command ends (or at interpreter exit) and opens in ``chrome://tracing`` /
Perfetto.  Disabled, a span costs one global read.
"""

import os
import threading
import time

_lock = threading.Lock()
_events = None
_path = None
_t0 = time.perf_counter_ns()


def enable(path):
    """Start recording; :func:`flush` writes ``path``."""
    global _events, _path
    with _lock:
        _events = []
        _path = path


def enabled():
    return _events is not None


class _NoSpan:
    __slots__ = ()

    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_SPAN = _NoSpan()


class _Span:
    __slots__ = ("ev", "name", "cat", "args", "start")

    def __init__(self, ev, name, cat, args):
        self.ev, self.name, self.cat, self.args = ev, name, cat, args

    def __enter__(self):
        self.start = time.perf_counter_ns()

    def __exit__(self, *exc):
        end = time.perf_counter_ns()
        rec = {"name": self.name, "cat": self.cat, "ph": "X", "pid": os.getpid(), "tid": threading.get_ident(),
               "ts": (self.start - _t0) / 1000.0, "dur": (end - self.start) / 1000.0}
        if self.args:
            rec["args"] = {k: str(v) for k, v in self.args.items()}
        with _lock:
            self.ev.append(rec)
        return False


def span(name, cat="phase", **args):
    """Context manager recording one complete event (a shared no-op while
    tracing is off)."""
    ev = _events
    if ev is None:
        return _NO_SPAN
    return _Span(ev, name, cat, args)


def events():
    with _lock:
        return list(_events or [])


def flush():
    """Write the trace file (keeps recording)."""
    if _events is None or not _path:
        return None
    with _lock:
        data = {"traceEvents": list(_events), "displayTimeUnit": "ms"}
    d = os.path.dirname(os.path.abspath(_path))
    os.makedirs(d, exist_ok=True)
    import json
    with open(_path, "w") as f:
        json.dump(data, f)
    return _path


def summary():
    """Total milliseconds per span name (for logs and benchmarks)."""
    tot = {}
    for e in events():
        tot[e["name"]] = tot.get(e["name"], 0.0) + e["dur"] / 1000.0
    return dict(sorted(tot.items(), key=lambda kv: -kv[1]))


if os.environ.get("M2K_TRACE"):
    import atexit
    enable(os.environ["M2K_TRACE"])
    atexit.register(flush)
