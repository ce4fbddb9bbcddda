"""Write-behind of output files during one ``translate``.

Serialising objects is Python work that holds the GIL; creating the files is
kernel work that the native ``write_files`` does with the GIL released.  Inside
a :func:`scope`, :func:`write` hands each batch to one background thread and
returns at once, so the next objects are serialised while the previous batch
is written.  Batches are written in submission order (a later batch to the
same path wins, as with sequential writes).  Completion callbacks - the
logging of failures and of created files - run on the submitting thread, in
order, at :func:`drain`; the translate drains before anything reads the output
(operator-sdk reads the Helm chart) and when the scope ends.  Outside a scope,
:func:`write` is synchronous.
"""

import threading

from . import native

_local = threading.local()


class _Writer:
    def __init__(self):
        import _queue
        self._q = _queue.SimpleQueue()
        self._done = []  # (callback, results or exception), in submission order
        self._pending = 0
        self._cv = threading.Condition()
        self._thread = threading.Thread(target=self._run, name="m2k-write-behind", daemon=True)
        self._thread.start()

    def _run(self):
        while True:
            job = self._q.get()
            if job is None:
                return
            items, callback = job
            try:
                res = native.write_files(items)
            except Exception as e:  # noqa: BLE001 - reported on the submitting thread
                res = e
            with self._cv:
                self._done.append((callback, res))
                self._pending -= 1
                self._cv.notify_all()

    def submit(self, items, callback):
        with self._cv:
            self._pending += 1
        self._q.put((items, callback))

    def drain(self):
        with self._cv:
            while self._pending:
                self._cv.wait()
            done, self._done = self._done, []
        for callback, res in done:
            if isinstance(res, Exception):
                raise res
            callback(res)

    def close(self):
        try:
            self.drain()
        finally:
            self._q.put(None)
            self._thread.join()


class scope:
    """Context manager: writes inside it are asynchronous until drained
    (``M2K_WRITE_BEHIND=0``: synchronous, for comparison runs)."""

    def __enter__(self):
        import os
        self._prev = getattr(_local, "writer", None)
        self._writer = None if os.environ.get("M2K_WRITE_BEHIND") == "0" else _Writer()
        _local.writer = self._writer
        return self

    def __exit__(self, *exc):
        _local.writer = self._prev
        if self._writer is not None:
            self._writer.close()
        return False


def write(items, callback):
    """Write ``[(path, data, mode)]`` and call ``callback(errors)`` (one
    ``OSError`` or None per item) - later, at :func:`drain`, inside a scope."""
    w = getattr(_local, "writer", None)
    if w is None:
        callback(native.write_files(items))
    else:
        w.submit(items, callback)


def drain():
    """Wait for every submitted batch and run their callbacks."""
    w = getattr(_local, "writer", None)
    if w is not None:
        w.drain()
