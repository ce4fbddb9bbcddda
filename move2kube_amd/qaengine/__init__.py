"""The QA engine: an ordered chain of answer sources (QA caches, defaults,
an interactive CLI, or the HTTP REST API the UI drives) plus a write cache
that checkpoints every answer."""

from .engine import (add_caches, add_engine, before_remove, engines, fetch_answer,  # noqa: F401
                     flush_write_cache, get_write_cache, reset, set_write_cache, start_engine)
