"""Cache engine: replays answers from a ``kind: QACache`` file, matching by
description (case-insensitive or regex) and solution type (reference
``internal/qaengine/cacheengine.go``)."""

from ..models import qa
from .engine import Engine


class CacheEngine(Engine):
    go_type = "*qaengine.CacheEngine"

    def __init__(self, cache_file):
        self.cache = qa.Cache(cache_file)

    def go_s(self):
        """``%s`` of ``*CacheEngine``: its Cache struct, problems and all."""
        c = self.cache
        return "&{{{%s %s} {%s} {%s [%s]}}}" % (qa.SCHEME_GROUP_VERSION, qa.QACACHE_KIND, "", c.file,
                                                " ".join(p.go_s() for p in c.problems))

    def start_engine(self):
        self.cache.load()

    def fetch_answer(self, prob):
        return self.cache.get_solution(prob)

    def __repr__(self):
        return "CacheEngine(%s)" % self.cache.file
