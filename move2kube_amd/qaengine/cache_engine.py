"""Cache engine: replays answers from a ``kind: QACache`` file, matching by
description (case-insensitive or regex) and solution type (reference
``internal/qaengine/cacheengine.go``)."""

from ..models import qa
from .engine import Engine


class CacheEngine(Engine):
    def __init__(self, cache_file):
        self.cache = qa.Cache(cache_file)

    def start_engine(self):
        self.cache.load()

    def fetch_answer(self, prob):
        return self.cache.get_solution(prob)

    def __repr__(self):
        return "CacheEngine(%s)" % self.cache.file
