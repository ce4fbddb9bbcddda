"""Default engine (``--qaskip``): answers every problem with its default
(reference ``internal/qaengine/defaultengine.go``)."""

from .engine import Engine


class DefaultEngine(Engine):
    def fetch_answer(self, prob):
        prob.set_answer(prob.default)
        return prob
