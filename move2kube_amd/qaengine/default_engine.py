"""Default engine (``--qaskip``): answers every problem with its default
(reference ``internal/qaengine/defaultengine.go``).

A password problem has no default; the reference then retries the last
engine forever.  Here it is answered with an empty password instead."""

from ..models import qa
from .engine import Engine


class DefaultEngine(Engine):
    go_type = "*qaengine.DefaultEngine"
    def fetch_answer(self, prob):
        if prob.type == qa.PASSWORD and not prob.default:
            prob.set_answer([""])
            return prob
        prob.set_answer(prob.default)
        return prob
