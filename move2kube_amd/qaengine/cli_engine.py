"""Interactive terminal engine (reference ``internal/qaengine/cliengine.go``).

On a terminal (stdin and stdout both TTYs) the questions are asked with the
survey-style raw-mode prompts of :mod:`.survey` - arrow-key Select and
MultiSelect with filtering, Confirm, Input, Multiline, masked Password - as
the reference does through AlecAivazis/survey.  When either side is not a
terminal (a pipe, a script; survey itself fails there) or ``M2K_QA_PLAIN=1``,
the same prompt text (``"<id>. <desc> \\nHints: \\n <context>\\n"``) is
printed with numbered options and answers are read line by line.
"""

import getpass
import os
import sys

from ..models import qa
from ..utils import log
from ..utils.gotemplate import go_sprint
from .engine import Engine


class CliEngine(Engine):
    go_type = "*qaengine.CliEngine"
    interactive = True  # may block on a person: the write cache is flushed first

    def __init__(self, stdin=None, stdout=None):
        self.stdin = stdin
        self.stdout = stdout

    @property
    def _in(self):
        return self.stdin or sys.stdin

    @property
    def _out(self):
        return self.stdout or sys.stdout

    def _message(self, prob):
        return "%d. %s \nHints: \n %s\n" % (prob.id, prob.desc, go_sprint(prob.context))

    def _readline(self):
        line = self._in.readline()
        if line == "":
            raise EOFError("end of input while answering a question")
        return line.rstrip("\n")

    def _write(self, s):
        self._out.write(s)
        self._out.flush()

    def _terminal(self):
        """A :class:`survey.Terminal` when both ends are TTYs, else None."""
        if os.environ.get("M2K_QA_PLAIN", "") not in ("", "0"):
            return None
        try:
            if not (os.isatty(self._in.fileno()) and os.isatty(self._out.fileno())):
                return None
        except (AttributeError, OSError, ValueError):
            return None
        from .survey import Terminal
        return Terminal(self._in, self._out)

    def fetch_answer(self, prob):
        term = self._terminal()
        if term is not None:
            return self._fetch_survey(term, prob)
        t = prob.type
        try:
            if t == qa.SELECT:
                return self._select(prob)
            if t == qa.MULTISELECT:
                return self._multiselect(prob)
            if t == qa.CONFIRM:
                return self._confirm(prob)
            if t == qa.INPUT:
                return self._input(prob)
            if t == qa.MULTILINE:
                return self._multiline(prob)
            if t == qa.PASSWORD:
                return self._password(prob)
        except EOFError as e:
            log.fatal("Error while asking a question : %s", e)
        log.fatal("Unknown type found: %s", t)

    def _fetch_survey(self, term, prob):
        """cliengine.go:38-197 with the survey-style prompts."""
        from . import survey
        msg = self._message(prob)
        t = prob.type
        try:
            if t == qa.SELECT:
                d = prob.default[0] if prob.default else prob.options[0]
                ans = [survey.select(term, msg, list(prob.options), d)]
            elif t == qa.MULTISELECT:
                ans = survey.multi_select(term, msg, list(prob.options), list(prob.default))
            elif t == qa.CONFIRM:
                d = False
                if prob.default:
                    try:
                        from ..utils.common import cast_to_bool
                        d = cast_to_bool(prob.default[0])
                    except ValueError as e:
                        log.warning("Unable to parse default value : %s", e)
                ans = ["true" if survey.confirm(term, msg, d) else "false"]
            elif t == qa.INPUT:
                ans = [survey.input_line(term, msg, prob.default[0] if prob.default else "")]
            elif t == qa.MULTILINE:
                ans = [survey.multiline(term, msg, prob.default[0] if prob.default else "")]
            elif t == qa.PASSWORD:
                ans = [survey.password(term, msg)]
            else:
                log.fatal("Unknown type found: %s", t)
        except (survey.Interrupt, EOFError, ValueError) as e:
            log.fatal("Error while asking a question : %s", e)
        prob.set_answer(ans)
        return prob

    def _select(self, prob):
        d = prob.default[0] if prob.default else prob.options[0]
        self._write("? " + self._message(prob))
        for i, o in enumerate(prob.options, 1):
            self._write("  %s%d) %s\n" % (">" if o == d else " ", i, o))
        while True:
            self._write("  [default: %s] > " % d)
            a = self._readline().strip()
            if a == "":
                a = d
            elif a.isdigit() and 1 <= int(a) <= len(prob.options):
                a = prob.options[int(a) - 1]
            try:
                prob.set_answer([a])
                return prob
            except qa.ProblemError as e:
                self._write("  invalid answer: %s\n" % e)

    def _multiselect(self, prob):
        self._write("? " + self._message(prob))
        for i, o in enumerate(prob.options, 1):
            self._write("  [%s] %d) %s\n" % ("✓" if o in prob.default else " ", i, o))
        while True:
            self._write("  comma separated numbers/names, '-' for none [default: %s] > " % ", ".join(prob.default))
            a = self._readline().strip()
            if a == "":
                ans = list(prob.default)
            elif a == "-":
                ans = []
            else:
                ans = []
                for tok in a.split(","):
                    tok = tok.strip()
                    if tok.isdigit() and 1 <= int(tok) <= len(prob.options):
                        ans.append(prob.options[int(tok) - 1])
                    elif tok:
                        ans.append(tok)
            try:
                prob.set_answer(ans)
                return prob
            except qa.ProblemError as e:
                self._write("  invalid answer: %s\n" % e)

    def _confirm(self, prob):
        d = False
        if prob.default:
            try:
                from ..utils.common import cast_to_bool
                d = cast_to_bool(prob.default[0])
            except ValueError as e:
                log.warning("Unable to parse default value : %s", e)
        self._write("? " + self._message(prob) + ("  (Y/n) > " if d else "  (y/N) > "))
        a = self._readline().strip().lower()
        val = d if a == "" else a in ("y", "yes", "true", "t", "1")
        prob.set_answer(["true" if val else "false"])
        return prob

    def _input(self, prob):
        d = prob.default[0] if prob.default else ""
        self._write("? " + self._message(prob) + "  (%s) > " % d)
        a = self._readline()
        prob.set_answer([a if a != "" else d])
        return prob

    def _multiline(self, prob):
        d = prob.default[0] if prob.default else ""
        self._write("? " + self._message(prob) + "  (end with an empty line; empty input keeps the default)\n")
        lines = []
        while True:
            line = self._readline()
            if line == "":
                break
            lines.append(line)
        prob.set_answer(["\n".join(lines) if lines else d])
        return prob

    def _password(self, prob):
        msg = "? " + self._message(prob) + "  > "
        if self._in is sys.stdin and sys.stdin.isatty():
            a = getpass.getpass(msg)
        else:
            self._write(msg)
            a = self._readline()
        prob.set_answer([a])
        return prob
