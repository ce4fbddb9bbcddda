"""Interactive terminal engine (reference ``internal/qaengine/cliengine.go``).

The reference uses AlecAivazis/survey prompts; this engine renders the same
prompt text (``"<id>. <desc> \\nHints: \\n <context>\\n"``) with numbered
options on plain stdin/stdout, so it also works when scripted through a pipe.
"""

import getpass
import sys

from ..models import qa
from ..utils import log
from ..utils.gotemplate import go_sprint
from .engine import Engine


class CliEngine(Engine):
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

    def fetch_answer(self, prob):
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
