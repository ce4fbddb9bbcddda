"""The survey-style terminal prompts of the CLI QA engine (reference
``internal/qaengine/cliengine.go`` on AlecAivazis/survey v2.2.3), driven
through a pseudo-terminal: keystrokes go in on the master side and the bytes
written back are replayed on a small VT100 screen model, so the assertions
are about what a user sees after survey-style redraws (prompt erased and
replaced by the answer), and about the answers."""

import os
import pty
import re
import threading
import tty

import pytest

from move2kube_amd.models import qa
from move2kube_amd.qaengine import survey
from move2kube_amd.qaengine.cli_engine import CliEngine
from move2kube_amd.utils import log

UP, DOWN, RIGHT, LEFT = "\x1b[A", "\x1b[B", "\x1b[C", "\x1b[D"

_CSI = re.compile(r"\x1b\[(\??)(\d*)(?:;(\d+))*([A-Za-z])")


class Screen:
    """Just enough of a VT100 for survey's output: text, CR/LF, cursor
    up/down/back/forward/column, erase line, SGR and cursor visibility."""

    def __init__(self):
        self.lines = [""]
        self.row = 0
        self.col = 0

    def _put(self, ch):
        line = self.lines[self.row].ljust(self.col)
        self.lines[self.row] = line[:self.col] + ch + line[self.col + 1:]
        self.col += 1

    def feed(self, data):
        i = 0
        while i < len(data):
            m = _CSI.match(data, i)
            if m:
                priv, n, _rest, cmd = m.groups()
                n = int(n) if n else None
                if not priv:
                    if cmd == "G":
                        self.col = max((n or 1) - 1, 0)
                    elif cmd == "K":
                        line = self.lines[self.row]
                        if n == 2:
                            self.lines[self.row] = ""
                        elif n == 1:
                            self.lines[self.row] = " " * self.col + line[self.col:]
                        else:
                            self.lines[self.row] = line[:self.col]
                    elif cmd == "F":
                        self.row = max(self.row - (n or 1), 0)
                        self.col = 0
                    elif cmd == "E":
                        self.row += n or 1
                        self.col = 0
                        while len(self.lines) <= self.row:
                            self.lines.append("")
                    elif cmd == "D":
                        self.col = max(self.col - (n or 1), 0)
                    elif cmd == "C":
                        self.col += n or 1
                i = m.end()
                continue
            ch = data[i]
            if ch == "\r":
                self.col = 0
            elif ch == "\n":
                self.row += 1
                self.col = 0
                while len(self.lines) <= self.row:
                    self.lines.append("")
            else:
                self._put(ch)
            i += 1

    def text(self):
        return "\n".join(line.rstrip() for line in self.lines).rstrip("\n")


class Pty:
    def __init__(self):
        self.master, self.slave = pty.openpty()
        tty.setraw(self.slave)
        os.set_blocking(self.master, True)
        self.fin = open(self.slave, "rb", buffering=0, closefd=False)
        self.fout = open(self.slave, "w", encoding="utf-8", closefd=False)
        self.out = []
        self._t = threading.Thread(target=self._drain, daemon=True)
        self._t.start()

    def _drain(self):
        while True:
            try:
                data = os.read(self.master, 4096)
            except OSError:
                return
            if not data:
                return
            self.out.append(data)

    def keys(self, *chunks):
        for c in chunks:
            os.write(self.master, c.encode())

    def _settle(self):
        """Wait until the drained output stops growing (the prompt has returned)."""
        import select
        import time
        n, stable = -1, 0
        while stable < 3:
            time.sleep(0.02)
            pending = select.select([self.master], [], [], 0)[0]
            m = sum(len(x) for x in self.out)
            stable = stable + 1 if (m == n and not pending) else 0
            n = m

    def screen(self):
        self._settle()
        s = Screen()
        s.feed(b"".join(self.out).decode("utf-8", "replace"))
        return s

    def wait_for(self, text, timeout=30.0):
        """The screen once ``text`` appears on it (a prompt thread renders)
        and the output has settled."""
        import time
        end = time.time() + timeout
        while True:
            s = Screen()
            s.feed(b"".join(self.out).decode("utf-8", "replace"))
            if text in s.text():
                self._settle()
                s = Screen()
                s.feed(b"".join(self.out).decode("utf-8", "replace"))
                return s
            assert time.time() < end, "timed out waiting for %r; screen:\n%s" % (text, s.text())
            time.sleep(0.02)

    def raw_output(self):
        self._settle()
        return b"".join(self.out).decode("utf-8", "replace")

    def close(self):
        # slave side first: the drain thread's read then fails and it exits
        # before the master's fd number can be reused by the next test's pty
        self.fin.close()
        self.fout.close()
        os.close(self.slave)
        self._t.join(10)
        os.close(self.master)


@pytest.fixture
def term():
    p = Pty()
    yield p
    p.close()


def _t(p):
    return survey.Terminal(p.fin, p.fout)


MSG = "1. Select the thing: \nHints: \n [pick one]\n"


def test_select_arrows_and_answer_line(term):
    term.keys(DOWN, DOWN, UP, "\r")
    assert survey.select(_t(term), MSG, ["alpha", "beta", "gamma"], "alpha") == "beta"
    assert term.screen().text() == "? 1. Select the thing:\nHints:\n [pick one]\n beta"
    raw = term.raw_output()
    assert "\x1b[1;92m?" in raw and "\x1b[36m[Use arrows to move, type to filter]" in raw
    assert "\x1b[1;36m> " in raw and "\x1b[?25l" in raw and "\x1b[?25h" in raw


def test_select_default_filter_and_wraparound(term):
    term.keys("\r")
    assert survey.select(_t(term), MSG, ["alpha", "beta", "gamma"], "gamma") == "gamma"
    term.out.clear()
    term.keys(UP, "\r")  # wraps from the top to the bottom
    assert survey.select(_t(term), MSG, ["alpha", "beta", "gamma"], "alpha") == "gamma"
    term.out.clear()
    term.keys("gam", "\r")
    assert survey.select(_t(term), MSG, ["alpha", "beta", "gamma"], "alpha") == "gamma"
    term.out.clear()
    term.keys("zz", "\x7f\x7f", "et", "\r")  # backspace clears the filter
    assert survey.select(_t(term), MSG, ["alpha", "beta", "gamma"], "alpha") == "beta"


def _background(fn):
    import time
    res = {}
    t = threading.Thread(target=lambda: res.setdefault("v", fn()), daemon=True)
    t.start()
    time.sleep(0.05)
    return t, res


def test_select_pages_seven_options_around_the_cursor(term):
    opts = ["opt%02d" % i for i in range(12)]
    term.keys(*([DOWN] * 9))
    t, res = _background(lambda: survey.select(_t(term), MSG, opts, opts[0]))
    shown = term.wait_for("> opt09").text().splitlines()
    assert shown[3] == "  [Use arrows to move, type to filter]"
    # survey paginate: the last half page shows opt05..opt11 with the cursor on opt09
    assert shown[4:] == ["  opt05", "  opt06", "  opt07", "  opt08", "> opt09", "  opt10", "  opt11"]
    term.keys("\r")
    t.join(5)
    assert res["v"] == "opt09"


def test_multiselect_space_right_left_and_marks(term):
    term.keys(" ", DOWN, DOWN, " ", "\r")
    got = survey.multi_select(_t(term), MSG, ["a", "b", "c"], ["b"])
    assert got == ["a", "b", "c"]
    assert term.screen().text().endswith(" a, b, c")
    term.out.clear()
    term.keys(LEFT, "\r")
    assert survey.multi_select(_t(term), MSG, ["a", "b", "c"], ["a", "c"]) == []
    term.out.clear()
    term.keys("b", RIGHT, "\r")  # right marks every filtered option
    assert survey.multi_select(_t(term), MSG, ["ab", "bc", "cd"], []) == ["ab", "bc"]


def test_multiselect_renders_reference_marks(term):
    t, res = _background(lambda: survey.multi_select(_t(term), MSG, ["x", "y"], ["y"]))
    lines = term.wait_for("[✓]  y").text().splitlines()
    assert lines[3] == "  [Use arrows to move, space to select, <right> to all, <left> to none, type to filter]"
    assert lines[4:] == ["> [ ]  x", "  [✓]  y"]
    term.keys("\r")
    t.join(5)
    assert res["v"] == ["y"]


def test_confirm_default_yes_no_and_invalid(term):
    term.keys("\r")
    assert survey.confirm(_t(term), MSG, True) is True
    assert term.screen().text().endswith(" Yes")
    term.out.clear()
    term.keys("maybe\r", "N\r")
    assert survey.confirm(_t(term), MSG, True) is False
    raw = term.raw_output()
    assert 'Sorry, your reply was invalid: "maybe" is not a valid answer, please try again.' in raw
    assert "(Y/n) " in raw


def test_input_editing_and_default(term):
    term.keys("helo", LEFT, "l", "\x1b[F", "!", "\r")
    assert survey.input_line(_t(term), MSG, "dflt") == "hello!"
    assert term.screen().text().endswith(" hello!")
    term.out.clear()
    term.keys("\r")
    assert survey.input_line(_t(term), MSG, "dflt") == "dflt"
    assert "(dflt) " in term.raw_output()


def test_password_is_masked(term):
    term.keys("s3cr3t\r")
    assert survey.password(_t(term), MSG) == "s3cr3t"
    raw = term.raw_output()
    assert "s3cr3t" not in raw and "******" in raw


def test_multiline_two_empty_lines(term):
    term.keys("line one\r", "line two\r", "\r", "\r")
    assert survey.multiline(_t(term), MSG, "") == "line one\nline two"
    assert "[Enter 2 empty lines to finish]" in term.raw_output()


def test_interrupt(term):
    term.keys("\x03")
    with pytest.raises(survey.Interrupt):
        survey.select(_t(term), MSG, ["a"], "a")


def test_cli_engine_uses_the_tty_prompts(term, monkeypatch):
    monkeypatch.delenv("M2K_QA_PLAIN", raising=False)
    eng = CliEngine(stdin=term.fin, stdout=term.fout)
    prob = qa.new_select_problem("Choose the cluster type:", ["pick one"], "Kubernetes",
                                 ["Kubernetes", "Openshift", "AWS-EKS"])
    term.keys(DOWN, "\r")
    out = eng.fetch_answer(prob)
    assert out.answer == ["Openshift"] and out.resolved
    prob = qa.new_confirm_problem("Enable it?", ["hint"], False)
    term.keys("y\r")
    assert eng.fetch_answer(prob).answer == ["true"]
    prob = qa.new_select_problem("Choose:", [], "a", ["a", "b"])
    term.keys("\x03")
    with pytest.raises(log.FatalError):
        eng.fetch_answer(prob)


def test_cli_engine_plain_mode_without_a_tty(monkeypatch):
    import io
    eng = CliEngine(stdin=io.StringIO("2\n"), stdout=io.StringIO())
    prob = qa.new_select_problem("Choose:", [], "a", ["a", "b"])
    assert eng.fetch_answer(prob).answer == ["b"]


def test_color_codes_like_mgutz_ansi():
    assert survey.color_code("green+hb") == "\x1b[1;92m"
    assert survey.color_code("default+hb") == "\x1b[1;99m"
    assert survey.color_code("cyan") == "\x1b[36m"
    assert survey.color_code("cyan+b") == "\x1b[1;36m"
    assert survey.color_code("reset") == "\x1b[0m"
    assert survey.color_code("red:white") == "\x1b[31;47m"


def test_paginate_like_survey():
    ch = list(range(10))
    assert survey.paginate(7, ch, 0) == ([0, 1, 2, 3, 4, 5, 6], 0)
    assert survey.paginate(7, ch, 5) == ([2, 3, 4, 5, 6, 7, 8], 3)
    assert survey.paginate(7, ch, 9) == ([3, 4, 5, 6, 7, 8, 9], 6)
    assert survey.paginate(7, [1, 2], 1) == ([1, 2], 1)


def test_cli_engine_every_tty_prompt_type(term, monkeypatch, capsys):
    """cliengine.go:38-197: each problem type through its survey prompt; a
    confirm default that strconv.ParseBool refuses is warned about and read
    as false."""
    monkeypatch.delenv("M2K_QA_PLAIN", raising=False)
    eng = CliEngine(stdin=term.fin, stdout=term.fout)
    prob = qa.new_multiselect_problem("Pick services:", ["hint"], ["a"], ["a", "b", "c"])
    term.keys(DOWN, " ", "\r")
    assert eng.fetch_answer(prob).answer == ["a", "b"]
    prob = qa.new_input_problem("Name:", ["hint"], "dflt")
    term.keys("\r")
    assert eng.fetch_answer(prob).answer == ["dflt"]
    prob = qa.new_multiline_input_problem("Text:", ["hint"], "")
    term.keys("x\r", "\r", "\r")
    assert eng.fetch_answer(prob).answer == ["x"]
    prob = qa.new_password_problem("Password:", ["hint"])
    term.keys("pw\r")
    assert eng.fetch_answer(prob).answer == ["pw"]
    prob = qa.new_confirm_problem("Sure?", ["hint"], False)
    prob.default = ["maybe"]
    term.keys("\r")
    assert eng.fetch_answer(prob).answer == ["false"]
    import logparse
    assert logparse.logged(capsys.readouterr().err, 'Unable to parse default value : strconv.ParseBool: parsing '
                           '"maybe": invalid syntax', "warning")
    prob = qa.new_input_problem("Odd:", [], "")
    prob.type = "Unknown"
    with pytest.raises(log.FatalError):
        eng.fetch_answer(prob)


def _plain(monkeypatch, text):
    import io
    monkeypatch.delenv("M2K_QA_PLAIN", raising=False)
    out = io.StringIO()
    return CliEngine(stdin=io.StringIO(text), stdout=out), out


def test_plain_select_retries_an_unknown_answer(monkeypatch):
    eng, out = _plain(monkeypatch, "nope\n\n")
    prob = qa.new_select_problem("Choose:", ["ctx"], "b", ["a", "b"])
    assert eng.fetch_answer(prob).answer == ["b"]
    text = out.getvalue()
    assert text.startswith("? %d. Choose: \nHints: \n [ctx]\n   1) a\n  >2) b\n" % prob.id)
    assert "  invalid answer: Unknown options selected\n" in text


@pytest.mark.parametrize("typed,want", [
    ("\n", ["a"]), ("-\n", []), ("2, c\n", ["b", "c"]), ("1,,3\n", ["a", "c"]),
    ("9\nb\n", ["b"]),                      # out of range is a name, and no option has it: asked again
])
def test_plain_multiselect(monkeypatch, typed, want):
    eng, out = _plain(monkeypatch, typed)
    prob = qa.new_multiselect_problem("Pick:", [], ["a"], ["a", "b", "c"])
    assert eng.fetch_answer(prob).answer == want
    assert "  [✓] 1) a\n  [ ] 2) b\n" in out.getvalue()


def test_plain_confirm_input_multiline_password(monkeypatch, capsys):
    eng, out = _plain(monkeypatch, "yes\n\nfirst\nsecond\n\nsecret\n")
    c = qa.new_confirm_problem("Sure?", [], False)
    assert eng.fetch_answer(c).answer == ["true"] and "(y/N) > " in out.getvalue()
    i = qa.new_input_problem("Name:", [], "dflt")
    assert eng.fetch_answer(i).answer == ["dflt"] and "(dflt) > " in out.getvalue()
    m = qa.new_multiline_input_problem("Text:", [], "keep")
    assert eng.fetch_answer(m).answer == ["first\nsecond"]
    p = qa.new_password_problem("Password:", [])
    assert eng.fetch_answer(p).answer == ["secret"]
    eng, out = _plain(monkeypatch, "\n\n")
    m = qa.new_multiline_input_problem("Text:", [], "keep")
    assert eng.fetch_answer(m).answer == ["keep"]
    c = qa.new_confirm_problem("Sure?", [], True)
    c.default = ["sometimes"]
    assert eng.fetch_answer(c).answer == ["false"] and "(y/N) > " in out.getvalue()
    assert "Unable to parse default value : " in capsys.readouterr().err


def test_plain_end_of_input_and_unknown_type_are_fatal(monkeypatch):
    eng, _ = _plain(monkeypatch, "")
    with pytest.raises(log.FatalError):
        eng.fetch_answer(qa.new_input_problem("Name:", [], "d"))
    eng, _ = _plain(monkeypatch, "x\n")
    prob = qa.new_input_problem("Odd:", [], "")
    prob.type = "Unknown"
    with pytest.raises(log.FatalError):
        eng.fetch_answer(prob)


def test_plain_mode_forced_on_a_tty(term, monkeypatch):
    monkeypatch.setenv("M2K_QA_PLAIN", "1")
    eng = CliEngine(stdin=term.fin, stdout=term.fout)
    assert eng._terminal() is None
