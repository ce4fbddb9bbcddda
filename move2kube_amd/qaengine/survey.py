"""Terminal prompts in the manner of AlecAivazis/survey v2.2.3, the library the
reference's CLI engine drives (``internal/qaengine/cliengine.go``;
``go.mod:8``): Select, MultiSelect, Confirm, Input, Multiline and Password on
a raw-mode TTY.

What is reproduced: the prompt layout (``? <message>`` in bold, the cyan
``[Use arrows to move, type to filter]`` hint, ``>`` on the focused option,
``[✓]``/``[ ]`` marks - the reference overrides survey's ``[x]`` - and the
cyan answer that replaces the prompt when it is done), pagination of 7
options around the cursor, the key bindings (arrows and Tab, type to filter,
Backspace / Ctrl-W / Ctrl-U on the filter, Space to toggle, Right / Left to
mark / unmark every filtered option, Esc for vim ``j``/``k``, Ctrl-C as an
interrupt, Ctrl-D as Enter), line editing for the text prompts, ``*`` masking
for passwords, the Confirm re-prompt with ``Sorry, your reply was invalid``,
and survey's redraw strategy (erase the lines it rendered last time,
wrap-aware).  Colours are mgutz/ansi codes.  The exact byte stream of cursor
movements is not pinned (the Go library is not available here: "parity
unpinned").
"""

import os

# survey/terminal key codes (runes after escape-sequence decoding)
KEY_ARROW_LEFT = "\x02"
KEY_ARROW_RIGHT = "\x06"
KEY_ARROW_UP = "\x10"
KEY_ARROW_DOWN = "\x0e"
KEY_SPACE = " "
KEY_BACKSPACE = "\b"
KEY_DELETE = "\x7f"
KEY_INTERRUPT = "\x03"
KEY_END_TRANSMISSION = "\x04"
KEY_ESCAPE = "\x1b"
KEY_DELETE_WORD = "\x17"
KEY_DELETE_LINE = "\x18"
KEY_TAB = "\t"
KEY_ENTER = "\r"
SPECIAL_KEY_HOME = "\x01"
SPECIAL_KEY_END = "\x11"
SPECIAL_KEY_DELETE = "\x12"
IGNORE_KEY = "\x00"

PAGE_SIZE = 7
HELP_INPUT = "?"
DEFAULT_TERM_WIDTH = 80


class Interrupt(Exception):
    """``terminal.InterruptErr``."""

    def __init__(self):
        super().__init__("interrupt")


# -- mgutz/ansi ---------------------------------------------------------------

_COLORS = {"black": 0, "red": 1, "green": 2, "yellow": 3, "blue": 4, "magenta": 5, "cyan": 6, "white": 7,
           "default": 9}


def color_code(style):
    """``ansi.ColorCode(style)``: ``"green+hb"`` -> ``"\\x1b[1;92m"``."""
    if style == "":
        return ""
    if style == "reset":
        return "\x1b[0m"
    fg, _, bg = style.partition(":")
    fg_key, _, fg_style = fg.partition("+")
    parts = []
    base = 30
    for flag, code in (("b", "1"), ("B", "5"), ("u", "4"), ("i", "7"), ("s", "9")):
        if flag in fg_style:
            parts.append(code)
    if "h" in fg_style:
        base = 90
    if fg_key.isdigit():
        parts.append("38;5;%s" % fg_key)
    elif fg_key in _COLORS:
        parts.append(str(base + _COLORS[fg_key]))
    if bg:
        bg_key, _, bg_style = bg.partition("+")
        if bg_key.isdigit():
            parts.append("48;5;%s" % bg_key)
        elif bg_key in _COLORS:
            parts.append(str((100 if "h" in bg_style else 40) + _COLORS[bg_key]))
    return "\x1b[" + ";".join(parts) + "m" if parts else ""


def _no_color(_style):
    return ""


# icons of survey's default IconSet, MarkedOption as cliengine.go:92-94 sets it
ICON_QUESTION = ("?", "green+hb")
ICON_HELP = ("?", "cyan")
ICON_ERROR = ("X", "red")
ICON_FOCUS = (">", "cyan+b")
ICON_MARKED = ("[✓]", "green")
ICON_UNMARKED = ("[ ]", "default+hb")


# -- terminal -------------------------------------------------------------------

class Terminal:
    """Raw-mode reads from ``fin`` and writes to ``fout`` (file objects on a TTY)."""

    def __init__(self, fin, fout):
        self.fin = fin
        self.fout = fout
        self.fd = fin.fileno()
        self._buf = b""
        self._saved = None

    # survey's RuneReader.SetTermMode: no echo, no canonical mode, no signals
    def set_raw(self):
        import termios
        self._saved = termios.tcgetattr(self.fd)
        new = termios.tcgetattr(self.fd)
        new[3] &= ~(termios.ECHO | termios.ECHONL | termios.ICANON | termios.ISIG)
        new[6][termios.VMIN] = 1
        new[6][termios.VTIME] = 0
        termios.tcsetattr(self.fd, termios.TCSANOW, new)

    def restore(self):
        if self._saved is not None:
            import termios
            termios.tcsetattr(self.fd, termios.TCSANOW, self._saved)
            self._saved = None

    def write(self, s):
        self.fout.write(s)
        self.fout.flush()

    def width(self):
        try:
            w = os.get_terminal_size(self.fout.fileno()).columns
        except (OSError, ValueError, AttributeError):
            w = 0
        return w or DEFAULT_TERM_WIDTH

    def _fill(self):
        data = os.read(self.fd, 1024)
        if not data:
            raise EOFError("EOF")
        self._buf += data

    def _byte(self):
        if not self._buf:
            self._fill()
        b, self._buf = self._buf[:1], self._buf[1:]
        return b

    def read_rune(self):
        """One key: a character, or a key code for an escape sequence."""
        b = self._byte()
        if b == b"\x1b":
            if not self._buf:  # nothing buffered after it: the Esc key itself
                return KEY_ESCAPE
            nxt = self._byte()
            if nxt != b"[":
                return IGNORE_KEY
            c = self._byte()
            keys = {b"D": KEY_ARROW_LEFT, b"C": KEY_ARROW_RIGHT, b"A": KEY_ARROW_UP, b"B": KEY_ARROW_DOWN,
                    b"H": SPECIAL_KEY_HOME, b"F": SPECIAL_KEY_END}
            if c in keys:
                return keys[c]
            if self._buf[:1] == b"~":  # ESC [ 3 ~ (Delete) and other tilde keys
                self._buf = self._buf[1:]
            return SPECIAL_KEY_DELETE if c == b"3" else IGNORE_KEY
        n = 1
        if b[0] >= 0xF0:
            n = 4
        elif b[0] >= 0xE0:
            n = 3
        elif b[0] >= 0xC0:
            n = 2
        while n > 1 and len(b) < n:
            b += self._byte()
        return b.decode("utf-8", "replace")

    # survey/terminal cursor and erase sequences
    def cursor_hide(self):
        self.write("\x1b[?25l")

    def cursor_show(self):
        self.write("\x1b[?25h")

    def back(self, n):
        if n > 0:
            self.write("\x1b[%dD" % n)

    def forward(self, n):
        if n > 0:
            self.write("\x1b[%dC" % n)

    def previous_line(self, n):
        self.write("\x1b[%dF" % n)

    def next_line(self, n):
        self.write("\x1b[%dE" % n)

    def erase_line(self, mode):
        self.write("\x1b[%dK" % mode)

    def read_line(self, mask=""):
        """``RuneReader.ReadLine``: echoed (or masked) line editing until Enter."""
        line, index = [], 0
        while True:
            r = self.read_rune()
            if r in ("\r", "\n", KEY_END_TRANSMISSION):
                self.write("\r\n")
                return "".join(line)
            if r == KEY_INTERRUPT:
                self.write("\r\n")
                raise Interrupt()
            if r in (KEY_BACKSPACE, KEY_DELETE):
                if index > 0 and line:
                    del line[index - 1]
                    index -= 1
                    self.back(1)
                    self.erase_line(0)
                    rest = line[index:]
                    if rest:
                        self.write("".join(mask * len(rest) if mask else rest))
                        self.back(len(rest))
                continue
            if r == SPECIAL_KEY_DELETE:
                if index < len(line):
                    del line[index]
                    self.erase_line(0)
                    rest = line[index:]
                    if rest:
                        self.write("".join(mask * len(rest) if mask else rest))
                        self.back(len(rest))
                continue
            if r == KEY_ARROW_LEFT:
                if index > 0:
                    self.back(1)
                    index -= 1
                continue
            if r == KEY_ARROW_RIGHT:
                if index < len(line):
                    self.forward(1)
                    index += 1
                continue
            if r == SPECIAL_KEY_HOME:
                self.back(index)
                index = 0
                continue
            if r == SPECIAL_KEY_END:
                self.forward(len(line) - index)
                index = len(line)
                continue
            if r == IGNORE_KEY or (len(r) == 1 and (ord(r) < 32 or ord(r) == 127)):
                continue
            line.insert(index, r)
            index += 1
            rest = line[index:]
            self.write(mask if mask else r)
            if rest:
                self.write("".join(mask * len(rest) if mask else rest))
                self.back(len(rest))


class Renderer:
    """survey's Renderer: remembers what it drew (without colours) so the next
    render first erases exactly those lines, counting wrapped ones."""

    def __init__(self, term):
        self.term = term
        self.rendered = ""
        self.rendered_errors = ""

    def count_lines(self, text):
        w = self.term.width()
        count, curr = 0, 0
        while curr < len(text):
            rel = text.find("\n", curr)
            if rel != -1:
                count += 1
                end = rel
            else:
                end = len(text)
            width = len(text[curr:end])
            if width > w:
                count += width // w
                if width % w == 0:
                    count -= 1
            curr = end + 1
        return count

    def reset_prompt(self, lines):
        t = self.term
        t.write("\x1b[0G")
        t.erase_line(2)
        for _ in range(lines):
            t.previous_line(1)
            t.erase_line(2)

    def render(self, template, data):
        self.reset_prompt(self.count_lines(self.rendered))
        self.term.write(template(data, color_code))
        self.rendered = template(data, _no_color)

    def error(self, message):
        self.reset_prompt(self.count_lines(self.rendered_errors))
        self.rendered_errors = ""
        self.reset_prompt(self.count_lines(self.rendered))
        self.rendered = ""

        def tmpl(_d, c):
            return "%s%s Sorry, your reply was invalid: %s%s\n" % (c(ICON_ERROR[1]), ICON_ERROR[0], message,
                                                                    c("reset"))
        self.term.write(tmpl(None, color_code))
        self.rendered_errors = tmpl(None, _no_color)


# -- templates ------------------------------------------------------------------

def _head(d, c):
    out = []
    if d.get("show_help"):
        out += [c(ICON_HELP[1]), ICON_HELP[0], " ", d["help"], c("reset"), "\n"]
    out += [c(ICON_QUESTION[1]), ICON_QUESTION[0], " ", c("reset")]
    return out


def _select_template(d, c):
    out = _head(d, c)
    out += [c("default+hb"), d["message"], d.get("filter_message", ""), c("reset")]
    if d.get("show_answer"):
        out += [c("cyan"), " ", d["answer"], c("reset"), "\n"]
        return "".join(out)
    more = ", %s for more help" % HELP_INPUT if d.get("help") and not d.get("show_help") else ""
    out += ["  ", c("cyan"), "[Use arrows to move, type to filter", more, "]", c("reset"), "\n"]
    for ix, (_idx, value) in enumerate(d["page"]):
        if ix == d["selected"]:
            out += [c(ICON_FOCUS[1]), ICON_FOCUS[0], " "]
        else:
            out += [c("default"), "  "]
        out += [value, c("reset"), "\n"]
    return "".join(out)


def _multiselect_template(d, c):
    out = _head(d, c)
    out += [c("default+hb"), d["message"], d.get("filter_message", ""), c("reset")]
    if d.get("show_answer"):
        out += [c("cyan"), " ", d["answer"], c("reset"), "\n"]
        return "".join(out)
    more = ", %s for more help" % HELP_INPUT if d.get("help") and not d.get("show_help") else ""
    out += ["  ", c("cyan"), "[Use arrows to move, space to select, <right> to all, <left> to none, type to filter",
            more, "]", c("reset"), "\n"]
    for ix, (idx, value) in enumerate(d["page"]):
        if ix == d["selected"]:
            out += [c(ICON_FOCUS[1]), ICON_FOCUS[0], c("reset")]
        else:
            out += [" "]
        icon = ICON_MARKED if d["checked"].get(idx) else ICON_UNMARKED
        out += [c(icon[1]), " ", icon[0], " ", c("reset"), " ", value, "\n"]
    return "".join(out)


def _line_prompt_template(d, c):
    """Input / Confirm / Password / Multiline share the head and the answer."""
    out = _head(d, c)
    out += [c("default+hb"), d["message"], " ", c("reset")]
    kind = d["kind"]
    if d.get("show_answer"):
        if kind == "multiline":
            out += ["\n", c("cyan"), d["answer"], c("reset")]
            if d["answer"]:
                out.append("\n")
        else:
            out += [c("cyan"), d["answer"], c("reset"), "\n"]
        return "".join(out)
    if kind != "multiline" and d.get("help") and not d.get("show_help"):
        out += [c("cyan"), "[", HELP_INPUT, " for help]", c("reset"), " "]
    if kind == "confirm":
        out += [c("white"), "(Y/n) " if d["default"] else "(y/N) ", c("reset")]
    elif kind in ("input", "multiline") and d.get("default"):
        out += [c("white"), "(", d["default"], ") ", c("reset")]
    if kind == "multiline":
        out += [c("cyan"), "[Enter 2 empty lines to finish]", c("reset")]
    return "".join(out)


def paginate(page_size, choices, sel):
    """survey ``paginate``: the visible window and the cursor inside it."""
    n = len(choices)
    if n < page_size:
        start, end, cursor = 0, n, sel
    elif sel < page_size // 2:
        start, end, cursor = 0, page_size, sel
    elif n - sel - 1 < page_size // 2:
        start, end = n - page_size, n
        cursor = sel - start
    else:
        above = page_size // 2
        start, end, cursor = sel - above, sel + page_size - above, above
    return choices[start:end], cursor


def _filtered(options, flt):
    """survey's DefaultFilterFn: ``strings.Contains(strings.ToLower(option),
    strings.ToLower(filter))``."""
    from ..utils.common import go_lower
    f = go_lower(flt)
    return [(i, o) for i, o in enumerate(options) if f in go_lower(o)]


# -- prompts --------------------------------------------------------------------

def select(term, message, options, default=None, help_text=""):
    if not options:
        raise ValueError("please provide options to select from")
    r = Renderer(term)
    sel = options.index(default) if default in options else 0
    flt, showing_help, vim, use_default = "", False, False, True

    def draw(opts, idx, **extra):
        page, cur = paginate(PAGE_SIZE, opts, idx)
        d = {"message": message, "help": help_text, "show_help": showing_help, "page": page, "selected": cur,
             "filter_message": " " + flt if flt else ""}
        d.update(extra)
        r.render(_select_template, d)

    draw(_filtered(options, ""), sel)
    term.set_raw()
    term.cursor_hide()
    try:
        while True:
            k = term.read_rune()
            if k == KEY_INTERRUPT:
                raise Interrupt()
            if k == KEY_END_TRANSMISSION:
                break
            opts = _filtered(options, flt)
            old = flt
            if k in (KEY_ENTER, "\n"):
                if opts and sel < len(opts):
                    break
                continue
            if (k == KEY_ARROW_UP or (vim and k == "k")) and opts:
                use_default = False
                sel = len(opts) - 1 if sel == 0 else sel - 1
            elif (k in (KEY_TAB, KEY_ARROW_DOWN) or (vim and k == "j")) and opts:
                use_default = False
                sel = 0 if sel == len(opts) - 1 else sel + 1
            elif k == HELP_INPUT and help_text:
                showing_help = True
            elif k == KEY_ESCAPE:
                vim = not vim
            elif k in (KEY_DELETE_WORD, KEY_DELETE_LINE):
                flt = ""
            elif k in (KEY_DELETE, KEY_BACKSPACE):
                flt = flt[:-1]
            elif k >= KEY_SPACE and k not in (KEY_DELETE,):
                flt += k
                vim = False
                use_default = False
            if old != flt:
                opts = _filtered(options, flt)
                if opts and len(opts) <= sel:
                    sel = len(opts) - 1
            if use_default or sel >= len(opts):
                for j, (_i, o) in enumerate(opts):
                    if o == default:
                        sel = j
                        break
            draw(opts, sel)
        opts = _filtered(options, flt)
        if use_default or sel >= len(opts):
            val = default if default is not None else (opts[0][1] if opts else "")
        else:
            val = opts[sel][1]
    finally:
        term.restore()
        term.cursor_show()
    flt = ""
    draw([], 0, show_answer=True, answer=val)
    return val


def multi_select(term, message, options, defaults=(), help_text=""):
    if not options:
        raise ValueError("please provide options to select from")
    r = Renderer(term)
    checked = {}
    for dflt in defaults:
        if dflt in options:
            checked[options.index(dflt)] = True
    sel, flt, showing_help, vim = 0, "", False, False

    def draw(opts, idx, **extra):
        page, cur = paginate(PAGE_SIZE, opts, idx)
        d = {"message": message, "help": help_text, "show_help": showing_help, "page": page, "selected": cur,
             "checked": checked, "filter_message": " " + flt if flt else ""}
        d.update(extra)
        r.render(_multiselect_template, d)

    term.cursor_hide()
    draw(_filtered(options, ""), sel)
    term.set_raw()
    try:
        while True:
            k = term.read_rune()
            if k in (KEY_ENTER, "\n"):
                break
            if k == KEY_INTERRUPT:
                raise Interrupt()
            if k == KEY_END_TRANSMISSION:
                break
            opts = _filtered(options, flt)
            old = flt
            if k == KEY_ARROW_UP or (vim and k == "k"):
                sel = len(opts) - 1 if sel == 0 else sel - 1
            elif k in (KEY_TAB, KEY_ARROW_DOWN) or (vim and k == "j"):
                sel = 0 if sel == len(opts) - 1 else sel + 1
            elif k == KEY_SPACE:
                if sel < len(opts):
                    i = opts[sel][0]
                    checked[i] = not checked.get(i, False)
                    flt = ""
            elif k == HELP_INPUT and help_text:
                showing_help = True
            elif k == KEY_ESCAPE:
                vim = not vim
            elif k in (KEY_DELETE_WORD, KEY_DELETE_LINE):
                flt = ""
            elif k in (KEY_DELETE, KEY_BACKSPACE):
                flt = flt[:-1]
            elif k > KEY_SPACE:
                flt += k
                vim = False
            elif not vim and k == KEY_ARROW_RIGHT:
                for i, _o in opts:
                    checked[i] = True
                flt = ""
            elif not vim and k == KEY_ARROW_LEFT:
                for i, _o in opts:
                    checked[i] = False
                flt = ""
            if old != flt:
                opts = _filtered(options, flt)
                if opts and len(opts) <= sel:
                    sel = len(opts) - 1
            draw(opts, sel)
    finally:
        term.restore()
        term.cursor_show()
    answers = [o for i, o in enumerate(options) if checked.get(i)]
    flt = ""
    draw([], 0, show_answer=True, answer=", ".join(answers))
    return answers


_YES = ("y", "yes")
_NO = ("n", "no")


def confirm(term, message, default=False, help_text=""):
    r = Renderer(term)
    d = {"kind": "confirm", "message": message, "default": default, "help": help_text}
    r.render(_line_prompt_template, d)
    term.set_raw()
    try:
        while True:
            line = term.read_line()
            term.previous_line(1)  # compensate for the echoed newline
            low = line.lower()
            if low in _YES:
                ans = True
            elif low in _NO:
                ans = False
            elif line == "":
                ans = default
            elif line == HELP_INPUT and help_text:
                d["show_help"] = True
                r.render(_line_prompt_template, d)
                continue
            else:
                from ..utils.log import go_quote
                r.error("%s is not a valid answer, please try again." % go_quote(line))
                r.render(_line_prompt_template, d)
                continue
            break
    finally:
        term.restore()
    r.render(_line_prompt_template, dict(d, show_answer=True, answer="Yes" if ans else "No"))
    return ans


def input_line(term, message, default="", help_text=""):
    r = Renderer(term)
    d = {"kind": "input", "message": message, "default": default, "help": help_text}
    r.render(_line_prompt_template, d)
    term.set_raw()
    try:
        line = term.read_line()
        term.previous_line(1)
    finally:
        term.restore()
    ans = line if line != "" else default
    r.render(_line_prompt_template, dict(d, show_answer=True, answer=ans))
    return ans


def password(term, message, help_text=""):
    r = Renderer(term)
    d = {"kind": "password", "message": message, "help": help_text}
    r.render(_line_prompt_template, d)
    term.set_raw()
    try:
        return term.read_line(mask="*")
    finally:
        term.restore()


def multiline(term, message, default=""):
    r = Renderer(term)
    d = {"kind": "multiline", "message": message, "default": default}
    r.render(_line_prompt_template, d)
    term.set_raw()
    lines, empty_once = [], False
    try:
        while True:
            line = term.read_line()
            if line == "":
                if empty_once:
                    n = len(lines) + 2
                    term.previous_line(n)
                    for _ in range(n):
                        term.erase_line(2)
                        term.next_line(1)
                    term.previous_line(n)
                    break
                empty_once = True
            else:
                empty_once = False
            lines.append(line)
    finally:
        term.restore()
    val = "\n".join(lines).strip()
    ans = val if val else default
    r.render(_line_prompt_template, dict(d, show_answer=True, answer=ans))
    return ans
