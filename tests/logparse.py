"""Reading back the logger's lines in tests: ``time="..." level=info
msg="..."`` when stderr is not a terminal (as under pytest), the coloured
``INFO[0000] message`` layout on a terminal (``utils/log.py``)."""

import re

_KV = re.compile(r'time="[^"]*" level=(\w+)(?: msg=("(?:[^"\\]|\\.)*"|\S+))?$')
_TTY = re.compile(r"\x1b\[\d+m(\w{4})\x1b\[0m\[\d{4}\] (.*?) ?$")
_LEVELS = {"DEBU": "debug", "INFO": "info", "WARN": "warning", "ERRO": "error", "FATA": "fatal"}
_ESC = {"a": "\a", "b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v", "\\": "\\", '"': '"'}


def go_unquote(q):
    """strconv.Unquote of a double-quoted Go string."""
    s, out, i = q[1:-1], [], 0
    while i < len(s):
        c = s[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        e = s[i + 1]
        if e in _ESC:
            out.append(_ESC[e])
            i += 2
        elif e == "x":
            out.append(chr(int(s[i + 2:i + 4], 16)))
            i += 4
        elif e == "u":
            out.append(chr(int(s[i + 2:i + 6], 16)))
            i += 6
        elif e == "U":
            out.append(chr(int(s[i + 2:i + 10], 16)))
            i += 10
        else:
            raise ValueError("bad escape in %r" % q)
    return "".join(out)


def messages(text):
    """[(level, message)] of every log line in ``text`` (other lines skipped)."""
    out = []
    for line in text.splitlines():
        m = _KV.match(line)
        if m:
            msg = m.group(2) or ""
            out.append((m.group(1), go_unquote(msg) if msg.startswith('"') else msg))
            continue
        m = _TTY.match(line)
        if m:
            out.append((_LEVELS[m.group(1)], m.group(2).rstrip(" ")))
    return out


def logged(text, message, level=None):
    """Whether a line with exactly this message (and level) was logged."""
    return any(m == message and (level is None or lv == level) for lv, m in messages(text))


def logged_containing(text, part, level=None):
    return any(part in m and (level is None or lv == level) for lv, m in messages(text))
