"""Logging in the format of the reference's logger: logrus v1.7.0
(``go.mod:28``) with its default ``TextFormatter``, Info level, Debug with
``-v`` (``cmd/move2kube/move2kube.go:41-46``).

The formatter looks at its output once: on a terminal each line is
``\x1b[36mINFO\x1b[0m[0012] <message padded to 44 runes> `` (level colour,
seconds since start; one trailing newline of the message dropped), anywhere
else ``time="<RFC 3339 local time>" level=info msg=<message>`` with the
message ``%q``-quoted unless it only has letters, digits and ``-._/@^+``.
``fatal`` logs and raises :class:`FatalError` (the CLI turns it into exit
code 1) instead of calling ``os.Exit``, so the library works in-process.
"""

import sys
import threading
import time

_START = time.time()
DEBUG, INFO, WARNING, ERROR, CRITICAL = 10, 20, 30, 40, 50
_LEVEL_NAMES = {DEBUG: "DEBU", INFO: "INFO", WARNING: "WARN", ERROR: "ERRO", CRITICAL: "FATA"}
_LEVEL_WORDS = {DEBUG: "debug", INFO: "info", WARNING: "warning", ERROR: "error", CRITICAL: "fatal"}
_LEVEL_COLORS = {DEBUG: 37, INFO: 36, WARNING: 33, ERROR: 31, CRITICAL: 31}   # gray, blue, yellow, red
_BARE = frozenset("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-._/@^+")


_GO_ESC = {"\a": "\\a", "\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r", "\t": "\\t",
           "\v": "\\v", "\\": "\\\\", '"': '\\"'}


def go_quote(s):
    """``strconv.Quote``: what the reference's ``%q`` prints for a string.
    Bytes that were not UTF-8 (surrogateescape) come out as ``\\xNN``."""
    if s.isascii() and s.isprintable() and '"' not in s and "\\" not in s:
        return '"' + s + '"'
    out = ['"']
    for ch in s:
        e = _GO_ESC.get(ch)
        if e is not None:
            out.append(e)
            continue
        o = ord(ch)
        if 0xDC80 <= o <= 0xDCFF:
            out.append("\\x%02x" % (o - 0xDC00))
        elif o < 0x20 or o == 0x7F:
            out.append("\\x%02x" % o)
        elif ch.isprintable() or ch == " ":
            out.append(ch)
        elif o < 0x10000:
            out.append("\\u%04x" % o)
        else:
            out.append("\\U%08x" % o)
    out.append('"')
    return "".join(out)


class _GoQ(str):
    """A string argument of a ``%r`` in a log format: printed as Go's ``%q``
    (double quotes) rather than Python's repr; ``%s`` is unchanged."""

    __slots__ = ()

    def __repr__(self):
        return go_quote(self)


class _GoVal:
    """A slice or map argument: ``%s`` prints Go's ``%v`` (``[a b]``,
    ``map[k:v]``), ``%r`` Go's ``%q`` (``["a" "b"]``)."""

    __slots__ = ("v", "q")

    def __init__(self, a):
        from .gofmt import sprint_one
        self.v = sprint_one(a)
        if type(a) is list:
            self.q = "[" + " ".join(go_quote(x) if type(x) is str else sprint_one(x) for x in a) + "]"
        else:
            self.q = self.v

    def __str__(self):
        return self.v

    def __repr__(self):
        return self.q


def _format(msg, args):
    if any(type(a) in (list, dict) for a in args):
        args = tuple(_GoVal(a) if type(a) in (list, dict) else a for a in args)
    if "%r" in msg:
        args = tuple(_GoQ(a) if type(a) is str else a for a in args)
    return msg % args


class FatalError(RuntimeError):
    """Raised where the reference calls ``log.Fatalf``."""


_stamp = (None, "")  # (whole second, its RFC3339 text): a run logs many lines per second


def _rfc3339(t):
    """time.RFC3339 of a local time (logrus' default timestamp format)."""
    global _stamp
    sec = int(t)
    cached = _stamp   # one tuple, replaced whole: threads never see a torn pair
    if cached[0] == sec:
        return cached[1]
    text = _rfc3339_uncached(sec)
    _stamp = (sec, text)
    return text


def _rfc3339_uncached(t):
    lt = time.localtime(t)
    off = lt.tm_gmtoff
    stamp = time.strftime("%Y-%m-%dT%H:%M:%S", lt)
    if off == 0:
        return stamp + "Z"
    sign = "+" if off > 0 else "-"
    off = abs(off)
    return "%s%s%02d:%02d" % (stamp, sign, off // 3600, off % 3600 // 60)


def format_line(level, text, now, colored):
    """One logrus TextFormatter line."""
    if colored:
        if text.endswith("\n"):
            text = text[:-1]
        return "\x1b[%dm%s\x1b[0m[%04d] %-44s \n" % (_LEVEL_COLORS.get(level, 36), _LEVEL_NAMES.get(level, "INFO"),
                                                     int(now - _START), text)
    line = 'time="%s" level=%s' % (_rfc3339(now), _LEVEL_WORDS.get(level, "info"))
    if text:
        line += " msg=" + (text if _BARE.issuperset(text) else go_quote(text))
    return line + "\n"


class _Logger:
    """Minimal logrus-style logger on stderr.  The stdlib ``logging`` package
    is not imported: it is a measurable part of a cold CLI start and nothing
    here needs handlers or hierarchies."""

    def __init__(self):
        self.level = INFO
        self.stream = None  # None = the current sys.stderr
        self._lock = threading.Lock()
        self._tty_of = None   # the stream whose terminal check is cached
        self._tty = False

    def _colored(self, stream):
        """logrus checks once whether its output is a terminal; a process has
        one stderr, so the check is cached per stream object."""
        if stream is not self._tty_of:
            try:
                self._tty = stream.isatty()
            except (AttributeError, ValueError, OSError):
                self._tty = False
            self._tty_of = stream
        return self._tty

    def isEnabledFor(self, level):
        return level >= self.level

    def setLevel(self, level):
        self.level = level
        _rebind()

    def log(self, level, msg, *args):
        if level < self.level:
            return
        try:
            text = _format(msg, args) if args else msg
        except (TypeError, ValueError):
            text = "%s %r" % (msg, args)
        stream = self.stream or sys.stderr
        line = format_line(level, text, time.time(), self._colored(stream))
        held = getattr(_held, "lines", None)
        if held is not None:
            held.append(line)
            return
        with self._lock:
            stream.write(line)
            stream.flush()

    def debug(self, msg, *args):
        if DEBUG >= self.level:
            self.log(DEBUG, msg, *args)

    def info(self, msg, *args):
        if INFO >= self.level:
            self.log(INFO, msg, *args)

    def warning(self, msg, *args):
        if WARNING >= self.level:
            self.log(WARNING, msg, *args)

    def error(self, msg, *args):
        if ERROR >= self.level:
            self.log(ERROR, msg, *args)

    def critical(self, msg, *args):
        self.log(CRITICAL, msg, *args)


logger = _Logger()
_held = threading.local()


class hold:
    """Context manager: this thread's log lines are kept (``.lines``) instead
    of written, so work run on several threads can be logged in a fixed order
    afterwards with :func:`emit`."""

    def __enter__(self):
        self.lines = []
        self._prev = getattr(_held, "lines", None)
        _held.lines = self.lines
        return self

    def __exit__(self, *exc):
        _held.lines = self._prev
        return False


def emit(lines):
    """Write lines kept by :class:`hold` (into this thread's own held lines
    when it is holding too)."""
    held = getattr(_held, "lines", None)
    if held is not None:
        held.extend(lines)
        return
    stream = logger.stream or sys.stderr
    with logger._lock:
        for line in lines:
            stream.write(line)
        stream.flush()


def set_verbose(verbose=True):
    logger.setLevel(DEBUG if verbose else INFO)


def set_quiet():
    logger.setLevel(ERROR)


def _debug(msg, *args):
    logger.debug(msg, *args)


def _off(msg, *args):
    """``log.debug`` while debug logging is off: one call, no level test or
    formatting (hot loops log per item)."""


debug = _off


def debug_enabled():
    """Whether ``log.debug`` writes anything (guards debug-only work)."""
    return debug is not _off


def _rebind():
    # ``log.debug`` is looked up on the module at every call site
    global debug
    debug = _debug if logger.level <= DEBUG else _off


def info(msg, *args):
    logger.info(msg, *args)


def warning(msg, *args):
    logger.warning(msg, *args)


warn = warning


def error(msg, *args):
    logger.error(msg, *args)


def fatal(msg, *args):
    logger.critical(msg, *args)
    raise FatalError(_format(msg, args) if args else msg)
