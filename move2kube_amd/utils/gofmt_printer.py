"""The ``fmt`` printer (``print.go`` / ``format.go``) behind :mod:`.gofmt`'s
``sprintf`` and the ``%v`` of composite values; loaded on first use, so a
process that only prints strings and numbers never builds it."""

from .gofmt import (LDIGITS, NO_VALUE, UDIGITS, _MASK64, _MAX_RUNE, _RUNE_ERROR, GoUint8, can_backquote,
                    format_float, is_print, quote, quote_rune, quote_to_ascii, sorted_keys, type_string,
                    utf8_bytes)


def _parsenum(s, start, end):
    """print.go: parsenum."""
    if start >= end:
        return 0, False, end
    num = 0
    isnum = False
    i = start
    while i < end and "0" <= s[i] <= "9":
        if num > 1000000 or num < -1000000:  # tooLarge
            return 0, False, end
        num = num * 10 + ord(s[i]) - 48
        isnum = True
        i += 1
    return num, isnum, i


def _parse_arg_number(fmt):
    """print.go: parseArgNumber -> (index, wid, ok); fmt[0] == '['."""
    if len(fmt) < 3:
        return 0, 1, False
    for i in range(1, len(fmt)):
        if fmt[i] == "]":
            width, ok, newi = _parsenum(fmt, 1, i)
            if not ok or newi != i:
                return 0, i + 1, False
            return width - 1, i + 1, True
    return 0, 1, False


def _int_from_arg(a, arg_num):
    """print.go: intFromArg -> (num, isInt, newArgNum)."""
    num, is_int, new = 0, False, arg_num
    if arg_num < len(a):
        v = a[arg_num]
        if isinstance(v, int) and not isinstance(v, bool):
            num, is_int = v, True
        new = arg_num + 1
        if num > 1000000 or num < -1000000:
            num, is_int = 0, False
    return num, is_int, new


class _Printer:
    __slots__ = ("buf", "plus", "minus", "sharp", "space", "zero", "plusV", "sharpV", "wid", "prec",
                 "widPresent", "precPresent", "reordered", "goodArgNum")

    def __init__(self):
        self.buf = []
        self.clearflags()
        self.reordered = False
        self.goodArgNum = True

    def clearflags(self):
        self.plus = self.minus = self.sharp = self.space = self.zero = False
        self.plusV = self.sharpV = False
        self.wid = self.prec = 0
        self.widPresent = self.precPresent = False

    # -- padding (format.go) ---------------------------------------------------
    def write_padding(self, n):
        if n > 0:
            self.buf.append(("0" if self.zero else " ") * n)

    def pad(self, s):
        """format.go: pad / padString (width counts runes)."""
        if not self.widPresent or self.wid == 0:
            self.buf.append(s)
            return
        width = self.wid - len(s)
        if not self.minus:
            self.write_padding(width)
            self.buf.append(s)
        else:
            self.buf.append(s)
            self.write_padding(width)

    # -- verbs -----------------------------------------------------------------
    def bad_verb(self, verb, v, nil=False):
        """print.go: badVerb -- %!verb(type=value), %!verb(<nil>)."""
        buf = self.buf
        buf.append("%!" + verb + "(")
        if nil or v is None or v is NO_VALUE:
            buf.append("<nil>")
        else:
            buf.append(type_string(v))
            buf.append("=")
            self.print_arg(v, "v")
        buf.append(")")

    def fmt_bool(self, v, verb):
        if verb in "tv":
            self.pad("true" if v else "false")
        else:
            self.bad_verb(verb, v)

    def fmt_integer(self, v, signed, verb):
        """print.go: fmtInteger (v the Go value; a negative signed value is its
        two's complement for %c %q %U, as uint64(f))."""
        u = v & _MASK64
        if verb == "v":
            if self.sharpV and not signed:
                self.fmt0x64(u, True)
            else:
                self.fmt_int(u, 10, signed, verb, LDIGITS)
        elif verb == "d":
            self.fmt_int(u, 10, signed, verb, LDIGITS)
        elif verb == "b":
            self.fmt_int(u, 2, signed, verb, LDIGITS)
        elif verb in "oO":
            self.fmt_int(u, 8, signed, verb, LDIGITS)
        elif verb == "x":
            self.fmt_int(u, 16, signed, verb, LDIGITS)
        elif verb == "X":
            self.fmt_int(u, 16, signed, verb, UDIGITS)
        elif verb == "c":
            r = u if u <= _MAX_RUNE and not 0xD800 <= u <= 0xDFFF else _RUNE_ERROR
            self.pad(chr(r))
        elif verb == "q":
            if u <= _MAX_RUNE:
                self.pad(quote_rune(u, self.plus))
            else:
                self.bad_verb(verb, v)
        elif verb == "U":
            self.fmt_unicode(u)
        else:
            self.bad_verb(verb, v)

    def fmt0x64(self, u, leading0x):
        sharp = self.sharp
        self.sharp = leading0x
        self.fmt_int(u, 16, False, "v", LDIGITS)
        self.sharp = sharp

    def fmt_int(self, u, base, signed, verb, digits):
        """format.go: fmtInteger."""
        negative = signed and u >= 1 << 63
        if negative:
            u = (-u) & _MASK64
        prec = 0
        if self.precPresent:
            prec = self.prec
            if prec == 0 and u == 0:
                old = self.zero
                self.zero = False
                self.write_padding(self.wid)
                self.zero = old
                return
        elif self.zero and self.widPresent:
            prec = self.wid
            if negative or self.plus or self.space:
                prec -= 1
        if base == 10:
            s = str(u)
        elif base == 16:
            s = format(u, "x")
            if digits is UDIGITS:
                s = s.upper()
        elif base == 8:
            s = format(u, "o")
        else:
            s = format(u, "b")
        if prec > len(s):
            s = "0" * (prec - len(s)) + s
        if self.sharp:
            if base == 2:
                s = "0b" + s
            elif base == 8:
                if s[0] != "0":
                    s = "0" + s
            elif base == 16:
                s = "0" + digits[16] + s
        if verb == "O":
            s = "0o" + s
        if negative:
            s = "-" + s
        elif self.plus:
            s = "+" + s
        elif self.space:
            s = " " + s
        old = self.zero
        self.zero = False
        self.pad(s)
        self.zero = old

    def fmt_unicode(self, u):
        """format.go: fmtUnicode (U+0041, %#U adds ' 'A'')."""
        prec = 4
        if self.precPresent and self.prec > 4:
            prec = self.prec
        tail = ""
        if self.sharp and u <= _MAX_RUNE and is_print(u):
            tail = " '" + chr(u) + "'"
        h = format(u, "X")
        if len(h) < prec:
            h = "0" * (prec - len(h)) + h
        old = self.zero
        self.zero = False
        self.pad("U+" + h + tail)
        self.zero = old

    def fmt_float(self, v, verb):
        """print.go: fmtFloat -> format.go: fmtFloat (size 64)."""
        if verb == "v":
            self._float(v, "g", -1)
        elif verb in "bgGxX":
            self._float(v, verb, -1)
        elif verb in "feE":
            self._float(v, verb, 6)
        elif verb == "F":
            self._float(v, "f", 6)
        else:
            self.bad_verb(verb, v)

    def _float(self, v, verb, prec):
        if self.precPresent:
            prec = self.prec
        num = format_float(v, verb, prec)
        if num[0] in "-+":
            sign, body = num[0], num[1:]
        else:
            sign, body = "+", num
        if self.space and sign == "+" and not self.plus:
            sign = " "
        if body[0] in "IN":
            old = self.zero
            self.zero = False
            if body[0] == "N" and not self.space and not self.plus:
                self.pad(body)
            else:
                self.pad(sign + body)
            self.zero = old
            return
        if self.sharp and verb != "b":
            digits = 0
            if verb in "vgGx":
                digits = prec if prec != -1 else 6
            tail = ""
            has_point = False
            i = 0
            out = []
            while i < len(body):
                c = body[i]
                if c == ".":
                    has_point = True
                elif c in "pP":
                    tail = body[i:]
                    break
                elif c in "eE" and verb not in "xX":
                    tail = body[i:]
                    break
                else:
                    digits -= 1
                out.append(c)
                i += 1
            body = "".join(out)
            if not has_point:
                body += "."
            if digits > 0:
                body += "0" * digits
            body += tail
        if self.plus or sign != "+":
            if self.zero and self.widPresent and self.wid > len(body) + 1:
                self.buf.append(sign)
                self.write_padding(self.wid - len(body) - 1)
                self.buf.append(body)
                return
            self.pad(sign + body)
            return
        self.pad(body)

    def fmt_complex(self, v, verb):
        if verb in "vbgGxXfFeE":
            old = self.plus
            self.buf.append("(")
            self.fmt_float(v.real, verb)
            self.plus = True
            self.fmt_float(v.imag, verb)
            self.buf.append("i)")
            self.plus = old
        else:
            self.bad_verb(verb, v)

    def truncate(self, s):
        if self.precPresent and self.prec < len(s):
            return s[:self.prec]
        return s

    def fmt_q(self, s):
        s = self.truncate(s)
        if self.sharp and can_backquote(s):
            self.pad("`" + s + "`")
            return
        self.pad(quote_to_ascii(s) if self.plus else quote(s))

    def fmt_sbx(self, b, digits):
        """format.go: fmtSbx over the bytes b."""
        length = len(b)
        if self.precPresent and self.prec < length:
            length = self.prec
        width = 2 * length
        if width > 0:
            if self.space:
                if self.sharp:
                    width *= 2
                width += length - 1
            elif self.sharp:
                width += 2
        else:
            if self.widPresent:
                self.write_padding(self.wid)
            return
        if self.widPresent and self.wid > width and not self.minus:
            self.write_padding(self.wid - width)
        out = []
        if self.sharp:
            out.append("0" + digits[16])
        for i in range(length):
            if self.space and i > 0:
                out.append(" ")
                if self.sharp:
                    out.append("0" + digits[16])
            c = b[i]
            out.append(digits[c >> 4] + digits[c & 15])
        self.buf.append("".join(out))
        if self.widPresent and self.wid > width and self.minus:
            self.write_padding(self.wid - width)

    def fmt_string(self, s, verb):
        if verb == "v":
            if self.sharpV:
                self.fmt_q(s)
            else:
                self.pad(self.truncate(s))
        elif verb == "s":
            self.pad(self.truncate(s))
        elif verb == "x":
            self.fmt_sbx(utf8_bytes(s), LDIGITS)
        elif verb == "X":
            self.fmt_sbx(utf8_bytes(s), UDIGITS)
        elif verb == "q":
            self.fmt_q(s)
        else:
            self.bad_verb(verb, s)

    def fmt_bytes(self, b, verb, type_name):
        if verb in "vd":
            if self.sharpV:
                self.buf.append(type_name + "{")
                for i, c in enumerate(b):
                    if i > 0:
                        self.buf.append(", ")
                    self.fmt0x64(c, True)
                self.buf.append("}")
            else:
                self.buf.append("[")
                for i, c in enumerate(b):
                    if i > 0:
                        self.buf.append(" ")
                    self.fmt_int(c, 10, False, verb, LDIGITS)
                self.buf.append("]")
        elif verb == "s":
            self.pad(self.truncate(bytes(b).decode("utf-8", "surrogateescape")))
        elif verb == "x":
            self.fmt_sbx(bytes(b), LDIGITS)
        elif verb == "X":
            self.fmt_sbx(bytes(b), UDIGITS)
        elif verb == "q":
            self.fmt_q(bytes(b).decode("utf-8", "surrogateescape"))
        else:
            self.print_value(list(GoUint8(c) for c in b), verb, 0)

    def fmt_pointer(self, v, verb):
        if isinstance(v, (list, tuple, dict)) or callable(v):
            u = id(v)
            if verb == "v" and self.sharpV:
                self.buf.append("(" + type_string(v) + ")(0x%x)" % u)
                return
            if verb in "vp":
                old = self.sharp
                self.sharp = not self.sharp
                self.fmt_int(u, 16, False, "v", LDIGITS)
                self.sharp = old
                return
            if verb in "bodxX":
                self.fmt_integer(u, False, verb)
                return
        self.bad_verb(verb, v)

    def print_arg(self, arg, verb):
        """print.go: printArg."""
        if arg is None or arg is NO_VALUE:
            if verb in "Tv":
                self.pad("<nil>")
            else:
                self.bad_verb(verb, None, nil=True)
            return
        if verb == "T":
            self.pad(self.truncate(type_string(arg)))
            return
        if verb == "p":
            self.fmt_pointer(arg, "p")
            return
        t = type(arg)
        if t is str:
            self.fmt_string(arg, verb)
        elif t is int:
            self.fmt_integer(arg, True, verb)
        elif t is float:
            self.fmt_float(arg, verb)
        elif t is bool:
            self.fmt_bool(arg, verb)
        elif t is GoUint8:
            self.fmt_integer(arg, False, verb)
        elif t is complex:
            self.fmt_complex(arg, verb)
        elif t in (bytes, bytearray):
            self.fmt_bytes(arg, verb, "[]byte")
        else:
            self.print_value(arg, verb, 0)

    def print_value(self, v, verb, depth):
        """print.go: printValue over the composite values."""
        buf = self.buf
        if v is None or v is NO_VALUE:
            # an interface element holding nil (or the zero reflect.Value)
            if depth == 0 and v is NO_VALUE:
                buf.append("<invalid reflect.Value>")
            elif self.sharpV:
                buf.append("interface {}(nil)")
            elif verb == "v" or depth > 0:
                buf.append("<nil>")
            else:
                self.bad_verb(verb, None, nil=True)
            return
        if isinstance(v, bool):
            self.fmt_bool(v, verb)
        elif isinstance(v, GoUint8):
            self.fmt_integer(v, False, verb)
        elif isinstance(v, int):
            self.fmt_integer(v, True, verb)
        elif isinstance(v, float):
            self.fmt_float(v, verb)
        elif isinstance(v, complex):
            self.fmt_complex(v, verb)
        elif isinstance(v, str):
            self.fmt_string(v, verb)
        elif isinstance(v, (bytes, bytearray)):
            self.fmt_bytes(v, verb, "[]uint8")
        elif isinstance(v, dict):
            if self.sharpV:
                buf.append(type_string(v) + "{")
            else:
                buf.append("map[")
            for i, k in enumerate(sorted_keys(v)):
                if i > 0:
                    buf.append(", " if self.sharpV else " ")
                self.print_value(k, verb, depth + 1)
                buf.append(":")
                self.print_value(v[k], verb, depth + 1)
            buf.append("}" if self.sharpV else "]")
        elif isinstance(v, (list, tuple)):
            if self.sharpV:
                buf.append(type_string(v) + "{")
                for i, x in enumerate(v):
                    if i > 0:
                        buf.append(", ")
                    self.print_value(x, verb, depth + 1)
                buf.append("}")
            else:
                buf.append("[")
                for i, x in enumerate(v):
                    if i > 0:
                        buf.append(" ")
                    self.print_value(x, verb, depth + 1)
                buf.append("]")
        elif callable(v):
            self.fmt_pointer(v, verb)
        else:
            fields = [(k, x) for k, x in vars(v).items() if not k.startswith("_")] if hasattr(v, "__dict__") else []
            if self.sharpV:
                buf.append(type_string(v))
            buf.append("{")
            for i, (k, x) in enumerate(fields):
                if i > 0:
                    buf.append(", " if self.sharpV else " ")
                if self.plusV or self.sharpV:
                    buf.append(k + ":")
                self.print_value(x, verb, depth + 1)
            buf.append("}")

    # -- Printf ----------------------------------------------------------------
    def arg_number(self, arg_num, fmt, i, num_args):
        """print.go: argNumber -> (newArgNum, newi, found)."""
        if len(fmt) <= i or fmt[i] != "[":
            return arg_num, i, False
        self.reordered = True
        index, wid, ok = _parse_arg_number(fmt[i:])
        if ok and 0 <= index < num_args:
            return index, i + wid, True
        self.goodArgNum = False
        return arg_num, i + wid, ok

    def do_printf(self, fmt, a):
        """print.go: doPrintf."""
        end = len(fmt)
        arg_num = 0
        after_index = False
        self.reordered = False
        buf = self.buf
        i = 0
        while i < end:
            self.goodArgNum = True
            j = fmt.find("%", i)
            if j < 0:
                j = end
            if j > i:
                buf.append(fmt[i:j])
            i = j
            if i >= end:
                break
            i += 1
            self.clearflags()
            simple = False
            while i < end:
                c = fmt[i]
                if c == "#":
                    self.sharp = True
                elif c == "0":
                    self.zero = not self.minus
                elif c == "+":
                    self.plus = True
                elif c == "-":
                    self.minus = True
                    self.zero = False
                elif c == " ":
                    self.space = True
                else:
                    if "a" <= c <= "z" and arg_num < len(a):
                        if c == "v":
                            self.sharpV, self.sharp = self.sharp, False
                            self.plusV, self.plus = self.plus, False
                        self.print_arg(a[arg_num], c)
                        arg_num += 1
                        i += 1
                        simple = True
                    break
                i += 1
            if simple:
                continue
            arg_num, i, after_index = self.arg_number(arg_num, fmt, i, len(a))
            if i < end and fmt[i] == "*":
                i += 1
                self.wid, self.widPresent, arg_num = _int_from_arg(a, arg_num)
                if not self.widPresent:
                    buf.append("%!(BADWIDTH)")
                if self.wid < 0:
                    self.wid = -self.wid
                    self.minus = True
                    self.zero = False
                after_index = False
            else:
                self.wid, self.widPresent, i = _parsenum(fmt, i, end)
                if after_index and self.widPresent:
                    self.goodArgNum = False
            if i + 1 < end and fmt[i] == ".":
                i += 1
                if after_index:
                    self.goodArgNum = False
                arg_num, i, after_index = self.arg_number(arg_num, fmt, i, len(a))
                if i < end and fmt[i] == "*":
                    i += 1
                    self.prec, self.precPresent, arg_num = _int_from_arg(a, arg_num)
                    if self.prec < 0:
                        self.prec = 0
                        self.precPresent = False
                    if not self.precPresent:
                        buf.append("%!(BADPREC)")
                    after_index = False
                else:
                    self.prec, self.precPresent, i = _parsenum(fmt, i, end)
                    if not self.precPresent:
                        self.prec = 0
                        self.precPresent = True
            if not after_index:
                arg_num, i, after_index = self.arg_number(arg_num, fmt, i, len(a))
            if i >= end:
                buf.append("%!(NOVERB)")
                break
            verb = fmt[i]
            i += 1
            if verb == "%":
                buf.append("%")
            elif not self.goodArgNum:
                buf.append("%!" + verb + "(BADINDEX)")
            elif arg_num >= len(a):
                buf.append("%!" + verb + "(MISSING)")
            else:
                if verb == "v":
                    self.sharpV, self.sharp = self.sharp, False
                    self.plusV, self.plus = self.plus, False
                self.print_arg(a[arg_num], verb)
                arg_num += 1
        if not self.reordered and arg_num < len(a):
            self.clearflags()
            buf.append("%!(EXTRA ")
            for k, arg in enumerate(a[arg_num:]):
                if k > 0:
                    buf.append(", ")
                if arg is None or arg is NO_VALUE:
                    buf.append("<nil>")
                else:
                    buf.append(type_string(arg) + "=")
                    self.print_arg(arg, "v")
            buf.append(")")
