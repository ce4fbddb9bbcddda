"""The command-line parsing of spf13/cobra v1.1.1 + spf13/pflag v1.0.5, the
libraries the reference's ``cmd/move2kube/*.go`` are built on (``go.mod:30``).

Only what move2kube's command tree uses: sub-commands, persistent root flags,
bool / string / int / string-slice flags with shorthands, hidden and required
flags, ``-h/--help``, the implicit ``help [command]`` sub-command, and cobra's
help / usage / error texts byte for byte (usage and help templates, pflag's
``FlagUsages`` column layout, "unknown command" suggestions).  Parsing follows
pflag's ``parseArgs``: interspersed flags and arguments, ``--`` ends the flags,
``--flag=v`` / ``--flag v`` / ``-fv`` / ``-f v`` / ``-f=v`` / grouped boolean
shorthands, and the first error stops the parse.

Written without ``argparse``: argparse's help strings go through ``gettext``
and ``locale`` on every run, which on a host whose system bytecode caches are
stale (the MI355X image, ``profiles/r03_cold_diag``) recompiles three modules
per process.
"""

import sys


class FlagError(Exception):
    """A parse or validation error (cobra prints it with the usage)."""


class HelpRequested(Exception):
    """``flag.ErrHelp``: print the command's help and exit 0."""


class Flag:
    __slots__ = ("name", "shorthand", "kind", "default", "usage", "hidden", "value", "changed")

    def __init__(self, name, shorthand, kind, default, usage, hidden=False):
        self.name = name
        self.shorthand = shorthand
        self.kind = kind  # "bool" | "string" | "int" | "stringSlice"
        self.default = default
        self.usage = usage
        self.hidden = hidden
        self.reset()

    def reset(self):
        self.value = list(self.default) if self.kind == "stringSlice" else self.default
        self.changed = False

    @property
    def no_opt_default(self):
        return "true" if self.kind == "bool" else ""

    @property
    def def_value(self):
        """pflag ``DefValue`` (the default rendered as text)."""
        if self.kind == "bool":
            return "true" if self.default else "false"
        if self.kind == "stringSlice":
            return "[" + ",".join(self.default) + "]"
        return str(self.default)

    def default_is_zero(self):
        return self.def_value in {"bool": ("false",), "string": ("",), "int": ("0",),
                                  "stringSlice": ("[]",)}[self.kind]

    def set(self, text):
        try:
            if self.kind == "bool":
                v = _parse_bool(text)
            elif self.kind == "int":
                v = _parse_int(text)
            elif self.kind == "stringSlice":
                items = _read_csv(text)
                v = (self.value + items) if self.changed else items
            else:
                v = text
        except ValueError as e:
            from ..utils.log import go_quote
            flag_name = "-%s, --%s" % (self.shorthand, self.name) if self.shorthand else "--" + self.name
            raise FlagError("invalid argument %s for %s flag: %s" % (go_quote(text), go_quote(flag_name), e))
        self.value = v
        self.changed = True


def _go_q(s):
    from ..utils.log import go_quote
    return go_quote(s)


def _parse_bool(s):
    from ..utils.common import go_parse_bool
    return go_parse_bool(s)


def _parse_int(s):
    from ..utils.common import go_parse_int
    return go_parse_int(s)


def _read_csv(val):
    """pflag ``readAsCSV``: one record of encoding/csv (quoted fields, ``""``
    escapes; a bare quote in an unquoted field is an error)."""
    if val == "":
        return []
    val = val.split("\n", 1)[0].rstrip("\r")
    out, i, n = [], 0, len(val)
    while True:
        if i < n and val[i] == '"':
            j, buf = i + 1, []
            while True:
                k = val.find('"', j)
                if k < 0:
                    raise ValueError('parse error on line 1, column %d: extraneous or missing " in quoted-field'
                                     % (n + 1))
                buf.append(val[j:k])
                if k + 1 < n and val[k + 1] == '"':
                    buf.append('"')
                    j = k + 2
                    continue
                i = k + 1
                break
            if i < n and val[i] != ",":
                raise ValueError('parse error on line 1, column %d: extraneous or missing " in quoted-field' % (i + 1))
            out.append("".join(buf))
        else:
            k = val.find(",", i)
            field = val[i:] if k < 0 else val[i:k]
            q = field.find('"')
            if q >= 0:
                raise ValueError('parse error on line 1, column %d: bare " in non-quoted-field' % (i + q + 1))
            out.append(field)
            i = n if k < 0 else k
        if i >= n:
            return out
        i += 1  # the comma
        if i == n:
            out.append("")
            return out


class Command:
    def __init__(self, use, short="", long="", run=None, hidden=False):
        self.use = use
        self.name = use.split(" ", 1)[0]
        self.short = short
        self.long = long
        self.run = run
        self.hidden = hidden
        self.parent = None
        self.commands = []
        self.local = []       # Flags()
        self.persistent = []  # PersistentFlags()
        self.required = []
        self.help_cmd = None
        self._help_flag = None

    # -- tree -----------------------------------------------------------------
    def add(self, *cmds):
        for c in cmds:
            c.parent = self
            self.commands.append(c)

    def flag(self, name, shorthand, kind, default, usage, hidden=False, persistent=False):
        f = Flag(name, shorthand, kind, default, usage, hidden)
        (self.persistent if persistent else self.local).append(f)
        return f

    def mark_required(self, name):
        self.required.append(name)

    @property
    def runnable(self):
        return self.run is not None

    def command_path(self):
        return self.parent.command_path() + " " + self.name if self.parent else self.name

    def root(self):
        return self.parent.root() if self.parent else self

    def sorted_commands(self):
        return sorted(self.commands, key=lambda c: c.name)

    def is_available(self):
        if self.hidden:
            return False
        if self.parent is not None and self.parent.help_cmd is self:
            return False
        return self.runnable or self.has_available_subcommands()

    def has_available_subcommands(self):
        return any(c.is_available() for c in self.commands)

    # -- flag sets --------------------------------------------------------------
    def init_help_flag(self):
        if self._help_flag is None:
            self._help_flag = Flag("help", "h", "bool", False, "help for " + self.name)
            self.local.append(self._help_flag)

    def parents_persistent(self):
        out, p = [], self.parent
        while p is not None:
            out.extend(p.persistent)
            p = p.parent
        return out

    def all_flags(self):
        """Flags() after mergePersistentFlags: local, own persistent, inherited."""
        seen, out = set(), []
        for f in self.local + self.persistent + self.parents_persistent():
            if f.name not in seen:
                seen.add(f.name)
                out.append(f)
        return out

    def local_flags(self):
        inherited = {f.name for f in self.parents_persistent()}
        return [f for f in self.local + self.persistent if f.name not in inherited]

    def inherited_flags(self):
        own = {f.name for f in self.local + self.persistent}
        return [f for f in self.parents_persistent() if f.name not in own]

    # -- parsing (pflag parseArgs) ----------------------------------------------
    def parse_flags(self, args):
        flags = self.all_flags()
        for f in flags:
            f.reset()
        longs = {f.name: f for f in flags}
        shorts = {f.shorthand: f for f in flags if f.shorthand}
        positional = []
        args = list(args)
        while args:
            s = args.pop(0)
            if len(s) < 2 or s[0] != "-":
                positional.append(s)
                continue
            if s[1] == "-":
                if len(s) == 2:  # "--" terminates the flags
                    positional.extend(args)
                    break
                name = s[2:]
                if name[0] in "-=":
                    raise FlagError("bad flag syntax: %s" % s)
                name, eq, value = name.partition("=")
                f = longs.get(name)
                if f is None:
                    if name == "help":
                        raise HelpRequested()
                    raise FlagError("unknown flag: --%s" % name)
                if eq:
                    pass
                elif f.no_opt_default:
                    value = f.no_opt_default
                elif args:
                    value = args.pop(0)
                else:
                    raise FlagError("flag needs an argument: %s" % s)
                f.set(value)
                continue
            shorthands = s[1:]
            while shorthands:
                c = shorthands[0]
                rest = shorthands[1:]
                f = shorts.get(c)
                if f is None:
                    if c == "h":
                        raise HelpRequested()
                    raise FlagError("unknown shorthand flag: %s in -%s" % (_go_char(c), shorthands))
                if len(shorthands) > 2 and shorthands[1] == "=":
                    value, rest = shorthands[2:], ""
                elif f.no_opt_default:
                    value = f.no_opt_default
                elif len(shorthands) > 1:
                    value, rest = shorthands[1:], ""
                elif args:
                    value = args.pop(0)
                else:
                    raise FlagError("flag needs an argument: %s in -%s" % (_go_char(c), shorthands))
                f.set(value)
                shorthands = rest
        return positional

    def value(self, name):
        for f in self.all_flags():
            if f.name == name:
                return f.value
        raise KeyError(name)

    def changed(self, name):
        for f in self.all_flags():
            if f.name == name:
                return f.changed
        return False

    # -- texts ---------------------------------------------------------------------
    def use_line(self):
        line = (self.parent.command_path() + " " + self.use) if self.parent else self.use
        if any(not f.hidden for f in self.all_flags()) and "[flags]" not in line:
            line += " [flags]"
        return line

    def usage_string(self):
        out = ["Usage:"]
        if self.runnable:
            out.append("\n  " + self.use_line())
        subs = self.has_available_subcommands()
        if subs:
            out.append("\n  %s [command]" % self.command_path())
            out.append("\n\nAvailable Commands:")
            pad = max([11] + [len(c.name) for c in self.commands if c.is_available()])
            for c in self.sorted_commands():
                if c.is_available() or c.name == "help":
                    out.append("\n  %s %s" % (c.name.ljust(pad), c.short))
        local = [f for f in self.local_flags() if not f.hidden]
        if local:
            out.append("\n\nFlags:\n" + flag_usages(local).rstrip())
        inherited = [f for f in self.inherited_flags() if not f.hidden]
        if inherited:
            out.append("\n\nGlobal Flags:\n" + flag_usages(inherited).rstrip())
        if subs:
            out.append('\n\nUse "%s [command] --help" for more information about a command.' % self.command_path())
        return "".join(out) + "\n"

    def help_string(self):
        text = (self.long or self.short).rstrip()
        head = text + "\n\n" if text else ""
        return head + (self.usage_string() if self.runnable or self.commands else "")

    # -- command lookup (cobra Find / legacyArgs) -------------------------------------
    def find(self, args):
        cmd, rest = self, list(args)
        while True:
            words = _strip_flags(rest, cmd)
            if not words:
                break
            nxt = next((c for c in cmd.commands if c.name == words[0]), None)
            if nxt is None:
                break
            i = rest.index(words[0])
            rest = rest[:i] + rest[i + 1:]
            cmd = nxt
        if cmd.commands and cmd.parent is None:
            words = _strip_flags(rest, cmd)
            if words:
                raise FlagError("unknown command %s for %s%s" % (_go_q(words[0]), _go_q(cmd.command_path()),
                                                                   cmd.suggestions(words[0])))
        return cmd, rest

    def suggestions(self, typed):
        from ..ops.editdistance import wagner_fischer_py
        names = []
        for c in self.commands:
            ld = wagner_fischer_py(typed.lower(), c.name.lower(), 1, 1, 1)  # cobra ld(), ignoreCase
            if c.is_available() and (ld <= 2 or c.name.lower().startswith(typed.lower())):
                names.append(c.name)
        if not names:
            return ""
        return "\n\nDid you mean this?\n" + "".join("\t%s\n" % n for n in names)


def _go_char(c):
    """Go ``%q`` of a byte: a quoted character literal."""
    if c == "'":
        return "'\\''"
    if c == "\\":
        return "'\\\\'"
    if " " <= c <= "~":
        return "'%s'" % c
    return "'\\x%02x'" % (ord(c) & 0xFF)


def _strip_flags(args, cmd):
    """cobra ``stripFlags``: the non-flag words of ``args``."""
    flags = cmd.all_flags() + [Flag("help", "h", "bool", False, "")]
    bool_long = {f.name for f in flags if f.kind == "bool"}
    bool_short = {f.shorthand for f in flags if f.kind == "bool" and f.shorthand}
    words, args = [], list(args)
    while args:
        s = args.pop(0)
        if s == "--":
            break
        if s.startswith("--") and "=" not in s and s[2:] not in bool_long:
            if len(args) <= 1:
                break
            args.pop(0)
            continue
        if s.startswith("-") and "=" not in s and len(s) == 2 and s[1:] not in bool_short:
            if len(args) <= 1:
                break
            args.pop(0)
            continue
        if s and not s.startswith("-"):
            words.append(s)
    return words


def flag_usages(flags):
    """pflag ``FlagSet.FlagUsages`` (sorted by name, no wrapping)."""
    lines, maxlen = [], 0
    for f in sorted(flags, key=lambda f: f.name):
        line = "  -%s, --%s" % (f.shorthand, f.name) if f.shorthand else "      --" + f.name
        varname = {"bool": "", "string": "string", "int": "int", "stringSlice": "strings"}[f.kind]
        if varname:
            line += " " + varname
        line += "\x00"
        maxlen = max(maxlen, len(line))
        line += f.usage
        if not f.default_is_zero():
            line += " (default %s)" % (_go_q(f.def_value) if f.kind == "string" else f.def_value)
        lines.append(line)
    out = []
    for line in lines:
        sidx = line.index("\x00")
        out.append("%s %s %s\n" % (line[:sidx], " " * (maxlen - sidx), line[sidx + 1:]))
    return "".join(out)


def add_help_command(root):
    """cobra ``InitDefaultHelpCmd``."""
    def run(cmd, args):
        try:
            target, _ = root.find(args)
        except FlagError:
            target = None
        if target is None:
            sys.stderr.write("Unknown help topic [%s]\n" % " ".join("`%s`" % a for a in args))
            sys.stderr.write(root.usage_string())
            return 0
        target.init_help_flag()
        sys.stdout.write(target.help_string())
        return 0
    h = Command("help [command]", "Help about any command",
                "Help provides help for any command in the application.\n"
                "Simply type %s help [path to command] for full details." % root.name, run=run)
    root.add(h)
    root.help_cmd = h
    return h


def execute(root, argv):
    """cobra ``ExecuteC``: returns (command, its positional args) to run, or an
    int exit status after printing help or an error (``"Error: ..."`` lines
    like cobra, then the reference's ``log.Fatalf("Error: %q", err)``)."""
    from ..utils import log
    try:
        cmd, rest = root.find(argv)
    except FlagError as e:
        sys.stderr.write("Error: %s\n" % e)
        sys.stderr.write("Run '%s --help' for usage.\n" % root.command_path())
        return _fatal(log, e)
    cmd.init_help_flag()
    try:
        positional = cmd.parse_flags(rest)
        if cmd.value("help"):
            raise HelpRequested()
        if not cmd.runnable:
            raise HelpRequested()
        missing = [n for n in cmd.required if not cmd.changed(n)]
        if missing:
            raise FlagError("required flag(s) %s not set" % ", ".join(_go_q(n) for n in sorted(missing)))
    except HelpRequested:
        sys.stdout.write(cmd.help_string())
        return 0
    except FlagError as e:
        sys.stderr.write("Error: %s\n" % e)
        sys.stderr.write(cmd.usage_string() + "\n")
        return _fatal(log, e)
    return cmd, positional


def _fatal(log, e):
    try:
        log.fatal("Error: %r", str(e))
    except log.FatalError:
        pass
    return 1
