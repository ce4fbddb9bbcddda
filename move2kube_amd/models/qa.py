"""QA problems and the QA cache (``kind: QACache``).

Reference: ``types/qaengine/problem.go:33-291`` and ``types/qaengine/cache.go:29-138``.
Problem validation rules (auto-resolution of single-option selects and
empty multi-selects, default checks), answer validation and cache matching
(case-insensitive description equality *or* regex match) follow the reference
so that caches written by either tool replay in the other.
"""

import functools
import re
import threading

from ..utils import common, log, yamlio
from ..utils.constants import SCHEME_GROUP_VERSION
from .base import as_bool, as_list, as_map, as_str, as_str_list

SELECT = "Select"
MULTISELECT = "MultiSelect"
INPUT = "Input"
MULTILINE = "MultiLine"
PASSWORD = "Password"
CONFIRM = "Confirm"

QACACHE_KIND = "QACache"

_id_lock = threading.Lock()
_last_id = 0


def _next_id():
    global _last_id
    with _id_lock:
        _last_id += 1
        return _last_id


class ProblemError(ValueError):
    pass


def _parse_bool(s):
    return common.cast_to_bool(s)


class Problem:
    __slots__ = ("id", "desc", "context", "type", "default", "options", "answer", "resolved")

    def __init__(self, id=0, desc="", context=None, type="", default=None, options=None,
                 answer=None, resolved=False):
        self.id = id
        self.desc = desc
        self.context = context if context is not None else []
        self.type = type
        self.default = default if default is not None else []
        self.options = options if options is not None else []
        self.answer = answer
        self.resolved = resolved

    def go_s(self):
        """fmt ``%s`` of the Go struct (ints and bools print as ``%!s(...)``)."""
        def lst(xs):
            return "[" + " ".join(xs or ()) + "]"
        return "{%%!s(int=%d) %s %s {%s %s %s %s} %%!s(bool=%s)}" % (
            self.id, self.desc, lst(self.context), self.type, lst(self.default), lst(self.options),
            lst(self.answer), "true" if self.resolved else "false")

    def go_plus_v(self):
        """fmt ``%+v`` of the Go struct: field names, nil slices as ``[]``."""
        def lst(xs):
            return "[" + " ".join(xs or ()) + "]"
        return "{ID:%d Desc:%s Context:%s Solution:{Type:%s Default:%s Options:%s Answer:%s} Resolved:%s}" % (
            self.id, self.desc, lst(self.context), self.type, lst(self.default), lst(self.options),
            lst(self.answer), "true" if self.resolved else "false")

    def copy(self):
        return Problem(self.id, self.desc, list(self.context), self.type, list(self.default),
                       list(self.options), None if self.answer is None else list(self.answer), self.resolved)

    # -- answers -------------------------------------------------------------
    def set_answer(self, answer):
        answer = list(answer or [])
        if self.type != MULTISELECT and len(answer) == 0:
            raise ProblemError("The answer slice is empty")
        if self.type != MULTISELECT and len(answer) > 1:
            raise ProblemError("The question type is not multiselect, but there are multiple answers")
        if self.type in (SELECT, MULTISELECT):
            ok = True
            self.answer = []
            folded = {common.go_fold(o) for o in self.options} if len(answer) > 1 else None
            for a in answer:
                if (common.go_fold(a) not in folded) if folded is not None else not common.is_string_present(self.options, a):
                    log.warning("No matching value in options for %s. Ignoring.", a)
                    ok = False
                    continue
                self.answer.append(a)
            if not ok:
                raise ProblemError("Unknown options selected")
            self.resolved = True
            return
        if self.type == CONFIRM:
            try:
                _parse_bool(answer[0])
            except ValueError as e:
                log.warning("Error while parsing answer for confirm question type : %s", e)
                raise ProblemError(str(e))
        self.answer = [answer[0]]
        self.resolved = True

    def get_slice_answer(self):
        if not self.resolved:
            raise ProblemError("Problem yet to be resolved")
        if self.type != MULTISELECT:
            raise ProblemError("This question type does not support this answer type")
        return list(self.answer or [])

    def get_bool_answer(self):
        if not self.resolved:
            raise ProblemError("Problem yet to be resolved")
        if self.type != CONFIRM:
            raise ProblemError("This question type does not support this answer type")
        if not self.answer or len(self.answer) != 1:
            raise ProblemError("No answer available")
        return _parse_bool(self.answer[0])

    def get_string_answer(self):
        if not self.resolved:
            raise ProblemError("Problem yet to be resolved")
        if self.type in (MULTISELECT, CONFIRM):
            raise ProblemError("This question type does not support this answer type")
        if not self.answer or len(self.answer) != 1:
            raise ProblemError("Wrong number of answers")
        return self.answer[0]

    def matches(self, other):
        return _match_string(self.desc, other.desc) and self.type == other.type

    # -- encoding ------------------------------------------------------------
    def to_yaml(self):
        d = {"description": self.desc}
        if self.context:
            d["context"] = list(self.context)
        sol = {"type": self.type}
        if self.default:
            sol["default"] = list(self.default)
        if self.options:
            sol["options"] = list(self.options)
        sol["answer"] = list(self.answer) if self.answer is not None else None
        if sol["answer"] is None:
            sol["answer"] = []
        d["solution"] = sol
        if self.resolved:
            d["resolved"] = True
        return d

    def to_json(self):
        d = {"id": self.id, "description": self.desc}
        if self.context:
            d["context"] = list(self.context)
        sol = {"type": self.type}
        if self.default:
            sol["default"] = list(self.default)
        if self.options:
            sol["options"] = list(self.options)
        sol["answer"] = list(self.answer) if self.answer is not None else None
        d["solution"] = sol
        if self.resolved:
            d["resolved"] = True
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        sol = as_map(d.get("solution"))
        ans = sol.get("answer")
        return cls(0, as_str(d.get("description")), as_str_list(d.get("context")), as_str(sol.get("type")),
                   as_str_list(sol.get("default")), as_str_list(sol.get("options")),
                   as_str_list(ans) if ans is not None else None, as_bool(d.get("resolved")))

    def __repr__(self):
        return "Problem(%r)" % (self.to_json(),)


_NOT_COMPILED = object()
_QUANTIFIERS = "*?{"


def required_literals(pattern):
    """Literal substrings every match of ``pattern`` must contain (a
    conservative subset), or None when the pattern has alternation or inline
    flags and no such guarantee is cheap to give.

    Only runs outside groups and character classes count, and a character
    followed by ``*``, ``?`` or ``{`` is dropped: so if one of them is missing
    from a string, ``re.search(pattern, string)`` is None for certain and the
    pattern need not be compiled (question descriptions in a QA cache are
    prose; almost none of them match each other)."""
    if "|" in pattern or "(?" in pattern:
        return None
    if _SIMPLE_PATTERN_OUT.isdisjoint(pattern):
        return _simple_required_literals(pattern)
    return _required_literals_scan(pattern)


# patterns made only of literal characters, "." "^" "$" "+" and the "*" / "?"
# quantifiers (most question texts) are split with str methods
_SIMPLE_PATTERN_OUT = frozenset("\\[](){}|\x00\x01")
_TO_FLUSH = str.maketrans(".^$+", "\x00\x00\x00\x00")
_TO_QUANT = str.maketrans("*?", "\x01\x01")


def _simple_required_literals(pattern):
    """:func:`required_literals` of a pattern without escapes, classes,
    groups, repeat counts or alternation: runs between "." "^" "$" "+", with a
    character followed by "*" or "?" dropped (it is optional)."""
    out = []
    for seg in pattern.translate(_TO_FLUSH).split("\x00"):
        parts = seg.translate(_TO_QUANT).split("\x01")
        for p in parts[:-1]:
            if len(p) > 1:
                out.append(p[:-1])
        if parts[-1]:
            out.append(parts[-1])
    return out


def _required_literals_scan(pattern):
    out, seg, depth, i, n = [], [], 0, 0, len(pattern)

    def flush():
        if seg and depth == 0:
            out.append("".join(seg))
        seg.clear()

    while i < n:
        c = pattern[i]
        if c == "\\":
            nxt = pattern[i + 1] if i + 1 < n else ""
            if nxt == "" or nxt.isalnum():
                # class, anchor, back-reference or a numeric escape (\000,
                # \x41, \x{41}, \pL, \p{Greek}): what follows it up to the
                # next non-alphanumeric is part of it or not required
                flush()
                i += 2
                while i < n and pattern[i].isalnum():
                    i += 1
                if i < n and pattern[i] == "{":
                    j = pattern.find("}", i)
                    i = n if j < 0 else j + 1
                continue
            if i + 2 < n and pattern[i + 2] in _QUANTIFIERS:
                flush()
            else:
                seg.append(nxt)
            i += 2
            continue
        if c == "[":
            flush()
            j = i + 1
            if j < n and pattern[j] == "^":
                j += 1
            if j < n and pattern[j] == "]":
                j += 1
            while j < n and pattern[j] != "]":
                j += 2 if pattern[j] == "\\" else 1
            i = j + 1
            continue
        if c == "(":
            flush()
            depth += 1
        elif c == ")":
            flush()
            depth = max(0, depth - 1)
        elif c in ".^$+":
            flush()
        elif c == "{":
            # a repeat count (or a literal brace): nothing up to "}" is required
            flush()
            j = pattern.find("}", i)
            i = n if j < 0 else j + 1
            continue
        elif c in _QUANTIFIERS:
            flush()
        elif i + 1 < n and pattern[i + 1] in _QUANTIFIERS:
            flush()
        else:
            seg.append(c)
        i += 1
    flush()
    return out


@functools.lru_cache(maxsize=4096)
def _matcher(s1):
    """[casefolded s1, required literals, regex] - cache lookups compare every
    new problem against every cached one.  The regex is compiled on the first
    comparison its literals do not rule out (``_NOT_COMPILED`` until then,
    None if it does not compile)."""
    return [common.go_fold(s1), required_literals(s1), _NOT_COMPILED]


def _match_string(s1, s2):
    """``strings.EqualFold(s1, s2)`` or ``regexp.MatchString(s1, s2)``
    (reference ``internal/types/qaengine/problem.go:matchString``)."""
    m = _matcher(s1)
    if m[0] == common.go_fold(s2):
        return True
    lits = m[1]
    if lits is not None:
        for lit in lits:
            if lit not in s2:
                return False
    rx = m[2]
    if rx is _NOT_COMPILED:
        try:
            import warnings
            with warnings.catch_warnings():     # "[--" etc.: Python's FutureWarning; RE2 is silent
                warnings.simplefilter("ignore", FutureWarning)
                rx = re.compile(_go_regex(s1))
        except re.error as e:
            log.debug("Unable to compile string %s : %s", s1, e)
            rx = None
        m[2] = rx
    return rx is not None and rx.search(s2) is not None


def _go_regex(p):
    """Translate the few RE2-only constructs to Python syntax."""
    return p.replace("(?P<", "(?P<").replace("\\z", "\\Z")


def _new_problem(t, desc, context, default, opts):
    resolved = False
    answer = []
    if desc == "":
        raise ProblemError("Empty Description")
    default = [d for d in (default or [])]
    opts = list(opts or [])
    if t == MULTISELECT:
        if len(opts) == 0:
            resolved = True
        folded = {common.go_fold(o) for o in opts}   # common.is_string_present for every default at once
        for d in default:
            if common.go_fold(d) not in folded:
                raise ProblemError("Default value [%s] not present in options [%s]" % (d, opts))
    elif t == SELECT:
        if len(opts) == 0:
            raise ProblemError("Atleast one option is required for question %s" % desc)
        if len(opts) == 1:
            answer = list(opts)
            resolved = True
        if len(default) > 1:
            log.warning("Only one default is allowed for question %s. Setting default as first value %s", desc, default)
            default = [default[0]]
        if len(default) == 0:
            default = [opts[0]]
        elif not common.is_string_present(opts, default[0]):
            raise ProblemError("Default value [%s] not present in options [%s]" % (default[0], opts))
    elif t == CONFIRM:
        if opts:
            log.warning("Options is not required for confirm question type : %s", desc)
        if len(default) > 1:
            log.warning("Only one default is allowed for question %s.", desc)
        if len(default) == 0:
            default = ["false"]
        else:
            try:
                _parse_bool(default[0])
                default = [default[0]]
            except ValueError:
                log.warning("Unable to parse default value %s. Setting as false", default[0])
                default = ["false"]
    elif t in (INPUT, MULTILINE):
        if len(default) > 1:
            log.warning("Only one default value supported for %s. Ignoring others.", desc)
            default = [default[0]]
        if opts:
            log.warning("Options not supported for %s. Ignoring options.", desc)
            opts = []
    elif t == PASSWORD:
        if default:
            log.warning("Default not supported for %s. Ignoring default.", desc)
            default = []
        if opts:
            log.warning("Options not supported for %s. Ignoring options.", desc)
            opts = []
    return Problem(_next_id(), desc, list(context or []), t, default, opts, answer, resolved)


def new_select_problem(desc, context, default, opts):
    return _new_problem(SELECT, desc, context, [default], opts)


def new_multiselect_problem(desc, context, default, opts):
    return _new_problem(MULTISELECT, desc, context, default, opts)


def new_confirm_problem(desc, context, default):
    return _new_problem(CONFIRM, desc, context, ["true" if default else "false"], [])


def new_input_problem(desc, context, default):
    return _new_problem(INPUT, desc, context, [default], [])


def new_multiline_input_problem(desc, context, default):
    return _new_problem(MULTILINE, desc, context, [default], [])


def new_password_problem(desc, context):
    return _new_problem(PASSWORD, desc, context, [], [])


class _DescIndex:
    """Which problems of a list may ``match`` a new one (``_match_string``:
    case-folded equality, or the listed description as a regex found in the
    new description).  The reference scans the whole list for every lookup
    (``types/qaengine/cache.go:84-111``), which makes a QA session over n
    services quadratic; this index bounds a lookup by the new description's
    length.

    A listed description is filed under its case-folded text and under one
    ``Q``-character piece of its required literals (:func:`required_literals`),
    the piece whose bucket is smallest when it is filed.  Any string the regex
    matches contains every required literal, hence that piece, so a lookup
    only visits the buckets of the pieces of the new description, plus the
    descriptions without a literal of ``Q`` characters.  Candidates are then
    checked with the full ``matches``, in list order."""

    Q = 6

    def __init__(self, problems):
        self.problems = problems
        self.size = 0
        self.fold = {}
        self.grams = {}
        self.always = set()
        self.where = {}
        for i, p in enumerate(problems):
            self.add(i, p.desc)

    def fresh(self, problems):
        return problems is self.problems and len(problems) == self.size

    def add(self, pos, desc):
        fold = common.go_fold(desc)
        self.fold.setdefault(fold, set()).add(pos)
        lits = _matcher(desc)[1]
        gram = None
        if lits:
            best = None
            q = self.Q
            for lit in lits:
                for j in range(len(lit) - q, -1, -1):
                    g = lit[j:j + q]
                    n = len(self.grams.get(g, ()))
                    if best is None or n < best[0]:
                        best = (n, g)
                        if n == 0:
                            break
                if best is not None and best[0] == 0:
                    break
            if best is not None:
                gram = best[1]
        if gram is None:
            self.always.add(pos)
        else:
            self.grams.setdefault(gram, set()).add(pos)
        self.where[pos] = (fold, gram)
        if pos >= self.size:
            self.size = pos + 1

    def remove(self, pos):
        fold, gram = self.where.pop(pos)
        self.fold[fold].discard(pos)
        if gram is None:
            self.always.discard(pos)
        else:
            self.grams[gram].discard(pos)

    def candidates(self, desc):
        out = set(self.fold.get(common.go_fold(desc), ()))
        out |= self.always
        grams, q = self.grams, self.Q
        windows = len(desc) - q + 1
        if len(grams) < windows:
            # fewer filed pieces than windows of the description (a small
            # cache): the same set, found by substring tests of the pieces
            for g, b in grams.items():
                if b and g in desc:
                    out |= b
        else:
            for i in range(windows):
                b = grams.get(desc[i:i + q])
                if b:
                    out |= b
        return sorted(out)

    def first_match(self, p, pred=None):
        """Index of the first listed problem that ``matches(p)`` (and passes
        ``pred``), or -1: the result of the reference's linear scan."""
        problems = self.problems
        for i in self.candidates(p.desc):
            cp = problems[i]
            if cp.matches(p) and (pred is None or pred(cp)):
                return i
        return -1


class Cache:
    """``kind: QACache`` file (cache.go)."""

    def __init__(self, file=""):
        self.api_version = SCHEME_GROUP_VERSION
        self.kind = QACACHE_KIND
        self.name = ""
        self.file = file
        self.problems = []
        self._lock = threading.Lock()
        self._chunks = {}  # id(problem) -> (problem, its to_yaml(), emitted YAML of its list item)
        # write-behind: answers are persisted at the engine chain's flush points
        # (before a blocking prompt, when the command ends) instead of one full
        # rewrite per answer
        self.write_behind = False
        self.dirty = False

    def _head(self):
        d = {}
        if self.api_version:
            d["apiVersion"] = self.api_version
        d["kind"] = self.kind
        if self.name:
            d["metadata"] = {"name": self.name}
        return d

    def to_yaml(self):
        d = self._head()
        if self.problems:
            d["spec"] = {"solutions": [p.to_yaml() for p in self.problems]}
        return d

    @classmethod
    def from_yaml(cls, d, file=""):
        d = as_map(d)
        c = cls(file)
        c.api_version = as_str(d.get("apiVersion"))
        c.kind = as_str(d.get("kind"))
        c.name = as_str(as_map(d.get("metadata")).get("name"))
        c.problems = [Problem.from_yaml(x) for x in as_list(as_map(d.get("spec")).get("solutions"))]
        return c

    def load(self):
        """Load and merge the cache file (cache.go:45-60)."""
        from .base import read_document
        try:
            other = read_document(self.file, lambda d: Cache.from_yaml(d, self.file), "QA_CACHE")
        except Exception as e:  # noqa: BLE001 - logged, then returned to StartEngine
            log.error("Unable to load cache : %s", common.go_error_text(e))
            raise
        self._merge(other)
        for p in self.problems:
            p.resolved = True

    _ITEM_PREFIX = "spec:\n  solutions:\n"

    def _item_text(self, p):
        d = p.to_yaml()
        hit = self._chunks.get(id(p))
        if hit is not None and hit[0] is p and hit[1] == d:
            return hit[2]
        text = yamlio.dump({"spec": {"solutions": [d]}})[len(self._ITEM_PREFIX):]
        self._chunks[id(p)] = (p, d, text)
        return text

    def render(self):
        """The cache file text.  Every solution's list item is emitted once and
        reused (the reference re-encodes the whole cache on every answer, which
        makes a QA session quadratic); the result is byte-identical to encoding
        :meth:`to_yaml` in one go."""
        if not self.problems:
            return yamlio.dump(self.to_yaml())
        head = self._head()
        live = {id(p) for p in self.problems}
        for k in [k for k in self._chunks if k not in live]:
            del self._chunks[k]
        return yamlio.dump(head) + self._ITEM_PREFIX + "".join(self._item_text(p) for p in self.problems)

    def write(self):
        try:
            common.write_text(self.file, self.render())
        except OSError as e:
            log.warning("Unable to write cache : %s", e)
            raise

    def add_problem_solution(self, p):
        if p.type == PASSWORD:
            log.debug("Passwords are not added to the cache.")
            return False
        if not p.resolved:
            log.warning("Unresolved problem. Not going to be added to cache.")
            return False
        with self._lock:
            idx = self._index()
            i = idx.first_match(p)
            if i >= 0:
                log.warning("A solution already exists in cache for [%s], rewriting", p.desc)
                self.problems[i] = p.copy()
                idx.remove(i)
                idx.add(i, p.desc)
            else:
                idx.add(len(self.problems), p.desc)
                self.problems.append(p.copy())
            if self.write_behind:
                self.dirty = True
            else:
                try:
                    self.write()
                except OSError as e:
                    log.error("Unable to persist cache : %s", e)
        return True

    def flush(self):
        """Write pending answers (write-behind mode)."""
        with self._lock:
            if not self.dirty:
                return
            self.dirty = False
            try:
                self.write()
            except OSError as e:
                log.error("Unable to persist cache : %s", e)

    def discard_pending(self):
        """The file is about to be deleted: pending answers need no write (the
        reference's writes of them would be deleted with it)."""
        with self._lock:
            self.dirty = False

    def get_solution(self, p):
        if p.resolved:
            log.warning("Problem already solved.")
            return p
        with self._lock:
            i = self._index().first_match(p, lambda cp: cp.resolved)
        if i >= 0:
            p.set_answer(self.problems[i].answer)
            return p
        raise ProblemError("The problem %s was not found in the cache" % p.go_plus_v())   # cache.go:125 (%+v)

    def _index(self):
        idx = self.__dict__.get("_desc_index")
        if idx is None or not idx.fresh(self.problems):
            idx = self._desc_index = _DescIndex(self.problems)
        return idx

    def _merge(self, other):
        # the reference's inner ``continue`` does not skip duplicates;
        # "fixed" compat drops later duplicates as the log message intends.
        from ..utils.constants import settings
        idx = self._index()
        for p in other.problems:
            if idx.first_match(p) >= 0:
                log.warning("There are two answers for %s in cache. Ignoring latter ones.", p.desc)
                if settings.fixed:
                    continue
            idx.add(len(self.problems), p.desc)
            self.problems.append(p)
