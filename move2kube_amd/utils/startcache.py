"""Reader of the build's start-up cache (``move2kube_amd/_startcache.bin``).

Every CLI run is a fresh process, and a few things it does on its first use of
them cost the same in every process although their inputs ship with the
package: parsing the packaged Go templates (``utils/gotemplate.py``, a
character-level lexer in Python: 10-300 us per template) and compiling the
package's regular expressions (``sre_compile`` is Python too: 100-400 us for a
non-trivial pattern).  ``ops/startcache_build.py`` does both at build time and
stores the results; a process reads the file once, on the first lookup.

* templates: the parse tree (:meth:`gotemplate.Template.to_data`) keyed by the
  template's source text, so an edited or user-supplied template simply misses
  and is parsed as before; the whole section is ignored when
  ``utils/gotemplate.py`` is not the file the trees were built by (size and
  mtime, the ``.pyc`` rule, or else its SHA-1).
* regular expressions: the arguments ``sre_compile.compile`` hands to
  ``_sre.compile`` for ``(pattern, flags)``; only used by an interpreter whose
  version string and ``_sre`` engine (``MAGIC``, ``CODESIZE``) match the
  builder's.  The build checks each entry compiles to a pattern equal to
  ``re.compile(pattern, flags)`` (``Pattern.__eq__`` compares the compiled
  code), and so does ``tests/test_startcache.py``.

A missing, unreadable or foreign file disables the cache; nothing else
changes.  ``M2K_STARTCACHE=0`` turns it off.
"""

import _thread

import marshal
import os
import sys

FILENAME = "_startcache.bin"
_HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(os.path.dirname(_HERE), FILENAME)
GOTEMPLATE_SRC = os.path.join(_HERE, "gotemplate.py")          # the node classes
GOTEMPLATE_PARSE_SRC = os.path.join(_HERE, "gotemplate_parse.py")  # the parser


def parser_sources():
    return (GOTEMPLATE_SRC, GOTEMPLATE_PARSE_SRC)

_state = None  # None: not read yet; False: unusable; else (templates, regexes)
_lock = _thread.RLock()


def interpreter_tag():
    import _sre
    return "%s|%s|%d|%d" % (sys.version, sys.implementation.cache_tag, _sre.MAGIC, _sre.CODESIZE)


def source_stamp(paths):
    """(newest mtime, total size) of the files ``paths``."""
    sts = [os.stat(p) for p in ((paths,) if isinstance(paths, str) else paths)]
    return max(int(st.st_mtime) for st in sts), sum(st.st_size for st in sts)


def source_digest(paths):
    import hashlib
    h = hashlib.sha1()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _load():
    with _lock:   # threads asking at once read the file once; none sees it half read
        return _state if _state is not None else _read()


def _read():
    """Read the file (under ``_lock``).  ``_state`` is assigned once, when the
    outcome is known: the lock-free readers in :func:`template` and
    :func:`regex` must never see a provisional value (a thread that saw
    ``False`` while another was still reading would parse from source)."""
    global _state
    st = False
    try:
        st = _read_file()
    finally:
        _state = st
    return _state


def _read_file():
    if os.environ.get("M2K_STARTCACHE", "1") == "0":
        return False
    try:
        with open(PATH, "rb") as f:
            tag, stamp, templates, regexes = marshal.loads(f.read())
    except (OSError, ValueError, EOFError, TypeError):
        return False
    if tag != interpreter_tag():
        return False
    if not _same_parser(stamp):
        templates = {}
    return (templates, regexes)


def _same_parser(stamp):
    """Whether utils/gotemplate.py is the file the trees were built by: its
    size and mtime, or (an installed copy has new mtimes) its SHA-1."""
    try:
        mtime, size, digest = stamp
        if (mtime, size) == source_stamp(parser_sources()):
            return True
        return source_digest(parser_sources()) == digest
    except (OSError, ValueError, TypeError):
        return False


def template(src):
    """The parse-tree data of the packaged template ``src``, or None."""
    st = _state if _state is not None else _load()
    if not st:
        return None
    blob = st[0].get(src)
    return None if blob is None else marshal.loads(blob)


def regex(pattern, flags=0):
    """A compiled pattern equal to ``re.compile(pattern, flags)`` built from
    the cache without ``sre_compile``, or None when it is not cached."""
    st = _state if _state is not None else _load()
    if not st:
        return None
    blob = st[1].get((pattern, int(flags)))
    if blob is None:
        return None
    import _sre
    final_flags, code, groups, groupindex, indexgroup = marshal.loads(blob)
    try:
        return _sre.compile(pattern, final_flags, code, groups, groupindex, indexgroup)
    except (TypeError, ValueError, RuntimeError):
        return None


def reset():
    """Forget what was read (tests)."""
    global _state
    _state = None
