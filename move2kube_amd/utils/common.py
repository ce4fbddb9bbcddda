"""Common helpers (reference ``internal/common/utils.go:47-718``).

File-system discovery goes through :mod:`move2kube_amd.utils.fsindex` (one
indexed walk shared by every planner instead of the reference's >=8 serial
``filepath.Walk`` passes); the hashing/naming primitives are bit-exact with
the reference (CRC-64/ECMA, FNV-64a, SHA-256 truncation).
"""

import os
import shutil

from . import log, yamlio
from .constants import (DEFAULT_FILE_PERMISSION, GROUP_NAME, SCHEME_VERSION)
from .lazyre import lazy as _lazy_re

_ATOMS = (str, int, float, bool, type(None))


def deep_copy(o):
    """``copy.deepcopy`` of a JSON-shaped tree (plain dicts/lists of scalars)
    without the copy module's memo and dispatch; anything else goes to
    ``copy.deepcopy``."""
    t = type(o)
    if t is dict:
        return {k: (v if type(v) in _ATOMS else deep_copy(v)) for k, v in o.items()}
    if t is list:
        return [v if type(v) in _ATOMS else deep_copy(v) for v in o]
    if t in _ATOMS:
        return o
    import copy
    return copy.deepcopy(o)


def shallow_copy(obj):
    """``copy.copy`` of a plain class instance (``__dict__`` and ``__slots__``)."""
    cls = type(obj)
    new = cls.__new__(cls)
    d = getattr(obj, "__dict__", None)
    if d is not None:
        new.__dict__.update(d)
    for klass in cls.__mro__:
        for name in klass.__dict__.get("__slots__", ()):
            if name not in ("__dict__", "__weakref__") and hasattr(obj, name):
                setattr(new, name, getattr(obj, name))
    return new


# ---------------------------------------------------------------------------
# hashing primitives (native when available; pure-python fallback is exact)
# ---------------------------------------------------------------------------

_CRC64_ECMA_POLY = 0xC96C5795D7870F42
_CRC_TABLE = None


def _crc64_table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        tbl = []
        for i in range(256):
            crc = i
            for _ in range(8):
                crc = (crc >> 1) ^ _CRC64_ECMA_POLY if crc & 1 else crc >> 1
            tbl.append(crc)
        _CRC_TABLE = tbl
    return _CRC_TABLE


def crc64_ecma_py(data):
    """Go ``crc64.Checksum(data, crc64.MakeTable(0xC96C5795D7870F42))``."""
    tbl = _crc64_table()
    crc = 0xFFFFFFFFFFFFFFFF
    for b in data:
        crc = tbl[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFFFFFFFFFF


def fnv64a_py(data):
    """Go ``hash/fnv`` New64a over ``data``."""
    h = 0xCBF29CE484222325
    for b in data:
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def go_bytes(s):
    """The bytes of a Go string held as ``str``: UTF-8, with the
    surrogate-escaped bytes of a name or file that is not UTF-8 given back as
    they were read (``str.encode()`` would fail on them)."""
    try:
        return s.encode("utf-8", "surrogateescape")
    except UnicodeEncodeError:   # a lone surrogate from elsewhere: keep it encodable
        return s.encode("utf-8", "surrogatepass")


def crc64_ecma(data):
    from ..ops import native
    if isinstance(data, str):
        data = go_bytes(data)
    return native.crc64_ecma(data)


def fnv64a(data):
    from ..ops import native
    if isinstance(data, str):
        data = go_bytes(data)
    return native.fnv64a(data)


def get_sha256_hash(s):
    import hashlib  # OpenSSL start-up cost; only long names need it
    return hashlib.sha256(s.encode("utf-8", "surrogateescape")).hexdigest()


# ---------------------------------------------------------------------------
# file discovery
# ---------------------------------------------------------------------------

def get_files_by_ext(input_path, exts):
    """Files under ``input_path`` whose extension is in ``exts`` (lexical walk order).

    Raises FileNotFoundError if ``input_path`` does not exist (reference returns an error)."""
    from .fsindex import get_index
    files = get_index(input_path).files_by_ext(exts)
    log.debug("No of files with %s ext identified : %d", "[" + " ".join(exts) + "]", len(files))
    return files


def get_files_by_name(input_path, names):
    from .fsindex import get_index
    files = get_index(input_path).files_by_name(names)
    log.debug("No of files with %s names identified : %d", "[" + " ".join(names) + "]", len(files))
    return files


# ---------------------------------------------------------------------------
# YAML / JSON IO
# ---------------------------------------------------------------------------

def read_bytes(path):
    """Contents of a regular file found in a source tree.  Opened without
    blocking and checked with fstat, so a FIFO, socket or device that happens
    to carry a .yaml/.py/Dockerfile name is an error, not a hang (ReadFile
    in the reference blocks forever on a FIFO with no writer)."""
    import errno
    import stat
    fd = os.open(path, os.O_RDONLY | os.O_NONBLOCK | os.O_CLOEXEC)
    try:
        mode = os.fstat(fd).st_mode
        if stat.S_ISDIR(mode):   # Go opens a directory and fails on the read
            e = IsADirectoryError(errno.EISDIR, os.strerror(errno.EISDIR), path)
            e.go_op = "read"
            raise e
        if not stat.S_ISREG(mode):
            raise OSError(errno.EINVAL, "not a regular file", path)
        with open(fd, "rb", closefd=False) as f:
            return f.read()
    finally:
        os.close(fd)


_GO_SPACE = ("\t\n\v\f\r \x85\xa0\u1680\u2000\u2001\u2002\u2003\u2004\u2005\u2006\u2007\u2008\u2009"
             "\u200a\u2028\u2029\u202f\u205f\u3000")


def go_trim_space(s):
    """``strings.TrimSpace`` / ``bytes.TrimSpace``: Unicode white space
    (``unicode.IsSpace``), not Python's wider ``str.strip()`` set."""
    return s.strip(_GO_SPACE)


def go_scan_lines(data):
    """``bufio.Scanner`` with ``ScanLines`` over ``data`` (bytes): lines split at
    LF with one CR before it dropped, a last line without LF kept; a line of
    64 KiB or more stops the scan (``ErrTooLong``).  -> (lines, too_long)."""
    lines = []
    start, n = 0, len(data)
    while start < n:
        end = data.find(b"\n", start)
        stop = n if end < 0 else end
        if stop - start >= 64 * 1024 or (end < 0 and n - start >= 64 * 1024):
            return lines, True
        line = data[start:stop]
        if line.endswith(b"\r"):
            line = line[:-1]
        lines.append(line)
        if end < 0:
            break
        start = end + 1
    return lines, False


def read_text(path):
    return read_bytes(path).decode("utf-8", errors="surrogateescape")


def write_text(path, text, mode=DEFAULT_FILE_PERMISSION):
    """``ioutil.WriteFile(path, data, mode)``: a new file is created with
    ``mode & ~umask``; an existing one is truncated and keeps its permissions."""
    data = text.encode("utf-8", errors="surrogateescape") if isinstance(text, str) else text
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_CLOEXEC, mode)
    with open(fd, "wb") as f:
        f.write(data)


def yaml_attr_present(path, attr):
    """``YamlAttrPresent`` (utils.go:122-140): decode into a
    ``map[string]interface{}`` and look the attribute up."""
    try:
        text = read_text(path)
    except OSError as e:
        log.warning("Error in reading yaml file %s: %s. Skipping", path, go_path_error(e, "open"))
        return False, None
    try:
        data = yamlio.load(text)
    except yamlio.YAMLError as e:
        log.warning("Error in unmarshalling yaml file %s: %s. Skipping", path, e)
        return False, None
    if data is not None and not isinstance(data, dict):
        tag = "!!seq" if isinstance(data, list) else "!!bool" if isinstance(data, bool) else \
            "!!int" if isinstance(data, int) else "!!float" if isinstance(data, float) else "!!str"
        log.warning("Error in unmarshalling yaml file %s: %s. Skipping", path,
                    "yaml: unmarshal errors:\n  line 1: cannot unmarshal %s into map[string]interface {}" % tag)
        return False, None
    if isinstance(data, dict) and attr in data:
        log.debug("%s file has %s attribute", path, attr)
        return True, data[attr]
    return False, None


def write_yaml(output_path, data, sort_maps=False):
    """Write ``data`` (a plain structure or an object with ``to_yaml()``) like
    go-yaml v3; a write error is logged as ``common.WriteYaml`` logs it
    (utils.go:159-176) and raised for the caller's own line."""
    if hasattr(data, "to_yaml"):
        data = data.to_yaml()
    text = yamlio.dump(data, sort_maps=sort_maps)
    try:
        write_text(output_path, text)
    except OSError as e:
        log.error("Error writing yaml to file. error: %s,  outputPath %s", go_path_error(e, "open"), output_path)
        raise


def read_yaml(path):
    return yamlio.load(read_text(path))


def parse_group_version(gv):
    """k8s ``schema.ParseGroupVersion``."""
    if gv == "" or gv == "/":
        return "", ""
    parts = gv.split("/")
    if len(parts) == 1:
        return "", parts[0]
    if len(parts) == 2:
        return parts[0], parts[1]
    raise ValueError("unexpected GroupVersion string: %s" % gv)


class Move2KubeYamlError(ValueError):
    pass


def read_move2kube_yaml(path, raw=True):
    """Read a move2kube-group YAML (plan, cache, cluster metadata ...).

    Checks that ``apiVersion``'s group is ``move2kube.konveyor.io`` and warns on a
    version mismatch (``internal/common/utils.go:210-251``).  Returns the decoded
    document (scalars kept as raw strings when ``raw``)."""
    return read_move2kube_yaml_text(path, raw)[1]


def read_move2kube_yaml_text(path, raw=True):
    """:func:`read_move2kube_yaml` -> (file text, document)."""
    try:
        text = read_text(path)
    except OSError as e:
        log.debug("Failed to read the yaml file at path %s Error: %r", path, go_path_error(e, "open"))
        raise
    try:
        data = yamlio.load(text)
    except yamlio.YAMLError as e:
        log.debug("Error occurred while unmarshalling yaml file at path %s Error: %r", path, str(e))
        raise
    if data is None:
        data = {}
    if not isinstance(data, dict):
        err = Move2KubeYamlError(yamlio.go_unmarshal_type_error(text, data))
        log.debug("Error occurred while unmarshalling yaml file at path %s Error: %r", path, str(err))
        raise err
    if "apiVersion" not in data:
        err = Move2KubeYamlError("Did not find apiVersion in the yaml file at path %s" % path)
        log.debug(str(err))
        raise err
    gv = data["apiVersion"]
    if not isinstance(gv, str):
        err = Move2KubeYamlError("The apiVersion is not a string in the yaml file at path %s" % path)
        log.debug(str(err))
        raise err
    try:
        group, version = parse_group_version(gv)
    except ValueError as e:
        log.debug("Failed to parse the apiVersion %s Error: %r", gv, str(e))
        raise Move2KubeYamlError(str(e))
    if group != GROUP_NAME:
        err = Move2KubeYamlError("The file at path %s doesn't have the correct group. Expected group %s Actual group %s"
                                 % (path, GROUP_NAME, group))
        log.debug(str(err))
        raise err
    if version != SCHEME_VERSION:
        log.warning("The file at path %s was generated using a different version. File version is %s and move2kube version is %s",
                    path, version, SCHEME_VERSION)
    return text, (yamlio.load_raw(text) if raw else data)


def write_json(output_path, data):
    import json
    write_text(output_path, json.dumps(data, separators=(",", ":")) + "\n")


def read_json(path):
    from . import fastjson
    with open(path, "rb") as f:
        return fastjson.loads(f.read())


# ---------------------------------------------------------------------------
# naming
# ---------------------------------------------------------------------------

def get_image_name_and_tag(image):
    parts = image.split("/")
    it = parts[-1].split(":")
    name = it[0]
    tag = "latest" if len(it) == 1 else it[1]
    return name, tag


def normalize_for_filename(name):
    processed = make_file_name_compliant(name)
    if len(processed) > 15:
        processed = processed[:15]
    return processed + "-" + format(crc64_ecma(go_bytes(name)), "x")


def go_lower(s):
    """Go ``strings.ToLower``: the simple (one-to-one) lowercase mapping of
    every rune.  ``str.lower`` applies the full mapping, which differs for one
    character only: U+0130 (capital I with dot) becomes "i" + U+0307 there and
    "i" in Go."""
    if s.isascii():
        return s.lower()
    return s.replace("\u0130", "i").lower()


_FOLD = {}


def _go_fold_char(c):
    f = c.casefold()
    if len(f) != 1:        # a full (one-to-many) folding: Go folds simply
        f = c.lower()
        if len(f) != 1:
            f = c
    _FOLD[c] = f
    return f


def go_fold(s):
    """Key under which Go ``strings.EqualFold`` calls two strings equal: the
    simple case folding of every rune.  ``str.casefold`` applies the full
    folding, so it equates "Straße" with "STRASSE", which EqualFold does not."""
    if s.isascii():
        return s.lower()
    fold = _FOLD
    return "".join([fold.get(c) or _go_fold_char(c) for c in s])


def normalize_for_service_name(svc_name):
    new = go_lower(svc_name.replace(".", "-").replace("_", "-"))  # [._] -> "-" (utils.go:297-305)
    if new != svc_name:
        log.info("Changing service name to %s from %s", svc_name, new)
    return new


def is_string_present(lst, value):
    """Case-insensitive membership (Go ``strings.EqualFold``)."""
    if not lst:
        return False
    if value in lst:  # an exact match: the common case, no folding
        return True
    v = go_fold(value)
    for x in lst:
        if go_fold(x) == v:
            return True
    return False


def is_int_present(lst, value):
    return value in (lst or [])


def merge_string_slices(a, b):
    """``a`` plus the items of ``b`` not already in it (``strings.EqualFold``),
    in order; linear, where ``IsStringPresent`` per item is quadratic."""
    a = list(a or [])
    if not b:
        return a
    seen = {go_fold(x) for x in a}
    for item in b:
        f = go_fold(item)
        if f not in seen:
            seen.add(f)
            a.append(item)
    return a


def merge_int_slices(a, b):
    a = list(a or [])
    for item in b or []:
        if item not in a:
            a.append(item)
    return a


def merge_string_maps(a, b):
    out = dict(a or {})
    out.update(b or {})
    return out


def get_string_from_template(tpl, config):
    """GetStringFromTemplate (utils.go:347-357): a template that fails to
    execute is reported with its text and data before the error is returned
    (a parse error panics in the reference, ``template.Must``; it raises here)."""
    from . import gotemplate
    t = gotemplate.compiled(tpl)
    try:
        return t.execute(config)
    except gotemplate.TemplateError:
        log.warning("Unable to translate template %s to string using the data %s", log.go_quote(tpl),
                    gotemplate.go_sprint(config))
        raise


def write_template_to_file(tpl, config, write_path, mode):
    write_text(write_path, get_string_from_template(tpl, config), mode)


_TOKEN_RE = _lazy_re(r"[^a-zA-Z0-9]+")


def get_closest_matching_string(options, search):
    """Option with least Wagner-Fischer distance (ins=1, del=1, sub=2) to ``search``
    after stripping non-alphanumerics and lower-casing (``utils.go:377-401``)."""
    if not options:
        return ""
    return get_closest_matching_strings(options, [search])[0]


_FILENAME_INVALID = _lazy_re(r"[^a-zA-Z0-9\-.]+")
_ASCII_ALNUM = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"
# str.translate tables deleting the allowed characters: an empty result means
# there is nothing to replace, and the regex is never compiled
_DROP_FILENAME_OK = str.maketrans("", "", _ASCII_ALNUM + "-.")
_DROP_DNS_OK = str.maketrans("", "", _ASCII_ALNUM[:26] + _ASCII_ALNUM[52:] + "-.")


def make_file_name_compliant(name):
    if not name:
        log.error("The input name is empty.")
        return ""
    base = os.path.basename(name.rstrip("/")) or "/"
    processed = _FILENAME_INVALID.sub("-", base) if base.translate(_DROP_FILENAME_OK) else base
    if len(processed) > 63:
        log.debug("Warning: The processed name %r is longer than 63 characters long.", processed)
    if processed[0] in "-." or processed[-1] in "-.":
        log.debug("Warning: The first and/or last characters of the name %r are not alphanumeric.", processed)
    return processed


_DNS_INVALID = _lazy_re(r"[^a-z0-9\-.]")


def make_string_dns_name_compliant(s):
    low = go_lower(s)
    name = _DNS_INVALID.sub("-", low) if low.translate(_DROP_DNS_OK) else low
    if name and (name[0] in "-." or name[-1] in "-."):
        log.warning("The first and/or last characters of the string %r are not alphanumeric.", s)
    return name


def _go_byte_prefix(s, n):
    """``s[:n]`` of a Go string: its first n UTF-8 bytes.  A rune cut in two
    leaves bytes that Go reads one invalid byte at a time; here they become
    one lone surrogate each, which the DNS pattern replaces like Go does."""
    return s.encode("utf-8", "surrogateescape")[:n].decode("utf-8", "surrogateescape")


def make_string_dns_subdomain_name_compliant(s):
    """MakeStringDNSSubdomainNameCompliant (utils.go:461-469): lengths are
    UTF-8 byte counts, as in Go."""
    name = s
    if len(name.encode("utf-8", "surrogateescape")) > 253:
        h = get_sha256_hash(name)
        name = _go_byte_prefix(name, 253 - 65) + "-" + h
    return make_string_dns_name_compliant(name)


def make_string_dns_label_name_compliant(s):
    """MakeStringDNSLabelNameCompliant (utils.go:477-486), byte lengths."""
    name = s
    if len(name.encode("utf-8", "surrogateescape")) > 63:
        h = get_sha256_hash(name)[:32]
        name = _go_byte_prefix(name, 63 - 33) + "-" + h
    return make_string_dns_name_compliant(name)


def clean_and_find_common_directory(paths):
    return find_common_directory([go_clean(p) for p in paths])


def find_common_directory(paths):
    if not paths:
        return ""
    common = paths[0]
    while common != "/":
        if all((p + "/").startswith(common + "/") for p in paths):
            break
        nxt = go_dir(common)
        if nxt == common:  # relative paths bottom out at "." (the reference would spin here)
            break
        common = nxt
    return common


def copy_file(dst, src):
    """``CopyFile`` (utils.go:587-615): the destination is opened like
    ``os.OpenFile(dst, O_WRONLY|O_CREATE|O_TRUNC, DefaultFilePermission)``."""
    with open(src, "rb") as fsrc, open(os.open(dst, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_CLOEXEC,
                                               DEFAULT_FILE_PERMISSION), "wb") as fdst:
        shutil.copyfileobj(fsrc, fdst)


def unique_strings(xs):
    seen = set()
    out = []
    for x in xs:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def go_errno_text(errno_):
    """Go's ``syscall.Errno`` text (``no such file or directory``)."""
    msg = os.strerror(errno_) if errno_ else ""
    return msg[:1].lower() + msg[1:]


def go_path_error(e, op):
    """An OSError as Go's ``*os.PathError`` prints it: ``<op> <path>: <errno
    text>`` (``mkdir /out: permission denied``, ``open /x/plan: not a
    directory``).  ``os.MkdirAll`` over an existing non-directory reports
    ENOTDIR where Python's ``makedirs`` says EEXIST.  Errors without a path
    keep Python's text."""
    path = getattr(e, "filename", None)
    if path is None or not getattr(e, "errno", None):
        return str(e)
    import errno as _errno
    op = getattr(e, "go_op", op)
    code = e.errno
    if op == "mkdir" and code == _errno.EEXIST:
        code = _errno.ENOTDIR
    return "%s %s: %s" % (op, os.fsdecode(path), go_errno_text(code))


def go_error_text(e, op="open"):
    """Text of an error caught broadly: an OSError with a path as Go's
    ``*os.PathError`` (:func:`go_path_error`), anything else as it is."""
    if isinstance(e, OSError):
        return go_path_error(e, op)
    return str(e)


class GoExecNotFoundError(FileNotFoundError):
    """A command that could not be started, worded as Go's ``os/exec`` does:
    ``exec: "cf": executable file not found in $PATH`` for a name looked up on
    PATH, ``fork/exec /x/cf: no such file or directory`` for a path."""

    def __str__(self):
        return self.args[1] if len(self.args) > 1 else super().__str__()


def go_exec_error(e, name):
    """``e`` (a FileNotFoundError from starting ``name``) with Go's message."""
    if "/" in name:
        text = "fork/exec %s: no such file or directory" % name
    else:
        text = "exec: %s: executable file not found in $PATH" % log.go_quote(name)
    err = GoExecNotFoundError(e.errno, text)
    err.filename = name
    return err


_GO_SIGNALS = ("", "hangup", "interrupt", "quit", "illegal instruction", "trace/breakpoint trap", "aborted",
               "bus error", "floating point exception", "killed", "user defined signal 1", "segmentation fault",
               "user defined signal 2", "broken pipe", "alarm clock", "terminated", "stack fault", "child exited",
               "continued", "stopped (signal)", "stopped", "stopped (tty input)", "stopped (tty output)",
               "urgent I/O condition", "CPU time limit exceeded", "file size limit exceeded",
               "virtual timer expired", "profiling timer expired", "window changed", "I/O possible",
               "power failure", "bad system call")


def go_exit_status(returncode):
    """Go's ``*exec.ExitError`` text for a subprocess return code
    (``exit status 2``, ``signal: killed``; linux/amd64 signal names)."""
    if returncode >= 0:
        return "exit status %d" % returncode
    sig = -returncode
    return "signal: " + (_GO_SIGNALS[sig] if 0 < sig < len(_GO_SIGNALS) else "signal %d" % sig)


def unnamed_temp_file():
    """A read/write binary file with no name, gone when closed - what
    ``tempfile.TemporaryFile`` makes on Linux (``O_TMPFILE`` in the temp dir),
    without importing ``tempfile`` and ``random`` into a cold CLI process."""
    try:
        fd = os.open(os.environ.get("TMPDIR") or "/tmp", os.O_RDWR | os.O_TMPFILE | os.O_CLOEXEC, 0o600)
    except (AttributeError, OSError):
        import tempfile
        return tempfile.TemporaryFile()
    return open(fd, "w+b")


def run_command(argv, **kw):
    """``subprocess.run`` whose missing-executable error reads like Go's."""
    import subprocess
    try:
        return subprocess.run(argv, **kw)
    except FileNotFoundError as e:
        if e.filename in (argv[0], os.fsencode(argv[0]) if isinstance(argv[0], str) else argv[0]):
            raise go_exec_error(e, os.fsdecode(argv[0])) from None
        raise


def _go_not_found(e, argv0):
    return isinstance(e, FileNotFoundError) and e.filename in (argv0, os.fsencode(argv0) if isinstance(argv0, str)
                                                                else argv0)


def run_tool(argv, **kw):
    """:func:`utils.proc.run` (no ``subprocess`` import) whose
    missing-executable error reads like Go's."""
    from . import proc
    try:
        return proc.run(argv, **kw)
    except FileNotFoundError as e:
        if _go_not_found(e, argv[0]):
            raise go_exec_error(e, os.fsdecode(argv[0])) from None
        raise


def run_tools(argvs, **kw):
    """:func:`utils.proc.run_many` with Go's missing-executable errors."""
    from . import proc
    out = proc.run_many(argvs, **kw)
    for i, r in enumerate(out):
        if _go_not_found(r, argvs[i][0]):
            out[i] = go_exec_error(r, os.fsdecode(argvs[i][0]))
    return out


def go_rel(base, target):
    """Go ``filepath.Rel`` (lexical; error if one is absolute and the other is not)."""
    if os.path.isabs(base) != os.path.isabs(target):
        raise ValueError("Rel: can't make %s relative to %s" % (target, base))
    return os.path.relpath(os.path.normpath(target), os.path.normpath(base))


def go_join(*parts):
    """Go ``filepath.Join``: joins non-empty parts and cleans (an absolute later part
    does NOT reset the path, unlike os.path.join)."""
    ps = [p for p in parts if p]
    if not ps:
        return ""
    return os.path.normpath("/".join(ps)).replace("//", "/")


def go_clean(p):
    if p == "":
        return "."
    c = os.path.normpath(p)
    if c.startswith("//"):
        c = "/" + c.lstrip("/")
    return c


def go_abs(p):
    """Go ``filepath.Abs``: joined with the working directory and cleaned
    (``os.path.abspath`` keeps a leading ``//``, which POSIX allows and Go's
    Clean folds to ``/``)."""
    return go_clean(os.path.abspath(p))


def go_ext(p):
    """Go ``filepath.Ext``: suffix from the final dot in the final element."""
    base = p.rsplit("/", 1)[-1]
    i = base.rfind(".")
    return base[i:] if i >= 0 else ""


def go_base(p):
    if p == "":
        return "."
    p = p.rstrip("/")
    if p == "":
        return "/"
    return p.rsplit("/", 1)[-1]


def go_dir(p):
    d = os.path.dirname(p)
    return go_clean(d) if d else "."


# ---------------------------------------------------------------------------
# strconv / spf13/cast (v1.3.1) parsing
# ---------------------------------------------------------------------------

def go_parse_bool(s):
    """strconv.ParseBool."""
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    raise ValueError("strconv.ParseBool: parsing %s: invalid syntax" % log.go_quote(s))


def _underscore_ok(s):
    """strconv ``underscoreOK``: ``_`` only between digits or after a base prefix."""
    s = s[1:] if s[:1] in "+-" else s
    saw, i, hexa = "^", 0, False
    if len(s) >= 2 and s[0] == "0" and s[1] in "bBoOxX":
        i, saw, hexa = 2, "0", s[1] in "xX"
    for ch in s[i:]:
        if "0" <= ch <= "9" or (hexa and ch in "abcdefABCDEF"):
            saw = "0"
        elif ch == "_":
            if saw != "0":
                return False
            saw = "_"
        elif saw == "_":
            return False
        else:
            saw = "!"
    return saw != "_"


_DIGITS = {16: "0123456789abcdefABCDEF", 10: "0123456789", 8: "01234567", 2: "01"}


def go_parse_int(s, bits=64):
    """strconv.ParseInt(s, 0, bits): sign, base prefixes 0x/0o/0b and a
    leading 0 for octal, underscores by Go's rules, range checked."""
    err = "strconv.ParseInt: parsing %s: " % log.go_quote(s)
    t = s[1:] if s[:1] in "+-" else s
    base, body = 10, t
    if len(t) >= 2 and t[0] == "0":
        p = t[1]
        base, body = ({"x": 16, "X": 16, "o": 8, "O": 8, "b": 2, "B": 2}[p], t[2:]) if p in "xXoObB" else (8, t[1:])
    if "_" in body:
        if not _underscore_ok(s):
            raise ValueError(err + "invalid syntax")
        body = body.replace("_", "")
    if not body or any(c not in _DIGITS[base] for c in body):
        raise ValueError(err + "invalid syntax")
    v = int(body, base)
    v = -v if s[:1] == "-" else v
    if not -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
        raise ValueError(err + "value out of range")
    return v


_FLOAT_DEC = _lazy_re(r"(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?\Z")
_FLOAT_HEX = _lazy_re(r"0[xX](?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?[0-9]+\Z")


def go_parse_float(s):
    """strconv.ParseFloat(s, 64): Go float syntax only (no surrounding
    spaces, no ``+nan``, hexadecimal mantissas need a ``p`` exponent,
    underscores by Go's rules); a finite-looking value beyond float64 is a
    range error rather than infinity."""
    err = "strconv.ParseFloat: parsing %s: " % log.go_quote(s)
    body = s[1:] if s[:1] in "+-" else s
    low = body.lower()
    if low in ("inf", "infinity"):
        return float("-inf") if s[:1] == "-" else float("inf")
    if low == "nan" and body == s:
        return float("nan")
    if not s.isascii():
        raise ValueError(err + "invalid syntax")
    if "_" in body:
        if not _underscore_ok(s):
            raise ValueError(err + "invalid syntax")
        body = body.replace("_", "")
    try:
        if _FLOAT_HEX.match(body):
            v = float.fromhex(body)
        elif _FLOAT_DEC.match(body):
            v = float(body)
        else:
            raise ValueError(err + "invalid syntax")
    except OverflowError:
        v = float("inf")
    if v in (float("inf"), float("-inf")):
        raise ValueError(err + "value out of range")
    return -v if s[:1] == "-" else v


def cast_to_bool(s):
    """spf13/cast ToBoolE (strconv.ParseBool for strings)."""
    if isinstance(s, bool):
        return s
    if isinstance(s, (int, float)):
        return s != 0
    if s is None:
        return False
    return go_parse_bool(str(s))


def cast_to_int(s):
    """spf13/cast v1.3.1 ToIntE: strings through strconv.ParseInt(s, 0, 0),
    no trimming; nil is 0."""
    if s is None:
        return 0
    if isinstance(s, bool):
        return int(s)
    if isinstance(s, int):
        return s
    if isinstance(s, float):
        return go_float_to_int64(s)
    t = str(s)
    try:
        return go_parse_int(t)
    except ValueError:
        raise ValueError("unable to cast %s of type string to int" % log.go_quote(t)) from None


def cast_to_float(s):
    """spf13/cast v1.3.1 ToFloat64E: strings through strconv.ParseFloat."""
    if s is None:
        return 0.0
    if isinstance(s, (bool, int, float)):
        return float(s)
    t = str(s)
    try:
        return go_parse_float(t)
    except ValueError:
        raise ValueError("unable to cast %s of type string to float64" % log.go_quote(t)) from None


def go_float_to_int64(f):
    """Go ``int64(f)`` on amd64: truncation toward zero; NaN, infinities and
    out-of-range values give the CVTTSD2SI "integer indefinite" value,
    math.MinInt64."""
    if f != f or f in (float("inf"), float("-inf")) or not -9.223372036854775808e18 <= f < 9.223372036854775808e18:
        return -(1 << 63)
    return int(f)


def go_bool_str(b):
    return "true" if b else "false"


def get_closest_matching_strings(options, searches):
    """Batched :func:`get_closest_matching_string`: one fused distance+argmin pass
    (gfx950 kernel when large, native bit-parallel CPU otherwise)."""
    from ..ops import editdistance
    if not options or not searches:
        return [""] * len(searches)
    toks = [go_lower(_TOKEN_RE.sub("", o)) for o in options]
    qs = [go_lower(_TOKEN_RE.sub("", s)) for s in searches]
    idx, _ = editdistance.closest_index_list(toks, qs)
    return [options[i] for i in idx]
