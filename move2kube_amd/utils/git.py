"""Git repository discovery without a git library.

Replaces the reference's go-git calls (``internal/common/utils.go:636-718``):
``PlainOpenWithOptions(path, DetectDotGit)``, remotes, HEAD branch and work
tree root, read directly from ``.git/config`` and ``.git/HEAD``.
"""

import os

from . import fsindex
from .lazyre import lazy as _lazy_re


class GitError(Exception):
    pass


def find_repo(path):
    """Walk up from ``path`` to the first directory holding a ``.git`` entry
    (go-git ``dotGitToOSFilesystems`` with ``DetectDotGit``): a ``.git``
    directory is the repository, a ``.git`` file must point at one with
    ``gitdir: ``; either way the walk stops there, and a repository without
    ``HEAD`` does not exist (``Open``: ``ErrRepositoryNotExists``).

    Returns (worktree_root, git_dir).  Inside an ``fsindex.scope()`` every
    directory visited remembers the answer, so the per-service lookups of one
    command share their walks up the tree."""
    cache = fsindex.scoped_cache("git-find")
    p = os.path.abspath(path)
    visited = []
    while True:
        if cache is not None and p in cache:
            result = cache[p]
            break
        visited.append(p)
        dotgit = os.path.join(p, ".git")
        if os.path.isdir(dotgit):
            result = (p, dotgit)
            break
        if os.path.lexists(dotgit):
            result = (p, _gitdir_file(p, dotgit))
            break
        parent = os.path.dirname(p)
        if parent == p:
            result = None
            break
        p = parent
    if cache is not None:
        for v in visited:
            cache[v] = result
    if result is None or isinstance(result[1], GitError):
        raise result[1] if result is not None else GitError("repository does not exist")
    if not os.path.exists(os.path.join(result[1], "HEAD")):
        raise GitError("repository does not exist")
    return result


def _gitdir_file(root, dotgit):
    """``dotGitFileToOSFilesystem``: the first line after ``gitdir: ``,
    relative to the work tree; a GitError (kept in the cache) otherwise."""
    try:
        with open(dotgit, encoding="utf-8", errors="surrogateescape") as f:
            line = f.read()
    except OSError as e:
        from .common import go_path_error
        return GitError(go_path_error(e, "open"))
    prefix = "gitdir: "
    if not line.startswith(prefix):
        return GitError(".git file has no %s prefix" % prefix)
    gd = line[len(prefix):].split("\n")[0].strip()
    return gd if os.path.isabs(gd) else os.path.join(root, gd)


class GitConfigError(GitError):
    pass


def parse_config(text):
    """``git-config`` syntax as go-git's decoder (``gcfg``) reads it: ``[section]``
    and ``[section "subsection"]`` headers (section and variable names are
    case-insensitive, subsections are not; ``[section.sub]`` is the old form of a
    lower-cased subsection), ``name = value`` with double quotes, the escapes
    ``\\ \" \n \t \b``, backslash-newline continuations and ``;``/``#``
    comments outside quotes, and a bare ``name`` (no ``=``).  Returns
    ``[(section, subsection, name, value)]`` in file order."""
    out = []
    section = subsection = None
    i, n, line = 0, len(text), 1

    def fail(what):
        raise GitConfigError("bad config line %d in file config: %s" % (line, what))

    while i < n:
        ch = text[i]
        if ch == "\n":
            line += 1
            i += 1
            continue
        if ch in " \t\r":
            i += 1
            continue
        if ch in "#;":
            while i < n and text[i] != "\n":
                i += 1
            continue
        if ch == "[":
            j = i + 1
            while j < n and (text[j].isalnum() or text[j] in "-."):
                j += 1
            name = text[i + 1:j]
            k = j
            while k < n and text[k] in " \t":
                k += 1
            sub = None
            if k < n and text[k] == '"':
                buf = []
                k += 1
                while k < n and text[k] != '"':
                    if text[k] == "\n":
                        fail("unterminated subsection name")
                    if text[k] == "\\" and k + 1 < n and text[k + 1] != "\n":
                        k += 1
                    buf.append(text[k])
                    k += 1
                if k >= n:
                    fail("unterminated subsection name")
                sub = "".join(buf)
                k += 1
            elif "." in name:
                name, sub = name.split(".", 1)
                sub = sub.lower()
            if k >= n or text[k] != "]" or not name:
                fail("bad section header")
            section, subsection = name.lower(), sub
            i = k + 1
            continue
        if not ch.isalpha():
            fail("bad variable name")
        j = i
        while j < n and (text[j].isalnum() or text[j] == "-"):
            j += 1
        name = text[i:j].lower()
        while j < n and text[j] in " \t":
            j += 1
        if section is None:
            fail("variable outside a section")
        if j >= n or text[j] in "\r\n#;":
            out.append((section, subsection, name, None))
            i = j
            continue
        if text[j] != "=":
            fail("bad variable")
        j += 1
        while j < n and text[j] in " \t":
            j += 1
        buf, keep, quoted = [], 0, False
        while j < n:
            c = text[j]
            if c == "\n" and not quoted:
                break
            if c == "\n":
                fail("unterminated quoted value")
            if c == "\r" and not quoted and text[j + 1:j + 2] == "\n":
                j += 1
                continue
            if c == '"':
                quoted = not quoted
                keep = len(buf)
                j += 1
                continue
            if c in "#;" and not quoted:
                while j < n and text[j] != "\n":
                    j += 1
                break
            if c == "\\":
                e = text[j + 1:j + 2]
                if e == "\n":
                    line += 1
                    j += 2
                    continue
                esc = {"\\": "\\", '"': '"', "n": "\n", "t": "\t", "b": "\b"}.get(e)
                if esc is None:
                    fail("bad escape")
                buf.append(esc)
                keep = len(buf)
                j += 2
                continue
            buf.append(c)
            if c not in " \t" or quoted:
                keep = len(buf)
            j += 1
        if quoted:
            fail("unterminated quoted value")
        out.append((section, subsection, name, "".join(buf[:keep])))
        i = j
    return out


def _read_config(git_dir):
    """Remote name -> URLs (in file order; ``remote.Config().URLs``) from the
    repository's config (the common dir's for a linked work tree).  A config
    go-git cannot parse raises :class:`GitConfigError`."""
    cfg = os.path.join(git_dir, "config")
    if not os.path.exists(cfg):
        cfg = os.path.join(_common_dir(git_dir), "config")
    try:
        with open(cfg, encoding="utf-8", errors="surrogateescape") as f:
            text = f.read()
    except OSError:
        return {}
    remotes = {}
    for section, sub, name, value in parse_config(text):
        if section == "remote" and sub is not None:
            urls = remotes.setdefault(sub, [])
            if name == "url":
                urls.append(value if value is not None else "")
    return remotes


def remote_names(path):
    _, git_dir = find_repo(path)
    return list(_read_config(git_dir).keys())


def _common_dir(git_dir):
    common_file = os.path.join(git_dir, "commondir")
    try:
        with open(common_file) as f:
            return os.path.normpath(os.path.join(git_dir, f.read().strip()))
    except OSError:
        return git_dir


def _ref_exists(git_dir, ref):
    """A loose ``refs/...`` file or a ``packed-refs`` line names ``ref``."""
    for d in (git_dir, _common_dir(git_dir)):
        if os.path.isfile(os.path.join(d, ref)):
            return True
        try:
            with open(os.path.join(d, "packed-refs")) as f:
                for line in f:
                    parts = line.split()
                    if len(parts) == 2 and parts[1] == ref and not line.startswith(("#", "^")):
                        return True
        except OSError:
            pass
    return False


def head_branch(git_dir):
    """``filepath.Base(repo.Head().Name())``: go-git resolves HEAD, so a branch
    without any commit (no ref yet) is an error and gives ''; a detached HEAD
    is named ``HEAD``."""
    try:
        with open(os.path.join(git_dir, "HEAD")) as f:
            head = f.read().strip()
    except OSError:
        return ""
    if not head.startswith("ref:"):
        return "HEAD" if head else ""
    ref = head[4:].strip()
    if not _ref_exists(git_dir, ref):
        return ""
    return go_base(ref)


def repo_details(path, remote_name):
    """(remote_urls, branch, repo_dir) like ``GetGitRepoDetails``
    (utils.go:653-680), with its debug lines; go-git's errors are
    ``reference not found`` and ``remote not found``."""
    from . import log
    try:
        root, git_dir = find_repo(path)
    except GitError as e:
        log.debug("Unable to open the path %r as a git repo. Error: %r", path, str(e))
        raise
    branch = head_branch(git_dir)
    if branch == "":
        log.debug("Unable to get the current branch. Error: %r", "reference not found")
    try:
        remotes = _read_config(git_dir)
    except GitConfigError as e:
        log.debug("Unable to get remote named %s Error: %r", remote_name, str(e))
        return [], branch, root
    if remote_name not in remotes:
        log.debug("Unable to get remote named %s Error: %r", remote_name, "remote not found")
    urls = remotes.get(remote_name, [])
    return list(urls), branch, root


def go_base(p):
    """Go ``filepath.Base``: '' -> '.', only slashes -> '/', trailing slashes dropped."""
    if p == "":
        return "."
    p = p.rstrip("/")
    if p == "":
        return "/"
    return p.rsplit("/", 1)[-1]


def go_ext(p):
    """Go ``filepath.Ext``: the suffix from the last dot of the last element
    (``.cfg`` for ``.cfg``; Python's splitext treats that as no extension)."""
    i = len(p) - 1
    while i >= 0 and p[i] != "/":
        if p[i] == ".":
            return p[i:]
        i -= 1
    return ""


_SCP_HOST_RE = _lazy_re(r"^(?:[\w.\-]+@)?([\w.\-]+):(?!//)")
_SCHEME_RE = _lazy_re(r"^([A-Za-z][A-Za-z0-9+.\-]*):")
_HEX = "0123456789abcdefABCDEF"


def go_url_path(raw):
    """``url.Parse(raw).Path`` for the subset of ``net/url`` rules that a git
    remote can hit; raises ValueError where Go returns an error."""
    if any(ord(c) < 0x20 or ord(c) == 0x7f for c in raw):
        raise ValueError("net/url: invalid control character in URL")
    rest = raw.split("#", 1)[0]
    if rest.count("?") == 1 and rest.endswith("?"):
        rest = rest[:-1]
    else:
        rest = rest.split("?", 1)[0]
    if rest.startswith(":"):
        raise ValueError("missing protocol scheme")
    m = _SCHEME_RE.match(rest)
    scheme = ""
    if m:
        scheme = m.group(1)
        rest = rest[m.end():]
    if scheme and not rest.startswith("/"):
        return ""  # opaque URL: Path stays empty
    if not scheme:
        seg = rest.split("/", 1)[0]
        if ":" in seg:
            raise ValueError("first path segment in URL cannot contain colon")
    if rest.startswith("//"):
        auth, slash, rest = rest[2:].partition("/")
        rest = slash + rest
        host = auth.rsplit("@", 1)[-1]
        if not host.startswith("["):
            _h, colon, port = host.rpartition(":")
            if colon and port and not port.isdigit():
                raise ValueError('invalid port ":%s" after host' % port)
    i = rest.find("%")
    while i >= 0:
        if i + 2 >= len(rest) or rest[i + 1] not in _HEX or rest[i + 2] not in _HEX:
            raise ValueError("invalid URL escape %r" % rest[i:i + 3])
        i = rest.find("%", i + 3)
    import urllib.parse
    return urllib.parse.unquote(rest)


def repo_name(path):
    """(name, root) of the repo's ``origin`` remote, or ('', '') (``GetGitRepoName``,
    ``internal/common/utils.go:682-718``)."""
    from . import log
    try:
        root, git_dir = find_repo(path)
    except GitError as e:
        log.debug("Unable to open %s as a git repo : %s", path, e)
        return "", ""
    try:
        remotes = _read_config(git_dir)
    except GitConfigError as e:
        log.debug("Unable to get origin remote : %s", e)
        return "", ""
    if "origin" not in remotes:
        log.debug("Unable to get origin remote : %s", "remote not found")
        return "", ""
    urls = remotes["origin"]
    if not urls:
        log.debug("Unable to get origins")
        return "", ""
    u = urls[0]
    if u.startswith("git"):
        parts = u.split(":")
        if len(parts) != 2:
            return "", ""
        u = parts[1]
    try:
        upath = go_url_path(u)
    except ValueError as e:
        log.debug("Unable to get origin remote host : %s", e)
        return "", ""
    name = go_base(upath)
    ext = go_ext(name)
    if ext and name.endswith(ext):
        name = name[:-len(ext)]
    return name, root


def url_hostname(giturl):
    """Hostname of a git URL (scp-like ``git@host:org/repo`` or URL forms); '' if none."""
    if not giturl:
        return ""
    m = _SCP_HOST_RE.match(giturl)
    if m and "://" not in giturl:
        return m.group(1)
    try:
        import urllib.parse
        return urllib.parse.urlparse(giturl).hostname or ""
    except ValueError:
        return ""
