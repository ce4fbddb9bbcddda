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
    """Walk up from ``path`` to the directory containing ``.git``.

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
            if os.path.exists(os.path.join(dotgit, "HEAD")):
                result = (p, dotgit)
                break
        elif os.path.isfile(dotgit):
            try:
                with open(dotgit) as f:
                    line = f.read().strip()
            except OSError as e:
                raise GitError(str(e))
            if line.startswith("gitdir:"):
                gd = line[len("gitdir:"):].strip()
                if not os.path.isabs(gd):
                    gd = os.path.normpath(os.path.join(p, gd))
                result = (p, gd)
                break
        parent = os.path.dirname(p)
        if parent == p:
            result = None
            break
        p = parent
    if cache is not None:
        for v in visited:
            cache[v] = result
    if result is None:
        raise GitError("repository does not exist")
    return result


_REMOTE_RE = _lazy_re(r'^remote\s+"(.*)"$')


def _read_config(git_dir):
    cfg = os.path.join(git_dir, "config")
    # worktrees keep the shared config in the common dir
    common_file = os.path.join(git_dir, "commondir")
    if not os.path.exists(cfg) and os.path.exists(common_file):
        with open(common_file) as f:
            cfg = os.path.join(os.path.normpath(os.path.join(git_dir, f.read().strip())), "config")
    import configparser
    parser = configparser.RawConfigParser(strict=False, allow_no_value=True)
    try:
        with open(cfg) as f:
            parser.read_string(f.read())
    except (OSError, configparser.Error):
        return {}
    remotes = {}
    for sect in parser.sections():
        m = _REMOTE_RE.match(sect.strip())
        if m:
            urls = []
            for k, v in parser.items(sect):
                if k == "url" and v:
                    urls.append(v.strip())
            remotes[m.group(1)] = urls
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
    remotes = _read_config(git_dir)
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
    remotes = _read_config(git_dir)
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
