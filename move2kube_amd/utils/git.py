"""Git repository discovery without a git library.

Replaces the reference's go-git calls (``internal/common/utils.go:636-718``):
``PlainOpenWithOptions(path, DetectDotGit)``, remotes, HEAD branch and work
tree root, read directly from ``.git/config`` and ``.git/HEAD``.
"""

import os
import re

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


def repo_details(path, remote_name):
    """(remote_urls, branch, repo_dir) like ``GetGitRepoDetails``."""
    root, git_dir = find_repo(path)
    branch = ""
    try:
        with open(os.path.join(git_dir, "HEAD")) as f:
            head = f.read().strip()
        if head.startswith("ref:"):
            branch = os.path.basename(head[4:].strip())
        else:
            branch = "HEAD"
    except OSError:
        pass
    urls = _read_config(git_dir).get(remote_name, [])
    return list(urls), branch, root


def repo_name(path):
    """(name, root) of the repo's ``origin`` remote, or ('', '') (``GetGitRepoName``)."""
    try:
        root, git_dir = find_repo(path)
    except GitError:
        return "", ""
    urls = _read_config(git_dir).get("origin")
    if not urls:
        return "", ""
    u = urls[0]
    if u.startswith("git"):
        parts = u.split(":")
        if len(parts) != 2:
            return "", ""
        u = parts[1]
    try:
        import urllib.parse
        parsed = urllib.parse.urlparse(u)
    except ValueError:
        return "", ""
    name = os.path.basename(parsed.path.rstrip("/")) if parsed.path else "."
    base, ext = os.path.splitext(name)
    if ext:
        name = base
    return name, root


def url_hostname(giturl):
    """Hostname of a git URL (scp-like ``git@host:org/repo`` or URL forms); '' if none."""
    if not giturl:
        return ""
    m = re.match(r"^(?:[\w.\-]+@)?([\w.\-]+):(?!//)", giturl)
    if m and "://" not in giturl:
        return m.group(1)
    try:
        import urllib.parse
        return urllib.parse.urlparse(giturl).hostname or ""
    except ValueError:
        return ""
