"""``move2kube`` command line (reference ``cmd/move2kube/*.go``).

Verbs and flags match the reference: ``collect [-a] [-o] [-s]``,
``plan -s [-p] [-n]``, ``translate [-p] [-c] [-s] [-o] [-n] [-q] [--ignoreenv]``
(+ hidden ``--qadisablecli --qaskip --qaport``), ``version [-l]``; global ``-v``.
"""

import argparse
import errno
import os
import stat
import sys

from .. import assets
from ..models import plan as plantypes
from ..utils import fsindex, log, yamlio
from ..utils.constants import (APP_NAME_SHORT, DEFAULT_DIRECTORY_PERMISSION, DEFAULT_PLAN_FILE, DEFAULT_PROJECT_NAME,
                               QA_CACHE_FILE, settings)
from ..utils.lazyre import LazyModule

# the orchestration layer (translators, QA engine, transformers) loads on
# first use: `collect` and `version` never need it
move2kube = LazyModule("move2kube_amd.move2kube")
qaengine = LazyModule("move2kube_amd.qaengine")


class _StringSlice(argparse.Action):
    """cobra StringSlice: repeatable, each value comma-separated."""

    def __call__(self, parser, namespace, values, option_string=None):
        cur = list(getattr(namespace, self.dest) or [])
        cur.extend(v for v in values.split(",") if v != "")
        setattr(namespace, self.dest, cur)


def _abs(p):
    return os.path.abspath(p) if p else p


def _go_stat(path):
    """``os.Stat``: (stat result, None) or (None, (errno, Go error string))."""
    try:
        return os.stat(path), None
    except OSError as e:
        msg = os.strerror(e.errno) if e.errno else str(e)
        return None, (e.errno, "stat %s: %s" % (path, msg[:1].lower() + msg[1:]))


def check_source_path(src):
    """translate.go:54-65: only ENOENT is "does not exist"; any other stat
    error (ENOTDIR, EACCES, ELOOP...) is an access error."""
    st, err = _go_stat(src)
    if err and err[0] == errno.ENOENT:
        log.fatal("The given source directory %s does not exist. Error: %r", src, err[1])
    if err:
        log.fatal("Error while accessing the given source directory %s Error: %r", src, err[1])
    if not stat.S_ISDIR(st.st_mode):
        log.fatal("The given source path %s is a file. Expected a directory. Exiting.", src)


def check_output_path(out):
    """translate.go:67-80 (an output path under a regular file is an access
    error here, before any planning, not a failed MkdirAll afterwards)."""
    st, err = _go_stat(out)
    if err and err[0] == errno.ENOENT:
        log.debug("Translated artifacts will be written to %s", out)
        return
    if err:
        log.fatal("Error while accessing output directory at path %s Error: %r . Exiting", out, err[1])
    if not stat.S_ISDIR(st.st_mode):
        log.fatal("Output path %s is a file. Expected a directory. Exiting", out)
    log.info("Output directory %s exists. The contents might get overwritten.", out)


def create_output_directory_and_cache_file(out):
    try:
        os.makedirs(out, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
    except OSError as e:
        log.fatal("Failed to create the output directory at path %s Error: %r", out, str(e))
    cache = os.path.join(out, QA_CACHE_FILE)
    log.debug("Creating the cache file at path %s", cache)
    try:
        qaengine.set_write_cache(cache)
    except OSError as e:
        log.warning("Unable to write the cache file to path %r Error: %r", cache, str(e))


def translate_handler(a):
    planfile = _abs(a.plan)
    srcpath = _abs(a.source) if a.source else ""
    outpath = _abs(a.outpath)
    settings.ignore_environment = a.ignoreenv
    qaengine.start_engine(a.qaskip, a.qaport, a.qadisablecli)
    qaengine.add_caches(list(reversed(a.qacache or [])))
    if os.path.isdir(planfile):
        planfile = os.path.join(planfile, DEFAULT_PLAN_FILE)
    if not os.path.exists(planfile):
        log.debug("No plan file found.")
        if a.plan_changed or not a.source_changed:
            log.fatal("Error while accessing plan file at path %s Error: %r", planfile,
                      "stat %s: no such file or directory" % planfile)
        check_source_path(srcpath)
        log.debug("Creating a new plan.")
        p = move2kube.create_plan(srcpath, a.name,
                                  keep_index=fsindex.handoff_allowed(srcpath, os.path.join(outpath, a.name)))
        outpath = os.path.join(outpath, p.name)
        check_output_path(outpath)
        create_output_directory_and_cache_file(outpath)
        p = move2kube.curate_plan(p)
    else:
        log.info("Detected a plan file at path %s. Will translate using this plan.", planfile)
        try:
            p = plantypes.read_plan(planfile)
        except Exception as e:  # noqa: BLE001
            log.fatal("Unable to read the plan at path %s Error: %r", planfile, str(e))
        if a.name_changed:
            p.name = a.name
        if a.source_changed:
            try:
                p.set_root_dir(srcpath)
            except Exception as e:  # noqa: BLE001
                log.fatal("Failed to set the root directory to %r Error: %r", srcpath, str(e))
        check_source_path(p.root_dir)
        outpath = os.path.join(outpath, p.name)
        check_output_path(outpath)
        create_output_directory_and_cache_file(outpath)
        if a.curate:
            p = move2kube.curate_plan(p)
    move2kube.translate(p, outpath, a.qadisablecli)
    log.info("Translated target artifacts can be found at [%s].", outpath)


def plan_handler(a):
    planfile = _abs(a.plan)
    srcpath = _abs(a.source)
    st, err = _go_stat(srcpath)
    if err:
        log.fatal("Unable to access source directory : %s", err[1])
    if not stat.S_ISDIR(st.st_mode):
        log.fatal("Input is a file, expected directory: %s", srcpath)
    pst, err = _go_stat(planfile)
    if err and err[0] != errno.ENOENT:
        log.fatal("Error while accessing plan file path %s : %s ", planfile, err[1])
    if err:
        # (the reference tests the trailing separator on the already-cleaned
        # absolute path, so only an extension-less base name selects a directory)
        if planfile.endswith(os.sep) or "." not in os.path.basename(planfile):
            planfile = os.path.join(planfile, DEFAULT_PLAN_FILE)
    elif stat.S_ISDIR(pst.st_mode):
        planfile = os.path.join(planfile, DEFAULT_PLAN_FILE)
    p = move2kube.create_plan(srcpath, a.name)
    try:
        d = os.path.dirname(planfile)
        if d and settings.fixed:
            # the reference writes with ioutil.WriteFile: a missing directory is an error
            os.makedirs(d, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        plantypes.write_plan(planfile, p)
    except OSError as e:
        log.error("Unable to write plan file (%s) : %s", planfile, e)
        return
    log.info("Plan can be found at [%s].", planfile)


def collect_handler(a):
    outpath = _abs(a.outpath) if a.outpath else a.outpath
    srcpath = ""
    if a.source:
        srcpath = _abs(a.source)
        st, err = _go_stat(srcpath)
        if err and err[0] == errno.ENOENT:
            log.fatal("Source directory does not exist: %s.", err[1])
        if err:
            log.fatal("Error while accessing directory: %s. ", srcpath)
        if not stat.S_ISDIR(st.st_mode):
            log.fatal("Source path is a file, expected directory: %s.", srcpath)
    outpath = os.path.join(os.path.normpath(outpath), APP_NAME_SHORT + "_collect")
    annotations = a.annotations.split(",") if a.annotations else []
    from .. import collector  # move2kube.collect without loading the orchestration layer
    collector.collect(srcpath, outpath, annotations)
    log.info("Collect Output in [%s]. Copy this directory into the source directory to be used for planning.", outpath)


def version_handler(a):
    from ..models import info
    print(info.get_version() if not a.long else yamlio.dump(info.get_version_info().to_yaml()))


_VERBS = ("collect", "plan", "translate", "version")


def _verb_of(argv):
    """The sub-command named on the command line (after the root flags), or None."""
    for arg in argv:
        if arg in ("-v", "--verbose"):
            continue
        return arg if arg in _VERBS else None
    return None


def build_parser(only=None):
    """The cobra command tree as argparse.  ``only`` = the verb being run: its
    arguments are the only ones built (argparse translates every help string
    through gettext as it is added, a measurable share of a cold run); the
    other verbs stay registered, so choices and errors are unchanged."""
    root = argparse.ArgumentParser(prog="move2kube", description="A tool to modernize to kubernetes/openshift")
    root.add_argument("-v", "--verbose", action="store_true", help="Enable verbose output")
    sub = root.add_subparsers(dest="command")

    def wanted(verb):
        return only is None or only == verb

    c = sub.add_parser("collect", help="Collect and process metadata from multiple sources.")
    if wanted("collect"):
        c.add_argument("-a", "--annotations", default="", help="Specify annotations to select collector subset.")
        c.add_argument("-o", "--outpath", default=".", help="Specify output directory for collect.")
        c.add_argument("-s", "--source", default="", help="Specify source directory for the artifacts to be considered while collecting.")
        c.set_defaults(func=collect_handler)

    p = sub.add_parser("plan", help="Plan out a move")
    if wanted("plan"):
        p.add_argument("-s", "--source", required=True, help="Specify source directory.")
        p.add_argument("-p", "--plan", default=DEFAULT_PLAN_FILE, help="Specify a file path to save plan to.")
        p.add_argument("-n", "--name", default=DEFAULT_PROJECT_NAME, help="Specify the project name.")
        p.set_defaults(func=plan_handler)

    t = sub.add_parser("translate", help="Translate using move2kube plan")
    if wanted("translate"):
        t.add_argument("-p", "--plan", default=None, help="Specify a plan file to execute.")
        t.add_argument("-c", "--curate", action="store_true", help="Specify whether to curate the plan with a q/a.")
        t.add_argument("-s", "--source", default=None, help="Specify source directory to translate.")
        t.add_argument("-o", "--outpath", default=".", help="Path for output. Default will be directory with the project name.")
        t.add_argument("-n", "--name", default=None, help="Specify the project name.")
        t.add_argument("-q", "--qacache", action=_StringSlice, default=[], help="Specify qa cache file locations")
        t.add_argument("--ignoreenv", action="store_true", help="Ignore data from local machine.")
        t.add_argument("--qadisablecli", action="store_true", help=argparse.SUPPRESS)
        t.add_argument("--qaskip", action="store_true", help=argparse.SUPPRESS)
        t.add_argument("--qaport", type=int, default=0, help=argparse.SUPPRESS)
        t.set_defaults(func=translate_handler)

    v = sub.add_parser("version", help="Print the client version information")
    if wanted("version"):
        v.add_argument("-l", "--long", action="store_true", help="print the version details")
        v.set_defaults(func=version_handler)
    return root


def main(argv=None):
    if argv is None:
        argv = sys.argv[1:]
    parser = build_parser(_verb_of(argv))
    a = parser.parse_args(argv)
    if a.verbose:
        log.set_verbose(True)
    if not getattr(a, "func", None):
        parser.print_help()
        return 0
    if a.command == "translate":
        a.plan_changed = a.plan is not None
        a.source_changed = a.source is not None
        a.name_changed = a.name is not None
        a.plan = a.plan if a.plan is not None else DEFAULT_PLAN_FILE
        a.source = a.source or ""
        a.name = a.name if a.name is not None else DEFAULT_PROJECT_NAME
    try:
        assets.setup()
    except OSError as e:
        log.error("Unable to create the assets directory. Error: %r", str(e))
        return 1
    try:
        with yamlio.parse_cache():  # one command = one parse of each YAML document
            a.func(a)
    except log.FatalError:
        return 1
    finally:
        assets.cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
