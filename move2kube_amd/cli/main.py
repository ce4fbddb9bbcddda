"""``move2kube`` command line (reference ``cmd/move2kube/*.go``).

Verbs and flags match the reference: ``collect [-a] [-o] [-s]``,
``plan -s [-p] [-n]``, ``translate [-p] [-c] [-s] [-o] [-n] [-q] [--ignoreenv]``
(+ hidden ``--qadisablecli --qaskip --qaport``), ``version [-l]``; global ``-v``.
"""

import errno
import os
import stat
import sys

from .. import assets
from ..models import plan as plantypes
from ..utils import fsindex, log, yamlio
from ..utils.common import go_abs, go_clean, go_error_text, go_join, go_path_error
from ..utils.constants import (APP_NAME_SHORT, DEFAULT_DIRECTORY_PERMISSION, DEFAULT_PLAN_FILE, DEFAULT_PROJECT_NAME,
                               QA_CACHE_FILE, settings)
from ..utils.lazyre import LazyModule

# the orchestration layer (translators, QA engine, transformers) loads on
# first use: `collect` and `version` never need it
move2kube = LazyModule("move2kube_amd.move2kube")
qaengine = LazyModule("move2kube_amd.qaengine")


def _abs(p, what=None):
    """filepath.Abs of a flag value; the reference's commands stop with
    ``Failed to make the <what> path %q absolute`` when it fails (the working
    directory is gone)."""
    if not p:
        return p
    try:
        return go_abs(p)
    except OSError as e:
        if what is None:
            raise
        log.fatal("Failed to make the %s path %r absolute. Error: %r", what, p,
                  "getwd: " + (e.strerror or str(e)).lower())


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
        log.fatal("Failed to create the output directory at path %s Error: %r", out, go_path_error(e, "mkdir"))
    cache = os.path.join(out, QA_CACHE_FILE)
    log.debug("Creating the cache file at path %s", cache)
    try:
        qaengine.set_write_cache(cache)
    except OSError as e:
        log.warning("Unable to write the cache file to path %r Error: %r", cache, go_path_error(e, "open"))


def translate_handler(a):
    planfile = _abs(a.plan, "plan file")
    srcpath = _abs(a.source, "source directory") if a.source else ""
    outpath = _abs(a.outpath, "output directory")
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
            log.fatal("Unable to read the plan at path %s Error: %r", planfile, go_error_text(e))
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
    planfile = _abs(a.plan, "plan file")
    srcpath = _abs(a.source, "source directory")
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
        log.error("Unable to write plan file (%s) : %s", planfile, go_path_error(e, "open"))
        return
    log.info("Plan can be found at [%s].", planfile)


def collect_handler(a):
    outpath = _abs(a.outpath, "output directory") if a.outpath else a.outpath
    srcpath = ""
    if a.source:
        srcpath = _abs(a.source, "source directory")
        st, err = _go_stat(srcpath)
        if err and err[0] == errno.ENOENT:
            log.fatal("Source directory does not exist: %s.", err[1])
        if err:
            log.fatal("Error while accessing directory: %s. ", srcpath)
        if not stat.S_ISDIR(st.st_mode):
            log.fatal("Source path is a file, expected directory: %s.", srcpath)
    outpath = go_join(go_clean(outpath), APP_NAME_SHORT + "_collect")
    annotations = a.annotations.split(",") if a.annotations else []
    from .. import collector  # move2kube.collect without loading the orchestration layer
    collector.collect(srcpath, outpath, annotations)
    log.info("Collect Output in [%s]. Copy this directory into the source directory to be used for planning.", outpath)


def version_handler(a):
    from ..models import info
    print(info.get_version() if not a.long else yamlio.dump(info.get_version_info().to_yaml()))


class _Args:
    """The parsed flags of one command (cobra flag values by name)."""

    def __init__(self, cmd):
        for f in cmd.all_flags():
            setattr(self, f.name, f.value)
        self.command = cmd.name
        self.cmd = cmd


def build_command_tree():
    """The reference's cobra command tree (``cmd/move2kube/move2kube.go:37-51``,
    ``collect.go:78-89``, ``plan.go:90-103``, ``translate.go:187-214``,
    ``version.go:30-39``)."""
    from .cobra import Command, add_help_command
    root = Command("move2kube", "A tool to modernize to kubernetes/openshift",
                   "move2kube is a tool to help optimally translate from platforms such as docker-swarm, CF to "
                   "Kubernetes.")
    root.flag("verbose", "v", "bool", False, "Enable verbose output", persistent=True)

    c = Command("collect", "Collect and process metadata from multiple sources.",
                "Collect metadata from multiple sources (cluster, image repo etc.), filter and summarize it into a "
                "yaml.", run=collect_handler)
    c.flag("annotations", "a", "string", "", "Specify annotations to select collector subset.")
    c.flag("outpath", "o", "string", ".", "Specify output directory for collect.")
    c.flag("source", "s", "string", "", "Specify source directory for the artifacts to be considered while "
                                         "collecting.")

    p = Command("plan", "Plan out a move", "Discover and create a plan file based on an input directory",
                run=plan_handler)
    p.flag("source", "s", "string", ".", "Specify source directory.")
    p.flag("plan", "p", "string", DEFAULT_PLAN_FILE, "Specify a file path to save plan to.")
    p.flag("name", "n", "string", DEFAULT_PROJECT_NAME, "Specify the project name.")
    p.mark_required("source")

    t = Command("translate", "Translate using move2kube plan", "Translate artifacts using move2kube plan",
                run=translate_handler)
    t.flag("plan", "p", "string", DEFAULT_PLAN_FILE, "Specify a plan file to execute.")
    t.flag("curate", "c", "bool", False, "Specify whether to curate the plan with a q/a.")
    t.flag("source", "s", "string", "", "Specify source directory to translate. If you already have a m2k.plan "
                                         "then this will override the rootdir value specified in that plan.")
    t.flag("outpath", "o", "string", ".", "Path for output. Default will be directory with the project name.")
    t.flag("name", "n", "string", DEFAULT_PROJECT_NAME, "Specify the project name.")
    t.flag("qacache", "q", "stringSlice", [], "Specify qa cache file locations")
    t.flag("ignoreenv", "", "bool", False, "Ignore data from local machine.")
    t.flag("qadisablecli", "", "bool", False, "Enable/disable the QA Cli sub-system. Without this system, you will "
           "have to use the REST API to interact.", hidden=True)
    t.flag("qaskip", "", "bool", False, "Enable/disable the default answers to questions posed in QA Cli "
           "sub-system. If disabled, you will have to answer the questions posed by QA during interaction.",
           hidden=True)
    t.flag("qaport", "", "int", 0, "Port for the QA service. By default it chooses a random free port.", hidden=True)

    v = Command("version", "Print the client version information", "Print the client version information",
                run=version_handler)
    v.flag("long", "l", "bool", False, "print the version details")

    root.add(c, p, t, v)
    add_help_command(root)
    return root


def main(argv=None):
    from . import cobra
    if argv is None:
        argv = sys.argv[1:]
    res = cobra.execute(build_command_tree(), argv)
    if isinstance(res, int):
        return res
    cmd, positional = res
    a = _Args(cmd)
    if a.verbose:
        log.set_verbose(True)
    if cmd.name == "help":
        return cmd.run(cmd, positional)
    if a.command == "translate":
        a.plan_changed = cmd.changed("plan")
        a.source_changed = cmd.changed("source")
        a.name_changed = cmd.changed("name")
    try:
        assets.setup()
    except OSError as e:
        log.error("Unable to create the assets directory. Error: %r", go_path_error(e, "mkdir"))
        return 1
    try:
        with yamlio.parse_cache():  # one command = one parse of each YAML document
            cmd.run(a)
    except log.FatalError:
        return 1
    finally:
        assets.cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
