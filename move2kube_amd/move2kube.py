"""Top-level operations behind the CLI verbs (reference ``internal/move2kube/``):
``collect``, ``create_plan``, ``curate_plan``, ``translate``, ``get_version``."""

import os

from . import customizer, metadata, optimizer, parameterizer, qaengine, transformer
from .ops import native
from .models import info, qa
from .models import plan as plantypes
from .source import translator as source_translator
from .utils import common, fsindex, log, trace, yamlio
from .utils.constants import DEFAULT_CLUSTER_TYPE


def collect(input_path, output_path, annotations=()):
    """``Collect`` (collector.go): run the annotation-selected collectors."""
    from . import collector
    collector.collect(input_path, output_path, list(annotations))


def create_plan(input_path, project_name, keep_index=False):
    """``CreatePlan`` (planner.go:30-64): every source translator proposes
    service options, then metadata loaders annotate the plan.  All planners
    share one cached directory index of ``input_path``; ``keep_index`` hands
    it (and the detector results) to the translate of the same command."""
    p = plantypes.new_plan()
    p.name = project_name
    p.root_dir = input_path
    with fsindex.scope(keep_for=input_path if keep_index else None), trace.span("plan", "command"):
        log.info("Planning Translation")
        # the CNB builders' runtime probes run while the translators walk the tree
        from .containerizer.cnb import prefetch_builder_probes
        prefetch_builder_probes()
        for t in source_translator.get_source_loaders():
            log.info("[%r] Planning translation", t)
            try:
                with trace.span(type(t).__name__, "plan"):
                    services = t.get_service_options(input_path, p)
            except Exception as e:  # noqa: BLE001
                if isinstance(e, log.FatalError):
                    raise
                log.warning("[%r] Failed : %s", t, e)
                continue
            p.add_services_to_plan(services)
            log.info("[%r] Done", t)
        log.info("Translation planning done")
        log.info("Planning Metadata")
        for loader in metadata.get_loaders():
            log.info("[%r] Planning metadata", loader)
            try:
                with trace.span(type(loader).__name__, "plan-metadata"):
                    loader.update_plan(input_path, p)
            except Exception as e:  # noqa: BLE001
                if isinstance(e, log.FatalError):
                    raise
                log.warning("[%r] Failed : %s", loader, e)
                continue
            log.info("[%r] Done", loader)
        log.info("Metadata planning done")
    return p


_CONVERTED_BUILD_TYPES = [plantypes.NEW_DOCKERFILE, plantypes.REUSE_DOCKERFILE, plantypes.S2I]


def _ask(prob):
    return qaengine.fetch_answer(prob)


def curate_plan(p):
    """``CuratePlan`` (planner.go:66-222): QA-driven selection of services,
    containerization modes, artifact type and target cluster."""
    qaengine.add_caches(list(reversed(p.qa_caches)))
    names = sorted(p.services)
    sel = _ask(qa.new_multiselect_problem("Select all services that are needed:",
                                          ["The services unselected here will be ignored."], names, names)).get_slice_answer()
    p.services = {s: p.services[s] for s in sel if s in p.services}

    con_types = []
    for sn in sorted(p.services):
        for so in p.services[sn]:
            if not common.is_string_present(con_types, so.container_build_type):
                con_types.append(so.container_build_type)
    sel_types = _ask(qa.new_multiselect_problem(
        "Select all containerization modes that is of interest:",
        ["The services which does not support any of the containerization technique you are interested will be ignored."],
        con_types, con_types)).get_slice_answer()
    if not sel_types:
        log.fatal("No containerization technique was selected; Terminating.")

    services = {}
    for sn in sorted(p.services):
        options = p.services[sn]
        s_types = [so.container_build_type for so in options if common.is_string_present(sel_types, so.container_build_type)]
        if not s_types:
            log.warning("Ignoring service %s, since it does not support any selected containerization technique.", sn)
            continue
        chosen = s_types[0]
        if len(s_types) > 1:
            chosen = _ask(qa.new_select_problem("Select containerization technique for service " + sn + ":",
                                                ["Choose the containerization technique of interest."], chosen,
                                                s_types)).get_string_answer()
        for so in options:
            if so.container_build_type != chosen:
                continue
            conv = common.is_string_present(_CONVERTED_BUILD_TYPES, so.container_build_type)
            if len(so.target_options) > 1:
                opts = so.target_options
                if conv:
                    opts = []
                    for o in so.target_options:
                        try:
                            opts.append(p.get_relative_path(o))
                        except ValueError as e:
                            log.error("Failed to make the option path %r relative to the root directory. Error: %r",
                                      o, str(e))
                if not opts:   # options[0] panics in the reference (planner.go:169): keep the options
                    services[sn] = [so]
                    break
                mode = _ask(qa.new_select_problem("Select containerization technique's mode for service " + sn + ":",
                                                  ["Choose the containerization technique mode of interest."], opts[0],
                                                  opts)).get_string_answer()
                if conv:
                    try:
                        mode = p.get_absolute_path(mode)
                    except ValueError as e:
                        log.error("Failed to make the option path %r absolute. Error: %r", mode, str(e))
                so.target_options = [mode]
            services[sn] = [so]
            break
    p.services = services

    art = _ask(qa.new_select_problem("Choose the artifact type:",
                                     ["Yamls - Generate Kubernetes Yamls", "Helm - Generate Helm chart",
                                      "Knative - Create Knative artifacts"],
                                     plantypes.YAMLS, [plantypes.YAMLS, plantypes.HELM, plantypes.KNATIVE])).get_string_answer()
    p.kubernetes.artifact_type = art

    clusters = sorted(metadata.ClusterMDLoader.get_clusters(p))
    ctype = _ask(qa.new_select_problem("Choose the cluster type:", ["Choose the cluster type you would like to target"],
                                       DEFAULT_CLUSTER_TYPE, clusters)).get_string_answer()
    p.kubernetes.target_cluster_type = ctype
    p.kubernetes.target_cluster_path = ""
    return p


def translate(p, outpath, qadisablecli=False):
    """``Translate`` (translator.go:31-107): plan -> IR -> metadata ->
    optimize -> compose output -> customize -> (helm) parameterize -> CI/CD
    -> k8s/knative output."""
    try:
        with trace.span("translate", "command", services=len(p.services)):
            _translate(p, outpath, qadisablecli)
    finally:
        qaengine.flush_write_cache()
        trace.flush()


def _translate(p, outpath, qadisablecli):
    # source -> IR and metadata loading only read the source tree: one shared
    # directory index for all translators/containerizers of this stage (the
    # plan's, when the same command just planned this tree)
    with fsindex.scope(adopt=p.root_dir):
        ir = _to_ir(p)
    ir = optimizer.optimize(ir)
    log.debug("Total services optimized : %d", len(ir.services))
    _emit(p, ir, outpath, qadisablecli)


def _to_ir(p):
    try:
        ir = source_translator.translate(p)
    except Exception as e:  # noqa: BLE001
        if isinstance(e, log.FatalError):
            raise
        log.fatal("Failed to translate the plan to intermediate representation. Error: %r", str(e))
    log.debug("Total storages loaded : %d", len(ir.storages))

    log.info("Begin Metadata loading")
    for loader in metadata.get_loaders():
        log.debug("[%r] Begin metadata loading", loader)
        try:
            with trace.span(type(loader).__name__, "metadata"):
                loader.load_to_ir(p, ir)
        except Exception as e:  # noqa: BLE001
            if isinstance(e, log.FatalError):
                raise
            log.warning("[%r] Failed : %s", loader, e)
        else:
            log.debug("[%r] Done", loader)
    log.info("Metadata loading done")
    log.debug("Total services loaded : %d", len(ir.services))
    log.debug("Total containers loaded : %d", len(ir.containers))
    return ir


def _remove_stale_trash(parent, base):
    """Delete ``.<base>.m2k-old-<pid>-<tid>`` trees left by a run that was
    killed before its background delete finished (the next plan would walk
    them as part of the source tree).  A tree whose pid is still alive belongs
    to a concurrent run and is left alone."""
    prefix = ".%s.m2k-old-" % base
    try:
        names = [n for n in os.listdir(parent) if n.startswith(prefix)]
    except OSError:
        return
    for n in names:
        pid = n[len(prefix):].split("-", 1)[0]
        if not pid.isdigit():
            continue
        try:
            os.kill(int(pid), 0)
            continue                     # alive (or not ours to signal): keep
        except ProcessLookupError:
            pass
        except (PermissionError, OverflowError, ValueError):
            continue
        try:
            native.remove_tree(os.path.join(parent, n))
        except OSError as e:
            log.debug("Unable to remove the stale output %s : %s", n, e)


def _remove_output(outpath):
    """``os.RemoveAll(out)`` (translator.go:64).  The old tree is renamed out of
    the way (one syscall) and deleted on a thread - the native delete releases
    the GIL - while the new artifacts are generated; :func:`_emit` joins it
    before returning, so nothing is left behind.  Falls back to a synchronous
    delete when the rename is not possible."""
    import threading
    parent, base = os.path.split(os.path.abspath(outpath))
    _remove_stale_trash(parent, base)
    trash = os.path.join(parent, ".%s.m2k-old-%d-%d" % (base, os.getpid(), threading.get_ident()))
    try:
        if os.path.lexists(trash):
            native.remove_tree(trash)
        os.rename(outpath, trash)
    except OSError:
        native.remove_tree(outpath)
        return None
    errors = []

    def work():
        try:
            native.remove_tree(trash)
        except OSError as e:
            errors.append(e)
    t = threading.Thread(target=work, name="m2k-remove-old-output", daemon=True)
    t.start()
    return t, errors


def _emit(p, ir, outpath, qadisablecli):
    remover = None
    if os.path.lexists(outpath):
        qaengine.before_remove(outpath)
        try:
            remover = _remove_output(outpath)
        except OSError as e:
            log.error("Failed to remove the existing file/directory at the output path %r Error: %r", outpath,
                      common.go_path_error(e, "unlinkat"))
            log.error("Anything in the output path will get overwritten.")
    try:
        _emit_artifacts(p, ir, outpath, qadisablecli, remover[0].join if remover is not None else None)
    finally:
        if remover is not None:
            remover[0].join()
            for e in remover[1]:
                log.warning("Failed to remove the previous output: %s", e)


def _emit_artifacts(p, ir, outpath, qadisablecli, join_remover=None):
    # For a Helm chart the main transformer starts operator-sdk once the chart
    # is written and waits for it at the end; the writes of the compose file,
    # the CI/CD objects and the QA cache do not feed the chart, so they are
    # done in that wait (same bytes, same files; every question is still asked
    # in the reference's order, before the chart is written).
    overlap = [] if p.kubernetes.artifact_type == plantypes.HELM else None

    def later(fn):
        if overlap is None:
            fn()
        else:
            overlap.append(fn)

    dct = transformer.ComposeTransformer()

    def write_compose():
        try:
            dct.write_objects(outpath)
        except Exception as e:  # noqa: BLE001
            if isinstance(e, log.FatalError):
                raise
            log.error("Unable to write docker compose objects : %s", e)
    try:
        with trace.span("ComposeTransformer", "transform"):
            dct.transform(ir)
    except Exception as e:  # noqa: BLE001
        if isinstance(e, log.FatalError):
            raise
        log.error("Error during translate docker compose file : %s", e)
    else:
        later(write_compose)

    try:
        ir = customizer.customize(ir)
        log.debug("Total storages customized : %d", len(ir.storages))
        if p.kubernetes.artifact_type == plantypes.HELM:
            ir = parameterizer.parameterize(ir)

        if any(c.new for c in ir.containers):
            # translator.go:92-102: the CI/CD transform (the git secrets ask
            # for known hosts and SSH keys) runs before the main transformer,
            # so its questions, and a fatal error among them, come before
            # anything of the chart is written; only the write of the Tekton
            # objects, which the chart does not read, waits for operator-sdk
            cicd = transformer.CICDTransformer()
            try:
                with trace.span("CICDTransformer", "transform"):
                    cicd.transform(ir)
            except Exception as e:  # noqa: BLE001
                if isinstance(e, log.FatalError):
                    raise
                log.error("Error while genrationg CI/CD resource fomr the IR. Error: %r", str(e))  # sic
            else:
                def write_cicd():
                    try:
                        cicd.write_objects(outpath)
                    except Exception as e:  # noqa: BLE001
                        if isinstance(e, log.FatalError):
                            raise
                        log.error("Unable to write the CI/CD artifacts to files. Error: %r", str(e))
                later(write_cicd)

        ir.add_copy_sources_warning = qadisablecli
        t = transformer.get_transformer(ir)
        try:
            with trace.span(type(t).__name__ + ".transform", "transform"):
                t.transform(ir)
        except Exception as e:  # noqa: BLE001
            if isinstance(e, log.FatalError):
                raise
            log.fatal("Error during translate. Error: %r", str(e))
        if overlap is not None:
            overlap.append(qaengine.flush_write_cache)
            t.overlap_work = overlap
            # the previous tree is unlinked on a thread; let it finish before
            # operator-sdk copies the chart: both on one tmpfs, the unlinks slow
            # the tool's writes (box A/B, profiles/r05_rmab/remove_ab.jsonl)
            t.before_operator = join_remover
        try:
            with trace.span(type(t).__name__ + ".write_objects", "transform"):
                t.write_objects(outpath)
        except Exception as e:  # noqa: BLE001
            if isinstance(e, log.FatalError):
                raise
            log.fatal("Unable to write objects Error: %r", str(e))
    finally:
        # deferred writes not yet run (no Helm wait reached, or an error before it)
        while overlap:
            overlap.pop(0)()
    log.info("Execution completed")


def get_version(long=False):
    if not long:
        return info.get_version()
    return yamlio.dump(info.get_version_info().to_yaml())
