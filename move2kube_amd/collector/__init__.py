"""Metadata collectors for ``move2kube collect`` (reference ``internal/collector/``).

Each collector shells out to the platform CLI that already holds the user's
credentials (kubectl/oc, docker, cf) and writes a move2kube metadata YAML
under ``<out>/m2k_collect/<area>/``.  Collectors are selected by annotation
(``-a k8s,cf``); a failing collector is logged and skipped.
"""

import os
import threading

from ..utils import log


class Collector:
    annotations = ()

    def get_annotations(self):
        return list(self.annotations)

    def collect(self, input_path, output_path):
        raise NotImplementedError

    def __repr__(self):
        return "*collector.%s" % type(self).__name__


class CommandError(RuntimeError):
    def __init__(self, argv, code, output=b""):
        from ..utils.common import go_exit_status
        super().__init__(go_exit_status(code))
        self.argv = argv
        self.code = code
        self.output = output


_SERIAL_CLIS = {"cf": threading.Lock()}


def run(argv, combined=False, timeout=300):
    """Run a command; stdout bytes (stdout+stderr with ``combined``). Raises
    :class:`CommandError` on a non-zero exit and FileNotFoundError if missing
    (worded like Go's ``exec: "cf": executable file not found in $PATH``).

    Collectors run concurrently, but two ``cf`` commands never do: the cf
    CLI rewrites ``~/.cf/config.json`` when it refreshes its token."""
    from ..utils import proc
    from ..utils.common import run_tool
    lock = _SERIAL_CLIS.get(os.path.basename(argv[0])) if argv else None
    kw = dict(stdout=proc.PIPE, stderr=proc.STDOUT if combined else proc.PIPE, timeout=timeout)
    if lock is not None:
        with lock:
            p = run_tool(argv, **kw)
    else:
        p = run_tool(argv, **kw)
    if p.returncode != 0:
        raise CommandError(argv, p.returncode, p.stdout)
    return p.stdout


def concurrently(*fns, workers=8):
    """Run the callables on up to ``workers`` threads (they wait on external
    CLIs); returns their results in order, a raised ``Exception`` in its slot.
    The log lines of each are held and written in call order, as a sequential
    run prints them."""
    import threading
    n = len(fns)
    out = [None] * n
    held = [None] * n
    nxt = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= n:
                return
            with log.hold() as h:
                try:
                    out[i] = fns[i]()
                except Exception as e:  # noqa: BLE001
                    out[i] = e
            held[i] = h.lines
    threads = [threading.Thread(target=worker, name="m2k-collect-worker") for _ in range(max(1, min(workers, n)))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for lines in held:
        log.emit(lines or [])
    return out


# (module, class, annotations) in the reference's order (collector.go:38-44);
# a collector's module is only imported when the annotations select it
# (cluster metadata pulls in the Kubernetes scheme)
REGISTRY = (("cluster", "ClusterCollector", ("k8s",)),
            ("images", "ImagesCollector", ("k8s", "dockerswarm", "dockercompose")),
            ("cf", "CFContainerTypesCollector", ("cloudfoundry", "cf")),
            ("cf", "CfAppsCollector", ("cf", "cloudfoundry")))


def get_collectors(annotations=()):
    """The collectors, or those whose annotations overlap ``annotations``."""
    import importlib
    out = []
    for mod, cls, ann in REGISTRY:
        if annotations and not has_overlap(annotations, ann):
            continue
        out.append(getattr(importlib.import_module("." + mod, __name__), cls)())
    return out


def has_overlap(a, b):
    from ..utils.common import go_fold
    return any(go_fold(x) == go_fold(y) for x in a for y in b)


def collect(input_path, output_path, annotations=()):
    from ..utils.constants import DEFAULT_DIRECTORY_PERMISSION
    try:
        os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
    except OSError as e:
        from ..utils.common import go_path_error
        log.fatal("Unable to create output directory at path %r Error: %r", output_path, go_path_error(e, "mkdir"))
    log.info("Begin collection")
    selected = [c for c in get_collectors(annotations)
                if not annotations or has_overlap(annotations, c.get_annotations())]
    # The collectors are independent (their own CLIs and output sub-directories)
    # and wait on external tools - cluster discovery, `docker`, `cf curl`, a
    # container runtime - so they run at the same time; the reference runs them
    # one after another.  Each one's log lines are held and written in
    # collector order, as a sequential run prints them.
    results = [None] * len(selected)

    def run_one(i):
        c = selected[i]
        with log.hold() as held:
            fatal = None
            log.info("[%r] Begin collection", c)
            try:
                c.collect(input_path, output_path)
            except log.FatalError as e:
                fatal = e
            except Exception as e:  # noqa: BLE001
                log.warning("[%r] failed. Error: %r", c, str(e))
            else:
                log.info("[%r] Done", c)
        results[i] = (held.lines, fatal)

    if len(selected) == 1:
        run_one(0)
    else:
        import threading
        threads = [threading.Thread(target=run_one, args=(i,), name="m2k-collect-%d" % i) for i in range(len(selected))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    for r in results:
        if r is None:  # the thread died outside Exception (interrupted)
            continue
        lines, fatal = r
        log.emit(lines)
        if fatal is not None:
            raise fatal
    log.info("Collection done")
