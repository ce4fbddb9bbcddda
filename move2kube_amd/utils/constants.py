"""Global constants and mutable process-wide settings.

Mirrors the reference's ``internal/common/constants.go:27-73`` and
``types/types.go:23-52``.  The mutable settings (``IGNORE_ENVIRONMENT``,
``TEMP_PATH``, ``ASSETS_PATH``) live on the :data:`settings` object so that
every module sees the same values after the CLI (or a test) changes them.
"""

import os

APP_NAME = "move2kube"
APP_NAME_SHORT = "m2k"
GROUP_NAME = APP_NAME + ".konveyor.io"
SCHEME_VERSION = "v1alpha1"
SCHEME_GROUP_VERSION = GROUP_NAME + "/" + SCHEME_VERSION

DEFAULT_PROJECT_NAME = "myproject"
DEFAULT_PLAN_FILE = APP_NAME_SHORT + ".plan"
TEMP_DIR_PREFIX = APP_NAME_SHORT + "-"
ASSETS_DIR = APP_NAME_SHORT + "assets"
VOLUME_PREFIX = "vol"
DEFAULT_STORAGE_CLASS_NAME = "default"
DEFAULT_DIRECTORY_PERMISSION = 0o755
DEFAULT_EXECUTABLE_PERMISSION = 0o744
DEFAULT_FILE_PERMISSION = 0o644
DEFAULT_REGISTRY_URL = "docker.io"
IMAGE_PULL_SECRET_PREFIX = "imagepullsecret"
QA_CACHE_FILE = APP_NAME_SHORT + "qacache.yaml"
DEFAULT_CLUSTER_TYPE = "Kubernetes"
IGNORE_FILENAME = "." + APP_NAME_SHORT + "ignore"
EXPOSE_SELECTOR = GROUP_NAME + "/service.expose"
ANNOTATION_LABEL_VALUE = "true"
DEFAULT_SERVICE_PORT = 8080
DEFAULT_PVC_SIZE = "100Mi"


def _cgroup_cpu_limit(root="/sys/fs/cgroup"):
    """CPUs granted by the cgroup CPU quota (v2 ``cpu.max``, v1
    ``cpu.cfs_quota_us``/``cpu.cfs_period_us``), or None when unlimited.  A
    container or pod limited to N CPUs usually still sees every host CPU in
    its affinity mask; sizing pools from the mask oversubscribes the quota and
    gets the whole process throttled."""
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) / int(period)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f:
            quota = int(f.read())
        with open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as f:
            period = int(f.read())
        if quota > 0 and period > 0:
            return max(1, quota // period)
    except (OSError, ValueError):
        pass
    return None


def host_threads(cap, local=None):
    """Threads this process should use: the CPUs it may run on (affinity, not
    the whole machine, and no more than the cgroup CPU quota), shared among
    the ``local`` processes of this node (default: the ranks torchrun placed
    here, LOCAL_WORLD_SIZE), capped."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 4
    limit = _cgroup_cpu_limit()
    if limit is not None:
        n = min(n, limit)
    if local is None:
        try:
            local = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
        except ValueError:
            local = 1
    forced = os.environ.get("M2K_HOST_THREADS", "")
    if forced.isdigit() and int(forced) > 0:   # scaling-rehearsal knob: every pool this size
        return min(cap, int(forced))
    return max(1, min(cap, n // max(1, local)))


class _Settings:
    """Process-wide mutable configuration (the reference's package globals)."""

    def __init__(self):
        self.ignore_environment = False
        self.temp_path = TEMP_DIR_PREFIX + "temp"
        self.assets_path = os.path.join(self.temp_path, ASSETS_DIR)
        # Behaviour switch for output-affecting quirks of the reference
        # (SURVEY.md section 2.13).  "reference" keeps byte-compatible output,
        # "fixed" applies the documented bug fixes.  Crash/hang bugs are always
        # fixed regardless of this switch.
        self.compat = os.environ.get("M2K_COMPAT", "reference")
        # Number of parallel workers used for detector scripts and file sniffing.
        self.workers = int(os.environ.get("M2K_WORKERS", "0") or 0) or host_threads(32)

    @property
    def fixed(self):
        return self.compat == "fixed"


settings = _Settings()

