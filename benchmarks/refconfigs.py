"""The five BASELINE.json configurations over the reference's own ``samples/``
corpus, shared by ``bench.py``, ``benchmarks/baseline_configs.py`` and
``tests/test_reference_configs.py``.

Each configuration is a command a user of the reference would type, run
against a private copy of its inputs laid out the same way every time
(``<work>/samples``, ``<work>/out``), so that paths embedded in the output
(``copysources.sh``) are reproducible:

====================  ==========================================================
``golang``            ``move2kube translate -s samples/golang --qaskip``
``docker-compose``    ``move2kube translate -s samples/docker-compose --qaskip``
``java-cnb``          ``move2kube translate -s java --qaskip -q java-cnb-qacache.yaml``
                      where ``java/`` holds ``samples/java-maven`` and
                      ``samples/java-gradle``; the cache picks the CNB mode, and
                      a ``podman`` stand-in on ``PATH`` answers the reference's
                      container-runtime CNB provider
                      (``internal/containerizer/cnb/containerruntimeprovider.go``)
``cf``                ``move2kube collect -a cf -s cf -o collect`` (``cf`` CLI
                      stand-in), the collected ``m2k_collect/`` copied into the
                      source tree, then ``move2kube translate -s cf --qaskip``
``helm-openshift``    ``move2kube translate -s samples --qaskip -q
                      helm-openshift-qacache.yaml``: the whole corpus to a Helm
                      chart for the Openshift profile (DeploymentConfig, Route,
                      ImageStream group/versions), plus the operator
                      (``operator-sdk`` stand-in)
====================  ==========================================================

The expected output trees live in ``tests/golden/reference/<config>/``.  They
are derived from the reference's code and fixtures (``PROVENANCE.md`` there)
and are never rewritten by a test run; allowed byte differences from what the
Go binary would write are listed with their reason in ``DEVIATIONS.md``.

External tools are stand-ins on ``PATH`` (``tests/fixtures/configs/bin``);
``HOME`` points at an empty directory so ``~/.docker/config.json`` of the host
does not leak into the registry questions (``registrycustomizer.go:71``).
"""

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAMPLES = os.path.join(ROOT, "samples")
FIXTURES = os.path.join(ROOT, "tests", "fixtures")
CONFIG_FIXTURES = os.path.join(FIXTURES, "configs")
STUB_BIN = os.path.join(CONFIG_FIXTURES, "bin")
CF_APP = os.path.join(FIXTURES, "extra_samples", "cfapp")
GOLDEN_REF = os.path.join(ROOT, "tests", "golden", "reference")
PROJECT = "myproject"  # the CLI default (-n)

# name -> (layout, source dir relative to <work>, QA caches, CNB probing on, collect annotations
#          [, extra environment])
CONFIGS = {
    "golang": ("samples", "samples/golang", [], False, None),
    "docker-compose": ("samples", "samples/docker-compose", [], False, None),
    "java-cnb": ("java", "java", ["java-cnb-qacache.yaml"], True, None),
    "cf": ("cf", "cf", [], True, ["cf"]),
    "helm-openshift": ("samples", "samples", ["helm-openshift-qacache.yaml"], False, None),
}
HEADLINE = "helm-openshift"
# Not a BASELINE configuration: the headline corpus with every default
# (Yamls, Kubernetes profile, no operator) - the per-service reference point
# for the cost of the Helm/Openshift output.
EXTRA_CONFIGS = {
    "samples-yamls": ("samples", "samples", [], False, None),
}

# The capability surface beyond the five BASELINE configurations, pinned by
# expected trees in ``tests/golden/reference/coverage/<name>``
# (``tests/test_coverage_trees.py``).  QA answers are given as a dict
# {question: answer} and written to a cache file when the run is prepared.
PROFILES = ("AWS-EKS", "Azure-AKS", "GCP-GKE", "IBM-IKS", "IBM-Openshift", "Kubernetes", "Openshift")
GOLDEN_COVERAGE = os.path.join(GOLDEN_REF, "coverage")
CARRIED_OVER = os.path.join(FIXTURES, "carried_over")
CARRIED_OVER_KINDS = os.path.join(FIXTURES, "carried_over_kinds")
GIT_REPOS = os.path.join(FIXTURES, "git_repos")
STORAGE_CLASS = os.path.join(FIXTURES, "storage_class")
FIXED = {"M2K_COMPAT": "fixed"}
Q_ARTIFACT = "Choose the artifact type:"
Q_CLUSTER = "Choose the cluster type:"


def _coverage_configs():
    out = {}
    for p in PROFILES:
        # samples/ in Yamls mode on every built-in cluster profile
        out["profiles/" + p] = ("samples", "samples", {Q_CLUSTER: p}, False, None)
    out["artifacts/knative-kubernetes"] = ("samples", "samples", {Q_ARTIFACT: "Knative"}, False, None)
    out["artifacts/knative-openshift"] = ("samples", "samples", {Q_ARTIFACT: "Knative", Q_CLUSTER: "Openshift"},
                                          False, None)
    out["artifacts/helm-kubernetes"] = ("samples", "samples", {Q_ARTIFACT: "Helm"}, False, None)
    for p in ("Kubernetes", "Openshift", "AWS-EKS", "IBM-Openshift"):
        # old-version Kubernetes/OpenShift YAMLs carried over to each profile
        out["carried-over/" + p] = ("carried", "carried", {Q_CLUSTER: p}, False, None)
    # kinds the target cluster lacks (Route/Ingress/LoadBalancer and NodePort
    # Services, Pods, Jobs, ReplicationControllers, ConfigMaps/Secrets) carried
    # over or generated for Kubernetes, Openshift and a custom cluster profile
    # found in the source tree (ClusterMetadata "minimal-cluster")
    for p in ("Kubernetes", "Openshift", "minimal-cluster"):
        out["carried-over-kinds/" + p] = ("carried-kinds", "carried", {Q_CLUSTER: p}, False, None)
    # source trees that are git repos with an origin remote
    out["git-repos"] = ("git", "git", {}, False, None)
    # two compose services with a named volume each: two PVCs, one storage
    # class question for all of them (the reference assigns
    # the answer to a loop copy, so no PVC gets it)
    out["storage-class"] = ("storage", "storage", {}, False, None)
    # M2K_COMPAT=fixed wherever it changes bytes (DEVIATIONS.md section 5):
    # cf (app2 containerized as Manual, Manualimages.md written) and the
    # storage class applied to the PVCs
    out["compat-fixed/cf"] = ("cf", "cf", {}, True, ["cf"], FIXED)
    out["compat-fixed/storage-class"] = ("storage", "storage", {}, False, None, FIXED)
    # ... the version conversion of carried-over objects (k8s/convert.py:convert_fixed)
    for p in ("Kubernetes", "Openshift", "AWS-EKS", "IBM-Openshift"):
        out["compat-fixed/carried-over/" + p] = ("carried", "carried", {Q_CLUSTER: p}, False, None, FIXED)
    # ... and the generated Ingress on the profiles that prefer networking.k8s.io/v1beta1
    for p in ("AWS-EKS", "Azure-AKS", "GCP-GKE"):
        out["compat-fixed/profiles/" + p] = ("samples", "samples", {Q_CLUSTER: p}, False, None, FIXED)
    return out


COVERAGE_CONFIGS = _coverage_configs()


def _lookup(name):
    for table in (CONFIGS, EXTRA_CONFIGS, COVERAGE_CONFIGS):
        if name in table:
            return table[name]
    raise KeyError(name)


def golden_dir(name):
    return os.path.join(GOLDEN_COVERAGE if name in COVERAGE_CONFIGS else GOLDEN_REF, name)


def qacache_text(answers):
    """A ``QACache`` file answering Select questions (``types/qaengine/cache.go``)."""
    lines = ["apiVersion: move2kube.konveyor.io/v1alpha1", "kind: QACache", "spec:", "  solutions:"]
    for desc, ans in answers.items():
        lines += ["    - description: '%s'" % desc, "      solution:", "        type: Select",
                  "        answer:", "          - %s" % ans, "      resolved: true"]
    return "\n".join(lines) + "\n"


def _copy_git_repos(dst):
    """``tests/fixtures/git_repos``: every ``dot-git`` directory becomes ``.git``
    (a nested ``.git`` cannot be committed)."""
    shutil.copytree(GIT_REPOS, dst, symlinks=True)
    for dp, dns, _fns in os.walk(dst):
        if "dot-git" in dns:
            os.rename(os.path.join(dp, "dot-git"), os.path.join(dp, ".git"))
            dns.remove("dot-git")


class Run:
    """One prepared configuration: inputs copied under ``work``."""

    def __init__(self, name, work):
        self.name = name
        self.work = os.path.abspath(work)
        layout, src, caches, cnb, collect, *extra = _lookup(name)
        self.extra_env = dict(extra[0]) if extra else {}
        self.layout = layout
        self.src = os.path.join(self.work, src)
        self.answers = caches if isinstance(caches, dict) else None
        if self.answers is not None:
            self.caches = [os.path.join(self.work, "qacache.yaml")] if self.answers else []
        else:
            self.caches = [os.path.join(CONFIG_FIXTURES, c) for c in caches]
        self.cnb = cnb
        self.collect_annotations = collect
        self.outdir = os.path.join(self.work, "out")
        self.home = os.path.join(self.work, "home")

    @property
    def out(self):
        return os.path.join(self.outdir, PROJECT)

    def prepare(self):
        os.makedirs(self.home, exist_ok=True)
        if self.layout == "samples":
            shutil.copytree(SAMPLES, os.path.join(self.work, "samples"), symlinks=True)
        elif self.layout == "java":
            root = os.path.join(self.work, "java")
            os.makedirs(root)
            with open(os.path.join(root, ".m2kignore"), "w") as f:
                f.write(".\n")
            for d in ("java-maven", "java-gradle"):
                shutil.copytree(os.path.join(SAMPLES, d), os.path.join(root, d), symlinks=True)
        elif self.layout == "cf":
            shutil.copytree(CF_APP, os.path.join(self.work, "cf"), symlinks=True)
        elif self.layout == "carried":
            shutil.copytree(CARRIED_OVER, self.src, symlinks=True)
        elif self.layout == "carried-kinds":
            shutil.copytree(CARRIED_OVER_KINDS, self.src, symlinks=True)
        elif self.layout == "git":
            _copy_git_repos(self.src)
        elif self.layout == "storage":
            shutil.copytree(STORAGE_CLASS, self.src, symlinks=True)
        if self.answers:
            with open(self.caches[0], "w") as f:
                f.write(qacache_text(self.answers))
        return self

    def env(self, base=None):
        """Environment of a configuration run (stand-in tools, private HOME)."""
        env = dict(os.environ if base is None else base)
        env["PATH"] = STUB_BIN + os.pathsep + env.get("PATH", "")
        env["HOME"] = self.home
        env["M2K_NO_NETWORK"] = "1"
        env["M2K_DISABLE_CNB"] = "0" if self.cnb else "1"
        env.update(self.extra_env)
        return env

    # -- in-process -------------------------------------------------------
    def apply_env(self):
        """Switch this process to the configuration's environment; returns an undo."""
        keys = ("PATH", "HOME", "M2K_NO_NETWORK", "M2K_DISABLE_CNB") + tuple(self.extra_env)
        saved = {k: os.environ.get(k) for k in keys}
        os.environ.update(self.env())
        from move2kube_amd.utils.constants import settings
        saved_compat = settings.compat
        settings.compat = os.environ.get("M2K_COMPAT", "reference")   # read once at start-up by the CLI

        def restore():
            settings.compat = saved_compat
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        return restore

    def collect_inprocess(self, session):
        # what `collect -o <work>/collect` does (cmd/move2kube/collect.go:41-73)
        cdir = os.path.join(self.work, "collect", "m2k_collect")
        shutil.rmtree(cdir, ignore_errors=True)
        session.collect(self.src, os.path.dirname(cdir), self.collect_annotations)
        dst = os.path.join(self.src, "m2k_collect")
        shutil.rmtree(dst, ignore_errors=True)
        shutil.copytree(cdir, dst)

    def step(self, session):
        """One in-process run of the configuration's commands (``session`` is an
        ``api.Session(qaskip=True, qacaches=run.caches, ignore_env=False)``)."""
        if self.collect_annotations:
            self.collect_inprocess(session)
        return session.translate(self.src, self.outdir, name=PROJECT)

    def session(self):
        from move2kube_amd import api
        return api.Session(qaskip=True, qacaches=self.caches, ignore_env=False)

    # -- CLI processes ------------------------------------------------------
    def cli_commands(self):
        """argv lists (after ``python -m move2kube_amd``) of the user's commands."""
        cmds = []
        if self.collect_annotations:
            cmds.append(["collect", "-a", ",".join(self.collect_annotations), "-s", self.src,
                         "-o", os.path.join(self.work, "collect")])
        t = ["translate", "-s", self.src, "-o", self.outdir, "--qaskip"]
        for c in self.caches:
            t += ["-q", c]
        cmds.append(t)
        return cmds

    def run_cli(self, extra_env=None, cwd=None, launcher=None):
        """Run the commands as separate ``python -m move2kube_amd`` processes
        (or ``launcher + argv``, e.g. :func:`release_launcher`)."""
        env = self.env()
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        if extra_env:
            env.update(extra_env)
        prefix = launcher or [sys.executable, "-m", "move2kube_amd"]
        for argv in self.cli_commands():
            p = subprocess.run(prefix + argv, env=env, cwd=cwd or self.work,
                               stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            if p.returncode != 0:
                raise RuntimeError("%s failed: %s" % (argv[0], p.stderr.decode(errors="replace")[-2000:]))
            if argv[0] == "collect":
                dst = os.path.join(self.src, "m2k_collect")
                shutil.rmtree(dst, ignore_errors=True)
                shutil.copytree(os.path.join(self.work, "collect", "m2k_collect"), dst)
        return self.out


def release_launcher(dirpath):
    """argv prefix of what ``bin/move2kube`` of a release archive runs
    (``scripts/builddist.py``: ``python3 -S bin/m2k_main.py``), with the entry
    script written to ``dirpath`` and pointed at this tree."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import builddist
    entry = os.path.join(dirpath, "m2k_main.py")
    with open(entry, "w") as f:
        f.write(builddist.ENTRY.replace("os.path.dirname(os.path.dirname(os.path.abspath(__file__)))", repr(ROOT)))
    return [sys.executable, "-S", entry]


def workdir_root(choice):
    """Where the inputs and output trees of the run live.  ``auto``: a tmpfs
    (``/dev/shm``) when one is writable with room to spare, else the default
    temp dir.  Every step deletes the previous output tree and writes a new one
    (~500 file creations and deletions per step); on the GPU hosts' ext4 /
    overlay scratch disks (mounted with ``discard``) that churn builds a
    backlog that slows every later run on the machine - a 1-rank step went
    from 20 to 50 ms after a few multi-rank runs - so a disk-backed number
    depends on what ran before.  ``disk`` forces the default temp dir."""
    if choice == "disk":
        return None, "disk"
    if choice != "auto":
        return choice, "given"
    shm = "/dev/shm"
    try:
        st = os.statvfs(shm)
        if os.access(shm, os.W_OK) and st.f_bavail * st.f_frsize >= (512 << 20):
            return shm, "tmpfs"
    except OSError:
        pass
    return None, "disk"


def tree_files(root):
    out = {}
    for dp, _dn, fns in os.walk(root):
        for fn in fns:
            p = os.path.join(dp, fn)
            out[os.path.relpath(p, root)] = p
    return out


WORK_PLACEHOLDER = b"$WORK"


def diff_files(actual_root, expected_root, work=None):
    """Relative paths that differ, are missing or are extra (sorted).  With
    ``work``, that directory's path in the actual files reads as ``$WORK``
    (the QA cache records absolute ``~/.ssh`` paths under the run's HOME)."""
    a, g = tree_files(actual_root), tree_files(expected_root)
    bad = sorted(set(a) ^ set(g))
    for rel in sorted(set(a) & set(g)):
        with open(a[rel], "rb") as fa, open(g[rel], "rb") as fg:
            data = fa.read()
            if work:
                data = data.replace(os.fsencode(work), WORK_PLACEHOLDER)
            if data != fg.read():
                bad.append(rel)
    return sorted(bad)


def write_expected_tree(name, actual_root, work):
    """Copy a run's output to ``golden_dir(name)`` with the work directory
    replaced by ``$WORK``.  Only ``python benchmarks/refconfigs.py --write``
    calls this: expected trees change by reviewed commits, never from tests."""
    dst = golden_dir(name)
    shutil.rmtree(dst, ignore_errors=True)
    for rel, src in tree_files(actual_root).items():
        out = os.path.join(dst, rel)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(src, "rb") as f:
            data = f.read().replace(os.fsencode(work), WORK_PLACEHOLDER)
        with open(out, "wb") as f:
            f.write(data)
        shutil.copymode(src, out)
    return dst


def _main(argv):
    import argparse
    import tempfile
    ap = argparse.ArgumentParser(description="write expected trees of coverage configurations")
    ap.add_argument("--write", nargs="+", required=True, metavar="NAME",
                    help="coverage configurations (or 'all') whose expected tree is (re)written")
    args = ap.parse_args(argv)
    names = sorted(COVERAGE_CONFIGS) if args.write == ["all"] else args.write
    sys.path.insert(0, ROOT)
    for name in names:
        if name not in COVERAGE_CONFIGS:
            raise SystemExit("not a coverage configuration: %s" % name)
        work = tempfile.mkdtemp(prefix="m2k-cov-")
        try:
            run = Run(name, work).prepare()
            undo = run.apply_env()
            try:
                with run.session() as s:
                    out = run.step(s)
            finally:
                undo()
            print(write_expected_tree(name, out, run.work))
        finally:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    _main(sys.argv[1:])


def manifest_diff_vs_ref(name, actual_root):
    """Number of files differing from the reference-derived expected tree."""
    golden = golden_dir(name)
    if not os.path.isdir(golden):
        return None
    return len(diff_files(actual_root, golden))
