"""Target-cluster metadata (reference ``internal/collector/clustercollector.go``).

Storage classes come from ``<kubectl|oc> get sc -o yaml``.  The kind ->
group/version map is taken from the discovery API first - one in-process pass
over ``/api``, ``/apis`` and every group/version document, straight to the
API server named by the kubeconfig (``kubeapi.py``; a single ``kubectl
proxy`` process when the kubeconfig needs a credential plugin) - and, if
that fails, from the CLI (``api-resources -o name`` + ``explain``).
Versions are finally ordered by the global group policy: ``*.openshift.io``,
``*.k8s.io``, ``apps``, ``extensions``, other named groups, then the core
group.
"""

import functools
import os
import re
import shutil

from ..k8s import scheme
from ..models import collection
from ..utils import common, log, yamlio
from ..utils.constants import DEFAULT_DIRECTORY_PERMISSION, settings
from ..utils.lazyre import lazy as _lazy_re
from . import Collector, CommandError, run

GLOBAL_GROUP_ORDER = [r"^.+\.openshift\.io$", r"^.+\.k8s\.io$", r"^apps$", r"^extensions$"]

# Masterminds/semver v3.1.1 (go.mod:9): NewVersion's pattern and Compare
_SEMVER_RE = _lazy_re(r"v?([0-9]+)(\.[0-9]+)?(\.[0-9]+)?(-([0-9A-Za-z\-]+(\.[0-9A-Za-z\-]+)*))?"
                       r"(\+([0-9A-Za-z\-]+(\.[0-9A-Za-z\-]+)*))?\Z")


def _semver(v):
    """(major, minor, patch, prerelease) or None when NewVersion fails."""
    m = _SEMVER_RE.match(v)
    if not m:
        return None
    pre = m.group(5) or ""
    for part in pre.split(".") if pre else ():
        if part.isdigit() and len(part) > 1 and part[0] == "0":
            return None               # ErrInvalidPrerelease: numeric identifier with a leading zero
    nums = [int(x.lstrip(".")) if x else 0 for x in (m.group(1), m.group(2), m.group(3))]
    if any(n >= 1 << 64 for n in nums):
        return None
    return nums[0], nums[1], nums[2], pre


def _semver_pre_part(s, o):
    if s == o:
        return 0
    if s == "":
        return -1
    if o == "":
        return 1
    sn, on = s.isdigit() and int(s) < 1 << 64, o.isdigit() and int(o) < 1 << 64
    if not sn and not on:
        return 1 if s > o else -1
    if not sn:
        return 1
    if not on:
        return -1
    return 1 if int(s) > int(o) else -1


def _semver_compare(a, b):
    for x, y in zip(a[:3], b[:3]):
        if x != y:
            return 1 if x > y else -1
    ps, po = a[3], b[3]
    if ps == po == "":
        return 0
    if ps == "":
        return 1
    if po == "":
        return -1
    sp, op = ps.split("."), po.split(".")
    for i in range(max(len(sp), len(op))):
        d = _semver_pre_part(sp[i] if i < len(sp) else "", op[i] if i < len(op) else "")
        if d:
            return d
    return 0


def _gv_string(group, version):
    return version if group == "" else "%s/%s" % (group, version)


def _parse_gv(gv):
    g, v = common.parse_group_version(gv)
    return g, v


class ClusterCollector(Collector):
    annotations = ("k8s",)

    def __init__(self):
        self.cluster_cmd = ""

    # -- helpers -----------------------------------------------------------
    def get_cluster_command(self):
        if self.cluster_cmd:
            return self.cluster_cmd
        for cmd in ("kubectl", "oc"):
            if shutil.which(cmd):
                self.cluster_cmd = cmd
                return cmd
            log.warning('Unable to find the %s command. Error: %r', cmd,
                        'exec: "%s": executable file not found in $PATH' % cmd)
        return ""

    def _run(self, *args, combined=False):
        return run([self.get_cluster_command()] + list(args), combined=combined)

    def get_cluster_context_name(self):
        name = self._run("config", "current-context").decode("utf-8", "replace")
        # the reference keeps kubectl's trailing newline in the name
        return name.strip() if settings.fixed else name

    def interpret_error(self, output):
        for term in ("Unauthorized", "Username"):
            if self.get_cluster_command() == "oc" and term in output:
                return "Please login to cluster before running collect. (e.g. oc login <cluster url> --token=<token string>)"
            if self.get_cluster_command() == "kubectl" and term in output:
                return ("Please configure the cluster authentication with following instructions: "
                        "[https://kubernetes.io/docs/reference/kubectl/cheatsheet/#kubectl-context-and-configuration]")
        return ""

    def get_storage_classes(self):
        try:
            out = self._run("get", "sc", "-o", "yaml", combined=True)
        except CommandError as e:
            desc = self.interpret_error(e.output.decode("utf-8", "replace"))
            if desc:
                log.warning("Error while running %s. %s", self.get_cluster_command(), desc)
            else:
                # exec.Cmd's String(): the looked-up path and the arguments
                log.warning("Error while fetching storage classes using command [%s get sc -o yaml]",
                            shutil.which(self.get_cluster_command()) or self.get_cluster_command())
            raise
        try:
            doc = yamlio.load(out.decode("utf-8", "replace")) or {}
        except yamlio.YAMLError as e:
            log.error("Error in unmarshalling yaml: %s. Skipping.", e)
            raise
        names = []
        for sc in (doc.get("items") if isinstance(doc, dict) else None) or []:
            if isinstance(sc, dict):
                names.append(str((sc.get("metadata") or {}).get("name", "")))
            else:
                # %T of the failed assertion's zero value (clustercollector.go:150-156)
                log.warning("Unknown type detected in cluster metadata [%s]", "map[string]interface {}")
        return names

    # -- discovery API -----------------------------------------------------
    def get_server_groups(self, client):
        """[(name, preferred_gv, [gv...])] like ``ServerGroups()`` (core group first)."""
        groups = []
        core = client.get_json("/api")
        versions = core.get("versions") or []
        if versions:
            groups.append(("", versions[0], list(versions)))
        for g in client.get_json("/apis").get("groups") or []:
            gvs = [v.get("groupVersion", "") for v in g.get("versions") or []]
            pref = (g.get("preferredVersion") or {}).get("groupVersion", gvs[0] if gvs else "")
            groups.append((g.get("name", ""), pref, gvs))
        return groups

    def get_preferred_resources_using_api(self, groups):
        gv_list = []
        for name, pref, gvs in groups:
            if pref == "":
                continue
            gv_list.append(pref)
            for pgv in scheme.prioritized_versions_for_group(name):
                if pgv == pref:
                    continue
                if pgv in gvs:
                    gv_list.append(pgv)
            for gv in gvs:
                if gv not in gv_list:
                    gv_list.append(gv)
        return gv_list

    def get_kinds_for_groups(self, client, groups):
        """``ServerGroupsAndResources``: every group/version document, fetched
        concurrently.  Subresources count too (``deployments/scale`` makes
        ``Scale`` an apps/v1 kind), as in the reference.  A failed group makes
        client-go return an error and the reference fall back to the CLI;
        "fixed" compat keeps the groups that answered."""
        gvs_all = [gv for _n, _p, gvs in groups for gv in gvs]
        docs = client.get_many(["/api/" + gv if "/" not in gv else "/apis/" + gv for gv in gvs_all])
        kinds = {}
        for gv in gvs_all:
            res = docs["/api/" + gv if "/" not in gv else "/apis/" + gv]
            if isinstance(res, Exception):
                if not settings.fixed:
                    raise RuntimeError("unable to retrieve the complete list of server APIs: %s" % res)
                log.warning("Ignoring group-version [%s]. %s", gv, res)
                continue
            for r in res.get("resources") or []:
                lst = kinds.setdefault(r.get("kind", ""), [])
                if gv not in lst:
                    lst.append(gv)
        return kinds

    def sort_gv_by_preference(self, pref, kinds):
        for kind, gvs in kinds.items():
            ordered = [p for p in pref if p in gvs]
            if settings.fixed:
                # the reference's inverted parse check drops every version that is not preferred
                rest = [p for p in gvs if p not in ordered]
                ordered.extend(self.cluster_by_groups_and_sort_versions(rest))
            kinds[kind] = ordered

    def collect_using_api(self):
        from . import kubeapi  # http.client/ssl: only when the k8s collector runs
        try:
            client = kubeapi.open_client(self.get_cluster_command())
        except kubeapi.ClientConfigError as e:      # getAPI (clustercollector.go:179-186, 301-306)
            log.warning("Failed to get the default config for the cluster API client. Error: %r", str(e))
            log.warning("Failed to api handle for cluster")
            raise
        try:
            err = "Failed to retrieve preferred group information from cluster"
            try:
                groups = self.get_server_groups(client)
            except kubeapi.DiscoveryError:
                log.error("API request for server-group list failed")
                log.warning(err)
                raise
            gv_list = self.get_preferred_resources_using_api(groups)
            if not gv_list:
                log.warning(err)
                raise RuntimeError(err)
            err = "Failed to retrieve <kind, group-version> information from cluster"
            try:
                kinds = self.get_kinds_for_groups(client, groups)
            except (kubeapi.DiscoveryError, RuntimeError):
                log.warning(err)
                raise
            if not kinds:
                log.warning(err)
                raise RuntimeError(err)
        finally:
            client.close()
        self.sort_gv_by_preference(gv_list, kinds)
        return kinds

    # -- CLI fallback ------------------------------------------------------
    def get_gvk_using_name_cli(self, name):
        out = self._run("explain", name).decode("utf-8", "replace")
        lines = out.split("\n")
        if len(lines) < 2:
            raise ValueError("Description incomplete")
        if "KIND" not in lines[0]:
            # clustercollector.go:622 returns the command's nil error here: an
            # explain that starts with another line (newer kubectl prints GROUP
            # first) gives kind "" and version "" without an error
            if settings.fixed:
                raise ValueError("no KIND")
            return "", ""
        kind = lines[0].split(":")[1].strip()
        group, version = "", ""
        if "VERSION" in lines[1]:
            parts = lines[1].split(":")[1].strip().split("/")
            if len(parts) == 2:
                group, version = parts
            else:
                version = parts[0]
        return kind, _gv_string(group, version)

    def is_supported_gv(self, kind, gv):
        """``isSupportedGV``: (supported, error text)."""
        try:
            out = self._run("explain", kind, "--api-version=" + gv, "--recursive").decode("utf-8", "replace")
        except (CommandError, OSError) as e:
            log.debug("Error while running %s for verifying [%s]\n", self.get_cluster_command(), gv)
            return False, str(e) if isinstance(e, CommandError) else common.go_exit_status(127)
        lines = out.split("\n")
        if len(lines) < 2:
            return False, "Description incomplete"
        if "VERSION" in lines[1]:
            return True, None
        return False, "GV [%s] not found" % gv

    def get_preferred_gv_using_cli(self, kind, groups):
        out = []
        for group, _v in groups:
            prio = scheme.prioritized_versions_for_group(group)
            if prio:
                for gv in prio:
                    ok, err = self.is_supported_gv(kind, gv)
                    if ok:
                        out.append(gv)
                    else:
                        log.debug("Group version not found by CLI for kind [%s] : %s", kind, err)
            else:
                try:
                    out.append(self.get_gvk_using_name_cli(kind)[1])
                except (CommandError, OSError, ValueError):
                    pass
        return out

    def collect_using_cli(self):
        try:
            out = self._run("api-resources", "-o", "name").decode("utf-8", "replace")
        except (CommandError, OSError) as e:
            log.error("Error while running kubectl api-resources: %s", e)
            raise
        log.debug("Got kind information for cluster")
        kinds = {}
        for name in out.split("\n"):
            parts = name.split(".")
            try:
                kind, gv = self.get_gvk_using_name_cli(parts[0])
            except (CommandError, OSError, ValueError):
                log.debug("Erroring parsing kind from CLI output")
                continue
            group = ".".join(p.strip() if i > 0 else p for i, p in enumerate(parts[1:]))
            if group:
                kinds.setdefault(kind, []).append((group, ""))
            else:
                kinds[kind] = [("", gv)]
        api = {}
        for kind in sorted(kinds):
            groups = kinds[kind]
            if len(groups) == 1 and groups[0][0] == "":
                api[kind] = [groups[0][1]]
                continue
            api[kind] = self.get_preferred_gv_using_cli(kind, groups)
        return api

    # -- ordering ----------------------------------------------------------
    @staticmethod
    def _matching(group_regex, gvs):
        rx = re.compile(group_regex)
        out = []
        for gv in gvs:
            g, _ = _parse_gv(gv)
            if g and rx.search(g):
                out.append(gv)
        return out

    def group_order_policy(self, kinds):
        for kind, gvs in kinds.items():
            ordered = []
            for rx in GLOBAL_GROUP_ORDER:
                ordered.extend(self._matching(rx, gvs))
            for gv in gvs:
                g, _ = _parse_gv(gv)
                if common.is_string_present(ordered, gv):
                    continue
                if g != "":
                    ordered.append(gv)
            for gv in gvs:
                g, _ = _parse_gv(gv)
                if g == "":
                    ordered.append(gv)
            kinds[kind] = ordered if ordered else gvs

    @staticmethod
    def sort_versions(versions):
        """``sortVersionList`` (clustercollector.go:412-456): ``alpha``/``beta``
        become ``-alpha.``/``-beta.`` so Masterminds semver v3 reads ``v1beta2``
        as 1.0.0-beta.2, the list is sorted newest first by semver precedence
        (``v2beta1`` ranks above ``v1``), and the names are restored.  A
        version semver rejects is logged and, where the reference's sort would
        dereference its nil entry and panic, kept after the others."""
        parsed, bad = [], []
        for v in versions:
            for key in ("alpha", "beta"):
                if key in v:
                    v = v.replace(key, "-%s." % key)
                    break
            sv = _semver(v)
            if sv is None:
                log.warning("Skipping Version: %s", v)
                bad.append(v)
            else:
                parsed.append((sv, v))
        parsed.sort(key=functools.cmp_to_key(lambda a, b: _semver_compare(a[0], b[0])), reverse=True)
        out = []
        for _sv, v in parsed + [(None, b) for b in bad]:
            for key in ("alpha", "beta"):
                if "-%s." % key in v:
                    v = v.replace("-%s." % key, key)
                    break
            out.append(v)
        return out

    def cluster_by_groups_and_sort_versions(self, gvs):
        """``clusterByGroupsAndSortVersions``; groups in sorted order (the
        reference ranges over a map)."""
        by_group = {}
        for gv in gvs:
            g, v = _parse_gv(gv)
            by_group.setdefault(g, []).append(v)
        out = []
        for g in sorted(by_group):
            for v in self.sort_versions(by_group[g]):
                out.append(_gv_string(g, v))
        return out

    # -- entry point -------------------------------------------------------
    def collect(self, input_path, output_path):
        output_path = os.path.join(output_path, "clusters")
        try:
            os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        except OSError as e:
            err = common.go_path_error(e, "mkdir")
            log.error("Unable to create output directory at path %r Error: %r", output_path, err)
            raise RuntimeError(err) from e
        if self.get_cluster_command() == "":
            msg = "No kubectl or oc in path. Add kubectl to path and rerun to collect data about the cluster in context."
            log.warning(msg)
            raise RuntimeError(msg)
        try:
            name = self.get_cluster_context_name()
        except (CommandError, OSError) as e:
            log.warning("Unable to access cluster in context : %s", e)
            raise
        cm = collection.ClusterMetadata(name)
        try:
            cm.spec.storage_classes = self.get_storage_classes()
        except Exception:  # noqa: BLE001
            cm.spec.storage_classes = []
        try:
            kinds = self.collect_using_api()
        except Exception as e:  # noqa: BLE001
            log.warning("Failed to collect using the API. Error: %r . Falling back to using the CLI.", str(e))
            try:
                kinds = self.collect_using_cli()
            except Exception as e2:  # noqa: BLE001
                log.warning("Failed to collect using the CLI. Error: %r", str(e2))
                raise
        self.group_order_policy(kinds)
        cm.spec.api_kind_version_map = kinds
        common.write_yaml(os.path.join(output_path, common.normalize_for_filename(cm.name) + ".yaml"), cm)
