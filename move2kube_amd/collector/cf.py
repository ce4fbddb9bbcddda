"""Cloud Foundry collectors (reference ``internal/collector/cfappscollector.go``,
``cfcontainertypescollector.go``).

* :class:`CfAppsCollector` - running apps via ``cf curl /v2/apps``.
* :class:`CFContainerTypesCollector` - maps every buildpack in use (manifests
  under the source dir, or the foundation's ``cf buildpacks`` + app list) to
  the CNB builder whose buildpack list holds its closest match.  The matching
  is one batched all-pairs edit-distance matrix (GPU kernel for large
  foundations) instead of the reference's per-name nested scans.
"""

import os

from ..models import collection
from ..models import plan as plantypes
from ..utils import common, fastjson, log
from ..utils.constants import DEFAULT_DIRECTORY_PERMISSION, settings
from . import Collector, concurrently, run


def _cf_apps():
    out = run(["cf", "curl", "/v2/apps"])
    log.debug("Cf Curl output %s", out)
    try:
        data = fastjson.loads(out)
    except ValueError as e:
        log.error("Error in unmarshalling yaml: %s. Skipping.", e)
        raise
    res = []
    for r in (data or {}).get("resources") or []:
        res.append((r or {}).get("entity") or {})
    return res


def _s(v):
    return "" if v is None else str(v)


class CfAppsCollector(Collector):
    annotations = ("cf", "cloudfoundry")

    def collect(self, input_path, output_path):
        try:
            apps = _cf_apps()
        except Exception as e:  # noqa: BLE001
            log.error("%s", e)
            raise
        output_path = os.path.join(output_path, "cf")
        try:
            os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        except OSError as e:
            log.error("Unable to create outputPath %s : %s", output_path, common.go_path_error(e, "mkdir"))
        inst = collection.CfInstanceApps()
        file_name = "instanceapps_"
        log.debug("Detected %d apps", len(apps))
        for ent in apps:
            app = collection.CfApplication(_s(ent.get("name")))
            log.debug("Reading info about %s", app.name)
            if _s(ent.get("buildpack")) != "null":
                app.buildpack = _s(ent.get("buildpack"))
            if _s(ent.get("detected_buildpack")) != "null":
                app.detected_buildpack = _s(ent.get("detected_buildpack"))
            if _s(ent.get("dockerimage")) != "null":
                app.docker_image = _s(ent.get("dockerimage"))
            app.instances = int(ent.get("instances") or 0)
            app.memory = int(ent.get("memory") or 0)
            app.env = {k: _s(v) for k, v in (ent.get("environment_json") or {}).items()}
            app.ports = [int(p) for p in ent.get("ports") or []]
            inst.applications.append(app)
            file_name += app.name
        path = os.path.join(output_path, common.normalize_for_filename(file_name) + ".yaml")
        common.write_yaml(path, inst)


def get_all_cf_instance_buildpacks():
    out = run(["cf", "buildpacks"]).decode("utf-8", "replace")
    bps = []
    for line in out.split("\n"):
        if line == "Getting buildpacks...":
            continue
        f = line.split()
        if not f or f[0] == "buildpack":
            continue
        bps.append(f[0])
    return bps


def get_all_cf_app_buildpacks():
    bps = []
    for ent in _cf_apps():
        if _s(ent.get("buildpack")):
            bps.append(_s(ent.get("buildpack")))
        if _s(ent.get("detected_buildpack")):
            bps.append(_s(ent.get("detected_buildpack")))
    return bps


def get_all_used_buildpacks(directory):
    from ..source.cfmanifest import read_application_manifest
    bps = []
    for path in common.get_files_by_ext(directory, [".yml", ".yaml"]):
        try:
            apps, _ = read_application_manifest(path, "", plantypes.YAMLS)
        except Exception as e:  # noqa: BLE001
            log.debug("Error while trying to parse manifest : %s", e)
            continue
        for a in apps:
            if a.buildpack.is_set:
                bps.append(a.buildpack.value)
            bps.extend(a.buildpacks)
    return bps


def get_cf_buildpack_names(input_path):
    names = []

    def add(found, what):
        if isinstance(found, Exception):
            log.warning(what, found)
            return
        for b in found:
            if not common.is_string_present(names, b):
                names.append(b)

    if input_path:
        try:
            found = get_all_used_buildpacks(input_path)
        except Exception as e:  # noqa: BLE001
            found = e
        add(found, "Unable to find used buildpacks : %s")
    else:
        for src, what in ((get_all_cf_instance_buildpacks, "Unable to collect buildpacks from cf instance : %s"),
                          (get_all_cf_app_buildpacks, "Unable to find used buildpacks : %s")):
            try:
                found = src()
            except Exception as e:  # noqa: BLE001
                found = e
            add(found, what)
    return names


def get_buildpack_containerizers(names, options):
    """For each buildpack name: the CNB target option (builder image) whose
    closest buildpack is the closest overall (``getBuildpackContainerizer``).

    ``options`` maps builder -> [buildpack ids].  Stage 1 picks, per builder,
    the buildpack closest to the name; stage 2 picks the closest of those
    winners (the first builder claiming a buildpack keeps it)."""
    builders = sorted(options)
    out = []
    if not names:
        return out
    stage1 = {}
    for b in builders:
        stage1[b] = common.get_closest_matching_strings(options[b], names)
    for j, name in enumerate(names):
        bpoptions, bps = {}, []
        for b in builders:
            opt = stage1[b][j]
            if opt not in bpoptions:
                bpoptions[opt] = b
                bps.append(opt)
        bp = common.get_closest_matching_string(bps, name)
        out.append(collection.BuildpackContainerizer(name, plantypes.CNB, [bpoptions.get(bp, "")]))
    return out


class CFContainerTypesCollector(Collector):
    annotations = ("cloudfoundry", "cf")

    def collect(self, input_path, output_path):
        from ..containerizer.cnb import CNBContainerizer
        output_path = os.path.join(output_path, "cf")
        os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        cz = collection.CfContainerizers()
        cnb = CNBContainerizer()
        cnb.init("")
        # the buildpack names (manifests or the foundation) and the builders'
        # buildpack lists (a container runtime) are gathered at the same time
        names, buildpacks = concurrently(lambda: get_cf_buildpack_names(input_path), cnb.get_all_buildpacks)
        for r in (names, buildpacks):
            if isinstance(r, Exception):
                raise r
        log.debug("buildpackNames : %s", names)
        log.debug("buildpacks : %s", buildpacks)
        cz.buildpack_containerizers = get_buildpack_containerizers(names, buildpacks)
        file_name = "cfcontainertypes_" + "".join(names)
        path = os.path.join(output_path, common.normalize_for_filename(file_name) + ".yaml")
        common.write_yaml(path, cz)
        if settings.fixed and not names:
            raise RuntimeError("No buildpacks found")
