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
from ..utils import common, gojson, log
from ..utils.constants import DEFAULT_DIRECTORY_PERMISSION, settings
from . import Collector, concurrently, run


# sourcetypes.CfInstanceApps and the types under it (internal/collector/sourcetypes)
_CF_APP = ("struct", "sourcetypes.CfSourceApplication", (
    ("name", gojson.STRING), ("buildpack", gojson.STRING), ("detected_buildpack", gojson.STRING),
    ("memory", ("int", "int64", 64)), ("instances", ("int", "int", 64)), ("dockerimage", gojson.STRING),
    ("ports", ("slice", "[]int32", ("int", "int32", 32))),
    ("environment_json", ("map", "map[string]string", gojson.STRING))))
_CF_APPS = ("struct", "sourcetypes.CfInstanceApps", (
    ("resources", ("slice", "[]sourcetypes.CfResource",
                   ("struct", "sourcetypes.CfResource", (("entity", _CF_APP),)))),))


def decode_cf_apps(output):
    """The entity of every resource of ``cf curl /v2/apps`` output; ValueError
    with encoding/json's text when Go would fail the Unmarshal."""
    res = gojson.unmarshal(output, _CF_APPS)
    return [(r or {}).get("entity") or {} for r in (res or {}).get("resources") or []]


def _cf_apps(skipping):
    """``cf curl /v2/apps`` decoded; the command's and the decode's errors are
    logged as the reference's two callers log them."""
    try:
        out = run(["cf", "curl", "/v2/apps"])
    except Exception as e:  # noqa: BLE001
        log.error("%s", e)
        raise
    log.debug("Cf Curl output %s", out)
    try:
        apps = decode_cf_apps(out)
    except ValueError as e:
        log.error("Error in unmarshalling yaml: %s. " + skipping, e)
        raise
    log.debug("Detected %d apps", len(apps))
    return apps


def _s(v):
    return "" if v is None else str(v)


class CfAppsCollector(Collector):
    annotations = ("cf", "cloudfoundry")

    def collect(self, input_path, output_path):
        apps = _cf_apps("Skipping.")
        output_path = os.path.join(output_path, "cf")
        try:
            os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        except OSError as e:
            log.error("Unable to create outputPath %s : %s", output_path, common.go_path_error(e, "mkdir"))
        inst = collection.CfInstanceApps()
        file_name = "instanceapps_"
        for ent in apps:
            app = collection.CfApplication(ent.get("name", ""))
            log.debug("Reading info about %s", app.name)
            if ent.get("buildpack", "") != "null":
                app.buildpack = ent.get("buildpack", "")
            if ent.get("detected_buildpack", "") != "null":
                app.detected_buildpack = ent.get("detected_buildpack", "")
            if ent.get("dockerimage", "") != "null":
                app.docker_image = ent.get("dockerimage", "")
            app.instances = ent.get("instances", 0)
            app.memory = ent.get("memory", 0)
            app.env = ent.get("environment_json") or {}
            app.ports = ent.get("ports") or []
            inst.applications.append(app)
            file_name += app.name
        path = os.path.join(output_path, common.normalize_for_filename(file_name) + ".yaml")
        try:
            common.write_yaml(path, inst)
        except OSError as e:
            err = common.go_path_error(e, "open")
            log.error("Unable to write collect output : %s", err)
            raise RuntimeError(err) from e


def get_all_cf_instance_buildpacks():
    try:
        out = run(["cf", "buildpacks"]).decode("utf-8", "replace")
    except Exception as e:  # noqa: BLE001
        log.warning("Error while getting buildpacks : %s", e)
        raise
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
    for ent in _cf_apps("Skipping"):
        if ent.get("buildpack"):
            bps.append(ent["buildpack"])
        if ent.get("detected_buildpack"):
            bps.append(ent["detected_buildpack"])
    return bps


def get_all_used_buildpacks(directory):
    from ..source.cfmanifest import read_application_manifest
    bps = []
    try:
        files = common.get_files_by_ext(directory, [".yml", ".yaml"])
    except (OSError, ValueError) as e:
        log.warning("Unable to fetch yaml files and recognize application manifest yamls : %s", e)
        files = []
    for path in files:
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
        try:
            os.makedirs(output_path, mode=DEFAULT_DIRECTORY_PERMISSION, exist_ok=True)
        except OSError as e:
            err = common.go_path_error(e, "mkdir")
            log.error("Unable to create output path %s : %s", output_path, err)
            raise RuntimeError(err) from e
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
        try:
            common.write_yaml(path, cz)
        except OSError as e:
            err = common.go_path_error(e, "open")
            log.error("Unable to write cf container type output %s : %s", file_name, err)
            raise RuntimeError(err) from e
        if settings.fixed and not names:
            raise RuntimeError("No buildpacks found")
