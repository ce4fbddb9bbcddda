"""``move2kube collect`` output kinds (reference ``types/collection/*.go``).

ClusterMetadata, ImageMetadata (ImageInfo), CfInstanceApps, CfContainerizers.
"""

from ..utils import common
from ..utils.constants import DEFAULT_STORAGE_CLASS_NAME, SCHEME_GROUP_VERSION
from .base import (GoMap, as_int, as_list, as_map, as_str, as_str_list, as_str_list_map,
                   as_str_map)

CLUSTER_METADATA_KIND = "ClusterMetadata"
IMAGE_METADATA_KIND = "ImageMetadata"
CF_INSTANCE_APPS_KIND = "CfInstanceApps"
CF_CONTAINERIZERS_KIND = "CfContainerizers"


def _typemeta(obj, d):
    if obj.api_version:
        d["apiVersion"] = obj.api_version
    d["kind"] = obj.kind
    if obj.name:
        d["metadata"] = {"name": obj.name}
    return d


def _read_typemeta(obj, d):
    obj.api_version = as_str(d.get("apiVersion"))
    obj.kind = as_str(d.get("kind"))
    obj.name = as_str(as_map(d.get("metadata")).get("name"))


class ClusterMetadataSpec:
    def __init__(self, storage_classes=None, api_kind_version_map=None, host=""):
        self.storage_classes = list(storage_classes) if storage_classes is not None else []
        self.api_kind_version_map = dict(api_kind_version_map) if api_kind_version_map is not None else {}
        self.host = host

    def to_yaml(self):
        d = {"storageClasses": list(self.storage_classes),
             "apiKindVersionMap": GoMap({k: list(v) for k, v in self.api_kind_version_map.items()})}
        if self.host:
            d["host"] = self.host
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        return cls(as_str_list(d.get("storageClasses")), as_str_list_map(d.get("apiKindVersionMap")),
                   as_str(d.get("host")))

    def copy(self):
        return ClusterMetadataSpec(list(self.storage_classes),
                                   {k: list(v) for k, v in self.api_kind_version_map.items()}, self.host)

    def merge(self, new):
        """``ClusterMetadataSpec.Merge``: intersect storage classes/kinds, take new host."""
        self.storage_classes = [sc for sc in self.storage_classes if common.is_string_present(new.storage_classes, sc)]
        m = {}
        for kind, gvs in new.api_kind_version_map.items():
            if kind in self.api_kind_version_map:
                m[kind] = gvs
        self.api_kind_version_map = m
        self.host = new.host
        return True

    def get_supported_versions(self, kind):
        gvs = self.api_kind_version_map.get(kind)
        if gvs:
            return gvs
        return None


class ClusterMetadata:
    def __init__(self, name=""):
        self.api_version = SCHEME_GROUP_VERSION
        self.kind = CLUSTER_METADATA_KIND
        self.name = name
        self.spec = ClusterMetadataSpec()

    def to_yaml(self):
        d = _typemeta(self, {})
        d["spec"] = self.spec.to_yaml()
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        c = cls()
        _read_typemeta(c, d)
        c.spec = ClusterMetadataSpec.from_yaml(d.get("spec"))
        return c

    def is_empty(self):
        return self.kind == ""

    def merge(self, new):
        """``ClusterMetadata.Merge`` (types/collection/cluster.go:46-78)."""
        if new.is_empty():
            return True
        if self.is_empty():
            self.kind = new.kind
            self.name = new.name
        elif self.kind != new.kind:
            return False
        if new.name:
            self.name = new.name
        self.spec.storage_classes = [sc for sc in self.spec.storage_classes
                                     if common.is_string_present(new.spec.storage_classes, sc)]
        if not self.spec.storage_classes:
            self.spec.storage_classes = [DEFAULT_STORAGE_CLASS_NAME]
        m = {}
        for kind, gvs in new.spec.api_kind_version_map.items():
            if kind in self.spec.api_kind_version_map:
                m[kind] = gvs
        self.spec.api_kind_version_map = m
        self.spec.host = new.spec.host
        return True


def new_cluster_metadata(context_name):
    return ClusterMetadata(context_name)


class ImageInfo:
    def __init__(self):
        self.api_version = SCHEME_GROUP_VERSION
        self.kind = IMAGE_METADATA_KIND
        self.name = ""
        self.tags = []
        self.ports = []
        self.accessed_dirs = []
        self.user_id = 0

    def go_v(self):
        """fmt ``%v`` of the Go struct: ``{{apiVersion kind} {name} {[tags] [ports] [dirs] userID}}``."""
        def lst(xs):
            return "[" + " ".join(str(x) for x in xs) + "]"
        return "{{%s %s} {%s} {%s %s %s %d}}" % (self.api_version, self.kind, self.name, lst(self.tags),
                                                 lst(self.ports), lst(self.accessed_dirs), self.user_id)

    def to_yaml(self):
        d = _typemeta(self, {})
        d["spec"] = {"tags": list(self.tags), "ports": list(self.ports),
                     "accessedDirs": list(self.accessed_dirs), "userID": self.user_id}
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        i = cls()
        _read_typemeta(i, d)
        spec = as_map(d.get("spec"))
        i.tags = as_str_list(spec.get("tags"))
        i.ports = [as_int(p) for p in as_list(spec.get("ports"))]
        i.accessed_dirs = as_str_list(spec.get("accessedDirs"))
        i.user_id = as_int(spec.get("userID"))
        return i


def _go_list(xs):
    return "[" + " ".join(str(x) for x in xs) + "]"


class CfApplication:
    def go_plus_v(self):
        """fmt ``%+v`` of the Go struct."""
        env = "map[" + " ".join("%s:%s" % (k, self.env[k]) for k in sorted(self.env)) + "]"
        return ("{Name:%s Buildpack:%s DetectedBuildpack:%s Memory:%d Instances:%d DockerImage:%s Ports:%s Env:%s}"
                % (self.name, self.buildpack, self.detected_buildpack, self.memory, self.instances, self.docker_image,
                   _go_list(self.ports), env))

    def __init__(self, name=""):
        self.name = name
        self.buildpack = ""
        self.detected_buildpack = ""
        self.memory = 0
        self.instances = 0
        self.docker_image = ""
        self.ports = []
        self.env = {}

    def to_yaml(self):
        d = {"name": self.name}
        if self.buildpack:
            d["buildpack"] = self.buildpack
        if self.detected_buildpack:
            d["detectedBuildpack"] = self.detected_buildpack
        d["memory"] = self.memory
        d["instances"] = self.instances
        if self.docker_image:
            d["dockerImage"] = self.docker_image
        d["ports"] = list(self.ports)
        if self.env:
            d["env"] = GoMap(self.env)
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        a = cls(as_str(d.get("name")))
        a.buildpack = as_str(d.get("buildpack"))
        a.detected_buildpack = as_str(d.get("detectedBuildpack"))
        a.memory = as_int(d.get("memory"))
        a.instances = as_int(d.get("instances"))
        a.docker_image = as_str(d.get("dockerImage"))
        a.ports = [as_int(p) for p in as_list(d.get("ports"))]
        a.env = as_str_map(d.get("env"))
        return a


class CfInstanceApps:
    def __init__(self):
        self.api_version = SCHEME_GROUP_VERSION
        self.kind = CF_INSTANCE_APPS_KIND
        self.name = ""
        self.applications = []

    def to_yaml(self):
        d = _typemeta(self, {})
        d["spec"] = {"applications": [a.to_yaml() for a in self.applications]}
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        c = cls()
        _read_typemeta(c, d)
        c.applications = [CfApplication.from_yaml(x) for x in as_list(as_map(d.get("spec")).get("applications"))]
        return c


class BuildpackContainerizer:
    def go_plus_v(self):
        return "{BuildpackName:%s ContainerBuildType:%s ContainerizationTargetOptions:%s}" % (
            self.buildpack_name, self.container_build_type, _go_list(self.target_options))

    def __init__(self, buildpack_name="", container_build_type="", target_options=None):
        self.buildpack_name = buildpack_name
        self.container_build_type = container_build_type
        self.target_options = list(target_options or [])

    def to_yaml(self):
        d = {"buildpackName": self.buildpack_name, "containerBuildType": self.container_build_type}
        if self.target_options:
            d["targetOptions"] = list(self.target_options)
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        return cls(as_str(d.get("buildpackName")), as_str(d.get("containerBuildType")),
                   as_str_list(d.get("targetOptions")))


class CfContainerizers:
    def __init__(self):
        self.api_version = SCHEME_GROUP_VERSION
        self.kind = CF_CONTAINERIZERS_KIND
        self.name = ""
        self.buildpack_containerizers = []

    def to_yaml(self):
        d = _typemeta(self, {})
        d["spec"] = {"buildpackContainerizers": [b.to_yaml() for b in self.buildpack_containerizers]}
        return d

    @classmethod
    def from_yaml(cls, d):
        d = as_map(d)
        c = cls()
        _read_typemeta(c, d)
        c.buildpack_containerizers = [BuildpackContainerizer.from_yaml(x) for x in
                                      as_list(as_map(d.get("spec")).get("buildpackContainerizers"))]
        return c
