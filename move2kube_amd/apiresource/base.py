"""API resource framework (reference ``internal/apiresource/apiresource.go``).

A handler knows a set of kinds, creates new objects from the IR and converts
objects (new or cached from input YAMLs) into kinds the target cluster
supports.  :class:`APIResource` wraps a handler with the cluster context and
de-duplicates by namespace+name+GroupKind (a later object replaces an earlier
one, the reference's ``DeepCopyInto`` merge).

Objects are JSON-shaped dicts.  ``__gotype`` records the Go type an object was
created as when it differs from its ``apiVersion`` (the reference builds some
objects with placeholder TypeMeta and relies on the Go type); it is stripped
before marshalling.
"""

from ..utils import common, log
from ..utils.constants import GROUP_NAME

SELECTOR = GROUP_NAME + "/service"
GOTYPE = "__gotype"


def gotype(obj):
    return obj.get(GOTYPE) or "%s.%s" % (obj.get("apiVersion", ""), obj.get("kind", ""))


def is_type(obj, gv, kind):
    return gotype(obj) == "%s.%s" % (gv, kind)


def kind_of(obj):
    return obj.get("kind", "")


def object_meta_copy(m):
    out = {}
    for k, v in (m or {}).items():
        out[k] = dict(v) if isinstance(v, dict) else (list(v) if isinstance(v, list) else v)
    return out


def get_service_labels(name):
    return {SELECTOR: name}


def get_annotations(service):
    return dict(service.annotations or {})


def get_pod_labels(name, networks):
    from .others import get_network_policy_labels
    return common.merge_string_maps(get_service_labels(name), get_network_policy_labels(networks))


class IAPIResource:
    def get_supported_kinds(self):
        return []

    def create_new_resources(self, ir, supported_kinds):
        return []

    def convert_to_cluster_supported_kinds(self, obj, supported_kinds, other_objs, ir):
        """Return (objs, ok)."""
        return None, False


class APIResource:
    def __init__(self, handler, cluster=None):
        self.handler = handler
        self.cluster = cluster
        self.cached = None
        self._index = None  # resource key -> position in cached (first occurrence)

    def set_cluster_context(self, cluster):
        self.cluster = cluster

    def get_cluster_supported_kinds(self):
        kinds = []
        for k in self.handler.get_supported_kinds():
            if self.cluster is not None and self.cluster.get_supported_versions(k) is not None:
                kinds.append(k)
        return kinds

    def _is_supported_kind(self, obj):
        return common.is_string_present(self.handler.get_supported_kinds(), kind_of(obj))

    def load_resources(self, objs, ir):
        ignored = []
        for obj in objs:
            if obj is None:
                continue
            if not self._load(obj, objs, ir):
                ignored.append(obj)
        return ignored

    def get_updated_resources(self, ir):
        objs = self.handler.create_new_resources(ir, self.get_cluster_supported_kinds()) or []
        for obj in objs:
            if not self._load(obj, objs, ir):
                log.error("Object created seems to be of an incompatible type : %r", obj.get("kind"))
        return self.cached or []

    def _load(self, obj, others, ir):
        if not self._is_supported_kind(obj):
            return False
        sup, ok = self.handler.convert_to_cluster_supported_kinds(obj, self.get_cluster_supported_kinds(), others, ir)
        if not ok:
            return False
        if self.cached is None:
            self.cached = list(sup)
            self._index = {}
            for i, c in enumerate(self.cached):
                k = _resource_key(c)
                if k is not None:
                    self._index.setdefault(k, i)
            return True
        # merge: an object replaces the first cached one with the same
        # namespace+name and group/kind (apiresource.go:86-101), else appends
        for s in sup:
            k = _resource_key(s)
            i = self._index.get(k) if k is not None else None
            if i is not None:
                self.cached[i] = s
            else:
                if k is not None:
                    self._index[k] = len(self.cached)
                self.cached.append(s)
        return True


def _object_id(obj):
    md = obj.get("metadata") or {}
    return (md.get("namespace") or "") + (md.get("name") or "")


def _group_kind(obj):
    gv = obj.get("apiVersion", "")
    group = gv.split("/", 1)[0] if "/" in gv else ""
    return group, obj.get("kind", "")


def _resource_key(obj):
    """``isSameResource`` (apiresource.go): namespace + name and group/kind, or
    None for an object without a name (such an object never matches another)."""
    oid = _object_id(obj)
    return None if oid == "" else (oid, _group_kind(obj))

