"""Go types of the move2kube documents, for go-yaml v3's typed-decode errors.

``yaml.Unmarshal(data, &plan)`` (``ReadMove2KubeYaml``,
``internal/common/utils.go:246``) does not stop at the first field of the
wrong shape: ``decoder.terror`` records ``line N: cannot unmarshal <tag>
[`value`] into <Go type>`` and decoding goes on, and the error is
``yaml: unmarshal errors:`` followed by every such line.  The typed decoders
in this package (``models/base.py``) work on plain loaded data and stop at the
first problem; when they do, :func:`unmarshal_errors` walks the composed YAML
nodes against the Go type of the document (declared here from
``types/plan/plan.go``, ``types/qaengine/{cache,problem}.go`` and
``types/collection/*.go``) and rebuilds go-yaml's text.

The walk follows ``gopkg.in/yaml.v3`` ``decode.go`` (``unmarshal``,
``scalar``, ``sequence``, ``mapping``, ``mappingStruct``, ``terror``) and
``resolve.go`` (which scalars are ints, floats, bools, nulls).  No Go
toolchain is here, so the texts are pinned by those sources only.
"""

import math

from ..utils import yamlio

_INT_RANGES = {"int": 64, "int64": 64, "int32": 32, "int16": 16, "int8": 8}


class GoType:
    __slots__ = ("kind", "name", "elem", "key", "fields")

    def __init__(self, kind, name, elem=None, key=None, fields=None):
        self.kind, self.name, self.elem, self.key, self.fields = kind, name, elem, key, fields


def string(name="string"):
    return GoType("string", name)


def boolean():
    return GoType("bool", "bool")


def integer(name="int"):
    return GoType("int", name)


def slice_of(elem):
    return GoType("slice", "[]" + elem.name, elem=elem)


def map_of(key, elem):
    return GoType("map", "map[%s]%s" % (key.name, elem.name), elem=elem, key=key)


def struct(name, fields):
    """``fields``: yaml key -> GoType (inline structs already flattened)."""
    return GoType("struct", name, fields=fields)


ANY = GoType("any", "interface {}")

# types/types.go: TypeMeta (inline) and ObjectMeta (``metadata``)
OBJECT_META = struct("types.ObjectMeta", {"name": string()})


def _document(name, spec):
    return struct(name, {"apiVersion": string(), "kind": string(), "metadata": OBJECT_META, "spec": spec})


# types/plan/plan.go
_STR_LIST = slice_of(string())
REPO_INFO = struct("plan.RepoInfo", {"gitRepoDir": string(), "gitRepoURL": string(), "gitRepoBranch": string(),
                                     "targetPath": string()})
SERVICE = struct("plan.Service", {
    "serviceName": string(),
    "serviceRelPath": string(),
    "image": string(),
    "translationType": string("plan.TranslationTypeValue"),
    "containerBuildType": string("plan.ContainerBuildTypeValue"),
    "sourceType": slice_of(string("plan.SourceTypeValue")),
    "targetOptions": _STR_LIST,
    "sourceArtifacts": map_of(string("plan.SourceArtifactTypeValue"), _STR_LIST),
    "buildArtifacts": map_of(string("plan.BuildArtifactTypeValue"), _STR_LIST),
    "updateContainerBuildPipeline": boolean(),
    "updateDeployPipeline": boolean(),
    "repoInfo": REPO_INFO,
})
PLAN = _document("plan.Plan", struct("plan.PlanSpec", {
    "inputs": struct("plan.Inputs", {
        "rootDir": string(),
        "kubernetesYamls": _STR_LIST,
        "qaCaches": _STR_LIST,
        "services": map_of(string(), slice_of(SERVICE)),
        "targetInfoArtifacts": map_of(string("plan.TargetInfoArtifactTypeValue"), _STR_LIST),
    }),
    "outputs": struct("plan.Outputs", {
        "kubernetes": struct("plan.KubernetesOutput", {
            "registryURL": string(),
            "registryNamespace": string(),
            "artifactType": string("plan.TargetArtifactTypeValue"),
            "targetCluster": struct("plan.TargetClusterType", {"type": string(), "path": string()}),
            "ignoreUnsupportedKinds": boolean(),
        }),
    }),
}))

# types/qaengine/cache.go, problem.go
QA_CACHE = _document("qaengine.Cache", struct("qaengine.CacheSpec", {
    "solutions": slice_of(struct("qaengine.Problem", {
        "description": string(),
        "context": _STR_LIST,
        "solution": struct("qaengine.SolutionForm", {
            "type": string("qaengine.SolutionFormType"),
            "default": _STR_LIST,
            "options": _STR_LIST,
            "answer": _STR_LIST,
        }),
        "resolved": boolean(),
    })),
}))

# types/collection/*.go
CLUSTER_METADATA = _document("collection.ClusterMetadata", struct("collection.ClusterMetadataSpec", {
    "storageClasses": _STR_LIST,
    "apiKindVersionMap": map_of(string(), _STR_LIST),
    "host": string(),
}))
IMAGE_INFO = _document("collection.ImageInfo", struct("collection.ImageInfoSpec", {
    "tags": _STR_LIST,
    "ports": slice_of(integer()),
    "accessedDirs": _STR_LIST,
    "userID": integer(),
}))
CF_INSTANCE_APPS = _document("collection.CfInstanceApps", struct("collection.CfInstanceAppsSpec", {
    "applications": slice_of(struct("collection.CfApplication", {
        "name": string(),
        "buildpack": string(),
        "detectedBuildpack": string(),
        "memory": integer("int64"),
        "instances": integer(),
        "dockerImage": string(),
        "ports": slice_of(integer("int32")),
        "env": map_of(string(), string()),
    })),
}))
CF_CONTAINERIZERS = _document("collection.CfContainerizers", struct("collection.CfContainerizersSpec", {
    "buildpackContainerizers": slice_of(struct("collection.BuildpackContainerizer", {
        "buildpackName": string(),
        "containerBuildType": string("plan.ContainerBuildTypeValue"),
        "targetOptions": _STR_LIST,
    })),
}))


# ---------------------------------------------------------------------------
# the walk
# ---------------------------------------------------------------------------

def _short_tag(tag):
    if tag.startswith("tag:yaml.org,2002:"):
        return "!!" + tag[len("tag:yaml.org,2002:"):]
    return tag


def _resolve(node):
    """(short tag, value) of a scalar as resolve.go sees it: an explicit tag
    is kept, a quoted or block scalar is a string, a plain one resolves to
    null, bool (only true/false), int, float or string."""
    explicit = getattr(node, "_m2k_tag", None)
    text = node.value
    if explicit is None:
        if node.style not in (None, ""):
            return "!!str", text
        if text in ("", "~", "null", "Null", "NULL"):
            return "!!null", None
        if text in ("true", "True", "TRUE"):
            return "!!bool", True
        if text in ("false", "False", "FALSE"):
            return "!!bool", False
        v = yamlio.go_resolve_number(text)
        if isinstance(v, str):
            return "!!str", text
        return ("!!int" if isinstance(v, int) else "!!float"), v
    short = _short_tag(node.tag)
    if short == "!!null":
        return short, None
    if short == "!!bool":
        return short, text in ("true", "True", "TRUE")
    if short in ("!!int", "!!float"):
        return short, yamlio.go_resolve_number(text)
    return short, text


class _Walk:
    def __init__(self):
        self.errors = []

    def terror(self, node, tag, t):
        import yaml
        value = ""
        if tag not in ("!!seq", "!!map"):
            v = node.value if isinstance(node, yaml.ScalarNode) else ""
            value = " `" + (v[:7] + "..." if len(v) > 10 else v) + "`"
        self.errors.append("line %d: cannot unmarshal %s%s into %s" % (node.start_mark.line + 1, tag, value, t.name))

    def unmarshal(self, node, t):
        import yaml
        if t.kind == "any":
            return
        if isinstance(node, yaml.ScalarNode):
            self.scalar(node, t)
        elif isinstance(node, yaml.SequenceNode):
            if t.kind != "slice":
                self.terror(node, "!!seq", t)
                return
            for item in node.value:
                self.unmarshal(item, t.elem)
        elif isinstance(node, yaml.MappingNode):
            if t.kind == "struct":
                for k, v in node.value:
                    if k.tag == "tag:yaml.org,2002:merge" or (isinstance(k, yaml.ScalarNode) and k.value == "<<"
                                                               and k.style is None):
                        self.unmarshal(v, t)   # merged mappings decode into the same struct
                        continue
                    if not isinstance(k, yaml.ScalarNode):
                        self.unmarshal(k, string())
                        continue
                    field = t.fields.get(k.value)
                    if field is not None:
                        self.unmarshal(v, field)
            elif t.kind == "map":
                for k, v in node.value:
                    self.unmarshal(k, t.key)
                    self.unmarshal(v, t.elem)
            else:
                self.terror(node, "!!map", t)

    def scalar(self, node, t):
        tag, value = _resolve(node)
        if tag == "!!null":
            return                   # the zero value
        if t.kind == "string":
            return                   # any scalar's text
        if t.kind == "bool":
            if isinstance(value, bool):
                return
            if isinstance(value, str) and value in ("y", "Y", "yes", "Yes", "YES", "on", "On", "ON",
                                            "n", "N", "no", "No", "NO", "off", "Off", "OFF"):
                return               # YAML 1.1 bools into a typed bool
        elif t.kind == "int" and not isinstance(value, bool):
            bits = _INT_RANGES.get(t.name, 64)
            lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
            if isinstance(value, int) and lo <= value <= hi:
                return
            if isinstance(value, float) and not math.isnan(value) and value <= 2 ** 63 - 1 and \
                    lo <= int(value) <= hi:
                return               # float64 truncated into an int field
        self.terror(node, tag, t)


def unmarshal_errors(text, t):
    """go-yaml v3's ``line N: ...`` type errors of decoding ``text`` into
    ``t`` (empty when it decodes)."""
    import yaml
    try:
        node = yaml.compose(text, Loader=getattr(yaml, "CSafeLoader", yaml.SafeLoader))
    except yaml.YAMLError:
        return []
    if node is None:
        return []
    _mark_explicit(node, text)
    w = _Walk()
    w.unmarshal(node, t)
    return w.errors


def _mark_explicit(root, text):
    """Flag scalars written with an explicit tag (the composer gives every
    plain scalar its resolved tag, so the tag is read back from the source:
    a node's start mark is at its properties, an anchor before a tag)."""
    import yaml
    stack, seen = [root], set()
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if isinstance(n, yaml.ScalarNode):
            i = n.start_mark.index
            if text.startswith("&", i):
                while i < len(text) and text[i] not in " \t\r\n":
                    i += 1
                while i < len(text) and text[i] in " \t\r\n":
                    i += 1
            if text.startswith("!", i):
                n._m2k_tag = n.tag
        elif isinstance(n, yaml.SequenceNode):
            stack.extend(n.value)
        elif isinstance(n, yaml.MappingNode):
            for k, v in n.value:
                stack.append(k)
                stack.append(v)


def error_text(text, t):
    """``yaml: unmarshal errors:`` text for ``text`` decoded into ``t``, or
    None when go-yaml would decode it."""
    errs = unmarshal_errors(text, t)
    if not errs:
        return None
    return "yaml: unmarshal errors:\n  " + "\n  ".join(errs)

