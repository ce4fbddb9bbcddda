"""Property tests: the go-yaml emitter round-trips through a YAML loader, the
native and Python walkers agree, edit-distance implementations agree."""

import os
import string

from hypothesis import given, settings, strategies as st

from move2kube_amd.ops import editdistance, native
from move2kube_amd.utils import yamlio


_text = st.text(alphabet=st.characters(blacklist_categories=("Cs",), blacklist_characters="﻿\x85  "),
                max_size=20)
_scalars = st.one_of(_text, st.integers(min_value=-10**12, max_value=10**12), st.booleans(), st.none())
_values = st.recursive(_scalars, lambda ch: st.one_of(st.lists(ch, max_size=4),
                                                      st.dictionaries(_text, ch, max_size=4)), max_leaves=12)


def _norm(v):
    # YAML has no distinction between "absent" and null inside lists/maps we emit; keep types
    return v


@settings(max_examples=300, deadline=None)
@given(st.dictionaries(_text, _values, max_size=5))
def test_dump_roundtrips_through_yaml_loader(doc):
    text = yamlio.dump(doc)
    # decoded with the go-yaml v3 resolution rules (PyYAML's YAML 1.1 SafeLoader
    # also resolves e.g. "=" (the 1.1 "value" type), which go-yaml emits plain)
    back = yamlio.load(text)
    assert back == (doc or {}), text


@settings(max_examples=200, deadline=None)
@given(st.text(alphabet=string.ascii_lowercase + string.digits + "_-", max_size=30),
       st.text(alphabet=string.ascii_lowercase + string.digits + "_-", max_size=30))
def test_edit_distance_native_equals_python(a, b):
    m = native.module()
    if m is None:
        return
    assert int(m.edit_distance_batch([a], [b], 1, 1, 2, 1)[0][0]) == editdistance.wagner_fischer_py(a, b)
    assert m.wagner_fischer(a, b, 1, 1, 2) == editdistance.wagner_fischer_py(a, b)


# strings biased towards what decides libyaml scalar styles: indicators,
# whitespace/breaks, control characters, numbers, YAML 1.1 keywords
_tricky_atoms = st.sampled_from(["-", "--", "---", "...", ":", ": ", " #", "#", "?", "'", '"', "\\", "|", ">",
                                 "\n", "\r", "\t", " ", "  ", "\x00", "\x7f", "\x1b", "y", "no", "null", "~",
                                 "true", "0x1F", "1_000", "1e3", ".5", "-.inf", "12:30", "2001-12-14", "+1",
                                 "007", "<<", "é", " ", "[", "{", ",", "%", "@", "`", "&a", "*a", "!t"])
_tricky = st.lists(st.one_of(_tricky_atoms, st.text(alphabet=string.printable, max_size=4)),
                   max_size=5).map("".join)
_keys = st.one_of(_tricky, st.integers(min_value=-5, max_value=120), st.sampled_from(["b10", "b9", "b09", "a0", "A"]))
_leaf = st.one_of(_tricky, st.integers(min_value=-2**70, max_value=2**70), st.floats(allow_nan=True),
                  st.booleans(), st.none())
_tree = st.recursive(_leaf, lambda ch: st.one_of(
    st.lists(ch, max_size=4), st.lists(ch, max_size=3).map(tuple),
    st.dictionaries(_keys, ch, max_size=4),
    st.dictionaries(_keys, ch, max_size=4).map(yamlio.GoMap)), max_leaves=16)


@settings(max_examples=int(os.environ.get("M2K_PROP_EXAMPLES", "600")), deadline=None)
@given(_tree, st.booleans())
def test_native_emitter_matches_python_specification(doc, sort_maps):
    if not yamlio._native():
        return
    assert yamlio.dump(doc, sort_maps) == yamlio.dump_py(doc, sort_maps)


# -- robustness: arbitrary compose documents never crash the loaders ---------

_FUZZ_KEYS = ["image", "build", "ports", "expose", "environment", "env_file", "volumes", "deploy", "healthcheck",
              "command", "entrypoint", "labels", "networks", "secrets", "configs", "tmpfs", "restart", "user",
              "working_dir", "hostname", "domainname", "privileged", "tty", "stdin_open", "cap_add", "cap_drop",
              "dns", "extra_hosts", "logging", "mem_limit", "cpu_shares", "pid", "stop_grace_period", "devices",
              "links", "depends_on", "container_name", "ulimits", "sysctls", "security_opt", "read_only",
              "shm_size", "init"]
_FUZZ_INNER = ["target", "published", "source", "type", "mode", "resources", "limits", "memory", "cpus",
               "replicas", "test", "interval", "disable", "external", "name", "driver", "file", "read_only",
               "size", "protocol", "x-a"]
_FUZZ_SCALARS = [None, True, False, 0, 1, -5, 80, 1.5, "", "x", "80:80", "1g", "a=b", "/tmp:/x:ro",
                 "8080-8081:80-81", "udp", "10s", "${X}", "$$", "CMD-SHELL", "127.0.0.1:5000:5000/udp",
                 "${N:-3}", "${B:-yes}", "${F:-0.5}", "$", "${X:?needed}", "${X-a}b", "$1",
                 "v:/x", "a::b", "8000-8002:80", "80/xyz", "5zz", "1.2.3m", "~/x:/y", "1m30s", "5x",
                 "[::1]:80:80", "::1:80:80", "0.0.0.0:1-2:3-4/sctp", "my web"]


def _fuzz_value(rng, depth=0):
    r = rng.random()
    if depth > 2 or r < 0.5:
        return rng.choice(_FUZZ_SCALARS)
    if r < 0.75:
        return [_fuzz_value(rng, depth + 1) for _ in range(rng.randint(0, 3))]
    return {rng.choice(_FUZZ_KEYS + _FUZZ_INNER): _fuzz_value(rng, depth + 1) for _ in range(rng.randint(0, 4))}


def test_compose_loaders_never_crash(tmp_path):
    """Randomly typed compose documents either load or fail with ComposeError
    (the reference's loaders reject them through the compose JSON schema)."""
    import random
    from move2kube_amd.models import plan as plantypes
    from move2kube_amd.source.compose import v1v2, v3
    rng = random.Random(1234)
    p = str(tmp_path / "docker-compose.yaml")
    plan = plantypes.new_plan()
    plan.root_dir = str(tmp_path)
    loaded = 0
    for _ in range(400):
        svc = {rng.choice(_FUZZ_KEYS): _fuzz_value(rng) for _ in range(rng.randint(1, 6))}
        doc = {"version": rng.choice(["3", "3.7", "2", "2.1"]), "services": {"s": svc}}
        for key in ("volumes", "networks", "secrets"):
            if rng.random() < 0.3:
                doc[key] = {"k": _fuzz_value(rng)}
        with open(p, "w") as f:
            f.write(yamlio.dump(doc))
        for loader in (v3.V3Loader, v1v2.V1V2Loader):
            try:
                loader().convert_to_ir(p, plan, plantypes.Service("s", plantypes.COMPOSE2KUBE))
                loaded += 1
            except v3.ComposeError:
                pass
    assert loaded > 0


_K8S_KINDS = [("apps/v1", "Deployment"), ("v1", "Service"), ("networking.k8s.io/v1", "Ingress"),
              ("extensions/v1beta1", "Ingress"), ("v1", "Pod"), ("apps/v1", "StatefulSet"), ("apps/v1", "DaemonSet"),
              ("batch/v1", "Job"), ("v1", "ConfigMap"), ("v1", "Secret"), ("v1", "PersistentVolumeClaim"),
              ("serving.knative.dev/v1", "Service"), ("route.openshift.io/v1", "Route"),
              ("apps.openshift.io/v1", "DeploymentConfig"), ("networking.k8s.io/v1", "NetworkPolicy")]
_K8S_KEYS = ["spec", "template", "containers", "ports", "containerPort", "port", "targetPort", "name", "image",
             "replicas", "selector", "matchLabels", "rules", "http", "paths", "path", "backend", "serviceName",
             "servicePort", "service", "number", "volumes", "volumeMounts", "env", "value", "resources", "data",
             "type", "host", "to", "kind", "tls", "hosts", "labels", "clusterIP", "protocol", "accessModes"]
_K8S_SCALARS = [None, True, False, 0, 80, "80", "x", "http", "/", 1.5, "", "TCP", "ClusterIP", "1Gi"]


def test_translate_never_crashes_on_arbitrary_manifests(tmp_path, monkeypatch):
    """Randomly shaped Kubernetes/Knative/OpenShift manifests: translate either
    completes or stops with the reference's fatal "nothing to containerize";
    objects that do not fit their Go types are skipped at decode time."""
    import random
    from move2kube_amd import api
    from move2kube_amd.utils import log
    monkeypatch.setenv("M2K_NO_NETWORK", "1")
    monkeypatch.setenv("M2K_DISABLE_CNB", "1")
    rng = random.Random(99)

    def val(d=0):
        r = rng.random()
        if d > 5 or r < 0.3:
            return rng.choice(_K8S_SCALARS)
        if r < 0.55:
            return [val(d + 1) for _ in range(rng.randint(0, 2))]
        return {rng.choice(_K8S_KEYS): val(d + 1) for _ in range(rng.randint(1, 4))}

    done = 0
    for it in range(40):
        src = tmp_path / ("src%d" % it)
        src.mkdir()
        for i in range(rng.randint(1, 3)):
            gv, kind = rng.choice(_K8S_KINDS)
            obj = {"apiVersion": gv, "kind": kind, "metadata": {"name": rng.choice("abc")}}
            for _ in range(rng.randint(1, 3)):
                obj[rng.choice(["spec", "data", "status"])] = val()
            (src / ("o%d.yaml" % i)).write_text(yamlio.dump(obj))
        try:
            api.translate(str(src), str(tmp_path / ("out%d" % it)))
            done += 1
        except log.FatalError as e:
            assert "No containerization technique was selected" in str(e), str(e)
    assert done > 0


_qa_atoms = st.sampled_from(["a", "b c", "", " lead", "trail ", "x:y", "- d", "#h", "'q'", '"dq"', "\\", "é", "中", "1",
                             "1.5", "true", "null", "~", "yes", "0x1f", "a\nb", "*a", "&b", "!t", "%p", "@", "`", "{}",
                             "[]", "a, b", "?", "--- x", "...", "<<", " x", "\x85", "\x7f", "\x01"])
_qa_text = st.lists(_qa_atoms, min_size=1, max_size=3).map("".join)


@settings(max_examples=int(os.environ.get("M2K_PROP_EXAMPLES", "300")), deadline=None)
@given(st.lists(st.tuples(_qa_text, _qa_text, _qa_text), min_size=1, max_size=4))
def test_qa_cache_answers_survive_a_write_and_read(tmp_path_factory, answers):
    """A QA cache written by this emitter reads back with the same
    descriptions, contexts and answers (go-yaml's emitter and reader agree on
    these strings: NEL double-quoted, LS kept raw with the indentation after)."""
    from move2kube_amd.models import qa
    path = str(tmp_path_factory.mktemp("qa") / "cache.yaml")
    c = qa.Cache(path)
    seen = set()
    for desc, ctx, ans in answers:
        if desc in seen:
            continue
        try:
            p = qa.new_input_problem(desc, [ctx], "d")
            p.set_answer([ans])
        except qa.ProblemError:   # not a problem the engine would accept
            continue
        seen.add(desc)
        c.add_problem_solution(p)
    if not seen:
        return
    c.write()
    back = qa.Cache(path)
    back.load()
    assert [p.to_yaml() for p in back.problems] == [p.to_yaml() for p in c.problems]
