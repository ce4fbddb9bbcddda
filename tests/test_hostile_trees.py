"""Source trees with special files and undecodable YAML: the planner and the
translator skip what they cannot read instead of hanging or dropping a whole
translator (crashes and hangs are fixed)."""

import os
import shutil
import threading

import pytest

from move2kube_amd import api
from move2kube_amd.utils import common

SAMPLES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "samples")  # the reference's corpus, byte for byte


def _bounded(fn, seconds=20):
    out = {}

    def run():
        try:
            out["value"] = fn()
        except BaseException as e:  # noqa: BLE001
            out["error"] = e
    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(seconds)
    assert not t.is_alive(), "hung"
    if "error" in out:
        raise out["error"]
    return out.get("value")


def test_read_bytes_rejects_a_fifo_without_blocking(tmp_path):
    fifo = tmp_path / "x.yaml"
    os.mkfifo(str(fifo))
    with pytest.raises(OSError):
        _bounded(lambda: common.read_bytes(str(fifo)), 5)
    (tmp_path / "ok.yaml").write_bytes(b"a: 1\n")
    assert common.read_bytes(str(tmp_path / "ok.yaml")) == b"a: 1\n"


def _tree(tmp_path, name):
    src = tmp_path / name
    shutil.copytree(os.path.join(SAMPLES, "nodejs"), str(src / "app"))
    shutil.copytree(os.path.join(SAMPLES, "docker-compose"), str(src / "dc"))
    (src / "app" / "requirements.txt").write_text("flask\n")  # the python detectors then read *.py files
    return src


def test_translate_a_tree_with_fifos_and_bad_utf8(tmp_path):
    """Same services as the clean tree; FIFOs named like YAML, Dockerfiles and
    Python files, a Latin-1 compose file and binary junk are skipped."""
    clean = _tree(tmp_path / "a", "src")   # same root name: it names a service
    src = _tree(tmp_path / "b", "src")
    for name in ("app/pipe.yaml", "app/Dockerfile.fifo", "app/main.py", "dc/fifo.yml"):
        os.mkfifo(str(src / name))
    (src / "latin1.yml").write_bytes(b'version: "3"\nservices:\n  web:\n    image: "caf\xe9:1"\n')
    (src / "junk.yaml").write_bytes(bytes(range(256)) * 4)
    with api.Session(qaskip=True) as s:
        want = s.translate(str(clean), str(tmp_path / "out-clean"))
        got = _bounded(lambda: s.translate(str(src), str(tmp_path / "out")), 60)
    assert sorted(os.listdir(os.path.join(got, "myproject"))) == sorted(os.listdir(os.path.join(want, "myproject")))
    with open(os.path.join(got, "docker-compose.yaml")) as a, open(os.path.join(want, "docker-compose.yaml")) as b:
        assert a.read() == b.read()


def test_a_deeply_nested_yaml_only_loses_itself(tmp_path):
    """A document nested deeper than the recursive walks allow is skipped as a
    file; the other manifests of every translator are still planned."""
    src = tmp_path / "src"
    src.mkdir()
    deep = "".join("  " * (i + 1) + "k%d:\n" % i for i in range(1500)) + "  " * 1501 + "v\n"
    (src / "crd.yaml").write_text("apiVersion: example.com/v1\nkind: Widget\nmetadata:\n  name: w\nspec:\n" + deep)
    (src / "compose.yml").write_text("version: '3'\nservices:\n  deep:\n    image: x\n    labels:\n" + deep)
    (src / "dep.yaml").write_text(
        "apiVersion: apps/v1\nkind: Deployment\nmetadata:\n  name: web\nspec:\n  selector:\n    matchLabels:\n"
        "      app: web\n  template:\n    metadata:\n      labels:\n        app: web\n    spec:\n      containers:\n"
        "      - name: web\n        image: nginx:1.19\n")
    with api.Session(qaskip=True) as s:
        out = _bounded(lambda: s.translate(str(src), str(tmp_path / "out")), 120)
    assert "web-deployment.yaml" in os.listdir(os.path.join(out, "myproject"))


def test_translate_a_tree_with_non_utf8_file_names(tmp_path):
    """A file or directory name that is not UTF-8 does not fail the walk: the
    services of the tree are still planned and translated."""
    clean = _tree(tmp_path / "a", "src")
    src = _tree(tmp_path / "b", "src")
    bsrc = os.fsencode(str(src))
    os.makedirs(os.path.join(bsrc, b"caf\xe9"))
    with open(os.path.join(bsrc, b"caf\xe9", b"notes\xff.txt"), "wb") as f:
        f.write(b"x\n")
    with api.Session(qaskip=True) as s:
        want = s.translate(str(clean), str(tmp_path / "out-clean"))
        got = _bounded(lambda: s.translate(str(src), str(tmp_path / "out")), 60)
    assert sorted(os.listdir(os.path.join(got, "myproject"))) == sorted(os.listdir(os.path.join(want, "myproject")))


def _laughs(levels=10, width=9):
    lines = ['a0: &a0 [%s]' % ",".join(['"x"'] * width)]
    for i in range(1, levels):
        lines.append("a%d: &a%d [%s]" % (i, i, ",".join(["*a%d" % (i - 1)] * width)))
    return "\n".join("  " + ln for ln in lines) + "\n"


def test_yaml_alias_expansion_is_refused_like_go_yaml():
    """go-yaml v3 fails "document contains excessive aliasing" and "anchor
    value contains itself"; the loaded tree would otherwise be expanded by
    every later walk (9**10 nodes here)."""
    from move2kube_amd.utils import yamlio
    with pytest.raises(yamlio._lz().yaml.YAMLError, match="excessive aliasing"):
        _bounded(lambda: yamlio.load("data:\n" + _laughs()), 10)
    with pytest.raises(yamlio._lz().yaml.YAMLError, match="contains itself"):
        yamlio.load("a: &a [1, *a]\n")
    legit = "a: &a {" + ", ".join("k%d: v" % i for i in range(30)) + "}\nl:\n" + "- *a\n" * 50
    assert len(yamlio.load(legit)["l"]) == 50 and yamlio.load("b: &b {x: 1}\nm:\n  <<: *b\n  y: 2\n")["m"] == {
        "x": 1, "y": 2}


def test_a_yaml_bomb_only_loses_itself(tmp_path):
    src = tmp_path / "src"
    src.mkdir()
    (src / "bomb.yaml").write_text("apiVersion: v1\nkind: ConfigMap\nmetadata:\n  name: b\ndata:\n" + _laughs())
    (src / "compose.yml").write_text("version: '3'\nx-b:\n" + _laughs() + "services:\n  web:\n    image: nginx\n")
    (src / "dep.yaml").write_text(
        "apiVersion: apps/v1\nkind: Deployment\nmetadata:\n  name: web\nspec:\n  selector:\n    matchLabels:\n"
        "      app: web\n  template:\n    metadata:\n      labels:\n        app: web\n    spec:\n      containers:\n"
        "      - name: web\n        image: nginx:1.19\n")
    with api.Session(qaskip=True) as s:
        out = _bounded(lambda: s.translate(str(src), str(tmp_path / "out")), 60)
    assert "web-deployment.yaml" in os.listdir(os.path.join(out, "myproject"))


def test_compose_service_in_a_non_utf8_directory(tmp_path):
    """A compose file under a directory whose name is not UTF-8: the volume
    hash is taken over the name's bytes, as Go hashes its string, instead of
    failing the whole compose translation on the undecodable byte."""
    bsrc = os.fsencode(str(tmp_path / "src"))
    d = os.path.join(bsrc, b"caf\xe9")
    os.makedirs(os.path.join(d, b"data"))
    with open(os.path.join(d, b"docker-compose.yaml"), "wb") as f:
        f.write(b'version: "3"\nservices:\n  web:\n    image: nginx\n    volumes:\n      - ./data:/data\n'
                b'    ports:\n      - "80:80"\n')
    with api.Session(qaskip=True) as s:
        out = _bounded(lambda: s.translate(str(tmp_path / "src"), str(tmp_path / "out")), 60)
    assert sorted(os.listdir(os.path.join(out, "myproject"))) == ["web-deployment.yaml", "web-ingress.yaml",
                                                                  "web-service.yaml"]
    assert common.fnv64a(os.fsdecode(b"caf\xe9")) == common.fnv64a(b"caf\xe9")
    assert common.normalize_for_filename(os.fsdecode(b"\xff")) == "--" + format(common.crc64_ecma(b"\xff"), "x")
