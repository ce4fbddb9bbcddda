"""The plan of a one-shot ``translate`` hands its directory listings and
detector results to the translate of the same command (one walk per
command), only when the output directory lies outside the source tree."""

import os
import shutil

from move2kube_amd import api
from move2kube_amd.utils import fsindex

SAMPLES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "samples")  # the reference's corpus, byte for byte


def test_handoff_allowed():
    assert fsindex.handoff_allowed("/w/src", "/w/out/proj")
    assert fsindex.handoff_allowed("/w/src", "/w/src2/proj")
    assert not fsindex.handoff_allowed("/w/src", "/w/src/proj")
    assert not fsindex.handoff_allowed("/w/src", "/w/src")
    assert not fsindex.handoff_allowed("/w/src/", "/w/src/out/p")


def test_kept_listing_is_adopted_once_and_only_for_its_root(tmp_path):
    (tmp_path / "a").mkdir()
    with fsindex.scope(keep_for=str(tmp_path)):
        first = fsindex.get_index(str(tmp_path))
    with fsindex.scope(adopt="/elsewhere"):
        assert fsindex.get_index(str(tmp_path)) is not first   # other root: fresh listing, kept one dropped
    with fsindex.scope(keep_for=str(tmp_path)):
        first = fsindex.get_index(str(tmp_path))
    with fsindex.scope(adopt=str(tmp_path)):
        assert fsindex.get_index(str(tmp_path)) is first
    with fsindex.scope(adopt=str(tmp_path)):
        assert fsindex.get_index(str(tmp_path)) is not first   # single use


def _tree(root):
    out = {}
    for dp, _dn, fns in os.walk(root):
        for fn in fns:
            p = os.path.join(dp, fn)
            with open(p, "rb") as f:
                out[os.path.relpath(p, root)] = f.read()
    return out


def _walks(monkeypatch):
    n = []
    real = fsindex.walk

    def counting(root):
        n.append(root)
        return real(root)
    monkeypatch.setattr(fsindex, "walk", counting)
    return n


def test_same_output_with_and_without_handoff(tmp_path, monkeypatch):
    src = tmp_path / "samples"
    shutil.copytree(SAMPLES, str(src), symlinks=True)
    walks = _walks(monkeypatch)
    with api.Session(qaskip=True) as s:
        a = s.translate(str(src), str(tmp_path / "o1"))
    with_handoff = [w for w in walks if w == str(src)]
    monkeypatch.setattr(fsindex, "handoff_allowed", lambda *_: False)
    del walks[:]
    with api.Session(qaskip=True) as s:
        b = s.translate(str(src), str(tmp_path / "o2"))
    without = [w for w in walks if w == str(src)]
    assert len(with_handoff) == 1 and len(without) == 2
    assert _tree(a) == _tree(b)


def test_output_inside_source_walks_again(tmp_path, monkeypatch):
    src = tmp_path / "app"
    shutil.copytree(os.path.join(SAMPLES, "nodejs"), str(src))
    walks = _walks(monkeypatch)
    with api.Session(qaskip=True) as s:
        s.translate(str(src), str(src))
    assert len([w for w in walks if w == str(src)]) == 2


def test_compose_files_parsed_once_per_command(tmp_path, monkeypatch):
    """The planner and the translator of one command share each compose
    file's parse (``source/compose/utils.py:command_memo``)."""
    from move2kube_amd.source.compose import v3
    src = tmp_path / "dc"
    shutil.copytree(os.path.join(SAMPLES, "docker-compose"), str(src))
    calls = []
    real = v3.parse_v3.__wrapped__

    def counting(path):
        calls.append(path)
        return real(path)
    monkeypatch.setattr(v3, "parse_v3", v3.cu.command_memo("compose-v3", v3.ComposeError, "%s %s")(counting))
    with api.Session(qaskip=True) as s:
        s.translate(str(src), str(tmp_path / "out"))
    compose_files = [c for c in calls if c.endswith("docker-compose.yaml") or c.endswith("docker-compose.yml")]
    assert compose_files and len(compose_files) == len(set(compose_files))
