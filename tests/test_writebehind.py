"""Write-behind of output files (``ops/writebehind.py``)."""

import os

import pytest

from move2kube_amd.ops import writebehind


def test_synchronous_outside_a_scope(tmp_path):
    seen = []
    writebehind.write([(str(tmp_path / "a"), "1", 0o644)], seen.append)
    assert seen == [[None]] and (tmp_path / "a").read_text() == "1"


def test_batches_in_order_callbacks_at_drain(tmp_path):
    seen = []
    with writebehind.scope():
        for i in range(20):
            writebehind.write([(str(tmp_path / "same"), str(i), 0o644), (str(tmp_path / ("f%d" % i)), "x", 0o644)],
                              lambda errs, i=i: seen.append((i, errs)))
        writebehind.write([(str(tmp_path / "nodir" / "g"), "x", 0o644)], lambda errs: seen.append(("bad", errs)))
        writebehind.drain()
        assert [s[0] for s in seen] == list(range(20)) + ["bad"]
        assert all(errs == [None, None] for _, errs in seen[:20])
        assert isinstance(seen[-1][1][0], OSError)
        assert (tmp_path / "same").read_text() == "19"   # the last batch wins
        writebehind.write([(str(tmp_path / "late"), "y", 0o644)], lambda errs: seen.append(("late", errs)))
    assert seen[-1] == ("late", [None])                  # the scope drains on exit
    assert sorted(os.listdir(str(tmp_path))) == sorted(["same", "late"] + ["f%d" % i for i in range(20)])


def test_callback_errors_surface_on_the_submitting_thread(tmp_path):
    def boom(errs):
        raise RuntimeError("callback failed")
    with pytest.raises(RuntimeError, match="callback failed"):
        with writebehind.scope():
            writebehind.write([(str(tmp_path / "a"), "1", 0o644)], boom)


def test_disabled_by_env(tmp_path, monkeypatch):
    monkeypatch.setenv("M2K_WRITE_BEHIND", "0")
    seen = []
    with writebehind.scope():
        writebehind.write([(str(tmp_path / "a"), "1", 0o644)], seen.append)
        assert seen == [[None]]
