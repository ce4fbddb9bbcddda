"""The hand-written action lexer (``gotemplate._scan_token``) returns what the
token regex (``gotemplate._TOKEN_RE``) matches, at every position of every
template asset and of generated inputs."""

import glob
import os

from hypothesis import given, settings, strategies as st

from move2kube_amd.utils import gotemplate

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _regex(src, pos):
    m = gotemplate._TOKEN_RE.match(src, pos)
    return None if m is None else (m.lastgroup, m.end())


def _check_all_positions(src):
    for pos in range(len(src)):
        assert gotemplate._scan_token(src, pos) == _regex(src, pos), (src, pos)


def test_every_position_of_the_template_assets():
    files = sorted(glob.glob(os.path.join(ROOT, "move2kube_amd", "assets", "templates", "*")))
    assert files
    for f in files:
        with open(f) as fh:
            _check_all_positions(fh.read())


_PIECES = st.sampled_from(["0x1F", "0b", "0o7", "0x", "1_0", "1.", ".5", "1.5e-3", "2e", "3i", "-", "+", "+.5", "-1", "e5",
                           "\"a\\\"b\"", "\"", "'c'", "''", "'\\", "`raw`", "`", "/*c*/", "/*", "/", ":=", ":", "=", "|",
                           "(", ")", ",", "$", "$x", "$x.Y", ".", ".A.b_1", "..", ".1", "abc", "_x", " ", "\t\n", "é", "١",
                           " ", "\\", "*", "x0"])


@settings(max_examples=1500, deadline=None)
@given(st.lists(_PIECES, min_size=1, max_size=6).map("".join))
def test_generated_inputs(src):
    _check_all_positions(src)


@settings(max_examples=500, deadline=None)
@given(st.text(alphabet="0123456789._eEixXbBoOaf+-", min_size=1, max_size=10))
def test_numbers(src):
    _check_all_positions(src)
