"""Compose v1/v2 interpolation as the reference's libcompose (57bd716502dc,
``config/interpolation.go``) does it, reached through ``ParseV2``
(``internal/source/compose/v1v2.go:93-129``): a hand-written scanner with no
``?`` forms, defaults that land in a package-level map and so outlive the
value (and the file) that set them, leading ``:``/``-`` of a default
skipped, an empty OS variable read as unset, the error naming the service
field.  ``ParseV2`` runs at logrus FatalLevel, so none of this is logged."""

import pytest

from move2kube_amd.source.compose import v1v2
from move2kube_amd.source.compose.interpolate import InterpolationError, interpolate_v1v2
from move2kube_amd.utils import fsindex, log

ENV = {"A": "a", "E": ""}


def _run(value, defaults=None, env=ENV, key="image"):
    d = {} if defaults is None else defaults
    out = interpolate_v1v2({"web": {key: value}}, env.get, d)
    return out["web"][key]


@pytest.mark.parametrize("value,want", [
    ("plain", "plain"),
    ("$$A", "$A"),
    ("$A-x", "a-x"),
    ("${A}${A}", "aa"),
    ("${UNSET:-d} ${UNSET-d}", "d d"),
    ("${E-d}", "d"),                                 # "-" also covers an empty value
    ("${A:-d}", "a"),
    ("${UNSET:--1}", "1"),                           # leading ":" and "-" of a default are skipped
    ("${UNSET-:x}", "x"),
    ("${1A}", ""),                                   # digits may start a braced name
    ("${UNSET:-a b}", "a b"),
    (["$A", {"k": "${A}"}], ["a", {"k": "a"}]),
    (5, 5),
])
def test_values(value, want):
    assert _run(value) == want


def test_defaults_outlive_the_value_that_set_them():
    d = {}
    assert _run(["${X:-first}", "$X", "${X}"], d) == ["first", "first", "first"]
    assert _run("$X", d) == "first"                  # a later value, or a later file
    assert _run("${X-second} $X", d) == "second second"
    assert _run("$E", {"E": "dflt"}) == "dflt"       # set but empty: the default too


@pytest.mark.parametrize("value", ["cost 5$", "$1", "${}", "${A:x}", "${A?x}", "${A:?x}", "${A", "${A:-x",
                                   "${A:", "${:-x}", "${A B}", "$-"])
def test_invalid(value):
    with pytest.raises(InterpolationError) as ei:
        _run(value, key="environment")
    assert str(ei.value) == 'Invalid interpolation format for key "environment": "%s"' % value


def test_unset_without_default_is_blank_and_the_parse_logs_nothing(tmp_path, monkeypatch, capsys):
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("NOPE", raising=False)
    monkeypatch.setenv("EMPTY", "")
    p = tmp_path / "docker-compose.yml"
    p.write_text('version: "2"\nservices:\n  web:\n    image: "nginx:${NOPE}${EMPTY}latest"\n'
                 '    env_file: missing.env\n')
    log.set_verbose(True)
    try:
        proj = v1v2.parse_v2(str(p))
    finally:
        log.set_verbose(False)
    assert proj["services"][0]["image"] == "nginx:latest"
    err = capsys.readouterr().err
    assert "variable is not set" not in err and "Unable to find env config file" not in err


def test_dotenv_value_wins_and_empty_dotenv_takes_the_default(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("TAG", "from-os")
    (tmp_path / ".env").write_text("TAG=from-dotenv\nBLANK=\n")
    p = tmp_path / "docker-compose.yml"
    p.write_text('version: "2"\nservices:\n  web:\n    image: "nginx:${TAG}-${BLANK:-d}"\n')
    assert v1v2.parse_v2(str(p))["services"][0]["image"] == "nginx:from-dotenv-d"


def test_defaults_carry_across_files_of_one_command_and_the_memo_keeps_that(tmp_path, monkeypatch):
    """Within one command (the reference's process) a file parsed again after
    another file recorded a default parses with it; the parse memo keys on the
    recorded defaults."""
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("TAG", raising=False)
    a = tmp_path / "a.yml"
    a.write_text('version: "2"\nservices:\n  web:\n    image: "web:$TAG"\n')
    b = tmp_path / "b.yml"
    b.write_text('version: "2"\nservices:\n  db:\n    image: "db:${TAG:-9}"\n')
    with fsindex.scope():
        assert v1v2.parse_v2(str(a))["services"][0]["image"] == "web:"
        assert v1v2.parse_v2(str(b))["services"][0]["image"] == "db:9"
        assert v1v2.parse_v2(str(a))["services"][0]["image"] == "web:9"
        assert v1v2.parse_v2(str(b))["services"][0]["image"] == "db:9"
    with fsindex.scope():                           # a new command starts with no defaults
        assert v1v2.parse_v2(str(a))["services"][0]["image"] == "web:"


def test_invalid_interpolation_fails_the_load(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    p = tmp_path / "docker-compose.yml"
    p.write_text('version: "2"\nservices:\n  web:\n    image: nginx\n    command: "echo ${A?required}"\n')
    with pytest.raises(v1v2.ComposeError) as ei:
        v1v2.parse_v2(str(p))
    assert str(ei.value) == ('Failed to load docker compose file at path %s Error: "Invalid interpolation format for '
                             'key \\"command\\": \\"echo ${A?required}\\""' % p)


def test_dotenv_lookup_takes_the_first_line_naming_the_key(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / ".env").write_text("TAG=one\nTAG=two\n")
    p = tmp_path / "docker-compose.yml"
    p.write_text('version: "2"\nservices:\n  web:\n    image: "nginx:${TAG}"\n')
    assert v1v2.parse_v2(str(p))["services"][0]["image"] == "nginx:one"


def test_scanner_never_crashes_or_hangs():
    """Any value: a string or an InterpolationError, never another exception
    or a loop (libcompose itself panics or rescans on some of these)."""
    from hypothesis import given, settings as hsettings, strategies as st
    alphabet = st.sampled_from(list("$${}:-?AB_1 x"))

    @hsettings(max_examples=400, deadline=None)
    @given(st.lists(alphabet, max_size=14).map("".join))
    def check(value):
        try:
            out = _run(value, env={"A": "a", "B": ""})
        except InterpolationError:
            return
        assert isinstance(out, str)
    check()
