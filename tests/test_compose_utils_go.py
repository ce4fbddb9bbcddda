"""Go library behaviour the compose loaders depend on (``source/compose/utils.py``):
``time.ParseDuration`` (healthcheck and stop-grace durations; the cases of Go's
own ``time_test.go`` table), docker/go-units ``RAMInBytes``, apimachinery
quantity strings, docker/go-connections ``ParsePortSpec`` and docker/cli's
``ParseVolume``."""

import os

import pytest

from move2kube_amd.source.compose import utils as cu

S, MS, US, M, H = 10 ** 9, 10 ** 6, 10 ** 3, 60 * 10 ** 9, 3600 * 10 ** 9


@pytest.mark.parametrize("text,want", [
    ("0", 0), ("5s", 5 * S), ("30s", 30 * S), ("1478s", 1478 * S), ("-5s", -5 * S), ("+5s", 5 * S),
    ("-0", 0), ("+0", 0), ("5.0s", 5 * S), ("5.6s", 5 * S + 600 * MS), ("5.s", 5 * S), (".5s", 500 * MS),
    ("1.0s", S), ("1.00s", S), ("1.004s", S + 4 * MS), ("1.0040s", S + 4 * MS), ("100.00100s", 100 * S + MS),
    ("10ns", 10), ("11us", 11 * US), ("12\u00b5s", 12 * US), ("12\u03bcs", 12 * US), ("13ms", 13 * MS),
    ("14s", 14 * S), ("15m", 15 * M), ("16h", 16 * H), ("3h30m", 3 * H + 30 * M),
    ("10.5s4m", 4 * M + 10 * S + 500 * MS), ("-2m3.4s", -(2 * M + 3 * S + 400 * MS)),
    ("1h2m3s4ms5us6ns", H + 2 * M + 3 * S + 4 * MS + 5 * US + 6), ("39h9m14.425s", 39 * H + 9 * M + 14 * S + 425 * MS),
    ("52763797000ns", 52763797000), ("0.3333333333333333333h", 20 * M), ("9007199254740993ns", (1 << 53) + 1),
    ("9223372036854775807ns", (1 << 63) - 1), ("9223372036854775.807us", (1 << 63) - 1),
    ("9223372036854ms775us807ns", (1 << 63) - 1), ("-9223372036854775807ns", -(1 << 63) + 1),
    ("0.100000000000000000000h", 6 * M), ("0.830103483285477580700h", 49 * M + 48 * S + 372539827),
])
def test_parse_duration_like_go(text, want):
    assert cu.parse_duration(text) == want


@pytest.mark.parametrize("text,err", [
    ("", 'time: invalid duration ""'), ("3", 'time: missing unit in duration "3"'),
    ("-", 'time: invalid duration "-"'), ("s", 'time: invalid duration "s"'), (".", 'time: invalid duration "."'),
    ("-.", 'time: invalid duration "-."'), (".s", 'time: invalid duration ".s"'),
    ("+.s", 'time: invalid duration "+.s"'), ("1d", 'time: unknown unit "d" in duration "1d"'),
    ("3000000h", 'time: invalid duration "3000000h"'),
    ("9223372036854775808ns", 'time: invalid duration "9223372036854775808ns"'),
    ("9223372036854775.808us", 'time: invalid duration "9223372036854775.808us"'),
    ("9223372036854ms775us808ns", 'time: invalid duration "9223372036854ms775us808ns"'),
    (None, 'time: invalid duration ""'),
])
def test_parse_duration_errors_like_go(text, err):
    with pytest.raises(ValueError) as ei:
        cu.parse_duration(text)
    assert str(ei.value) == err


@pytest.mark.parametrize("v,want", [
    (512, 512), (1.5, 1), ("512", 512), ("32k", 32 * 1024), ("32kb", 32 * 1024), ("32Ki", 32 * 1024),
    ("32KiB", 32 * 1024), ("1.5m", int(1.5 * 1024 ** 2)), ("2g", 2 * 1024 ** 3), ("1 t", 1024 ** 4),
    ("1p", 1024 ** 5), (" 7b ", 7),
])
def test_ram_in_bytes(v, want):
    assert cu.ram_in_bytes(v) == want


@pytest.mark.parametrize("v", [True, "", "abc", "1x", "-1m"])
def test_ram_in_bytes_errors(v):
    with pytest.raises(ValueError):
        cu.ram_in_bytes(v)


@pytest.mark.parametrize("milli,want", [
    (0, "0"), (500, "500m"), (1000, "1"), (1500, "1500m"), (2000000, "2k"), (-3000, "-3"),
    (5 * 10 ** 9, "5M"), (10 ** 21, "1E"),
])
def test_milli_quantity(milli, want):
    assert cu.format_milli_quantity(milli) == want


@pytest.mark.parametrize("value,want", [(0, "0"), (512, "512"), (536870912, "536870912"), (1000, "1e3"),
                                        (-2000000, "-2e6")])
def test_decimal_exponent_quantity(value, want):
    assert cu.format_quantity_decimal_exponent(value) == want


def test_shell_split():
    assert cu.shell_split("sh -c 'echo hi'") == ["sh", "-c", "echo hi"]
    assert cu.shell_split("echo 'unterminated") == ["echo", "'unterminated"]


@pytest.mark.parametrize("spec,want", [
    ("80", [("", 0, 80, "tcp")]),
    ("8080:80/UDP", [("", 8080, 80, "udp")]),
    ("127.0.0.1:8080:80", [("127.0.0.1", 8080, 80, "tcp")]),
    ("3000-3001:4000-4001", [("", 3000, 4000, "tcp"), ("", 3001, 4001, "tcp")]),
    ("9000:4000-4001", [("", 9000, 4000, "tcp"), ("", 9000, 4001, "tcp")]),
    ("[::1]:8080:80", [("::1", 8080, 80, "tcp")]),
    ("80/", [("", 0, 80, "tcp")]),
])
def test_parse_port_spec(spec, want):
    assert cu.parse_port_spec(spec) == want


@pytest.mark.parametrize("spec", ["8080:", "[::1:8080:80", "5-3", "1-3:4-5", "a:b:c:d"])
def test_parse_port_spec_errors(spec):
    with pytest.raises(ValueError):
        cu.parse_port_spec(spec)


@pytest.mark.parametrize("spec,want", [
    ("/data", {"type": "volume", "source": "", "target": "/data", "read_only": False}),
    ("vol:/data", {"type": "volume", "source": "vol", "target": "/data", "read_only": False}),
    ("./src:/app:ro", {"type": "bind", "source": "./src", "target": "/app", "read_only": True}),
    ("~/x:/app:ro,rw", {"type": "bind", "source": "~/x", "target": "/app", "read_only": False}),
    ("/abs:/app:z", {"type": "bind", "source": "/abs", "target": "/app", "read_only": False}),
])
def test_parse_volume(spec, want):
    assert cu.parse_volume_v3(spec) == want


def test_resolve_bind_source(monkeypatch, tmp_path):
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    assert cu.resolve_bind_source("~/data", "/w") == str(tmp_path / "home" / "data")
    assert cu.resolve_bind_source("./a/../b", "/w") == "/w/b"
    assert cu.resolve_bind_source("/abs", "/w") == "/abs"
    assert os.path.isabs(cu.resolve_bind_source("rel", str(tmp_path)))
