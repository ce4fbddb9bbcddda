"""Go library behaviour the compose loaders depend on (``source/compose/utils.py``):
``time.ParseDuration`` (healthcheck and stop-grace durations; the cases of Go's
own ``time_test.go`` table), docker/go-units ``RAMInBytes``, apimachinery
quantity strings, docker/go-connections ``ParsePortSpec`` and docker/cli's
``ParseVolume``."""

import os

import pytest

import logparse

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
    ("1p", 1024 ** 5), ("7b", 7), ("0012.50M", int(12.5 * 1024 ** 2)),
])
def test_ram_in_bytes(v, want):
    assert cu.ram_in_bytes(v) == want


@pytest.mark.parametrize("v,err", [
    (True, "invalid size"), ("", "invalid size: ''"), ("abc", "invalid size: 'abc'"), ("1x", "invalid size: '1x'"),
    ("-1m", "invalid size: '-1m'"), (" 7b ", "invalid size: ' 7b '"), ("5m\n", "invalid size: '5m\n'"),
    ("\u0661m", "invalid size: '\u0661m'"), ("1.2.3k", 'strconv.ParseFloat: parsing "1.2.3": invalid syntax'),
])
def test_ram_in_bytes_errors(v, err):
    """go-units v0.4.0 parseSize: RE2 semantics (ASCII digits, ``$`` at the
    very end, no trimming), then ParseFloat of the number part."""
    with pytest.raises(ValueError) as ei:
        cu.ram_in_bytes(v)
    assert str(ei.value) == err


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
    ("80", [(80, 0, "tcp", "ingress")]),
    (80, [(80, 0, "tcp", "ingress")]),
    ("8080:80/UDP", [(80, 8080, "udp", "ingress")]),
    ("127.0.0.1:8080:80", [(80, 8080, "tcp", "ingress")]),
    ("3000-3001:4000-4001", [(4000, 3000, "tcp", "ingress"), (4001, 3001, "tcp", "ingress")]),
    ("8000-8002:80", [(80, 8000, "tcp", "ingress"), (80, 8001, "tcp", "ingress"), (80, 8002, "tcp", "ingress")]),
    ("9-10:9-10", [(10, 10, "tcp", "ingress"), (9, 9, "tcp", "ingress")]),     # "10/tcp" sorts first
    ("[::1]:8080:80", [(80, 8080, "tcp", "ingress")]),
    ("80/", [(80, 0, "tcp", "ingress")]),
    ("80/sctp/x", [(80, 0, "sctp", "ingress")]),
    (":80", [(80, 0, "tcp", "ingress")]),
    ("1.2.3.4::80", [(80, 0, "tcp", "ingress")]),
    ("010.1.1.1:1:1", [(1, 1, "tcp", "ingress")]),
])
def test_to_service_port_configs(spec, want):
    """docker/cli toServicePortConfigs over go-connections nat (v0.4.0)."""
    assert cu.to_service_port_configs(str(spec)) == want


@pytest.mark.parametrize("spec,err", [
    ("8080:", "No port specified: 8080:<empty>"),
    ("", "No port specified: <empty>"),
    ("[::1:8080:80", "Invalid ip address [::1: address [::1:: missing ']' in address"),
    ("::1:8080:80", "Invalid ip address ::1: address ::1:: too many colons in address"),
    ("1.2.3:80:80", "Invalid ip address: 1.2.3"),
    ("fe80::1%eth0:80:80", "Invalid ip address fe80::1%eth0: address fe80::1%eth0:: too many colons in address"),
    ("5-3", "Invalid containerPort: 5-3"),
    ("70000", "Invalid containerPort: 70000"),
    ("+80", "Invalid containerPort: +80"),
    ("abc:80", "Invalid hostPort: abc"),
    ("1-3:4-5", "Invalid ranges specified for container and host Ports: 4-5 and 1-3"),
    ("9000:4000-4001", "Invalid ranges specified for container and host Ports: 4000-4001 and 9000"),
    ("80/xyz", "Invalid proto: xyz"),
    ("a:b:c:d", "Invalid ip address a:b: address a:b:: too many colons in address"),
])
def test_port_spec_errors(spec, err):
    with pytest.raises(ValueError) as ei:
        cu.to_service_port_configs(spec)
    assert str(ei.value) == err


def test_host_ip_warning(capsys):
    """opts.ConvertPortToPortConfig warns for a host IP other than 0.0.0.0."""
    cu.to_service_port_configs("0.0.0.0:80:80")
    cu.to_service_port_configs("127.0.0.1:8000-8001:80/udp")
    err = capsys.readouterr().err
    assert err.count("level=warning") == 1
    assert logparse.logged(err, "ignoring IP-address (127.0.0.1:8000-8001:80/udp) service will listen on "
                                "'0.0.0.0'", "warning")


@pytest.mark.parametrize("spec,want", [
    ("/data", {"type": "volume", "source": "", "target": "/data", "read_only": False}),
    ("vol:/data", {"type": "volume", "source": "vol", "target": "/data", "read_only": False}),
    ("./src:/app:ro", {"type": "bind", "source": "./src", "target": "/app", "read_only": True}),
    ("~/x:/app:ro,rw", {"type": "bind", "source": "~/x", "target": "/app", "read_only": False}),
    ("/abs:/app:z", {"type": "bind", "source": "/abs", "target": "/app", "read_only": False}),
    ("v:/data", {"type": "volume", "source": "", "target": "v:/data", "read_only": False}),   # a drive letter
    ("c:/d:/data", {"type": "bind", "source": "c:/d", "target": "/data", "read_only": False}),
    ("a:", {"type": "volume", "source": "", "target": "a:", "read_only": False}),           # two characters
    ("data:/x:nocopy,ro", {"type": "volume", "source": "data", "target": "/x", "read_only": True}),
])
def test_parse_volume(spec, want):
    """docker/cli loader.ParseVolume (cli/compose/loader/volume.go)."""
    assert cu.parse_volume_v3(spec) == want


@pytest.mark.parametrize("spec,err", [
    ("", "invalid empty volume spec"),
    ("vol::/x", "invalid spec: vol::/x: empty section between colons"),
    ("vol:/x:ro:z", "invalid spec: vol:/x:ro:z: too many colons"),
])
def test_parse_volume_errors(spec, err):
    with pytest.raises(ValueError) as ei:
        cu.parse_volume_v3(spec)
    assert str(ei.value) == err


def test_abs_path():
    assert cu.go_abs_path("/w", "./a/../b") == "/w/b"
    assert cu.go_abs_path("/w", "/abs") == "/abs"
    assert cu.go_abs_path("/w", "") == "/w"
    assert cu.go_abs_path("/w", "~/x") == "/w/~/x"


@pytest.mark.parametrize("hostport,want", [
    ("a:", ("a", "")), ("[::1]:80", ("::1", "80")), (":", ("", "")),
    ("x", "address x: missing port in address"),
    ("[::1]", "address [::1]: missing port in address"),
    ("[::1", "address [::1: missing ']' in address"),
    ("[a]b:", "address [a]b:: missing port in address"),
    ("[::1]:x:", "address [::1]:x:: too many colons in address"),
    ("a:b:", "address a:b:: too many colons in address"),
    ("a[b:", "address a[b:: unexpected '[' in address"),
    ("a]b:", "address a]b:: unexpected ']' in address"),
])
def test_split_host_port(hostport, want):
    """net.SplitHostPort (Go 1.15) and its *net.AddrError texts."""
    if isinstance(want, tuple):
        assert cu._split_host_port(hostport) == want
    else:
        with pytest.raises(ValueError) as ei:
            cu._split_host_port(hostport)
        assert str(ei.value) == want


@pytest.mark.parametrize("ip,ok", [
    ("1.2.3.4", True), ("001.02.3.255", True), ("1.2.3.4.5", False), ("1..2.3", False), ("256.1.1.1", False),
    ("1.2.3", False), ("::1", True), ("::ffff:1.2.3.4", True), ("fe80::1%eth0", False), ("::zz", False),
    ("abc", False), ("", False),
])
def test_go_parse_ip(ip, ok):
    assert cu.go_parse_ip_ok(ip) is ok
