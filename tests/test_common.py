"""Common helpers beyond ``internal/common/utils_test.go`` (whose subtests are
ported one by one in ``test_reference_utils.py``)."""

import json
import os

import pytest

from conftest import ref_path
from move2kube_amd.utils import common, tarutil


def test_is_string_present_is_case_insensitive():
    # utils_test.go's cases are in test_reference_utils.py; Go's IsStringPresent uses EqualFold
    assert common.is_string_present(["foo", "bar"], "FOO")


def test_tar_roundtrip(tmp_path):
    src = tmp_path / "src"
    (src / "d" / "e").mkdir(parents=True)
    (src / "a.txt").write_text("hello")
    (src / "d" / "b.yaml").write_text("k: v\n")
    os.chmod(str(src / "d" / "b.yaml"), 0o600)
    s = tarutil.tar_as_string(str(src), ["d/e"])
    dst = tmp_path / "dst"
    tarutil.untar_string(s, str(dst))
    assert (dst / "a.txt").read_text() == "hello"
    assert (dst / "d" / "b.yaml").read_text() == "k: v\n"
    assert oct(os.stat(str(dst / "d" / "b.yaml")).st_mode & 0o777) == "0o600"
    assert not (dst / "d" / "e").exists()


def test_tar_missing_path(tmp_path):
    with pytest.raises(tarutil.TarError):
        tarutil.tar_as_string(str(tmp_path / "nope"))


def test_untar_rejects_escaping_entries(tmp_path):
    import base64, io, tarfile
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as t:
        info = tarfile.TarInfo("../evil")
        info.size = 1
        t.addfile(info, io.BytesIO(b"x"))
    with pytest.raises(tarutil.TarError):
        tarutil.untar_string(base64.b64encode(buf.getvalue()).decode(), str(tmp_path / "d"))


@pytest.mark.reference
def test_untar_reference_tarstring(tmp_path):
    with open(ref_path("internal", "common", "testdata", "datafortestingtar", "untarstring.json")) as f:
        data = json.load(f)
    tarutil.untar_string(data["untar_a_valid_tarstring"], str(tmp_path))
    names = sorted(os.path.relpath(os.path.join(dp, f), str(tmp_path)) for dp, _, fs in os.walk(str(tmp_path)) for f in fs)
    assert names


def test_copy_file_like_go_copyfile(tmp_path):
    """``CopyFile`` (utils.go:587-615): new destination gets 0644 & ~umask; an
    existing one is truncated and keeps its mode."""
    umask = os.umask(0o022)
    os.umask(umask)
    src = tmp_path / "src"
    src.write_bytes(b"abc" * 1000)
    dst = tmp_path / "dst"
    common.copy_file(str(dst), str(src))
    assert dst.read_bytes() == src.read_bytes()
    assert dst.stat().st_mode & 0o777 == 0o644 & ~umask
    os.chmod(str(dst), 0o600)
    src.write_bytes(b"x")
    common.copy_file(str(dst), str(src))
    assert dst.read_bytes() == b"x" and dst.stat().st_mode & 0o777 == 0o600


def test_cgroup_cpu_limit(tmp_path):
    """Thread pools are sized within the cgroup CPU quota (v2 and v1)."""
    from move2kube_amd.utils.constants import _cgroup_cpu_limit
    v2 = tmp_path / "v2"
    v2.mkdir()
    (v2 / "cpu.max").write_text("1600000 100000\n")
    assert _cgroup_cpu_limit(str(v2)) == 16
    (v2 / "cpu.max").write_text("max 100000\n")
    assert _cgroup_cpu_limit(str(v2)) is None
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("250000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert _cgroup_cpu_limit(str(v1)) == 2
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert _cgroup_cpu_limit(str(v1)) is None
    assert _cgroup_cpu_limit(str(tmp_path / "none")) is None


def test_exec_errors_read_like_go(tmp_path):
    """os/exec start failures and *ExitError texts (collectors, CNB providers,
    operator-sdk) as the reference prints them."""
    import pytest as _pytest
    from move2kube_amd.utils import common as c
    with _pytest.raises(FileNotFoundError) as ei:
        c.run_command(["m2k-no-such-tool", "x"])
    assert str(ei.value) == 'exec: "m2k-no-such-tool": executable file not found in $PATH'
    missing = str(tmp_path / "nope")
    with _pytest.raises(FileNotFoundError) as ei:
        c.run_command([missing])
    assert str(ei.value) == "fork/exec %s: no such file or directory" % missing
    assert c.go_exit_status(0) == "exit status 0" and c.go_exit_status(3) == "exit status 3"
    assert c.go_exit_status(-9) == "signal: killed" and c.go_exit_status(-15) == "signal: terminated"
    assert c.go_exit_status(-11) == "signal: segmentation fault" and c.go_exit_status(-40) == "signal: signal 40"


def test_os_errors_read_like_go_path_errors(tmp_path):
    import errno
    import os
    from move2kube_amd.utils import common as c
    f = tmp_path / "file"
    f.write_text("x")
    try:
        os.makedirs(str(f), exist_ok=True)
    except OSError as e:
        # os.MkdirAll over an existing regular file: ENOTDIR
        assert c.go_path_error(e, "mkdir") == "mkdir %s: not a directory" % f
    try:
        open(str(f / "x"))
    except OSError as e:
        assert c.go_path_error(e, "open") == "open %s: not a directory" % (f / "x")
    e = PermissionError(errno.EACCES, "Permission denied", "/out")
    assert c.go_path_error(e, "mkdir") == "mkdir /out: permission denied"
    assert c.go_path_error(OSError("no path"), "open") == "no path"


def test_unnamed_temp_file(tmp_path, monkeypatch):
    from move2kube_amd.utils import common
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    with common.unnamed_temp_file() as f:
        f.write(b"operator output")
        f.seek(0)
        assert f.read() == b"operator output"
        assert os.listdir(str(tmp_path)) == []  # no name in the directory
    monkeypatch.setenv("TMPDIR", str(tmp_path / "missing"))
    with common.unnamed_temp_file() as f:  # falls back to tempfile's search
        f.write(b"x")


def test_go_case_helpers():
    """strings.ToLower / strings.EqualFold use simple (one-to-one) case
    mappings; Python's lower/casefold apply the full ones."""
    from move2kube_amd.utils import common
    assert common.go_lower("MyApp") == "myapp"
    assert common.go_lower("İstanbul") == "istanbul"          # str.lower: "i̇stanbul"
    assert common.go_fold("STRASSE") != common.go_fold("Straße")  # casefold equates them
    assert common.go_fold("ẞ") == common.go_fold("ß")        # capital sharp s folds to sharp s
    assert common.go_fold("K") == common.go_fold("k")             # Kelvin sign
    assert common.go_fold("ſ") == common.go_fold("S")             # long s
    assert common.go_fold("İ") != common.go_fold("i")
    assert common.is_string_present(["Straße"], "STRASSE") is False
    assert common.is_string_present(["STRAẞE"], "straße") is True
    assert common.normalize_for_service_name("İzmir_App.v2") == "izmir-app-v2"


def test_dns_names_count_utf8_bytes_like_go():
    """MakeStringDNSLabelNameCompliant / ...SubdomainNameCompliant
    (utils.go:461-486) compare and cut Go string lengths, i.e. UTF-8 bytes;
    a rune cut in two leaves one invalid byte each, replaced by '-'."""
    import hashlib
    from move2kube_amd.utils import common
    assert common.make_string_dns_label_name_compliant("My_App") == "my-app"
    s = "é" * 40                                  # 40 characters, 80 bytes
    h = hashlib.sha256(s.encode()).hexdigest()[:32]
    assert common.make_string_dns_label_name_compliant(s) == "-" * 15 + "-" + h
    s = "a" + "é" * 20                           # 41 bytes: cut at 30 splits the 15th rune
    s = s + "b" * 30                                   # 71 bytes
    h = hashlib.sha256(s.encode()).hexdigest()[:32]
    out = common.make_string_dns_label_name_compliant(s)
    assert out == "a" + "-" * 14 + "-" + "-" + h      # 14 whole runes, 1 stray byte, then the hyphen
    assert len(out) == 1 + 14 + 1 + 1 + 32   # each non-ASCII rune became one '-'
    s = "x" * 200 + "中" * 20                      # 260 bytes
    out = common.make_string_dns_subdomain_name_compliant(s)
    assert out == "x" * 188 + "-" + hashlib.sha256(s.encode()).hexdigest() and len(out) == 253
    assert common.make_string_dns_subdomain_name_compliant("x" * 200 + "中" * 17) == "x" * 200 + "-" * 17


@pytest.mark.parametrize("text,want", [
    ("1.5", 1.5), ("1_000.5", 1000.5), ("0x1p-2", 0.25), (".5", 0.5), ("5.", 5.0), ("-2e3", -2000.0),
    ("Infinity", float("inf")), ("-inf", float("-inf")), ("1e-400", 0.0),
    ("0x1.8", "invalid syntax"), ("+nan", "invalid syntax"), (" 1", "invalid syntax"), ("1e", "invalid syntax"),
    ("1__0", "invalid syntax"), ("٣", "invalid syntax"), ("1e400", "value out of range"),
])
def test_go_parse_float(text, want):
    """strconv.ParseFloat, not float(): no spaces, no signed NaN, hex needs
    'p', ASCII digits only, overflow is an error."""
    from move2kube_amd.utils import common
    if isinstance(want, str):
        with pytest.raises(ValueError) as ei:
            common.go_parse_float(text)
        assert str(ei.value).endswith(want)
    else:
        assert common.go_parse_float(text) == want


@pytest.mark.parametrize("text,want", [
    ("80", 80), ("010", 8), ("0x1F", 31), ("-0b101", -5), ("0o17", 15), ("1_000", 1000), ("0", 0), (None, 0),
    (7.9, 7), (True, 1),
    ("080", None), ("08", None), (" 80", None), ("80 ", None), ("1.0", None), ("", None), ("+", None),
    ("9223372036854775808", None), ("_1", None), ("١٢", None),
])
def test_cast_to_int_is_cast_v1_3_1(text, want):
    """spf13/cast v1.3.1 ToIntE = strconv.ParseInt(s, 0, 0): no trimming, no
    "1.0" (that came with cast v1.4), octal by a leading 0."""
    from move2kube_amd.utils import common
    if want is None:
        with pytest.raises(ValueError) as ei:
            common.cast_to_int(text)
        assert str(ei.value) == 'unable to cast "%s" of type string to int' % text
    else:
        assert common.cast_to_int(text) == want


def test_go_float_to_int64():
    from move2kube_amd.utils import common
    assert common.go_float_to_int64(2.9) == 2 and common.go_float_to_int64(-2.9) == -2
    for f in (float("nan"), float("inf"), float("-inf"), 1e19):
        assert common.go_float_to_int64(f) == -(1 << 63)


def test_go_abs_cleans_a_double_leading_slash(tmp_path, monkeypatch):
    from move2kube_amd.utils import common
    assert common.go_abs("//tmp//x/../y") == "/tmp/y"
    monkeypatch.chdir(str(tmp_path))
    assert common.go_abs("a/./b/") == os.path.join(os.path.realpath(str(tmp_path)), "a", "b") or \
        common.go_abs("a/./b/") == os.path.join(str(tmp_path), "a", "b")


def test_template_execution_failure_is_reported_with_its_data(capsys):
    """GetStringFromTemplate (utils.go:347-357) warns with the template (%q)
    and its data (%v) before returning the error; JSON numbers are float64."""
    import logparse
    from move2kube_amd.utils import common, log
    from move2kube_amd.utils.gotemplate import TemplateError
    log.set_verbose(False)
    with pytest.raises(TemplateError) as ei:
        common.get_string_from_template("FROM {{.port.x}}", {"port": 8080.0, "app": "a b", "n": None})
    # exec.go evalField: the receiver is a map element, of type interface {};
    # the error carries Go's location (the chain's second field) and context
    assert str(ei.value) == ('template: :1:12: executing "" at <.port.x>: '
                             "can't evaluate field x in type interface {}")
    assert logparse.logged(capsys.readouterr().err, 'Unable to translate template "FROM {{.port.x}}" to string '
                           "using the data map[app:a b n:<nil> port:8080]", "warning")


def test_image_info_without_tags_is_logged_as_go_value(capsys):
    import logparse
    from move2kube_amd.models import ir
    from move2kube_amd.models.collection import ImageInfo
    from move2kube_amd.utils import log
    log.set_verbose(False)
    info = ImageInfo()
    info.name, info.ports, info.accessed_dirs, info.user_id = "img", [8080], ["/app"], -1
    c = ir.new_container_from_image_info(info)
    assert c.image_names == []
    assert logparse.logged(capsys.readouterr().err, "The image info {{move2kube.konveyor.io/v1alpha1 ImageMetadata} "
                           "{img} {[] [8080] [/app] -1}} has no tags. Leaving the tag empty for the container.", "error")
