"""Compose v3 interpolation as docker/cli (the reference's pinned a4bedce16568)
does it: ``compose/template.Substitute`` with its substitution functions and
error variable, and ``compose/interpolation.Interpolate`` with the loader's
type casts (``cli/compose/loader/interpolate.go``) and ``newPathError``
texts.  Reached through ``compose.ParseV3`` (reference
``internal/source/compose/v3.go:93-121``)."""

import pytest

from move2kube_amd.source.compose import v3
from move2kube_amd.source.compose.interpolate import InterpolationError, interpolate_v3, substitute_v3

ENV = {"A": "a", "E": "", "N": "3"}


@pytest.mark.parametrize("template,want", [
    ("plain", "plain"),
    ("$$A", "$A"),
    ("$A-$A", "a-a"),
    ("${A}x", "ax"),
    ("$UNSET.", "."),
    ("${UNSET:-d} ${E:-d} ${A:-d}", "d d a"),
    ("${UNSET-d} ${E-d}", "d "),
    ("${A:?m} ${A?m} ${E?m}", "a a "),
    ("${a}", ""),                                     # names are case-sensitive, the pattern is not
    # strings.Contains order: a hard default ("-") is found before ":?" and "?"
    ("${UNSET:?no-value}", "value"),
    ("${A?x-y}", "y"),
    ("${A?x:-y}", "y"),
    ("${UNSET-x:?y}", "x:?y"),
    # the error variable is overwritten by every later substitution
    ("$ and ${A}", " and a"),
    ("${UNSET:?required} then $A", " then a"),
    ("${A:x} $N", "{A:x} 3"),                        # only the "$" is the invalid match
])
def test_substitute(template, want):
    got, err = substitute_v3(template, ENV.get)
    assert (got, err) == (want, None)


@pytest.mark.parametrize("template,err", [
    ("cost: 5$", "cost: 5$"),
    ("$1", "$1"),
    ("${A:x}", "${A:x}"),
    ("${}", "${}"),
    ("$A then $", "$A then $"),
    ("$A ${UNSET:?set it}", "required variable UNSET is missing a value: set it"),
    ("${E:?}", "required variable E is missing a value: "),
])
def test_substitute_errors(template, err):
    _, e = substitute_v3(template, ENV.get)
    assert e is not None and e.template == err


def test_interpolate_casts_only_what_changed():
    cfg = {"version": "3.7", "services": {"web": {
        "image": "${A}", "deploy": {"replicas": "${N}", "update_config": {"max_failure_ratio": "${R:-0.5}"}},
        "ports": [{"target": "${P:-80}", "published": "8080"}, "${N}000:80"],
        "tty": "${T:-on}", "read_only": "no", "ulimits": {"nofile": {"soft": "${N}", "hard": 4}, "nproc": "${N}"}}},
        "networks": {"n": {"external": "${X:-yes}"}}, "volumes": {"v": {"external": "${X:-off}"}}}
    out = interpolate_v3(cfg, ENV.get)
    web = out["services"]["web"]
    assert web["image"] == "a" and web["deploy"]["replicas"] == 3
    assert web["deploy"]["update_config"]["max_failure_ratio"] == 0.5
    assert web["ports"] == [{"target": 80, "published": "8080"}, "3000:80"]
    assert web["tty"] is True and web["read_only"] == "no"            # not interpolated: not cast
    assert web["ulimits"] == {"nofile": {"soft": 3, "hard": 4}, "nproc": 3}
    assert out["networks"]["n"]["external"] is True and out["volumes"]["v"]["external"] is False


@pytest.mark.parametrize("cfg,err", [
    ({"services": {"web": {"image": "$"}}},
     'invalid interpolation format for services.web.image: "$". You may need to escape any $ with another $.'),
    ({"services": {"web": {"environment": ["X=${UNSET:?needed}"]}}},
     'invalid interpolation format for services.web.environment.[]: "required variable UNSET is missing a value: '
     'needed". You may need to escape any $ with another $.'),
    ({"services": {"web": {"deploy": {"replicas": "${A}"}}}},
     'error while interpolating services.web.deploy.replicas: failed to cast to expected type: strconv.Atoi: '
     'parsing "a": invalid syntax'),
    ({"services": {"web": {"deploy": {"replicas": "${N}0000000000000000000000"}}}},
     'error while interpolating services.web.deploy.replicas: failed to cast to expected type: strconv.Atoi: '
     'parsing "30000000000000000000000": value out of range'),
    ({"services": {"web": {"tty": "${A}"}}},
     "error while interpolating services.web.tty: failed to cast to expected type: invalid boolean: a"),
    ({"services": {"web": {"deploy": {"rollback_config": {"max_failure_ratio": "${A}"}}}}},
     'error while interpolating services.web.deploy.rollback_config.max_failure_ratio: failed to cast to expected '
     'type: strconv.ParseFloat: parsing "a": invalid syntax'),
])
def test_interpolate_errors(cfg, err):
    with pytest.raises(InterpolationError) as ei:
        interpolate_v3(cfg, ENV.get)
    assert str(ei.value) == err


def test_interpolated_numbers_load(tmp_path, monkeypatch):
    """A replica count or port from the environment is a number to the
    schema, as docker/cli casts it; the same text written quoted is not."""
    monkeypatch.delenv("R", raising=False)
    p = tmp_path / "docker-compose.yaml"
    p.write_text('version: "3.7"\nservices:\n  web:\n    image: nginx\n    deploy:\n      replicas: ${R:-2}\n'
                 '    ports:\n      - target: ${P:-80}\n        published: 8080\n    tty: ${T:-true}\n')
    (svc,) = v3.parse_v3(str(p))["services"]
    assert svc["deploy"]["replicas"] == 2 and svc["ports"][0]["target"] == 80 and svc["tty"] is True
    q = tmp_path / "quoted.yaml"
    q.write_text('version: "3.7"\nservices:\n  web:\n    image: nginx\n    deploy:\n      replicas: "2"\n')
    with pytest.raises(v3.ComposeError, match="replicas must be a integer"):
        v3.parse_v3(str(q))


def test_forbidden_properties_fail_before_interpolation(tmp_path):
    """loader.Load runs validateForbidden before interpolating: its error wins
    over a malformed ${...} in the same file."""
    p = tmp_path / "docker-compose.yaml"
    p.write_text('version: "3"\nservices:\n  web:\n    image: "$"\n    mem_limit: 1g\n')
    with pytest.raises(v3.ComposeError) as ei:
        v3.parse_v3(str(p))
    assert str(ei.value) == ('Unable to load Compose file at path %s Error: "Configuration contains forbidden '
                             'properties"' % p)


def test_version_is_read_before_interpolation_and_checked_after(tmp_path, monkeypatch):
    monkeypatch.setenv("V", "3.7")
    p = tmp_path / "docker-compose.yaml"
    p.write_text('version: "${V}"\nservices:\n  web:\n    image: "$"\n')
    with pytest.raises(v3.ComposeError) as ei:
        v3.parse_v3(str(p))
    assert "invalid interpolation format for services.web.image" in str(ei.value)
    p.write_text('version: "${V}"\nservices:\n  web:\n    image: nginx\n')
    with pytest.raises(v3.ComposeError, match=r"unsupported Compose file version: \$\{V\}"):
        v3.parse_v3(str(p))


def test_substitute_never_crashes():
    from hypothesis import given, settings as hsettings, strategies as st
    alphabet = st.sampled_from(list("$${}:-?AB_1 x"))

    @hsettings(max_examples=400, deadline=None)
    @given(st.lists(alphabet, max_size=14).map("".join))
    def check(value):
        out, err = substitute_v3(value, ENV.get)
        assert isinstance(out, str) and (err is None or isinstance(err.template, str))
    check()


@pytest.mark.parametrize("body,err", [
    ("    healthcheck:\n      interval: 5x\n", "services.web.healthcheck.interval Does not match format 'duration'"),
    ("    healthcheck:\n      start_period: 1\n", "services.web.healthcheck.start_period must be a string"),
    ("    stop_grace_period: 1d\n", "services.web.stop_grace_period Does not match format 'duration'"),
    ("    deploy:\n      restart_policy:\n        window: 10\n",
     "services.web.deploy.restart_policy.window must be a string"),
    ("    deploy:\n      update_config:\n        monitor: 1h1\n",
     "services.web.deploy.update_config.monitor Does not match format 'duration'"),
])
def test_duration_format_fails_the_load(tmp_path, body, err):
    """docker/cli's schema.go checks the "duration" format with
    time.ParseDuration, so a bad duration refuses the whole file (v3.go:93-121)
    instead of only its health check."""
    p = tmp_path / "docker-compose.yaml"
    p.write_text('version: "3.7"\nservices:\n  web:\n    image: nginx\n' + body)
    with pytest.raises(v3.ComposeError) as ei:
        v3.parse_v3(str(p))
    assert str(ei.value) == 'Unable to load Compose file at path %s Error: "%s"' % (p, err)


def test_durations_from_the_environment(tmp_path, monkeypatch):
    monkeypatch.setenv("HC", "1m30s")
    p = tmp_path / "docker-compose.yaml"
    p.write_text('version: "3.7"\nservices:\n  web:\n    image: nginx\n    stop_grace_period: 2h45m.5s\n'
                 '    healthcheck:\n      interval: ${HC}\n      timeout: "-1.5us"\n')
    (svc,) = v3.parse_v3(str(p))["services"]
    assert svc["healthcheck"]["interval"] == "1m30s"
