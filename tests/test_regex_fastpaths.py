"""String-operation fast paths that stand in for regexes on the cold-start path
agree with the regexes they replace (or, for prefilters, never reject a string
the regex accepts)."""

import re

from hypothesis import given, settings, strategies as st

from move2kube_amd.optimizer import strip_quotation
from move2kube_amd.utils import common, fsindex, yamlio

_TEXT = st.text(alphabet="aZ09_./ -:+eE'\",\n\té", max_size=12)


@settings(max_examples=800, deadline=None)
@given(_TEXT)
def test_simple_scalar(s):
    assert yamlio._is_simple_scalar(s) == bool(yamlio._SIMPLE_SCALAR.match(s))


@settings(max_examples=800, deadline=None)
@given(_TEXT)
def test_base60_and_float_prefilters(s):
    assert yamlio._is_base60(s) == bool(yamlio._BASE60.match(s))
    if yamlio._YAML_FLOAT.match(s):
        assert yamlio._maybe_float(s)


@settings(max_examples=500, deadline=None)
@given(st.text(alphabet="0123456789-:T.Z+ ", max_size=24))
def test_resolves_to_string_timestamp_prefilter(s):
    ts = any(rx.match(s) for rx in yamlio._TIMESTAMP_FORMATS)
    if ts and s[:1].isdigit():
        assert not yamlio.resolves_to_string(s)


@settings(max_examples=800, deadline=None)
@given(_TEXT)
def test_strip_quotation_is_re2(s):
    # RE2: "." excludes newline, "$" is the end of text
    m = re.fullmatch(r"[',\"]([^\n]*)[',\"]", s)
    assert strip_quotation(s) == (m.group(1) if m else s)


@settings(max_examples=800, deadline=None)
@given(_TEXT)
def test_name_helpers(s):
    low = s.lower()
    assert common.make_string_dns_name_compliant(s) == re.sub(r"[^a-z0-9\-.]", "-", low)
    base = s.rstrip("/")
    if base and "/" not in base:
        assert common.make_file_name_compliant(s) == re.sub(r"[^a-zA-Z0-9\-.]+", "-", base)
    assert common.normalize_for_service_name(s) == re.sub(r"[._]", "-", s).lower()


@settings(max_examples=500, deadline=None)
@given(st.text(alphabet="*.ab+_-?[]\n", max_size=8))
def test_suffix_pattern(p):
    assert fsindex._is_suffix_pattern(p) == bool(re.fullmatch(r"\*\.[A-Za-z0-9_+-]+", p))
