"""Host-side logic of the hot path's callers (no GPU): predicate literal parsing and HyperLogLog estimates."""
import os
import numpy as np
import pytest

import oracle
from pinot_amd import parse_sql
from pinot_amd import predicate as P
from pinot_amd.hll import HyperLogLog


def test_hll_all_registers_nonzero_small_estimate():
    """Every register set but the estimate in the small range: linearCounting(m, 0) = m * log(m / 0.0) = +Infinity in
    stream-lib, and Math.round(+Infinity) == Long.MAX_VALUE (no ZeroDivisionError)."""
    h = HyperLogLog(8, np.ones(256, dtype=np.uint8))
    assert h.cardinality() == (1 << 63) - 1
    h = HyperLogLog(4, np.ones(16, dtype=np.uint8))
    assert h.cardinality() == (1 << 63) - 1
    # one zero register: the ordinary linear-counting branch
    r = np.ones(256, dtype=np.uint8)
    r[0] = 0
    assert HyperLogLog(8, r).cardinality() == round(256 * np.log(256.0))


@pytest.mark.parametrize("lit,dtype,ok", [
    ("17", "INT", 17), ("-17", "INT", -17), ("+5", "INT", 5), ("2147483647", "INT", 2147483647),
    ("2147483648", "INT", None), ("1.5", "INT", None), ("1.0", "INT", None), ("1e3", "LONG", None),
    (" 7", "INT", None), ("1_000", "INT", None), ("9223372036854775807", "LONG", (1 << 63) - 1),
    ("9223372036854775808", "LONG", None), ("123456789012345678", "LONG", 123456789012345678),
])
def test_integral_literals_parse_like_java(lit, dtype, ok):
    """Integer.parseInt / Long.parseLong: a non-integral or out-of-range literal on an INT/LONG column is a
    NumberFormatException in the reference (IntDictionary.insertionIndexOf, RangePredicateEvaluatorFactory.java:80-85),
    never a truncated bound; LONG literals past 2^53 parse exactly. The oracle's restatement agrees."""
    if ok is None:
        with pytest.raises(ValueError):
            P.stored_value(lit, dtype)
        with pytest.raises(ValueError):
            oracle._parse(lit, dtype)
    else:
        assert P.stored_value(lit, dtype) == ok
        assert oracle._parse(lit, dtype) == ok


def test_fractional_bound_on_int_column_is_refused():
    from pinot_amd.segment import create_segment
    seg = create_segment("s", {"m": np.arange(10, dtype=np.int32)}, {"m": "INT"})
    q = parse_sql("SELECT COUNT(*) FROM t WHERE m >= 1.5")
    with pytest.raises(ValueError):
        P.dictionary_leaf(q.filter, seg.column("m"))


def test_build_rebuilds_when_any_header_changes(monkeypatch):
    """build() recompiles when any header under csrc/ (pa_keys.h included) or the JIT kernel source is newer than the
    library (pinot_amd/build.py _stale): HEADERS is globbed, so a new header is covered without an edit."""
    from pinot_amd import build as B
    assert "pa_keys.h" in B.HEADERS and "pa_gdense.h" in B.HEADERS
    lib_t = 1_000_000.0
    real_exists = os.path.exists

    def mtime(newer):
        return lambda p: lib_t if p == B.LIB else (lib_t + 10 if p.endswith(newer) else lib_t - 10)

    monkeypatch.setattr(os.path, "exists", lambda p: True if p == B.LIB else real_exists(p))
    monkeypatch.setattr(os.path, "getmtime", mtime("no-such-file"))
    assert not B._stale()
    for name in ("pa_keys.h", "pa_device.h", "gdl_jit.hip", "pinot_amd.h"):
        monkeypatch.setattr(os.path, "getmtime", mtime(name))
        assert B._stale(), name


def test_build_covers_every_source_and_rebuilds_objects_by_includes(monkeypatch):
    """Every .hip translation unit under csrc/ (the JIT kernels aside: hiprtc compiles them) is in build.SOURCES, the
    library is stale when any of them is newer, and an object is rebuilt exactly when its source or a header it includes
    (recursively) is newer (build._stale_objs): a host-only header such as pa_host.h rebuilds the host units, not the
    scan kernels."""
    from pinot_amd import build as B
    units = sorted(f for f in os.listdir(B.CSRC) if f.endswith(".hip") and f not in B.JIT_SOURCES)
    assert units == sorted(B.SOURCES)
    for name in ("pa_plan.hip", "pa_jit.hip", "pa_stats_host.hip", "pa_fetch.hip", "pa_segment.hip"):
        assert name in B.SOURCES
    deps = {s: {os.path.basename(d) for d in B._deps(os.path.join(B.CSRC, s))} for s in B.SOURCES}
    assert "pa_host.h" in deps["pa_capi.hip"] and "pa_jit_abi.h" in deps["pa_jit.hip"]
    assert "pa_host.h" not in deps["pa_scan_std.hip"] and "pa_scan.h" in deps["pa_scan_std.hip"]
    t0 = 1_000_000.0
    real_exists = os.path.exists

    def mtime(newer):
        return lambda p: t0 + 10 if os.path.basename(p) == newer else t0

    monkeypatch.setattr(os.path, "exists", lambda p: True if p.endswith(".o") or p == B.LIB else real_exists(p))
    monkeypatch.setattr(os.path, "getmtime", mtime("pa_host.h"))
    stale = set(B._stale_objs())
    assert stale == {s for s in B.SOURCES if "pa_host.h" in deps[s]} and "pa_scan_std.hip" not in stale
    monkeypatch.setattr(os.path, "getmtime", mtime("pa_plan.hip"))
    assert B._stale_objs() == ["pa_plan.hip"]
