"""Aggregation-only queries on the per-lane register path (STRAT_LANE, lane-major tiles) against the oracle.

The path picks, per tile and aggregation (pa_scan.h lane_acc_tile):
  raw columns        sparse tiles: per-doc loads of the matching docs; dense tiles: the whole tile as coalesced 16-byte
                     loads with every value's match bit fetched from the lane that owns its doc (ds_bpermute)
  dictionary columns few matches per lane: decode + gather of those docs only; else the static-unpack full-tile path
                     (MIN / MAX of a sorted dictionary on dictIds)
so the selectivities below (~0.02 % .. 100 %) drive every branch, over INT / LONG / FLOAT / DOUBLE raw values and
dictionary columns, on ragged segments (a partial last tile). Reference semantics: AggregationOperator ->
Sum/Min/MaxAggregationFunction.aggregate. Bars: bit-exact COUNT, integer SUM, MIN, MAX; DOUBLE SUM within 1e-9.
"""
import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.segment import create_segment
from test_gpu_parity import assert_same
import oracle

pytestmark = pytest.mark.gpu

DOUBLE_REL = 1e-9


def _segment(seed, n):
    rng = np.random.default_rng(seed)
    data = {
        "day": rng.integers(0, 4000, size=n).astype(np.int32),     # 12-bit dictionary filter column
        "ri": rng.integers(-(1 << 30), 1 << 30, size=n).astype(np.int32),
        "rl": rng.integers(-(1 << 40), 1 << 40, size=n).astype(np.int64),
        "rf": rng.normal(0, 1e3, size=n).astype(np.float32),
        "rd": rng.normal(0, 1e6, size=n),
        "dl": rng.integers(0, 1 << 14, size=n).astype(np.int64) * 37 - 99999,  # dictionary LONG metric
        "dd": np.round(rng.normal(0, 100, size=n), 2),                          # dictionary DOUBLE metric
        "rs": rng.integers(-(1 << 31), 1 << 31, size=n).astype(np.int64),      # raw LONG in int32 range (SUM_I64)
        "g": rng.integers(0, 700, size=n).astype(np.int32),                    # group-by dimension
    }
    data["rs"][:2] = [-(1 << 31), (1 << 31) - 1]
    schema = {"day": "INT", "ri": "INT", "rl": "LONG", "rf": "FLOAT", "rd": "DOUBLE", "dl": "LONG", "dd": "DOUBLE",
              "rs": "LONG", "g": "INT"}
    return create_segment("lane%d" % seed, data, schema, no_dictionary_columns=("ri", "rl", "rf", "rd", "rs"))


@pytest.fixture(scope="module")
def lane_segments():
    segs = [_segment(1, 300_001), _segment(2, 65_536), _segment(3, 2049)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


# day < hi keeps ~hi/4000 of the docs
SELECTIVITY = {"0.02pct": 1, "1pct": 40, "5pct": 200, "30pct": 1200, "all": 4000}
AGGS = [
    "COUNT(*), SUM(ri), MIN(ri), MAX(ri)",
    "SUM(rl), MIN(rl), MAX(rl)",
    "SUM(rf), MIN(rf), MAX(rf), COUNT(*)",
    "SUM(rd), MIN(rd), MAX(rd)",
    "COUNT(*), SUM(dl), MIN(dl), MAX(dl)",
    "SUM(dd), MIN(dd), MAX(dd), SUM(rl)",
    "COUNT(*), SUM(rs), MIN(rs), MAX(rs)",
]


@pytest.mark.parametrize("sel", list(SELECTIVITY))
@pytest.mark.parametrize("aggs", AGGS)
def test_lane_aggregations(lane_segments, sel, aggs):
    segs, gs = lane_segments
    q = parse_sql("SELECT %s FROM t WHERE day < %d" % (aggs, SELECTIVITY[sel]))
    ex = GpuQueryExecutor(q, gs)
    try:
        st = ex.stats()["plan"]
        assert st["strategy"] == "lane" and st["lane_major"] == 1, st
        got = ex.run()
    finally:
        ex.close()
    assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


def test_lane_no_filter_and_empty_result(lane_segments):
    segs, gs = lane_segments
    for sql in ("SELECT SUM(rl), MIN(rd), MAX(ri), SUM(dl) FROM t",
                "SELECT COUNT(*), SUM(rl), MIN(rd) FROM t WHERE day < 0"):
        q = parse_sql(sql)
        ex = GpuQueryExecutor(q, gs)
        try:
            got = ex.run()
        finally:
            ex.close()
        assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


@pytest.mark.parametrize("flags", [0, L.PA_QF_NO_LANE_HIST])
def test_lane_sum_over_shared_dictionary(flags):
    """SUM over a dictionary every bound segment shares: dictId counts in the workgroup's LDS histogram, values folded in
    once at the end (exact split sums for 64-bit values, here up to 2^40 over ~2^18 docs: past 2^53 in total) — against
    the oracle and against the per-doc gather path (PA_QF_NO_LANE_HIST)."""
    rng = np.random.default_rng(11)
    n = 200_003
    pool_l = np.unique(rng.integers(-(1 << 40), 1 << 40, size=9000))
    pool_d = np.unique(np.round(rng.normal(0, 1e5, size=5000), 3))
    data = {"day": rng.integers(0, 4000, size=n).astype(np.int32), "dl": pool_l[rng.integers(0, len(pool_l), n)],
            "dd": pool_d[rng.integers(0, len(pool_d), n)], "di": rng.integers(-1000, 1000, size=n).astype(np.int32)}
    seg = create_segment("shared", data, {"day": "INT", "dl": "LONG", "dd": "DOUBLE", "di": "INT"})
    g = GpuSegment(seg)
    try:
        # (dense filters take the histogram; a 1 % filter and three histograms at once gather per doc)
        for sql in ("SELECT COUNT(*), SUM(dl), SUM(dd), SUM(di) FROM t WHERE day < 3000",
                    "SELECT SUM(dl), SUM(di) FROM t WHERE day < 3950", "SELECT SUM(dl) FROM t WHERE day < 40",
                    "SELECT SUM(dd), MAX(dl) FROM t"):
            q = parse_sql(sql)
            ex = GpuQueryExecutor(q, [g, g, g], flags=flags)  # three segments, one dictionary per column
            try:
                assert ex.stats()["plan"]["strategy"] == "lane"
                got = ex.run()
            finally:
                ex.close()
            assert_same(got, oracle.run_query(q, [seg, seg, seg]), DOUBLE_REL)
    finally:
        g.close()


GROUP_AGGS = ["COUNT(*), SUM(rs)", "SUM(rl), MIN(rl)", "SUM(rd), MAX(rd), COUNT(*)", "SUM(ri), MIN(rf), MAX(ri)",
              "SUM(dl), SUM(rs)"]


@pytest.mark.parametrize("sel", ["1pct", "30pct", "all"])
@pytest.mark.parametrize("aggs", GROUP_AGGS)
def test_lds_group_by_raw_metrics(lane_segments, sel, aggs):
    """Filter + GROUP BY over raw metrics on the LDS-accumulator strategy, lane-major tiles (pa_scan.h
    accumulate_lds_lm; accumulate_lds_raw_dense when every non-COUNT aggregation reads one raw column and the wave's tile
    is dense): INT / LONG (int32-range: one int64 slot; wider: the split pair) / FLOAT / DOUBLE values and 700 groups.
    PA_QF_NO_DENSE_GROUP keeps the query on the LDS strategy (the planner may otherwise pick the dense GROUP BY kernel,
    tests/test_gpu_dense.py); the default plan is checked against the oracle too."""
    segs, gs = lane_segments
    q = parse_sql("SELECT g, %s FROM t WHERE day < %d GROUP BY g LIMIT 1000" % (aggs, SELECTIVITY[sel]))
    want = oracle.run_query(q, segs)
    for flags in (L.PA_QF_NO_DENSE_GROUP, 0):
        ex = GpuQueryExecutor(q, gs, flags=flags)
        try:
            st = ex.stats()["plan"]
            if flags:
                assert st["strategy"] == "lds" and st["lane_major"] == 1, st
            got = ex.run()
        finally:
            ex.close()
        assert_same(got, want, DOUBLE_REL)


@pytest.mark.parametrize("sel", ["1pct", "30pct", "all"])
@pytest.mark.parametrize("flags", [L.PA_QF_NO_DENSE_GROUP, L.PA_QF_LAZY_POST])
def test_lds_group_by_dictionary_metrics(lane_segments, sel, flags):
    """Filter + GROUP BY over dictionary metrics on the LDS strategy (PA_QF_NO_DENSE_GROUP: not the dense GROUP BY
    kernel), with the post-filter columns staged with the filter column or read per matching doc from HBM
    (PA_QF_LAZY_POST)."""
    segs, gs = lane_segments
    q = parse_sql("SELECT g, COUNT(*), SUM(dl), MIN(dd), MAX(dl), SUM(dd) FROM t WHERE day < %d GROUP BY g LIMIT 1000"
                  % SELECTIVITY[sel])
    ex = GpuQueryExecutor(q, gs, flags=flags)
    try:
        assert ex.stats()["plan"]["strategy"] == "lds"
        got = ex.run()
    finally:
        ex.close()
    assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)
