"""Dense filter + GROUP BY on the staged-column kernel (STRAT_GDENSE, pinot_amd/csrc/pa_gdense.h) against the oracle.

The kernel stages every column a query reads (raw metrics too), keeps value dictionaries and group-key remaps in LDS per
segment, and accumulates over the box of group keys the filter admits, with per-lane replicas of each key. The cases
below drive each of its value sources and LDS operations:
  raw INT / LONG (int32 range: one int64 slot; wider: the exact split pair) / FLOAT / DOUBLE metrics;
  dictionary metrics: int32 / int64 / double value tables, the affine shared dictionary (SUM from the dictId sum),
  MIN / MAX on dictIds of a shared sorted dictionary;
  segments with their own dictionaries (group-key remaps and value tables swapped between segments) and one dictionary
  bound three times (one table load per workgroup);
  key boxes from a BETWEEN / IN unit clause on a group-by column (few keys: 8-32 replicas), two group-by columns;
  sparse (lane-major) and dense (step-major) tiles, ragged segments.
Reference semantics: DefaultGroupByExecutor.java:131-158 + {Count,Sum,Min,Max}AggregationFunction.aggregateGroupBySV.
Bars: bit-exact COUNT, integer SUM, MIN, MAX and group keys; DOUBLE SUM within 1e-9 relative (LDS atomic order).
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
    wide = np.unique(rng.integers(-(1 << 40), 1 << 40, size=3000))
    dpool = np.unique(np.round(rng.normal(0, 100, size=3000), 2))
    data = {
        "day": rng.integers(0, 4000, size=n).astype(np.int32),                  # 12-bit filter column
        "g": rng.integers(0, 700, size=n).astype(np.int32),                     # group-by dimension
        "h": rng.integers(0, 5, size=n).astype(np.int32),                       # second group-by dimension
        "w": rng.integers(0, 40, size=n).astype(np.int32),                      # small dimension (key boxes)
        "ri": rng.integers(-(1 << 30), 1 << 30, size=n).astype(np.int32),
        "rl": rng.integers(-(1 << 40), 1 << 40, size=n).astype(np.int64),
        "rs": rng.integers(-(1 << 31), 1 << 31, size=n).astype(np.int64),      # raw LONG in int32 range
        "rf": rng.normal(0, 1e3, size=n).astype(np.float32),
        "rd": rng.normal(0, 1e6, size=n),
        "dl": rng.integers(0, 1 << 12, size=n).astype(np.int64) * 37 - 99999,  # dictionary LONG, int32 values
        "dw": wide[rng.integers(0, len(wide), size=n)],                         # dictionary LONG beyond int32
        "dd": dpool[rng.integers(0, len(dpool), size=n)],                       # dictionary DOUBLE
        "db": np.round(rng.normal(0, 100, size=n), 2),                          # ~50K-value dictionary: no LDS table
        "da": rng.integers(0, 1000, size=n).astype(np.int64) * 3 + 7,           # affine when every value occurs
    }
    schema = {"day": "INT", "g": "INT", "h": "INT", "w": "INT", "ri": "INT", "rl": "LONG", "rs": "LONG", "rf": "FLOAT",
              "rd": "DOUBLE", "dl": "LONG", "dw": "LONG", "dd": "DOUBLE", "da": "LONG",
              "db": "DOUBLE"}
    return create_segment("dense%d" % seed, data, schema, no_dictionary_columns=("ri", "rl", "rs", "rf", "rd"))


@pytest.fixture(scope="module")
def own_dicts():
    """Three segments with their own dictionaries (remaps, per-segment value tables); ragged sizes."""
    segs = [_segment(1, 300_001), _segment(2, 65_536), _segment(3, 2049)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


@pytest.fixture(scope="module")
def shared_dict():
    """One segment bound three times: every dictionary shared (affine / dictId MIN-MAX paths, one table load)."""
    seg = _segment(7, 200_003)
    g = GpuSegment(seg)
    yield [seg, seg, seg], [g, g, g]
    g.close()


# day < hi keeps ~hi/4000 of the docs: 30 % -> sparse tiles (lane-major walk, below kGdDenseMin matches per tile), all ->
# dense tiles (step-major); 5 % takes the dense kernel only when the post-filter columns are narrow (staging break-even)
SELECTIVITY = {"5pct": 200, "30pct": 1200, "all": 4000}
AGGS = [
    "COUNT(*), SUM(rs), MAX(rs), SUM(ri)",
    "SUM(rl), MIN(rl)",
    "SUM(rd), MIN(rf), MAX(rf)",
    "COUNT(*), SUM(dl), MIN(dl), MAX(dd)",
    "SUM(dw), MAX(dw), SUM(dd)",
    "SUM(da), MIN(da), MAX(rd)",
]


def _run(q, gs, flags=0, expect_dense=True):
    ex = GpuQueryExecutor(q, gs, flags=flags)
    try:
        st = ex.stats()["plan"]
        if expect_dense is not None:
            assert (st["strategy"] == "lds_dense") == expect_dense, st
        return ex.run()
    finally:
        ex.close()


@pytest.mark.parametrize("sel", list(SELECTIVITY))
@pytest.mark.parametrize("aggs", AGGS)
@pytest.mark.parametrize("dicts", ["own", "shared"])
def test_dense_group_by(own_dicts, shared_dict, dicts, sel, aggs):
    segs, gs = own_dicts if dicts == "own" else shared_dict
    q = parse_sql("SELECT g, %s FROM t WHERE day < %d GROUP BY g LIMIT 1000" % (aggs, SELECTIVITY[sel]))
    got = _run(q, gs, expect_dense=None if sel == "5pct" else True)
    assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


@pytest.mark.parametrize("dicts", ["own", "shared"])
def test_dense_key_boxes(own_dicts, shared_dict, dicts):
    """Key boxes from unit clauses on group-by columns: 3 keys (32 replicas), 16 (8 replicas), a 2-column box (4
    replicas), an IN list, and a box whose filter column is the group-by column itself (the configs[0] shape)."""
    segs, gs = own_dicts if dicts == "own" else shared_dict
    for sql in (
            "SELECT h, COUNT(*), SUM(dl), SUM(rs) FROM t WHERE h BETWEEN 1 AND 3 GROUP BY h",
            "SELECT w, COUNT(*), SUM(ri), MIN(dd) FROM t WHERE w BETWEEN 10 AND 25 GROUP BY w",
            "SELECT w, h, COUNT(*), SUM(ri) FROM t WHERE w BETWEEN 10 AND 17 AND day < 3000 GROUP BY w, h",
            "SELECT h, w, MAX(rl) FROM t WHERE w IN (3, 17, 20, 21, 30) AND day >= 100 GROUP BY h, w",
            "SELECT day, SUM(da), MAX(dw) FROM t WHERE day BETWEEN 1500 AND 2500 GROUP BY day LIMIT 2000"):
        q = parse_sql(sql)
        got = _run(q, gs)
        assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


def test_dense_no_filter_and_agrees_with_lds_path(own_dicts):
    """No filter at all (every doc), and the same results as the LDS strategy (PA_QF_NO_DENSE_GROUP)."""
    segs, gs = own_dicts
    for sql in ("SELECT g, COUNT(*), SUM(rl), MAX(dl) FROM t GROUP BY g LIMIT 1000",
                "SELECT h, SUM(dw), SUM(rs) FROM t WHERE day < 2000 GROUP BY h"):
        q = parse_sql(sql)
        got = _run(q, gs)
        ref = _run(q, gs, flags=L.PA_QF_NO_DENSE_GROUP, expect_dense=False)
        assert_same(got, ref, DOUBLE_REL)
        assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


def test_dense_not_chosen_for_sparse_or_wide(own_dicts):
    """A filter keeping ~0.03 % of the docs reads post-filter columns per doc (LDS strategy); a group-by column without a
    dictionary, a key box over kGdMaxKeys keys or a value dictionary too large for LDS leave the dense kernel too — and
    the results still match."""
    segs, gs = own_dicts
    for sql, dense in (("SELECT g, SUM(rl) FROM t WHERE day = 17 GROUP BY g LIMIT 1000", False),
                       ("SELECT ri, COUNT(*) FROM t WHERE day < 10 GROUP BY ri LIMIT 100000", False),
                       ("SELECT g, day, COUNT(*) FROM t WHERE day < 3000 GROUP BY g, day LIMIT 3000000 "
                        "OPTION(numGroupsLimit=3000000)", False),
                       ("SELECT g, SUM(db) FROM t WHERE day < 2000 GROUP BY g LIMIT 1000", False),
                       ("SELECT g, SUM(rl) FROM t WHERE day < 2000 GROUP BY g LIMIT 1000", True)):
        q = parse_sql(sql)
        got = _run(q, gs, expect_dense=dense)
        assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


@pytest.mark.parametrize("flags", [0, L.PA_QF_BOX_FILTER, L.PA_QF_NO_BOX_FILTER, L.PA_QF_BOX_FILTER | L.PA_QF_NO_REG_STAGE])
@pytest.mark.parametrize("dicts", ["own", "shared"])
def test_dense_box_filter(own_dicts, shared_dict, dicts, flags):
    """The key box as the filter (unit range clauses on group-by columns only: every doc box-checked, no filter pass,
    no walk), forced at any selectivity, disabled, and automatic; filters the box does not capture exactly (a second
    column, disjoint or empty ranges) keep the filter path. Groups and numDocsScanned identical to the oracle."""
    segs, gs = own_dicts if dicts == "own" else shared_dict
    for sql in (
            "SELECT day, COUNT(*), SUM(dl), MAX(rd) FROM t WHERE day BETWEEN 1500 AND 2500 GROUP BY day LIMIT 2000",
            "SELECT day, COUNT(*), SUM(da), MIN(rl) FROM t WHERE day >= 3900 GROUP BY day LIMIT 2000",
            "SELECT w, h, COUNT(*), SUM(ri), SUM(dd) FROM t WHERE w BETWEEN 10 AND 17 AND h >= 2 GROUP BY w, h",
            "SELECT w, SUM(rs), MAX(dw) FROM t WHERE w > 5 AND w < 30 AND w <= 20 GROUP BY w",
            "SELECT w, COUNT(*) FROM t WHERE w > 30 AND w < 10 GROUP BY w",
            "SELECT w, COUNT(*), SUM(ri) FROM t WHERE w BETWEEN 10 AND 12 AND day < 3000 GROUP BY w",
            "SELECT w, h, COUNT(*) FROM t WHERE w BETWEEN 100 AND 200 GROUP BY w, h"):
        q = parse_sql(sql)
        got = _run(q, gs, flags=flags, expect_dense=None)
        assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)


PACKABLE = (
    # COUNT + two SUMs whose terms fit one word: dl's values as offsets from their minimum (negative values), da's
    # dictIds (affine shared dictionary) or offsets (own dictionaries)
    "SELECT g, COUNT(*), SUM(dl), SUM(da) FROM t WHERE day < 1200 GROUP BY g LIMIT 1000",
    "SELECT h, w, SUM(dl) FROM t WHERE w BETWEEN 10 AND 25 AND day >= 100 GROUP BY h, w",
    "SELECT g, COUNT(*) FROM t WHERE day < 2000 GROUP BY g LIMIT 1000",
    "SELECT day, SUM(da) FROM t WHERE day BETWEEN 1500 AND 2500 GROUP BY day LIMIT 2000",
)
NOT_PACKABLE = (
    "SELECT g, SUM(dw), SUM(da) FROM t WHERE day < 1200 GROUP BY g LIMIT 1000",   # dw spans 2^41: no field fits
    "SELECT g, COUNT(*), MIN(dl), SUM(rs) FROM t WHERE day < 3000 GROUP BY g LIMIT 1000",
)


@pytest.mark.parametrize("flags", [0, L.PA_QF_GD_DRAIN_EACH_TILE, L.PA_QF_NO_JIT, L.PA_QF_NO_JIT | L.PA_QF_GD_DRAIN_EACH_TILE,
                                   L.PA_QF_NO_GD_PACK, L.PA_QF_NO_GDENSE_LM])
@pytest.mark.parametrize("dicts", ["own", "shared"])
def test_dense_lane_major_walk(own_dicts, shared_dict, dicts, flags):
    """The lane-major walk (STRAT_GDENSE_LM*: each lane unpacks its 16 docs of every column) with packed accumulation
    (one word per matching doc: COUNT + SUM terms, drained per wave; drained after every tile to exercise the drain),
    with one atomic per aggregation, and the step-major kernels (PA_QF_NO_GDENSE_LM): identical to the oracle."""
    segs, gs = own_dicts if dicts == "own" else shared_dict
    lm = not (flags & L.PA_QF_NO_GDENSE_LM)
    packed_runs = lm_runs = jit_runs = 0
    for sql, packable in [(x, True) for x in PACKABLE] + [(x, False) for x in NOT_PACKABLE]:
        q = parse_sql(sql)
        ex = GpuQueryExecutor(q, gs, flags=flags)
        try:
            st = ex.stats()["plan"]
            assert st["strategy"] == "lds_dense", (sql, st)
            # (a wide raw column can leave no room for two images per wave: a step-major variant then runs)
            if not lm:
                assert not st["variant"].startswith("gdense_lm"), (sql, st)
            lm_runs += st["variant"].startswith("gdense_lm")
            # (a packable query runs unpacked when the waves' packed rows do not fit LDS beside its tables)
            if not (lm and packable and not (flags & L.PA_QF_NO_GD_PACK)):
                assert st["dense_packed"] == 0, (sql, st)
            packed_runs += st["dense_packed"] > 0
            # (the kernel specialised to the query's shape: never under PA_QF_NO_JIT)
            if flags & L.PA_QF_NO_JIT:
                assert st["dense_packed"] != 2, (sql, st)
            jit_runs += st["dense_packed"] == 2
            got = ex.run()
        finally:
            ex.close()
        assert_same(got, oracle.run_query(q, segs), DOUBLE_REL)
    if lm:
        assert lm_runs >= 4
    if lm and not (flags & L.PA_QF_NO_GD_PACK):
        assert packed_runs >= 2
        if not flags & L.PA_QF_NO_JIT:  # (own dictionaries too: width classes, remaps, per-segment tables)
            assert jit_runs >= 3, jit_runs
