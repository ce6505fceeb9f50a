"""GPU parity for multi-value columns (through the C-ABI) against the oracle.

Covers: MV filter leaves (MVScanDocIdIterator + applyMV: ANY value for IN / = / ranges, ALL values for NOT IN / <>)
alone and behind single-value clauses (always evaluated lazily, per doc), MV group-by (one key per value, the
cartesian product over several MV columns, duplicates included: DictionaryBasedGroupKeyGenerator.getIntRawKeys),
the *MV aggregations (COUNTMV, SUMMV, MINMV, MAXMV, AVGMV, DISTINCTCOUNTHLLMV), per-segment dictionaries (table-wide
key remap), both tile layouts and both accumulator strategies, numDocsScanned, and the BASELINE configs[4] shape
(raw DOUBLE SUM + DISTINCTCOUNTHLLMV + 4-dim GROUP BY). Bar as in test_gpu_parity: bit-exact except DOUBLE sums
(relative 1e-9).
"""
import ctypes

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.segment import create_segment
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from test_gpu_parity import DOUBLE_REL, run_both

pytestmark = pytest.mark.gpu


def mv_segment(seed, n, mv_cols=(("tags", 30, 4),), sv_cols=(("a", 6), ("b", 50)), raw_double=False, skew=False):
    """SV INT dims, a LONG metric m, MV INT columns (name, cardinality, max values per doc) and optionally a raw
    DOUBLE metric r."""
    rng = np.random.default_rng(seed)
    data, schema = {}, {}
    for name, card in sv_cols:
        data[name] = (rng.integers(0, card, size=n) * 3 + 11).astype(np.int32)
        schema[name] = "INT"
    data["m"] = rng.integers(-5000, 100000, size=n).astype(np.int64)
    schema["m"] = "LONG"
    for name, card, max_len in mv_cols:
        lens = rng.integers(1, max_len + 1, size=n)
        if skew:
            lens[rng.random(n) < 0.7] = 1
        # the cardinality varies with the seed, so segments get different dictionaries (table-wide key remaps)
        data[name] = [(rng.integers(0, card + seed % 3, size=k) * 7 + 100).astype(np.int32) for k in lens]
        schema[name] = "INT"
    no_dict = ()
    if raw_double:
        data["r"] = rng.normal(0, 100, size=n)
        schema["r"] = "DOUBLE"
        no_dict = ("r",)
    return create_segment("mv%d" % seed, data, schema, no_dictionary_columns=no_dict,
                          multi_value_columns=tuple(c[0] for c in mv_cols))


MV_FILTERS = [
    "tags IN (107, 121, 163)",
    "tags NOT IN (107, 121)",
    "tags = 128",
    "tags <> 128",
    "tags BETWEEN 150 AND 240",
    "tags > 250",
    "a = 14 AND tags IN (107, 114)",
    "a = 14 OR tags = 121",
    "NOT (tags IN (107, 114)) AND b < 80",
]


@pytest.mark.parametrize("flt", MV_FILTERS)
def test_mv_filters(flt):
    segs = [mv_segment(1, 20011), mv_segment(2, 4099)]
    run_both("SELECT COUNT(*), SUM(m), MIN(m), MAX(b) FROM t WHERE %s" % flt, segs)
    run_both("SELECT a, COUNT(*), SUM(m) FROM t WHERE %s GROUP BY a LIMIT 100" % flt, segs)


@pytest.mark.parametrize("sql", [
    "SELECT tags, COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t GROUP BY tags LIMIT 1000",
    "SELECT a, tags, COUNT(*), SUM(m), DISTINCTCOUNTHLL(b) FROM t GROUP BY a, tags LIMIT 10000",
    "SELECT tags, a, COUNT(*), SUM(m) FROM t WHERE b > 60 GROUP BY tags, a LIMIT 10000",
    "SELECT tags, tags2, COUNT(*), SUM(m) FROM t GROUP BY tags, tags2 LIMIT 10000",
    "SELECT a, tags2, tags, COUNT(*), MAX(m) FROM t WHERE tags IN (107, 121, 135) GROUP BY a, tags2, tags "
    "LIMIT 10000",
])
def test_mv_group_by(sql):
    mv = (("tags", 30, 4), ("tags2", 9, 3))
    segs = [mv_segment(5, 15013, mv_cols=mv), mv_segment(6, 3001, mv_cols=mv)]
    got, exp, _ = run_both(sql, segs)
    assert got.groups


@pytest.mark.parametrize("sql", [
    "SELECT COUNTMV(tags), SUMMV(tags), MINMV(tags), MAXMV(tags), AVGMV(tags), DISTINCTCOUNTHLLMV(tags), COUNT(*) "
    "FROM t",
    "SELECT COUNTMV(tags), SUMMV(tags), MINMV(tags), MAXMV(tags), AVGMV(tags) FROM t WHERE a = 14 AND b < 70",
    "SELECT a, COUNTMV(tags), SUMMV(tags), MINMV(tags), MAXMV(tags), AVGMV(tags), DISTINCTCOUNTHLLMV(tags) FROM t "
    "GROUP BY a LIMIT 100",
    "SELECT tags, COUNTMV(tags), SUMMV(tags), DISTINCTCOUNTHLLMV(tags) FROM t WHERE b > 40 GROUP BY tags LIMIT 1000",
    "SELECT COUNT(*), SUMMV(tags) FROM t WHERE tags = 999999",
    "SELECT a, DISTINCTCOUNTMV(tags), MINMAXRANGEMV(tags), DISTINCTCOUNT(b), MINMAXRANGE(m) FROM t WHERE b > 20 "
    "GROUP BY a LIMIT 100",
    "SELECT DISTINCTCOUNTMV(tags), MINMAXRANGEMV(tags) FROM t WHERE a = 14",
])
def test_mv_aggregations(sql):
    segs = [mv_segment(7, 12007), mv_segment(8, 2048)]
    run_both(sql, segs)


@pytest.mark.parametrize("flags", [0, L.PA_QF_FORCE_GLOBAL, L.PA_QF_NO_LANE_MAJOR, L.PA_QF_STAGE_ALL,
                                   L.PA_QF_FORCE_LDS, L.PA_QF_NO_LANE_MAJOR | L.PA_QF_FORCE_GLOBAL | L.PA_QF_NO_LAZY])
def test_mv_plan_variants(flags):
    segs = [mv_segment(9, 30011, skew=True), mv_segment(10, 777)]
    for sql in ("SELECT a, tags, COUNT(*), SUM(m), SUMMV(tags) FROM t WHERE b < 100 AND tags NOT IN (107) "
                "GROUP BY a, tags LIMIT 10000",
                "SELECT b, COUNT(*), AVGMV(tags), MAXMV(tags) FROM t WHERE a IN (11, 14) GROUP BY b LIMIT 1000"):
        run_both(sql, segs, flags=flags)


def test_mv_num_docs_scanned_vs_group_counts():
    """With an MV group-by a doc lands in several groups: numDocsScanned counts docs, the group counts key hits."""
    segs = [mv_segment(12, 9001)]
    got, exp, _ = run_both("SELECT tags, COUNT(*) FROM t WHERE a = 14 GROUP BY tags LIMIT 1000", segs)
    assert sum(v[0] for v in got.groups.values()) > got.num_docs_scanned == exp.num_docs_scanned


def test_star_schema_config4_shape():
    """BASELINE configs[4] shape at oracle size: raw (no-dictionary) DOUBLE metric SUM + DISTINCTCOUNTHLLMV over a
    multi-value column, 4-dim GROUP BY."""
    sv = (("d1", 7), ("d2", 5), ("d3", 11), ("d4", 3))
    segs = [mv_segment(20 + i, n, mv_cols=(("tags", 200, 5),), sv_cols=sv, raw_double=True)
            for i, n in enumerate((40009, 17011))]
    run_both("SELECT d1, d2, d3, d4, SUM(r), DISTINCTCOUNTHLLMV(tags), COUNT(*) FROM t WHERE d4 <> 14 "
             "GROUP BY d1, d2, d3, d4 LIMIT 100000", segs, rel=DOUBLE_REL)


@pytest.mark.parametrize("flags,max_len,skew", [(0, 6, False), (L.PA_QF_NO_PARTITION, 6, False),
                                                (L.PA_QF_NO_SPLIT_EMIT, 6, False), (0, 20, False), (0, 24, True)])
def test_star_schema_partitioned_hll(flags, max_len, skew):
    """configs[4] shape over a key space that takes the partitioned path: one record per MV value carries the HLL
    register and rank, COUNT / SUM(r) count each doc once; HLL registers bit-exact, SUM(r) within DOUBLE_REL. Also an SV
    DISTINCTCOUNTHLL and a COUNT-only HLL query. Rows of up to 6 values take the doc-reserved emit path, longer rows
    (up to 20, or skewed: mostly 1 value, some up to 24) the value-parallel one in the same batches; the V and H
    records are emitted by two launches by default, by one with PA_QF_NO_SPLIT_EMIT."""
    sv = (("d1", 64), ("d2", 32), ("d3", 16), ("d4", 8))
    segs = [mv_segment(30 + i, n, mv_cols=(("tags", 300, max_len),), sv_cols=sv, raw_double=True, skew=skew)
            for i, n in enumerate((50021, 20011))]
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        for sql in ("SELECT d1, d2, d3, d4, SUM(r), DISTINCTCOUNTHLLMV(tags), COUNT(*) FROM t GROUP BY d1, d2, d3, d4 "
                    "LIMIT 1000000 OPTION(numGroupsLimit=1000000)",
                    "SELECT d1, d2, d3, d4, DISTINCTCOUNTHLL(m), MAX(m) FROM t GROUP BY d1, d2, d3, d4 "
                    "LIMIT 1000000 OPTION(numGroupsLimit=1000000)",
                    "SELECT d4, d3, d2, d1, DISTINCTCOUNTHLLMV(tags) FROM t GROUP BY d4, d3, d2, d1 "
                    "LIMIT 1000000 OPTION(numGroupsLimit=1000000)"):
            got, exp, _ = run_both(sql, segs, gsegs=gsegs, flags=flags, rel=DOUBLE_REL)
            assert len(got.groups) > 30000
            ex = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags)
            strategy = ex.stats()["plan"]["strategy"]
            ex.close()
            assert strategy == ("global" if flags & L.PA_QF_NO_PARTITION else "partitioned"), (sql, strategy)
    finally:
        for g in gsegs:
            g.close()


@pytest.mark.parametrize("max_len,skew,flags", [(4, False, 0), (20, True, 0), (6, False, L.PA_QF_NO_PARTITION)])
def test_mv_group_by_partitioned(max_len, skew, flags):
    """GROUP BY an MV column over a key space that takes the partitioned path: one V record per (doc, value) pair
    (getIntRawKeys expansion, duplicates included), each carrying the doc's payload — a dictionary LONG (value ids) or
    a raw DOUBLE (64-bit records) — with the MV component least or most significant in the key; a second MV group-by
    column keeps the per-doc global path. Identical to the oracle (DOUBLE sums within DOUBLE_REL)."""
    sv = (("a", 64), ("b", 7))
    segs = [mv_segment(40 + i, n, mv_cols=(("tags", 3000, max_len), ("tags2", 5, 2)), sv_cols=sv, raw_double=True,
                       skew=skew) for i, n in enumerate((60013, 20011))]
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        for sql, part in (
                ("SELECT a, tags, COUNT(*), SUM(r) FROM t GROUP BY a, tags LIMIT 1000000 "
                 "OPTION(numGroupsLimit=1000000)", True),
                ("SELECT tags, a, COUNT(*), SUM(m), MIN(m) FROM t GROUP BY tags, a LIMIT 1000000 "
                 "OPTION(numGroupsLimit=1000000)", True),
                ("SELECT tags, b, COUNT(*) FROM t WHERE a < 60 GROUP BY tags, b LIMIT 1000000 "
                 "OPTION(numGroupsLimit=1000000)", None),
                ("SELECT a, tags, tags2, COUNT(*), MAX(r) FROM t GROUP BY a, tags, tags2 LIMIT 1000000 "
                 "OPTION(numGroupsLimit=1000000)", False)):
            got, exp, _ = run_both(sql, segs, gsegs=gsegs, flags=flags, rel=DOUBLE_REL)
            assert len(got.groups) > 10000
            ex = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags)
            strategy = ex.stats()["plan"]["strategy"]
            ex.close()
            if part is not None:
                assert strategy == ("partitioned" if part and not flags else "global"), (sql, strategy)
    finally:
        for g in gsegs:
            g.close()


def test_malformed_mv_index_rejected():
    """The C-ABI validates the row-start bitmap and chunk offsets of an MV forward index."""
    lib = L.lib()
    seg = mv_segment(30, 5000)
    col = seg.column("tags")
    h = L.check_ptr(lib.pa_segment_create(seg.num_docs), "create")
    dv = np.ascontiguousarray(col.dictionary, dtype=np.int64)
    bad = col.fwd_bytes.copy()
    _, _, boff, _ = col.mv_layout(seg.num_docs)
    bad[boff] ^= 0x40  # flip a row-start bit: one doc more or fewer
    rc = lib.pa_segment_add_mv_dict_column(h, 0, bad.ctypes.data, bad.nbytes, col.num_bits, col.cardinality,
                                           col.total_num_values, L.PA_INT, dv.ctypes.data, None)
    assert rc == -1 and b"MV" in lib.pa_last_error()
    good = np.ascontiguousarray(col.fwd_bytes)
    assert lib.pa_segment_add_mv_dict_column(h, 0, good.ctypes.data, good.nbytes, col.num_bits, col.cardinality,
                                             col.total_num_values, L.PA_INT, dv.ctypes.data, None) == 0
    lib.pa_segment_destroy(h)


@pytest.mark.parametrize("limit", [1, 37, 101, 700])
def test_mv_num_groups_limit_trimming(limit):
    """numGroupsLimit binding inside a doc's key expansion: group ids follow getIntRawKeys order (last group-by
    column first; a later MV column's value index is the more significant digit), so the cut falls between two keys
    of one doc exactly where the reference's IntGroupIdMap would put it. Two MV group-by columns take the sorted form
    (first positions, mode 1); one MV column the walk form (mode 2: a doc-order walk over (doc, value) keys, then
    per-key admission), also with the walk disabled (sorted form) for comparison."""
    from pinot_amd import parse_sql
    from pinot_amd.engine import GpuQueryExecutor, GpuSegment
    mv = (("tags", 30, 4), ("tags2", 9, 3))
    segs = [mv_segment(11, 9001, mv_cols=mv), mv_segment(12, 2500, mv_cols=mv)]
    for sql, mode, flags in (
            ("SELECT a, tags2, tags, COUNT(*), SUM(m), MAX(m) FROM t WHERE b > 10 GROUP BY a, tags2, tags "
             "LIMIT 100000 OPTION(numGroupsLimit=%d)" % limit, 1, 0),
            ("SELECT tags, COUNT(*), SUMMV(tags), DISTINCTCOUNTHLLMV(tags2) FROM t GROUP BY tags LIMIT 100000 "
             "OPTION(numGroupsLimit=%d)" % (limit % 31 + 1), 2, 0),
            ("SELECT a, tags, b, COUNT(*), SUM(m) FROM t WHERE b > 10 GROUP BY a, tags, b LIMIT 100000 "
             "OPTION(numGroupsLimit=%d)" % limit, 2, 0),
            ("SELECT tags, b, COUNT(*), MIN(m) FROM t GROUP BY tags, b LIMIT 100000 "
             "OPTION(numGroupsLimit=%d)" % limit, 2, 0),
            ("SELECT tags, b, COUNT(*), MIN(m) FROM t GROUP BY tags, b LIMIT 100000 "
             "OPTION(numGroupsLimit=%d)" % limit, 1, L.PA_QF_NO_LIMIT_WALK)):
        gsegs = [GpuSegment(s) for s in segs]
        try:
            ex = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags)
            assert ex.stats()["plan"]["limit_trimming"] == mode, sql
            ex.close()
        finally:
            for g in gsegs:
                g.close()
        got, exp, _ = run_both(sql, segs, flags=flags)
        assert got.num_groups_limit_reached


@pytest.mark.parametrize("limit", [5000, 60000])
def test_mv_num_groups_limit_partitioned(limit):
    """The walk form of numGroupsLimit on the partitioned MV path (the mvgroup shape at oracle size: 64 x 3000 keys,
    dense): the count and emit passes admit each (doc, value) record by the segment's bitmap."""
    sv = (("a", 64),)
    segs = [mv_segment(50 + i, n, mv_cols=(("tags", 3000, 5),), sv_cols=sv, raw_double=True)
            for i, n in enumerate((60013, 20011))]
    sql = ("SELECT a, tags, COUNT(*), SUM(r) FROM t GROUP BY a, tags LIMIT 1000000 OPTION(numGroupsLimit=%d)" % limit)
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        got, exp, _ = run_both(sql, segs, gsegs=gsegs, rel=DOUBLE_REL)
        assert got.num_groups_limit_reached
        ex = GpuQueryExecutor(parse_sql(sql), gsegs)
        p = ex.stats()["plan"]
        ex.close()
        assert p["strategy"] == "partitioned" and p["limit_trimming"] == 2, p
    finally:
        for g in gsegs:
            g.close()
