"""GPU parity: the HIP path (through the C-ABI) against the oracle and the reference's golden results.

Bar: bit-exact for COUNT, integer/long SUM (exact int64 accumulation == the reference's double accumulation while
partial sums stay below 2^53, true for every case here), MIN/MAX, group keys and HLL registers; DOUBLE/FLOAT sums
within a relative tolerance of 1e-9 (summation order differs from the reference's docId order).
"""
import ctypes

import numpy as np
import pytest

import oracle
from conftest import golden_rows, rows_match
from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd.engine import AvgPair, GpuQueryExecutor, GpuSegment, MinMaxRangePair
from pinot_amd.hll import HyperLogLog
from pinot_amd.reduce import final_result_table, merge_intermediate, server_trim
from synth import make_segment

pytestmark = pytest.mark.gpu

DOUBLE_REL = 1e-9


def _close(a, b, rel):
    if isinstance(b, HyperLogLog):
        return isinstance(a, HyperLogLog) and a == b
    if isinstance(b, set):  # DISTINCTCOUNT value sets: exact
        return isinstance(a, set) and a == b
    if isinstance(b, MinMaxRangePair):
        return _close(a.min, b.min, rel) and _close(a.max, b.max, rel)
    if isinstance(b, AvgPair):
        return a.count == b.count and _close(a.sum, b.sum, rel)
    if isinstance(b, int) and not isinstance(b, bool):
        return a == b
    a, b = float(a), float(b)
    if a == b:
        return True
    if np.isinf(b) or np.isinf(a):
        return False
    return rel > 0 and abs(a - b) <= rel * max(abs(b), 1.0)


def assert_same(gpu, ora, rel=0.0):
    assert gpu.num_docs_scanned == ora.num_docs_scanned
    assert gpu.num_groups_limit_reached == ora.num_groups_limit_reached
    if ora.group_by:
        assert set(gpu.groups) == set(ora.groups), (sorted(set(gpu.groups) ^ set(ora.groups))[:5])
        for k, vals in ora.groups.items():
            for a, b in zip(gpu.groups[k], vals):
                assert _close(a, b, rel), (k, a, b)
    else:
        for a, b in zip(gpu.row, ora.row):
            assert _close(a, b, rel), (a, b)


def run_both(sql, segments, gsegs=None, flags=0, rel=0.0):
    q = parse_sql(sql)
    own = gsegs is None
    if own:
        gsegs = [GpuSegment(s) for s in segments]
    ex = GpuQueryExecutor(q, gsegs, flags=flags)
    try:
        got = ex.run()
    finally:
        ex.close()
        if own:
            for g in gsegs:
                g.close()
    exp = oracle.run_query(q, segments)
    assert_same(got, exp, rel)
    return got, exp, ex


# ------------------------------------------------------------------ reference golden results on the GPU
def test_golden_cases_gpu(golden_spec, golden_segment):
    g = GpuSegment(golden_segment)
    failures = []
    try:
        for case in golden_spec["cases"]:
            q = parse_sql(case["sql"])
            ex = GpuQueryExecutor(q, [g, g])  # one server = 2 copies of the segment
            ex.execute()
            server = ex.fetch(execution_stats=True)  # + the DataTable statistics (GPU leaf bitmaps)
            ex.close()
            exp = oracle.run_query(q, [golden_segment] * 2)
            assert_same(server, exp)
            broker = merge_intermediate([server_trim(server, q)] * 2)
            got = final_result_table(broker, q)
            if case["rows"] is not None and not rows_match(golden_rows(got, case), case["rows"], case["delta"]):
                failures.append((case["source"], got[:3], case["rows"][:3]))
            if "limit_reached" in case and broker.num_groups_limit_reached != case["limit_reached"]:
                failures.append((case["source"], "numGroupsLimitReached", broker.num_groups_limit_reached))
            # testInterSegmentsResult: numDocsScanned, numEntriesScannedInFilter, numEntriesScannedPostFilter,
            # numTotalDocs summed over the broker's servers
            stats = [broker.num_docs_scanned, broker.num_entries_scanned_in_filter,
                     broker.num_entries_scanned_post_filter, broker.num_total_docs]
            if case["stats"] is not None and stats != case["stats"]:
                failures.append((case["source"], "stats", stats, case["stats"]))
    finally:
        g.close()
    assert not failures, failures


def test_query_executor_cases_gpu(query_executor_spec, query_executor_segments):
    """QueryExecutorTest.java:152-190 on the GPU: one server of 2 x simpleData200001 + 2 empty segments; the
    AggregationResultsBlock value (COUNT long, SUM/MIN/MAX double) and numDocsScanned."""
    gs = [GpuSegment(s) for s in query_executor_segments]
    try:
        for case in query_executor_spec["cases"]:
            ex = GpuQueryExecutor(parse_sql(case["sql"]), gs)
            res = ex.run()
            ex.close()
            assert res.row[0] == case["value"] and type(res.row[0]) is type(case["value"]), (case["source"], res.row)
            assert res.num_docs_scanned == 400002 and res.num_total_docs == 400002
        # only the empty segments: the aggregation functions' empty results, as the oracle gives them
        q = parse_sql("SELECT COUNT(*), SUM(met), MIN(met), MAX(met) FROM testTable_OFFLINE")
        ex = GpuQueryExecutor(q, gs[2:])
        res = ex.run()
        ex.close()
        exp = oracle.run_query(q, query_executor_segments[2:])
        assert res.row == exp.row and res.num_docs_scanned == 0, (res.row, exp.row)
    finally:
        for g in gs:
            g.close()


# ------------------------------------------------------------------ randomized parity vs the oracle
COLS = {"d1": ("INT", 50), "d2": ("STRING", 20), "d3": ("LONG", 3000), "m1": ("INT", 500), "m2": ("LONG", 10000),
        "f1": ("DOUBLE", 200), "f2": ("FLOAT", 300), "r1": ("DOUBLE", 0), "r2": ("INT", 0), "r3": ("LONG", 0)}
RAW = ("r1", "r2", "r3")

QUERIES = [
    "SELECT COUNT(*), SUM(m1), SUM(m2), MIN(m1), MAX(m2) FROM t",
    "SELECT COUNT(*), SUM(m1) FROM t WHERE d1 BETWEEN {d1a} AND {d1b}",
    "SELECT COUNT(*), SUM(m2), MIN(d3), MAX(d3) FROM t WHERE d3 > {d3a} AND d2 IN ('s00003_xxx', 's00007_', 's00011_xxxx')",
    "SELECT d1, COUNT(*), SUM(m1), SUM(m2), MIN(m1), MAX(m1) FROM t GROUP BY d1 ORDER BY d1 LIMIT 100",
    "SELECT d1, d2, COUNT(*), SUM(m2), AVG(m1) FROM t WHERE d3 <= {d3a} OR d2 NOT IN ('s00001_x', 's00002_xx') "
    "GROUP BY d1, d2 LIMIT 2000",
    "SELECT d2, DISTINCTCOUNTHLL(m2), DISTINCTCOUNTHLL(d2), DISTINCTCOUNTHLL(f1) FROM t GROUP BY d2 LIMIT 100",
    "SELECT DISTINCTCOUNTHLL(d3), DISTINCTCOUNTHLL(m1, 10), DISTINCTCOUNTHLL(r2), DISTINCTCOUNTHLL(r1) FROM t "
    "WHERE NOT (d1 < {d1a})",
    "SELECT d1, SUM(f1), MIN(f1), MAX(f2), SUM(r1), MIN(r1), MAX(r3), SUM(r2) FROM t GROUP BY d1 LIMIT 100",
    "SELECT COUNT(*), SUM(r1), MAX(r2) FROM t WHERE r2 > 100 AND r1 <= 50.5",
    "SELECT d3, COUNT(*) FROM t WHERE r3 IN (5, 7, 11, -3) OR d1 = {d1a} GROUP BY d3 LIMIT 5000",
    "SELECT COUNT(*) FROM t WHERE d1 != {d1a} AND NOT (d2 = 's00004_xxxx' OR m1 >= {m1a})",
    "SELECT d1, d2, d3, COUNT(*), SUM(m1) FROM t WHERE f1 < 0 GROUP BY d1, d2, d3 LIMIT 100000 "
    "OPTION(numGroupsLimit=1000000)",
    # exact DISTINCTCOUNT (per-group value presence over the table-wide value dictionary) and MINMAXRANGE
    "SELECT d1, MINMAXRANGE(m1), DISTINCTCOUNT(d3), DISTINCTCOUNT(d2), MINMAXRANGE(f2), COUNT(*) FROM t "
    "WHERE d3 > {d3a} GROUP BY d1 LIMIT 100",
    "SELECT MINMAXRANGE(f1), MINMAXRANGE(m2), DISTINCTCOUNT(m1), DISTINCTCOUNT(f2), DISTINCTCOUNT(d2) FROM t "
    "WHERE d2 NOT IN ('s00001_x') OR m1 < {m1a}",
]


def _fill(sql, seg):
    vals = {}
    for c in ("d1", "d3", "m1"):
        d = seg.column(c).dictionary
        vals[c + "a"] = int(d[len(d) // 3])
        vals[c + "b"] = int(d[(2 * len(d)) // 3])
    return sql.format(**vals)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_random_queries(seed, qi):
    sizes = [(20011, 5000), (8191, 70001), (1, 2049)][seed - 1]
    segs = [make_segment(seed * 100 + i, n, COLS, no_dict=RAW) for i, n in enumerate(sizes)]
    sql = _fill(QUERIES[qi], segs[0])
    rel = DOUBLE_REL if any(c in sql for c in ("f1", "f2", "r1")) else 0.0
    run_both(sql, segs, rel=rel)


@pytest.mark.parametrize("flags", [L.PA_QF_FORCE_GLOBAL, L.PA_QF_STAGE_ALL, L.PA_QF_FORCE_GLOBAL | L.PA_QF_STAGE_ALL,
                                   L.PA_QF_NO_LANE_MAJOR, L.PA_QF_NO_LANE_MAJOR | L.PA_QF_FORCE_GLOBAL,
                                   L.PA_QF_NO_LANE_MAJOR | L.PA_QF_STAGE_ALL | L.PA_QF_NO_LAZY, L.PA_QF_NO_LANE_ACC,
                                   L.PA_QF_NO_LANE_ACC | L.PA_QF_NO_LANE_MAJOR])
def test_strategies_agree(flags):
    """LDS-privatised vs global accumulators, staged vs lazy post-filter columns, lane-major vs step-major tiles:
    identical results."""
    segs = [make_segment(11 + i, n, COLS, no_dict=RAW) for i, n in enumerate((30001, 4096))]
    for sql in QUERIES[:8]:
        sql = _fill(sql, segs[0])
        rel = DOUBLE_REL if any(c in sql for c in ("f1", "f2", "r1")) else 0.0
        run_both(sql, segs, flags=flags, rel=rel)


LAZY_QUERIES = [
    # the headline shape: a very selective clause leads, the day range is evaluated lazily on its survivors
    "SELECT day, SUM(clicks), SUM(imps), COUNT(*) FROM t WHERE day BETWEEN {da} AND {db} AND acct IN ({acct}) "
    "GROUP BY day LIMIT 1000",
    "SELECT COUNT(*), SUM(clicks), MIN(imps), MAX(day) FROM t WHERE acct = {acct0} AND (day < {da} OR imps > {ia}) "
    "AND NOT (clicks = {c0})",
    "SELECT day, COUNT(*), DISTINCTCOUNTHLL(clicks) FROM t WHERE acct IN ({acct}) AND r1 < 0.5 GROUP BY day "
    "LIMIT 1000",
    "SELECT COUNT(*), SUM(r1) FROM t WHERE acct NOT IN ({acct}) AND day = {da}",
]


@pytest.mark.parametrize("flags", [0, L.PA_QF_NO_LAZY, L.PA_QF_FORCE_LDS, L.PA_QF_STAGE_ALL,
                                   (4 << L.PA_QF_WG_SHIFT) | (2 << L.PA_QF_RING_SHIFT) | L.PA_QF_STEPS16,
                                   L.PA_QF_NO_LANE_MAJOR, L.PA_QF_NO_LANE_MAJOR | L.PA_QF_NO_LAZY,
                                   (2 << L.PA_QF_WG_SHIFT) | (3 << L.PA_QF_RING_SHIFT)])
def test_lazy_clauses(flags):
    """Late materialisation: clauses behind a very selective lead clause run only on its survivors, from HBM.
    Every plan variant must return the oracle's result; the default plan must actually defer clauses."""
    cols = {"day": ("INT", 512), "acct": ("INT", 50000), "clicks": ("LONG", 1000), "imps": ("LONG", 9000),
            "r1": ("DOUBLE", 0)}
    # even seeds: uniform (unskewed) values, so the dictId-fraction estimate holds and the lead clause is lazy-worthy
    segs = [make_segment(42 + 2 * i, n, cols, no_dict=("r1",)) for i, n in enumerate((300007, 65536, 5000))]
    d = segs[0].column("day").dictionary
    a = segs[0].column("acct").dictionary
    vals = {"da": int(d[100]), "db": int(d[300]), "acct0": int(a[7]), "acct": ", ".join(str(int(v)) for v in a[5:9]),
            "ia": int(segs[0].column("imps").dictionary[4000]), "c0": int(segs[0].column("clicks").dictionary[3])}
    gsegs = [GpuSegment(s) for s in segs]
    try:
        for sql in LAZY_QUERIES:
            sql = sql.format(**vals)
            _, _, ex = run_both(sql, segs, gsegs=gsegs, flags=flags, rel=DOUBLE_REL if "r1" in sql else 0.0)
        if flags == 0:
            ex = GpuQueryExecutor(parse_sql(LAZY_QUERIES[0].format(**vals)), gsegs)
            st = ex.stats()
            lm = L.lib().pa_query_lane_major(ex.handle)
            ex.close()
            assert st["plan"]["eager_literals"] == 1, st
            assert lm == 1, "the headline shape must run the lane-major kernel"
    finally:
        for g in gsegs:
            g.close()


@pytest.mark.parametrize("n", [1, 63, 64, 65, 2047, 2048, 2049, 4095, 4097, 100003])
def test_ragged_segment_sizes(n):
    cols = {"a": ("INT", 37), "b": ("LONG", 1500), "m": ("LONG", 777)}
    seg = make_segment(n, n, cols)
    run_both("SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE b > %d" % int(seg.column("b").dictionary[0]), [seg])
    run_both("SELECT a, COUNT(*), SUM(m), MAX(b) FROM t GROUP BY a LIMIT 100", [seg])


def test_empty_and_no_match():
    """Zero-doc segment and a filter matching nothing: aggregation-only returns COUNT 0, SUM 0.0,
    MIN +inf, MAX -inf (Min/MaxAggregationFunction DEFAULT_VALUE) and an empty HLL."""
    cols = {"a": ("INT", 10), "m": ("LONG", 50)}
    seg = make_segment(6, 1000, cols)
    got, _, _ = run_both("SELECT COUNT(*), SUM(m), MIN(m), MAX(m), DISTINCTCOUNTHLL(m) FROM t WHERE a > 2147483000",
                         [seg])
    assert got.row[0] == 0 and got.row[1] == 0.0 and got.row[2] == np.inf and got.row[3] == -np.inf
    assert got.row[4].cardinality() == 0
    got, _, _ = run_both("SELECT a, COUNT(*) FROM t WHERE a > 2147483000 GROUP BY a", [seg])
    assert got.groups == {}


def test_zero_doc_segment_in_set():
    from pinot_amd.segment import Segment, build_column
    cols = {"a": ("INT", 10), "m": ("LONG", 50)}
    seg = make_segment(7, 5000, cols)
    z = Segment("empty", 0)
    for c, (dt, _) in cols.items():
        col = build_column(c, seg.column(c).dictionary[:1], dt)  # one-value dictionary, no docs
        col.fwd_bytes = np.zeros(0, dtype=np.uint8)
        z.columns[c] = col
    run_both("SELECT a, COUNT(*), SUM(m) FROM t GROUP BY a", [z, seg, z])


def test_different_dictionaries_remap():
    """Segments with different dictionaries: group keys merge by value (GroupByCombineOperator semantics)."""
    cols = {"k1": ("INT", 40), "k2": ("STRING", 15), "m": ("INT", 100)}
    segs = [make_segment(s, 7000 + s, cols) for s in (21, 22, 23, 24)]
    run_both("SELECT k1, k2, COUNT(*), SUM(m), MIN(m), DISTINCTCOUNTHLL(m) FROM t GROUP BY k1, k2 LIMIT 10000", segs)
    # DISTINCTCOUNT over per-segment dictionaries: segment dictIds remapped to the table-wide value ids
    run_both("SELECT k1, DISTINCTCOUNT(m), DISTINCTCOUNT(k2), MINMAXRANGE(m) FROM t GROUP BY k1 LIMIT 10000", segs)
    run_both("SELECT DISTINCTCOUNT(m), DISTINCTCOUNT(k2) FROM t WHERE k1 > 0", segs)


def test_long_sum_beyond_2_53():
    """Past 2^53 the reference's docId-order double accumulation rounds; the GPU's exact int64 sum converted once
    is the correctly rounded value. Agreement is then within the reference's own rounding error (n ulps)."""
    from pinot_amd.segment import create_segment
    rng = np.random.default_rng(5)
    n = 50000
    vals = rng.integers(1 << 60, (1 << 61), size=n, dtype=np.int64)
    seg = create_segment("big", {"m": vals, "k": rng.integers(0, 4, size=n).astype(np.int32)},
                         {"m": "LONG", "k": "INT"})
    run_both("SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t", [seg], rel=1e-12)
    run_both("SELECT k, SUM(m) FROM t GROUP BY k", [seg], rel=1e-12)
    exact = int(vals.astype(object).sum())
    q = parse_sql("SELECT SUM(m) FROM t")
    g = GpuSegment(seg)
    ex = GpuQueryExecutor(q, [g])
    assert ex.run().row[0] == float(exact)
    ex.close()
    g.close()


def test_high_cardinality_global_fallback():
    """~1M-key space (LDS cannot hold it): global-memory accumulators."""
    cols = {"k1": ("INT", 1000), "k2": ("LONG", 1000), "m": ("LONG", 5000)}
    seg = make_segment(30, 300000, cols)
    got, exp, ex = run_both("SELECT k1, k2, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t GROUP BY k1, k2 LIMIT 1000000 "
                            "OPTION(numGroupsLimit=2000000)", [seg])
    assert len(got.groups) > 100000


def test_large_fetch_hll_registers_and_count_probe():
    """Accumulator block > 1 MiB with HLL registers: GPU compaction narrows registers to bytes, the host copies them
    as-is; >65536 keys makes fetch_arrays probe the group count first (capacity-0 call). Registers bit-exact."""
    cols = {"k1": ("INT", 300), "k2": ("INT", 400), "v": ("LONG", 70000), "m": ("LONG", 100)}
    seg = make_segment(31, 200000, cols)
    got, exp, _ = run_both("SELECT k1, k2, COUNT(*), DISTINCTCOUNTHLL(v), SUM(m) FROM t GROUP BY k1, k2 "
                           "LIMIT 1000000 OPTION(numGroupsLimit=2000000)", [seg])
    assert len(got.groups) > 20000  # synth draws skewed dictIds; the key space is 120000 (> 65536: probe)
    gs = [GpuSegment(seg)]
    ex = GpuQueryExecutor(parse_sql("SELECT k1, COUNT(*), DISTINCTCOUNTHLL(v, 12) FROM t WHERE k2 < 100 GROUP BY k1"),
                          gs)
    ex.execute()
    keys, counts, outs = ex.fetch_arrays()
    hi = [i for i, a in enumerate(ex.pa_aggs) if a[0] == L.PA_AGG_DISTINCTCOUNTHLL][0]
    assert outs[hi].dtype == np.uint8 and len(outs[hi]) == len(keys) << 12
    ora = oracle.run_query(ex.query, [seg])
    assert len(keys) == len(ora.groups)
    ex.close()
    gs[0].close()


@pytest.mark.parametrize("flags", [0, L.PA_QF_NO_LANE_MAJOR, L.PA_QF_NO_PARTITION, L.PA_QF_STAGE_ALL,
                                   1 << L.PA_QF_PART_SHIFT, 2 << L.PA_QF_PART_SHIFT,
                                   3 << L.PA_QF_PART_SHIFT | 1 << L.PA_QF_WG_SHIFT])
def test_partitioned_aggregation(flags):
    """High-cardinality dense GROUP BY (BASELINE configs[2] shape): records partitioned by key range, aggregated per
    partition in LDS. INT / LONG (beyond int32) / DOUBLE / FLOAT values, SUM MIN MAX AVG, with and without a filter,
    several segments with different dictionaries; identical to the oracle and to the per-doc atomic path."""
    cols = {"k1": ("INT", 700), "k2": ("LONG", 900), "m": ("INT", 5000), "big": ("LONG", 3000), "f": ("DOUBLE", 800),
            "g": ("FLOAT", 600)}
    segs = [make_segment(70 + i, n, cols) for i, n in enumerate((120011, 40009))]
    # (the second query's records carry three 64-bit payloads over a 2.5M-key space: their LDS bins may not fit next
    # to the tile ring, and then the per-doc global-atomic path runs it — same results either way)
    queries = [
        ("SELECT k1, k2, COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t GROUP BY k1, k2 LIMIT 1000000 "
         "OPTION(numGroupsLimit=2000000)", True),
        ("SELECT k2, k1, SUM(big), MIN(big), MAX(f), SUM(f), MIN(g) FROM t WHERE m > {m} GROUP BY k2, k1 "
         "LIMIT 1000000 OPTION(numGroupsLimit=2000000)", False),
        ("SELECT k1, k2, COUNT(*) FROM t GROUP BY k1, k2 LIMIT 1000000 OPTION(numGroupsLimit=2000000)", True),
        # one 64-bit payload (value ids, negative values): pass C's one-int64 SUM when the partition bounds it
        ("SELECT k1, k2, SUM(big), MIN(big), MAX(big) FROM t GROUP BY k1, k2 LIMIT 1000000 "
         "OPTION(numGroupsLimit=2000000)", True),
    ]
    mv = int(segs[0].column("m").dictionary[len(segs[0].column("m").dictionary) // 4])
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        for sql, must in queries:
            sql = sql.format(m=mv)
            got, exp, _ = run_both(sql, segs, gsegs=gsegs, flags=flags, rel=DOUBLE_REL)
            assert len(got.groups) > 50000
            ex = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags)
            strategy = ex.stats()["plan"]["strategy"]
            ex.close()
            if flags & L.PA_QF_NO_PARTITION:
                assert strategy == "global", strategy
            elif must and not flags & (3 << L.PA_QF_PART_SHIFT):  # (smaller partitions may not fit the bins' LDS)
                assert strategy == "partitioned", strategy
    finally:
        for g in gsegs:
            g.close()


def test_partitioned_generic_records():
    """V records with several payloads (V_FMT_GEN: LONG beyond int32, DOUBLE, FLOAT widened to double) over one shared
    table-wide key space small enough for the emit pass's bins; identical to the oracle."""
    cols = {"k1": ("INT", 400), "k2": ("INT", 300), "big": ("LONG", 3000), "f": ("DOUBLE", 800), "g": ("FLOAT", 600)}
    base = make_segment(77, 150011, cols)
    segs = [base, base]  # one dictionary per column: the key space stays 400 x 300
    sql = ("SELECT k2, k1, COUNT(*), SUM(big), MIN(big), MAX(f), SUM(f), MIN(g) FROM t GROUP BY k2, k1 "
           "LIMIT 1000000 OPTION(numGroupsLimit=2000000)")
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        got, exp, _ = run_both(sql, segs, gsegs=gsegs, rel=DOUBLE_REL)
        ex = GpuQueryExecutor(parse_sql(sql), gsegs)
        strategy = ex.stats()["plan"]["strategy"]
        ex.close()
        assert strategy == "partitioned", strategy
        assert len(got.groups) > 10000
    finally:
        for g in gsegs:
            g.close()


def test_partitioned_raw_values():
    """Partitioned aggregation with raw (no-dictionary) value columns: INT and LONG (32/64-bit record payloads), DOUBLE
    (bits), FLOAT (widened: generic emit), 4 group-by columns, a value column dictionary-encoded in one segment and raw
    in the other; identical to the oracle (DOUBLE sums within DOUBLE_REL)."""
    cols = {"k1": ("INT", 40), "k2": ("INT", 30), "k3": ("LONG", 20), "k4": ("INT", 16), "ri": ("INT", 500),
            "rl": ("LONG", 0), "rd": ("DOUBLE", 0), "rf": ("FLOAT", 0)}
    segs = [make_segment(90, 150007, cols, no_dict=("ri", "rl", "rd", "rf")),
            make_segment(92, 60001, cols, no_dict=("rl", "rd", "rf"))]
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        # single LONG / DOUBLE aggregations: 3-word records (pass C's batched 64-bit path)
        for agg in ("SUM(ri), MIN(ri)", "SUM(rl), MAX(rl)", "SUM(rd), MIN(rd), MAX(rd)", "SUM(rf)", "COUNT(*)",
                    "MAX(rl)", "SUM(rd)", "MIN(rd)", "SUM(rl)"):
            sql = ("SELECT k1, k2, k3, k4, COUNT(*), %s FROM t GROUP BY k1, k2, k3, k4 LIMIT 10000000 "
                   "OPTION(numGroupsLimit=10000000)" % agg)
            got, exp, _ = run_both(sql, segs, gsegs=gsegs, rel=DOUBLE_REL)
            ex = GpuQueryExecutor(parse_sql(sql), gsegs)
            strategy = ex.stats()["plan"]["strategy"]
            ex.close()
            assert strategy == "partitioned", (agg, strategy)
            assert len(got.groups) > 100000
    finally:
        for g in gsegs:
            g.close()


@pytest.mark.parametrize("flags", [0, L.PA_QF_NO_LANE_MAJOR])
def test_raw_group_by_hashed(flags):
    """GROUP BY raw (no-dictionary) columns — INT, LONG, DOUBLE, and mixed with dictionary columns — through the hashed
    key space (NoDictionarySingle/MultiColumnGroupKeyGenerator semantics: groups by value), small and large fetch
    paths, filters on the same raw columns; identical to the oracle."""
    cols = {"d1": ("INT", 40), "m": ("LONG", 300), "r2": ("INT", 0), "r3": ("LONG", 0), "r1": ("DOUBLE", 0)}
    small = [make_segment(80 + i, n, cols, no_dict=("r1", "r2", "r3")) for i, n in enumerate((9001, 3001))]
    queries = [
        "SELECT r2, COUNT(*), SUM(m), MAX(m) FROM t GROUP BY r2 LIMIT 100000",
        "SELECT d1, r2, COUNT(*), MIN(m), SUM(r3) FROM t WHERE r2 > 0 GROUP BY d1, r2 LIMIT 100000",
        "SELECT r3, COUNT(*), MIN(m), SUM(r2) FROM t WHERE r2 > 0 GROUP BY r3 LIMIT 100000",
        "SELECT r2, d1, AVG(m), DISTINCTCOUNTHLL(m) FROM t WHERE d1 < {d1} GROUP BY r2, d1 LIMIT 100000",
        "SELECT r1, COUNT(*) FROM t WHERE r1 > 50 GROUP BY r1 LIMIT 100000",
    ]
    d1 = int(small[0].column("d1").dictionary[20])
    for sql in queries:
        got, exp, _ = run_both(sql.format(d1=d1), small, flags=flags, rel=DOUBLE_REL)
        assert got.groups
    # large fetch path (accumulator block > 1 MiB): many distinct raw values
    rng = np.random.default_rng(5)
    from pinot_amd.segment import create_segment
    n = 200_000
    big = create_segment("big", {"r": rng.integers(-(1 << 40), 1 << 40, size=n), "m": rng.integers(0, 100, size=n)},
                         {"r": "LONG", "m": "INT"}, no_dictionary_columns=("r",))
    got, exp, _ = run_both("SELECT r, COUNT(*), SUM(m) FROM t GROUP BY r LIMIT 1000000 OPTION(numGroupsLimit=1000000)",
                           [big], flags=flags)
    assert len(got.groups) > 190_000


@pytest.mark.parametrize("flags", [0, L.PA_QF_NO_LANE_MAJOR])
def test_group_keys_wider_than_64_bits(flags):
    """Group keys wider than one 64-bit word (NoDictionaryMultiColumnGroupKeyGenerator's composite keys): a dictionary
    column + a raw LONG, two raw LONGs, raw DOUBLE + INT + dictionary take two key words ([k0, k1, state] slots,
    pa_keys.h ht_slot2); small and large fetch paths, a multi-value group-by column with a raw LONG, and the default
    numGroupsLimit (first-seen trimming over two-word keys); identical to the oracle."""
    cols = {"d1": ("INT", 40), "m": ("LONG", 300), "r2": ("INT", 0), "r3": ("LONG", 0), "r1": ("DOUBLE", 0),
            "r4": ("LONG", 0)}
    segs = [make_segment(85 + i, n, cols, no_dict=("r1", "r2", "r3", "r4")) for i, n in enumerate((9001, 3001))]
    queries = [
        "SELECT d1, r3, COUNT(*), SUM(m), MAX(m) FROM t GROUP BY d1, r3 LIMIT 100000",
        "SELECT r3, r4, COUNT(*), MIN(m), SUM(r2) FROM t WHERE r2 > 0 GROUP BY r3, r4 LIMIT 100000",
        "SELECT r1, r2, d1, AVG(m), DISTINCTCOUNTHLL(m) FROM t GROUP BY r1, r2, d1 LIMIT 100000",
        "SELECT r3, d1, COUNT(*) FROM t WHERE d1 < 20 GROUP BY r3, d1 LIMIT 100000",
    ]
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        for sql in queries:
            got, exp, _ = run_both(sql, segs, gsegs=gsegs, flags=flags, rel=DOUBLE_REL)
            assert got.groups
            ex = GpuQueryExecutor(parse_sql(sql), gsegs)
            assert ex.hashed and ex.key_words == 2, sql
            ex.close()
        # the default numGroupsLimit binds (first-seen trimming of two-word keys)
        got, exp, _ = run_both("SELECT r3, r4, COUNT(*) FROM t GROUP BY r3, r4 LIMIT 100000 OPTION(numGroupsLimit=500)",
                               segs, gsegs=gsegs, flags=flags)
        assert got.num_groups_limit_reached
    finally:
        for g in gsegs:
            g.close()
    # large fetch path: many distinct (LONG, LONG) pairs
    rng = np.random.default_rng(7)
    from pinot_amd.segment import create_segment
    n = 150_000
    big = create_segment("bigw", {"a": rng.integers(-(1 << 40), 1 << 40, size=n), "b": rng.integers(0, 3, size=n),
                                  "m": rng.integers(0, 100, size=n)},
                         {"a": "LONG", "b": "LONG", "m": "INT"}, no_dictionary_columns=("a", "b"))
    got, exp, _ = run_both("SELECT a, b, COUNT(*), SUM(m) FROM t GROUP BY a, b LIMIT 1000000 "
                           "OPTION(numGroupsLimit=1000000)", [big], flags=flags)
    assert len(got.groups) > 140_000


def test_hashed_dictionary_key_space():
    """A dictionary-only key space too large to address directly (product of cardinalities > 2^27) is hashed."""
    cols = {"a": ("INT", 900), "b": ("LONG", 800), "c": ("INT", 400), "m": ("LONG", 1000)}
    segs = [make_segment(90 + i, n, cols) for i, n in enumerate((30011, 7001))]
    sql = "SELECT a, b, c, COUNT(*), SUM(m), MIN(m) FROM t GROUP BY a, b, c LIMIT 100000 OPTION(numGroupsLimit=1000000)"
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        got, exp, ex = run_both(sql, segs, gsegs=gsegs)
        ex = GpuQueryExecutor(parse_sql(sql), gsegs)
        assert ex.hashed
        ex.close()
    finally:
        for g in gsegs:
            g.close()


# ------------------------------------------------------------------ numGroupsLimit first-seen trimming
# trimming modes (pa_query_limit_trimming): 0 none, 1 first positions + sort, 2 prefix walk
WALK = 2
SORTED = 1
LIMIT_PATHS = [(0, WALK), (L.PA_QF_NO_LIMIT_WALK, SORTED)]


def _limit_run(sql, segs, expect_trim=SORTED, rel=0.0, flags=0):
    q = parse_sql(sql)
    gsegs = [GpuSegment(sg) for sg in segs]
    try:
        ex = GpuQueryExecutor(q, gsegs, flags=flags)
        try:
            assert ex.stats()["plan"]["limit_trimming"] == int(expect_trim)
            got = ex.run()
        finally:
            ex.close()
    finally:
        for g in gsegs:
            g.close()
    exp = oracle.run_query(q, segs)
    assert_same(got, exp, rel)
    return got, exp


@pytest.mark.parametrize("flags,mode", LIMIT_PATHS)
@pytest.mark.parametrize("limit", [1, 7, 300, 5000, 30000])
def test_num_groups_limit_trimming_sv(limit, flags, mode):
    """Two dictionary dims (~1M possible keys) over segments of different sizes, filtered: each segment keeps its
    first `limit` groups in docId order (IntGroupIdMap.getGroupId) and drops later keys' docs; the union over segments
    and numGroupsLimitReached match the oracle's first-seen maps exactly."""
    cols = {"k1": ("INT", 1000), "k2": ("LONG", 1000), "m": ("LONG", 5000), "f": ("INT", 10)}
    segs = [make_segment(500 + i, n, cols) for i, n in enumerate((40000, 9001, 123))]
    sql = ("SELECT k1, k2, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE f <> 3 GROUP BY k1, k2 LIMIT 100000000 "
           "OPTION(numGroupsLimit=%d)" % limit)
    got, exp = _limit_run(sql, segs, mode, flags=flags)
    assert got.num_groups_limit_reached
    assert len(exp.groups) <= limit * len(segs)


@pytest.mark.parametrize("flags", [0, L.PA_QF_FORCE_GLOBAL, L.PA_QF_NO_PARTITION, L.PA_QF_NO_LANE_MAJOR])
def test_num_groups_limit_walk_every_strategy(flags):
    """The walk's admitted keys are tested inside every scan strategy (partitioned count + emit passes, global
    atomics, step-/lane-major tiles): dense 2-dim keys, segments whose crossing round is the first, a later one, or
    never comes (fewer matching groups than the limit)."""
    cols = {"k1": ("INT", 1000), "k2": ("LONG", 1000), "m": ("LONG", 5000), "f": ("INT", 10)}
    segs = [make_segment(700 + i, n, cols) for i, n in enumerate((60000, 16000, 2500, 47000))]
    sql = ("SELECT k1, k2, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE f <> 3 GROUP BY k1, k2 LIMIT 100000000 "
           "OPTION(numGroupsLimit=15000)")
    got, exp = _limit_run(sql, segs, WALK, flags=flags)
    assert got.num_groups_limit_reached


@pytest.mark.parametrize("limit", [5, 50, 119])
def test_num_groups_limit_walk_small_key_space(limit):
    """A key space of 120 keys (10 x 12) under a binding limit: nearly every 64-doc replay step of the walk holds the same
    key in several lanes (the replay's first-lane table resolves them; two keys in one table slot fall back to comparing
    every lane); same first-seen groups as the oracle on both trimming paths."""
    cols = {"k1": ("INT", 10), "k2": ("LONG", 12), "m": ("LONG", 500)}
    segs = [make_segment(760 + i, n, cols) for i, n in enumerate((20000, 3001))]
    for flags, mode in LIMIT_PATHS:
        got, exp = _limit_run("SELECT k1, k2, COUNT(*), SUM(m) FROM t GROUP BY k1, k2 LIMIT 100000000 "
                              "OPTION(numGroupsLimit=%d)" % limit, segs, mode, flags=flags)
        assert got.num_groups_limit_reached


def test_num_groups_limit_walk_hbm_bitmap():
    """Key spaces beyond the walk's LDS bitmap (1.28M keys: 1500 x 1000 here) keep the admitted-key bitmap in HBM
    (limit_walk_kernel<true>); same first-seen groups as the oracle."""
    cols = {"k1": ("INT", 1500), "k2": ("LONG", 1000), "m": ("LONG", 5000)}
    segs = [make_segment(740 + i, n, cols) for i, n in enumerate((30000, 12000))]
    got, exp = _limit_run("SELECT k1, k2, COUNT(*), SUM(m) FROM t GROUP BY k1, k2 LIMIT 100000000 "
                          "OPTION(numGroupsLimit=9000)", segs, WALK)
    assert got.num_groups_limit_reached


def test_num_groups_limit_default_binds():
    """Default numGroupsLimit (100000) on a segment with more distinct keys: trimmed on the GPU like the reference."""
    cols = {"k1": ("INT", 1000), "k2": ("LONG", 1000)}
    segs = [make_segment(32, 200000, cols)]
    for flags, mode in LIMIT_PATHS:
        got, exp = _limit_run("SELECT k1, k2, COUNT(*) FROM t GROUP BY k1, k2 LIMIT 100000000", segs, mode, flags=flags)
        assert len(got.groups) == 100000 and got.num_groups_limit_reached


def test_num_groups_limit_not_reached():
    """The limit can bind in principle (key space > limit) but the filter leaves fewer groups: nothing is trimmed and
    numGroupsLimitReached stays false."""
    cols = {"k1": ("INT", 1000), "k2": ("LONG", 1000), "f": ("INT", 1000)}
    segs = [make_segment(70 + i, 30000, cols) for i in range(2)]
    for flags, mode in LIMIT_PATHS:
        got, exp = _limit_run("SELECT k1, k2, COUNT(*) FROM t WHERE f < 2 GROUP BY k1, k2 LIMIT 100000 "
                              "OPTION(numGroupsLimit=20000)", segs, mode, flags=flags)
        assert not got.num_groups_limit_reached


def test_num_groups_limit_hll_avg_double():
    """DISTINCTCOUNTHLL, AVG and DOUBLE sums under trimming."""
    cols = {"k1": ("INT", 300), "k2": ("INT", 200), "u": ("LONG", 50000), "d": ("DOUBLE", 5000)}
    segs = [make_segment(80 + i, 20000, cols) for i in range(2)]
    for flags, mode in LIMIT_PATHS:
        _limit_run("SELECT k1, k2, DISTINCTCOUNTHLL(u), AVG(d), SUM(d) FROM t GROUP BY k1, k2 LIMIT 100000 "
                   "OPTION(numGroupsLimit=1000)", segs, mode, rel=DOUBLE_REL, flags=flags)


def test_num_groups_limit_raw_hashed():
    """No-dictionary group-by (NoDictionarySingle/MultiColumnGroupKeyGenerator: same first-seen cap) through the
    hashed key space."""
    cols = {"r": ("INT", 0), "k": ("INT", 50), "m": ("LONG", 1000)}
    segs = [make_segment(90 + i, 25000, cols, no_dict=("r",)) for i in range(2)]
    _limit_run("SELECT r, k, COUNT(*), SUM(m) FROM t GROUP BY r, k LIMIT 1000000 OPTION(numGroupsLimit=777)", segs)
    _limit_run("SELECT r, COUNT(*), MAX(m) FROM t GROUP BY r LIMIT 1000000 OPTION(numGroupsLimit=500)", segs)


def test_num_groups_limit_not_triggered_below_bound():
    """A key space smaller than the limit never runs the trimming passes."""
    cols = {"k1": ("INT", 20), "k2": ("INT", 30)}
    segs = [make_segment(99, 5000, cols)]
    _limit_run("SELECT k1, k2, COUNT(*) FROM t GROUP BY k1, k2 LIMIT 1000 OPTION(numGroupsLimit=601)", segs,
               expect_trim=0)


@pytest.mark.parametrize("flags", [0, L.PA_QF_NO_LANE_MAJOR])
@pytest.mark.parametrize("nb", list(range(1, 32)))
def test_bit_widths_through_capi(nb, flags):
    """Raw C-ABI use: an nb-bit column with no dictionary values (STRING type), DICT_RANGE filter count (plain and
    negated) and a DICT_SET filter, against numpy on the same ids — every bit width, both tile layouts."""
    from pinot_amd.segment import pack_bits
    lib = L.lib()
    n = 50_000 + nb
    rng = np.random.default_rng(nb)
    ids = rng.integers(0, 1 << nb, size=n, dtype=np.int64).astype(np.uint32)
    card = (1 << nb) if nb < 31 else (1 << 31) - 1
    ids = np.minimum(ids, card - 1)
    fwd = pack_bits(ids, nb)
    seg = L.check_ptr(lib.pa_segment_create(n), "create")
    L.check(lib.pa_segment_add_sv_dict_column(seg, 0, fwd.ctypes.data, fwd.nbytes, nb, card, L.PA_STRING, None, None),
            "add")
    lo, hi = int(card // 5), int(card // 2) + 1
    for kind, negate in ((L.PA_LEAF_DICT_RANGE, 0), (L.PA_LEAF_DICT_RANGE, 1), (L.PA_LEAF_DICT_SET, 0)):
        if kind == L.PA_LEAF_DICT_SET and nb > 20:
            continue
        spec = L.QuerySpec()
        spec.flags = flags
        spec.num_leaves = 1
        spec.leaves[0].column_id = 0
        spec.leaves[0].kind = kind
        spec.num_ops = 1
        spec.ops[0] = L.PA_OP_LEAF
        spec.num_aggs = 1
        spec.aggs[0].type = L.PA_AGG_COUNT
        q = L.check_ptr(lib.pa_query_create(ctypes.byref(spec), 1), "qcreate")
        lp = (L.LeafParams * 1)()
        lut = None
        lp[0].negate = negate
        if kind == L.PA_LEAF_DICT_RANGE:
            lp[0].lo, lp[0].hi = lo, hi
            expected = int(((ids >= lo) & (ids < hi)).sum())
            if negate:
                expected = n - expected
        else:
            sel = np.arange(0, card, 3, dtype=np.int64)
            lut = np.zeros((card + 31) // 32, dtype=np.uint32)
            np.bitwise_or.at(lut, sel >> 5, (np.uint32(1) << (sel & 31).astype(np.uint32)))
            lp[0].lut = lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
            expected = int((ids % 3 == 0).sum())
        L.check(lib.pa_query_bind_segment(q, 0, seg, lp, None), "bind")
        L.check(lib.pa_query_prepare(q), "prepare")
        assert lib.pa_query_lane_major(q) == (0 if flags else 1)
        L.check(lib.pa_query_execute(q, None), "execute")
        keys = np.zeros(1, np.int64)
        counts = np.zeros(1, np.int64)
        outs = np.zeros(1, np.float64)
        ptrs = (ctypes.c_void_p * 1)(outs.ctypes.data)
        assert L.check(lib.pa_query_fetch(q, None, 1, keys.ctypes.data, counts.ctypes.data, ptrs), "fetch") == 1
        assert counts[0] == expected
        lib.pa_query_destroy(q)
    lib.pa_segment_destroy(seg)


def test_large_segment_properties():
    """A 10M-doc segment (the BASELINE configs' segment size): filter+group-by counts sum to the filter-only count,
    both equal to the oracle, and the group-by sums are exact."""
    from pinot_amd.segment import segment_from_dict_ids
    n = 10_000_000
    rng = np.random.default_rng(99)
    specs = {}
    for name, card in (("day", 512), ("acct", 1 << 17), ("clicks", 1024)):
        nb = int(card - 1).bit_length()
        ids = rng.integers(0, card, size=n, dtype=np.int64).astype(np.uint32)
        from pinot_amd.segment import pack_bits
        specs[name] = ("LONG" if name == "clicks" else "INT", np.arange(card, dtype=np.int64) * 3 + 17000,
                       pack_bits(ids, nb))
    seg = segment_from_dict_ids("big", n, specs)
    g = GpuSegment(seg)
    sql_f = "SELECT COUNT(*), SUM(clicks) FROM t WHERE day BETWEEN 17300 AND 17400"
    sql_g = "SELECT day, COUNT(*), SUM(clicks) FROM t WHERE day BETWEEN 17300 AND 17400 GROUP BY day LIMIT 1000"
    a, _, _ = run_both(sql_f, [seg], gsegs=[g])
    b, _, _ = run_both(sql_g, [seg], gsegs=[g])
    assert sum(v[0] for v in b.groups.values()) == a.row[0]
    assert sum(v[1] for v in b.groups.values()) == a.row[1]
    g.close()
