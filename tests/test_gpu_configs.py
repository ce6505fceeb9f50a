"""Every BASELINE.json config at its own shape through the HIP path, against the oracle, with the plan it must run.

  configs[0]  10M-doc segment, COUNT(*), SUM(m) WHERE day BETWEEN a AND b (LONG metric, non-arithmetic dictionary)
  configs[1]  the README AdAnalytics query over a 10M-doc segment of bench.py's column shapes (+ a wide IN list, so
              the GROUP BY SUM has real groups), lane-major tiles, the day range deferred behind the accountId clause
  configs[2]  GROUP BY d1, d2 over the exact 1024 x 1024 key space with SUM/MIN/MAX, 3M docs: partitioned aggregation,
              untrimmed and at the default numGroupsLimit (walk-form first-seen trimming)
  configs[3]  two executors (two ranks' segment sets, table-wide dictionaries) merged element-wise plus a world-size-1
              RCCL reduce (the N>1 collective path); N>1 itself runs only in the driver's scaling bench
  configs[4]  the star query over the exact 16 x 32 x 64 x 8 key space: raw DOUBLE SUM + DISTINCTCOUNTHLLMV over a
              4096-value MV column, 2.4M docs, partitioned, untrimmed and at the default numGroupsLimit

Bars as in test_gpu_parity: bit-exact COUNT / LONG SUM (all sums here stay below 2^53) / MIN / MAX / group keys / HLL
registers; DOUBLE sums within 1e-9 relative. Large key spaces are compared as arrays (oracle.run_query_arrays).
"""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch

import oracle
from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOUBLE_REL = 1e-9


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


BENCH = _load("pa_bench_main", "bench.py")
CFG = _load("pa_bench_configs", "tools/bench_configs.py")


def _plan(ex):
    st = ex.stats()["plan"]
    return st


def _compare_arrays(ex, q, segs, rel=0.0):
    """GPU fetch_arrays vs oracle.run_query_arrays: keys, counts, every aggregation; numDocsScanned and
    numGroupsLimitReached."""
    keys, counts, outs = ex.fetch_arrays()
    exp = oracle.run_query_arrays(q, segs)
    assert int(L.lib().pa_query_matched_docs(ex.handle)) == exp["matched"]
    assert (int(L.lib().pa_query_num_groups_limit_reached(ex.handle)) > 0) == exp["limit_reached"]
    np.testing.assert_array_equal(keys, exp["keys"])
    np.testing.assert_array_equal(counts, exp["counts"])
    oaggs, amap = exp["oaggs"], exp["amap"]
    for a, gi, oi in zip(q.aggregations, ex.agg_map, amap):
        if a.function == "COUNT":
            continue
        got, want = outs[gi], exp["accs"][oi]
        if a.function.startswith("DISTINCTCOUNTHLL"):
            np.testing.assert_array_equal(got.reshape(want.shape), want, err_msg=a.function)
        elif rel:
            np.testing.assert_allclose(got, want, rtol=rel, atol=0, err_msg=a.function)
        else:
            np.testing.assert_array_equal(got, want, err_msg=a.function)
    return len(keys)


# ------------------------------------------------------------------ configs[0]
@pytest.fixture(scope="module")
def sumscan():
    seg = CFG.sumscan_segment(3, 10_000_000)
    g = GpuSegment(seg)
    yield seg, g
    g.close()


@pytest.mark.parametrize("plan", ["sel_10pct", "sel_50pct", "sel_100pct"])
def test_configs0_count_sum_day_range(sumscan, plan):
    seg, g = sumscan
    sql = dict((n, s) for n, s, _ in CFG.WORKLOADS["sumscan"][1])[plan]
    q = parse_sql(sql)
    ex = GpuQueryExecutor(q, [g])
    try:
        p = _plan(ex)
        assert p["lane_major"] == 1 and p["strategy"] == "lane", p
        got = ex.run()
    finally:
        ex.close()
    exp = oracle.run_query(q, [seg])
    assert_same(got, exp)
    # the LDS-accumulator path (the strategy before per-lane registers) agrees
    ex = GpuQueryExecutor(q, [g], flags=L.PA_QF_NO_LANE_ACC)
    try:
        assert _plan(ex)["strategy"] != "lane"
        assert_same(ex.run(), exp)
    finally:
        ex.close()
    frac = got.row[0] / seg.num_docs
    assert {"sel_10pct": 0.1, "sel_50pct": 0.5, "sel_100pct": 1.0}[plan] == pytest.approx(frac, abs=0.02)


# ------------------------------------------------------------------ configs[1]
@pytest.fixture(scope="module")
def adanalytics():
    seg = BENCH.make_segment(1000, 10_000_000)
    g = GpuSegment(seg)
    yield seg, g
    g.close()


def test_configs1_readme_query(adanalytics):
    seg, g = adanalytics
    q = parse_sql(BENCH.QUERY)
    ex = GpuQueryExecutor(q, [g])
    try:
        p = _plan(ex)
        assert p["lane_major"] == 1 and p["eager_literals"] == 1, p  # accountId leads, the day range is lazy
        got = ex.run()
    finally:
        ex.close()
    assert_same(got, oracle.run_query(q, [seg]))


def test_configs1_wide_in_list(adanalytics):
    """Same shape with 2000 accounts in the IN list: ~150k matching docs over 8 days, real GROUP BY SUM work."""
    seg, g = adanalytics
    accts = seg.column("accountId").dictionary[::64][:2000]
    sql = ("SELECT daysSinceEpoch, sum(clicks), sum(impressions), COUNT(*) FROM AdAnalyticsTable WHERE daysSinceEpoch "
           "BETWEEN 17849 AND 17856 AND accountId IN (%s) GROUP BY daysSinceEpoch TOP 100"
           % ", ".join(str(int(a)) for a in accts))
    q = parse_sql(sql)
    ex = GpuQueryExecutor(q, [g])
    try:
        assert _plan(ex)["lane_major"] == 1
        got = ex.run()
    finally:
        ex.close()
    exp = oracle.run_query(q, [seg])
    assert_same(got, exp)
    assert len(got.groups) == 8 and got.num_docs_scanned > 1000


@pytest.fixture(scope="module")
def adanalytics3():
    """Three bench.py segments of the bench's own size (10M docs each) sharing their dictionaries, as the bench's 100
    segments do: 29,298 1024-doc tiles, so every wave of the packed-row kernel runs past JIT_DRAIN tiles and its
    mid-loop drain fires, as it does at the bench's 1B docs."""
    segs = [BENCH.make_segment(2000 + i, 10_000_000) for i in range(3)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


# the dense GROUP BY kernel variant the bench's secondary lines run (pa_query_plan; engine.STRATEGY_VARIANTS)
BENCH_SECONDARY_VARIANT = "gdense_lm8"  # (dense_packed 2: the query-shape specialised kernel)


@pytest.mark.parametrize("drain", [0, L.PA_QF_GD_DRAIN_EACH_TILE])
@pytest.mark.parametrize("n_ids,frac", [(17476, 0.1), (87381, 0.5)])
def test_configs1_secondary_lines(adanalytics3, n_ids, frac, drain):
    """bench.py's secondary lines at their plan: the accountId IN list widened to 10 % / 50 % of the docs (a 2^17-bit
    bitmap held in LDS), the 384-day key box, two dictionary SUMs over segments that share dictionaries, on the
    query-shape specialised kernel (dense_packed 2: gdl_jit.hip) at the bench's own drain period and with a drain after
    every tile."""
    segs, gs = adanalytics3
    q = parse_sql(BENCH.secondary_query(n_ids))
    ex = GpuQueryExecutor(q, gs, flags=drain)
    try:
        p = _plan(ex)
        assert p["strategy"] == "lds_dense" and p["variant"] == BENCH_SECONDARY_VARIANT, p
        assert p["dense_packed"] == 2, p  # the JIT compiled and loaded (not the generic packed kernel)
        got = ex.run()
    finally:
        ex.close()
    exp = oracle.run_query(q, segs)
    assert_same(got, exp)
    assert len(got.groups) == 384
    assert got.num_docs_scanned / sum(s.num_docs for s in segs) == pytest.approx(frac, abs=0.01)


@pytest.fixture(scope="module")
def adanalytics_own():
    """Three of bench.py's own-dictionary segments (4M docs each): 4-day time partitions, a random half of the accounts,
    per-segment clicks / impressions value runs."""
    segs = [BENCH.make_segment_own(6000 + i, 4_000_000, i) for i in range(3)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


@pytest.mark.parametrize("drain", [0, L.PA_QF_GD_DRAIN_EACH_TILE])
@pytest.mark.parametrize("n_ids,frac", [(13107, 0.1), (65536, 0.5)])
def test_configs1_own_dictionary_lines(adanalytics_own, n_ids, frac, drain):
    """bench.py's own-dictionary secondary lines at their plan: every segment's own dictionaries (per-segment accountId
    IN bitmaps in LDS table slots, day keys shifted per partition, SUM terms offset per segment) on the query-shape
    specialised kernel, at the packed rows' own drain period and drained after every tile."""
    segs, gs = adanalytics_own
    q = parse_sql(BENCH.secondary_query_own(n_ids, len(segs)))
    ex = GpuQueryExecutor(q, gs, flags=drain)
    try:
        p = _plan(ex)
        assert p["strategy"] == "lds_dense" and p["dense_packed"] == 2, p
        got = ex.run()
    finally:
        ex.close()
    exp = oracle.run_query(q, segs)
    assert_same(got, exp)
    assert len(got.groups) == BENCH.OWN_DAYS * len(segs)
    assert got.num_docs_scanned / sum(s.num_docs for s in segs) == pytest.approx(frac, abs=0.01)


# ------------------------------------------------------------------ configs[2]
@pytest.fixture(scope="module")
def highcard():
    segs = [CFG.highcard_segment(200 + i, 1_500_000) for i in range(2)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


@pytest.mark.parametrize("count_free", [True, False])
@pytest.mark.parametrize("variant", ["untrimmed", "default_limit", "filtered"])
def test_configs2_high_cardinality_group_by(highcard, variant, count_free):
    """configs[2] (GROUP BY d1, d2 over ~1M keys, SUM / MIN / MAX) on the partitioned path against the oracle: with the
    count-free emit (pve_jit.hip: whole record chunks per workgroup, partitions read through chunk lists) where it
    applies (untrimmed, filtered, and the default numGroupsLimit: the walk form's admitted-key bitmaps checked per record),
    and with the count + emit passes (PA_QF2_NO_COUNT_FREE)."""
    segs, gs = highcard
    sql = {"untrimmed": "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                        "OPTION(numGroupsLimit=2000000)",
           "default_limit": "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000",
           "filtered": "SELECT d1, d2, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE m < 6554 GROUP BY d1, d2 "
                       "LIMIT 2000000 OPTION(numGroupsLimit=2000000)"}[variant]
    q = parse_sql(sql)
    ex = GpuQueryExecutor(q, gs, flags=0 if count_free else L.PA_QF2_NO_COUNT_FREE)
    try:
        p = _plan(ex)
        assert p["strategy"] == "partitioned", p
        assert p["limit_trimming"] == (2 if variant == "default_limit" else 0), p
        assert p["count_free_emit"] == (1 if count_free else 0), p
        ex.execute()
        n = _compare_arrays(ex, q, segs)
    finally:
        ex.close()
    if variant == "untrimmed":
        assert n > 900_000  # 3M docs over 1M keys
    elif variant == "default_limit":
        assert n <= 2 * 100_000


@pytest.fixture(scope="module")
def highcard_own():
    segs = [CFG.highcard_own_segment(201 + i, 1_500_000) for i in range(2)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


@pytest.mark.parametrize("count_free", [True, False])
@pytest.mark.parametrize("variant", ["untrimmed", "default_limit", "filtered"])
def test_configs2_own_dictionaries(highcard_own, variant, count_free):
    """configs[2] over segments that built their own dictionaries (d1 / d2 / m shifted runs of the table-wide
    dictionaries): the count-free emit maps each segment's dictIds by its key and value id offsets (pve_jit.hip
    PVE_KOFF / PVE_VOFF); the count + emit passes through the remap tables. Table-wide keys against the oracle's."""
    segs, gs = highcard_own
    assert not np.array_equal(segs[0].column("d1").dictionary, segs[1].column("d1").dictionary)
    sql = {"untrimmed": "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                        "OPTION(numGroupsLimit=2000000)",
           "default_limit": "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000",
           "filtered": "SELECT d1, d2, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE m < 6554 GROUP BY d1, d2 "
                       "LIMIT 2000000 OPTION(numGroupsLimit=2000000)"}[variant]
    q = parse_sql(sql)
    ex = GpuQueryExecutor(q, gs, flags=0 if count_free else L.PA_QF2_NO_COUNT_FREE)
    try:
        p = _plan(ex)
        assert p["strategy"] == "partitioned", p
        assert p["count_free_emit"] == (1 if count_free else 0), p
        # (about 1025 x 1027 keys: 257 partitions of 4096 keys, or under the count-free emit one per CU: pve_repartition)
        nk = int(L.lib().pa_query_num_keys(ex.handle))
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        assert nk > 256 * 4096 and p["partition_keys"] == (-(-nk // cus) if count_free else 4096), (nk, p)
        ex.execute()
        _compare_arrays(ex, q, segs)
    finally:
        ex.close()


def test_configs2_non_affine_values():
    """configs[2] with a non-arithmetic value dictionary (pass C looks every SUM value up)."""
    segs = [CFG.highcard_rd_segment(300, 2_000_000)]
    gs = [GpuSegment(s) for s in segs]
    q = parse_sql("SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                  "OPTION(numGroupsLimit=2000000)")
    ex = GpuQueryExecutor(q, gs)
    try:
        assert _plan(ex)["strategy"] == "partitioned"
        ex.execute()
        _compare_arrays(ex, q, segs)
    finally:
        ex.close()
        for g in gs:
            g.close()


# ------------------------------------------------------------------ configs[4]
@pytest.fixture(scope="module")
def star():
    segs = [CFG.star_segment(400 + i, 1_200_000) for i in range(2)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


@pytest.mark.parametrize("count_free", [True, False])
@pytest.mark.parametrize("variant", ["untrimmed", "default_limit", "filtered"])
def test_configs4_star_query(star, variant, count_free):
    """configs[4] (raw DOUBLE SUM + DISTINCTCOUNTHLLMV over 262144 keys) on the partitioned path against the oracle: with
    the count-free emit of both record streams where it applies (pve_jit.hip: V records of key offset + the raw value,
    H records per MV value, each stream in whole chunks per workgroup read through chunk lists; the default
    numGroupsLimit's admitted-key bitmaps checked per record) and with the count + emit passes."""
    segs, gs = star
    assert segs[0].column("tags").cardinality == 4096 and not segs[0].column("r").has_dictionary
    opt = "" if variant == "default_limit" else " OPTION(numGroupsLimit=1000000)"
    where = " WHERE d4 <> 5 AND d3 < 40" if variant == "filtered" else ""
    q = parse_sql("SELECT d1, d2, d3, d4, COUNT(*), SUM(r), DISTINCTCOUNTHLLMV(tags) FROM t" + where +
                  " GROUP BY d1, d2, d3, d4 LIMIT 1000000" + opt)
    ex = GpuQueryExecutor(q, gs, flags=0 if count_free else L.PA_QF2_NO_COUNT_FREE)
    try:
        p = _plan(ex)
        assert ex.num_keys == 16 * 32 * 64 * 8
        assert p["strategy"] == "partitioned", p
        assert p["limit_trimming"] == (2 if variant == "default_limit" else 0), p
        assert p["count_free_emit"] == (2 if count_free else 0), p
        ex.execute()
        n = _compare_arrays(ex, q, segs, rel=DOUBLE_REL)
    finally:
        ex.close()
    assert n > 250_000 if variant == "untrimmed" else n <= 200_000


def test_configs4_hll_only_keeps_count_pass(star):
    """DISTINCTCOUNTHLLMV without a V stream (COUNT from the H records' first-value flags) keeps the count + emit
    passes."""
    segs, gs = star
    q = parse_sql("SELECT d1, d2, d3, d4, DISTINCTCOUNTHLLMV(tags) FROM t GROUP BY d1, d2, d3, d4 LIMIT 1000000 "
                  "OPTION(numGroupsLimit=1000000)")
    ex = GpuQueryExecutor(q, gs)
    try:
        p = _plan(ex)
        assert p["strategy"] == "partitioned" and p["count_free_emit"] == 0, p
        ex.execute()
        _compare_arrays(ex, q, segs, rel=DOUBLE_REL)
    finally:
        ex.close()


# ------------------------------------------------------------------ configs[3]
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_configs3_two_rank_merge_and_rccl_reduce(adanalytics):
    """configs[3]'s data path on one GPU: two executors stand for two ranks' segment sets (different segments, the
    agreed table-wide dictionaries from parallel.table_layout), their accumulator blocks merge element-wise (what the
    RCCL reduce does across GPUs), and a world-size-1 RCCL group runs DistributedAccumulators' real reduce."""
    import torch
    import torch.distributed as dist
    from pinot_amd.parallel import SECTION_OP, DistributedAccumulators, key_space_fingerprint, table_layout
    seg0, g0 = adanalytics
    seg1 = BENCH.make_segment(1001, 3_000_000)
    g1 = GpuSegment(seg1)
    accts = seg0.column("accountId").dictionary[::32][:4000]
    sql = ("SELECT daysSinceEpoch, sum(clicks), sum(impressions), COUNT(*), DISTINCTCOUNTHLL(accountId) "
           "FROM AdAnalyticsTable WHERE daysSinceEpoch BETWEEN 17800 AND 17900 AND accountId IN (%s) "
           "GROUP BY daysSinceEpoch TOP 1000" % ", ".join(str(int(a)) for a in accts))
    q = parse_sql(sql)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % _port(),
                            device_id=torch.device("cuda", 0))
    exs = []
    try:
        kw = table_layout(q, [seg0, seg1]).executor_kwargs()
        exs = [GpuQueryExecutor(q, [g], **kw) for g in (g0, g1)]
        assert key_space_fingerprint(exs[0]) == key_space_fingerprint(exs[1])
        accs = [DistributedAccumulators(e, torch.device("cuda", 0)) for e in exs]
        for e in exs:
            e.execute()
        torch.cuda.synchronize()
        for (k0, t0), (k1, t1) in zip(accs[0].views, accs[1].views):
            op = SECTION_OP[k0]
            if op == dist.ReduceOp.SUM:
                t0.add_(t1)
            elif op == dist.ReduceOp.MIN:
                torch.minimum(t0, t1, out=t0)
            else:
                torch.maximum(t0, t1, out=t0)
        accs[0].reduce(dst=0)
        got = exs[0].fetch()
    finally:
        for e in exs:
            e.close()
        dist.destroy_process_group()
        g1.close()
    exp = oracle.run_query(q, [seg0, seg1])
    assert_same(got, exp)
    assert len(got.groups) == 101 and got.num_docs_scanned > 10_000


def test_configs4_count_free_relocated_accumulators(star):
    """configs[4] on the count-free emit with the accumulator block moved into a torch buffer (what the cross-GPU
    reduce does, parallel.DistributedAccumulators under a world-size-1 RCCL group): both streams' kernels write through
    the relocated numDocsScanned counter and pass C into the new block."""
    import torch
    import torch.distributed as dist
    from pinot_amd.parallel import DistributedAccumulators
    segs, gs = star
    q = parse_sql("SELECT d1, d2, d3, d4, COUNT(*), SUM(r), DISTINCTCOUNTHLLMV(tags) FROM t WHERE d2 < 20 "
                  "GROUP BY d1, d2, d3, d4 LIMIT 1000000 OPTION(numGroupsLimit=1000000)")
    dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % _port(),
                            device_id=torch.device("cuda", 0))
    ex = GpuQueryExecutor(q, gs)
    try:
        assert _plan(ex)["count_free_emit"] == 2
        acc = DistributedAccumulators(ex, torch.device("cuda", 0))
        ex.execute()
        acc.reduce(dst=0)
        torch.cuda.synchronize()
        _compare_arrays(ex, q, segs, rel=DOUBLE_REL)
    finally:
        ex.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("agg", ["SUM(r)", "MIN(r), MAX(r)"])
def test_configs4_raw_value_stream_count_free(star, agg):
    """The V stream alone with a raw DOUBLE value (three-word records: key offset + the value's 64 bits, the raw column
    staged by the count-free emit's DMA ring) against the oracle."""
    segs, gs = star
    q = parse_sql("SELECT d1, d2, d3, d4, COUNT(*), %s FROM t WHERE d3 >= 7 GROUP BY d1, d2, d3, d4 LIMIT 1000000 "
                  "OPTION(numGroupsLimit=1000000)" % agg)
    ex = GpuQueryExecutor(q, gs)
    try:
        p = _plan(ex)
        assert p["strategy"] == "partitioned" and p["count_free_emit"] == 1, p
        ex.execute()
        _compare_arrays(ex, q, segs, rel=DOUBLE_REL)
    finally:
        ex.close()
