"""Secondary measurements for BASELINE.json configs[2] and configs[4] (the headline configs[1] line is bench.py).

  highcard : configs[2] — GROUP BY 2 dictionary dims (1024 x 1024 = ~1M groups) with SUM/MIN/MAX over every doc
             (and over a 10 % filter); the key space does not fit LDS, so accumulators are global
  star     : configs[4] shape on one GPU — raw DOUBLE SUM + DISTINCTCOUNTHLLMV over a multi-value column, 4-dim
             GROUP BY

python tools/bench_configs.py [--workload highcard|star|all] [--segments S] [--docs D] [--reps R]
Prints one JSON line per (workload, plan): scan-kernel ms per launch (HIP events around back-to-back launches on
the launch stream), rows/s, forward-index bytes staged per launch and GB/s, fetch ms, groups.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def sv_spec(rng, docs, card, dtype="INT", base=0):
    from pinot_amd.segment import num_bits_per_value, pack_bits
    nb = num_bits_per_value(card - 1)
    if card == 1 << nb:  # uniform dictIds over [0, 2^nb) == uniformly random bytes
        fwd = np.frombuffer(rng.bytes((docs * nb + 7) // 8), dtype=np.uint8)
    else:
        fwd = pack_bits(rng.integers(0, card, size=docs).astype(np.uint32), nb)
    return (dtype, np.arange(card, dtype=np.int64) + base, fwd)


def highcard_segment(seed, docs):
    from pinot_amd.segment import segment_from_dict_ids
    rng = np.random.default_rng(seed)
    return segment_from_dict_ids("hc%d" % seed, docs, {
        "d1": sv_spec(rng, docs, 1024, base=1000), "d2": sv_spec(rng, docs, 1024, base=5000),
        "m": sv_spec(rng, docs, 1 << 16, "LONG")})


def highcard_own_segment(seed, docs):
    """configs[2] where every segment built its own dictionaries (SegmentDictionaryCreator.java:104): d1 / d2 runs of 1024
    values starting at a per-segment shift (0..7) of the table-wide 1031-value dictionaries (~1.06M keys), m 65536
    values from a per-segment offset (the table-wide value dictionary is their union)."""
    from pinot_amd.segment import segment_from_dict_ids
    rng = np.random.default_rng(seed)
    return segment_from_dict_ids("hco%d" % seed, docs, {
        "d1": sv_spec(rng, docs, 1024, base=1000 + seed % 8), "d2": sv_spec(rng, docs, 1024, base=5000 + (3 * seed) % 8),
        "m": sv_spec(rng, docs, 1 << 16, "LONG", base=(611 * seed) % 4096)})


def highcard_rd_segment(seed, docs):
    """configs[2] with a non-arithmetic value dictionary: m's 65536 values are sorted random distinct longs, so pass C
    looks every SUM value up in the dictionary (the affine shortcut does not apply)."""
    seg = highcard_segment(seed, docs)
    rng = np.random.default_rng(10_000 + seed)
    vals = np.unique(rng.integers(0, 1 << 40, size=70_000))[:1 << 16]
    assert len(vals) == 1 << 16
    seg.columns["m"].dictionary = np.sort(vals).astype(np.int64)
    return seg


def sumscan_segment(seed, docs):
    """configs[0]: a fixed-bit dictionary-encoded INT dimension (daysSinceEpoch, 1024 days = 10 bits) and a LONG metric
    m whose 16384 dictionary values (14 bits) are sorted random longs below 2^29 (no arithmetic shortcut: every SUM value
    is a dictionary lookup; a 10M-doc segment's sum stays below 2^53, where the reference's double accumulation is
    exact)."""
    from pinot_amd.segment import segment_from_dict_ids
    rng = np.random.default_rng(seed)
    vals = np.unique(np.random.default_rng(777).integers(0, 1 << 29, size=20_000))[:1 << 14].astype(np.int64)
    assert len(vals) == 1 << 14
    return segment_from_dict_ids("ss%d" % seed, docs, {
        "daysSinceEpoch": sv_spec(rng, docs, 1024, base=17000),
        "m": ("LONG", vals, sv_spec(rng, docs, 1 << 14)[2])})


def sumscan_raw_segment(seed, docs):
    """configs[0] with the LONG metric stored raw (no dictionary: Pinot's usual metric layout, noDictionaryColumns):
    8 bytes per doc, read straight from HBM."""
    from pinot_amd.segment import Column
    seg = sumscan_segment(seed, docs)
    m = Column(name="m", data_type="LONG", has_dictionary=False)
    m.raw_values = np.random.default_rng(seed + 5).integers(0, 1 << 29, size=docs, dtype=np.int64)
    seg.columns["m"] = m
    return seg


def star_segment(seed, docs, avg_mv=3):
    from pinot_amd.segment import Column, mv_column_from_flat, segment_from_dict_ids
    rng = np.random.default_rng(seed)
    seg = segment_from_dict_ids("st%d" % seed, docs, {
        "d1": sv_spec(rng, docs, 16), "d2": sv_spec(rng, docs, 32), "d3": sv_spec(rng, docs, 64),
        "d4": sv_spec(rng, docs, 8)})
    lengths = rng.integers(1, 2 * avg_mv, size=docs)
    flat = rng.integers(0, 4096, size=int(lengths.sum())).astype(np.uint32)
    seg.columns["tags"] = mv_column_from_flat("tags", lengths, flat, np.arange(4096, dtype=np.int64) * 11, "INT")
    r = Column(name="r", data_type="DOUBLE", has_dictionary=False)
    r.raw_values = rng.normal(100.0, 30.0, size=docs)
    seg.columns["r"] = r
    return seg


WORKLOADS = {
    # configs[0]: COUNT(*), SUM(m) WHERE day BETWEEN a AND b at ~10 % / ~50 % / 100 % selectivity (day dictionary
    # 17000..17999, uniform)
    "sumscan": (sumscan_segment, [
        ("sel_0p1pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch = 17100", 0),
        ("sel_1pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17109", 0),
        ("count_10pct", "SELECT COUNT(*) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17201", 0),
        ("count_100pct", "SELECT COUNT(*) FROM t WHERE daysSinceEpoch BETWEEN 17000 AND 18023", 0),
        ("min_100pct", "SELECT MIN(m) FROM t WHERE daysSinceEpoch BETWEEN 17000 AND 18023", 0),
        ("sel_10pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17201", 0),
        ("sel_50pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17611", 0),
        ("sel_100pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17000 AND 18023", 0),
    ]),
    "sumscan_raw": (sumscan_raw_segment, [
        ("sel_10pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17201", 0),
        ("sel_50pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17611", 0),
        ("sel_100pct", "SELECT COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17000 AND 18023", 0),
    ]),
    # the north-star shape on configs[0]'s columns: filter + GROUP BY SUM (1024-day key space, raw LONG metric)
    "sumgroup": (sumscan_raw_segment, [
        ("sel_10pct", "SELECT daysSinceEpoch, COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17201 "
                      "GROUP BY daysSinceEpoch LIMIT 2000", 0),
        ("sel_50pct", "SELECT daysSinceEpoch, COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17611 "
                      "GROUP BY daysSinceEpoch LIMIT 2000", 0),
    ]),
    "sumgroup_dict": (sumscan_segment, [
        ("sel_10pct", "SELECT daysSinceEpoch, COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17201 "
                      "GROUP BY daysSinceEpoch LIMIT 2000", 0),
        ("sel_50pct", "SELECT daysSinceEpoch, COUNT(*), SUM(m) FROM t WHERE daysSinceEpoch BETWEEN 17100 AND 17611 "
                      "GROUP BY daysSinceEpoch LIMIT 2000", 0),
    ]),
    # configs[1]: bench.py's AdAnalytics segments and README query (execution statistics: --exec-stats)
    "adanalytics": (lambda seed, docs: _bench().make_segment(seed, docs), [
        ("readme", None, 0),
    ]),
    # configs[1]'s columns with the accountId IN list widened (bench.py's secondary lines): 10 % / 50 % of the docs
    "adanalytics_in": (lambda seed, docs: _bench().make_segment(seed, docs), [
        ("sel_10pct", "@17476", 0),
        ("sel_50pct", "@87381", 0),
    ]),
    "highcard": (highcard_segment, [
        ("all_docs", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                     "OPTION(numGroupsLimit=2000000)", 0),
        ("filtered_10pct", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t WHERE m < 6554 GROUP BY d1, d2 "
                           "LIMIT 2000000 OPTION(numGroupsLimit=2000000)", 0),
        # decomposition of all_docs (which part of the work costs what)
        ("count_only", "SELECT d1, d2, COUNT(*) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                       "OPTION(numGroupsLimit=2000000)", 0),
        ("minmax_only", "SELECT d1, d2, MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                        "OPTION(numGroupsLimit=2000000)", 0),
        ("sum_only", "SELECT d1, d2, SUM(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                     "OPTION(numGroupsLimit=2000000)", 0),
        # the default numGroupsLimit (100000 < 1M keys): first-seen trimming per segment (a11)
        ("default_limit", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000", 0),
    ]),
    # configs[2] over segments with their own dictionaries (count-free emit: per-segment key / value id offsets)
    "highcard_own": (highcard_own_segment, [
        ("all_docs", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                     "OPTION(numGroupsLimit=2000000)", 0),
        ("filtered_10pct", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t WHERE m < 6554 GROUP BY d1, d2 "
                           "LIMIT 2000000 OPTION(numGroupsLimit=2000000)", 0),
        ("default_limit", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000", 0),
    ]),
    "highcard_rd": (highcard_rd_segment, [
        ("all_docs", "SELECT d1, d2, SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1, d2 LIMIT 2000000 "
                     "OPTION(numGroupsLimit=2000000)", 0),
    ]),
    "star": (star_segment, [
        ("all_docs", "SELECT d1, d2, d3, d4, SUM(r), DISTINCTCOUNTHLLMV(tags) FROM t GROUP BY d1, d2, d3, d4 "
                     "LIMIT 1000000 OPTION(numGroupsLimit=1000000)", 0),
        # decomposition of all_docs (which part of the work costs what)
        ("count_only", "SELECT d1, d2, d3, d4, COUNT(*) FROM t GROUP BY d1, d2, d3, d4 "
                       "LIMIT 1000000 OPTION(numGroupsLimit=1000000)", 0),
        ("sum_only", "SELECT d1, d2, d3, d4, SUM(r) FROM t GROUP BY d1, d2, d3, d4 "
                     "LIMIT 1000000 OPTION(numGroupsLimit=1000000)", 0),
        ("hll_only", "SELECT d1, d2, d3, d4, DISTINCTCOUNTHLLMV(tags) FROM t GROUP BY d1, d2, d3, d4 "
                     "LIMIT 1000000 OPTION(numGroupsLimit=1000000)", 0),
        # the default numGroupsLimit (100000 < 262144 keys): first-seen trimming per segment (walk form: SV group-by)
        ("default_limit", "SELECT d1, d2, d3, d4, SUM(r), DISTINCTCOUNTHLLMV(tags) FROM t GROUP BY d1, d2, d3, d4 "
                          "LIMIT 1000000", 0),
    ]),
    # MV group-by (a doc expands into one key per value of tags): 64 x 4096 keys, so the default numGroupsLimit (100000)
    # binds in every segment and the sorted-form first-seen trimming runs (a11'); untrimmed for comparison
    "mvgroup": (star_segment, [
        ("untrimmed", "SELECT d3, tags, COUNT(*), SUM(r) FROM t GROUP BY d3, tags LIMIT 1000000 "
                      "OPTION(numGroupsLimit=1000000)", 0),
        ("default_limit", "SELECT d3, tags, COUNT(*), SUM(r) FROM t GROUP BY d3, tags LIMIT 1000000", 0),
    ]),
}


CHECK_LINES = ("all_docs", "filtered_10pct", "default_limit")


def oracle_check(ex, q, host_segs, sp, rel=0.0):
    """The full-size line's result (every segment of the run) against the oracle's server-level result of the same
    segments, outside the timed region (--check; test infrastructure, as bench.py's oracle_check): keys, counts,
    numDocsScanned, numGroupsLimitReached and every aggregation bit-exact (tests/test_gpu_configs.py _compare_arrays),
    except a SUM over a raw DOUBLE column (rel: the tests' DOUBLE_REL, the atomic order differs from docId order)."""
    import numpy as np
    import oracle
    from pinot_amd import _lib as L
    ex.execute(sp)
    keys, counts, outs = ex.fetch_arrays(sp)
    t0 = time.perf_counter()
    exp = oracle.run_query_arrays(q, host_segs)
    res = {"docs": int(sum(s.num_docs for s in host_segs)), "groups": int(len(exp["keys"])),
           "oracle_s": round(time.perf_counter() - t0, 1)}
    try:
        assert int(L.lib().pa_query_matched_docs(ex.handle)) == exp["matched"], "numDocsScanned"
        assert (int(L.lib().pa_query_num_groups_limit_reached(ex.handle)) > 0) == exp["limit_reached"], "limit"
        np.testing.assert_array_equal(keys, exp["keys"])
        np.testing.assert_array_equal(counts, exp["counts"])
        for a, gi, oi in zip(q.aggregations, ex.agg_map, exp["amap"]):
            if a.function != "COUNT":
                got, want = outs[gi], exp["accs"][oi]
                if rel and a.function == "SUM":
                    np.testing.assert_allclose(got, want, rtol=rel, atol=0, err_msg=a.function)
                    res["sum_max_rel"] = float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-300)))
                else:
                    np.testing.assert_array_equal(got.reshape(want.shape), want, err_msg=a.function)
        res["checked"] = True
    except AssertionError as e:
        res["checked"] = False
        res["error"] = str(e)[:300]
    return res


def cpu_port_baseline(sql, host_segs):
    """bench.py's cpu_baseline (the C oracle port, one segment per thread) over the kept host segments."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("pa_bench_main", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from pinot_amd import parse_sql
    return bench.cpu_baseline(parse_sql(sql), host_segs)


_BENCH = []


def _bench():
    if not _BENCH:
        import importlib.util
        spec = importlib.util.spec_from_file_location("bench_main", os.path.join(ROOT, "bench.py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        _BENCH.append(m)
    return _BENCH[0]


def run(workload, nseg, docs, reps, only=None, no_stepmajor=False, variants=None, cpu_sample=0, exec_stats=False,
        warm=0, check=False):
    import torch
    from pinot_amd import parse_sql
    from pinot_amd import _lib as L
    from pinot_amd.engine import GpuQueryExecutor, GpuSegment
    make, queries = WORKLOADS[workload]
    t0 = time.perf_counter()
    gsegs, cids, host = [], None, []
    for i in range(nseg):
        seg = make(100 + i, docs)
        if cids is None:
            cids = {n: j for j, n in enumerate(sorted(seg.columns))}
        gsegs.append(GpuSegment(seg, column_ids=cids, device=0))
        if check or len(host) < cpu_sample:
            host.append(seg)  # (kept whole for the CPU baseline)
            continue
        for c in seg.columns.values():  # HBM holds the data now; keep only the dictionaries
            c.fwd_bytes = None
            c.raw_values = None
        if (i + 1) % 10 == 0:
            log("  %d/%d segments resident, %.1f s" % (i + 1, nseg, time.perf_counter() - t0))
    log("%s: %d segments x %d docs resident (%.1f GB), %.1f s" % (
        workload, nseg, docs, sum(g.device_bytes for g in gsegs) / 1e9, time.perf_counter() - t0))
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for name, sql, flags in queries:
        if only and name != only:
            continue
        sql = sql or _bench().QUERY
        if sql.startswith("@"):
            sql = _bench().secondary_query(int(sql[1:]))
        vs = variants or (((0, ""),) if no_stepmajor else ((0, ""), (L.PA_QF_NO_LANE_MAJOR, "_stepmajor")))
        def extra_flags(vs_, tag_):
            return dict((t_, f_) for f_, t_ in vs_)[tag_]
        for extra, tag in vs:
            ex = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags | extra | (L.PA_QF_NO_FILTER_STATS if exec_stats else 0))
            ex.execute(sp)
            for _ in range(warm):  # (untimed: the clocks reach their steady state)
                ex.scan(sp)
            torch.cuda.synchronize()
            ex.reset(sp)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(reps):
                ex.scan(sp)
            b.record(stream)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / reps
            ex.execute(sp)
            torch.cuda.synchronize()  # fetch_ms = compaction + copies (+ host decode of small blocks) only
            ex.fetch_arrays(sp, pooled=True)  # (first use grows the process's pinned output pool)
            ex.fetch(sp, execution_stats=False)  # (numDocsScanned of this scan)
            t1 = time.perf_counter()
            keys, counts, outs = ex.fetch_arrays(sp, pooled=True)
            fetch_ms = (time.perf_counter() - t1) * 1e3
            # end to end: accumulator reset + scan + fetch of the groups into host arrays, one query after another
            t2 = time.perf_counter()
            for _ in range(3):
                ex.execute(sp)
                ex.fetch_arrays(sp, pooled=True)
            e2e_ms = (time.perf_counter() - t2) * 1e3 / 3
            st = ex.stats()
            extra = {}
            if check and name in CHECK_LINES:
                extra["check"] = oracle_check(ex, parse_sql(sql), host, sp, rel=1e-9 if workload == "star" else 0.0)
                log("%s %s%s: oracle check %s" % (workload, name, tag, extra["check"]))
            # roofline of the fused scan on the byte model every line shares (bench.algorithmic_bytes): staged columns
            # whole, columns read per surviving doc (and multi-value offsets / values) at 64-byte-sector granularity
            matched = int(L.lib().pa_query_matched_docs(ex.handle))
            algo = _bench().algorithmic_bytes(ex, matched)
            extra["roofline"] = {"bound": "hbm", "achieved": algo / (ms * 1e-3) / 1e9, "peak": 8000.0,
                                 "unit": "GB/s", "frac": algo / (ms * 1e-3) / 1e9 / 8000.0,
                                 "algorithmic_bytes_per_launch": algo}
            if cpu_sample:
                extra["cpu_baseline"] = cpu_port_baseline(sql, host)
            if exec_stats:
                # numEntriesScannedInFilter / PostFilter of every segment: (a) an executor whose scan does not count
                # (PA_QF_NO_FILTER_STATS: pa_query_execution_stats' GPU engine over leaf bitmaps); (b) the default
                # executor, whose scan counts a two-leaf AND's leaps itself where that applies: its scan time and the
                # statistics call after it, against the plain scan (ms)
                from pinot_amd import filter_stats as FS
                docs_total = int(L.lib().pa_query_matched_docs(ex.handle))
                ex.execution_stats(sp, docs_total)  # (warms the allocator)
                t3 = time.perf_counter()
                in_f, post = ex.execution_stats(sp, docs_total)
                plain_ms = (time.perf_counter() - t3) * 1e3
                fx = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags | extra_flags(vs, tag))
                fx.execute(sp)
                torch.cuda.synchronize()
                fx.reset(sp)
                a.record(stream)
                for _ in range(reps):
                    fx.scan(sp)
                b.record(stream)
                torch.cuda.synchronize()
                fused_scan_ms = a.elapsed_time(b) / reps
                fx.execute(sp)
                fx.fetch_arrays(sp, pooled=True)  # (numDocsScanned of this scan)
                fdocs = int(L.lib().pa_query_matched_docs(fx.handle))
                fx.execution_stats(sp, fdocs)
                t4 = time.perf_counter()
                f_in, f_post = fx.execution_stats(sp, fdocs)
                fused_host_ms = (time.perf_counter() - t4) * 1e3
                fused = int(L.lib().pa_query_leap_leaf(fx.handle)) >= 0
                fx.close()
                assert (f_in, f_post) == (in_f, post), ((f_in, f_post), (in_f, post))
                extra["exec_stats"] = {"scan_ms": round(ms, 4), "plain_stats_ms": round(plain_ms, 3),
                                       "fused": fused, "fused_scan_ms": round(fused_scan_ms, 4),
                                       "fused_host_ms": round(fused_host_ms, 3),
                                       "overhead_vs_scan": round((fused_scan_ms + fused_host_ms) / ms - 1.0, 4),
                                       "entries_in_filter": in_f, "entries_post_filter": post}
            print(json.dumps(dict({"workload": workload, "plan_name": name + tag, "kernel_ms": round(ms, 4),
                              "rows_per_s": st["num_docs"] / (ms * 1e-3), "staged_bytes": st["staged_bytes"],
                              "staged_GBps": st["staged_bytes"] / (ms * 1e-3) / 1e9, "fetch_ms": round(fetch_ms, 2), "e2e_ms": round(e2e_ms, 2),
                              "groups": int(len(keys)), "matched_docs": int(L.lib().pa_query_matched_docs(ex.handle)),
                              "plan": st["plan"], "segments": nseg, "docs_per_segment": docs}, **extra)), flush=True)
            ex.close()
    for g in gsegs:
        g.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="all")
    ap.add_argument("--segments", type=int, default=20)
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm", type=int, default=0, help="untimed scans before each line's timed ones")
    ap.add_argument("--check", action="store_true",
                    help="keep every segment on the host and check the full-size results against the oracle")
    ap.add_argument("--plan", default=None, help="only this plan name (e.g. all_docs)")
    ap.add_argument("--no-stepmajor", action="store_true", help="skip the forced step-major variants")
    ap.add_argument("--sweep-part", action="store_true",
                    help="partitioned aggregation: sweep LDS per partition x workgroups per CU")
    ap.add_argument("--flags", type=int, default=None, help="run this one PA_QF_* flag set only")
    ap.add_argument("--exec-stats", action="store_true", help="also time the execution statistics per plan")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="keep this many segments on the host: roofline + the C-port CPU baseline per line")
    args = ap.parse_args()
    variants = None if args.flags is None else [(args.flags, "_f%d" % args.flags)]
    if args.sweep_part:
        from pinot_amd import _lib as L
        variants = [(ps << L.PA_QF_PART_SHIFT | wg << L.PA_QF_WG_SHIFT, "_part%d_wg%d" % (ps, wg))
                    for ps in (1, 2, 3) for wg in (0, 1, 2)]
    import torch
    torch.cuda.set_device(0)
    for w in (WORKLOADS if args.workload == "all" else [args.workload]):
        run(w, args.segments, args.docs, args.reps, args.plan, args.no_stepmajor, variants, args.cpu_sample,
            args.exec_stats, args.warm, args.check)


if __name__ == "__main__":
    main()
