"""Headline benchmark: rows/sec scanned + %HBM roofline for filter + GROUP BY SUM (BASELINE.json).

Workload (BASELINE.json configs[1]): the README AdAnalytics query
  SELECT sum(clicks), sum(impressions) FROM AdAnalyticsTable
  WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789)
  GROUP BY daysSinceEpoch TOP 100
over 1B rows = 100 synthetic segments x 10M docs PER GPU (weak scaling: N GPUs scan N billion rows; configs[3]).
Columns are dictionary-encoded fixed-bit forward indexes (daysSinceEpoch INT 512 days = 9 bits, accountId INT
2^17 accounts = 17 bits, clicks LONG 1024 values = 10 bits, impressions LONG 16384 values = 14 bits), with
uniformly random dictIds; data is synthetic, generated on the host and resident in HBM before timing.

A step = one execution of the query over the rank's whole segment set: accumulator reset + the fused HIP scan
kernel + (N>1) the RCCL reduce of partial aggregates to rank 0 + rank 0's fetch/decode of the groups.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rows/sec scanned + %HBM roofline, filter+GROUP BY SUM at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
QUERY = ("SELECT sum(clicks), sum(impressions) FROM AdAnalyticsTable WHERE daysSinceEpoch BETWEEN 17849 AND 17856 "
         "AND accountId IN (123456789) GROUP BY daysSinceEpoch TOP 100")
COLUMNS = {  # name: (type, cardinality, dictionary values)
    "daysSinceEpoch": ("INT", 512, lambda: np.arange(17532, 17532 + 512, dtype=np.int64)),
    "accountId": ("INT", 1 << 17, lambda: 123456789 + (np.arange(1 << 17, dtype=np.int64) - (1 << 16)) * 997),
    "clicks": ("LONG", 1024, lambda: np.arange(1024, dtype=np.int64)),
    "impressions": ("LONG", 1 << 14, lambda: np.arange(1 << 14, dtype=np.int64) * 3),
}


# Secondary lines (same columns and segments): the accountId IN list widened so the filter + GROUP BY SUM aggregates a
# tenth / half of the docs (day range: 384 of the 512 days, 75 %; IN list: 13.3 % / 66.7 % of the 2^17 account ids).
DAY_RANGE = (17532, 17915)
SECONDARY = (("sel_10pct", 17476), ("sel_50pct", 87381))


# Own-dictionary lines: the same columns where every segment built its own dictionaries (SegmentDictionaryCreator.java:104,
# one per segment), as in a time-partitioned table: a 4-day slice of daysSinceEpoch (2 bits), a random half of the 2^17
# accounts (16 bits), clicks a run of 1024 values and impressions 16384 values of step 3, each from a per-segment
# offset. The day range covers every segment's slice; the IN list keeps a tenth / half of the docs.
OWN_DAYS = 4
OWN_SECONDARY = (("sel_10pct_own_dicts", 13107), ("sel_50pct_own_dicts", 65536))


def make_segment_own(seed, docs, index):
    from pinot_amd.segment import segment_from_dict_ids
    rng = np.random.default_rng(seed)
    accts = np.sort(rng.choice(COLUMNS["accountId"][2](), size=1 << 16, replace=False))
    d0 = DAY_RANGE[0] + OWN_DAYS * index
    dicts = {"daysSinceEpoch": ("INT", np.arange(d0, d0 + OWN_DAYS, dtype=np.int64)),
             "accountId": ("INT", accts),
             "clicks": ("LONG", np.arange(1024, dtype=np.int64) + (index * 37) % 500),
             "impressions": ("LONG", (np.arange(1 << 14, dtype=np.int64) + (index * 101) % 2000) * 3)}
    specs = {}
    for name, (dt, d) in dicts.items():
        nb = int(len(d) - 1).bit_length()  # (every cardinality a power of two: uniform dictIds = random bytes)
        specs[name] = (dt, d, np.frombuffer(rng.bytes((docs * nb + 7) // 8), dtype=np.uint8))
    return segment_from_dict_ids("AdAnalyticsOwn_%d" % seed, docs, specs)


def secondary_query_own(n_ids, num_segments):
    ids = np.sort(np.random.default_rng(4243).choice(COLUMNS["accountId"][2](), size=n_ids, replace=False))
    return ("SELECT sum(clicks), sum(impressions) FROM AdAnalyticsTable WHERE daysSinceEpoch BETWEEN %d AND %d "
            "AND accountId IN (%s) GROUP BY daysSinceEpoch TOP 1000" % (
                DAY_RANGE[0], DAY_RANGE[0] + OWN_DAYS * num_segments - 1, ",".join(map(str, ids))))


def secondary_query(n_ids):
    ids = np.sort(np.random.default_rng(4242).choice(COLUMNS["accountId"][2](), size=n_ids, replace=False))
    return ("SELECT sum(clicks), sum(impressions) FROM AdAnalyticsTable WHERE daysSinceEpoch BETWEEN %d AND %d "
            "AND accountId IN (%s) GROUP BY daysSinceEpoch TOP 100" % (DAY_RANGE + (",".join(map(str, ids)),)))


def L_lib():
    from pinot_amd import _lib
    return _lib.lib()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _touched(p, per_sector):
    """Fraction of 64-byte sectors holding at least one doc of a uniform selection of density p."""
    p = min(1.0, max(0.0, p))
    return 1.0 - (1.0 - p) ** max(1.0, per_sector)


def algorithmic_bytes(ex, matched):
    """HBM bytes one launch of the query's scan must read (the byte model of every roofline line): a column
    the plan stages is read whole (nb / 8 bytes per doc for a dictionary column, the value bytes for a raw one); a column
    read per surviving doc costs the 64-byte sectors holding a surviving doc, at the query's final density (lazy filter
    clauses run at a density >= that: the model undercounts them); a multi-value column also its per-doc value offsets
    (4 bytes) and its values' bits, sector-wise."""
    from pinot_amd import _lib as L
    q = ex.query
    from pinot_amd.query import query_columns
    names = query_columns(q)
    docs = sum(sg.num_docs for sg in ex.segs)
    p = matched / max(1, docs)
    total = 0.0
    for name in names:
        staged = L.lib().pa_query_column_staged(ex.handle, ex.gsegs[0].column_ids[name]) == 1
        for sg in ex.segs:
            c = sg.column(name)
            if not c.has_dictionary:
                vb = 4 if c.data_type in ("INT", "FLOAT") else 8
                total += sg.num_docs * vb * (1.0 if staged else _touched(p, 64 / vb))
            elif c.single_value:
                total += sg.num_docs * c.num_bits / 8 * (1.0 if staged else _touched(p, 512 / c.num_bits))
            else:
                total += sg.num_docs * 4 * _touched(p, 16)
                total += c.total_num_values * c.num_bits / 8 * _touched(p * c.total_num_values / max(1, sg.num_docs),
                                                                         512 / c.num_bits)
    return int(total)


def make_segment(seed, docs):
    from pinot_amd.segment import segment_from_dict_ids
    rng = np.random.default_rng(seed)
    specs = {}
    for name, (dt, card, dvals) in COLUMNS.items():
        nb = int(card - 1).bit_length()
        nbytes = (docs * nb + 7) // 8
        # uniform dictIds over [0, 2^nb) == uniformly random bytes, because card == 2^nb
        specs[name] = (dt, dvals(), np.frombuffer(rng.bytes(nbytes), dtype=np.uint8))
    return segment_from_dict_ids("AdAnalytics_%d" % seed, docs, specs)


def load_traffic(workload, docs, nseg):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), if it matches this shape."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if d.get("docs_per_segment") == docs and d.get("segments") == nseg:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def cpu_baseline(query, host_segments, min_wall_s=1.0):
    """Oracle (the scalar C port of the reference's per-doc path) on the host cores, one segment per thread like the
    reference's combine operator's per-segment tasks; passes over the segment sample repeat until min_wall_s so the
    sample is ~10-20 CPU-seconds at 16 threads."""
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cores = max(1, min(16, cores, len(host_segments)))
    oracle.lib()
    passes = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        while True:
            list(ex.map(lambda s: oracle.run_segment(query, s), host_segments))
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= min_wall_s:
                break
    rows = passes * sum(s.num_docs for s in host_segments)
    return {"value": rows / dt, "unit": "rows/s", "cores": cores, "kind": "port",
            "sample": "%d pass(es) over %d segments x %d docs, %d threads, %.2f s wall" % (
                passes, len(host_segments), host_segments[0].num_docs, cores, dt)}


def oracle_check(q, gsegs, host_segments, sptr):
    """A line's own result checked outside the timed region: the same query over the host sample's segments (the first
    len(host_segments) of the rank's set, whose forward indexes the host kept) on the GPU, against the oracle's
    server-level result of those segments (one oracle task per segment, merged by group key: COUNT and SUM add).
    Bar as in tests/: bit-exact group keys, COUNT, numDocsScanned and LONG SUMs (all below 2^53 here)."""
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    from pinot_amd.engine import GpuQueryExecutor
    assert all(a.function in ("COUNT", "SUM") for a in q.aggregations)
    ex = GpuQueryExecutor(q, gsegs[:len(host_segments)])
    try:
        plan = ex.stats()["plan"]
        got = ex.run(sptr)
    finally:
        ex.close()
    with ThreadPoolExecutor(max(1, min(16, len(host_segments)))) as tp:
        parts = list(tp.map(lambda s: oracle.run_query(q, [s]), host_segments))
    groups, scanned = {}, 0
    for r in parts:
        scanned += r.num_docs_scanned
        for k, v in r.groups.items():
            groups[k] = [a + b for a, b in zip(groups[k], v)] if k in groups else list(v)
    ok = got.num_docs_scanned == scanned and set(got.groups) == set(groups) and all(
        list(got.groups[k]) == list(v) for k, v in groups.items())
    if not ok:
        log("oracle check FAILED: %d vs %d docs, %d vs %d groups" % (got.num_docs_scanned, scanned, len(got.groups),
                                                                    len(groups)))
    return {"checked": bool(ok), "check_segments": len(host_segments), "check_docs": scanned,
            "check_groups": len(groups), "check_plan": plan["variant"], "check_dense_packed": plan["dense_packed"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (20 warmup steps, ~10 ms of scans: with 3 the first timed launches still ran at the clocks of the idle setup
    # phase, ~4 % slower than the same plan measured warm by tools/sweep.py)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--segments", type=int, default=100, help="segments per GPU")
    ap.add_argument("--docs", type=int, default=10_000_000, help="docs per segment")
    ap.add_argument("--cpu-sample", type=int, default=16, help="segments in the CPU baseline sample (0 = skip)")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--no-secondary", action="store_true", help="skip the widened-IN-list secondary lines")
    ap.add_argument("--secondary", default="all",
                    help="run only this secondary line (sel_10pct | sel_50pct | sel_10pct_own_dicts | sel_50pct_own_dicts)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    # under a torch.distributed launcher (RANK set) the RCCL path runs even at world size 1 (rehearsal of N>1)
    distributed = world > 1 or "RANK" in os.environ
    if distributed:
        import torch.distributed as dist
        # RCCL prints its version banner on stdout when the first communicator comes up: send it to stderr, so that
        # stdout holds only the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("nccl", device_id=device)
            dist.barrier()
            torch.cuda.synchronize()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    from pinot_amd import parse_sql
    from pinot_amd.engine import GpuQueryExecutor, GpuSegment
    from pinot_amd.parallel import DistributedAccumulators, shard_segments, table_layout

    q = parse_sql(QUERY)
    total_segments = args.segments * world
    mine = shard_segments(total_segments, rank, world)
    t_setup = time.perf_counter()
    gsegs, host_sample = [], []
    cids = None
    for i in mine:
        seg = make_segment(1000 + i, args.docs)
        if cids is None:
            cids = {n: j for j, n in enumerate(sorted(seg.columns))}
        gsegs.append(GpuSegment(seg, column_ids=cids, device=local))
        if rank == 0 and len(host_sample) < args.cpu_sample:
            host_sample.append(seg)
        else:
            for c in seg.columns.values():  # HBM holds the forward index now; keep only the dictionaries
                c.fwd_bytes = None
    log("rank %d: %d segments (%d rows) resident, %.1f GB HBM, setup %.1f s" % (
        rank, len(gsegs), sum(g.segment.num_docs for g in gsegs), sum(g.device_bytes for g in gsegs) / 1e9,
        time.perf_counter() - t_setup))

    # N>1: every rank groups over the same table-wide dictionaries (union over all ranks' segments), so key ids line up
    # across GPUs and the partial aggregates reduce element-wise
    # (and on the SUM accumulator widths), so the accumulator blocks line up element for element
    kw = table_layout(q, [g.segment for g in gsegs]).executor_kwargs() if distributed else {}
    ex = GpuQueryExecutor(q, gsegs, flags=args.flags, **kw)
    dacc = DistributedAccumulators(ex, device) if distributed else None
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    def step():
        ex.execute(sptr)
        if dacc is not None:
            dacc.reduce(dst=0, execution_stats=False)
        if rank == 0:
            return ex.fetch(sptr, execution_stats=False)
        return None

    def step_with_stats():
        """The same step plus the DataTable execution statistics every results block carries (BaseResultsBlock.java:194):
        each rank (server) counts numEntriesScannedInFilter of its own segments after its scan."""
        ex.execute(sptr)
        in_filter, _ = ex.execution_stats(sptr, docs_total=0)
        if dacc is not None:
            dacc.reduce(dst=0, execution_stats=False)
        if rank == 0:
            r = ex.fetch(sptr, execution_stats=False)
            r.num_entries_scanned_in_filter = in_filter
            return r
        return None

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()

    def kernel_time(e, n):
        """Per-launch scan time: HIP events on the launch stream around n back-to-back launches (one accumulator reset
        before the first event; the scans keep accumulating, which changes no byte the kernel reads)."""
        e.reset(sptr)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(n):
            e.scan(sptr)
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n

    # scan-kernel-only timing (per-launch duration = elapsed / steps, the figure rocprofv3 --stats averages)
    kernel_ms = kernel_time(ex, args.steps)
    multi = None
    if distributed:
        # per-rank evidence for a scaling record: each rank's scan time, the merge's time (the RCCL collective of the
        # partial aggregates alone, back to back) and the ranks the process group holds
        torch.cuda.synchronize()
        ma, mb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ma.record(stream)
        for _ in range(args.steps):
            dacc.reduce(dst=0, execution_stats=False)
        mb.record(stream)
        torch.cuda.synchronize()
        merge_ms = ma.elapsed_time(mb) / args.steps
        per = torch.tensor([kernel_ms, merge_ms], dtype=torch.float64, device=device)
        allr = [torch.zeros_like(per) for _ in range(world)]
        dist.all_gather(allr, per)
        multi = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                 "kernel_ms_per_rank": [float(x[0].item()) for x in allr],
                 "merge_ms_per_rank": [float(x[1].item()) for x in allr]}

    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the stats-inclusive step, timed the same way
    for _ in range(max(1, args.warmup)):
        sres = step_with_stats()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        sres = step_with_stats()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed_stats = time.perf_counter() - t1
    if distributed:
        t = torch.tensor([elapsed, elapsed_stats], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_stats = float(t[0].item()), float(t[1].item())

    # secondary lines: the same segments under the widened IN lists (kernel time, roofline on the same byte model)
    secondary = []
    own = {}  # the own-dictionary segment set, built for its lines only

    def own_segments():
        if not own:
            t = time.perf_counter()
            own["g"], own["host"] = [], []
            for i in mine:
                seg = make_segment_own(5000 + i, args.docs, i)
                own["g"].append(GpuSegment(seg, column_ids=cids, device=local))
                if rank == 0 and len(own["host"]) < args.cpu_sample:
                    own["host"].append(seg)
                else:
                    for c in seg.columns.values():
                        c.fwd_bytes = None
            own["kw"] = table_layout(q, [g.segment for g in own["g"]]).executor_kwargs() if distributed else {}
            log("rank %d: own-dictionary segments resident, %.1f s" % (rank, time.perf_counter() - t))
        return own["g"], own["host"], own["kw"]

    if not args.no_secondary:
        from pinot_amd import _lib as L
        lines = [(n, k, False) for n, k in SECONDARY] + [(n, k, True) for n, k in OWN_SECONDARY]
        for name, n_ids, own_dicts in lines:
            if args.secondary not in ("all", name):
                continue
            sql = secondary_query_own(n_ids, args.segments * world) if own_dicts else secondary_query(n_ids)
            lsegs, lhost, lkw = own_segments() if own_dicts else (gsegs, host_sample, kw)
            e2 = GpuQueryExecutor(parse_sql(sql), lsegs, flags=args.flags, **lkw)
            for _ in range(args.warmup):
                e2.execute(sptr)
            torch.cuda.synchronize()
            ms = kernel_time(e2, args.steps)
            e2.execute(sptr)
            r2 = e2.fetch(sptr) if rank == 0 else None
            matched = int(L.lib().pa_query_matched_docs(e2.handle))
            algo = algorithmic_bytes(e2, matched)
            st2 = e2.stats()
            secondary.append({
                "workload": "adanalytics_in_list_" + name, "matched_fraction": matched / st2["num_docs"],
                "query": sql[:sql.index("IN (") + 4] + "... %d account ids) GROUP BY daysSinceEpoch" % n_ids,
                "own_dictionaries": own_dicts,
                "kernel_ms": ms, "rows_per_s": st2["num_docs"] / (ms * 1e-3),
                "groups": len(r2.groups) if r2 is not None else None,
                "roofline": {"bound": "hbm", "achieved": algo / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": algo,
                             "traffic": load_traffic("adanalytics_in_list_" + name, args.docs, len(lsegs)),
                             "plan": st2["plan"]}})
            e2.close()
            if rank == 0 and lhost:
                secondary[-1].update(oracle_check(parse_sql(sql), lsegs, lhost, sptr))

    st = ex.stats()
    rows_per_gpu = st["num_docs"]
    total_rows = rows_per_gpu * world
    if rank == 0:
        # algorithmic bytes (algorithmic_bytes): the staged accountId forward index + the sectors of the lazily read
        # columns at the ~100 surviving docs
        algo_bytes = algorithmic_bytes(ex, int(res.num_docs_scanned))
        achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9
        cpu = cpu_baseline(q, host_sample) if host_sample else None
        out = {
            "metric": METRIC,
            "value": total_rows * args.steps / elapsed,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": "adanalytics_readme_query",
                "query": QUERY,
                "rows_per_gpu": rows_per_gpu,
                "segments_per_gpu": len(gsegs),
                "docs_per_segment": args.docs,
                "columns": {k: {"type": v[0], "cardinality": v[1], "bits": int(v[1] - 1).bit_length()}
                            for k, v in COLUMNS.items()},
                "parallelism": "segment-sharded dp%d, RCCL reduce of partial aggregates" % world,
                "groups": len(res.groups) if res is not None else None,
                "matched_docs_rank0": res.num_docs_scanned if res is not None else None,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_traffic("adanalytics", args.docs, len(gsegs)),
                "kernel_ms": kernel_ms,
                "algorithmic_bytes_per_launch": algo_bytes,
                "plan": st["plan"],
            },
            "cpu_baseline": cpu,
            # the same step with the execution statistics (numEntriesScannedInFilter of every segment: the scan's own
            # leap counts for this two-scan AND, pa_query_execution_stats)
            "stats_step": {"ms_per_step": elapsed_stats * 1e3 / args.steps,
                           "vs_plain_step": elapsed_stats / elapsed,
                           "num_entries_scanned_in_filter_rank0": sres.num_entries_scanned_in_filter,
                           "fused": int(L_lib().pa_query_leap_leaf(ex.handle)) >= 0},
            "secondary": secondary,
        }
        if multi is not None:
            out["multi_gpu"] = multi
        print(json.dumps(out), flush=True)
    ex.close()
    for g in gsegs + own.get("g", []):
        g.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
