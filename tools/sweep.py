"""Tile-planner sweep on the headline workload: one process, many kernel plans, HIP-event kernel times.

python tools/sweep.py [--segments 50] [--reps 10]
Prints one JSON line per configuration (plan, kernel ms, staged GB/s) and checks every non-debug configuration
returns the same groups as the automatic plan.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from pinot_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=50)
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--query", default=bench.QUERY)
    ap.add_argument("--quick", action="store_true", help="only the automatic plans")
    ap.add_argument("--only", default=None, help="run just this configuration name")
    ap.add_argument("--mode", choices=("both", "full", "stream"), default="both")
    args = ap.parse_args()
    import torch
    from pinot_amd import parse_sql
    from pinot_amd.engine import GpuQueryExecutor, GpuSegment
    torch.cuda.set_device(0)
    gsegs = []
    cids = None
    for i in range(args.segments):
        seg = bench.make_segment(1000 + i, args.docs)
        if cids is None:
            cids = {n: j for j, n in enumerate(sorted(seg.columns))}
        gsegs.append(GpuSegment(seg, column_ids=cids, device=0))
        for c in seg.columns.values():
            c.fwd_bytes = None
    q = parse_sql(args.query)
    stream = torch.cuda.current_stream()
    configs = [("auto", 0), ("auto_nolazy", L.PA_QF_NO_LAZY), ("auto_stepmajor", L.PA_QF_NO_LANE_MAJOR),
               ("auto_nolazy_stepmajor", L.PA_QF_NO_LAZY | L.PA_QF_NO_LANE_MAJOR)]
    for lazy_name, lazy_flag in (("", 0), ("_nolazy", L.PA_QF_NO_LAZY)):
        for steps_flag, steps in ((L.PA_QF_STEPS32, 32), (L.PA_QF_STEPS16, 16)):
            for ring in (2, 3, 4):
                for wg in (2, 3, 4):
                    configs.append(("s%d_r%d_wg%d%s" % (steps, ring, wg, lazy_name),
                                    lazy_flag | steps_flag | (ring << L.PA_QF_RING_SHIFT) | (wg << L.PA_QF_WG_SHIFT)))
    if args.quick:
        configs = configs[:4]
    if args.only:
        configs = [c for c in configs if c[0] == args.only]
    modes = {"both": (0, L.PA_QF_DEBUG_STREAM_ONLY), "full": (0,), "stream": (L.PA_QF_DEBUG_STREAM_ONLY,)}[args.mode]
    ref = None
    for name, flags in configs:
        for dbg in modes:
            try:
                ex = GpuQueryExecutor(q, gsegs, flags=flags | dbg)
            except L.PinotAmdError as e:
                if dbg == 0:
                    print(json.dumps({"config": name, "skipped": str(e)[:80]}), flush=True)
                break
            ex.execute(stream.cuda_stream)
            torch.cuda.synchronize()
            # back-to-back scans between one event pair (per-launch duration, as in bench.py)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(args.reps):
                ex.scan(stream.cuda_stream)
            b.record(stream)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.reps
            ex.execute(stream.cuda_stream)
            st = ex.stats()
            rec = {"config": name, "stream_only": bool(dbg), "plan": st["plan"], "kernel_ms": round(ms, 4),
                   "GBps": round(st["staged_bytes"] / ms / 1e6, 1),
                   "Grows_per_s": round(st["num_docs"] / ms / 1e6, 1)}
            if not dbg:
                res = ex.fetch(stream.cuda_stream)
                snap = {k: tuple(v) for k, v in res.groups.items()}
                if ref is None:
                    ref = snap
                rec["same_result"] = snap == ref
            print(json.dumps(rec), flush=True)
            ex.close()


if __name__ == "__main__":
    main()
