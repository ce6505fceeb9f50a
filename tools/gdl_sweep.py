"""Measurement of the query-shape specialised dense kernel (gdl_jit.hip) on bench.py's secondary lines: one segment set
built once, then every knob setting (environment variables read at query prepare) timed with HIP events around
back-to-back scans. Settings: default plan; waves / docs per lane / rows shared by two waves (PA_GDL_W, PA_GDL_ND,
PA_GDL_RS), tile images per wave (PA_GDL_RING); the decomposition stream-only / + filter / + keys and terms without
the row atomics (PA_GDL_DBG=1 / 2 / 3: results invalid, not checked). Every other
setting's groups must equal the default plan's.

python tools/gdl_sweep.py [--segments 100] [--docs 10000000] [--own] [--lines sel_10pct,sel_50pct] [--reps 10]
Prints one JSON line per (line, setting).
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SETTINGS = [
    ("default", {}),
    ("stream_only", {"PA_GDL_DBG": "1"}),
    ("stream_filter", {"PA_GDL_DBG": "2"}),
    ("w16_nd8_rs2", {"PA_GDL_W": "16", "PA_GDL_ND": "8", "PA_GDL_RS": "2"}),
    ("w8_nd8", {"PA_GDL_W": "8", "PA_GDL_ND": "8", "PA_GDL_RS": "1"}),
    ("w8_nd16_rs2", {"PA_GDL_W": "8", "PA_GDL_ND": "16", "PA_GDL_RS": "2"}),
    ("rr1", {"PA_GDL_RR": "1"}),
    ("w16_nd8", {"PA_GDL_W": "16", "PA_GDL_ND": "8", "PA_GDL_RS": "1"}),
    ("walk_no_atomics", {"PA_GDL_DBG": "3"}),
    ("w12_nd8", {"PA_GDL_W": "12", "PA_GDL_ND": "8", "PA_GDL_RS": "1"}),
    ("w12_nd16", {"PA_GDL_W": "12", "PA_GDL_ND": "16", "PA_GDL_RS": "1"}),
    ("w8_nd8_pin", {"PA_GDL_W": "8", "PA_GDL_ND": "8", "PA_GDL_RS": "1"}),
    ("w16_nd16", {"PA_GDL_W": "16", "PA_GDL_ND": "16", "PA_GDL_RS": "1"}),
    ("ring3", {"PA_GDL_RING": "3"}),
    ("ring4", {"PA_GDL_RING": "4"}),
    ("ring3_w8_nd8", {"PA_GDL_RING": "3", "PA_GDL_W": "8", "PA_GDL_ND": "8"}),
    ("ring3_w8_nd16", {"PA_GDL_RING": "3", "PA_GDL_W": "8", "PA_GDL_ND": "16"}),
    ("ring3_w16_nd8", {"PA_GDL_RING": "3", "PA_GDL_W": "16", "PA_GDL_ND": "8"}),
    ("ring3_rr1", {"PA_GDL_RING": "3", "PA_GDL_RR": "1"}),
    ("default_b", {}),
]
KNOBS = ("PA_GDL_W", "PA_GDL_ND", "PA_GDL_RS", "PA_GDL_DBG", "PA_GDL_RR", "PA_GDL_RING")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=100)
    ap.add_argument("--docs", type=int, default=10_000_000)
    ap.add_argument("--own", action="store_true", help="the own-dictionary segment set and lines")
    ap.add_argument("--lines", default=None)
    ap.add_argument("--settings", default=None, help="comma-separated setting names")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm", type=int, default=0, help="untimed scans before the timed ones (clocks at steady state)")
    args = ap.parse_args()
    spec = importlib.util.spec_from_file_location("bench_main", os.path.join(ROOT, "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    import torch
    from pinot_amd import _lib as L
    from pinot_amd import parse_sql
    from pinot_amd.engine import GpuQueryExecutor, GpuSegment
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    gsegs, cids = [], None
    for i in range(args.segments):
        seg = B.make_segment_own(5000 + i, args.docs, i) if args.own else B.make_segment(1000 + i, args.docs)
        if cids is None:
            cids = {n: j for j, n in enumerate(sorted(seg.columns))}
        gsegs.append(GpuSegment(seg, column_ids=cids, device=0))
        for c in seg.columns.values():
            c.fwd_bytes = None
    print("segments resident %.1f s" % (time.perf_counter() - t0), file=sys.stderr, flush=True)
    lines = B.OWN_SECONDARY if args.own else B.SECONDARY
    if args.lines:
        lines = [x for x in lines if x[0] in args.lines.split(",")]
    settings = SETTINGS if not args.settings else [s for s in SETTINGS if s[0] in args.settings.split(",")]
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for name, n_ids in lines:
        sql = B.secondary_query_own(n_ids, args.segments) if args.own else B.secondary_query(n_ids)
        ref = None
        for sname, env in settings:
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(env)
            ex = GpuQueryExecutor(parse_sql(sql), gsegs)
            try:
                plan = ex.stats()["plan"]
                ex.execute(sp)
                torch.cuda.synchronize()
                for _ in range(args.warm):
                    ex.scan(sp)
                ex.reset(sp)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(args.reps):
                    ex.scan(sp)
                b.record(stream)
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / args.reps
                ex.execute(sp)
                keys, counts, outs = ex.fetch_arrays(sp)
                matched = int(L.lib().pa_query_matched_docs(ex.handle))
                algo = B.algorithmic_bytes(ex, matched)
                same = None
                if "PA_GDL_DBG" not in env:
                    cur = (keys.tolist(), counts.tolist(), [o.tolist() for o in outs])
                    ref = cur if ref is None else ref
                    same = cur == ref
            finally:
                ex.close()
            print(json.dumps({"line": name, "own_dictionaries": args.own, "setting": sname, "env": env,
                              "kernel_ms": round(ms, 4), "frac": round(algo / (ms * 1e-3) / 8e12, 4),
                              "algorithmic_bytes": algo, "dense_packed": plan["dense_packed"],
                              "variant": plan["variant"], "lds_bytes": plan["lds_bytes"], "same_groups": same}),
                  flush=True)
    for k in KNOBS:
        os.environ.pop(k, None)
    for g in gsegs:
        g.close()


if __name__ == "__main__":
    main()
