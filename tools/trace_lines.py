"""Per-line rocprof summary of bench.py's secondary lines from one `rocprofv3 --kernel-trace` run of bench.py: the
gdl_jit dispatches in launch order, one block of (warmup + 1 + steps) per secondary line, next to the line's own
HIP-event kernel_ms (bench.py's JSON line of the same run).

python tools/trace_lines.py <kernel_trace.csv> <bench json> <out json> [kernel prefix] [dispatches per line]
"""
import csv
import json
import sys


def main(trace, bench, out, prefix="gdl_jit", per_line=71):  # (bench.py defaults: 20 warmup + 50 steps + 1)
    per_line = int(per_line)
    rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].startswith(prefix)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    line = json.loads(open(bench).readline())
    res = {"source": trace, "kernel": prefix, "dispatches_per_line": per_line, "lines": []}
    for i, s in enumerate(line.get("secondary", [])):
        blk = dur[per_line * i:per_line * (i + 1)]
        if len(blk) < per_line:
            break
        avg = sum(blk) / len(blk)
        res["lines"].append({"workload": s["workload"], "bench_kernel_ms": s["kernel_ms"],
                             "rocprof_avg_ms": round(avg, 5),
                             "rocprof_avg_last_steps_ms": round(sum(blk[-20:]) / 20, 5),
                             "rel_diff": round(avg / s["kernel_ms"] - 1.0, 4),
                             "bench_frac": s["roofline"]["frac"]})
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for x in res["lines"]:
        print(x["workload"], x["bench_kernel_ms"], x["rocprof_avg_ms"], x["rel_diff"])


if __name__ == "__main__":
    main(*sys.argv[1:6])
