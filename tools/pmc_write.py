"""Write profiles/pmc_<workload>.json (bench.py's roofline.traffic source) from a tools/profile.sh output directory:
HBM bytes per launch of one kernel from the separate FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE KiB x 1024 x 2 on
gfx950, MI355X_MICROARCH.md HBM section), its rocprof average duration from the kernel-trace pass, and the SQ pass.

python tools/pmc_write.py <profile dir> <workload> <kernel name substring> <docs per segment> <segments> <tree> <out>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d, workload, kname, docs, nseg, tree, out):
    pmc = defaultdict(list)
    kernels = set()
    for sub in ("sq", "fetch", "write"):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            if kname in r.get("Kernel_Name", ""):
                kernels.add(r["Kernel_Name"].split("(")[0])
                pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    agg = {k: sum(v) / len(v) for k, v in pmc.items() if v}
    stats = [r for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")) if kname in r["Name"]]
    res = {
        "workload": workload,
        "docs_per_segment": int(docs),
        "segments": int(nseg),
        "kernel": sorted(kernels),
        "tree": tree,
        "source": "%s (tools/profile.sh: rocprofv3 --kernel-trace --stats, then --pmc SQ_*, FETCH_SIZE, WRITE_SIZE "
                  "in separate passes over bench.py)" % d,
        "correction": "FETCH_SIZE (KiB) x 1024 x 2: gfx950 reports half the bytes of wide coalesced streaming reads "
                      "(MI355X_MICROARCH.md HBM)",
        "dispatches": len(pmc.get("FETCH_SIZE", [])),
        "fetch_size_kib_avg": agg.get("FETCH_SIZE"),
        "write_size_kib_avg": agg.get("WRITE_SIZE"),
    }
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        res["hbm_read_bytes_per_launch"] = agg["FETCH_SIZE"] * 1024 * 2
        res["hbm_write_bytes_per_launch"] = agg["WRITE_SIZE"] * 1024
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    if stats:
        res["rocprof_avg_kernel_ns"] = float(stats[0]["AverageNs"])
        res["rocprof_calls"] = int(stats[0]["Calls"])
    res["sq"] = {k: v for k, v in sorted(agg.items()) if k.startswith("SQ_")}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res.get(k) for k in ("kernel", "dispatches", "hbm_read_bytes_per_launch",
                                              "hbm_write_bytes_per_launch", "rocprof_avg_kernel_ns")}))


if __name__ == "__main__":
    main(*sys.argv[1:8])
