"""Per-kernel average of every PMC counter in the rocprofv3 counter_collection CSVs under a directory (one row per
kernel name prefix), plus derived per-dispatch figures: HBM read bytes (FETCH_SIZE KiB x2 on gfx950, see
MI355X_MICROARCH.md HBM section), write bytes, and the SQ cycle split (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as
fractions of WAVE_CYCLES)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name.replace("void ", ""))
    return name[:90]


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        a["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in a:
            a["hbm_read_MB"] = a["FETCH_SIZE"] * 1024 * 2 / 1e6
        if "WRITE_SIZE" in a:
            a["hbm_write_MB"] = a["WRITE_SIZE"] * 1024 / 1e6
        w = a.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if c in a:
                    a["frac_" + c[3:]] = round(a[c] / w, 3)
        out[k] = {c: (round(v, 3) if isinstance(v, float) else v) for c, v in sorted(a.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
