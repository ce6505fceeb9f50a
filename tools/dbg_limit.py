"""Diagnostic (GPU): numGroupsLimit reached flag per trimming mode on test_num_groups_limit_not_reached's shape."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from synth import make_segment
from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment

cols = {"k1": ("INT", 1000), "k2": ("LONG", 1000), "f": ("INT", 1000)}
segs = [make_segment(70 + i, 30000, cols) for i in range(2)]
gsegs = [GpuSegment(s) for s in segs]
for sql in ("SELECT k1, k2, COUNT(*) FROM t WHERE f < 2 GROUP BY k1, k2 LIMIT 100000 OPTION(numGroupsLimit=20000)",
            "SELECT k1, k2, COUNT(*) FROM t WHERE f < 200 GROUP BY k1, k2 LIMIT 100000 OPTION(numGroupsLimit=20000)",
            "SELECT k1, k2, COUNT(*) FROM t GROUP BY k1, k2 LIMIT 100000 OPTION(numGroupsLimit=40000)"):
    for flags in (0, L.PA_QF_NO_LIMIT_WALK):
        ex = GpuQueryExecutor(parse_sql(sql), gsegs, flags=flags)
        st = ex.stats()["plan"]
        r = ex.run()
        print(sql[40:75], flags, "trim", st.get("limit_trimming"), "strategy", st.get("strategy"), "reached",
              r.num_groups_limit_reached, "groups", len(r.groups), "scanned", r.num_docs_scanned, flush=True)
        ex.close()
for g in gsegs:
    g.close()
