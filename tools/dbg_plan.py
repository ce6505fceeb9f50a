import sys; sys.path.insert(0, '.')
from tests.synth import make_segment
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
cols = {"k1": ("INT", 40), "k2": ("INT", 30), "k3": ("LONG", 20), "k4": ("INT", 16), "ri": ("INT", 500),
        "rl": ("LONG", 0), "rd": ("DOUBLE", 0), "rf": ("FLOAT", 0)}
segs = [make_segment(90, 150007, cols, no_dict=("ri", "rl", "rd", "rf")), make_segment(92, 60001, cols, no_dict=("rl", "rd", "rf"))]
gsegs = [GpuSegment(sg) for sg in segs]
for agg in ("SUM(ri), MIN(ri)", "SUM(rl), MAX(rl)"):
    sql = ("SELECT k1, k2, k3, k4, COUNT(*), %s FROM t GROUP BY k1, k2, k3, k4 LIMIT 10000000 OPTION(numGroupsLimit=10000000)" % agg)
    ex = GpuQueryExecutor(parse_sql(sql), gsegs)
    print(agg, ex.stats()["plan"], flush=True)
    ex.close()
