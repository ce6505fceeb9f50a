import sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_gpu_parity import make_segment
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
cols = {"k1": ("INT", 700), "k2": ("LONG", 900), "m": ("INT", 5000), "big": ("LONG", 3000), "f": ("DOUBLE", 800), "g": ("FLOAT", 600)}
segs = [make_segment(70 + i, n, cols) for i, n in enumerate((120011, 40009))]
gsegs = [GpuSegment(sg) for sg in segs]
for sql in ["SELECT k1, k2, COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t GROUP BY k1, k2 LIMIT 1000000 OPTION(numGroupsLimit=2000000)",
            "SELECT k2, k1, SUM(big), MIN(big), MAX(f), SUM(f), MIN(g) FROM t WHERE m > 10 GROUP BY k2, k1 LIMIT 1000000 OPTION(numGroupsLimit=2000000)"]:
    ex = GpuQueryExecutor(parse_sql(sql), gsegs)
    print(ex.stats())
