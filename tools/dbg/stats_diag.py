"""Diagnostic: pa_query_filter_counts vs host bitmaps per leaf / pair (GPU), 3 segments in one executor."""
import sys
sys.path[:0] = [".", "tests"]
import numpy as np
from pinot_amd import filter_stats as FS, parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from test_gpu_stats import _segment
from test_filter_stats import np_leaps

segs = [_segment(1, 200_003), _segment(2, 70_000), _segment(3, 1025)]
gs = [GpuSegment(s) for s in segs]
q = parse_sql("SELECT COUNT(*) FROM t WHERE a < 30 AND b < 30")
ex = GpuQueryExecutor(q, gs)
reqs = {}
for si in range(3):
    for k in [((0,), ()), ((1,), ()), ((0,), (1,))]:
        reqs[(si,) + k] = len(reqs)
out = FS.device_counts(ex, ex.segs, reqs)
for si in range(3):
    bm = ex.leaf_bitmaps(si)
    a, b = bm[0], bm[1]
    print(si, "dev", out[3 * si:3 * si + 3].tolist())
    print(si, "host", [int(a.sum()), int(b.sum()), int((a & b).sum()), np_leaps(a, b)])
print(ex.execution_stats(), FS.server_stats(q, ex.segs, lambda si: ex.leaf_bitmaps(si)))
ex.close()
