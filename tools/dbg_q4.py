import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import oracle
from pinot_amd import parse_sql, _lib as L
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from synth import make_segment
from test_gpu_parity import COLS, RAW, QUERIES, _fill
seed = 3
sizes = [(20011, 5000), (8191, 70001), (1, 2049)][seed - 1]
segs = [make_segment(seed * 100 + i, n, COLS, no_dict=RAW) for i, n in enumerate(sizes)]
for qi in (4, 3, 1):
    sql = _fill(QUERIES[qi], segs[0])
    q = parse_sql(sql)
    exp = oracle.run_query(q, segs)
    for flags in (0, L.PA_QF_FORCE_GLOBAL, L.PA_QF_NO_LANE_MAJOR, L.PA_QF_STAGE_ALL):
        for subset in ([0], [1], [0, 1]):
            gs = [GpuSegment(segs[i]) for i in subset]
            ex = GpuQueryExecutor(q, gs, flags=flags)
            got = ex.run()
            st = ex.stats()
            e2 = oracle.run_query(q, [segs[i] for i in subset])
            print(qi, flags, subset, "gpu", got.num_docs_scanned, "ora", e2.num_docs_scanned,
                  "groups", len(got.groups), len(e2.groups), st["plan"], flush=True)
            ex.close()
            for g in gs:
                g.close()
