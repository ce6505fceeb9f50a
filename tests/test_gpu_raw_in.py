"""IN / NOT IN on no-dictionary columns as one RAW_SET leaf (RawValueBasedInPredicateEvaluatorFactory.java's value
sets: Int/Long/Float/DoubleRawValueBasedInPredicateEvaluator), any list size (each value used to be an equality leaf,
so a list longer than the 16 leaves of a query spec was refused): INT / LONG / FLOAT / DOUBLE columns, lists of 1 to
5000 values with present and absent values, NOT IN, inside AND / OR, on the scan's eager and lazy clauses, the per-doc
group-by paths and the execution statistics; identical to the oracle (which evaluates the list value by value)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same
import oracle
from pinot_amd import _lib as L
from pinot_amd import filter_stats as FS
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.segment import create_segment

pytestmark = pytest.mark.gpu


def _segment(seed, n):
    rng = np.random.default_rng(seed)
    data = {
        "d": rng.integers(0, 40, n).astype(np.int32),
        "m": rng.integers(0, 1000, n).astype(np.int64),
        "ri": rng.integers(-5000, 5000, n).astype(np.int32),
        "rl": rng.integers(-(1 << 40), 1 << 40, n) // 1000 * 1000,
        "rf": (rng.integers(-2000, 2000, n) / 8.0).astype(np.float32),
        "rd": rng.integers(-3000, 3000, n) / 16.0,
    }
    schema = {"d": "INT", "m": "LONG", "ri": "INT", "rl": "LONG", "rf": "FLOAT", "rd": "DOUBLE"}
    return create_segment("rin%d" % seed, data, schema, no_dictionary_columns=("ri", "rl", "rf", "rd"))


def _literal(v, dt):
    if dt in ("INT", "LONG"):
        return str(int(v))
    return repr(float(np.float32(v))) if dt == "FLOAT" else repr(float(v))


def _in_list(seg, col, dt, n, rng):
    """n values: about two thirds drawn from the column, the rest absent from it (or outside its range)."""
    present = np.unique(seg.column(col).raw_values)
    take = rng.choice(present, size=min(len(present), max(1, 2 * n // 3)), replace=False)
    if dt in ("INT", "LONG"):
        absent = rng.integers(1 << 20, 1 << 21, size=n - len(take)) * (7 if dt == "LONG" else 1)
    else:
        absent = rng.integers(1, 1000, size=n - len(take)) + 0.3
    vals = list(take) + list(absent)
    rng.shuffle(vals)
    return ", ".join(_literal(v, dt) for v in vals)


@pytest.fixture(scope="module")
def raw_segments():
    segs = [_segment(11, 60_001), _segment(12, 25_000)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


@pytest.mark.parametrize("col,dt", [("ri", "INT"), ("rl", "LONG"), ("rf", "FLOAT"), ("rd", "DOUBLE")])
@pytest.mark.parametrize("n", [1, 20, 300, 5000])
def test_raw_in_lists(raw_segments, col, dt, n):
    segs, gs = raw_segments
    rng = np.random.default_rng(n * 31 + len(col))
    lst = _in_list(segs[0], col, dt, n, rng)
    wheres = ["%s IN (%s)" % (col, lst), "%s NOT IN (%s) AND d < 20" % (col, lst),
              "d = 3 OR %s IN (%s)" % (col, lst), "%s IN (%s) AND m < 500" % (col, lst)]
    for where in wheres:
        for sql in ("SELECT COUNT(*), SUM(m) FROM t WHERE " + where,
                    "SELECT d, COUNT(*), MAX(m) FROM t WHERE %s GROUP BY d LIMIT 100" % where):
            q = parse_sql(sql)
            ex = GpuQueryExecutor(q, gs)
            try:
                kinds = [ex.spec.leaves[i].kind for i in range(ex.spec.num_leaves)]
                # (a one-value IN is an equality: MergeEqInFilterOptimizer's rewrite, a RAW_RANGE leaf; NOT IN stays)
                want = (L.PA_LEAF_RAW_RANGE, L.PA_LEAF_RAW_SET) if n == 1 else (L.PA_LEAF_RAW_SET,)
                assert any(k in kinds for k in want) and ex.spec.num_leaves <= 3, (sql[:80], kinds)
                got = ex.run()
            finally:
                ex.close()
            assert_same(got, oracle.run_query(q, segs))


def test_raw_in_execution_statistics(raw_segments):
    """numEntriesScannedInFilter / PostFilter with long raw IN lists: the GPU engine (one leaf per list) = the host
    replay of the reference's iterators, the replay unused."""
    segs, gs = raw_segments
    rng = np.random.default_rng(5)
    lst = _in_list(segs[0], "ri", "INT", 400, rng)
    for where in ["ri IN (%s)" % lst, "ri IN (%s) AND d < 9" % lst, "d < 30 AND ri NOT IN (%s)" % lst,
                  "ri IN (%s) OR m < 5" % lst]:
        ex = GpuQueryExecutor(parse_sql("SELECT d, SUM(m) FROM t WHERE %s GROUP BY d" % where), gs)
        try:
            ex.execute()
            res = ex.fetch()
            got = (res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter)
            want = FS.server_stats(ex.query, ex.segs, lambda si: ex.leaf_bitmaps(si))
            replayed = ex.stats_replayed_segments
        finally:
            ex.close()
        assert got == want, where
        assert replayed == 0, where
