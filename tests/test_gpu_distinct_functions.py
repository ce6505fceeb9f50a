"""DISTINCTCOUNTBITMAP (the values' Java hash codes, DistinctCountBitmapAggregationFunction.java) and
DISTINCTCOUNTRAWHLL (serialized HyperLogLog registers, DistinctCountRawHLLAggregationFunction.java) with their MV
forms on the GPU: the intermediate results (hash-code sets, register sets) and the final values equal the oracle's,
over INT / LONG / FLOAT / DOUBLE / STRING dictionaries, with and without a filter, grouped and not."""
import numpy as np
import pytest

import oracle
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.reduce import final_result_table, merge_intermediate
from pinot_amd.segment import create_segment, mv_column_from_flat
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _segment(seed, n):
    rng = np.random.default_rng(seed)
    data = {"d": rng.integers(0, 12, n).astype(np.int32), "i": rng.integers(-300, 300, n).astype(np.int32),
            "l": (rng.integers(0, 60, n) * (1 << 32) + rng.integers(0, 4, n)).astype(np.int64),
            "f": (rng.integers(-200, 200, n) / 4.0).astype(np.float32), "g": rng.integers(-900, 900, n) / 8.0,
            "s": np.array(["Aa", "BB", "C#", "x%d" % seed, "hello", "world", "ab", "ba"])[rng.integers(0, 8, n)]}
    seg = create_segment("dbm%d" % seed, data, {"d": "INT", "i": "INT", "l": "LONG", "f": "FLOAT", "g": "DOUBLE",
                                                "s": "STRING"})
    lengths = rng.integers(1, 4, size=n)
    seg.columns["tags"] = mv_column_from_flat("tags", lengths, rng.integers(0, 50, size=int(lengths.sum())).astype(
        np.uint32), np.arange(50, dtype=np.int64) * 7, "INT")
    return seg


@pytest.fixture(scope="module")
def segments():
    segs = [_segment(31, 40_000), _segment(32, 9_000)]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


QUERIES = [
    "SELECT DISTINCTCOUNTBITMAP(i), DISTINCTCOUNTBITMAP(l), DISTINCTCOUNTBITMAP(f), DISTINCTCOUNTBITMAP(g), "
    "DISTINCTCOUNTBITMAP(s) FROM t",
    "SELECT d, DISTINCTCOUNTBITMAP(l), DISTINCTCOUNTBITMAP(s), DISTINCTCOUNT(l) FROM t WHERE i > 0 GROUP BY d LIMIT 100",
    "SELECT DISTINCTCOUNTRAWHLL(i), DISTINCTCOUNTRAWHLL(s, 10), DISTINCTCOUNTHLL(i) FROM t WHERE d < 5",
    "SELECT d, DISTINCTCOUNTRAWHLL(l), DISTINCTCOUNTBITMAPMV(tags), DISTINCTCOUNTRAWHLLMV(tags) FROM t GROUP BY d "
    "ORDER BY DISTINCTCOUNTRAWHLL(l) DESC LIMIT 5",
]


@pytest.mark.parametrize("sql", QUERIES)
def test_distinct_functions(segments, sql):
    segs, gs = segments
    q = parse_sql(sql)
    ex = GpuQueryExecutor(q, gs)
    try:
        got = ex.run()
    finally:
        ex.close()
    exp = oracle.run_query(q, segs)
    assert_same(got, exp)
    assert final_result_table(merge_intermediate([got]), q) == final_result_table(merge_intermediate([exp]), q)
