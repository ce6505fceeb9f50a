"""REGEXP_LIKE / LIKE / NOT LIKE on STRING dictionary columns through the GPU path: each segment resolves the pattern to
its matching dictIds (DictionaryBasedRegexpLikePredicateEvaluator), a DICT_SET / DICT_RANGE leaf on the GPU; results
and execution statistics (always a scan leaf: FilterOperatorUtils.java:108-117) against the oracle and the host
replay. Segments with their own dictionaries (different word sets) take different dictIds per segment."""
import numpy as np
import pytest

import oracle
from pinot_amd import filter_stats as FS
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.segment import create_segment
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

WORDS = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta", "iota", "kappa", "lambda", "mu", "nu",
         "xi", "omicron", "pi", "rho", "sigma", "tau", "upsilon", "phi", "chi", "psi", "omega", "C++", "C#", "a_b", "a+b"]


def _segment(seed, n, words):
    rng = np.random.default_rng(seed)
    w = np.array(words)
    data = {"s": w[rng.integers(0, len(w), n)], "t": w[rng.integers(0, len(w), n)],
            "d": rng.integers(0, 30, n).astype(np.int32), "m": rng.integers(0, 1000, n).astype(np.int64)}
    return create_segment("rx%d" % seed, data, {"s": "STRING", "t": "STRING", "d": "INT", "m": "LONG"},
                          inverted_index_columns=("t",))


@pytest.fixture(scope="module")
def string_segments():
    segs = [_segment(21, 70_001, WORDS), _segment(22, 30_000, WORDS[3:20]), _segment(23, 5_000, WORDS[:8])]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


WHERES = ["REGEXP_LIKE(s, 'ta$')", "s LIKE '%ta'", "s NOT LIKE 'a%'", "s LIKE 'C_+'", "s LIKE 'a\\_b'",
          "REGEXP_LIKE(s, 'e.a') AND d < 15", "REGEXP_LIKE(s, '^(alpha|omega)$') OR m < 20",
          "REGEXP_LIKE(s, 'nomatch')", "NOT REGEXP_LIKE(t, 'a') AND s LIKE '%i%'", "REGEXP_LIKE(t, 'ta') AND d = 4"]


@pytest.mark.parametrize("where", WHERES)
def test_regexp_like_results(string_segments, where):
    segs, gs = string_segments
    for sql in ("SELECT COUNT(*), SUM(m) FROM t WHERE " + where,
                "SELECT s, COUNT(*), MAX(m) FROM t WHERE %s GROUP BY s LIMIT 100" % where,
                "SELECT d, DISTINCTCOUNTHLL(t) FROM t WHERE %s GROUP BY d LIMIT 100" % where):
        q = parse_sql(sql)
        ex = GpuQueryExecutor(q, gs)
        try:
            got = ex.run()
        finally:
            ex.close()
        assert_same(got, oracle.run_query(q, segs))


@pytest.mark.parametrize("where", WHERES)
def test_regexp_like_execution_statistics(string_segments, where):
    segs, gs = string_segments
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
