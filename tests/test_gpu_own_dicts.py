"""Segments that build their own dictionaries on the query-shape specialised dense kernel (gdl_jit.hip, pa_jit.hip
jit_plan), against the oracle.

In the reference every segment builds and reads its own dictionary (SegmentDictionaryCreator.java:104,
DictionaryBasedGroupKeyGenerator.java:122); a time-partitioned table's daysSinceEpoch differs per segment by
construction. The cases drive each per-segment mechanism of the kernel:
  * column widths per segment (width classes: one tile body per class),
  * group keys shifted by a per-segment offset (each segment's dictionary a contiguous run of the table's) and group
    keys through per-segment remap tables in LDS slots (non-contiguous dictionaries),
  * DICT_SET bitmaps and value tables per segment in the workgroup's LDS table slots,
  * SUMs over per-segment arithmetic dictionaries (a dictId offset per segment) and over value tables,
  * a leaf negated in some segments only (an empty range becomes NOT(full range); NOT EQUALS of a value some segments
    lack), and segments a unit clause empties (left out of the kernel's tiles),
  * packed rows indexed by each segment's local keys, replicated per lane (PA_GDL_RR) and drained at segment switches,
  * 16 or 8 docs per lane (PA_GDL_ND), drained after every tile (PA_QF_GD_DRAIN_EACH_TILE).
Bars: bit-exact COUNT, LONG SUM, group keys, numDocsScanned.
"""
import numpy as np
import pytest

import oracle
from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.segment import create_segment
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

ACCOUNTS = np.arange(6000, dtype=np.int64) * 7 + 1000


def _tp_segment(seed, n, day0, ndays, acct_n):
    """A time partition: days [day0, day0 + ndays), acct_n of the 6000 accounts, clicks a run of 300 values and imps
    2000 values of step 3 from per-segment offsets, pv sorted random values (no arithmetic dictionary), g a random
    subset of 400 group values (a non-contiguous run of the table dictionary)."""
    rng = np.random.default_rng(seed)
    accts = np.sort(rng.choice(ACCOUNTS, size=acct_n, replace=False))
    pv = np.unique(rng.integers(-(1 << 20), 1 << 20, size=600))
    gvals = np.sort(rng.choice(np.arange(1000, dtype=np.int64) * 5, size=400, replace=False))
    data = {
        "day": rng.integers(day0, day0 + ndays, size=n).astype(np.int32),
        "acct": accts[rng.integers(0, len(accts), size=n)].astype(np.int32),
        "clicks": (rng.integers(0, 300, size=n) + (seed * 13) % 100).astype(np.int64),
        "imps": ((rng.integers(0, 2000, size=n) + (seed * 29) % 300) * 3).astype(np.int64),
        "pv": pv[rng.integers(0, len(pv), size=n)].astype(np.int64),
        "g": gvals[rng.integers(0, len(gvals), size=n)].astype(np.int32),
    }
    schema = {"day": "INT", "acct": "INT", "clicks": "LONG", "imps": "LONG", "pv": "LONG", "g": "INT"}
    return create_segment("tp%d" % seed, data, schema)


@pytest.fixture(scope="module")
def partitions():
    """Five time partitions of 5 days each (days 100..124), ragged sizes, account sets of 512..6000 (9..13-bit
    accountIds: several width classes)."""
    specs = [(1, 300_001, 100, 5, 6000), (2, 150_000, 105, 5, 3000), (3, 2049, 110, 5, 400), (4, 700_000, 115, 5, 512),
             (5, 65_536, 120, 5, 5000)]
    segs = [_tp_segment(*sp) for sp in specs]
    gs = [GpuSegment(s) for s in segs]
    yield segs, gs
    for g in gs:
        g.close()


def _in_list(frac, seed=9):
    ids = np.sort(np.random.default_rng(seed).choice(ACCOUNTS, size=int(len(ACCOUNTS) * frac), replace=False))
    return ", ".join(str(int(v)) for v in ids)


QUERIES = (
    # per-segment DICT_SET bitmaps, affine key offsets, per-segment SUM offsets, width classes
    "SELECT day, COUNT(*), SUM(clicks), SUM(imps) FROM t WHERE day BETWEEN 100 AND 124 AND acct IN (%s) GROUP BY day "
    "LIMIT 1000" % _in_list(0.3),
    # a day range two partitions lie outside (left out of the tiles) and one it cuts
    "SELECT day, COUNT(*), SUM(imps) FROM t WHERE day BETWEEN 107 AND 117 AND acct IN (%s) GROUP BY day LIMIT 1000"
    % _in_list(0.6, 3),
    # a SUM through per-segment value tables
    "SELECT day, SUM(pv), SUM(clicks) FROM t WHERE acct IN (%s) GROUP BY day LIMIT 1000" % _in_list(0.5, 4),
    # group keys through per-segment remap tables (g: non-contiguous runs of the table dictionary)
    "SELECT g, COUNT(*), SUM(clicks) FROM t WHERE acct IN (%s) AND day >= 103 GROUP BY g LIMIT 5000" % _in_list(0.4, 5),
    # an OR whose day range is empty in some partitions (NOT(full range) there: negation per segment)
    "SELECT day, COUNT(*), SUM(imps) FROM t WHERE (day < 108 OR acct IN (%s)) AND clicks >= 40 GROUP BY day "
    "LIMIT 1000" % _in_list(0.2, 6),
    # NOT EQUALS of a day only one partition holds (negated there, the full range elsewhere)
    "SELECT day, COUNT(*), SUM(clicks) FROM t WHERE day <> 112 AND acct IN (%s) GROUP BY day LIMIT 1000"
    % _in_list(0.5, 7),
)


@pytest.mark.parametrize("rr", ["64", "1"])
@pytest.mark.parametrize("nd", ["16", "8"])
@pytest.mark.parametrize("flags", [0, L.PA_QF_GD_DRAIN_EACH_TILE])
def test_own_dictionaries_on_the_specialised_kernel(partitions, monkeypatch, nd, flags, rr):
    """Every QUERIES shape with 16 or 8 docs per lane, the packed rows replicated per lane (as many replicas as fit, up
    to 64) or not."""
    segs, gs = partitions
    monkeypatch.setenv("PA_GDL_ND", nd)
    monkeypatch.setenv("PA_GDL_RR", rr)
    for sql in QUERIES:
        q = parse_sql(sql)
        ex = GpuQueryExecutor(q, gs, flags=flags)
        try:
            p = ex.stats()["plan"]
            assert p["dense_packed"] == 2 and p["strategy"] == "lds_dense", (sql[:80], p)
            got = ex.run()
        finally:
            ex.close()
        assert_same(got, oracle.run_query(q, segs))


def test_own_dictionaries_generic_kernel_agrees(partitions):
    """The same queries on the generic kernels (PA_QF_NO_JIT) give the same groups as the specialised one."""
    segs, gs = partitions
    for sql in QUERIES[:3]:
        q = parse_sql(sql)
        ex = GpuQueryExecutor(q, gs, flags=L.PA_QF_NO_JIT)
        try:
            assert ex.stats()["plan"]["dense_packed"] != 2
            got = ex.run()
        finally:
            ex.close()
        assert_same(got, oracle.run_query(q, segs))


def test_every_segment_excluded(partitions):
    """A unit clause no partition can match: no tile runs, no group, numDocsScanned 0."""
    segs, gs = partitions
    q = parse_sql("SELECT day, COUNT(*), SUM(clicks) FROM t WHERE day BETWEEN 300 AND 310 AND acct IN (%s) GROUP BY day "
                  "LIMIT 1000" % _in_list(0.5))
    ex = GpuQueryExecutor(q, gs)
    try:
        got = ex.run()
    finally:
        ex.close()
    exp = oracle.run_query(q, segs)
    assert_same(got, exp)
    assert not got.groups and got.num_docs_scanned == 0
