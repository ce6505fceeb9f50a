"""Execution statistics on the GPU (pa_query_execution_stats: pa_stats.hip's masks, counts and chunked leap-frogs;
the scan's fused counts) against the host iterator replay.

pa_bitmap_counts is checked against a numpy restatement of its four counts on random leaf bitmaps (one word to
multi-workgroup sizes, densities down to a few set bits so the cross-workgroup label carry is exercised); the
executor's execution_stats() against filter_stats.server_stats (the replay of the reference's iterators,
SVScanDocIdIterator / MVScanDocIdIterator / AndDocIdIterator / OrDocIdIterator / NotDocIdIterator) over the same GPU
leaf bitmaps, per filter shape, with the replay asserted unused for every shape the engine covers. Bit-exact
integers."""
import ctypes

import numpy as np
import pytest
import torch

from pinot_amd import _lib as L
from pinot_amd import filter_stats as FS
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.segment import create_segment
from test_filter_stats import ENGINE_WHERES, REPLAY_WHERES, _np_prog, np_leaps

pytestmark = pytest.mark.gpu

AND, OR, NOT = L.PA_BIT_AND, L.PA_BIT_OR, L.PA_BIT_NOT


def _device_counts(bits, n, a, b):
    lib = L.lib()
    nl, words = bits.shape
    dev = torch.device("cuda", torch.cuda.current_device())
    bm = torch.from_numpy(np.ascontiguousarray(bits).view(np.int32).reshape(-1)).to(dev)
    out = torch.zeros(4, dtype=torch.int64, device=dev)
    scratch = torch.empty(max(1, int(lib.pa_bitmap_counts_scratch_bytes(words)) // 4), dtype=torch.int32, device=dev)
    pa = (ctypes.c_int32 * max(1, len(a)))(*a)
    pb = (ctypes.c_int32 * max(1, len(b)))(*b)
    L.check(lib.pa_bitmap_counts(bm.data_ptr(), words, nl, n, pa, len(a), pb, len(b), scratch.data_ptr(),
                                 out.data_ptr(), None), "pa_bitmap_counts")
    torch.cuda.synchronize()
    return out.cpu().numpy().tolist()


@pytest.mark.parametrize("n", [1, 31, 32, 33, 5000, 32 * 1024 + 7, 3_000_001])
def test_bitmap_counts_kernel(n):
    rng = np.random.default_rng(n)
    words = (n + 127) // 128 * 4
    progs = [([0], [1]), ([0, 1, OR], [2, NOT]), ([0, NOT, 2, AND], [1]), ([2], []), ([0, 1, AND, 2, OR], [0, NOT])]
    for dens in ([0.5, 0.5, 0.5], [0.02, 0.3, 0.9], [3.0 / n, 2.0 / n, 0.5], [1.0, 1.0, 0.0]):
        masks = np.stack([rng.random(n) < d for d in dens])
        bits = np.zeros((3, words * 32), dtype=bool)
        bits[:, :n] = masks
        packed = np.packbits(bits, axis=1, bitorder="little").view(np.uint32)
        for a, b in progs:
            A = _np_prog(a, masks, n)
            B = _np_prog(b, masks, n) if b else np.zeros(n, dtype=bool)
            want = [int(A.sum()), int(B.sum()), int((A & B).sum()), np_leaps(A, B) if b else 0]
            assert _device_counts(packed, n, a, b) == want, (dens, a, b)


def test_bitmap_counts_rejects_bad_programs():
    lib = L.lib()
    for a in ([], [0, 1], [AND], [5], [0, -9], [0] * 17 + [AND] * 16):
        pa = (ctypes.c_int32 * max(1, len(a)))(*a)
        rc = lib.pa_bitmap_counts(None, 0, 3, 0, pa, len(a), None, 0, None, ctypes.c_void_p(8), None)
        assert rc < 0, a


def _segment(seed, n):
    rng = np.random.default_rng(seed)
    data = {"s": np.sort(rng.integers(0, 50, n)).astype(np.int32), "a": rng.integers(0, 100, n).astype(np.int32),
            "b": rng.integers(0, 100, n).astype(np.int32), "c": rng.integers(0, 20, n).astype(np.int32),
            "r": rng.integers(0, 5000, n).astype(np.int32), "w": rng.integers(0, 1 << 20, n).astype(np.int32)}
    return create_segment("st%d" % seed, data, {k: "INT" for k in data}, inverted_index_columns=("c",),
                          no_dictionary_columns=("r",))


def _stats_and_replay(ex):
    """(engine statistics, host replay) after a scan + fetch of the executor (the fetch fills the statistics)."""
    ex.execute()
    early = ex.execution_stats()  # before the fetch: numDocsScanned from the scan's own counter
    res = ex.fetch()
    got = (res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter)
    assert got == early == ex.execution_stats()  # (evaluated again over the same scan)
    # (the executor holds the reference's rewritten filter: optimizer.py)
    want = FS.server_stats(ex.query, ex.segs, lambda si: ex.leaf_bitmaps(si))
    return got, want


def test_execution_stats_device_vs_replay():
    """Every filter shape of test_filter_stats over 3 segments of up to 200K docs (the leap-frogs cross many 2048-doc
    chunks): the statistics the fetch fills = the host replay over the same GPU bitmaps, and the host replay is never
    used — the shapes outside the reduction (REPLAY_WHERES, a NOT child of a leap-frogging AND) are replayed iterator by
    iterator on the GPU (stat_replay_kernel)."""
    segs = [_segment(1, 200_003), _segment(2, 70_000), _segment(3, 1025)]
    gs = [GpuSegment(s) for s in segs]
    try:
        # (+ a raw column: per-doc leaf path; a 20-bit dictionary: wide lane-major decode)
        extra = ["r < 1000 AND a < 50", "r BETWEEN 10 AND 20 OR b = 3", "w < 300000 AND b < 40",
                 "w IN (5, 77, 1000) OR a = 1", "r IN (3, 5, 7, 4000) AND b < 50",
                 "w < 600000 AND (a < 5 OR r < 200) AND b > 20", "NOT (w < 900000 AND r > 40 AND b < 90)"]
        replay = REPLAY_WHERES + ["NOT r IN (3, 5) AND a < 9", "w < 500000 AND NOT (r < 100 OR b > 60)"]
        for where in ENGINE_WHERES + extra + replay:
            for sql in ("SELECT COUNT(*) FROM t WHERE " + where, "SELECT c, SUM(a) FROM t WHERE %s GROUP BY c" % where):
                ex = GpuQueryExecutor(parse_sql(sql), gs)
                try:
                    got, want = _stats_and_replay(ex)
                    replayed = ex.stats_replayed_segments
                finally:
                    ex.close()
                assert got == want, sql
                assert replayed == 0, sql
    finally:
        for g in gs:
            g.close()


def test_execution_stats_multi_value_scans():
    """Multi-value scans read every value of a doc (MVScanDocIdIterator): in applyAnd chains (value counts of the
    surviving docs) and in leap-frogs (the values of the docs between target and answer) = the host replay."""
    rng = np.random.default_rng(8)
    segs = []
    for i, n in enumerate((150_001, 4099)):
        data = {"c": rng.integers(0, 20, n).astype(np.int32), "a": rng.integers(0, 100, n).astype(np.int32),
                "s": np.sort(rng.integers(0, 40, n)).astype(np.int32),
                "tags": [rng.integers(0, 300, int(k)).astype(np.int32) for k in rng.integers(1, 6, n)]}
        segs.append(create_segment("mv%d" % i, data, {k: "INT" for k in data}, inverted_index_columns=("c",),
                                   multi_value_columns=("tags",)))
    gs = [GpuSegment(s) for s in segs]
    try:
        for where in ("tags IN (3, 5, 7) AND a < 50", "s < 20 AND tags < 100", "c = 3 AND tags > 250",
                      "tags < 30 OR a < 5", "a < 40 AND (tags = 7 OR a > 90)", "NOT (tags < 200 AND a < 70)",
                      "tags < 150 AND a < 60 AND c < 15"):
            ex = GpuQueryExecutor(parse_sql("SELECT c, SUM(a) FROM t WHERE %s GROUP BY c" % where), gs)
            try:
                got, want = _stats_and_replay(ex)
                assert ex.stats_replayed_segments == 0, where
            finally:
                ex.close()
            assert got == want, where
    finally:
        for g in gs:
            g.close()


def test_merged_range_is_one_scan_on_the_gpu():
    """MergeRangeFilterOptimizer feeds the GPU statistics path: `a >= 10 AND a <= 40` is ONE scan of a (the reference's
    rewritten RANGE predicate reads every entry once: numEntriesScannedInFilter = the docs), where the unrewritten AND
    of two scans (the host replay of the original tree over its two leaves) reads more; the groups are the same."""
    from pinot_amd.segment import unpack_bits
    segs = [_segment(5, 120_001), _segment(6, 9000)]
    gs = [GpuSegment(s) for s in segs]
    try:
        q = parse_sql("SELECT c, SUM(b) FROM t WHERE a >= 10 AND a <= 40 GROUP BY c")
        ex = GpuQueryExecutor(q, gs)
        try:
            assert isinstance(ex.query.filter, type(q.filter.children[0]))  # one RANGE predicate
            res = ex.run()
            in_filter, post = ex.execution_stats()
        finally:
            ex.close()
        total = sum(s.num_docs for s in segs)
        assert in_filter == total
        raw = 0
        for s in segs:
            col = s.column("a")
            v = col.dictionary[unpack_bits(col.fwd_bytes, s.num_docs, col.num_bits)]
            raw += FS.entries_scanned_in_filter(q.filter, s, np.asarray([v >= 10, v <= 40]))
        assert raw > in_filter
        assert post == res.num_docs_scanned * 2  # projected: c and b
    finally:
        for g in gs:
            g.close()


def _sparse_segment(seed, n, e_docs):
    """z: 16 values (an A leaf matching ~1/16 .. 1/4 of the docs), y: 4096 values (a sparse A leaf), e: 65536 values,
    with value 7 placed at e_docs (a sparse E leaf: segment ends, tile boundaries) plus a few random docs."""
    rng = np.random.default_rng(seed)
    e = rng.integers(8, 65536, n).astype(np.int32)
    e[[d for d in e_docs if d < n]] = 7
    e[rng.integers(0, n, 6)] = 7
    data = {"z": rng.integers(0, 16, n).astype(np.int32), "y": rng.integers(0, 4096, n).astype(np.int32), "e": e,
            "m": rng.integers(0, 1000, n).astype(np.int32)}
    return create_segment("sp%d" % seed, data, {k: "INT" for k in data})


def test_fused_execution_stats_match_the_replay():
    """The scan counts the leaps of `z-leaf AND e-leaf` itself by default (E = the sparse eager e leaf, found by
    neighbour searches from each E doc); the statistics equal the host replay, and no GPU statistics pass runs when
    every search finished. A sparse A leaf (y) makes searches give up: those segments take the statistics engine, with
    the same result. With E first in the reference's AND order the fused counts do not apply (engine)."""
    n0 = 300_007
    # (segments large enough that e's dictionary keeps e = 7 below 1 / 256 of the docs, which makes the planner
    # evaluate the z clause lazily: the fused count's precondition)
    segs = [_sparse_segment(1, n0, [0, 1, 2047, 2048, 4095, n0 - 1]), _sparse_segment(2, 70_000, [69_999]),
            _sparse_segment(3, 131_072, [65_536]), _sparse_segment(4, 200_000, [])]
    gs = [GpuSegment(s) for s in segs]
    try:
        cases = [("z < 2 AND e = 7", True), ("z BETWEEN 3 AND 6 AND e IN (7, 11)", True),
                 ("z = 5 AND e = 7", True), ("y = 17 AND e = 7", False), ("e = 7 AND z < 2", False)]
        for where, fused_only in cases:
            for sql in ("SELECT COUNT(*) FROM t WHERE " + where, "SELECT z, SUM(m) FROM t WHERE %s GROUP BY z" % where):
                for flags in (0, L.PA_QF_NO_FILTER_STATS):
                    ex = GpuQueryExecutor(parse_sql(sql), gs, flags=flags)
                    try:
                        ex.execute()
                        fz = ex.fused_leap_counts()
                        assert (fz is not None) == (flags == 0), sql  # (a sparse E: the scan counted by default)
                        res = ex.fetch()
                        got = (res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter)
                        if fused_only and flags == 0:
                            assert ex.stats_gpu_segments == 0, sql
                        want = FS.server_stats(ex.query, ex.segs, lambda si: ex.leaf_bitmaps(si))
                        if fz is not None:
                            assert fz[2][:, 0].sum() == res.num_docs_scanned
                    finally:
                        ex.close()
                    assert got == want, (sql, flags)
    finally:
        for g in gs:
            g.close()


def test_fused_statistics_on_the_steady_state_tile_loop():
    """The fused count's segment-start term (the segment's first labelled doc A-only) on waves that walk many tiles
    (ring of 2, one workgroup per CU: the hoisted steady-state loop, not the per-tile entry point): the statistics of
    an AND whose segments all start with an A-only doc equal the host replay."""
    segs = [_sparse_segment(11 + i, 4_000_000, [1_000_000 + 7 * i]) for i in range(2)]
    # (z < 8 matches half the docs, e = 7 a handful: every segment's first labelled doc is A-only)
    gs = [GpuSegment(s) for s in segs]
    try:
        q = parse_sql("SELECT COUNT(*) FROM t WHERE z < 8 AND e = 7")
        flags = (2 << L.PA_QF_RING_SHIFT) | (1 << L.PA_QF_WG_SHIFT)
        ex = GpuQueryExecutor(q, gs, flags=flags)
        try:
            ex.execute()
            fz = ex.fused_leap_counts()
            assert fz is not None and not fz[2][:, 2].any()
            res = ex.fetch()
            got = (res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter)
            assert ex.stats_gpu_segments == 0
            want = FS.server_stats(ex.query, ex.segs, lambda si: ex.leaf_bitmaps(si))
        finally:
            ex.close()
        assert got == want
    finally:
        for g in gs:
            g.close()
