"""Multi-GPU merge on one GPU: two executors stand for two ranks whose segments carry DIFFERENT dictionaries. With the
agreed table-wide dictionaries (parallel.table_dictionaries' union) their accumulator blocks line up key for key, so
the element-wise reduce of the merged section runs (what RCCL does across GPUs) equals the oracle over all segments.
A world-size-1 RCCL group runs the real DistributedAccumulators path (key-space check + reduce calls)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle
from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd.engine import GpuQueryExecutor, GpuSegment
from pinot_amd.parallel import SECTION_OP, DistributedAccumulators, key_space_fingerprint
from synth import make_segment
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

COLS = {"d1": ("INT", 60), "d2": ("STRING", 12), "m": ("LONG", 4000), "f": ("DOUBLE", 300)}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl_world1():
    dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % _port(),
                            device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("sql", [
    "SELECT d1, COUNT(*), SUM(m), MIN(m), MAX(f), DISTINCTCOUNTHLL(m) FROM t GROUP BY d1 LIMIT 1000",
    "SELECT d1, d2, COUNT(*), SUM(f), AVG(m) FROM t WHERE m > 0 GROUP BY d1, d2 LIMIT 10000",
    "SELECT COUNT(*), SUM(m), MIN(f), MAX(m) FROM t WHERE d1 < 0",
])
def test_two_rank_merge_with_table_dictionaries(sql, rccl_world1):
    shards = [[make_segment(500 + 10 * r + i, n, COLS) for i, n in enumerate((20011, 7001))] for r in range(2)]
    q = parse_sql(sql)
    td = {}
    for name in q.group_by:
        td[name] = np.unique(np.concatenate([s.column(name).dictionary for sh in shards for s in sh]))
    gsegs = [[GpuSegment(s) for s in sh] for sh in shards]
    exs = [GpuQueryExecutor(q, g, table_dicts=td) for g in gsegs]
    try:
        if q.group_by:
            assert key_space_fingerprint(exs[0]) == key_space_fingerprint(exs[1])
            plain = [GpuQueryExecutor(q, g) for g in gsegs]  # own-segment dictionaries: key spaces differ
            assert key_space_fingerprint(plain[0]) != key_space_fingerprint(plain[1])
            for e in plain:
                e.close()
        accs = [DistributedAccumulators(e, torch.device("cuda", 0)) for e in exs]
        for e in exs:
            e.execute()
        torch.cuda.synchronize()
        for (k0, t0), (k1, t1) in zip(accs[0].views, accs[1].views):
            assert k0 == k1 and t0.shape == t1.shape
            op = SECTION_OP[k0]
            if op == dist.ReduceOp.SUM:
                t0.add_(t1)
            elif op == dist.ReduceOp.MIN:
                torch.minimum(t0, t1, out=t0)
            else:
                torch.maximum(t0, t1, out=t0)
        accs[0].reduce(dst=0)  # world size 1: RCCL reduce in place (identity)
        got = exs[0].fetch()
        exp = oracle.run_query(q, shards[0] + shards[1])
        assert_same(got, exp, rel=1e-9)
    finally:
        for e in exs:
            e.close()
        for g in gsegs:
            for x in g:
                x.close()


@pytest.mark.parametrize("sql", [
    "SELECT r, COUNT(*), SUM(m), MIN(f), MAX(m), DISTINCTCOUNTHLL(d1) FROM t GROUP BY r LIMIT 100000",
    "SELECT d1, ri, COUNT(*), AVG(f) FROM t WHERE m > 0 GROUP BY d1, ri LIMIT 100000",
])
def test_hashed_key_space_device_merge(sql, rccl_world1):
    """HashedAccumulators on a hashed key space (GROUP BY a raw column): the block moves into a torch buffer, the
    RCCL merge (world size 1: all-to-all of this rank's compacted rows to their key owners, merge by packed key) rewrites it as groups
    [0, n) in key order, and the library's own fetch of the rewritten block equals the oracle."""
    from pinot_amd.parallel import HashedAccumulators
    cols = dict(COLS, r=("LONG", 0), ri=("INT", 0))
    segs = [make_segment(900 + i, n, cols, no_dict=("r", "ri")) for i, n in enumerate((15013, 9001))]
    q = parse_sql(sql)
    gsegs = [GpuSegment(s) for s in segs]
    ex = GpuQueryExecutor(q, gsegs)
    try:
        assert ex.hashed
        acc = HashedAccumulators(ex, torch.device("cuda", 0))
        ex.execute()
        torch.cuda.synchronize()
        before = ex.fetch()
        n = acc.merge()
        torch.cuda.synchronize()
        got = ex.fetch()
        assert n == len(got.groups) == len(before.groups)
        exp = oracle.run_query(q, segs)
        assert_same(got, exp, rel=1e-9)
    finally:
        ex.close()
        for g in gsegs:
            g.close()


def test_rank_with_only_empty_segments_joins_the_merge(rccl_world1):
    """a rank whose segments are all empty plans a placeholder block from the agreed layout
    (parallel.table_layout: dictionaries, SUM widths, column schema), so its key-space fingerprint equals the other
    ranks', its reset block reduces as the identity, and as the reduce's destination it fetches the whole result."""
    from pinot_amd.parallel import TableLayout, wide_sum_columns_local
    from pinot_amd.segment import Segment
    q = parse_sql("SELECT d1, COUNT(*), SUM(m), MIN(f), MAX(m), DISTINCTCOUNTHLL(m) FROM t WHERE m > 0 GROUP BY d1 "
                  "LIMIT 1000")
    segs = [make_segment(610 + i, n, COLS) for i, n in enumerate((12011, 3001))]
    layout = TableLayout(dicts={"d1": np.unique(np.concatenate([s.column("d1").dictionary for s in segs]))},
                         wide=sorted(wide_sum_columns_local(q, segs)),
                         schema={n: (segs[0].column(n).data_type, True, True) for n in ("d1", "m", "f")})
    full = [GpuSegment(s) for s in segs]
    empty = [GpuSegment(Segment("e%d" % i, 0)) for i in range(2)]
    ex_full = GpuQueryExecutor(q, full, **layout.executor_kwargs())
    ex_empty = GpuQueryExecutor(q, empty, **layout.executor_kwargs())
    try:
        assert ex_empty.handle is not None and ex_empty.placeholder is not None
        assert key_space_fingerprint(ex_full) == key_space_fingerprint(ex_empty)
        a_full = DistributedAccumulators(ex_full, torch.device("cuda", 0))
        a_empty = DistributedAccumulators(ex_empty, torch.device("cuda", 0))
        ex_full.execute()
        ex_empty.execute()  # (reset only: nothing to scan)
        torch.cuda.synchronize()
        for (k0, t0), (k1, t1) in zip(a_empty.views, a_full.views):  # the placeholder rank as the reduce's destination
            op = SECTION_OP[k0]
            if op == dist.ReduceOp.SUM:
                t0.add_(t1)
            elif op == dist.ReduceOp.MIN:
                torch.minimum(t0, t1, out=t0)
            else:
                torch.maximum(t0, t1, out=t0)
        got = ex_empty.fetch()
        assert_same(got, oracle.run_query(q, segs), rel=1e-9)
    finally:
        for e in (ex_full, ex_empty):
            e.close()
        for g in full + empty:
            g.close()


@pytest.mark.parametrize("world,sql", [
    (2, "SELECT r, COUNT(*), SUM(m), SUM(f), MIN(f), MAX(m), DISTINCTCOUNTHLL(d1) FROM t GROUP BY r LIMIT 100000"),
    (3, "SELECT r, COUNT(*), SUM(m), SUM(f), MIN(f), MAX(m), DISTINCTCOUNTHLL(d1) FROM t GROUP BY r LIMIT 100000"),
    # two-word keys (two raw LONG columns: 128 bits)
    (3, "SELECT r, r2, COUNT(*), SUM(m), MAX(f) FROM t GROUP BY r, r2 LIMIT 100000"),
])
def test_library_pack_and_merge_rows_across_simulated_ranks(world, sql):
    """The hashed merge's local halves on the GPU (parallel.LibraryRows: pa_query_pack_rows / pa_query_merge_rows)
    with the all-to-all done by hand: `world` executors over disjoint segment sets stand for the ranks; each packs its
    groups into rows per owner rank, rank r merges every rank's rows for r into its own block. Every rank then holds
    exactly the groups key_owner gives it, and the union of the shares equals the oracle over all segments (COUNT,
    exact SUM of LONG, SUM of DOUBLE within 1e-9, MIN / MAX, HLL registers)."""
    from pinot_amd.parallel import LibraryRows, key_owner, key_owner2
    cols = dict(COLS, r=("LONG", 0), r2=("LONG", 0))
    q = parse_sql(sql)
    shards = [[make_segment(700 + 10 * w + i, n, cols, no_dict=("r", "r2")) for i, n in enumerate((9001, 4003))]
              for w in range(world)]
    for sh in shards:  # (r2 in a small range: (r, r2) pairs repeat across ranks)
        for sg in sh:
            sg.column("r2").raw_values = sg.column("r2").raw_values % 7
    # (make_segment draws r in [-1000, 1000): the ranks hold overlapping keys)
    gsegs = [[GpuSegment(s) for s in sh] for sh in shards]
    dev = torch.device("cuda", 0)
    bound = sum(s.num_docs for sh in shards for s in sh)
    exs = [GpuQueryExecutor(q, g, hash_keys_bound=bound) for g in gsegs]
    try:
        rows = [LibraryRows(e, dev) for e in exs]
        for e in exs:
            assert e.hashed
            e.execute()
        torch.cuda.synchronize()
        packed = [r.pack(world) for r in rows]
        us = []
        for w in range(world):
            parts = []
            for src in range(world):
                buf, counts = packed[src]
                lo = sum(counts[:w])
                parts.append(buf[lo:lo + counts[w]])
            u, over = rows[w].merge(torch.cat(parts))
            assert over == 0
            us.append(u)
        torch.cuda.synchronize()
        got_groups = {}
        docs_scanned = total_docs = 0
        for w, e in enumerate(exs):
            res = e.fetch()
            docs_scanned += res.num_docs_scanned  # (counters stay per rank: the broker sums them)
            total_docs += res.num_total_docs
            assert len(res.groups) == us[w]
            kw = e.key_words
            ks, _, _ = e.fetch_arrays()
            for k in (ks.tolist() if kw == 1 else [tuple(x) for x in ks.tolist()]):
                own = key_owner(torch.tensor([k]), world) if kw == 1 else \
                    key_owner2(torch.tensor([k[0]]), torch.tensor([k[1]]), world)
                assert int(own[0]) == w
            for key in res.groups:
                assert key not in got_groups
            got_groups.update(res.groups)
        exp = oracle.run_query(q, [s for sh in shards for s in sh])
        merged = exs[0].fetch()
        merged.groups = got_groups
        merged.num_docs_scanned, merged.num_total_docs = docs_scanned, total_docs
        assert_same(merged, exp, rel=1e-9)
    finally:
        for e in exs:
            e.close()
        for g in gsegs:
            for x in g:
                x.close()


def test_reduce_scatter_merge_path(rccl_world1):
    """DistributedAccumulators.merge on a key space at the scatter threshold runs reduce_scatter_sections over RCCL
    (world size 1: the rank's range is the whole key space) and the fetch of the rewritten block equals the oracle."""
    q = parse_sql("SELECT d1, d2, COUNT(*), SUM(m), MIN(f), MAX(m), DISTINCTCOUNTHLL(m) FROM t GROUP BY d1, d2 "
                  "LIMIT 10000")
    segs = [make_segment(820 + i, n, COLS) for i, n in enumerate((11003, 5001))]
    gsegs = [GpuSegment(s) for s in segs]
    ex = GpuQueryExecutor(q, gsegs)
    try:
        acc = DistributedAccumulators(ex, torch.device("cuda", 0))
        ex.execute()
        torch.cuda.synchronize()
        assert acc.merge(scatter_keys=1) is True
        torch.cuda.synchronize()
        assert_same(ex.fetch(), oracle.run_query(q, segs), rel=1e-9)
    finally:
        ex.close()
        for g in gsegs:
            g.close()


def test_reduce_execution_stats(rccl_world1):
    """numDocsScanned is summed by the element-wise reduce, so the merged block's execution statistics are the ranks'
    own pairs summed before the collective (reduce(execution_stats=True), the default); a reduce without them
    (execution_stats=False) makes a statistics fetch raise rather than recount this rank's segments against the merged
    counter or return (0, 0), and the next execute() returns to local counting.""" 
    q = parse_sql("SELECT d1, COUNT(*), SUM(m) FROM t WHERE m > 1000 AND d1 < 30 GROUP BY d1 LIMIT 10000")
    segs = [make_segment(840 + i, n, COLS) for i, n in enumerate((12007, 4001))]
    gsegs = [GpuSegment(s) for s in segs]
    ex = GpuQueryExecutor(q, gsegs)
    try:
        acc = DistributedAccumulators(ex, torch.device("cuda", 0))
        ex.execute()
        before = ex.fetch()
        local = (before.num_entries_scanned_in_filter, before.num_entries_scanned_post_filter)
        assert local[0] > 0 and local[1] > 0
        acc.reduce(dst=0, execution_stats=True)  # world size 1: the sum is this rank's own pair
        got = ex.fetch()
        assert (got.num_entries_scanned_in_filter, got.num_entries_scanned_post_filter) == local
        ex.execute()
        acc.reduce(dst=0)  # (the default gathers the statistics too)
        got = ex.fetch()
        assert (got.num_entries_scanned_in_filter, got.num_entries_scanned_post_filter) == local
        ex.execute()
        acc.reduce(dst=0, execution_stats=False)
        with pytest.raises(L.PinotAmdError):
            ex.fetch()  # (no statistics were gathered: no silent (0, 0))
        got = ex.fetch(execution_stats=False)
        assert (got.num_entries_scanned_in_filter, got.num_entries_scanned_post_filter) == (0, 0)
        ex.execute()
        again = ex.fetch()
        assert (again.num_entries_scanned_in_filter, again.num_entries_scanned_post_filter) == local
    finally:
        ex.close()
        for g in gsegs:
            g.close()
