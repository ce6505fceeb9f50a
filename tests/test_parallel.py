"""Multi-rank merge of partial aggregates (pinot_amd/parallel.py) on CPU with the gloo backend, world size 2.

Each rank owns a disjoint segment range (shard_segments) and holds its partial accumulators in the library's section
layout (pa_query_section kinds); reduce_sections must reproduce what one GPU would hold for the whole segment set:
the cross-server half of GroupByCombineOperator (IndexedTable upsert: COUNT/SUM +, MIN min, MAX max, HLL register max).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pinot_amd import _lib as L
from pinot_amd.parallel import SECTION_DTYPE, reduce_sections, shard_segments

K = 257  # keys
LOG2M = 8


def f64_order_encode(d):
    """pa_device.h f64_order_encode: signed int64 order == double order."""
    b = np.asarray(d, dtype=np.float64).view(np.int64)
    return np.where(b >= 0, b, b ^ np.int64(0x7FFFFFFFFFFFFFFF))


def f64_order_decode(e):
    e = np.asarray(e, dtype=np.int64)
    return np.where(e >= 0, e, e ^ np.int64(0x7FFFFFFFFFFFFFFF)).view(np.float64)


def partial(rank):
    """Partial accumulators of one rank's segments (random, seeded by rank)."""
    rng = np.random.default_rng(100 + rank)
    count = rng.integers(0, 1000, K).astype(np.int64)
    vals = rng.integers(-(1 << 62), 1 << 62, K)
    sum_x2 = np.empty(2 * K, dtype=np.int64)  # PA_ACC_SUM_I64X2: [2k] low-32 unsigned sum, [2k+1] high-32 signed sum
    sum_x2[0::2] = vals & 0xFFFFFFFF
    sum_x2[1::2] = vals >> 32
    dsum = rng.standard_normal(K)
    dmin = f64_order_encode(rng.standard_normal(K) * 1e6)
    imax = rng.integers(-(1 << 40), 1 << 40, K).astype(np.int64)
    hll = rng.integers(0, 26, K << LOG2M).astype(np.uint8)
    return [(L.PA_ACC_COUNT_U64, count), (L.PA_ACC_SUM_I64X2, sum_x2), (L.PA_ACC_SUM_F64, dsum),
            (L.PA_ACC_MIN_I64, dmin), (L.PA_ACC_MAX_I64, imax), (L.PA_ACC_HLL_U8, hll)], vals


def _worker(rank, world, port, all_reduce, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    secs, _ = partial(rank)
    views = [(k, torch.from_numpy(np.ascontiguousarray(a)).to(SECTION_DTYPE[k])) for k, a in secs]
    reduce_sections(views, dst=0, all_reduce=all_reduce)
    if rank == 0 or all_reduce:
        out[rank] = [t.numpy().copy() for _, t in views]
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("all_reduce", [False, True])
def test_gloo_reduce_matches_single_gpu_merge(all_reduce):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), all_reduce, out), nprocs=world, join=True)
    parts = [partial(r) for r in range(world)]
    exp_count = sum(p[0][0][1] for p in parts)
    exp_sum = sum(p[1].astype(object) for p in parts)  # exact big-int totals
    exp_dsum = sum(p[0][2][1] for p in parts)
    exp_min = np.minimum.reduce([f64_order_decode(p[0][3][1]) for p in parts])
    exp_max = np.maximum.reduce([p[0][4][1] for p in parts])
    exp_hll = np.maximum.reduce([p[0][5][1] for p in parts])
    for r in (range(world) if all_reduce else [0]):
        count, sx2, dsum, dmin, imax, hll = out[r]
        assert np.array_equal(count, exp_count)
        total = sx2[0::2].astype(object) + (sx2[1::2].astype(object) << 32)  # decode of pa_query_fetch
        assert all(a == b for a, b in zip(total, exp_sum))
        assert np.allclose(dsum, exp_dsum, rtol=1e-12, atol=0)
        assert np.array_equal(f64_order_decode(dmin), exp_min)
        assert np.array_equal(imax, exp_max)
        assert np.array_equal(hll, exp_hll)


def test_f64_order_encoding_is_monotone():
    rng = np.random.default_rng(0)
    d = np.concatenate([rng.standard_normal(1000) * 10.0 ** rng.integers(-300, 300, 1000),
                        [0.0, -0.0, np.inf, -np.inf, 5e-324, -5e-324]])
    e = f64_order_encode(d)
    # sorted by the encoding, the doubles are non-decreasing (-0.0 sorts just below 0.0, as Java's Math.min/max
    # order them)
    ds = d[np.argsort(e, kind="stable")]
    assert np.all(ds[1:] >= ds[:-1])
    assert f64_order_encode(-0.0) < f64_order_encode(0.0)
    assert np.array_equal(f64_order_decode(e).view(np.int64), d.view(np.int64))


@pytest.mark.parametrize("n,world", [(100, 1), (100, 2), (100, 8), (7, 8), (801, 3)])
def test_shard_segments_partition(n, world):
    parts = [shard_segments(n, r, world) for r in range(world)]
    flat = [i for p in parts for i in p]
    assert flat == list(range(n))  # disjoint, complete, contiguous
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _block_layout(secs):
    """pa_plan.hip plan_accumulators block: sections at 256-byte aligned offsets (gaps zero, as pa_query_reset leaves them)."""
    offs, total = [], 0
    for k, a in secs:
        offs.append(total)
        total += (a.nbytes + 255) & ~255
    buf = np.zeros(total, dtype=np.uint8)
    for o, (k, a) in zip(offs, secs):
        buf[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8)
    return buf, offs


def _secs_with_docs(rank):
    secs, _ = partial(rank)
    # the bench query's layout: COUNT, 2x SUM(LONG), numDocsScanned — then the rest
    return [secs[0], secs[1], (L.PA_ACC_SUM_I64X2, secs[1][1] * 3),
            (L.PA_ACC_DOCS_U64, np.array([5 + rank, 0, 1, 0], np.int64))] + secs[2:]


def test_section_runs_merge_adjacent_same_op():
    from pinot_amd.parallel import section_runs
    secs = _secs_with_docs(0)
    _, offs = _block_layout(secs)
    runs = section_runs([(k, o, a.size) for (k, a), o in zip(secs, offs)])
    # COUNT + SUM_I64X2 + SUM_I64X2 + DOCS -> one SUM run; then f64 SUM, MIN, MAX, HLL each on their own
    assert [r[0] for r in runs] == [L.PA_ACC_COUNT_U64, L.PA_ACC_SUM_F64, L.PA_ACC_MIN_I64, L.PA_ACC_MAX_I64,
                                    L.PA_ACC_HLL_U8]
    assert runs[0][2] == 0 and runs[0][3] == offs[3] + 4 * 8
    # a keys section (not element-wise reducible) never merges
    r2 = section_runs([(L.PA_ACC_COUNT_U64, 0, 4), (L.PA_ACC_KEYS_I64, 256, 4), (L.PA_ACC_DOCS_U64, 512, 3)])
    assert len(r2) == 3


def _runs_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd.parallel import section_runs
    secs = _secs_with_docs(rank)
    buf, offs = _block_layout(secs)
    t = torch.from_numpy(buf)
    runs = section_runs([(k, o, a.size) for (k, a), o in zip(secs, offs)])
    reduce_sections([(k, t[a:b].view(dt)) for k, dt, a, b in runs], dst=0)
    if rank == 0:
        out[0] = t.numpy().copy()
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_reduce_over_merged_section_runs():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_runs_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    parts = [_secs_with_docs(r) for r in range(world)]
    bufs = [_block_layout(p)[0] for p in parts]
    _, offs = _block_layout(parts[0])
    got = out[0]
    for i, (k, a) in enumerate(parts[0]):
        dt = a.dtype
        g = got[offs[i]:offs[i] + a.nbytes].view(dt)
        xs = [b[offs[i]:offs[i] + a.nbytes].view(dt) for b in bufs]
        if k in (L.PA_ACC_MIN_I64,):
            exp = np.minimum(*xs)
        elif k in (L.PA_ACC_MAX_I64, L.PA_ACC_HLL_U8):
            exp = np.maximum(*xs)
        else:
            exp = xs[0] + xs[1]
        if k == L.PA_ACC_SUM_F64:
            assert np.allclose(g, exp, rtol=1e-12, atol=0)
        else:
            assert np.array_equal(g, exp), k
    # the alignment gaps stay zero
    mask = np.ones(len(got), bool)
    for o, (k, a) in zip(offs, parts[0]):
        mask[o:o + a.nbytes] = False
    assert not got[mask].any()


def _dict_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd import parse_sql
    from pinot_amd.parallel import check_same_key_space, table_dictionaries
    from synth import make_segment
    q = parse_sql("SELECT d, s, COUNT(*) FROM t GROUP BY d, s")
    segs = [make_segment(40 + 2 * rank + i, 500, {"d": ("INT", 30 + 10 * rank), "s": ("STRING", 5 + rank)})
            for i in range(2)]
    td = table_dictionaries(q, segs)
    out[rank] = {k: v.tolist() for k, v in td.items()}
    check_same_key_space(12345, "cpu")  # same on both ranks: passes
    try:
        check_same_key_space(100 + rank, "cpu")
        out["raised%d" % rank] = False
    except L.PinotAmdError:
        out["raised%d" % rank] = True
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_table_dictionaries_and_key_space_check():
    """Ranks whose segments carry different dictionaries agree on one table-wide dictionary per group-by column (the
    union), and a key-space mismatch is refused on every rank instead of reducing misaligned accumulator rows."""
    from synth import make_segment
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_dict_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out[0] == out[1]
    for name in ("d", "s"):
        exp = set()
        for r in range(world):
            for i in range(2):
                cols = {"d": ("INT", 30 + 10 * r), "s": ("STRING", 5 + r)}
                exp |= set(make_segment(40 + 2 * r + i, 500, cols).column(name).dictionary.tolist())
        assert out[0][name] == sorted(exp)
    assert out["raised0"] and out["raised1"]


def test_key_space_fingerprint_distinguishes_dictionaries():
    from pinot_amd.parallel import key_space_fingerprint

    class _E:
        def __init__(self, n, dicts, secs=((L.PA_ACC_COUNT_U64, 6), (L.PA_ACC_SUM_I64, 6))):
            self.num_keys, self.global_dicts, self.handle, self._secs = n, dicts, None, secs

        def sections(self):
            return [(k, 0, n) for k, n in self._secs]
    a = key_space_fingerprint(_E(6, [np.array([1, 2, 3]), np.array(["x", "y"])]))
    # same key space, a SUM kept wide on one rank only: a different accumulator layout
    assert a != key_space_fingerprint(_E(6, [np.array([1, 2, 3]), np.array(["x", "y"])],
                                         ((L.PA_ACC_COUNT_U64, 6), (L.PA_ACC_SUM_I64X2, 12))))
    assert a == key_space_fingerprint(_E(6, [np.array([1, 2, 3]), np.array(["x", "y"])]))
    assert a != key_space_fingerprint(_E(6, [np.array([1, 2, 4]), np.array(["x", "y"])]))
    assert a != key_space_fingerprint(_E(6, [np.array([1, 2, 3]), np.array(["x", "z"])]))
    assert a != key_space_fingerprint(_E(6, [np.array([1, 2, 3]), None]))


def _layout_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd import parse_sql
    from pinot_amd.parallel import table_layout
    from pinot_amd.segment import create_segment
    q = parse_sql("SELECT k, SUM(m), AVG(n), SUM(i) FROM t GROUP BY k")
    rng = np.random.default_rng(rank)
    m = rng.integers(0, 1000, size=300).astype(np.int64)
    if rank == 1:
        m[7] = 1 << 40  # only rank 1 holds a LONG value outside int32
    seg = create_segment("s%d" % rank, {"k": rng.integers(0, 5, size=300).astype(np.int32), "m": m,
                                        "n": rng.integers(0, 9, size=300).astype(np.int64),
                                        "i": rng.integers(0, 9, size=300).astype(np.int32)},
                         {"k": "INT", "m": "LONG", "n": "LONG", "i": "INT"})
    lay = table_layout(q, [seg])
    out[rank] = (sorted(lay.dicts), list(lay.wide))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_table_layout_agrees_on_wide_sums():
    """A LONG column whose values fit int32 on one rank but not on the other: both ranks agree to keep the wide SUM
    accumulator (otherwise the ranks' accumulator blocks differ in size and RCCL reduces misaligned data)."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_layout_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out[0] == out[1] == (["k"], ["m"])


NS = 64  # hashed table slots per rank
HLOG = 4  # HLL log2m of the hashed-merge test (16 registers per key)


def _hashed_partial(rank):
    """One rank's hashed table: 20 groups at random slots (keys from a shared pool of 30, so ranks overlap), every
    other slot empty (key INT64_MAX, count 0, identities) — the block pa_query_scan leaves for a hashed key space."""
    rng = np.random.default_rng(700 + rank)
    pool = np.array([-(1 << 62), -5, 0, 3, (1 << 63) - 1] + list(range(100, 125)), dtype=np.int64)
    keys_used = rng.choice(pool, size=20, replace=False)
    slots = rng.choice(NS, size=20, replace=False)
    keys = np.full(NS, (1 << 63) - 1, np.int64)
    count = np.zeros(NS, np.int64)
    sx2 = np.zeros(2 * NS, np.int64)
    dsum = np.zeros(NS)
    dmin = np.full(NS, (1 << 63) - 1, np.int64)
    imax = np.full(NS, -(1 << 63), np.int64)
    hll = np.zeros(NS << HLOG, np.uint8)
    pres = np.zeros(NS * 16, np.uint8)
    groups = {}
    for k, s in zip(keys_used.tolist(), slots.tolist()):
        keys[s] = k
        count[s] = rng.integers(1, 50)
        v = int(rng.integers(-(1 << 40), 1 << 40))
        sx2[2 * s], sx2[2 * s + 1] = v & 0xFFFFFFFF, v >> 32
        dsum[s] = rng.standard_normal()
        dmin[s] = f64_order_encode(rng.standard_normal() * 100)
        imax[s] = rng.integers(-1000, 1000)
        hll[s << HLOG:(s + 1) << HLOG] = rng.integers(0, 20, 1 << HLOG)
        pres[s * 16:(s + 1) * 16] = rng.integers(0, 2, 16)
        groups[k] = (int(count[s]), v, float(dsum[s]), int(dmin[s]), int(imax[s]),
                     hll[s << HLOG:(s + 1) << HLOG].copy(), pres[s * 16:(s + 1) * 16].copy())
    secs = [(L.PA_ACC_COUNT_U64, count), (L.PA_ACC_SUM_I64X2, sx2), (L.PA_ACC_SUM_F64, dsum),
            (L.PA_ACC_MIN_I64, dmin), (L.PA_ACC_MAX_I64, imax), (L.PA_ACC_HLL_U8, hll),
            (L.PA_ACC_PRESENCE_U8, pres), (L.PA_ACC_KEYS_I64, keys),
            (L.PA_ACC_DOCS_U64, np.array([1000 + rank, 0, 0, 0], np.int64))]
    return secs, groups


def _hashed_worker(rank, world, port, out, partial_fn=None, extra=b""):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd.parallel import merge_hashed_sections
    from row_ops_ref import TorchRows
    secs, _ = (partial_fn or _hashed_partial)(rank)
    views = [(k, torch.from_numpy(np.ascontiguousarray(a)).to(SECTION_DTYPE[k])) for k, a in secs]
    try:
        u = merge_hashed_sections(views, NS, layout_extra=extra if isinstance(extra, bytes) else extra[rank],
                                  rows=TorchRows(views, NS))
        out[rank] = (u, [t.numpy().copy() for _, t in views])
    except L.PinotAmdError as e:
        out[rank] = ("raised", str(e))
    dist.barrier()
    dist.destroy_process_group()


def _expected_union(partials):
    exp = {}
    for groups in partials:
        for k, (c, v, ds, mn, mx, h, p) in groups.items():
            if k in exp:
                e = exp[k]
                exp[k] = (e[0] + c, e[1] + v, e[2] + ds, min(e[3], mn), max(e[4], mx), np.maximum(e[5], h),
                          np.maximum(e[6], p))
            else:
                exp[k] = (c, v, ds, mn, mx, h, p)
    return exp


def _check_shares(out, world, exp, docs_of):
    """Every rank's block holds its share (the keys key_owner assigns it) in ascending key order, every other slot
    empty; the shares are disjoint and their union is the merged result; numDocsScanned stays per rank."""
    from pinot_amd.parallel import key_owner
    seen = []
    for r in range(world):
        u, (count, sx2, dsum, dmin, imax, hll, pres, keys, docs) = out[r]
        share = sorted(k for k in exp if int(key_owner(torch.tensor([k], dtype=torch.int64), world)[0]) == r)
        assert u == len(share)
        assert keys[:u].tolist() == share and (keys[u:] == (1 << 63) - 1).all()
        assert (count[u:] == 0).all() and (dmin[u:] == (1 << 63) - 1).all() and (imax[u:] == -(1 << 63)).all()
        assert docs.tolist() == docs_of(r)
        for i, k in enumerate(share):
            c, v, ds, mn, mx, h, p = exp[k]
            assert count[i] == c
            assert int(sx2[2 * i]) + (int(sx2[2 * i + 1]) << 32) == v
            assert abs(dsum[i] - ds) <= 1e-12 * max(1.0, abs(ds))
            assert dmin[i] == mn and imax[i] == mx
            assert np.array_equal(hll[i << HLOG:(i + 1) << HLOG], h)
            assert np.array_equal(pres[i * 16:(i + 1) * 16], p)
        seen += share
    assert sorted(seen) == sorted(exp)  # disjoint + complete


def test_gloo_device_side_merge_of_hashed_key_spaces():
    """parallel.merge_hashed_sections (the RCCL path of hashed key spaces: rows sent to the rank owning their key by
    one all-to-all, merged by packed key there) reproduces the key-based merge of GroupByCombineOperator across the
    ranks' shares, in the block layout the library's fetch reads (groups in ascending key order, others empty)."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_hashed_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    exp = _expected_union([_hashed_partial(r)[1] for r in range(world)])
    _check_shares(out, world, exp, lambda r: [1000 + r, 0, 0, 0])


def _disjoint_partial(rank):
    """40 groups per rank with keys no other rank holds (the case hashed key spaces exist for: high-cardinality raw
    keys): the union (120 at world 3) is larger than one rank's table of NS slots."""
    rng = np.random.default_rng(900 + rank)
    keys_used = (np.arange(40, dtype=np.int64) * 7919 + rank) * (1 << 20) - (1 << 40)
    slots = rng.choice(NS, size=40, replace=False)
    keys = np.full(NS, (1 << 63) - 1, np.int64)
    count = np.zeros(NS, np.int64)
    sx2 = np.zeros(2 * NS, np.int64)
    dsum = np.zeros(NS)
    dmin = np.full(NS, (1 << 63) - 1, np.int64)
    imax = np.full(NS, -(1 << 63), np.int64)
    hll = np.zeros(NS << HLOG, np.uint8)
    pres = np.zeros(NS * 16, np.uint8)
    groups = {}
    for k, s in zip(keys_used.tolist(), slots.tolist()):
        keys[s] = k
        count[s] = rng.integers(1, 50)
        v = int(rng.integers(-(1 << 40), 1 << 40))
        sx2[2 * s], sx2[2 * s + 1] = v & 0xFFFFFFFF, v >> 32
        dsum[s] = rng.standard_normal()
        dmin[s] = f64_order_encode(rng.standard_normal() * 100)
        imax[s] = rng.integers(-1000, 1000)
        hll[s << HLOG:(s + 1) << HLOG] = rng.integers(0, 20, 1 << HLOG)
        pres[s * 16:(s + 1) * 16] = rng.integers(0, 2, 16)
        groups[k] = (int(count[s]), v, float(dsum[s]), int(dmin[s]), int(imax[s]),
                     hll[s << HLOG:(s + 1) << HLOG].copy(), pres[s * 16:(s + 1) * 16].copy())
    secs = [(L.PA_ACC_COUNT_U64, count), (L.PA_ACC_SUM_I64X2, sx2), (L.PA_ACC_SUM_F64, dsum),
            (L.PA_ACC_MIN_I64, dmin), (L.PA_ACC_MAX_I64, imax), (L.PA_ACC_HLL_U8, hll),
            (L.PA_ACC_PRESENCE_U8, pres), (L.PA_ACC_KEYS_I64, keys),
            (L.PA_ACC_DOCS_U64, np.array([7 * rank, 0, 0, 0], np.int64))]
    return secs, groups


def test_gloo_hashed_merge_of_disjoint_keys_larger_than_one_table():
    """World size 3, every rank's keys disjoint from the others' and the union (120 groups) larger than one rank's
    table (64 slots): the key-partitioned merge leaves each rank a share that fits, matching the single-process
    merge (the all-gather design it replaces had to raise here)."""
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_hashed_worker, args=(world, _free_port(), out, _disjoint_partial), nprocs=world, join=True)
    exp = _expected_union([_disjoint_partial(r)[1] for r in range(world)])
    assert len(exp) == 120 > NS
    _check_shares(out, world, exp, lambda r: [7 * r, 0, 0, 0])


def test_gloo_hashed_merge_refuses_mismatched_key_spaces():
    """Ranks whose key spaces differ (e.g. DISTINCTCOUNT value dictionaries of the same size but different values)
    all raise before any row is exchanged."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_hashed_worker, args=(world, _free_port(), out, None, [b"V0:abc|", b"V0:abd|"]), nprocs=world, join=True)
    assert out[0][0] == "raised" and out[1][0] == "raised"


def test_key_space_fingerprint_covers_distinct_value_dictionaries():
    """presence byte j must mean the same value on every rank before the uint8-MAX reduce."""
    from pinot_amd.parallel import key_space_fingerprint

    class _E:
        num_keys, global_dicts, handle = 6, [np.array([1, 2, 3])], None

        def __init__(self, vd):
            self.value_dicts = vd

        def sections(self):
            return [(L.PA_ACC_COUNT_U64, 0, 6), (L.PA_ACC_PRESENCE_U8, 0, 6 * 16)]
    a = key_space_fingerprint(_E({1: np.array([10, 20, 30])}))
    assert a == key_space_fingerprint(_E({1: np.array([10, 20, 30])}))
    assert a != key_space_fingerprint(_E({1: np.array([10, 20, 31])}))  # same size, different values


def _distinct_layout_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd import parse_sql
    from pinot_amd.parallel import table_layout
    from pinot_amd.segment import create_segment
    q = parse_sql("SELECT k, DISTINCTCOUNT(v), COUNT(*) FROM t GROUP BY k")
    rng = np.random.default_rng(rank)
    # disjoint, equal-sized value dictionaries: rank 0 holds 0..49, rank 1 holds 100..149
    v = (rng.permutation(50).repeat(4) + 100 * rank).astype(np.int32)
    seg = create_segment("s%d" % rank, {"k": rng.integers(0, 5, size=200).astype(np.int32), "v": v},
                         {"k": "INT", "v": "INT"})
    lay = table_layout(q, [seg])
    out[rank] = (lay.value_dicts["v"].tolist(), lay.hash_keys_bound, lay.executor_kwargs()["value_dicts"] is lay.value_dicts)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_table_layout_agrees_on_distinct_value_dictionaries():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_distinct_layout_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    exp = list(range(50)) + list(range(100, 150))
    assert out[0] == out[1] == (exp, 200, True)


def _empty_rank_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd import parse_sql
    from pinot_amd.engine import GpuQueryExecutor, GpuSegment
    from pinot_amd.parallel import DistributedAccumulators, HashedAccumulators, check_same_key_space, table_layout
    from pinot_amd.segment import Segment
    from synth import make_segment
    q = parse_sql("SELECT d, COUNT(*), SUM(m), MAX(f) FROM t WHERE d > 3 GROUP BY d")
    cols = {"d": ("INT", 30), "m": ("LONG", 400), "f": ("DOUBLE", 50)}
    # rank 1 holds only empty segments
    segs = [make_segment(70 + i, 300, cols) for i in range(2)] if rank == 0 else [Segment("e0", 0), Segment("e1", 0)]
    layout = table_layout(q, segs)
    out["schema%d" % rank] = sorted((k, tuple(v)) for k, v in layout.schema.items())
    out["dict%d" % rank] = layout.dicts["d"].tolist()
    if rank == 1:
        # built without the layout, the empty-only rank has no accumulator block: it still joins the key-space check
        # (with -1), so every rank raises instead of rank 0 blocking in the collective
        ex = GpuQueryExecutor(q, [GpuSegment(s) for s in segs])
        assert ex.handle is None
        for acc_cls in (DistributedAccumulators, HashedAccumulators):
            try:
                acc = acc_cls(ex, "cpu")
                if acc_cls is HashedAccumulators:
                    acc.merge()
                out["raised1_%s" % acc_cls.__name__] = False
            except L.PinotAmdError:
                out["raised1_%s" % acc_cls.__name__] = True
    else:
        for name in ("DistributedAccumulators", "HashedAccumulators"):
            try:  # (the planned rank's side of the same check: its own fingerprint)
                check_same_key_space(4242, "cpu")
                out["raised0_" + name] = False
            except L.PinotAmdError:
                out["raised0_" + name] = True
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_rank_with_only_empty_segments():
    """a rank whose segments are all empty. table_layout gathers the referenced columns' schema from the
    ranks that hold docs (so that rank can plan a placeholder block of the agreed layout: test_gpu_dist.py); an executor
    built without it has no block, and both merge paths still run the key-space collective on it so every rank raises
    together — no rank is left blocked."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_empty_rank_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out["schema0"] == out["schema1"] == [("d", ("INT", True, True)), ("f", ("DOUBLE", True, True)),
                                                ("m", ("LONG", True, True))]
    assert out["dict0"] == out["dict1"] and len(out["dict0"]) > 0
    for name in ("DistributedAccumulators", "HashedAccumulators"):
        assert out["raised0_" + name] and out["raised1_" + name]


def _rs_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pinot_amd.parallel import reduce_scatter_sections
    secs, _ = partial(rank)
    views = [(k, torch.from_numpy(np.ascontiguousarray(a)).to(SECTION_DTYPE[k])) for k, a in secs]
    lo, hi = reduce_scatter_sections(views, K)
    out[rank] = (lo, hi, [t.numpy().copy() for _, t in views])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_reduce_scatter_gives_each_rank_its_key_range(world):
    """parallel.reduce_scatter_sections (large direct key spaces): rank r holds the merged rows of keys
    [r K', (r + 1) K') (the last rank also the K mod world remainder), identities elsewhere; the ranges tile the key
    space and every merged row equals the whole-block reduce."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rs_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    parts = [partial(r) for r in range(world)]
    exp_count = sum(p[0][0][1] for p in parts)
    exp_sum = sum(p[1].astype(object) for p in parts)
    exp_dsum = sum(p[0][2][1] for p in parts)
    exp_min = np.minimum.reduce([p[0][3][1] for p in parts])
    exp_max = np.maximum.reduce([p[0][4][1] for p in parts])
    exp_hll = np.maximum.reduce([p[0][5][1] for p in parts])
    covered = np.zeros(K, dtype=int)
    for r in range(world):
        lo, hi, (count, sx2, dsum, dmin, imax, hll) = out[r]
        covered[lo:hi] += 1
        mine = np.zeros(K, dtype=bool)
        mine[lo:hi] = True
        assert np.array_equal(count[mine], exp_count[mine]) and (count[~mine] == 0).all()
        total = sx2[0::2].astype(object) + (sx2[1::2].astype(object) << 32)
        assert all(a == b for a, b in zip(total[mine], exp_sum[mine])) and (sx2.reshape(K, 2)[~mine] == 0).all()
        assert np.allclose(dsum[mine], exp_dsum[mine], rtol=1e-12, atol=0) and (dsum[~mine] == 0).all()
        assert np.array_equal(dmin[mine], exp_min[mine]) and (dmin[~mine] == (1 << 63) - 1).all()
        assert np.array_equal(imax[mine], exp_max[mine]) and (imax[~mine] == -(1 << 63)).all()
        h = hll.reshape(K, -1)
        assert np.array_equal(h[mine], exp_hll.reshape(K, -1)[mine]) and (h[~mine] == 0).all()
    assert (covered == 1).all()


def _wide_partial(rank):
    """Two-word keys ([k0, k1, state] per slot): 40 groups per rank, half of them shared with the other ranks (same
    (k0, k1)), some sharing k0 with a different k1."""
    rng = np.random.default_rng(950 + rank)
    k0 = np.concatenate([np.arange(20, dtype=np.int64) * 7919 - (1 << 50), np.full(20, 123456789 + rank, np.int64)])
    k1 = np.concatenate([np.arange(20, dtype=np.int64), np.arange(20, dtype=np.int64) * 31 + rank])
    slots = rng.choice(NS, size=40, replace=False)
    keys = np.full(3 * NS, (1 << 63) - 1, np.int64)
    count = np.zeros(NS, np.int64)
    dsum = np.zeros(NS)
    imax = np.full(NS, -(1 << 63), np.int64)
    groups = {}
    for a, b, s in zip(k0.tolist(), k1.tolist(), slots.tolist()):
        keys[3 * s], keys[3 * s + 1], keys[3 * s + 2] = a, b, 5
        count[s] = rng.integers(1, 50)
        dsum[s] = rng.standard_normal()
        imax[s] = rng.integers(-1000, 1000)
        groups[(a, b)] = (int(count[s]), float(dsum[s]), int(imax[s]))
    secs = [(L.PA_ACC_COUNT_U64, count), (L.PA_ACC_SUM_F64, dsum), (L.PA_ACC_MAX_I64, imax), (L.PA_ACC_KEYS_I64, keys),
            (L.PA_ACC_DOCS_U64, np.array([10 + rank, 0, 0, 0], np.int64))]
    return secs, groups


def test_gloo_hashed_merge_of_two_word_keys():
    """merge_hashed_sections with two-word keys (group keys wider than 64 bits): rows go to the rank key_owner2 picks,
    and every rank ends with its share merged by (k0, k1) — keys sharing k0 stay distinct."""
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_hashed_worker, args=(world, _free_port(), out, _wide_partial), nprocs=world, join=True)
    from pinot_amd.parallel import key_owner2
    exp = {}
    for r in range(world):
        for k, (c, ds, mx) in _wide_partial(r)[1].items():
            e = exp.get(k, (0, 0.0, -(1 << 63)))
            exp[k] = (e[0] + c, e[1] + ds, max(e[2], mx))
    seen = []
    for r in range(world):
        u, (count, dsum, imax, keys, docs) = out[r]
        share = sorted(k for k in exp
                       if int(key_owner2(torch.tensor([k[0]]), torch.tensor([k[1]]), world)[0]) == r)
        kk = keys.reshape(NS, 3)
        assert u == len(share)
        assert [tuple(x) for x in kk[:u, :2].tolist()] == share
        for i, k in enumerate(share):
            c, ds, mx = exp[k]
            assert count[i] == c and abs(dsum[i] - ds) <= 1e-12 * max(1.0, abs(ds)) and imax[i] == mx
        assert (count[u:] == 0).all()
        assert docs.tolist() == [10 + r, 0, 0, 0]
        seen += share
    assert sorted(seen) == sorted(exp) and len(exp) == 20 + 20 * world


def test_layout_records_round_trip_without_pickle():
    """table_layout's per-rank record crosses ranks as tensor bytes (JSON header + raw arrays), not pickles: numeric and
    string dictionaries, nested dicts, lists and scalars survive the round trip."""
    from pinot_amd.parallel import _decode_record, _encode_record
    rec = {"dicts": {"d": np.array([3, 1, 2], dtype=np.int64), "s": np.array(["b", "a"], dtype=object)},
           "vals": {"f": np.array([1.5, -2.0])}, "wide": ["m"], "hb": 12345678901,
           "schema": {"d": ("INT", True, True)}}
    out = _decode_record(_encode_record(rec))
    np.testing.assert_array_equal(out["dicts"]["d"], rec["dicts"]["d"])
    assert out["dicts"]["d"].dtype == np.int64
    assert list(out["dicts"]["s"]) == ["b", "a"]
    np.testing.assert_array_equal(out["vals"]["f"], rec["vals"]["f"])
    assert out["wide"] == ["m"] and out["hb"] == 12345678901 and tuple(out["schema"]["d"]) == ("INT", True, True)
    assert b"\x80\x04" not in _encode_record(rec)[:2]  # (not a pickle stream)
