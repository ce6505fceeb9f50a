"""Multi-GPU segment sharding + cross-GPU merge of partial aggregates.

One process per GPU. Every rank owns a disjoint segment set (segments shard naturally: no data-path exchange) and
accumulates it into the SAME table-wide key space; the GroupByCombineOperator / AggregationCombineOperator merge of
partial aggregates across GPUs then becomes one collective per accumulator section over RCCL (xGMI):
SUM for COUNT/SUM, MIN for MIN, MAX for MAX and for HLL registers (HyperLogLog.addAll == register max).
"""
import hashlib

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

SECTION_OP = {
    L.PA_ACC_COUNT_U64: dist.ReduceOp.SUM,
    L.PA_ACC_SUM_I64: dist.ReduceOp.SUM,
    L.PA_ACC_SUM_I64X2: dist.ReduceOp.SUM,
    L.PA_ACC_SUM_F64: dist.ReduceOp.SUM,
    L.PA_ACC_MIN_I64: dist.ReduceOp.MIN,
    L.PA_ACC_MAX_I64: dist.ReduceOp.MAX,
    L.PA_ACC_HLL_U8: dist.ReduceOp.MAX,
    L.PA_ACC_DOCS_U64: dist.ReduceOp.SUM,
    L.PA_ACC_PRESENCE_U8: dist.ReduceOp.MAX,  # DISTINCTCOUNT value presence bytes (set union)
    L.PA_ACC_KEYS_I64: None,  # not element-wise reducible (hashed key spaces)
}
SECTION_DTYPE = {
    L.PA_ACC_COUNT_U64: torch.int64,
    L.PA_ACC_SUM_I64: torch.int64,
    L.PA_ACC_SUM_I64X2: torch.int64,
    L.PA_ACC_SUM_F64: torch.float64,
    L.PA_ACC_MIN_I64: torch.int64,
    L.PA_ACC_MAX_I64: torch.int64,
    L.PA_ACC_HLL_U8: torch.uint8,  # one byte per register (HyperLogLog.addAll == register max)
    L.PA_ACC_DOCS_U64: torch.int64,
    L.PA_ACC_PRESENCE_U8: torch.uint8,
    L.PA_ACC_KEYS_I64: torch.int64,
}
# identity of each per-key section (what pa_query_reset leaves in an empty slot)
SECTION_IDENTITY = {
    L.PA_ACC_MIN_I64: (1 << 63) - 1,
    L.PA_ACC_MAX_I64: -(1 << 63),
    L.PA_ACC_KEYS_I64: (1 << 63) - 1,  # the empty-slot marker
}
_SCATTER_REDUCE = {dist.ReduceOp.SUM: "sum", dist.ReduceOp.MIN: "amin", dist.ReduceOp.MAX: "amax"}


def shard_segments(num_segments, rank, world_size):
    """Contiguous segment ranges per rank (each GPU owns a segment set; ranks differ by at most one segment)."""
    per = num_segments // world_size
    extra = num_segments % world_size
    start = rank * per + min(rank, extra)
    return list(range(start, start + per + (1 if rank < extra else 0)))


def reduce_sections(views, dst=0, group=None, all_reduce=False):
    """views: [(section kind, tensor)] -> reduced in place on `dst` (or everywhere)."""
    for kind, t in views:
        if all_reduce:
            dist.all_reduce(t, op=SECTION_OP[kind], group=group)
        else:
            dist.reduce(t, dst=dst, op=SECTION_OP[kind], group=group)


def merge_results_across_ranks(executor, dst=0, group=None):
    """Key-based merge for hashed key spaces (accumulator slots differ per GPU, so sections cannot be reduced element-
    wise): every rank fetches its groups and rank `dst` merges them by key value (GroupByCombineOperator / broker
    reduce semantics, reduce.merge_intermediate). Returns the merged IntermediateResult on `dst`, None elsewhere."""
    from .reduce import merge_intermediate
    res = executor.fetch()
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    gathered = [None] * world if rank == dst else None
    dist.gather_object(res, gathered, dst=dst, group=group)
    return merge_intermediate(gathered) if rank == dst else None


def merge_hashed_sections(views, num_slots, group=None):
    """Device-side merge of hashed key spaces across ranks (GroupByCombineOperator semantics, value-keyed: a packed key
    means the same group values on every rank once parallel.table_layout agreed the dictionaries, but sits in a
    different slot of each rank's table). views: [(section kind, 1-D tensor)] of ONE rank's accumulator block, the
    per-key sections holding num_slots rows each (row width = elements / num_slots) plus the PA_ACC_DOCS_U64 counters.

    Every rank: compact its occupied slots (count > 0) into byte rows, all-gather them over the collective backend
    (RCCL on GPUs), then merge by packed key on its own device — torch.unique over the keys and one scatter-reduce per
    section (SUM for counts/sums, MIN, MAX for maxima, HLL registers and DISTINCTCOUNT presence) — and write the merged
    groups back into the block: slots [0, groups) in ascending key order, every other slot empty. pa_query_fetch reads
    slots by count and key, not by position, so the executor's own fetch then returns the merged result on every rank.
    Raises when the merged groups do not fit the table."""
    kinds = [k for k, _ in views]
    if L.PA_ACC_KEYS_I64 not in kinds or L.PA_ACC_COUNT_U64 not in kinds:
        raise L.PinotAmdError("merge_hashed_sections: the block has no key or count section")
    docs = [t for k, t in views if k == L.PA_ACC_DOCS_U64]
    per_key = [(k, t) for k, t in views if k != L.PA_ACC_DOCS_U64]
    for t in docs:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    count = dict(per_key)[L.PA_ACC_COUNT_U64]
    dev = count.device
    occ = torch.nonzero(count.view(num_slots) > 0).flatten()
    m = int(occ.numel())
    # one byte row per occupied slot: every per-key section's row, concatenated
    parts, layout = [], []
    for k, t in per_key:
        w = t.numel() // num_slots
        rows = t.view(num_slots, w)[occ]
        b = rows.contiguous().view(torch.uint8).view(m, -1) if m else torch.empty(0, w * t.element_size(),
                                                                                  dtype=torch.uint8, device=dev)
        layout.append((k, t.dtype, w, b.shape[1]))
        parts.append(b)
    local = torch.cat(parts, dim=1) if parts else torch.empty(m, 0, dtype=torch.uint8, device=dev)
    rb = local.shape[1]
    world = dist.get_world_size(group)
    sizes = torch.tensor([m], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    ns = [int(s.item()) for s in all_sizes]
    mx = max(ns)
    padded = torch.zeros(mx, rb, dtype=torch.uint8, device=dev)
    padded[:m] = local
    gathered = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(gathered, padded, group=group)
    rows = torch.cat([g[:n] for g, n in zip(gathered, ns)], dim=0)
    # unpack per section, merge by packed key
    cols, o = {}, 0
    for k, dt, w, nb in layout:
        cols[k] = rows[:, o:o + nb].contiguous().view(dt).view(-1, w)
        o += nb
    keys = cols[L.PA_ACC_KEYS_I64][:, 0]
    uniq, inv = torch.unique(keys, sorted=True, return_inverse=True)
    u = int(uniq.numel())
    if u > num_slots:
        raise L.PinotAmdError("merged groups (%d) exceed the hashed table's %d slots" % (u, num_slots))
    for k, t in per_key:
        w = t.numel() // num_slots
        out = t.view(num_slots, w)
        out.fill_(SECTION_IDENTITY.get(k, 0))
        if k == L.PA_ACC_KEYS_I64:
            out[:u, 0] = uniq
            continue
        acc = torch.full((u, w), SECTION_IDENTITY.get(k, 0), dtype=t.dtype, device=dev)
        acc.scatter_reduce_(0, inv.view(-1, 1).expand(-1, w), cols[k], reduce=_SCATTER_REDUCE[SECTION_OP[k]],
                            include_self=True)
        out[:u] = acc
    return u


class HashedAccumulators:
    """The hashed-key-space counterpart of DistributedAccumulators: moves an executor's accumulator block into a
    torch-owned device buffer (construct it BEFORE executing the query: the block is relocated, not copied), and
    merge() runs merge_hashed_sections over it on every rank, after which executor.fetch() returns the merged groups
    on every rank."""

    def __init__(self, executor, device):
        if not getattr(executor, "hashed", False):
            raise L.PinotAmdError("HashedAccumulators: direct key spaces reduce element-wise (DistributedAccumulators)")
        lib = L.lib()
        nbytes = int(lib.pa_query_accumulator_bytes(executor.handle))
        self.buf = torch.zeros(nbytes + 512, dtype=torch.uint8, device=device)
        pad = (-self.buf.data_ptr()) % 256
        base = self.buf.data_ptr() + pad
        L.check(lib.pa_query_set_accumulator_buffer(executor.handle, base, nbytes), "set_accumulator_buffer")
        executor._acc_owner = self.buf  # the library reads and writes this block for the executor's lifetime
        self.num_slots = int(executor.num_keys)
        self.views = []
        for kind, ptr, n in executor.sections():
            off = ptr - self.buf.data_ptr()
            dt = SECTION_DTYPE[kind]
            es = torch.empty(0, dtype=dt).element_size()
            self.views.append((kind, self.buf[off:off + n * es].view(dt)))

    def merge(self, group=None):
        return merge_hashed_sections(self.views, self.num_slots, group=group)


def section_runs(sections):
    """[(kind, byte offset, elements)] -> [(kind, dtype, start byte, end byte)]: adjacent sections with the same reduce
    op and element type merge into one collective over the byte span they cover (the 256-B alignment gaps between
    them are zero and stay zero under SUM/MIN/MAX). The bench query's COUNT + 2x SUM(LONG) + numDocsScanned sections
    become one RCCL reduce per step instead of four: small-message latency, not bytes, is the cost of this merge."""
    runs = []
    for kind, off, n in sorted(sections, key=lambda s: s[1]):
        dt = SECTION_DTYPE[kind]
        es = torch.empty(0, dtype=dt).element_size()
        op = SECTION_OP[kind]
        if op is not None and runs and SECTION_OP[runs[-1][0]] == op and runs[-1][1] == dt:
            runs[-1][3] = off + n * es
        else:
            runs.append([kind, dt, off, off + n * es])
    return [tuple(r) for r in runs]


SUM_FUNCTIONS = ("SUM", "AVG", "SUMMV", "AVGMV")


def wide_sum_columns_local(query, segments):
    """Columns of this rank's segments whose SUM needs the 64-bit accumulator (PA_AGGF_WIDE_SUM): LONG columns that are
    raw or hold a dictionary value outside int32 (the library picks SUM_I64 for all-int32 columns, SUM_I64X2 else)."""
    out = set()
    for a in query.aggregations:
        if a.function not in SUM_FUNCTIONS or a.column in out:
            continue
        for s in segments:
            c = s.column(a.column)
            if c.data_type != "LONG":
                continue
            if not c.has_dictionary:
                out.add(a.column)
                break
            d = np.asarray(c.dictionary, dtype=np.int64)
            if len(d) and (d.min() < -(1 << 31) or d.max() >= (1 << 31)):
                out.add(a.column)
                break
    return out


def table_layout(query, segments, group=None):
    """Everything the ranks of one multi-GPU query must agree on before building their executors, in one all-gather:
    the table-wide dictionary of every dictionary-encoded group-by column (the union over all ranks' segments: the
    value-keyed combine of GroupByCombineOperator needs the same key id for the same value on every GPU) and the SUM
    columns that need the wide accumulator on some rank. Pass both to GpuQueryExecutor(table_dicts=...,
    wide_sum_columns=...) on every rank."""
    local = {"dicts": {}, "wide": sorted(wide_sum_columns_local(query, segments))}
    for name in query.group_by:
        ds = [s.column(name).dictionary for s in segments if s.column(name).has_dictionary]
        if ds:
            local["dicts"][name] = np.unique(np.concatenate(ds))
    world = dist.get_world_size(group)
    gathered = [None] * world
    dist.all_gather_object(gathered, local, group=group)
    dicts = {}
    for name in query.group_by:
        parts = [g["dicts"][name] for g in gathered if name in g["dicts"]]
        if parts:
            dicts[name] = np.unique(np.concatenate(parts))
    wide = sorted(set().union(*[set(g["wide"]) for g in gathered]))
    return dicts, wide


def table_dictionaries(query, segments, group=None):
    """Table-wide dictionaries of the query's dictionary-encoded group-by columns, agreed across ranks: the union of
    every rank's segment dictionaries (the value-keyed combine of GroupByCombineOperator needs the same key id for
    the same value on every GPU before accumulators can be reduced element-wise). Pass the result to
    GpuQueryExecutor(table_dicts=...) on every rank."""
    local = {}
    for name in query.group_by:
        ds = [s.column(name).dictionary for s in segments if s.column(name).has_dictionary]
        if ds:
            local[name] = np.unique(np.concatenate(ds))
    world = dist.get_world_size(group)
    gathered = [None] * world
    dist.all_gather_object(gathered, local, group=group)
    out = {}
    for name in query.group_by:
        parts = [g[name] for g in gathered if name in g]
        if parts:
            out[name] = np.unique(np.concatenate(parts))
    return out


def key_space_fingerprint(executor):
    """62-bit digest of everything an element-wise cross-GPU reduce relies on: the table-wide key space (key count +
    every group-by dictionary's values), whether it is hashed, and the accumulator block layout (every section's kind
    and element count, the block size) — a SUM over INT on one rank and over values beyond int32 on another would
    otherwise hand RCCL collectives of different lengths."""
    lib = L.lib()
    h = hashlib.blake2b(np.int64(executor.num_keys).tobytes(), digest_size=8)
    h.update(b"hashed" if getattr(executor, "hashed", False) else b"direct")
    h.update(np.int64(lib.pa_query_accumulator_bytes(executor.handle)).tobytes())
    for kind, _, n in executor.sections():
        h.update(np.array([kind, n], dtype=np.int64).tobytes())
    for gd in executor.global_dicts:
        if gd is None:
            h.update(b"<raw>")
        elif np.asarray(gd).dtype.kind in "USO":
            h.update("\x00".join(map(str, gd)).encode())
        else:
            h.update(np.ascontiguousarray(gd).tobytes())
        h.update(b"|")
    return int.from_bytes(h.digest(), "little") & ((1 << 62) - 1)


def check_same_key_space(fingerprint, device, group=None):
    """Raises on EVERY rank unless all ranks hold the same key space and accumulator layout (element-wise section
    reduces would hang or be silently wrong). A rank that cannot take part passes fingerprint -1: the collective still
    runs everywhere, so no rank is left blocked in it."""
    t = torch.tensor([fingerprint, -fingerprint], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if int(t[0]) != fingerprint or -int(t[1]) != fingerprint or fingerprint < 0:
        raise L.PinotAmdError("ranks hold different group-key spaces or accumulator layouts (or a hashed key space): "
                              "build the executors with parallel.table_layout(...)")


class DistributedAccumulators:
    """Moves an executor's accumulators into one torch-owned device block and reduces it across ranks (direct key
    spaces: the same key id addresses the same accumulator row on every GPU)."""

    def __init__(self, executor, device):
        hashed = getattr(executor, "hashed", False)
        if dist.is_initialized():
            # the collective first, on every rank (a hashed rank joins with -1 and every rank then raises)
            check_same_key_space(-1 if hashed else key_space_fingerprint(executor), device)
        if hashed:
            raise L.PinotAmdError("hashed key space: merge with merge_results_across_ranks (slots differ per GPU)")
        lib = L.lib()
        nbytes = int(lib.pa_query_accumulator_bytes(executor.handle))
        self.buf = torch.zeros(nbytes + 512, dtype=torch.uint8, device=device)
        base = self.buf.data_ptr()
        pad = (-base) % 256
        self.base = base + pad
        L.check(lib.pa_query_set_accumulator_buffer(executor.handle, self.base, nbytes), "set_accumulator_buffer")
        # the library now reads and writes this torch-owned block: the executor keeps it alive for as long as it lives
        # (pa_query_set_accumulator_buffer: the caller owns the block and must outlive the query)
        executor._acc_owner = self.buf
        runs = section_runs([(kind, ptr - self.base + pad, n) for kind, ptr, n in executor.sections()])
        self.views = [(kind, self.buf[a:b].view(dt)) for kind, dt, a, b in runs]

    def reduce(self, dst=0, all_reduce=False):
        reduce_sections(self.views, dst=dst, all_reduce=all_reduce)
