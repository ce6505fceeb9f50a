"""Multi-GPU segment sharding + cross-GPU merge of partial aggregates.

One process per GPU. Every rank owns a disjoint segment set (segments shard naturally: no data-path exchange) and
accumulates it into the SAME table-wide key space; the GroupByCombineOperator / AggregationCombineOperator merge of
partial aggregates across GPUs then becomes one collective per accumulator section over RCCL (xGMI):
SUM for COUNT/SUM, MIN for MIN, MAX for MAX and for HLL registers (HyperLogLog.addAll == register max).
"""
import ctypes
import hashlib
from dataclasses import dataclass, field

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


def shard_segments(num_segments, rank, world_size):
    """Contiguous segment ranges per rank (each GPU owns a segment set; ranks differ by at most one segment)."""
    per = num_segments // world_size
    extra = num_segments % world_size
    start = rank * per + min(rank, extra)
    return list(range(start, start + per + (1 if rank < extra else 0)))


# DistributedAccumulators.reduce(execution_stats=False): the merged block carries no execution statistics
NO_MERGED_STATS = "no merged execution statistics"


def reduce_sections(views, dst=0, group=None, all_reduce=False):
    """views: [(section kind, tensor)] -> reduced in place on `dst` (or everywhere)."""
    for kind, t in views:
        if all_reduce:
            dist.all_reduce(t, op=SECTION_OP[kind], group=group)
        else:
            dist.reduce(t, dst=dst, op=SECTION_OP[kind], group=group)


def key_owner(keys, world):
    """Rank that owns packed key `keys` in the cross-GPU merge of hashed key spaces: a multiplicative hash of the key,
    its high bits taken modulo the world size (int64 tensor ops: products wrap, the arithmetic shift is masked). The
    library's pack kernel computes the same function (pa_merge.hip owner_of)."""
    h = keys ^ (keys >> 31)
    h = h * -7046029254386353131  # 0x9E3779B97F4A7C15 as a signed int64
    return ((h >> 33) & 0x7FFFFFFF) % world


def _mix64(x):
    """pa_keys.h mix64 on int64 tensors (products wrap; logical shifts as masked arithmetic ones)."""
    x = x ^ ((x >> 33) & 0x7FFFFFFF)
    x = x * -49064778989728563  # 0xff51afd7ed558ccd as a signed int64
    x = x ^ ((x >> 33) & 0x7FFFFFFF)
    x = x * -4265267296055464877  # 0xc4ceb9fe1a85ec53
    return x ^ ((x >> 33) & 0x7FFFFFFF)


def key_owner2(k0, k1, world):
    """key_owner of a two-word key (pa_merge.hip owner_of): the first word mixed with the second's hash."""
    return key_owner(k0 ^ _mix64(k1), world)


def row_layout_fingerprint(views, num_slots, extra=b""):
    """62-bit digest of what the ranks of a hashed merge must share: every section's kind and row width (elements per
    slot, not the slot count) and `extra` (the key space: dictionaries and DISTINCTCOUNT value dictionaries)."""
    h = hashlib.blake2b(extra, digest_size=8)
    for k, t in views:
        w = t.numel() if k == L.PA_ACC_DOCS_U64 else t.numel() // max(1, num_slots)
        h.update(np.array([k, w, t.element_size()], dtype=np.int64).tobytes())
    return int.from_bytes(h.digest(), "little") & ((1 << 62) - 1)


def merge_hashed_sections(views, num_slots, group=None, layout_extra=b"", rows=None):
    """Device-side merge of hashed key spaces across ranks (GroupByCombineOperator semantics, value-keyed: a packed key
    means the same group values on every rank once parallel.table_layout agreed the dictionaries, but sits in a
    different slot of each rank's table). views: [(section kind, 1-D tensor)] of ONE rank's accumulator block, the
    per-key sections holding num_slots rows each (row width = elements / num_slots) plus the PA_ACC_DOCS_U64 counters.

    The key space is split across ranks by a hash of the packed key: every rank packs its occupied slots (count > 0)
    into byte rows grouped by the rank that owns their key, sends each row there (one all-to-all over the collective
    backend: RCCL on GPUs, so no rank ever holds the whole union), and merges the rows it receives by packed key into
    its own block. `rows` does the two local halves: rows.pack(world) -> (uint8 [m, row bytes] grouped by owner rank,
    rows per owner) and rows.merge(received) -> (groups held, rows that found no free slot); HashedAccumulators passes
    LibraryRows (the library's pack / merge kernels: pa_query_pack_rows / pa_query_merge_rows). The merged share is
    this rank's block afterwards, so the executor's own fetch returns it. The shares are disjoint and together are the
    merged result: each rank's fetch is one partial DataTable of disjoint groups, which the broker's reduce
    concatenates (numDocsScanned and the other counters stay per rank: the broker sums them).

    Before any exchange the ranks agree on the row layout (row_layout_fingerprint, one all-reduce: mismatched widths
    would hand the all-to-all rows of different sizes), and after the merge on whether every share fit its table
    (tables sized from parallel.table_layout's agreed key bound hold twice the largest rank's keys, and a share is
    ~1/world of the union); every rank raises together otherwise. Returns this rank's merged group count."""
    if rows is None:
        raise L.PinotAmdError("merge_hashed_sections: no row operations (HashedAccumulators passes the library's)")
    kinds = [k for k, _ in views]
    if L.PA_ACC_KEYS_I64 not in kinds or L.PA_ACC_COUNT_U64 not in kinds:
        raise L.PinotAmdError("merge_hashed_sections: the block has no key or count section")
    dev = dict(views)[L.PA_ACC_COUNT_U64].device
    check_same_key_space(row_layout_fingerprint(views, num_slots, layout_extra), dev, group=group,
                         what="hashed merge: ranks hold different accumulator row layouts or key spaces")
    world = dist.get_world_size(group)
    local, sn = rows.pack(world)
    send_n = torch.tensor(sn, dtype=torch.int64, device=dev)
    recv_n = torch.empty_like(send_n)
    dist.all_to_all_single(recv_n, send_n, group=group)
    rn = recv_n.tolist()
    received = torch.empty(sum(rn), local.shape[1], dtype=torch.uint8, device=dev)
    dist.all_to_all_single(received, local.contiguous(), output_split_sizes=rn, input_split_sizes=list(sn),
                           group=group)
    u, over = rows.merge(received)
    # every rank learns whether some share overflowed its table
    flag = torch.tensor([over], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag.item()) > 0:
        raise L.PinotAmdError("hashed merge: a rank's share of the merged groups exceeds its table by %d rows (size "
                              "the tables with parallel.table_layout's hash_keys_bound)" % int(flag.item()))
    return u


class LibraryRows:
    """The local halves of merge_hashed_sections on the device, through the library (pa_merge.hip): pack =
    pa_query_pack_rows (occupied slots -> rows grouped by owner rank), merge = pa_query_merge_rows (reset the block,
    insert every received row's packed key into the table, combine each accumulator with its section's operator)."""

    def __init__(self, executor, device):
        self.handle = executor.handle
        self.device = device
        self.row_bytes = L.check(L.lib().pa_query_row_bytes(self.handle), "pa_query_row_bytes")

    def pack(self, world):
        lib = L.lib()
        counts = np.zeros(world, dtype=np.int64)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        L.check(lib.pa_query_pack_rows(self.handle, world, None, counts.ctypes.data, stream), "pa_query_pack_rows")
        out = torch.empty(int(counts.sum()), self.row_bytes, dtype=torch.uint8, device=self.device)
        if out.shape[0]:
            L.check(lib.pa_query_pack_rows(self.handle, world, out.data_ptr(), counts.ctypes.data, stream),
                    "pa_query_pack_rows")
        return out, counts.tolist()

    def merge(self, received):
        groups, over = ctypes.c_int64(), ctypes.c_int64()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        L.check(L.lib().pa_query_merge_rows(self.handle, received.data_ptr() if received.shape[0] else None,
                                            int(received.shape[0]), ctypes.byref(groups), ctypes.byref(over), stream),
                "pa_query_merge_rows")
        return int(groups.value), int(over.value)


class HashedAccumulators:
    """The hashed-key-space counterpart of DistributedAccumulators: moves an executor's accumulator block into a
    torch-owned device buffer (construct it BEFORE executing the query: the block is relocated, not copied), and
    merge() runs merge_hashed_sections over it on every rank, after which executor.fetch() returns this rank's share
    of the merged groups (disjoint across ranks)."""

    def __init__(self, executor, device):
        self.device = device
        self.views = None
        if executor.handle is None:
            # a rank whose segments are all empty, built without the layout's schema (executor_kwargs): it has no block,
            # so merge() joins the layout check with -1 and every rank raises there (none is left blocked)
            return
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
        self.key_space = key_space_bytes(executor)
        self.rows = LibraryRows(executor, device)
        self.views = []
        for kind, ptr, n in executor.sections():
            off = ptr - self.buf.data_ptr()
            dt = SECTION_DTYPE[kind]
            es = torch.empty(0, dtype=dt).element_size()
            self.views.append((kind, self.buf[off:off + n * es].view(dt)))

    def merge(self, group=None):
        if self.views is None:
            check_same_key_space(-1, self.device, group=group,
                                 what="hashed merge: a rank holds only empty segments and no table layout (build its "
                                      "executor with parallel.table_layout(...).executor_kwargs())")
        return merge_hashed_sections(self.views, self.num_slots, group=group, layout_extra=self.key_space,
                                     rows=self.rows)


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
    hold a value outside int32, raw or in the dictionary (the library picks SUM_I64 for all-int32 columns, SUM_I64X2
    else: pa_segment.hip pa_segment_add_raw_column / upload_dict)."""
    out = set()
    for a in query.aggregations:
        if a.function not in SUM_FUNCTIONS or a.column in out:
            continue
        for s in segments:
            c = s.column(a.column)
            if c.data_type != "LONG":
                continue
            d = np.asarray(c.dictionary if c.has_dictionary else c.raw_values, dtype=np.int64)
            if len(d) and (d.min() < -(1 << 31) or d.max() >= (1 << 31)):
                out.add(a.column)
                break
    return out


def hash_keys_bound_local(query, segments):
    """The hashed key space's key bound of these segments (pa_plan.hip plan_key_space): every doc a key, or twice the
    values of a multi-value group-by column."""
    b = 0
    for s in segments:
        n = s.num_docs
        for name in query.group_by:
            c = s.column(name)
            if not c.single_value:
                n = max(n, int(c.total_num_values)) * 2
        b += n
    return b


@dataclass
class TableLayout:
    """What the ranks of one multi-GPU query agree on before building their executors (table_layout)."""
    dicts: dict = field(default_factory=dict)        # group-by column -> table-wide dictionary (sorted unique values)
    wide: list = field(default_factory=list)         # SUM columns that keep the 64-bit accumulator on every rank
    value_dicts: dict = field(default_factory=dict)  # DISTINCTCOUNT column -> table-wide value dictionary
    hash_keys_bound: int = 0                         # the largest rank's hashed key bound (equal tables everywhere)
    schema: dict = field(default_factory=dict)       # column -> (data type, has dictionary, single value): lets a rank
                                                     # whose segments are all empty plan the same accumulator block

    def executor_kwargs(self):
        """Keyword arguments of GpuQueryExecutor that make every rank's accumulator block line up."""
        return dict(table_dicts=self.dicts, wide_sum_columns=self.wide, value_dicts=self.value_dicts,
                    hash_keys_bound=self.hash_keys_bound, schema=self.schema)


from .query import DISTINCT_SET_FUNCTIONS as DISTINCT_FUNCTIONS, query_columns  # noqa: E402


def _encode_record(rec):
    """A rank's layout record as bytes without pickling: a JSON header (scalars, lists, and per array its dtype, shape
    and byte range; string dictionaries as JSON lists) followed by the numeric arrays' raw bytes."""
    import json
    blobs, off = [], 0

    def enc(v):
        nonlocal off
        if isinstance(v, np.ndarray):
            if v.dtype.kind in "USO":
                return {"strs": [str(x) for x in v.tolist()]}
            a = np.ascontiguousarray(v)
            blobs.append(a.tobytes())
            d = {"dtype": a.dtype.str, "shape": list(a.shape), "off": off, "n": a.nbytes}
            off += a.nbytes
            return {"array": d}
        if isinstance(v, dict):
            return {"dict": {k: enc(x) for k, x in v.items()}}
        if isinstance(v, (list, tuple)):
            return {"list": [enc(x) for x in v]}
        if isinstance(v, (bool, np.bool_)):
            return {"v": bool(v)}
        if isinstance(v, (int, np.integer)):
            return {"v": int(v)}
        return {"v": v}

    head = json.dumps(enc(rec)).encode()
    return len(head).to_bytes(8, "little") + head + b"".join(blobs)


def _decode_record(buf):
    import json
    hl = int.from_bytes(buf[:8], "little")
    head = json.loads(buf[8:8 + hl].decode())
    body = buf[8 + hl:]

    def dec(v):
        if "array" in v:
            a = v["array"]
            return np.frombuffer(body[a["off"]:a["off"] + a["n"]], dtype=np.dtype(a["dtype"])).reshape(a["shape"]).copy()
        if "strs" in v:
            return np.asarray(v["strs"], dtype=object)
        if "dict" in v:
            return {k: dec(x) for k, x in v["dict"].items()}
        if "list" in v:
            return [dec(x) for x in v["list"]]
        return v["v"]

    return dec(head)


def all_gather_records(rec, group=None):
    """Every rank's record (dicts / lists / scalars / numpy arrays) on every rank, through two tensor all-gathers (byte
    lengths, then the padded byte images) on the group's backend device: no pickles cross the wire."""
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    data = _encode_record(rec)
    n = torch.tensor([len(data)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    cap = int(max(int(x.item()) for x in ns))
    mine = torch.zeros(cap, dtype=torch.uint8, device=dev)
    if len(data):
        mine[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    outs = [torch.zeros(cap, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, mine, group=group)
    return [_decode_record(bytes(o[:int(k.item())].cpu().numpy().tobytes())) for o, k in zip(outs, ns)]


def table_layout(query, segments, group=None):
    """Everything the ranks of one multi-GPU query must agree on before building their executors, in one all-gather:
    the table-wide dictionary of every dictionary-encoded group-by column (the union over all ranks' segments: the
    value-keyed combine of GroupByCombineOperator needs the same key id for the same value on every GPU), the SUM
    columns that need the wide accumulator on some rank, the table-wide value dictionary of every DISTINCTCOUNT column
    (presence byte j must mean the same value on every rank before the uint8-MAX reduce ORs them) and the largest
    rank's hashed key bound (every rank's hashed table then has the same slots). Returns a TableLayout; build every
    rank's executor with GpuQueryExecutor(..., **layout.executor_kwargs())."""
    segments = [s for s in segments if s.num_docs > 0]  # (empty segments hold no columns: SegmentColumnarIndexCreator)
    local = {"dicts": {}, "vals": {}, "wide": sorted(wide_sum_columns_local(query, segments)),
             "hb": hash_keys_bound_local(query, segments), "schema": {}}
    for s in segments:
        for name in query_columns(query):
            c = s.column(name)
            local["schema"].setdefault(name, (c.data_type, bool(c.has_dictionary), bool(c.single_value)))
    for name in query.group_by:
        ds = [s.column(name).dictionary for s in segments if s.column(name).has_dictionary]
        if ds:
            local["dicts"][name] = np.unique(np.concatenate(ds))
    for a in query.aggregations:
        if a.function in DISTINCT_FUNCTIONS and a.column not in local["vals"]:
            ds = [s.column(a.column).dictionary for s in segments if s.column(a.column).has_dictionary]
            if ds:
                local["vals"][a.column] = np.unique(np.concatenate(ds))
    gathered = all_gather_records(local, group)
    out = TableLayout()
    for name in query.group_by:
        parts = [g["dicts"][name] for g in gathered if name in g["dicts"]]
        if parts:
            out.dicts[name] = np.unique(np.concatenate(parts))
    for name in sorted(set().union(*[set(g["vals"]) for g in gathered])):
        out.value_dicts[name] = np.unique(np.concatenate([g["vals"][name] for g in gathered if name in g["vals"]]))
    out.wide = sorted(set().union(*[set(g["wide"]) for g in gathered]))
    out.hash_keys_bound = max(int(g["hb"]) for g in gathered)
    for g in gathered:
        for name, meta in g["schema"].items():
            out.schema.setdefault(name, tuple(meta))
    return out



def table_dictionaries(query, segments, group=None):
    """Table-wide dictionaries of the query's dictionary-encoded group-by columns, agreed across ranks (table_layout's
    first half, for callers that need only the key space)."""
    return table_layout(query, segments, group=group).dicts


def _array_bytes(a):
    a = np.asarray(a)
    if a.dtype.kind in "USO":
        return "\x00".join(map(str, a.tolist())).encode()
    return np.ascontiguousarray(a).tobytes()


def key_space_bytes(executor):
    """Byte image of an executor's key space: every group-by dictionary (or <raw>) and every DISTINCTCOUNT value
    dictionary, in a fixed order."""
    parts = []
    for gd in executor.global_dicts:
        parts.append(b"<raw>" if gd is None else _array_bytes(gd))
        parts.append(b"|")
    for i in sorted(getattr(executor, "value_dicts", {}) or {}):
        parts.append(b"V%d:" % i + _array_bytes(executor.value_dicts[i]) + b"|")
    return b"".join(parts)


def key_space_fingerprint(executor):
    """62-bit digest of everything an element-wise cross-GPU reduce relies on: the table-wide key space (key count,
    every group-by dictionary's values and every DISTINCTCOUNT value dictionary), whether it is hashed, and the
    accumulator block layout (every section's kind and element count, the block size) — a SUM over INT on one rank and
    over values beyond int32 on another would otherwise hand RCCL collectives of different lengths, and presence bytes
    over different value dictionaries would OR unrelated values."""
    lib = L.lib()
    h = hashlib.blake2b(np.int64(executor.num_keys).tobytes(), digest_size=8)
    h.update(b"hashed" if getattr(executor, "hashed", False) else b"direct")
    h.update(np.int64(lib.pa_query_accumulator_bytes(executor.handle)).tobytes())
    for kind, _, n in executor.sections():
        h.update(np.array([kind, n], dtype=np.int64).tobytes())
    h.update(key_space_bytes(executor))
    return int.from_bytes(h.digest(), "little") & ((1 << 62) - 1)


def check_same_key_space(fingerprint, device, group=None, what=None):
    """Raises on EVERY rank unless all ranks hold the same key space and accumulator layout (element-wise section
    reduces would hang or be silently wrong). A rank that cannot take part passes fingerprint -1: the collective still
    runs everywhere, so no rank is left blocked in it."""
    t = torch.tensor([fingerprint, -fingerprint], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if int(t[0]) != fingerprint or -int(t[1]) != fingerprint or fingerprint < 0:
        raise L.PinotAmdError(what or "ranks hold different group-key spaces or accumulator layouts (or a hashed key "
                              "space): build the executors with parallel.table_layout(...).executor_kwargs()")


def reduce_scatter_sections(per_key, num_keys, group=None):
    """per_key: [(section kind, 1-D tensor)] of the per-key sections of a direct key space (num_keys rows each; the
    numDocsScanned counters excluded). Instead of reducing the whole block onto one rank, every rank ends up holding the
    merged rows of its own key range — keys [r K', (r + 1) K') with K' = floor(K / world), one reduce-scatter per
    section (each rank receives 1/world of the block: over xGMI every link carries 1/world of it per step instead of the
    whole block converging on one GPU), and the K mod world remainder keys (all-reduced) on the last rank. Every other
    row is reset to its section's identity (count 0: the executor's fetch skips it), so each rank's fetch returns its
    share of the groups, disjoint across ranks — partial DataTables the broker concatenates; numDocsScanned and the
    other counters stay per rank (the broker sums them). Returns the rank's key range (lo, hi)."""
    world, r = dist.get_world_size(group), dist.get_rank(group)
    K = int(num_keys)
    kr = K // world
    lo, hi = r * kr, (r + 1) * kr + (K - kr * world if r == world - 1 else 0)
    for kind, t in per_key:
        w = t.numel() // K
        op, ident = SECTION_OP[kind], SECTION_IDENTITY.get(kind, 0)
        out = torch.empty(kr * w, dtype=t.dtype, device=t.device)
        if kr:
            dist.reduce_scatter_tensor(out, t[:kr * world * w], op=op, group=group)
        rem = t[kr * world * w:]
        if rem.numel():
            dist.all_reduce(rem, op=op, group=group)
        t[:lo * w].fill_(ident)
        t[lo * w:(lo + kr) * w].copy_(out)
        if r != world - 1:
            t[(lo + kr) * w:].fill_(ident)
    return lo, hi


class DistributedAccumulators:
    """Moves an executor's accumulators into one torch-owned device block and reduces it across ranks (direct key
    spaces: the same key id addresses the same accumulator row on every GPU)."""

    def __init__(self, executor, device):
        hashed = getattr(executor, "hashed", False)
        if dist.is_initialized():
            # the collective first, on every rank (a hashed rank, or one holding only empty segments and built without the
            # layout's schema, joins with -1 and every rank then raises)
            check_same_key_space(-1 if (hashed or executor.handle is None) else key_space_fingerprint(executor), device)
        if executor.handle is None:
            raise L.PinotAmdError("a rank holds only empty segments and no table layout: build its executor with "
                                  "parallel.table_layout(...).executor_kwargs()")
        if hashed:
            raise L.PinotAmdError("hashed key space: merge with HashedAccumulators (slots differ per GPU)")
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
        self.executor = executor
        runs = section_runs([(kind, ptr - self.base + pad, n) for kind, ptr, n in executor.sections()])
        self.views = [(kind, self.buf[a:b].view(dt)) for kind, dt, a, b in runs]
        self.num_keys = int(executor.num_keys)
        self.per_key = []  # [(kind, 1-D view)] of every per-key section (the counters excluded)
        for kind, ptr, n in executor.sections():
            if kind == L.PA_ACC_DOCS_U64:
                continue
            dt = SECTION_DTYPE[kind]
            es = torch.empty(0, dtype=dt).element_size()
            off = ptr - self.base + pad
            self.per_key.append((kind, self.buf[off:off + n * es].view(dt)))

    def reduce(self, dst=0, all_reduce=False, execution_stats=True, group=None):
        """Element-wise merge onto rank `dst` (every rank with all_reduce; `dst` is a global rank, as torch.distributed's
        reduce takes it, also under a subgroup). numDocsScanned is summed too, so the merged results block's execution
        statistics are every rank's own pair summed before the collective (one extra 16-byte all-reduce and a host sync
        per query). execution_stats=False skips that (the timed bench steps, which fetch without statistics): the merged
        block then has no statistics, and a fetch that asks for them raises instead of returning (0, 0)."""
        ex = self.executor
        if execution_stats:
            local = torch.tensor(list(ex.execution_stats()), dtype=torch.int64, device=self.buf.device)
            if dist.is_initialized():
                dist.all_reduce(local, group=group)
            stats = tuple(int(v) for v in local.tolist())
        else:
            stats = NO_MERGED_STATS
        reduce_sections(self.views, dst=dst, group=group, all_reduce=all_reduce)
        if all_reduce or not dist.is_initialized() or dist.get_rank() == dst:
            ex.merged_stats = stats

    def reduce_scatter(self, group=None):
        """Large direct key spaces: every rank ends up holding the merged rows of its own key range
        (reduce_scatter_sections), so each rank's fetch returns its share of the groups. Returns the range (lo, hi)."""
        return reduce_scatter_sections(self.per_key, self.num_keys, group)

    def merge(self, dst=0, group=None, scatter_keys=1 << 20, execution_stats=True):
        """The cross-GPU merge this key space wants: key spaces of at least `scatter_keys` keys reduce-scatter (every
        rank then fetches its share: returns True), smaller ones reduce onto rank `dst`, the one rank that fetches
        (returns False)."""
        if self.num_keys >= scatter_keys:
            self.reduce_scatter(group)
            return True
        self.reduce(dst=dst, execution_stats=execution_stats, group=group)
        return False
