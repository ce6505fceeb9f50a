"""GPU segment residency + query execution through the C-ABI.

Host-side mirror of the Java operator layer that stays in the JVM in a real integration:
  GpuSegment            ~ ImmutableSegmentLoader handing forward-index PinotDataBuffers to the GPU
  GpuQueryExecutor      ~ AggregationPlanNode/GroupByPlanNode -> AggregationOperator / GroupByOperator on every
                          segment + AggregationCombineOperator / GroupByCombineOperator
                          (pinot-core/.../operator/query/GroupByOperator.java:84,
                           operator/combine/GroupByCombineOperator.java:110)
It resolves predicates per segment (predicate.py), builds the table-wide group-key dictionaries (the value-keyed
merge GroupByCombineOperator performs with IndexedTable.upsert), and decodes the GPU's accumulators into the
reference's intermediate results: COUNT -> long, SUM/MIN/MAX -> double, AVG -> (sum, count),
DISTINCTCOUNTHLL -> HyperLogLog.
"""
import ctypes
import dataclasses
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _lib as L
from . import predicate as P
from . import query as Q
from .hll import HyperLogLog, hash_value
from .java_hash import java_hash_code
from .optimizer import optimize_filter
from .segment import Segment

_VTYPE = {"INT": L.PA_INT, "LONG": L.PA_LONG, "FLOAT": L.PA_FLOAT, "DOUBLE": L.PA_DOUBLE, "STRING": L.PA_STRING}


class UnsupportedQuery(L.PinotAmdError):
    pass


def column_ids_for(segment: Segment) -> Dict[str, int]:
    """Table-level column id assignment (stable across the segments of one table)."""
    return {name: i for i, name in enumerate(sorted(segment.columns))}


class GpuSegment:
    """HBM-resident forward indexes + dictionaries of one immutable segment (a pa_segment)."""

    def __init__(self, segment: Segment, columns=None, column_ids=None, device=None):
        lib = L.lib()
        if device is not None:
            L.check(lib.pa_set_device(int(device)), "pa_set_device")
        self.device = None if device is None else int(device)  # (None: the caller's current device)
        self.segment = segment
        self.column_ids = dict(column_ids or column_ids_for(segment))
        self.handle = L.check_ptr(lib.pa_segment_create(segment.num_docs), "pa_segment_create")
        self._keep = []
        if segment.num_docs == 0:
            return  # an empty segment has no column indexes (SegmentColumnarIndexCreator.java:124 writes none)
        for name in (columns if columns is not None else segment.columns):
            self._add(name)

    def _add(self, name):
        lib = L.lib()
        col = self.segment.column(name)
        cid = self.column_ids[name]
        vt = _VTYPE[col.data_type]
        if col.has_dictionary:
            hashes = None
            if col.data_type in ("INT", "LONG"):
                dv = np.ascontiguousarray(col.dictionary, dtype=np.int64)
            elif col.data_type in ("FLOAT", "DOUBLE"):
                dv = np.ascontiguousarray(col.dictionary, dtype=np.float64)
            else:
                dv = None
                hashes = np.array([hash_value(v, "STRING") for v in col.dictionary.tolist()], dtype=np.int32)
            fwd = np.ascontiguousarray(col.fwd_bytes, dtype=np.uint8)
            if col.single_value:
                L.check(lib.pa_segment_add_sv_dict_column(
                    self.handle, cid, fwd.ctypes.data, fwd.nbytes, col.num_bits, col.cardinality, vt,
                    None if dv is None else dv.ctypes.data, None if hashes is None else hashes.ctypes.data),
                    "pa_segment_add_sv_dict_column(%s)" % name)
            else:
                L.check(lib.pa_segment_add_mv_dict_column(
                    self.handle, cid, fwd.ctypes.data, fwd.nbytes, col.num_bits, col.cardinality,
                    col.total_num_values, vt, None if dv is None else dv.ctypes.data,
                    None if hashes is None else hashes.ctypes.data),
                    "pa_segment_add_mv_dict_column(%s)" % name)
        else:
            raw = np.ascontiguousarray(col.raw_values)
            L.check(lib.pa_segment_add_raw_column(self.handle, cid, vt, raw.ctypes.data),
                    "pa_segment_add_raw_column(%s)" % name)

    @property
    def device_bytes(self):
        return int(L.lib().pa_segment_device_bytes(self.handle))

    def close(self):
        if self.handle:
            L.lib().pa_segment_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class AvgPair:
    """AvgAggregationFunction intermediate result (sum, count)."""
    sum: float
    count: int


@dataclass
class MinMaxRangePair:
    """MinMaxRangeAggregationFunction intermediate result (MinMaxRangePair: min, max; empty = (+inf, -inf))."""
    min: float
    max: float


@dataclass
class IntermediateResult:
    """What the server returns for the segment set (AggregationResultsBlock / GroupByResultsBlock contents)."""
    aggregations: List[Q.Aggregation]
    group_by: List[str]
    groups: Dict[tuple, list] = field(default_factory=dict)   # group-by: key values -> intermediate values
    row: Optional[list] = None                                # aggregation-only
    num_docs_scanned: int = 0
    num_total_docs: int = 0
    num_groups_limit_reached: bool = False
    # DataTable execution statistics (fetch(execution_stats=True); filter_stats.py)
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0


class PinnedPool:
    """Page-locked host buffers (pa_host_alloc) reused across fetches: pa_query_fetch DMAs every result column straight
    into them. Arrays handed out are views, valid until the pool's next fetch from the same thread. One pool per thread
    (OUTPUT_POOL is thread-local), so concurrent fetches from different threads never share a buffer; a slot that grows
    retires its old buffer instead of freeing it (views an earlier fetch returned stay readable until close())."""

    def __init__(self):
        self.bufs = {}  # slot -> (address, bytes)
        self.retired = []

    def array(self, slot, count, dtype):
        dt = np.dtype(dtype)
        need = max(16, int(count) * dt.itemsize)
        addr, size = self.bufs.get(slot, (None, 0))
        if size < need:
            if addr:
                self.retired.append(addr)
            size = max(need, size * 2)
            addr = L.check_ptr(L.lib().pa_host_alloc(size), "pa_host_alloc")
            self.bufs[slot] = (addr, size)
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(addr))
        return raw[:int(count) * dt.itemsize].view(dt)

    def close(self):
        for addr, _ in self.bufs.values():
            L.lib().pa_host_free(addr)
        for addr in self.retired:
            L.lib().pa_host_free(addr)
        self.bufs = {}
        self.retired = []


class _ThreadPools(threading.local):
    """OUTPUT_POOL: one PinnedPool per thread (attribute access forwards to this thread's pool)."""

    def __init__(self):
        self.pool = PinnedPool()

    def array(self, slot, count, dtype):
        return self.pool.array(slot, count, dtype)

    def close(self):
        self.pool.close()


OUTPUT_POOL = _ThreadPools()


def _flatten_filter(f, leaves, ops):
    """Filter tree -> leaves + postfix program (PA_OP_*)."""
    if isinstance(f, (Q.And, Q.Or)):
        for i, c in enumerate(f.children):
            _flatten_filter(c, leaves, ops)
            if i:
                ops.append(L.PA_OP_AND if isinstance(f, Q.And) else L.PA_OP_OR)
    elif isinstance(f, Q.Not):
        _flatten_filter(f.child, leaves, ops)
        ops.append(L.PA_OP_NOT)
    else:
        ops.append(L.PA_OP_LEAF | (len(leaves) << 8))
        leaves.append(f)


class GpuQueryExecutor:
    def __init__(self, query: Q.Query, gpu_segments: List[GpuSegment], flags=0, enforce_num_groups_limit=True,
                 table_dicts=None, wide_sum_columns=(), value_dicts=None, hash_keys_bound=0, schema=None):
        """table_dicts: optional {group-by column: sorted unique values} — the table-wide dictionary every rank of a
        multi-GPU query must share so that key ids address the same accumulator rows everywhere
        (parallel.table_layout builds it); by default it is the union of these segments' dictionaries.
        wide_sum_columns: columns whose SUM keeps the 64-bit (PA_AGGF_WIDE_SUM) accumulator layout even if these
        segments' values all fit int32 — agreed across ranks by parallel.table_layout.
        value_dicts: optional {DISTINCTCOUNT column: sorted unique values} — the table-wide value dictionary whose ids
        the presence bytes index (every rank of a multi-GPU query must share it); by default the union of these
        segments' dictionaries.
        hash_keys_bound: hashed key spaces: size the slot table for at least this many keys (parallel.table_layout
        agrees on the largest rank's bound so every rank's table can take its share of the cross-GPU merge).
        schema: {column: (data type, has dictionary, single value)} agreed across ranks (parallel.table_layout): when
        every segment given here is empty, the executor plans over a one-doc placeholder segment of that schema and never
        scans it, so the rank still holds a (zero) accumulator block of the agreed layout and joins the cross-GPU merge."""
        if not gpu_segments:
            raise ValueError("no segments")
        self.table_dicts = table_dicts or {}
        self.table_value_dicts = value_dicts or {}
        self.wide_sum_columns = set(wide_sum_columns or ())
        self.hash_keys_bound = int(hash_keys_bound or 0)
        self.query = query
        # empty segments hold no indexes and contribute nothing but their (zero) doc count: only the others are bound
        self.all_segs = [g.segment for g in gpu_segments]
        self.gsegs = [g for g in gpu_segments if g.segment.num_docs > 0]
        self.segs = [g.segment for g in self.gsegs]
        self.device = next((g.device for g in gpu_segments if g.device is not None), None)
        self.flags = flags
        self.enforce_num_groups_limit = enforce_num_groups_limit
        self.handle = None
        self.placeholder = None
        self.match_none = False  # the rewritten filter is FALSE: the block stays reset, nothing is scanned
        if not self.segs and schema:
            self.placeholder = GpuSegment(self._placeholder_segment(schema), column_ids=gpu_segments[0].column_ids,
                                          device=self.device)
            self.gsegs = [self.placeholder]
            self.segs = [self.placeholder.segment]
        if self.segs:
            self._plan()
        if self.placeholder is not None:
            self.segs = []  # (nothing to scan; the plan only fixes the accumulator layout)

    def _placeholder_segment(self, schema):
        """One doc per column of the agreed schema: dictionary columns hold one value of the agreed table-wide dictionary
        (group-by and DISTINCTCOUNT columns) or a zero, raw columns a zero, multi-value columns one value."""
        from .segment import create_segment
        data, types, raw, mv = {}, {}, [], []
        for name in Q.query_columns(self.query):
            dt, has_dict, sv = schema[name]
            d = self.table_dicts.get(name)
            if d is None:
                d = self.table_value_dicts.get(name)
            v = np.asarray(d)[:1] if d is not None and len(d) else np.array(["" if dt == "STRING" else 0])
            v = v.astype({"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}.get(dt, object))
            data[name] = v if sv else [v]
            types[name] = dt
            if not has_dict:
                raw.append(name)
            if not sv:
                mv.append(name)
        return create_segment("placeholder", data, types, no_dictionary_columns=raw, multi_value_columns=mv)

    # ------------------------------------------------------------------ planning
    def _plan(self):
        lib = L.lib()
        ids = self.gsegs[0].column_ids
        seg0 = self.segs[0]
        # the reference's compile-time filter rewrites (QueryOptimizer: merged ranges / IN lists, constant predicates),
        # so the leaves below and the execution statistics follow the operator tree the reference builds
        schema = {n: (c.data_type, bool(c.single_value)) for n, c in seg0.columns.items()}
        filt = optimize_filter(self.query.filter, schema)
        if isinstance(filt, Q.BoolFilter):
            self.match_none = not filt.value  # FALSE: EmptyFilterOperator, TRUE: MatchAllFilterOperator
            filt = None
        if _has_comparison(filt):
            raise UnsupportedQuery("comparison between two different columns")
        self.query = dataclasses.replace(self.query, filter=filt)
        q = self.query
        spec = L.QuerySpec()

        # aggregations -> GPU accumulators (AVG = SUM + group count, AVGMV = SUM + COUNT_MV over the MV column; the
        # *MV forms aggregate every value of a multi-value column)
        self.pa_aggs = []
        self.agg_map = []

        def acc_index(key):
            if key not in self.pa_aggs:
                self.pa_aggs.append(key)
            return self.pa_aggs.index(key)

        for a in q.aggregations:
            fn = a.function
            if fn.endswith("MV") and seg0.column(a.column).single_value:
                raise UnsupportedQuery("%s on single-value column %s" % (fn, a.column))
            if fn == "COUNT":
                self.agg_map.append(acc_index((L.PA_AGG_COUNT, -1, 0)))
            elif fn == "AVGMV":
                self.agg_map.append((acc_index((L.PA_AGG_SUM, ids[a.column], 0)),
                                     acc_index((L.PA_AGG_COUNT_MV, ids[a.column], 0))))
            elif fn == "COUNTMV":
                self.agg_map.append(acc_index((L.PA_AGG_COUNT_MV, ids[a.column], 0)))
            elif fn in ("SUM", "AVG", "SUMMV"):
                self.agg_map.append(acc_index((L.PA_AGG_SUM, ids[a.column], 0)))
            elif fn in ("MIN", "MINMV"):
                self.agg_map.append(acc_index((L.PA_AGG_MIN, ids[a.column], 0)))
            elif fn in ("MAX", "MAXMV"):
                self.agg_map.append(acc_index((L.PA_AGG_MAX, ids[a.column], 0)))
            elif fn in Q.HLL_FUNCTIONS:
                self.agg_map.append(acc_index((L.PA_AGG_DISTINCTCOUNTHLL, ids[a.column], a.log2m)))
            elif fn in ("MINMAXRANGE", "MINMAXRANGEMV"):
                # MinMaxRangePair(min, max): the MIN and MAX accumulators of the column
                self.agg_map.append((acc_index((L.PA_AGG_MIN, ids[a.column], 0)),
                                     acc_index((L.PA_AGG_MAX, ids[a.column], 0))))
            elif fn in Q.DISTINCT_SET_FUNCTIONS:
                if not all(sg.column(a.column).has_dictionary for sg in self.segs):
                    raise UnsupportedQuery("%s on a raw (no-dictionary) column %s" % (fn, a.column))
                self.agg_map.append(acc_index((L.PA_AGG_DISTINCTCOUNT, ids[a.column], 0)))
            else:
                raise UnsupportedQuery("aggregation %s" % fn)
        if len(self.pa_aggs) > L.PA_MAX_AGGS:
            raise UnsupportedQuery("too many aggregations")
        spec.num_aggs = len(self.pa_aggs)
        names = {cid: name for name, cid in ids.items()}
        # DISTINCTCOUNT: the table-wide value dictionary of the column (presence byte j <=> value value_dicts[j])
        self.value_dicts = {}
        for i, (t, cid, log2m) in enumerate(self.pa_aggs):
            spec.aggs[i].type = t
            spec.aggs[i].column_id = max(cid, 0)
            spec.aggs[i].log2m = log2m
            if t == L.PA_AGG_SUM and names.get(cid) in self.wide_sum_columns:
                spec.aggs[i].flags = L.PA_AGGF_WIDE_SUM
            if t == L.PA_AGG_DISTINCTCOUNT:
                name = names[cid]
                if name in self.table_value_dicts:
                    vd = np.asarray(self.table_value_dicts[name])
                else:
                    ds = [sg.column(name).dictionary for sg in self.segs]
                    same = all(d is ds[0] or (len(d) == len(ds[0]) and np.array_equal(d, ds[0])) for d in ds)
                    vd = ds[0] if same else np.unique(np.concatenate(ds))
                self.value_dicts[i] = vd
                spec.aggs[i].num_values = len(vd)

        # filter
        filt = q.filter
        leaves, ops = [], []
        if filt is not None:
            _flatten_filter(filt, leaves, ops)
        if len(leaves) > L.PA_MAX_LEAVES or len(ops) > L.PA_MAX_OPS:
            raise UnsupportedQuery("filter too large")
        per_seg = []
        for seg in self.segs:
            params = []
            for pred in leaves:
                col = seg.column(pred.column)
                params.append(P.dictionary_leaf(pred, col) if col.has_dictionary else P.raw_leaf(pred, col))
            per_seg.append(params)
        self.leaf_params = per_seg  # (also the execution statistics' leaf evaluators: filter_stats)
        spec.num_leaves = len(leaves)
        for li, pred in enumerate(leaves):
            kinds = {ps[li].kind for ps in per_seg}
            kind = L.PA_LEAF_DICT_SET if L.PA_LEAF_DICT_SET in kinds else kinds.pop()
            if not seg0.column(pred.column).single_value:  # MVScanDocIdIterator: ANY value (ALL for NOT IN / !=)
                kind = {L.PA_LEAF_DICT_RANGE: L.PA_LEAF_MV_DICT_RANGE, L.PA_LEAF_DICT_SET: L.PA_LEAF_MV_DICT_SET}[kind]
            spec.leaves[li].column_id = ids[pred.column]
            spec.leaves[li].kind = kind
        spec.num_ops = len(ops)
        for i, op in enumerate(ops):
            spec.ops[i] = op

        # group-by: table-wide dictionaries (value-keyed combine)
        self.global_dicts = []
        self.remaps = []  # [seg][gb] -> np.int32 or None
        spec.num_group_by = len(q.group_by)
        if spec.num_group_by > L.PA_MAX_GROUP_BY:
            raise UnsupportedQuery("too many group-by columns")
        self.raw_group_by = []
        for j, name in enumerate(q.group_by):
            has_dict = [s.column(name).has_dictionary for s in self.segs]
            if not any(has_dict):
                # raw (no-dictionary) column: grouped by value through the hashed key space
                # (NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator)
                self.global_dicts.append(None)
                self.raw_group_by.append(seg0.column(name).data_type)
                spec.group_by_columns[j] = ids[name]
                spec.group_by_cardinality[j] = 0
                continue
            if not all(has_dict):
                raise UnsupportedQuery("group-by column %s is dictionary-encoded in some segments only" % name)
            self.raw_group_by.append(None)
            dicts = [s.column(name).dictionary for s in self.segs]
            if name in self.table_dicts:
                gd = np.asarray(self.table_dicts[name])
                if not all(np.isin(d, gd).all() for d in dicts):
                    raise ValueError("table dictionary of %s misses values of a bound segment" % name)
            else:
                first = dicts[0]
                same = all(d is first or (len(d) == len(first) and np.array_equal(d, first)) for d in dicts)
                gd = first if same else np.unique(np.concatenate(dicts))
            self.global_dicts.append(gd)
            spec.group_by_columns[j] = ids[name]
            spec.group_by_cardinality[j] = len(gd)
        for seg in self.segs:
            rm = []
            for j, name in enumerate(q.group_by):
                d = seg.column(name).dictionary
                gd = self.global_dicts[j]
                if gd is None or d is gd or (len(d) == len(gd) and np.array_equal(d, gd)):
                    rm.append(None)
                else:
                    rm.append(np.searchsorted(gd, d).astype(np.int32))
            self.remaps.append(rm)
        spec.flags = ((self.flags & 0xffffffff) ^ 0x80000000) - 0x80000000  # (int32: PA_QF_NO_JIT is bit 31)
        spec.flags2 = (self.flags >> 32) & 0x7fffffff if self.flags >= 0 else 0
        spec.hash_keys_bound = self.hash_keys_bound

        # numGroupsLimit (DictionaryBasedGroupKeyGenerator._globalGroupIdUpperBound): the per-segment first-seen group
        # cap. The library decides whether it can bind and then runs the first-seen trimming passes on the GPU;
        # enforce_num_groups_limit=False drops the cap (measurement tools only: results then differ from the
        # reference whenever the cap binds).
        spec.num_groups_limit = int(min(q.num_groups_limit, 2**31 - 1)) if (q.group_by and self.enforce_num_groups_limit) else 0

        self.spec = spec
        self.handle = L.check_ptr(lib.pa_query_create(ctypes.byref(spec), len(self.segs)), "pa_query_create")
        self._keep = []
        for si, (g, params) in enumerate(zip(self.gsegs, per_seg)):
            arr = (L.LeafParams * max(1, len(params)))()
            for li, p in enumerate(params):
                lp = arr[li]
                if isinstance(p, P.DictLeaf):
                    lp.negate = int(p.negate)
                    if spec.leaves[li].kind in (L.PA_LEAF_DICT_SET, L.PA_LEAF_MV_DICT_SET):
                        ids_ = p.ids if p.ids is not None else np.arange(p.lo, p.hi, dtype=np.int32)
                        lut = P.DictLeaf(L.PA_LEAF_DICT_SET, ids=ids_).lut_words(self.segs[si].column(leaves[li].column).cardinality)
                        self._keep.append(lut)
                        lp.lut = lut.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
                    else:
                        lp.lo, lp.hi = p.lo, p.hi
                else:
                    lp.negate = int(p.negate)
                    lp.ilo = max(min(int(p.ilo), P.LONG_MAX), P.LONG_MIN)
                    lp.ihi = max(min(int(p.ihi), P.LONG_MAX), P.LONG_MIN)
                    lp.dlo, lp.dhi = float(p.dlo), float(p.dhi)
                    if p.kind == L.PA_LEAF_RAW_SET:
                        vals = np.ascontiguousarray(p.values)
                        self._keep.append(vals)
                        lp.values = vals.ctypes.data if len(vals) else None
                        lp.num_values = len(vals)
            rms = (ctypes.c_void_p * max(1, len(q.group_by)))()
            for j, rm in enumerate(self.remaps[si]):
                if rm is not None:
                    self._keep.append(rm)
                    rms[j] = rm.ctypes.data
            L.check(lib.pa_query_bind_segment(self.handle, si, g.handle, arr, rms), "pa_query_bind_segment")
            for i, vd in self.value_dicts.items():
                d = self.segs[si].column(names[self.pa_aggs[i][1]]).dictionary
                if d is vd or (len(d) == len(vd) and np.array_equal(d, vd)):
                    continue
                if not np.isin(d, vd).all():
                    raise ValueError("DISTINCTCOUNT value dictionary misses values of a bound segment")
                rm = np.searchsorted(vd, d).astype(np.int32)
                self._keep.append(rm)
                L.check(lib.pa_query_bind_value_remap(self.handle, si, i, rm.ctypes.data), "pa_query_bind_value_remap")
        L.check(lib.pa_query_prepare(self.handle), "pa_query_prepare")
        self.num_keys = int(lib.pa_query_num_keys(self.handle))
        hashed, shifts = ctypes.c_int32(), (ctypes.c_int32 * max(1, len(q.group_by)))()
        L.check(lib.pa_query_key_layout(self.handle, ctypes.byref(hashed), shifts), "pa_query_key_layout")
        self.hashed = bool(hashed.value)
        self.key_shifts = list(shifts)[:len(q.group_by)]
        self.key_words = int(lib.pa_query_key_words(self.handle))  # 2: two int64 per hashed key
        self.strides = []
        s = 1
        for gd in self.global_dicts:
            self.strides.append(s)
            s *= len(gd) if gd is not None else 1

    # ------------------------------------------------------------------ execution
    def execute(self, stream=None):
        if not self.segs or self.match_none:  # nothing to scan (a placeholder plan, a FALSE filter): block reset only
            if self.handle is not None:
                L.check(L.lib().pa_query_reset(self.handle, stream), "pa_query_reset")
            return
        L.check(L.lib().pa_query_execute(self.handle, stream), "pa_query_execute")
        self._scanned = True
        self.merged_stats = None

    def reset(self, stream=None):
        L.check(L.lib().pa_query_reset(self.handle, stream), "pa_query_reset")
        self._scanned = False
        self.merged_stats = None

    def scan(self, stream=None):
        if not self.segs or self.match_none:
            return
        L.check(L.lib().pa_query_scan(self.handle, stream), "pa_query_scan")
        self._scanned = True
        self.merged_stats = None

    def sections(self):
        """[(kind, device_ptr, num_elements)] accumulator sections (for the cross-GPU reduce)."""
        lib = L.lib()
        out = []
        for i in range(lib.pa_query_num_sections(self.handle)):
            kind, n = ctypes.c_int32(), ctypes.c_int64()
            p = L.check_ptr(lib.pa_query_section(self.handle, i, ctypes.byref(kind), ctypes.byref(n)), "section")
            out.append((kind.value, p, n.value))
        return out

    def stats(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        L.check(L.lib().pa_query_stats(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "stats")
        out = {"staged_bytes": a.value, "num_docs": b.value, "num_wave_tiles": c.value}
        vals = [ctypes.c_int32() for _ in range(7)]
        L.check(L.lib().pa_query_plan(self.handle, *[ctypes.byref(v) for v in vals]), "plan")
        names = ("strategy", "steps", "dma_slots", "ring", "wg_per_cu", "grid", "lds_bytes")
        out["plan"] = {n: v.value for n, v in zip(names, vals)}
        code = out["plan"]["strategy"]
        out["plan"]["strategy"] = {0: "lds", 1: "global", 2: "partitioned", 4: "lane", 5: "lane", 6: "lane", 7: "lane",
                                    8: "lds_dense", 9: "lds_dense", 10: "lds_dense", 11: "lds_dense", 12: "lds_dense",
                                    14: "lds_dense", 15: "lds_dense"}[code]
        out["plan"]["variant"] = STRATEGY_VARIANTS.get(code, str(code))
        out["plan"]["eager_literals"] = int(L.lib().pa_query_num_eager_literals(self.handle))
        out["plan"]["lane_major"] = int(L.lib().pa_query_lane_major(self.handle))
        out["plan"]["dense_packed"] = int(L.lib().pa_query_dense_packed(self.handle))
        out["plan"]["count_free_emit"] = int(L.lib().pa_query_count_free_emit(self.handle))
        out["plan"]["partition_keys"] = int(L.lib().pa_query_partition_keys(self.handle))
        out["plan"]["limit_trimming"] = int(L.lib().pa_query_limit_trimming(self.handle))
        return out

    def fetch_arrays(self, stream=None, pooled=False):
        """Non-empty groups in ascending table-wide key order as arrays: (keys int64[n], counts int64[n],
        [one array per GPU accumulator: float64[n], or uint8[n << log2m] HLL registers]). Synchronises `stream`.
        pooled=True: the arrays are views of the process's page-locked output pool (OUTPUT_POOL: each column arrives by
        one DMA; valid until the next pooled fetch of any executor) instead of fresh arrays."""
        lib = L.lib()
        alloc = (lambda slot, n, dt: OUTPUT_POOL.array(slot, n, dt)) if pooled else (lambda slot, n, dt: np.empty(n, dt))
        cap = 1 if not self.query.group_by else min(self.num_keys, 1 << 16)
        if self.query.group_by and self.num_keys > 1 << 16:
            # large key space: a capacity-0 call runs only the GPU count pass and returns the number of non-empty
            # groups, so the gather + copy run once, at the exact size
            cap = max(1, L.check(lib.pa_query_fetch(self.handle, stream, 0, None, None, None), "pa_query_fetch"))
        kw = getattr(self, "key_words", 1)
        while True:
            keys = alloc("keys", cap * kw, np.int64)
            counts = alloc("counts", cap, np.int64)
            outs, ptrs = [], (ctypes.c_void_p * max(1, len(self.pa_aggs)))()
            for i, (t, _, log2m) in enumerate(self.pa_aggs):
                if t == L.PA_AGG_DISTINCTCOUNTHLL:
                    o = alloc(i, cap << log2m, np.uint8)
                elif t == L.PA_AGG_DISTINCTCOUNT:
                    o = alloc(i, cap * self._presence_stride(i), np.uint8)
                else:
                    o = alloc(i, cap, np.float64)
                outs.append(o)
                ptrs[i] = o.ctypes.data
            n = L.check(lib.pa_query_fetch(self.handle, stream, cap, keys.ctypes.data, counts.ctypes.data, ptrs),
                        "pa_query_fetch")
            if n <= cap:
                break
            cap = n
        outs = [o[: n << self.pa_aggs[i][2]] if self.pa_aggs[i][0] == L.PA_AGG_DISTINCTCOUNTHLL else
                (o[: n * self._presence_stride(i)] if self.pa_aggs[i][0] == L.PA_AGG_DISTINCTCOUNT else o[:n])
                for i, o in enumerate(outs)]
        return (keys[:n] if kw == 1 else keys[:2 * n].reshape(n, 2)), counts[:n], outs

    def _presence_stride(self, i):
        """DISTINCTCOUNT presence bytes per group: the value count rounded up to 16 (PA_ACC_PRESENCE_U8)."""
        return (len(self.value_dicts[i]) + 15) & ~15

    def key_values(self, keys):
        """Keys -> one value array per group-by column (DictionaryBasedGroupKeyGenerator.getKeys). Direct key space:
        key = sum id_j * prod_{k<j} card_k. Hashed (pa_query_key_layout): component j at bit shift_j, a table-wide key
        id for dictionary columns, the value bits for raw ones (INT/FLOAT 32 bits, LONG/DOUBLE 64); two-word keys
        (keys of shape (n, 2)): component j in word shift_j // 64 at bit shift_j % 64."""
        if not self.hashed:
            return [gd[(keys // st) % len(gd)] for gd, st in zip(self.global_dicts, self.strides)]
        kk = np.asarray(keys, dtype=np.int64)
        words = [kk.view(np.uint64)] if kk.ndim == 1 else [np.ascontiguousarray(kk[:, w]).view(np.uint64)
                                                           for w in range(kk.shape[1])]
        out = []
        for gd, raw, shw in zip(self.global_dicts, self.raw_group_by, self.key_shifts):
            k, sh = words[shw // 64], shw % 64
            if gd is not None:
                bits = max(1, int(len(gd) - 1).bit_length())
            else:
                bits = 32 if raw in ("INT", "FLOAT") else 64
            comp = (k >> np.uint64(sh)) & np.uint64((1 << bits) - 1) if bits < 64 else (k >> np.uint64(sh))
            if gd is not None:
                out.append(gd[comp.astype(np.int64)])
            elif raw == "INT":
                out.append(comp.astype(np.uint32).view(np.int32))
            elif raw == "FLOAT":
                out.append(comp.astype(np.uint32).view(np.float32))
            elif raw == "LONG":
                out.append(comp.view(np.int64))
            else:
                out.append(comp.view(np.float64))
        return out

    def torch_device(self):
        """The GPU holding this executor's segments (GpuSegment(device=...)), else the current device."""
        import torch
        return torch.device("cuda", self.device if self.device is not None else torch.cuda.current_device())

    def leaf_bitmaps(self, segment_index, stream=None):
        """bool[leaves, num_docs]: every filter leaf (the engine's flattened leaf order) on every doc of one bound
        segment, computed on the GPU (pa_query_leaf_bitmaps). Synchronises `stream`."""
        import torch
        lib = L.lib()
        nl = int(self.spec.num_leaves)
        n = self.segs[segment_index].num_docs
        if nl == 0:
            return np.zeros((0, n), dtype=bool)
        words = L.check(lib.pa_query_leaf_bitmap_words(self.handle, segment_index), "pa_query_leaf_bitmap_words")
        dev = self.torch_device()
        buf = torch.zeros(nl * words, dtype=torch.int32, device=dev)
        L.check(lib.pa_query_leaf_bitmaps(self.handle, segment_index, buf.data_ptr(), stream), "pa_query_leaf_bitmaps")
        torch.cuda.synchronize(dev)  # (device-wide: covers `stream`)
        w = buf.cpu().numpy().view(np.uint8).reshape(nl, words * 4)
        return np.unpackbits(w, axis=1, bitorder="little")[:, :n].astype(bool)

    def fused_leap_counts(self, stream=None):
        """(E leaf, Z leaf, int64[segments, 3]) when the last scan counted the execution statistics of its two-leaf AND
        itself (the default where it applies; PA_QF_NO_FILTER_STATS turns it off. pa_query_leap_counts: per segment
        matched docs, leaps of AndDocIdIterator(A = Z, B = E), gave-up flag), else None. Synchronises `stream`."""
        lib = L.lib()
        if self.handle is None or not self.segs or not getattr(self, "_scanned", False):
            return None
        e = int(lib.pa_query_leap_leaf(self.handle))
        if e < 0:
            return None
        out = np.zeros((len(self.segs), 3), dtype=np.int64)
        L.check(lib.pa_query_leap_counts(self.handle, out.ctypes.data, stream), "pa_query_leap_counts")
        return e, 1 - e, out

    def execution_stats(self, stream=None, docs_total=None):
        """(numEntriesScannedInFilter, numEntriesScannedPostFilter) of this server's segments after the last scan: the
        reference's operator accounting counted by the library (pa_query_execution_stats) over the operator trees this
        host builds per segment (filter_stats.operator_trees = FilterOperatorUtils). Segments whose tree the engine
        does not express (filter_stats "device path") replay the iterators on the host over GPU leaf bitmaps;
        self.stats_replayed_segments counts them. docs_total: numDocsScanned of the scan (default: the last scan's own
        counter, so a call after execute() without a fetch is not stale)."""
        from . import filter_stats as FS
        self.stats_replayed_segments = self.stats_gpu_segments = 0
        if self.match_none or self.handle is None or not self.segs:
            return 0, 0  # EmptyFilterOperator: no entry read, no doc projected
        if getattr(self, "_stats_trees", None) is None:  # the operator trees of this prepared query, built once
            self._stats_trees = FS.operator_trees(self.query, self.segs, getattr(self, "leaf_params", None),
                                                  self.gsegs[0].column_ids)
        ops, roots, seg_tree = self._stats_trees
        out = np.zeros(3, dtype=np.int64)
        per = np.zeros(len(self.segs), dtype=np.int64)
        L.check(L.lib().pa_query_execution_stats(
            self.handle, len(ops), ops.ctypes.data, len(roots), roots.ctypes.data, seg_tree.ctypes.data,
            FS.projected_columns(self.query), -1 if docs_total is None else int(docs_total), out.ctypes.data,
            per.ctypes.data, stream), "pa_query_execution_stats")
        in_filter, post = int(out[0]), int(out[1])
        self.stats_gpu_segments = int(out[2])  # segments whose statistics took a GPU pass (not the scan's own counts)
        host = np.flatnonzero(per < 0).tolist()
        if host:
            self.stats_replayed_segments = len(host)
            hi, _ = FS.server_stats(self.query, [self.segs[i] for i in host],
                                    lambda i: self.leaf_bitmaps(host[i], stream))
            in_filter += hi
        return in_filter, post

    def fetch(self, stream=None, execution_stats=True) -> IntermediateResult:
        """The results block of the last scan. Like the reference's results blocks (BaseResultsBlock.java:194) it carries
        the execution statistics — numEntriesScannedInFilter / PostFilter from pa_query_execution_stats, after the groups
        (execution_stats): execution_stats=False leaves them 0."""
        lib = L.lib()
        q = self.query
        if self.handle is None:
            return self._empty_result()
        keys, counts, outs = self.fetch_arrays(stream, pooled=True)  # (converted to Python objects below)
        n = len(keys)
        res = IntermediateResult(list(q.aggregations), list(q.group_by))
        res.num_total_docs = sum(s.num_docs for s in self.all_segs)
        res.num_docs_scanned = int(lib.pa_query_matched_docs(self.handle))
        merged = getattr(self, "merged_stats", None)
        if merged is not None:
            # numDocsScanned was summed across GPUs (parallel.DistributedAccumulators.reduce): this rank's segments
            # cannot recount the statistics against it; the reduce summed every rank's own pair before its collective
            # (reduce(execution_stats=True), the default), or gathered none (NO_MERGED_STATS)
            if execution_stats:
                if isinstance(merged, str):  # (parallel.NO_MERGED_STATS)
                    raise L.PinotAmdError("the merged block has no execution statistics: reduce(execution_stats=True), "
                                          "or fetch(execution_stats=False)")
                res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter = merged
        elif execution_stats:
            res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter = self.execution_stats(
                stream, res.num_docs_scanned)
        key_cols = [kc.tolist() for kc in self.key_values(keys)]
        cols = []  # one python list per query aggregation
        for a, pi in zip(q.aggregations, self.agg_map):
            if a.function == "COUNT":
                cols.append(counts.tolist())
            elif a.function == "AVG":
                cols.append([AvgPair(s_, c_) for s_, c_ in zip(outs[pi].tolist(), counts.tolist())])
            elif a.function == "AVGMV":
                cols.append([AvgPair(s_, int(c_)) for s_, c_ in zip(outs[pi[0]].tolist(), outs[pi[1]].tolist())])
            elif a.function == "COUNTMV":
                cols.append([int(v) for v in outs[pi].tolist()])
            elif a.function in Q.HLL_FUNCTIONS:
                log2m = self.pa_aggs[pi][2]
                regs = outs[pi].reshape(n, 1 << log2m)
                cols.append([HyperLogLog(log2m, regs[r]) for r in range(n)])
            elif a.function in ("MINMAXRANGE", "MINMAXRANGEMV"):
                cols.append([MinMaxRangePair(lo, hi) for lo, hi in zip(outs[pi[0]].tolist(), outs[pi[1]].tolist())])
            elif a.function in Q.DISTINCT_SET_FUNCTIONS:
                # the value set of BaseDistinctAggregateAggregationFunction (DISTINCTCOUNT / DISTINCTSUM / DISTINCTAVG)
                vd = self.value_dicts[pi]
                pres = outs[pi].reshape(n, self._presence_stride(pi))[:, :len(vd)]
                if a.function in Q.BITMAP_FUNCTIONS:  # (DISTINCTCOUNTBITMAP: the values' Java hash codes)
                    dt = self.segs[0].column(a.column).data_type
                    hc = np.array([java_hash_code(v, dt) for v in vd.tolist()], dtype=np.int64)
                    cols.append([set(hc[np.flatnonzero(pres[r])].tolist()) for r in range(n)])
                else:
                    cols.append([set(vd[np.flatnonzero(pres[r])].tolist()) for r in range(n)])
            else:
                cols.append(outs[pi].tolist())
        rows = list(zip(*cols)) if cols else [()] * n
        if q.group_by:
            res.groups = {tuple(kc[r] for kc in key_cols): list(rows[r]) for r in range(n)}
            # GroupByOperator.java:112 per segment, OR-ed by GroupByCombineOperator.java:154
            res.num_groups_limit_reached = int(L.lib().pa_query_num_groups_limit_reached(self.handle)) > 0
        else:
            res.row = list(rows[0])
        return res

    def _empty_result(self):
        """The results block of a segment set without docs: no groups, or the aggregation functions' empty
        intermediate results (COUNT 0, SUM 0.0, MIN +inf, MAX -inf, AVG (0.0, 0), empty HLL / value set)."""
        q = self.query
        res = IntermediateResult(list(q.aggregations), list(q.group_by))
        if not q.group_by:
            row = []
            for a in q.aggregations:
                fn = Q.base_function(a.function)
                row.append({"COUNT": 0, "SUM": 0.0, "MIN": float("inf"), "MAX": float("-inf")}.get(fn) if fn in
                           ("COUNT", "SUM", "MIN", "MAX") else
                           AvgPair(0.0, 0) if fn == "AVG" else
                           HyperLogLog(a.log2m) if fn in ("DISTINCTCOUNTHLL", "DISTINCTCOUNTRAWHLL") else
                           MinMaxRangePair(float("inf"), float("-inf")) if fn == "MINMAXRANGE" else set())
            res.row = row
        return res

    def run(self, stream=None) -> IntermediateResult:
        self.execute(stream)
        return self.fetch(stream)

    def close(self):
        if self.handle:
            L.lib().pa_query_destroy(self.handle)
            self.handle = None
        if self.placeholder is not None:
            self.placeholder.close()
            self.placeholder = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# the kernel variant behind each pa_query_plan strategy code (pa_device.h Strategy)
STRATEGY_VARIANTS = {0: "lds", 1: "global", 2: "partitioned", 4: "lane", 5: "lane_cnt", 6: "lane_raw", 7: "lane_dict",
                     8: "gdense4", 9: "gdense8", 10: "gdense12", 11: "gdense_rs12", 12: "gdense_rs8", 14: "gdense_lm8",
                     15: "gdense_lm16"}


def _has_comparison(f):
    if isinstance(f, (Q.And, Q.Or)):
        return any(_has_comparison(c) for c in f.children)
    if isinstance(f, Q.Not):
        return _has_comparison(f.child)
    return isinstance(f, Q.Comparison)


def _py(v):
    if isinstance(v, np.generic):
        return v.item()
    return v
