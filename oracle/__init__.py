"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

Imported solely by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker; the product
path (pinot_amd) never imports it. Parity is pinned against the reference's own golden results
(tests/golden/sv_queries.json, transcribed with file:line from pinot-core/src/test/java/org/apache/pinot/queries)
on the reference's own test input (tests/golden/test_data_sv.npz, converted from
pinot-core/src/test/resources/data/test_data-sv.avro by tests/golden/make_golden.py).

The per-doc scan lives in pinot_oracle.c (scalar C restatement, see its header for the reference file:line map);
this module restates the dictionary-based predicate evaluators (value -> set of matching dictIds), drives the
per-segment scan, and merges segment results by group-key VALUE in segment order
(GroupByCombineOperator / IndexedTable.upsert semantics: SUM +, MIN min, MAX max, COUNT +, HLL register max).
"""
import ctypes
import os
import subprocess
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(BUILD, "liboracle.so")
SRC = os.path.join(HERE, "pinot_oracle.c")

_lock = threading.Lock()
_lib = None


def build(force=False):
    os.makedirs(BUILD, exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(SRC) > os.path.getmtime(LIB):
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-o", LIB + ".tmp", SRC, "-lm"], check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


class OCol(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("num_bits", ctypes.c_int32), ("cardinality", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("fwd", ctypes.c_void_p), ("raw", ctypes.c_void_p),
                ("dict_f64", ctypes.c_void_p), ("dict_hash", ctypes.c_void_p),
                ("mv_bitmap", ctypes.c_void_p), ("mv_num_values", ctypes.c_int64)]


class OLeaf(ctypes.Structure):
    _fields_ = [("col", ctypes.c_int32), ("kind", ctypes.c_int32), ("match", ctypes.c_void_p),
                ("dlo", ctypes.c_double), ("dhi", ctypes.c_double), ("ilo", ctypes.c_int64), ("ihi", ctypes.c_int64),
                ("lo_unbounded", ctypes.c_int32), ("hi_unbounded", ctypes.c_int32),
                ("lo_incl", ctypes.c_int32), ("hi_incl", ctypes.c_int32),
                ("exclusive", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class OQuery(ctypes.Structure):
    _fields_ = [("num_ops", ctypes.c_int32), ("ops", ctypes.c_void_p), ("num_leaves", ctypes.c_int32),
                ("leaves", ctypes.c_void_p), ("num_gb", ctypes.c_int32), ("gb_col", ctypes.c_void_p),
                ("num_groups_limit", ctypes.c_int64), ("num_aggs", ctypes.c_int32), ("agg_type", ctypes.c_void_p),
                ("agg_col", ctypes.c_void_p), ("agg_log2m", ctypes.c_void_p)]


def lib():
    global _lib
    with _lock:
        if _lib is None:
            _lib = ctypes.CDLL(build())
            _lib.oracle_read_int.restype = ctypes.c_int32
            _lib.oracle_read_int.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
            _lib.oracle_read_ints.restype = None
            _lib.oracle_read_ints.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                              ctypes.c_void_p]
            _lib.oracle_write_int.restype = None
            _lib.oracle_write_int.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
            _lib.oracle_hash_long.restype = ctypes.c_int32
            _lib.oracle_hash_long.argtypes = [ctypes.c_int64]
            _lib.oracle_hash_bytes.restype = ctypes.c_int32
            _lib.oracle_hash_bytes.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32]
            _lib.oracle_run_segment.restype = ctypes.c_int64
            _lib.oracle_run_segment.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(OQuery),
                                                ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
    return _lib


# ------------------------------------------------------------------ small helpers used by tests
def read_ints(buf, n, nb, start=0):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = np.zeros(n, dtype=np.int32)
    lib().oracle_read_ints(buf.ctypes.data, start, n, nb, out.ctypes.data)
    return out


def write_ints(values, nb):
    values = np.asarray(values, dtype=np.int32)
    buf = np.zeros((len(values) * nb + 7) // 8 + 1, dtype=np.uint8)
    for i, v in enumerate(values.tolist()):
        lib().oracle_write_int(buf.ctypes.data, i, nb, v)
    return buf[: (len(values) * nb + 7) // 8]


def murmur_hash(value, data_type):
    """MurmurHash.hash(Object) for the boxed dictionary value of a column of `data_type`."""
    L = lib()
    if data_type in ("INT", "LONG"):
        return L.oracle_hash_long(int(value))
    if data_type == "FLOAT":
        return L.oracle_hash_long(int(np.array([value], dtype=np.float32).view(np.int32)[0]))
    if data_type == "DOUBLE":
        return L.oracle_hash_long(int(np.array([value], dtype=np.float64).view(np.int64)[0]))
    b = str(value).encode("utf-8")  # String.getBytes() with the UTF-8 platform charset
    return L.oracle_hash_bytes(b, len(b), -1)


# ------------------------------------------------------------------ predicate evaluators (restated)
def _parse(raw, data_type):
    if data_type in ("INT", "LONG"):
        # Integer.parseInt / Long.parseLong: sign + decimal digits within range, else NumberFormatException
        s = str(raw)
        bits = 32 if data_type == "INT" else 64
        body = s[1:] if s[:1] in ("+", "-") else s
        if not body or not all("0" <= ch <= "9" for ch in body) or not -(1 << (bits - 1)) <= int(s) < (1 << (bits - 1)):
            raise ValueError("NumberFormatException: %r" % s)
        return int(s)
    if data_type == "FLOAT":
        return float(np.float32(float(raw)))
    if data_type == "DOUBLE":
        return float(raw)
    return str(raw)


def _dict_match(pred, col):
    """applySV(dictId) for every dictId of the (sorted) dictionary, as uint8[cardinality]."""
    from pinot_amd import query as Q  # query model only (data classes)
    d = col.dictionary
    card = len(d)
    m = np.zeros(card, dtype=np.uint8)
    values = d.tolist()
    dt = col.data_type

    def index_of(v):
        lo, hi = 0, card
        while lo < hi:  # Dictionary.indexOf on a sorted dictionary (binary search)
            mid = (lo + hi) // 2
            if values[mid] < v:
                lo = mid + 1
            else:
                hi = mid
        return lo if lo < card and values[lo] == v else -1

    def insertion_point(v):
        lo, hi = 0, card
        while lo < hi:
            mid = (lo + hi) // 2
            if values[mid] < v:
                lo = mid + 1
            else:
                hi = mid
        return lo

    if isinstance(pred, Q.EqPredicate):
        i = index_of(_parse(pred.value, dt))
        if i >= 0:
            m[i] = 1
    elif isinstance(pred, Q.NotEqPredicate):
        m[:] = 1
        i = index_of(_parse(pred.value, dt))
        if i >= 0:
            m[i] = 0
    elif isinstance(pred, Q.RegexpLikePredicate):
        # DictionaryBasedRegexpLikePredicateEvaluator.applySV: Matcher.find() on the dictionary value
        # (RegexpLikePredicateEvaluatorFactory.java), restated with re.search
        import re
        rx = re.compile(pred.pattern)
        for i, v in enumerate(values):
            m[i] = 1 if rx.search(str(v)) else 0
    elif isinstance(pred, Q.InPredicate):
        for v in pred.values:
            i = index_of(_parse(v, dt))
            if i >= 0:
                m[i] = 1
    elif isinstance(pred, Q.NotInPredicate):
        m[:] = 1
        for v in pred.values:
            i = index_of(_parse(v, dt))
            if i >= 0:
                m[i] = 0
    elif isinstance(pred, Q.RangePredicate):
        # SortedDictionaryBasedRangePredicateEvaluator: [startDictId, endDictId)
        if pred.lower == Q.UNBOUNDED:
            start = 0
        else:
            v = _parse(pred.lower, dt)
            p = insertion_point(v)
            start = p + 1 if (p < card and values[p] == v and not pred.lower_inclusive) else p
        if pred.upper == Q.UNBOUNDED:
            end = card
        else:
            v = _parse(pred.upper, dt)
            p = insertion_point(v)
            end = p + 1 if (p < card and values[p] == v and pred.upper_inclusive) else p
        if end > start:
            m[start:end] = 1
    else:
        raise TypeError(pred)
    return m


def _raw_leaf(pred, col, leaf):
    from pinot_amd import query as Q
    dt = col.data_type
    integral = dt in ("INT", "LONG")
    leaf.kind = 1
    leaf.lo_unbounded = leaf.hi_unbounded = 1
    leaf.lo_incl = leaf.hi_incl = 1

    def setb(which, raw, incl):
        v = _parse(raw, dt)
        if which == "lo":
            leaf.lo_unbounded, leaf.lo_incl = 0, int(incl)
            if integral:
                leaf.ilo = v
            else:
                leaf.dlo = v
        else:
            leaf.hi_unbounded, leaf.hi_incl = 0, int(incl)
            if integral:
                leaf.ihi = v
            else:
                leaf.dhi = v

    if isinstance(pred, Q.EqPredicate):
        setb("lo", pred.value, True)
        setb("hi", pred.value, True)
    elif isinstance(pred, Q.RangePredicate):
        if pred.lower != Q.UNBOUNDED:
            setb("lo", pred.lower, pred.lower_inclusive)
        if pred.upper != Q.UNBOUNDED:
            setb("hi", pred.upper, pred.upper_inclusive)
    else:
        raise TypeError("raw leaf %r" % (pred,))


def _flatten(f, leaves, ops, segment):
    from pinot_amd import query as Q
    if isinstance(f, (Q.And, Q.Or)):
        for i, c in enumerate(f.children):
            _flatten(c, leaves, ops, segment)
            if i:
                ops.append(1 if isinstance(f, Q.And) else 2)
    elif isinstance(f, Q.Not):
        _flatten(f.child, leaves, ops, segment)
        ops.append(3)
    elif isinstance(f, (Q.NotEqPredicate, Q.InPredicate, Q.NotInPredicate)) and not segment.column(f.column).has_dictionary:
        # raw: != -> NOT(=); IN -> OR(=...); NOT IN -> NOT(OR(=...))
        if isinstance(f, Q.NotEqPredicate):
            _flatten(Q.Not(Q.EqPredicate(f.column, f.value)), leaves, ops, segment)
        else:
            ors = Q.Or(tuple(Q.EqPredicate(f.column, v) for v in f.values))
            _flatten(Q.Not(ors) if isinstance(f, Q.NotInPredicate) else ors, leaves, ops, segment)
    else:
        ops.append(0 | (len(leaves) << 8))
        leaves.append(f)


_AGG = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "DISTINCTCOUNTHLL": 4, "COUNTMV": 5, "DISTINCTCOUNT": 6}
# query function -> oracle accumulators (the *MV forms read every value of the MV column; AVG = SUM + group count,
# AVGMV = SUM + COUNTMV over the column)
_ORACLE_FNS = {"SUM": ("SUM",), "AVG": ("SUM",), "MIN": ("MIN",), "MAX": ("MAX",),
               "DISTINCTCOUNTHLL": ("DISTINCTCOUNTHLL",), "SUMMV": ("SUM",), "MINMV": ("MIN",), "MAXMV": ("MAX",),
               "DISTINCTCOUNTHLLMV": ("DISTINCTCOUNTHLL",), "COUNTMV": ("COUNTMV",), "AVGMV": ("SUM", "COUNTMV"),
               "DISTINCTCOUNTRAWHLL": ("DISTINCTCOUNTHLL",), "DISTINCTCOUNTRAWHLLMV": ("DISTINCTCOUNTHLL",),
               "COUNT": ("COUNT",), "MINMAXRANGE": ("MIN", "MAX"), "MINMAXRANGEMV": ("MIN", "MAX"),
               "DISTINCTCOUNT": ("DISTINCTCOUNT",), "DISTINCTCOUNTMV": ("DISTINCTCOUNT",),
               "DISTINCTSUM": ("DISTINCTCOUNT",), "DISTINCTSUMMV": ("DISTINCTCOUNT",),
               "DISTINCTAVG": ("DISTINCTCOUNT",), "DISTINCTAVGMV": ("DISTINCTCOUNT",),
               "DISTINCTCOUNTBITMAP": ("DISTINCTCOUNT",), "DISTINCTCOUNTBITMAPMV": ("DISTINCTCOUNT",)}


def _java_hash(v, dt):
    """Object.hashCode of a stored value as DistinctCountBitmapAggregationFunction.convertToValueBitmap
    (DistinctCountBitmapAggregationFunction.java:410-446) adds it: Integer (the value), Long ((int)(v ^ v >>> 32)),
    Float (floatToIntBits), Double (doubleToLongBits folded like Long), String (s[0]*31^(n-1) + ... over UTF-16 units)."""
    import struct
    if dt == "INT":
        h = int(v)
    elif dt == "LONG":
        x = int(v) % (1 << 64)
        h = x ^ (x >> 32)
    elif dt == "FLOAT":
        h = 0x7FC00000 if v != v else struct.unpack("<I", struct.pack("<f", float(v)))[0]
    elif dt == "DOUBLE":
        x = 0x7FF8000000000000 if v != v else struct.unpack("<Q", struct.pack("<d", float(v)))[0]
        h = x ^ (x >> 32)
    else:
        h = 0
        u = str(v).encode("utf-16-le")
        for i in range(0, len(u), 2):
            h = (h * 31 + (u[i] | (u[i + 1] << 8))) % (1 << 32)
    h %= 1 << 32
    return h - (1 << 32) if h >= 1 << 31 else h


def _pack_msb(ids, nb):
    """PinotDataBitSet.writeInt layout (MSB-first), vectorised; for the oracle's virtual group-by dictionaries."""
    ids = np.asarray(ids, dtype=np.uint64)
    bits = ((ids[:, None] >> np.arange(nb - 1, -1, -1, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8).reshape(-1)
    return np.packbits(bits)


def _run_segment_raw(query, segment):
    """The C scan of one segment; results as arrays (_SegRaw)."""
    from pinot_amd import query as Q  # noqa: F401
    cols_order = sorted(query.columns())
    cidx = {c: i for i, c in enumerate(cols_order)}
    raw_gb = [c for c in query.group_by if not segment.column(c).has_dictionary]
    gbidx = {c: cidx[c] for c in query.group_by}
    virt = {}
    for c in raw_gb:
        gbidx[c] = len(cols_order) + len(virt)
        virt[c] = np.unique(segment.column(c).raw_values, return_inverse=True)
    ocols = (OCol * max(1, len(cols_order) + len(virt)))()
    keep = []
    hll_cols = {a.column for a in query.aggregations if a.function in Q.HLL_FUNCTIONS}
    for name, i in cidx.items():
        col = segment.column(name)
        oc = ocols[i]
        if col.has_dictionary:
            oc.kind = 0
            oc.num_bits = col.num_bits
            oc.cardinality = col.cardinality
            fwd = np.ascontiguousarray(col.fwd_bytes, dtype=np.uint8)
            keep.append(fwd)
            oc.fwd = fwd.ctypes.data
            if not col.single_value:  # FixedBitMVForwardIndexReader sections (chunk offsets | bitmap | values)
                _, _, boff, roff = col.mv_layout(segment.num_docs)
                oc.kind = 5
                oc.fwd = fwd.ctypes.data + roff
                oc.mv_bitmap = fwd.ctypes.data + boff
                oc.mv_num_values = col.total_num_values
            if col.data_type != "STRING":
                df = np.ascontiguousarray(col.dictionary, dtype=np.float64)
                keep.append(df)
                oc.dict_f64 = df.ctypes.data
            if name in hll_cols:
                hh = np.array([murmur_hash(v, col.data_type) for v in col.dictionary.tolist()], dtype=np.int32)
                keep.append(hh)
                oc.dict_hash = hh.ctypes.data
        else:
            oc.kind = {"INT": 1, "LONG": 2, "FLOAT": 3, "DOUBLE": 4}[col.data_type]
            raw = np.ascontiguousarray(col.raw_values)
            keep.append(raw)
            oc.raw = raw.ctypes.data

    for c, (uniq, inv) in virt.items():
        oc = ocols[gbidx[c]]
        nb = max(1, int(len(uniq) - 1).bit_length())
        packed = _pack_msb(inv, nb)
        keep.append(packed)
        oc.kind = 0
        oc.num_bits = nb
        oc.cardinality = len(uniq)
        oc.fwd = packed.ctypes.data

    # filter
    leaves, ops = [], []
    if query.filter is not None:
        _flatten(query.filter, leaves, ops, segment)
    oleaves = (OLeaf * max(1, len(leaves)))()
    for i, pred in enumerate(leaves):
        col = segment.column(pred.column)
        oleaves[i].col = cidx[pred.column]
        if col.has_dictionary:
            m = _dict_match(pred, col)
            keep.append(m)
            oleaves[i].kind = 0
            oleaves[i].match = m.ctypes.data
            # PredicateEvaluator.isExclusive (NOT_EQ, NOT_IN): applyMV requires every value to pass
            oleaves[i].exclusive = int(isinstance(pred, (Q.NotEqPredicate, Q.NotInPredicate)))
        else:
            _raw_leaf(pred, col, oleaves[i])
    ops_a = np.array(ops or [0], dtype=np.int32)

    # aggregations: one oracle accumulator per distinct (function, column)
    oaggs = []
    amap = []
    for a in query.aggregations:
        idx = []
        for fn in _ORACLE_FNS[a.function]:
            key = (fn, a.column if fn != "COUNT" else None, a.log2m if fn == "DISTINCTCOUNTHLL" else 0)
            if key not in oaggs:
                oaggs.append(key)
            idx.append(oaggs.index(key))
        amap.append(idx[0] if len(idx) == 1 else tuple(idx))
    at = np.array([_AGG[k[0]] for k in oaggs] or [0], dtype=np.int32)
    ac = np.array([cidx[k[1]] if k[1] else 0 for k in oaggs] or [0], dtype=np.int32)
    al = np.array([k[2] for k in oaggs] or [0], dtype=np.int32)
    gb = np.array([gbidx[c] for c in query.group_by] or [0], dtype=np.int32)

    oq = OQuery()
    oq.num_ops = len(ops)
    oq.ops = ops_a.ctypes.data
    oq.num_leaves = len(leaves)
    oq.leaves = ctypes.cast(oleaves, ctypes.c_void_p)
    oq.num_gb = len(query.group_by)
    oq.gb_col = gb.ctypes.data
    oq.num_groups_limit = query.num_groups_limit
    oq.num_aggs = len(oaggs)
    oq.agg_type = at.ctypes.data
    oq.agg_col = ac.ctypes.data
    oq.agg_log2m = al.ctypes.data

    if query.group_by:
        prod = 1
        for c in query.group_by:
            prod *= len(virt[c][0]) if c in virt else segment.column(c).cardinality
        mv = any(not segment.column(c).single_value for c in query.group_by)
        cap = max(1, min(prod, query.num_groups_limit) if mv else min(prod, segment.num_docs, query.num_groups_limit))
    else:
        cap = 1
    keys = np.zeros(cap, dtype=np.int64)
    counts = np.zeros(cap, dtype=np.int64)
    vals = np.zeros(max(1, len(oaggs)) * cap, dtype=np.float64)
    def _buf(k):
        if k[0] == "DISTINCTCOUNTHLL":
            return np.zeros(cap << k[2], dtype=np.uint8)
        if k[0] == "DISTINCTCOUNT":
            return np.zeros(cap * segment.column(k[1]).cardinality, dtype=np.uint8)
        return np.zeros(1, np.uint8)
    hll_bufs = [_buf(k) for k in oaggs] or [np.zeros(1, np.uint8)]
    hll_ptrs = (ctypes.c_void_p * len(hll_bufs))(*[b.ctypes.data for b in hll_bufs])
    matched = ctypes.c_int64()
    n = lib().oracle_run_segment(ctypes.cast(ocols, ctypes.c_void_p), segment.num_docs, ctypes.byref(oq), cap,
                                 keys.ctypes.data, counts.ctypes.data, vals.ctypes.data,
                                 ctypes.cast(hll_ptrs, ctypes.c_void_p), ctypes.byref(matched))
    if n < 0:
        raise MemoryError("oracle allocation failed")
    n = min(n, cap)
    return _SegRaw(n, keys, counts, vals, hll_bufs, oaggs, amap, int(matched.value), cap, virt)


class _SegRaw:
    """Array form of one segment's oracle result: raw keys (DictionaryBasedGroupKeyGenerator raw key over the segment's
    own dictionaries, column 0 least significant) in first-seen order, counts, per-accumulator values."""

    def __init__(self, n, keys, counts, vals, hll_bufs, oaggs, amap, matched, cap, virt):
        self.n, self.keys, self.counts, self.vals, self.hll_bufs = n, keys, counts, vals, hll_bufs
        self.oaggs, self.amap, self.matched, self.cap, self.virt = oaggs, amap, matched, cap, virt


def run_segment(query, segment):
    """Per-segment intermediate result: {key tuple (values): [count, per-oracle-agg values]}; () for agg-only.

    Raw (no-dictionary) group-by columns are grouped by value, as the reference's NoDictionarySingleColumn /
    NoDictionaryMultiColumnGroupKeyGenerator do (value -> group id map): the oracle gives each one a virtual sorted
    dictionary of its distinct values (its own column slot, so the same column can still be filtered or aggregated raw)."""
    r = _run_segment_raw(query, segment)
    n, keys, counts, vals, hll_bufs, oaggs, amap, cap, virt = (r.n, r.keys, r.counts, r.vals, r.hll_bufs, r.oaggs,
                                                               r.amap, r.cap, r.virt)
    out = {}
    for g in range(n):
        if query.group_by:
            rk = int(keys[g])
            kv = []
            for c in query.group_by:
                d = virt[c][0] if c in virt else segment.column(c).dictionary
                kv.append(d[rk % len(d)].item())
                rk //= len(d)
            key = tuple(kv)
        else:
            key = ()
        row = []
        for ai, k in enumerate(oaggs):
            if k[0] == "DISTINCTCOUNTHLL":
                mm = 1 << k[2]
                row.append(hll_bufs[ai][g * mm:(g + 1) * mm].copy())
            elif k[0] == "DISTINCTCOUNT":
                col = segment.column(k[1])
                card = col.cardinality
                row.append(set(col.dictionary[np.flatnonzero(hll_bufs[ai][g * card:(g + 1) * card])].tolist()))
            else:
                row.append(float(vals[ai * cap + g]))
        out[key] = (int(counts[g]), row)
    return out, oaggs, amap, r.matched


def _constant_filters(query, segments):
    """A filter with constant parts (TRUE / FALSE literals, literal = literal, column = same column) is folded first, as
    the reference's IdenticalPredicateFilterOptimizer does; a FALSE filter becomes `x = v AND NOT x = v` (no doc)."""
    import dataclasses
    from pinot_amd import query as Q
    from pinot_amd.optimizer import optimize_filter

    def has_const(f):
        if isinstance(f, (Q.And, Q.Or)):
            return any(has_const(c) for c in f.children)
        if isinstance(f, Q.Not):
            return has_const(f.child)
        return isinstance(f, (Q.BoolFilter, Q.Comparison))
    if query.filter is None or not has_const(query.filter):
        return query
    seg = next((s for s in segments if s.num_docs > 0), None)
    schema = {n: (c.data_type, bool(c.single_value)) for n, c in seg.columns.items()} if seg is not None else {}
    f = optimize_filter(query.filter, schema)
    if isinstance(f, Q.BoolFilter):
        if f.value or seg is None:
            f = None
        else:
            name = sorted(seg.columns)[0]
            leaf = Q.EqPredicate(name, str(seg.column(name).dictionary[0]) if seg.column(name).has_dictionary else "0")
            f = Q.And((leaf, Q.Not(leaf)))
    return dataclasses.replace(query, filter=f)


def run_query(query, segments):
    """Server-level intermediate result for a segment set, merged by key value in segment order."""
    query = _constant_filters(query, segments)
    from pinot_amd import query as Q  # query model only (data classes)
    from pinot_amd.engine import AvgPair, IntermediateResult, MinMaxRangePair
    from pinot_amd.hll import HyperLogLog
    merged = {}
    oaggs, amap = None, None
    scanned = 0
    limit_reached = False
    for seg in segments:
        res, oaggs, amap, matched = run_segment(query, seg)
        scanned += matched
        # GroupByOperator.java:112: a segment whose group table holds numGroupsLimit groups; OR over segments
        limit_reached |= bool(query.group_by) and len(res) >= query.num_groups_limit
        for key, (cnt, row) in res.items():
            if key not in merged:
                merged[key] = [cnt, [r.copy() if isinstance(r, np.ndarray) else r for r in row]]
                continue
            acc = merged[key]
            acc[0] += cnt
            for ai, k in enumerate(oaggs):
                if k[0] in ("SUM", "COUNTMV"):
                    acc[1][ai] = acc[1][ai] + row[ai]
                elif k[0] == "MIN":
                    acc[1][ai] = min(acc[1][ai], row[ai])
                elif k[0] == "MAX":
                    acc[1][ai] = max(acc[1][ai], row[ai])
                elif k[0] == "DISTINCTCOUNTHLL":
                    acc[1][ai] = np.maximum(acc[1][ai], row[ai])
                elif k[0] == "DISTINCTCOUNT":
                    acc[1][ai] = acc[1][ai] | row[ai]
    out = IntermediateResult(list(query.aggregations), list(query.group_by))
    out.num_total_docs = sum(s.num_docs for s in segments)
    out.num_docs_scanned = scanned
    out.num_groups_limit_reached = limit_reached
    if not query.group_by and () not in merged:
        merged[()] = [0, [np.zeros(1 << k[2], np.uint8) if k[0] == "DISTINCTCOUNTHLL" else
                          (set() if k[0] == "DISTINCTCOUNT" else
                           (0.0 if k[0] in ("SUM", "COUNT", "COUNTMV") else (np.inf if k[0] == "MIN" else -np.inf)))
                          for k in oaggs]]
    for key, (cnt, row) in merged.items():
        vals = []
        for a, ai in zip(query.aggregations, amap):
            if a.function == "COUNT":
                vals.append(cnt)
            elif a.function == "AVG":
                vals.append(AvgPair(row[ai], cnt))
            elif a.function == "AVGMV":
                vals.append(AvgPair(row[ai[0]], int(row[ai[1]])))
            elif a.function == "COUNTMV":
                vals.append(int(row[ai]))
            elif a.function in Q.HLL_FUNCTIONS:
                vals.append(HyperLogLog(a.log2m, row[ai] if isinstance(row[ai], np.ndarray) else None))
            elif a.function in ("MINMAXRANGE", "MINMAXRANGEMV"):
                vals.append(MinMaxRangePair(row[ai[0]], row[ai[1]]))
            elif a.function in ("DISTINCTCOUNTBITMAP", "DISTINCTCOUNTBITMAPMV"):
                dt = segments[0].column(a.column).data_type
                vals.append({_java_hash(x, dt) for x in row[ai]})
            elif a.function in ("DISTINCTCOUNT", "DISTINCTCOUNTMV", "DISTINCTSUM", "DISTINCTSUMMV", "DISTINCTAVG",
                                "DISTINCTAVGMV"):
                vals.append(set(row[ai]))
            else:
                vals.append(row[ai])
        if query.group_by:
            out.groups[key] = vals
        else:
            out.row = vals
    return out


def run_query_arrays(query, segments):
    """run_query's server-level merge in array form, for the BASELINE-sized configs tests (up to ~1M groups, where the
    per-group Python objects of run_query cost more than the scan). Every segment must share one dictionary per
    group-by column, so the oracle's raw key (column 0 least significant) IS the GPU's table-wide key. Returns a dict:
    keys (ascending int64), counts (int64), accs (one array per oracle accumulator, in `oaggs` order: float64[n], or
    uint8[n, 2^log2m] HLL registers), oaggs, amap, matched (numDocsScanned) and limit_reached. Segments with their own
    dictionaries: each segment's raw key is decomposed over its own cardinalities and recomposed over the table-wide
    dictionaries (the sorted union of the segments' values, as the GPU's key space is), so keys are table-wide keys."""
    for c in query.group_by:
        if not all(s.column(c).has_dictionary for s in segments):
            raise ValueError("run_query_arrays: group-by column %s needs a dictionary in every segment" % c)
    tables = []
    for c in query.group_by:
        ds = [s.column(c).dictionary for s in segments]
        same = all(d is ds[0] or (len(d) == len(ds[0]) and np.array_equal(d, ds[0])) for d in ds)
        tables.append(ds[0] if same else np.unique(np.concatenate(ds)))
    raws = [_run_segment_raw(query, s) for s in segments]
    oaggs, amap = raws[0].oaggs, raws[0].amap
    if any(k[0] == "DISTINCTCOUNT" for k in oaggs):
        raise ValueError("run_query_arrays: DISTINCTCOUNT is compared through run_query")

    def table_keys(r, seg):
        raw = r.keys[:r.n].astype(np.int64)
        out = np.zeros(r.n, np.int64)
        stride = 1
        for c, gd in zip(query.group_by, tables):
            d = seg.column(c).dictionary
            comp = raw % len(d)
            raw = raw // len(d)
            out += (comp if d is gd else np.searchsorted(gd, d)[comp]) * stride
            stride *= len(gd)
        return out
    seg_keys = [table_keys(r, s) if query.group_by else np.zeros(r.n, np.int64) for r, s in zip(raws, segments)]
    uniq = np.unique(np.concatenate(seg_keys)) if seg_keys else np.zeros(0, np.int64)
    if not query.group_by:
        uniq = np.zeros(1, np.int64)
    u = len(uniq)
    cnt = np.zeros(u, np.int64)
    accs = []
    for k in oaggs:
        if k[0] == "DISTINCTCOUNTHLL":
            accs.append(np.zeros((u, 1 << k[2]), np.uint8))
        else:
            accs.append(np.full(u, np.inf if k[0] == "MIN" else (-np.inf if k[0] == "MAX" else 0.0)))
    for r, sk in zip(raws, seg_keys):
        idx = np.searchsorted(uniq, sk)  # a key occurs once per segment: plain fancy-index updates
        cnt[idx] += r.counts[:r.n]
        for ai, k in enumerate(oaggs):
            if k[0] == "DISTINCTCOUNTHLL":
                m = 1 << k[2]
                part = r.hll_bufs[ai][:r.n * m].reshape(r.n, m)
                accs[ai][idx] = np.maximum(accs[ai][idx], part)
            else:
                part = r.vals[ai * r.cap: ai * r.cap + r.n]
                if k[0] == "MIN":
                    accs[ai][idx] = np.minimum(accs[ai][idx], part)
                elif k[0] == "MAX":
                    accs[ai][idx] = np.maximum(accs[ai][idx], part)
                else:
                    accs[ai][idx] += part
    limit_reached = bool(query.group_by) and any(r.n >= query.num_groups_limit for r in raws)
    return {"keys": uniq.astype(np.int64), "counts": cnt, "accs": accs, "oaggs": oaggs, "amap": amap,
            "matched": sum(r.matched for r in raws), "limit_reached": limit_reached}
