"""Server trim + broker reduce of intermediate results (the callers either side of the hot path).

  merge_intermediate   ~ GroupByDataTableReducer / AggregationDataTableReducer merging server DataTables
                         (AggregationFunction.merge: COUNT/SUM +, MIN min, MAX max, AVG pair +, HLL addAll,
                         MINMAXRANGE pair min/max, DISTINCTCOUNT / DISTINCTSUM / DISTINCTAVG set union)
  server_trim          ~ IndexedTable.finish on the server (IndexedTable.java:149): with ORDER BY keep the top
                         max(limit*5, minServerGroupTrimSize) groups (GroupByUtils.getTableCapacity); without
                         ORDER BY keep `limit` groups (GroupByCombineOperator.java:63-73)
  final_result_table   ~ broker: extractFinalResult (AVG sum/count, HLL cardinality), ORDER BY, LIMIT
"""
import math
from functools import cmp_to_key

from . import query as Q
from .engine import AvgPair, IntermediateResult, MinMaxRangePair
from .hll import HyperLogLog


def merge_value(fn, a, b):
    fn = Q.base_function(fn)
    if fn in ("COUNT", "SUM"):
        return a + b
    if fn == "MIN":
        return min(a, b)
    if fn == "MAX":
        return max(a, b)
    if fn == "AVG":
        return AvgPair(a.sum + b.sum, a.count + b.count)
    if fn in ("DISTINCTCOUNTHLL", "DISTINCTCOUNTRAWHLL"):
        return HyperLogLog(a.log2m, a.registers).add_all(b)
    if fn == "MINMAXRANGE":  # MinMaxRangePair.apply
        return MinMaxRangePair(min(a.min, b.min), max(a.max, b.max))
    if fn in ("DISTINCTCOUNT", "DISTINCTSUM", "DISTINCTAVG", "DISTINCTCOUNTBITMAP"):
        # BaseDistinctAggregateAggregationFunction.merge: union (DISTINCTCOUNTBITMAP: RoaringBitmap.or)
        return set(a) | set(b)
    raise ValueError(fn)


def final_value(fn, v):
    fn = Q.base_function(fn)
    if fn == "AVG":
        return v.sum / v.count if v.count else -math.inf
    if fn == "DISTINCTCOUNTHLL":
        return v.cardinality()
    if fn == "DISTINCTCOUNTRAWHLL":
        return SerializedHLL(v)
    if fn == "MINMAXRANGE":  # MinMaxRangeAggregationFunction.extractFinalResult: max - min
        return v.max - v.min
    if fn in ("DISTINCTCOUNT", "DISTINCTCOUNTBITMAP"):  # extractFinalResult: the set's size / the bitmap's cardinality
        return len(v)
    if fn in ("DISTINCTSUM", "DISTINCTAVG"):
        # DistinctSumAggregationFunction / DistinctAvgAggregationFunction.extractFinalResult: a double sum over the set
        # in its iteration order, divided by its size for the average (0/0 = NaN for an empty set, as in Java). The
        # reference iterates a Java HashSet, this a Python set: for non-integer FLOAT/DOUBLE values the sums can differ
        # in the last bits (parity unpinned: no golden vector sums fractional distinct values; tests compare those
        # with a relative tolerance)
        s = 0.0
        for x in v:
            s += float(x)
        if fn == "DISTINCTSUM":
            return s
        return s / len(v) if len(v) else math.nan
    return v


def merge_intermediate(results):
    results = list(results)
    out = IntermediateResult(results[0].aggregations, results[0].group_by)
    fns = [a.function for a in out.aggregations]
    for r in results:
        out.num_docs_scanned += r.num_docs_scanned
        out.num_total_docs += r.num_total_docs
        out.num_entries_scanned_in_filter += r.num_entries_scanned_in_filter
        out.num_entries_scanned_post_filter += r.num_entries_scanned_post_filter
        out.num_groups_limit_reached |= r.num_groups_limit_reached
        if out.group_by:
            for k, vals in r.groups.items():
                if k in out.groups:
                    out.groups[k] = [merge_value(f, a, b) for f, a, b in zip(fns, out.groups[k], vals)]
                else:
                    out.groups[k] = list(vals)
        elif out.row is None:
            out.row = list(r.row)
        else:
            out.row = [merge_value(f, a, b) for f, a, b in zip(fns, out.row, r.row)]
    return out


class SerializedHLL(str):
    """DISTINCTCOUNTRAWHLL's final result (SerializedHLL.java): the string is BytesUtils.toHexString of
    HyperLogLog.getBytes(); ORDER BY compares cardinalities (compareTo)."""

    def __new__(cls, hll):
        s = str.__new__(cls, hll.to_bytes().hex())
        s.cardinality = hll.cardinality()
        return s


def _sort_value(v):
    return v.cardinality if isinstance(v, SerializedHLL) else v


def _order_key_fn(query):
    """Comparator over (key, final values) following ORDER BY; ties broken by group key for determinism."""
    items = []
    for ob in query.order_by:
        if isinstance(ob.expr, Q.Aggregation):
            idx = None
            for i, a in enumerate(query.aggregations):
                if a == ob.expr:
                    idx = i
            if idx is None:
                raise ValueError("ORDER BY aggregation not in select list: %r" % (ob.expr,))
            items.append(("agg", idx, ob.asc))
        else:
            items.append(("key", query.group_by.index(ob.expr), ob.asc))

    def cmp(x, y):
        for kind, idx, asc in items:
            a = _sort_value(x[1][idx]) if kind == "agg" else x[0][idx]
            b = _sort_value(y[1][idx]) if kind == "agg" else y[0][idx]
            if a != b:
                c = -1 if a < b else 1
                return c if asc else -c
        return -1 if x[0] < y[0] else (1 if x[0] > y[0] else 0)
    return cmp_to_key(cmp)


def server_trim(res: IntermediateResult, query: Q.Query) -> IntermediateResult:
    if not query.group_by:
        return res
    fns = [a.function for a in query.aggregations]
    if query.order_by:
        trim = max(query.limit * 5, query.min_server_group_trim_size)
    else:
        trim = query.limit
    if len(res.groups) <= trim:
        return res
    rows = [(k, [final_value(f, v) for f, v in zip(fns, vals)], k) for k, vals in res.groups.items()]
    if query.order_by:
        rows.sort(key=_order_key_fn(query))
    else:
        rows.sort(key=lambda r: r[0])
    keep = {r[2] for r in rows[:trim]}
    out = IntermediateResult(res.aggregations, res.group_by, {k: v for k, v in res.groups.items() if k in keep})
    out.num_docs_scanned, out.num_total_docs = res.num_docs_scanned, res.num_total_docs
    out.num_entries_scanned_in_filter = res.num_entries_scanned_in_filter
    out.num_entries_scanned_post_filter = res.num_entries_scanned_post_filter
    out.num_groups_limit_reached = res.num_groups_limit_reached
    return out


def final_result_table(res: IntermediateResult, query: Q.Query):
    """Broker ResultTable rows: [select group-by columns..., final aggregation values...]."""
    fns = [a.function for a in query.aggregations]
    nsel = query.num_select_aggs if query.num_select_aggs >= 0 else len(fns)
    if not query.group_by:
        return [[final_value(f, v) for f, v in zip(fns, res.row)][:nsel]]
    rows = [(k, [final_value(f, v) for f, v in zip(fns, vals)]) for k, vals in res.groups.items()]
    if query.order_by:
        rows.sort(key=_order_key_fn(query))
    else:
        rows.sort(key=lambda r: r[0])
    rows = rows[: query.limit]
    sel = query.select_columns
    out = []
    for k, vals in rows:
        out.append([k[query.group_by.index(c)] for c in sel] + vals[:nsel])
    return out
