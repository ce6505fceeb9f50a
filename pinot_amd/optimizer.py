"""The reference's compile-time filter rewrites, restated over query.py's filter model.

QueryOptimizer.java (pinot-core/.../query/optimizer/QueryOptimizer.java:47-50) runs, in this order:
  FlattenAndOrFilterOptimizer      AND(AND(a, b), c) -> AND(a, b, c), same for OR
  IdenticalPredicateFilterOptimizer `col = col` -> TRUE, `col != col` -> FALSE (and literal comparisons, which the
                                   reference folds at compile time), then TRUE/FALSE propagated through AND / OR / NOT
                                   (BaseAndOrBooleanFilterOptimizer.optimizeCurrent)
  MergeEqInFilterOptimizer         EQ / IN children of an OR on one column -> one IN (EQ when one value), IN values
                                   de-duplicated
  NumericalFilterOptimizer         a numeric literal outside the column type's range / not representable in it: EQ, NEQ
                                   and single-bound ranges become TRUE / FALSE, others get the literal in the column type
  TimePredicateFilterOptimizer     (dateTimeConvert / timeConvert on the left-hand side: transform expressions are not
                                   on this path)
  MergeRangeFilterOptimizer        range children of an AND on one single-value column -> one RANGE (intersection)
  TextMatchFilterOptimizer         (TEXT_MATCH: no text index on this path)
The rewrites change the operator tree the server builds (FilterPlanNode), hence numEntriesScannedInFilter: a
`col >= a AND col <= b` filter is one scan of col, not two (filter_stats.py), and they give the same documents.
Pinned by the reference's own input / expected pairs (QueryOptimizerTest.java:188-249, tests/golden/
query_optimizer.json, tests/test_optimizer.py) and NumericalFilterOptimizerTest cases.
"""
from decimal import Decimal

import numpy as np

from . import query as Q

TRUE = Q.BoolFilter(True)
FALSE = Q.BoolFilter(False)
INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
NUMERIC = ("INT", "LONG", "FLOAT", "DOUBLE")


def optimize_filter(f, schema):
    """schema: {column: (data type, single value)} (FieldSpec type and isSingleValueField). None stays None."""
    if f is None:
        return None
    f = flatten(f)
    f = _bool_pass(f, _identical_child)
    f = merge_eq_in(f)
    f = _bool_pass(f, lambda c: _numerical_child(c, schema))
    f = merge_range(f, schema)
    return f


# ------------------------------------------------------------------ FlattenAndOrFilterOptimizer
def flatten(f):
    """FlattenAndOrFilterOptimizer.optimize (:43-64): only AND / OR nodes, recursively through AND / OR operands."""
    if isinstance(f, (Q.And, Q.Or)):
        kids = []
        for c in f.children:
            c = flatten(c)
            if type(c) is type(f):
                kids.extend(c.children)
            else:
                kids.append(c)
        return type(f)(tuple(kids))
    return f  # a NOT (and anything else) is returned as it is: its operand is not flattened (:48-51)


# ------------------------------------------------------------------ BaseAndOrBooleanFilterOptimizer
def _bool_pass(f, child_fn):
    """optimize(): AND / OR / NOT recurse into their operands then optimizeCurrent; other nodes go to child_fn."""
    if isinstance(f, (Q.And, Q.Or)):
        kids = [_bool_pass(c, child_fn) for c in f.children]
        if isinstance(f, Q.And):
            if FALSE in kids:
                return FALSE
            kids = [k for k in kids if k != TRUE]
            if not kids:
                return TRUE
        else:
            if TRUE in kids:
                return TRUE
            kids = [k for k in kids if k != FALSE]
            if not kids:
                return FALSE
        return type(f)(tuple(kids))  # (a single remaining operand keeps its AND / OR node, as in the reference)
    if isinstance(f, Q.Not):
        c = _bool_pass(f.child, child_fn)
        if c == TRUE:
            return FALSE
        if c == FALSE:
            return TRUE
        return Q.Not(c)
    return child_fn(f)


def _num(text):
    try:
        return Decimal(text)
    except Exception:
        return None


# ------------------------------------------------------------------ IdenticalPredicateFilterOptimizer
def _identical_child(f):
    if not isinstance(f, Q.Comparison):
        return f
    (lk, lv), (rk, rv) = f.lhs, f.rhs
    if lk == "id" and rk == "id":
        if lv != rv:
            return f  # two different columns: not rewritten (and not evaluable on this path)
        return TRUE if f.op == "=" else FALSE
    if lk == "lit" and rk == "lit":  # compile-time evaluation of a literal comparison
        a, b = _num(lv), _num(rv)
        eq = (a == b) if (a is not None and b is not None) else (lv == rv)
        return TRUE if eq == (f.op == "=") else FALSE
    return f


# ------------------------------------------------------------------ MergeEqInFilterOptimizer
def _eq_in_values(f):
    if isinstance(f, Q.EqPredicate):
        return [f.value]
    return list(f.values)


def _dedup(vals):
    out = []
    for v in vals:
        if v not in out:
            out.append(v)
    return out


def _eq_or_in(column, vals):
    return Q.EqPredicate(column, vals[0]) if len(vals) == 1 else Q.InPredicate(column, tuple(vals))


def _or_child(c):
    """An AND / NOT operand of an OR: its own operands optimized (MergeEqInFilterOptimizer.java:61-63), so a NOT is
    recursed into only here, as an OR's child."""
    if isinstance(c, Q.Not):
        return Q.Not(merge_eq_in(c.child))
    return merge_eq_in(c)


def merge_eq_in(f):
    """MergeEqInFilterOptimizer.optimize (:46-140): OR nodes merge their EQ / IN operands per column, AND nodes recurse
    into their operands, an IN node alone is de-duplicated; a NOT at the top or under an AND is returned as it is."""
    if isinstance(f, Q.Or):
        values, order, kids = {}, [], []
        recreate = False
        for c in f.children:
            if isinstance(c, (Q.And, Q.Not)):
                kids.append(_or_child(c))
            elif isinstance(c, (Q.EqPredicate, Q.InPredicate)):
                vals = _eq_in_values(c)
                if isinstance(c, Q.InPredicate):
                    uniq = _dedup(vals)
                    if len(uniq) == 1 or len(uniq) != len(vals):
                        recreate = True
                    vals = uniq
                if c.column in values:
                    values[c.column] = _dedup(values[c.column] + vals)
                    recreate = True
                else:
                    values[c.column] = list(vals)
                    order.append(c.column)
            else:
                kids.append(c)
        if not recreate:
            return Q.Or(tuple(_or_child(c) if isinstance(c, (Q.And, Q.Not)) else c for c in f.children))
        if not kids and len(values) == 1:
            return _eq_or_in(order[0], values[order[0]])
        return Q.Or(tuple(kids + [_eq_or_in(col, values[col]) for col in order]))
    if isinstance(f, Q.And):
        return Q.And(tuple(merge_eq_in(c) for c in f.children))
    if isinstance(f, Q.InPredicate):
        uniq = _dedup(list(f.values))
        if len(uniq) == 1 or len(uniq) != len(f.values):
            return _eq_or_in(f.column, uniq)
    return f


# ------------------------------------------------------------------ NumericalFilterOptimizer
def _is_int_text(text):
    return _num(text) is not None and all(ch not in text for ch in ".eE")


def _literal(text):
    """(kind, value) of a numeric literal as the reference's SQL compiler types it (RequestUtils.java:108-121): an exact
    integer -> INT (int range) or LONG (BigDecimal.longValue: the low 64 bits), anything else -> DOUBLE (the
    BigDecimal's correctly rounded double). (None, None) for a non-numeric literal."""
    d = _num(text)
    if d is None or not d.is_finite():
        return None, None
    if _is_int_text(text):
        i = int(d)
        if INT_MIN <= i <= INT_MAX:
            return "INT", i
        i &= (1 << 64) - 1
        return "LONG", i - (1 << 64) if i > LONG_MAX else i
    return "DOUBLE", float(d)


def _bd(x):
    """BigDecimal.valueOf: a long exactly, a double through Double.toString (the shortest repr that round-trips, as
    Python's repr and JDK >= 19's Double.toString give it)."""
    return Decimal(x) if isinstance(x, int) else Decimal(repr(float(x)))


def _f32_of_long(v):
    """(float) of a Java long: one IEEE rounding (numpy's int64 -> float32 cast), widened to double."""
    return float(np.float32(np.int64(v)))


def _f32_of_double(x):
    with np.errstate(over="ignore"):
        return float(np.float32(x))


def _cast_int(x, lo, hi):
    """(int) / (long) of a Java double: NaN -> 0, truncation toward zero, saturating at the type's bounds."""
    if x != x:
        return 0
    if x >= hi:
        return hi
    if x <= lo:
        return lo
    return int(x)


def _cmp(a, b):
    return (a > b) - (a < b)


def _numerical_child(f, schema):
    """NumericalFilterOptimizer.optimizeChild: only on a single-value numeric column (getDataType returns null for a
    multi-value one, :370-376), with a numeric literal."""
    dt, sv = schema.get(getattr(f, "column", None), (None, True))
    if dt not in NUMERIC or not sv:
        return f
    if isinstance(f, (Q.EqPredicate, Q.NotEqPredicate)):
        return _numerical_eq(f, dt)
    if isinstance(f, Q.RangePredicate) and ((f.lower == Q.UNBOUNDED) != (f.upper == Q.UNBOUNDED)):
        return _numerical_range(f, dt)
    return f


def _numerical_eq(f, dt):
    """rewriteEqualsExpression (NumericalFilterOptimizer.java:96-185)."""
    kind, v = _literal(str(f.value))
    const = TRUE if isinstance(f, Q.NotEqPredicate) else FALSE
    if kind == "LONG":
        if dt == "INT":
            return const  # (int) of a long outside INT differs from it
        if dt in ("FLOAT", "DOUBLE"):
            conv = _f32_of_long(v) if dt == "FLOAT" else float(v)
            if _bd(v) != _bd(conv):
                return const  # lossy conversion
            return type(f)(f.column, repr(conv))
    elif kind == "DOUBLE":
        if dt == "INT":
            conv = _cast_int(v, INT_MIN, INT_MAX)
            if conv != v:
                return const
            return type(f)(f.column, str(conv))
        if dt == "LONG":
            conv = _cast_int(v, LONG_MIN, LONG_MAX)
            if _bd(v) != _bd(conv):
                return const
            return type(f)(f.column, str(conv))
    return f


def _numerical_range(f, dt):
    """rewriteRangeExpression + rewriteRangeOperator (NumericalFilterOptimizer.java:187-360)."""
    lower_side = f.lower != Q.UNBOUNDED  # col > v / col >= v
    kind, v = _literal(str(f.lower if lower_side else f.upper))
    greater_true = TRUE if lower_side else FALSE  # the literal lies below every value of the type
    less_true = FALSE if lower_side else TRUE     # the literal lies above every value of the type

    def rewritten(conv_text, cmp):
        # rewriteRangeOperator: literal > converted: "> / >=" -> ">", "< / <=" -> "<="; literal < converted: "> / >="
        # -> ">=", "< / <=" -> "<"
        if lower_side:
            incl = f.lower_inclusive if cmp == 0 else cmp < 0
            return Q.RangePredicate(f.column, conv_text, incl, Q.UNBOUNDED, False)
        incl = f.upper_inclusive if cmp == 0 else cmp > 0
        return Q.RangePredicate(f.column, Q.UNBOUNDED, False, conv_text, incl)

    if kind == "LONG":
        if dt == "INT":
            return less_true if v > INT_MAX else greater_true
        if dt in ("FLOAT", "DOUBLE"):
            conv = _f32_of_long(v) if dt == "FLOAT" else float(v)
            return rewritten(repr(conv), _cmp(_bd(v), _bd(conv)))
    elif kind == "DOUBLE":
        if dt in ("INT", "LONG"):
            lo, hi = (INT_MIN, INT_MAX) if dt == "INT" else (LONG_MIN, LONG_MAX)
            conv = _cast_int(v, lo, hi)
            cmp = _cmp(v, conv) if dt == "INT" else _cmp(_bd(v), _bd(conv))  # Double.compare / BigDecimal.compareTo
            if cmp > 0 and conv == hi:
                return less_true
            if cmp < 0 and conv == lo:
                return greater_true
            return rewritten(str(conv), cmp)
        if dt == "FLOAT":
            c = _f32_of_double(v)
            if c == float("inf"):
                return less_true
            if c == float("-inf"):
                return greater_true
    return f


# ------------------------------------------------------------------ MergeRangeFilterOptimizer
def _typed(text, dt):
    """dataType.convertInternal of a literal: the comparable bound of a range."""
    if text == Q.UNBOUNDED:
        return None
    if dt in ("INT", "LONG"):
        # Integer.valueOf / Long.valueOf of the literal text: a fractional or exponent text ("1.5", "3.0", "1e3") is
        # a NumberFormatException in the reference, which fails the query
        if not _is_int_text(str(text)):
            raise ValueError("range bound %r of an %s column is not an integer (the reference's MergeRangeFilterOptimizer "
                             "rejects it: NumberFormatException)" % (text, dt))
        return int(Decimal(str(text)))
    if dt == "FLOAT":
        with np.errstate(over="ignore"):
            return float(np.float32(float(text)))
    if dt == "DOUBLE":
        return float(text)
    if dt == "BYTES":
        return bytes.fromhex(str(text))
    return str(text)


def _java_string_hash(s):
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h


def _hashmap_order(keys):
    """Iteration order of a java.util.HashMap<String, _> filled with `keys` in order (default capacity 16, no resize
    below 13 keys): bucket (h ^ h >>> 16) & (capacity - 1) ascending, insertion order within a bucket."""
    cap = 16
    while len(keys) > cap * 3 // 4:
        cap *= 2
    def bucket(k):
        h = _java_string_hash(k)
        return (h ^ (h >> 16)) & (cap - 1)
    return sorted(keys, key=lambda k: (bucket(k), keys.index(k)))


class _Range:
    """Range.java: bounds as typed comparables (None = unbounded), intersected in place."""

    def __init__(self, p, dt):
        self.lo, self.li = _typed(p.lower, dt), p.lower_inclusive
        self.hi, self.ui = _typed(p.upper, dt), p.upper_inclusive
        self.lt, self.ut = p.lower, p.upper  # literal texts of the bounds

    def intersect(self, o):
        if o.lo is not None:
            if self.lo is None or self.lo < o.lo:
                self.lo, self.li, self.lt = o.lo, o.li, o.lt
            elif self.lo == o.lo:
                self.li = self.li and o.li
        if o.hi is not None:
            if self.hi is None or self.hi > o.hi:
                self.hi, self.ui, self.ut = o.hi, o.ui, o.ut
            elif self.hi == o.hi:
                self.ui = self.ui and o.ui

    def predicate(self, column):
        return Q.RangePredicate(column, Q.UNBOUNDED if self.lo is None else self.lt, self.lo is not None and self.li,
                                Q.UNBOUNDED if self.hi is None else self.ut, self.hi is not None and self.ui)


def merge_range(f, schema):
    if isinstance(f, Q.And):
        ranges, order, kids = {}, [], []
        recreate = False
        for c in f.children:
            if isinstance(c, (Q.Or, Q.Not)):
                kids.append(merge_range(c, schema))
            elif isinstance(c, Q.RangePredicate):
                dt, sv = schema.get(c.column, (None, True))
                if dt is None or not sv:  # (multi-value: [0, 10] matches "col < 1 AND col > 9", not the merged range)
                    kids.append(c)
                    continue
                r = _Range(c, dt)
                if c.column in ranges:
                    ranges[c.column].intersect(r)
                    recreate = True
                else:
                    ranges[c.column] = r
                    order.append(c.column)
            else:
                kids.append(c)
        if not recreate:
            return Q.And(tuple(merge_range(c, schema) if isinstance(c, (Q.Or, Q.Not)) else c for c in f.children))
        if not kids and len(ranges) == 1:
            return ranges[order[0]].predicate(order[0])
        return Q.And(tuple(kids + [ranges[col].predicate(col) for col in _hashmap_order(order)]))
    if isinstance(f, (Q.Or,)):
        return Q.Or(tuple(merge_range(c, schema) for c in f.children))
    if isinstance(f, Q.Not):
        return Q.Not(merge_range(f.child, schema))
    return f
