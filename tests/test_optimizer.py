"""The reference's compile-time filter rewrites (pinot_amd/optimizer.py) against its own input / expected pairs
(QueryOptimizerTest.java testQueries, tests/golden/query_optimizer.json) and NumericalFilterOptimizer cases, and their
effect on the execution statistics (a merged range is one scan: filter_stats.py)."""
import json
import os
from decimal import Decimal

import numpy as np
import pytest

from conftest import GOLDEN
from pinot_amd import query as Q
from pinot_amd.optimizer import optimize_filter, _typed


def _spec():
    with open(os.path.join(GOLDEN, "query_optimizer.json")) as f:
        d = json.load(f)
    return d, {k: tuple(v) for k, v in d["schema"].items()}


def _norm(f, schema):
    """Canonical form of an optimized filter for comparePinotQuery's equality (QueryOptimizerTest.java:319-393): AND /
    OR children and IN values in any order, ranges by their typed bounds (the range string)."""
    if isinstance(f, (Q.And, Q.Or)):
        if len(f.children) == 1:  # (FilterOperatorUtils: an AND / OR of one child is that child)
            return _norm(f.children[0], schema)
        return (type(f).__name__, tuple(sorted((repr(_norm(c, schema)) for c in f.children))))
    if isinstance(f, Q.Not):
        return ("Not", _norm(f.child, schema))
    if isinstance(f, Q.RangePredicate):
        dt = schema[f.column][0]
        lo, hi = _typed(f.lower, dt), _typed(f.upper, dt)
        return ("Range", f.column, lo, lo is not None and f.lower_inclusive, hi, hi is not None and f.upper_inclusive)
    if isinstance(f, (Q.InPredicate, Q.NotInPredicate)):
        return (type(f).__name__, f.column, tuple(sorted(set(_lit(v) for v in f.values))))
    if isinstance(f, (Q.EqPredicate, Q.NotEqPredicate)):
        return (type(f).__name__, f.column, _lit(f.value))
    return f


def _lit(v):
    try:
        return ("n", Decimal(str(v)))
    except Exception:
        return ("s", str(v))


@pytest.mark.parametrize("i", range(40))
def test_reference_optimizer_pairs(i):
    d, schema = _spec()
    if i >= len(d["pairs"]):
        pytest.skip("fewer pairs")
    p = d["pairs"][i]
    got = optimize_filter(Q.parse_filter(p["input"]), schema)
    exp = optimize_filter(Q.parse_filter(p["expected"]), schema)
    assert _norm(got, schema) == _norm(exp, schema), (p, got, exp)


def test_golden_fixture_has_every_pair():
    d, _ = _spec()
    assert len(d["pairs"]) == 40


SCHEMA = {"intColumn": ("INT", True), "longColumn": ("LONG", True), "floatColumn": ("FLOAT", True),
          "doubleColumn": ("DOUBLE", True)}


@pytest.mark.parametrize("where,expected", [
    # NumericalFilterOptimizerTest.java (EQ / NEQ / ranges against the column type)
    ("intColumn = 5000000000", "false"),
    ("intColumn != 5000000000", "true"),
    ("intColumn = 5.5", "false"),
    ("intColumn != 5.5", "true"),
    ("intColumn = 5.0", "intColumn = 5"),
    ("longColumn = 5.5", "false"),
    ("intColumn > 5000000000", "false"),
    ("intColumn < 5000000000", "true"),
    ("intColumn > -5000000000", "true"),
    ("intColumn <= -5000000000", "false"),
    ("intColumn > 5.5", "intColumn > 5"),
    ("intColumn >= 5.5", "intColumn > 5"),
    ("intColumn < 5.5", "intColumn <= 5"),
    ("intColumn <= -5.5", "intColumn < -5"),
    ("intColumn > 3000000000.5", "false"),
    ("floatColumn > 1e40", "false"),
    ("floatColumn < -1e40", "false"),
    ("intColumn > 5000000000 AND longColumn = 3", "false"),
    ("intColumn < 5000000000 AND longColumn = 3", "longColumn = 3"),
])
def test_numerical_filter_rewrites(where, expected):
    got = optimize_filter(Q.parse_filter(where), SCHEMA)
    exp = Q.parse_filter(expected)
    assert _norm(got, SCHEMA) == _norm(exp, SCHEMA), (where, got)


def test_merged_range_is_one_scan_in_the_statistics():
    """MergeRangeFilterOptimizer feeds the execution statistics: `col >= a AND col <= b` reads col once per doc (one
    SVScanDocIdIterator over a RANGE predicate), where the unrewritten AND of two scans pays the leap-frogging."""
    from pinot_amd import filter_stats as FS
    from pinot_amd.segment import create_segment, unpack_bits
    n = 5000
    seg = create_segment("s", {"x": np.random.default_rng(3).integers(0, 100, n).astype(np.int32)}, {"x": "INT"})
    raw = Q.parse_filter("x >= 10 AND x <= 40")
    opt = optimize_filter(raw, {"x": ("INT", True)})
    assert isinstance(opt, Q.RangePredicate)
    col = seg.column("x")
    v = col.dictionary[unpack_bits(col.fwd_bytes, n, col.num_bits)]
    in_one = FS.entries_scanned_in_filter(opt, seg, np.asarray([(v >= 10) & (v <= 40)]))
    in_two = FS.entries_scanned_in_filter(raw, seg, np.asarray([v >= 10, v <= 40]))
    assert in_one == n  # one scan driven to EOF reads every entry once
    assert in_two > n


SCHEMA_MV = dict(SCHEMA, mvIntColumn=("INT", False))


@pytest.mark.parametrize("where,expected", [
    # FlattenAndOrFilterOptimizer returns a NOT as it is; MergeEqInFilterOptimizer recurses into a NOT only as an OR's
    # operand (FlattenAndOrFilterOptimizer.java:48-51, MergeEqInFilterOptimizer.java:61-63, :117)
    ("NOT (intColumn = 1 OR intColumn = 2)", "NOT (intColumn = 1 OR intColumn = 2)"),
    ("longColumn > 3 AND NOT (intColumn = 1 OR intColumn = 2)", "longColumn > 3 AND NOT (intColumn = 1 OR intColumn = 2)"),
    ("longColumn = 3 OR NOT (intColumn = 1 OR intColumn = 2)", "longColumn = 3 OR NOT (intColumn IN (1, 2))"),
    ("NOT (intColumn IN (1, 1))", "NOT (intColumn IN (1, 1))"),
    ("longColumn = 3 OR NOT (intColumn IN (1, 1))", "longColumn = 3 OR NOT (intColumn = 1)"),
    # numerical rewrites skip multi-value columns (getDataType returns null for them, NumericalFilterOptimizer.java:370)
    ("mvIntColumn = 5000000000", "mvIntColumn = 5000000000"),
    ("mvIntColumn > 5.5", "mvIntColumn > 5.5"),
    # a DOUBLE literal is compared as the double the SQL compiler made of it (RequestUtils.java:121)
    ("intColumn = 3.00000000000000001", "intColumn = 3"),
    ("longColumn >= 1.00000000000000001", "longColumn >= 1"),
    ("longColumn = 5.0", "longColumn = 5"),
])
def test_not_and_numerical_semantics(where, expected):
    got = optimize_filter(Q.parse_filter(where), SCHEMA_MV)
    exp = Q.parse_filter(expected)
    assert _canon(got) == _canon(exp), (where, got)


def _canon(f):
    """Structure-preserving form (unlike _norm, nested NOT / AND / OR nodes and IN duplicates stay as they are)."""
    if isinstance(f, (Q.And, Q.Or)):
        return (type(f).__name__, tuple(sorted(repr(_canon(c)) for c in f.children)))
    if isinstance(f, Q.Not):
        return ("Not", _canon(f.child))
    if isinstance(f, (Q.InPredicate, Q.NotInPredicate)):
        return (type(f).__name__, f.column, tuple(sorted(_lit(v) for v in f.values)))
    if isinstance(f, (Q.EqPredicate, Q.NotEqPredicate)):
        return (type(f).__name__, f.column, _lit(f.value))
    if isinstance(f, Q.RangePredicate):
        return ("Range", f.column, _lit(f.lower), f.lower_inclusive, _lit(f.upper), f.upper_inclusive)
    return f


@pytest.mark.parametrize("where", [
    "intColumn >= 1 AND intColumn BETWEEN 1.5 AND 10",
    "intColumn BETWEEN -1.5 AND 3 AND intColumn > -1",
    "longColumn BETWEEN 2.0 AND 5 AND doubleColumn = 1",
])
def test_fractional_range_bound_of_an_integer_column_fails(where):
    """MergeRangeFilterOptimizer converts every range operand of an AND with Integer.valueOf / Long.valueOf of the
    literal text (getComparable, :134): a fractional bound fails the query instead of merging to a wrong range."""
    with pytest.raises(ValueError, match="not an integer"):
        optimize_filter(Q.parse_filter(where), SCHEMA)


def test_integral_range_bounds_still_merge():
    got = optimize_filter(Q.parse_filter("intColumn >= 1 AND intColumn BETWEEN 2 AND 10"), SCHEMA)
    assert isinstance(got, Q.RangePredicate) and (got.lower, got.lower_inclusive, got.upper) == ("2", True, "10")
