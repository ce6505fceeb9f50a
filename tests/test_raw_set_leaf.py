"""Host side of the RAW_SET leaf (IN / NOT IN on a no-dictionary column, RawValueBasedInPredicateEvaluatorFactory.java):
the list becomes one leaf of the column type's stored values, sorted and unique (FLOAT literals rounded to float then
widened, NaN dropped), and matches what the oracle evaluates value by value. No GPU."""
import numpy as np

import oracle
from pinot_amd import _lib as L
from pinot_amd import parse_sql
from pinot_amd import predicate as P
from pinot_amd.engine import _flatten_filter
from pinot_amd.segment import create_segment


def _seg(n=4000, seed=2):
    rng = np.random.default_rng(seed)
    data = {"ri": rng.integers(-50, 50, n).astype(np.int32), "rl": rng.integers(-(1 << 40), 1 << 40, n),
            "rf": (rng.integers(-80, 80, n) / 4.0).astype(np.float32), "rd": rng.integers(-90, 90, n) / 8.0}
    return create_segment("rs", data, {"ri": "INT", "rl": "LONG", "rf": "FLOAT", "rd": "DOUBLE"},
                          no_dictionary_columns=tuple(data))


def test_raw_in_is_one_sorted_unique_leaf():
    seg = _seg()
    q = parse_sql("SELECT COUNT(*) FROM t WHERE ri IN (7, -3, 7, 40, 1000000) AND rf NOT IN (1.1, 0.25, -2.5)")
    leaves, ops = [], []
    _flatten_filter(q.filter, leaves, ops)
    assert len(leaves) == 2
    a = P.raw_leaf(leaves[0], seg.column("ri"))
    assert a.kind == L.PA_LEAF_RAW_SET and not a.negate and a.values.dtype == np.int64
    assert a.values.tolist() == [-3, 7, 40, 1000000]
    b = P.raw_leaf(leaves[1], seg.column("rf"))
    assert b.kind == L.PA_LEAF_RAW_SET and b.negate and b.values.dtype == np.float64
    # FLOAT literals: the stored float (Float.parseFloat), widened — 1.1 is not 1.1 as a double
    assert b.values.tolist() == sorted([float(np.float32(1.1)), 0.25, -2.5])


def test_raw_set_matches_the_oracle():
    seg = _seg()
    rng = np.random.default_rng(4)
    for col in ("ri", "rl", "rf", "rd"):
        vals = seg.column(col).raw_values
        pick = rng.choice(vals, 25)
        lits = ", ".join(repr(float(np.float32(v))) if col == "rf" else (repr(float(v)) if col == "rd" else str(int(v)))
                         for v in pick)
        for neg in (False, True):
            q = parse_sql("SELECT COUNT(*) FROM t WHERE %s %sIN (%s, 123456789)" % (col, "NOT " if neg else "", lits))
            lf = P.raw_leaf(q.filter, seg.column(col))
            m = np.isin(vals.astype(np.float64) if col in ("rf", "rd") else vals.astype(np.int64), lf.values)
            assert int((~m if neg else m).sum()) == oracle.run_query(q, [seg]).row[0], (col, neg)


def test_oracle_evaluates_lists_past_256_values():
    """The oracle expands a raw IN list into one equality leaf per value (its restatement of the reference's per-value
    set test); its postfix ops carry the leaf index in 24 bits (8 bits wrapped past 256 values)."""
    seg = _seg()
    vals = np.unique(seg.column("ri").raw_values)
    lits = ", ".join(str(int(v)) for v in vals[::2]) + ", " + ", ".join(str(10_000 + i) for i in range(300))
    q = parse_sql("SELECT COUNT(*) FROM t WHERE ri IN (%s)" % lits)
    lf = P.raw_leaf(q.filter, seg.column("ri"))
    assert len(lf.values) > 256
    want = int(np.isin(seg.column("ri").raw_values.astype(np.int64), lf.values).sum())
    assert oracle.run_query(q, [seg]).num_docs_scanned == want
