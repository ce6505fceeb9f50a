"""REGEXP_LIKE / LIKE on dictionary columns (host side; no GPU): LIKE -> regex as RegexpPatternConverterUtils.
likeToRegexpLike does (pinned by the reference's own test vectors, RegexpPatternConverterUtilsTest.java:28-128), the
parser's RequestContextUtils mapping (RequestContextUtils.java:231-236), the per-segment matching dictIds
(DictionaryBasedRegexpLikePredicateEvaluator: Matcher.find() on each dictionary value) against the oracle, and the
statistics' operator choice (a scan whatever the column's indexes, never the always-true / always-false operators:
FilterOperatorUtils.java:108-117)."""
import numpy as np
import pytest

import oracle
from pinot_amd import filter_stats as FS
from pinot_amd import parse_sql
from pinot_amd import predicate as P
from pinot_amd import query as Q
from pinot_amd.segment import create_segment

# RegexpPatternConverterUtilsTest.java: (LIKE pattern, likeToRegexpLike result)
LIKE_VECTORS = [
    ("%++", r"\+\+$"), ("C+%", r"^C\+"), ("%+%", r"\+"), ("C%+", r"^C.*\+$"), ("_++", r"^.\+\+$"),
    ("C+_", r"^C\+.$"), ("C_+", r"^C.\+$"), ("C_%", r"^C."), ("%%%%%%%%%%%%%zz", "zz$"), ("zz%%%%%%%%%%%%%", "^zz"),
    ("%z", "z$"), ("z%", "^z"), ("a\\_b_\\", "^a\\_b.\\\\$"),
]

WORDS = np.array(["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta", "iota", "kappa", "lambda", "mu",
                  "C++", "C#", "a_b", "a+b", "axb"])


def _seg(n=6000, seed=3, sorted_col=False):
    rng = np.random.default_rng(seed)
    s = WORDS[rng.integers(0, len(WORDS), n)]
    data = {"s": np.sort(s) if sorted_col else s, "d": rng.integers(0, 10, n).astype(np.int32),
            "m": rng.integers(0, 100, n).astype(np.int64)}
    return create_segment("rx%d" % seed, data, {"s": "STRING", "d": "INT", "m": "LONG"})


@pytest.mark.parametrize("like,regex", LIKE_VECTORS)
def test_like_to_regexp_reference_vectors(like, regex):
    assert Q.like_to_regexp(like) == regex


def test_parse_regexp_like_and_like():
    q = parse_sql("SELECT COUNT(*) FROM t WHERE REGEXP_LIKE(s, 'ta$') AND s NOT LIKE 'a%' OR s LIKE 'C_+'")
    a, b = q.filter.children
    assert a.children[0] == Q.RegexpLikePredicate("s", "ta$")
    assert a.children[1] == Q.Not(Q.RegexpLikePredicate("s", "^a"))
    assert b == Q.RegexpLikePredicate("s", r"^C.\+$")


@pytest.mark.parametrize("where", ["REGEXP_LIKE(s, 'ta$')", "s LIKE '%ta'", "s NOT LIKE 'a%'", "s LIKE 'C_+'",
                                   "s LIKE 'a\\_b'", "REGEXP_LIKE(s, 'e.a') AND d < 5", "REGEXP_LIKE(s, 'nomatch')",
                                   "REGEXP_LIKE(s, '')"])
def test_matching_dict_ids_equal_the_oracle(where):
    seg = _seg()
    q = parse_sql("SELECT COUNT(*) FROM t WHERE " + where)
    preds = []

    def walk(f):
        if isinstance(f, (Q.And, Q.Or)):
            for c in f.children:
                walk(c)
        elif isinstance(f, Q.Not):
            walk(f.child)
        elif isinstance(f, Q.RegexpLikePredicate):
            preds.append(f)
    walk(q.filter)
    col = seg.column("s")
    for p in preds:
        lf = P.dictionary_leaf(p, col)
        ids = np.arange(lf.lo, lf.hi) if lf.ids is None else np.unique(lf.ids)
        want = np.flatnonzero(oracle._dict_match(p, col))
        assert ids.tolist() == want.tolist(), p
    assert oracle.run_query(q, [seg]).row[0] >= 0


def test_regexp_like_on_a_non_string_column_is_refused():
    seg = _seg()
    with pytest.raises(ValueError):
        P.dictionary_leaf(Q.RegexpLikePredicate("d", "1"), seg.column("d"))


@pytest.mark.parametrize("sorted_col", [False, True])
@pytest.mark.parametrize("pattern", ["ta$", "nomatch", ""])
def test_statistics_take_the_scan_operator(sorted_col, pattern):
    seg = _seg(sorted_col=sorted_col)
    op = FS._leaf_op(Q.RegexpLikePredicate("s", pattern), seg, None, lambda c: (False, False, True))
    assert op.kind == "scan"


def test_distinct_quantifier_rewrites():
    """CalciteSqlParser.java:761-772: COUNT / SUM / AVG (DISTINCT x) are DISTINCTCOUNT / DISTINCTSUM / DISTINCTAVG; any
    other aggregation on DISTINCT is refused."""
    q = parse_sql("SELECT COUNT(DISTINCT a), SUM(DISTINCT b), AVG(DISTINCT c), COUNT(*) FROM t GROUP BY d")
    assert [(a.function, a.column) for a in q.aggregations] == [("DISTINCTCOUNT", "a"), ("DISTINCTSUM", "b"),
                                                               ("DISTINCTAVG", "c"), ("COUNT", None)]
    with pytest.raises(ValueError):
        parse_sql("SELECT MAX(DISTINCT a) FROM t")
