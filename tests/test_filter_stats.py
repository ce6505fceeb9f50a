"""DataTable execution statistics (pinot_amd/filter_stats.py): the reference's filter-operator accounting restated
over per-leaf doc bitmaps, checked against the statistics the reference's own tests assert
(QueriesTestUtils.testInterSegmentsResult in InterSegmentAggregationSingleValueQueriesTest /
InterSegmentGroupBySingleValueQueriesTest: numDocsScanned, numEntriesScannedInFilter, numEntriesScannedPostFilter,
numTotalDocs; tests/golden/sv_queries.json). Here the leaf bitmaps come from a numpy evaluation of each leaf on the
golden segment (test-side); the -m gpu golden test takes them from the GPU (pa_query_leaf_bitmaps)."""
import numpy as np
import pytest

import oracle
from pinot_amd import _lib as L
from pinot_amd import filter_stats as FS
from pinot_amd import parse_sql
from pinot_amd import predicate as P
from pinot_amd import query as Q
from pinot_amd.engine import _flatten_filter


def leaf_masks(query, seg):
    """bool[leaves, docs] in the engine's leaf order (expand_raw_in + postfix flattening), evaluated with numpy."""
    if query.filter is None:
        return None
    leaves, ops = [], []
    _flatten_filter(P.expand_raw_in(query.filter, seg), leaves, ops)
    out = np.zeros((len(leaves), seg.num_docs), dtype=bool)
    for i, pred in enumerate(leaves):
        col = seg.column(pred.column)
        assert col.has_dictionary and col.single_value
        ids = oracle.read_ints(col.fwd_bytes, seg.num_docs, col.num_bits)
        out[i] = oracle._dict_match(pred, col)[ids].astype(bool)
    return out


def golden_stats(case, seg, servers, per_server):
    q = parse_sql(case["sql"])
    segs = [seg] * per_server
    masks = leaf_masks(q, seg)
    in_f, post = FS.server_stats(q, segs, lambda si: masks)
    docs = oracle.run_query(q, segs).num_docs_scanned
    return [docs * servers, in_f * servers, post * servers, seg.num_docs * per_server * servers]


def test_golden_execution_statistics(golden_spec, golden_segment):
    """All four statistics of every golden case (51 queries: aggregation-only and group-by, with and without the
    reference's FILTER, whose numEntriesScannedInFilter 252256 follows from the sorted daysSinceEpoch range, the
    applyAnd chain over column1/column3 and the AndDocIdIterator/OrDocIdIterator leap-frog of column6's scan)."""
    bad = []
    for case in golden_spec["cases"]:
        if case["stats"] is None:  # (testNumGroupsLimit asserts no statistics)
            continue
        got = golden_stats(case, golden_segment, golden_spec["servers"], golden_spec["segments_per_server"])
        if got != case["stats"]:
            bad.append((case["source"], case["sql"][:80], got, case["stats"]))
    assert not bad, bad


def _seg(n=5000, seed=3):
    from pinot_amd.segment import create_segment
    rng = np.random.default_rng(seed)
    data = {"s": np.sort(rng.integers(0, 50, n)).astype(np.int32), "a": rng.integers(0, 100, n).astype(np.int32),
            "b": rng.integers(0, 100, n).astype(np.int32), "c": rng.integers(0, 20, n).astype(np.int32)}
    return create_segment("x", data, {k: "INT" for k in data}, inverted_index_columns=("c",))


@pytest.mark.parametrize("where,expect", [
    # one scan leaf: the projection's next() reads every doc
    ("a < 50", lambda m, n: n),
    # index-only filters read nothing
    ("s = 7", lambda m, n: 0),
    ("c IN (1, 2, 3)", lambda m, n: 0),
    ("s = 7 AND c = 3", lambda m, n: 0),
    # sorted + scans: applyAnd over the sorted range, then over its survivors
    ("s BETWEEN 10 AND 20 AND a < 50 AND b > 30",
     lambda m, n: m["s"].sum() + (m["s"] & m["a"]).sum()),
    # inverted + scan
    ("c = 4 AND a >= 10", lambda m, n: m["c"].sum()),
    # scans only: AndDocIdIterator leap-frogs (first scan reads up to each candidate, the second from it)
    ("a < 30 AND b < 30", None),
    # always-true / always-false leaves fold away (dictionary evaluators)
    ("a < 1000 AND s = 7", lambda m, n: 0),
    ("a > 1000 OR c = 2", lambda m, n: 0),
])
def test_filter_accounting_shapes(where, expect):
    seg = _seg()
    q = parse_sql("SELECT COUNT(*) FROM t WHERE " + where)
    masks = leaf_masks(q, seg)
    got = FS.entries_scanned_in_filter(q.filter, seg, masks)
    if expect is None:
        # reference: AndDocIdIterator.next() -> a.advance(t) reads [t, next a-match], b.advance reads [t, next b-match]
        a = masks[0]
        b = masks[1]
        n = seg.num_docs
        exp, t = 0, 0
        ia, ib = np.flatnonzero(a), np.flatnonzero(b)
        na = nb = -1  # not used by the protocol (advance always re-reads from the target)
        while True:
            j = np.searchsorted(ia, t)
            if j == len(ia):
                exp += n - t
                break
            x = int(ia[j]); exp += x - t + 1; mx = x
            while True:
                k = np.searchsorted(ib, mx)
                if k == len(ib):
                    exp += n - mx
                    break
                y = int(ib[k]); exp += y - mx + 1
                if y == mx:
                    break
                j = np.searchsorted(ia, y)
                if j == len(ia):
                    exp += n - y
                    mx = None
                    break
                x = int(ia[j]); exp += x - y + 1; mx = x
                if x == y:
                    break
            if mx is None or k == len(ib):
                break
            t = mx + 1
        assert got == exp
    else:
        names = {}
        for li, pred in enumerate(_leaves(q, seg)):
            names[pred.column] = masks[li]
        assert got == expect(names, seg.num_docs)


def test_range_index_serves_eq_but_not_in():
    """FilterOperatorUtils.java:118-130 / RangeIndexBasedFilterOperator.canEvaluate: a range index answers RANGE and (exact
    index) EQ predicates — no entries scanned — while IN still scans; an inverted index takes precedence."""
    from pinot_amd.segment import create_segment
    rng = np.random.default_rng(9)
    n = 3000
    data = {"a": rng.integers(0, 100, n).astype(np.int32), "b": rng.integers(0, 100, n).astype(np.int32)}
    seg = create_segment("ri", data, {"a": "INT", "b": "INT"}, range_index_columns=("a",))
    for where, scanned in (("a = 5", 0), ("a BETWEEN 3 AND 9", 0), ("a IN (1, 2)", n), ("b = 5", n)):
        q = parse_sql("SELECT COUNT(*) FROM t WHERE " + where)
        assert FS.entries_scanned_in_filter(q.filter, seg, leaf_masks(q, seg)) == scanned, where


def _leaves(q, seg):
    leaves, ops = [], []
    _flatten_filter(P.expand_raw_in(q.filter, seg), leaves, ops)
    return leaves


def test_post_filter_rules(golden_segment):
    """numEntriesScannedPostFilter: 0 for the non-scan plans (metadata/dictionary aggregations on a match-all filter,
    COUNT(*)), docs x projected columns otherwise (AggregationPlanNode.java:97-115, ProjectionOperator)."""
    seg = golden_segment
    for sql, cols in [("SELECT MAX(column1), MIN(column3) FROM t", 0), ("SELECT COUNT(*) FROM t", 0),
                      ("SELECT SUM(column1) FROM t", 1), ("SELECT SUM(column1), MAX(column3) FROM t", 2),
                      ("SELECT column9, MAX(column1) FROM t GROUP BY column9", 2),
                      ("SELECT COUNT(*) FROM t WHERE column1 > 100000000", 0),
                      ("SELECT MAX(column1) FROM t WHERE column1 > 100", 0),  # always true: match-all, non-scan
                      ("SELECT MAX(column1) FROM t WHERE column1 > 100000000", 1)]:
        q = parse_sql(sql)
        masks = leaf_masks(q, seg)
        _, post = FS.server_stats(q, [seg], lambda si: masks)
        docs = seg.num_docs if q.filter is None else int(masks[0].sum())
        assert post == docs * cols, sql


# ---------------------------------------------------------------- closed forms (filter_stats.server_stats_closed_form)
def _np_prog(prog, masks, n):
    from pinot_amd import _lib as L
    st = []
    for t in prog:
        if t >= 0:
            st.append(masks[t].copy())
        elif t == L.PA_BIT_NOT:
            st[-1] = ~st[-1]
        else:
            y = st.pop()
            st[-1] = (st[-1] & y) if t == L.PA_BIT_AND else (st[-1] | y)
    assert len(st) == 1
    return st[0][:n]


def np_leaps(a, b):
    """pa_bitmap_counts' leap count, restated doc by doc (test-side)."""
    lab = a.astype(np.int64) + 2 * b.astype(np.int64)
    seq = lab[lab != 0]
    prev = np.concatenate([[3], seq[:-1]])
    return int(np.sum(((seq == 1) & (prev == 3)) | ((seq != 3) & (prev != 3) & (seq != prev))))


def np_counts(masks_of, segments):
    """counts_fn of server_stats_closed_form emulated with numpy over host leaf masks (test-side pa_bitmap_counts)."""
    def fn(reqs):
        out = np.zeros((len(reqs), 4), dtype=np.int64)
        for (si, a, b), r in reqs.items():
            m, n = masks_of(si), segments[si].num_docs
            A = _np_prog(a, m, n)
            B = _np_prog(b, m, n) if b else np.zeros(n, dtype=bool)
            out[r] = [A.sum(), B.sum(), (A & B).sum(), np_leaps(A, B) if b else 0]
        return out
    return fn


def test_leap_count_closed_form_matches_and_iterator():
    """num_docs + popcount(A & B) + leaps = the reads of AndDocIdIterator over two SVScanDocIdIterators, on random masks
    of many densities (including empty, full, a match at the last doc)."""
    rng = np.random.default_rng(5)
    for trial in range(300):
        n = int(rng.integers(1, 400))
        pa, pb = rng.random(2) ** 2
        a, b = rng.random(n) < pa, rng.random(n) < pb
        if trial % 7 == 0:
            a[-1] = b[-1] = True
        it = FS._AndIt([FS._ScanIt(a), FS._ScanIt(b)])
        while it.next() != FS.EOF:
            pass
        replay = it.its[0].entries + it.its[1].entries
        assert replay == n + int((a & b).sum()) + np_leaps(a, b), (trial, n)


CLOSED_FORM_WHERES = [
    "a < 30 AND b < 30", "a < 90 AND b >= 5", "a = 3 AND b = 4", "a < 50", "NOT a < 50", "a < 10 OR b < 10",
    "s BETWEEN 10 AND 20 AND a < 50 AND b > 30", "c = 4 AND a >= 10", "c IN (1, 2) AND s < 30 AND a < 60",
    "NOT (c = 3 AND a < 20)", "NOT (a < 10 OR b < 20)", "a IN (1, 5, 7) AND b NOT IN (3, 4)",
    "s = 7", "c IN (1, 2, 3)", "a < 1000 AND s = 7",
]
HOST_WHERES = ["a < 30 AND b < 30 AND c < 10 AND s > 3 AND a > 2", "a < 50 AND (b < 10 OR s = 3)",
               "(a < 10 OR b < 10) AND c = 3", "NOT (a < 10 AND b < 20)"]


@pytest.mark.parametrize("where", CLOSED_FORM_WHERES + HOST_WHERES)
def test_closed_form_matches_replay(where):
    """server_stats_closed_form (counts emulated with numpy) = server_stats (iterator replay), and the closed form is
    taken for every shape in CLOSED_FORM_WHERES (the replay is never asked for)."""
    segs = [_seg(3000, 3), _seg(4097, 4)]
    for sql in ("SELECT COUNT(*) FROM t WHERE " + where, "SELECT SUM(a), MAX(b) FROM t WHERE " + where,
                "SELECT c, SUM(a) FROM t WHERE %s GROUP BY c" % where):
        q = parse_sql(sql)
        masks = [leaf_masks(q, s) for s in segs]
        want = FS.server_stats(q, segs, lambda si: masks[si])

        def host(si):
            assert where in HOST_WHERES, "closed form expected for " + where
            return masks[si]
        got = FS.server_stats_closed_form(q, segs, np_counts(lambda si: masks[si], segs), host)
        assert got == want, sql
        # with the executor's bound leaf parameters: operator trees shared by segments of one signature
        params = [[P.dictionary_leaf(pred, s.column(pred.column)) for pred in _leaves(q, s)] for s in segs]
        got = FS.server_stats_closed_form(q, segs + segs, np_counts(lambda si: masks[si % 2], segs + segs),
                                          lambda si: host(si % 2), params + params)
        assert got == tuple(2 * x for x in want), sql


def test_closed_form_golden_statistics(golden_spec, golden_segment):
    """The golden statistics through the closed forms (numpy-emulated counts)."""
    bad = []
    for case in golden_spec["cases"]:
        if case["stats"] is None:
            continue
        q = parse_sql(case["sql"])
        segs = [golden_segment] * golden_spec["segments_per_server"]
        masks = leaf_masks(q, golden_segment)
        got = FS.server_stats_closed_form(q, segs, np_counts(lambda si: masks, segs), lambda si: masks)
        want = FS.server_stats(q, segs, lambda si: masks)
        if got != want:
            bad.append((case["sql"][:80], got, want))
    assert not bad, bad


def _word_leaps(a, b, prev):
    """pa_kernels.hip word_leaps restated on Python ints (32-bit words): (leaps, new prev)."""
    m = 0xFFFFFFFF
    l = a | b
    if l == 0:
        return 0, prev
    a1, b1, c, z = a & ~b & m, b & ~a & m, a & b, ~l & m
    after = lambda x: (z + ((x << 1) & m)) & m & l
    n = bin(a1 & after(c)).count("1") + bin(a1 & after(b1)).count("1") + bin(b1 & after(a1)).count("1")
    p0 = (l & -l).bit_length() - 1
    first = ((a >> p0) & 1) | (((b >> p0) & 1) << 1)
    n += 1 if (first == 1 and prev == 3) or (first != 3 and prev != 3 and first != prev) else 0
    p1 = l.bit_length() - 1
    return n, ((a >> p1) & 1) | (((b >> p1) & 1) << 1)


def test_constant_time_word_leaps_match_the_sequence_rule():
    """The count kernel's per-word bit-parallel leap count (carry trick) over random words and densities = the leap
    rule applied doc by doc (np_leaps), chained across words."""
    rng = np.random.default_rng(12)
    for _ in range(200):
        nw = int(rng.integers(1, 12))
        pa, pb = rng.random(2) ** 2
        a = rng.random(32 * nw) < pa
        b = rng.random(32 * nw) < pb
        wa = np.packbits(a, bitorder="little").view(np.uint32)
        wb = np.packbits(b, bitorder="little").view(np.uint32)
        prev, total = 3, 0
        for x, y in zip(wa.tolist(), wb.tolist()):
            n, prev = _word_leaps(x, y, prev)
            total += n
        assert total == np_leaps(a, b)


def test_operator_trees_not_shared_across_index_configurations():
    """segments with the same data and dictionaries but different indexes on a filter column (none, an
    exact range index, an inverted index, an inexact v1 range index) must not share an operator tree in the closed-form
    planner (_tree_signature lists every index attribute _leaf_op reads): each gets its own accounting, equal to its
    own replay. An EQ on an inexact range index scans (RangeIndexBasedFilterOperator.canEvaluate needs isExact)."""
    from pinot_amd.segment import create_segment
    rng = np.random.default_rng(21)
    n = 4000
    data = {"a": rng.integers(0, 60, n).astype(np.int32), "b": rng.integers(0, 100, n).astype(np.int32),
            "c": rng.integers(0, 7, n).astype(np.int32)}
    types = {"a": "INT", "b": "INT", "c": "INT"}
    segs = [create_segment("plain", data, types), create_segment("ranged", data, types, range_index_columns=("a",)),
            create_segment("inverted", data, types, inverted_index_columns=("a",)),
            create_segment("v1", data, types, range_index_columns=("a",))]
    segs[3].column("a").range_index_exact = False
    q = parse_sql("SELECT c, SUM(b) FROM t WHERE a = 5 AND b < 50 GROUP BY c")
    masks = [leaf_masks(q, s) for s in segs]
    params = [[P.dictionary_leaf(pred, s.column(pred.column)) for pred in _leaves(q, s)] for s in segs]
    got = FS.server_stats_closed_form(q, segs, np_counts(lambda si: masks[si], segs), lambda si: masks[si], params)
    assert got == FS.server_stats(q, segs, lambda si: masks[si])
    per = [FS.server_stats_closed_form(q, [s], np_counts(lambda si: masks[i], [s]), lambda si: masks[i], [params[i]])
           for i, s in enumerate(segs)]
    assert per[0] == per[3] != per[1] == per[2]  # scan vs index-served EQ


@pytest.mark.parametrize("where", ["a < 50", "NOT a < 50", "a < 10 OR b < 10", "s = 7", "c IN (1, 2, 3)",
                                   "NOT (a < 10 OR b < 20)"])
def test_constant_cost_filters_need_no_counts(where):
    """A filter whose entries are a constant (every scan driven to EOF reads all docs; index-served operators none):
    given the scan's numDocsScanned the closed form never asks for counts, so the statistics cost no pass over the
    filter columns (configs[0]'s day BETWEEN a AND b)."""
    segs = [_seg(3000, 3), _seg(4097, 4)]

    def boom(*_):
        raise AssertionError("counts requested for a constant-cost filter")
    for sql in ("SELECT COUNT(*), SUM(a) FROM t WHERE " + where, "SELECT c, SUM(a) FROM t WHERE %s GROUP BY c" % where):
        q = parse_sql(sql)
        masks = [leaf_masks(q, s) for s in segs]
        want = FS.server_stats(q, segs, lambda si: masks[si])
        docs = sum(int(FS.filter_mask(q.filter, s, masks[i]).sum()) for i, s in enumerate(segs))
        assert FS.server_stats_closed_form(q, segs, boom, boom, docs_total=docs) == want, sql


def test_fused_counts_serve_only_their_requests():
    """filter_stats.fused_counts: the AND request (A = [Z], B = [E]) and the whole-filter popcount come from the scan's
    per-segment counts; other requests and gave-up segments from the fallback."""
    AND = L.PA_BIT_AND
    arr = np.array([[10, 4, 0], [3, 1, 1]], dtype=np.int64)
    reqs = {(0, (1,), (0,)): 0, (0, (1, 0, AND), ()): 1, (1, (1,), (0,)): 2, (0, (0,), (1,)): 3}
    asked = []

    def fallback(rest):
        asked.append(sorted(rest))
        return np.array([[100 + r, 0, 0, 0] for r in range(len(rest))], dtype=np.int64)

    out = FS.fused_counts(reqs, (0, 1, arr), fallback)
    assert out[0].tolist() == [-1, -1, 10, 4]
    assert out[1].tolist() == [10, -1, -1, -1]
    assert asked == [sorted([(1, (1,), (0,)), (0, (0,), (1,))])]
    assert out[2][0] >= 100 and out[3][0] >= 100


def test_fused_linear_form_equals_the_closed_forms(monkeypatch):
    """server_stats_device's fast path (the statistics as linear forms of the scan's per-segment matched docs and
    leaps, _StatsPlan.fused_form) gives what fused_counts + the closed forms give; a gave-up segment leaves it for the
    general path (which asks the device counts for that segment)."""
    segs = [_seg(4000, 11), _seg(3000, 12), _seg(5000, 13)]
    q = parse_sql("SELECT COUNT(*), SUM(b) FROM t WHERE a < 20 AND b = 7")
    plan = FS.plan_stats(q, segs)
    reqs = plan.flat()[0]
    e, z = None, None
    for (si, a, b) in reqs:  # the two-leaf AND's request names the leaves: A = [Z], B = [E]
        if len(a) == 1 and len(b) == 1:
            z, e = a[0], b[0]
    assert e is not None
    rng = np.random.default_rng(5)
    arr = np.stack([rng.integers(0, 500, 3), rng.integers(0, 900, 3), np.zeros(3, dtype=np.int64)], axis=1)

    class Ex:
        handle = None

        def fused_leap_counts(self, stream=None):
            return e, z, arr

    def no_fallback(rq):
        raise AssertionError(rq)

    want = FS.server_stats_closed_form(q, segs, lambda rq: FS.fused_counts(rq, (e, z, arr), no_fallback), None, None,
                                       777, plan)
    assert plan.fused_form(e, z, len(segs)) is not None
    assert FS.server_stats_device(q, segs, Ex(), None, 777, plan) == want
    arr[1, 2] = 1  # segment 1 gave up
    asked = []
    monkeypatch.setattr(FS, "device_counts", lambda ex, sg, rq, st=None: asked.append(sorted(rq)) or
                        np.zeros((len(rq), 4), dtype=np.int64))
    FS.server_stats_device(q, segs, Ex(), None, 777, plan)
    assert asked and all(k[0] == 1 for k in asked[0])
