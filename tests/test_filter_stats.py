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
    """bool[leaves, docs] in the engine's leaf order (postfix flattening), evaluated with numpy."""
    if query.filter is None:
        return None
    leaves, ops = [], []
    _flatten_filter(query.filter, leaves, ops)
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
    _flatten_filter(q.filter, leaves, ops)
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


# ---------------------------------------------------------------- the GPU statistics engine (pa_query_execution_stats)
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
    # the shapes the host used to replay: leap-frogs of more than two scans, an AND with an OR child, an OR of scans
    # under an AND with an index leaf, NOT of a leap-frogging AND
    "a < 30 AND b < 30 AND c < 10 AND s > 3 AND a > 2", "a < 50 AND (b < 10 OR s = 3)",
    "(a < 10 OR b < 10) AND c = 3", "NOT (a < 10 AND b < 20)",
    "a < 60 AND b < 70 AND c < 12", "a < 50 AND (b < 10 OR c < 3)", "(a < 10 OR b < 10) AND (a > 50 OR c = 3)",
    "a < 50 AND (b < 10 OR (s = 3 AND a > 20))",
    "(a < 20 AND b < 30) OR (c = 2 AND a > 70) OR NOT (b < 50 AND a > 10)", "NOT (a < 95 AND b < 95 AND c < 19)",
]
# outside the engine (documented in filter_stats "device path"): the host replays these segments
# the shapes outside the reduction (a NOT child of a leap-frogging AND, an AND / NOT under an OR inside a leap-frog, a
# NOT over a leap-frog with an OR child): the GPU iterator replay counts them (stat_replay_kernel)
REPLAY_WHERES = ["a < 50 AND NOT (b < 10 OR c = 2)", "a < 50 AND (b < 10 OR NOT c = 3)",
                 "NOT (a < 10 AND (b < 20 OR c = 1))", "NOT a IN (3, 5) AND b < 9",
                 "a < 60 AND (c = 3 OR (a > 7 AND b > 70))", "NOT (b > 40) AND (a < 30 OR NOT c = 1)"]
HOST_WHERES = REPLAY_WHERES  # (former name)
# (the same lists, by name, for the GPU test)
ENGINE_WHERES = CLOSED_FORM_WHERES


def _model_stats(q, segs, masks, chunk, params=None, replayed=None):
    import stats_model as M
    ops, roots, seg_tree = FS.operator_trees(q, segs, params, {})
    msegs = [M.Seg(s.num_docs, masks[i]) for i, s in enumerate(segs)]
    docs = sum(int(FS.filter_mask(q.filter, s, masks[i]).sum()) if q.filter is not None else s.num_docs
               for i, s in enumerate(segs))
    return M.execution_stats(ops, roots, seg_tree, msegs, FS.projected_columns(q), docs, chunk, replayed)


@pytest.mark.parametrize("where", CLOSED_FORM_WHERES + REPLAY_WHERES)
def test_engine_model_matches_replay(where):
    """The statistics engine's algorithm (tests/stats_model.py: the operator-tree reduction of pa_stats_host.hip, the
    chunked leap-frog of pa_stats.hip, restated on the CPU with small chunks so the chunk boundaries and the chaining
    are exercised, and the GPU iterator replay of the shapes outside the reduction: the REPLAY_WHERES) = the host's
    iterator replay (filter_stats.server_stats), per segment; no segment is left to the host."""
    segs = [_seg(3000, 3), _seg(4097, 4), _seg(257, 5)]
    for sql in ("SELECT COUNT(*) FROM t WHERE " + where, "SELECT c, SUM(a) FROM t WHERE %s GROUP BY c" % where):
        q = parse_sql(sql)
        masks = [leaf_masks(q, s) for s in segs]
        want_per = [FS.server_stats(q, [s], lambda si, i=i: masks[i]) for i, s in enumerate(segs)]
        for chunk in (64, 5, 2048):
            replayed = []
            in_f, post, per = _model_stats(q, segs, masks, chunk, replayed=replayed)
            for i in range(len(segs)):
                assert per[i] >= 0, (sql, i)
                assert per[i] == want_per[i][0], (sql, chunk, i)
            assert post == sum(w[1] for w in want_per), sql
            assert bool(replayed) == (where in REPLAY_WHERES), (where, replayed)


def test_engine_model_golden_statistics(golden_spec, golden_segment):
    """The golden statistics' numEntriesScannedInFilter through the engine's algorithm (CPU model)."""
    bad = []
    for case in golden_spec["cases"]:
        if case["stats"] is None:
            continue
        q = parse_sql(case["sql"])
        segs = [golden_segment] * golden_spec["segments_per_server"]
        masks = leaf_masks(q, golden_segment)
        got = _model_stats(q, segs, [masks] * len(segs), 2048)
        want = FS.server_stats(q, segs, lambda si: masks)
        if (got[0], got[1]) != want or min(got[2]) < 0:
            bad.append((case["sql"][:80], got[:2], want))
    assert not bad, bad


def test_leapfrog_model_on_random_masks():
    """The chunked leap-frog (per chunk and entry state, chained) = AndDocIdIterator over the same iterators, for random
    masks of many densities, 2..5 children, scan / index / OR-of-scans children, and several chunk sizes."""
    import stats_model as M
    rng = np.random.default_rng(17)
    for trial in range(120):
        n = int(rng.integers(1, 700))
        k = int(rng.integers(2, 6))
        nleaf = k + 3
        leaves = rng.random((nleaf, n)) < (rng.random(nleaf) ** 2)[:, None]
        if trial % 5 == 0:
            leaves[:, -1] = True
        seg = M.Seg(n, leaves)
        el, its = [], []
        nxt = 0
        for j in range(k):
            kind = int(rng.integers(0, 3)) if j else 1
            if kind == 2:  # an OR of two scans and an index doc set
                subs = [(M.LF_SCAN, [nxt], -1), (M.LF_SCAN, [nxt + 1], -1), (M.LF_DOCS, [nxt + 2], -1)]
                prog = [nxt, nxt + 1, L.PA_BIT_OR, nxt + 2, L.PA_BIT_OR]
                el.append((M.LF_OR, prog, -1, subs))
                its.append(FS._OrIt([FS._ScanIt(leaves[nxt]), FS._ScanIt(leaves[nxt + 1]),
                                     FS._DocsIt(np.flatnonzero(leaves[nxt + 2]), "bitmap")]))
                nxt += 3
            else:
                el.append((M.LF_SCAN if kind == 1 else M.LF_DOCS, [nxt], -1, []))
                its.append(FS._ScanIt(leaves[nxt]) if kind == 1 else FS._DocsIt(np.flatnonzero(leaves[nxt]), "bitmap"))
                nxt += 1
            if nxt + 3 > nleaf:
                break
        if len(el) < 2:
            continue
        scans = []
        for it in its:
            if isinstance(it, FS._ScanIt):
                scans.append(it)
            elif isinstance(it, FS._OrIt):
                scans += [x for x in it.its if isinstance(x, FS._ScanIt)]
        ai = FS._AndIt(its)
        matches = 0
        while ai.next() != FS.EOF:
            matches += 1
        want = sum(x.entries for x in scans)
        for chunk in (3, 32, 64, 1000):
            got, _, m = M.leapfrog(el, False, seg, chunk)
            assert (got, m) == (want, matches), (trial, chunk)


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
    exact range index, an inverted index, an inexact v1 range index) must not share an operator tree
    (filter_stats._tree_signature lists every index attribute _leaf_op reads): each gets its own tree, and its
    accounting equals its own replay. An EQ on an inexact range index scans (RangeIndexBasedFilterOperator.canEvaluate
    needs isExact)."""
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
    ops, roots, seg_tree = FS.operator_trees(q, segs, params, {})
    assert seg_tree[0] == seg_tree[3] != seg_tree[1] == seg_tree[2]  # scan vs index-served EQ
    got = _model_stats(q, segs, masks, 64, params)
    assert (got[0], got[1]) == FS.server_stats(q, segs, lambda si: masks[si])
    per = [FS.server_stats(q, [s], lambda si, i=i: masks[i])[0] for i, s in enumerate(segs)]
    assert got[2] == per


@pytest.mark.parametrize("where", ["a < 50", "NOT a < 50", "a < 10 OR b < 10", "s = 7", "c IN (1, 2, 3)",
                                   "NOT (a < 10 OR b < 20)"])
def test_constant_cost_filters_need_no_gpu_pass(where):
    """A filter whose entries are a constant (every scan driven to EOF reads all docs; index-served operators none)
    reduces to a constant: no applyAnd count and no leap-frog, so the statistics cost no pass over the filter columns
    (configs[0]'s day BETWEEN a AND b)."""
    import stats_model as M
    segs = [_seg(3000, 3), _seg(4097, 4)]
    for sql in ("SELECT COUNT(*), SUM(a) FROM t WHERE " + where, "SELECT c, SUM(a) FROM t WHERE %s GROUP BY c" % where):
        q = parse_sql(sql)
        ops, roots, seg_tree = FS.operator_trees(q, segs, None, {})
        for si, s in enumerate(segs):
            counts, leaps = [], []
            v = M._cost_next(ops, int(roots[seg_tree[si]]), M.Seg(s.num_docs, leaf_masks(q, s)), counts, leaps, False)
            assert not counts and not leaps, sql
            assert v == FS.server_stats(q, [s], lambda _: leaf_masks(q, s))[0], sql


def test_operator_tree_encoding():
    """operator_trees: pre-order pa_filter_op rows (kind, children, multi-value column, program), AND children in the
    reference's priority order (sorted index, inverted index, scans), constant leaves folded, one tree per signature."""
    segs = [_seg(3000, 3), _seg(3000, 3)]
    q = parse_sql("SELECT COUNT(*) FROM t WHERE a < 50 AND (b < 10 OR c = 3) AND s = 7")
    ops, roots, seg_tree = FS.operator_trees(q, segs, None, {})
    assert list(seg_tree) == [0, 0] and list(roots) == [0]
    kinds = [int(r[0]) for r in ops]
    assert kinds[0] == L.PA_FOP_AND and ops[0][1] == 3
    # s = 7 on the sorted column first (HIGH), then the OR (OR_P 400), then the scan of a (SCAN_P 500)
    assert kinds[1] == L.PA_FOP_SORTED and kinds[2] == L.PA_FOP_OR and kinds[5] == L.PA_FOP_SCAN
    assert kinds[3:5] == [L.PA_FOP_SCAN, L.PA_FOP_BITMAP]
    assert all(r[2] == -1 for r in ops)
    for r in ops:
        if r[0] in (L.PA_FOP_SORTED, L.PA_FOP_BITMAP, L.PA_FOP_SCAN):
            assert r[3] == 1 and 0 <= r[4] < 4
    q = parse_sql("SELECT COUNT(*) FROM t WHERE a > 1000 OR c = 2")  # always-false leaf folds: one bitmap leaf
    ops, roots, seg_tree = FS.operator_trees(q, segs, None, {})
    assert [int(r[0]) for r in ops] == [L.PA_FOP_BITMAP]
    q = parse_sql("SELECT SUM(a) FROM t")  # no filter: a match-all tree (the projection reads every doc)
    ops, roots, seg_tree = FS.operator_trees(q, segs, None, {})
    assert [int(r[0]) for r in ops] == [L.PA_FOP_MATCH_ALL]
    q = parse_sql("SELECT MAX(a) FROM t")  # non-scan plan
    assert list(FS.operator_trees(q, segs, None, {})[2]) == [L.PA_STATS_NON_SCAN] * 2


def test_non_scan_plan_chosen_per_segment_with_shared_trees():
    """segments sharing a filter signature share one operator tree, but the non-scan plan is chosen per
    segment (AggregationPlanNode.isFitForNonScanBasedPlan reads each IndexSegment's aggregation columns): with the
    aggregated column dictionary-encoded in one segment and raw in the other, only the first takes the non-scan plan,
    and each segment's accounting equals its own replay."""
    from pinot_amd.segment import create_segment
    rng = np.random.default_rng(5)
    n = 3000
    data = {"a": rng.integers(0, 60, n).astype(np.int32), "b": rng.integers(0, 100, n).astype(np.int32)}
    types = {"a": "INT", "b": "INT"}
    segs = [create_segment("dict", data, types), create_segment("raw", data, types, no_dictionary_columns=("b",))]
    q = parse_sql("SELECT DISTINCTCOUNT(b) FROM t WHERE a < 1000")  # (a match-all filter: every a < 60)
    params = [[P.dictionary_leaf(pred, s.column(pred.column)) for pred in _leaves(q, s)] for s in segs]
    ops, roots, seg_tree = FS.operator_trees(q, segs, params, {})
    assert seg_tree[0] == L.PA_STATS_NON_SCAN and seg_tree[1] >= 0
    for order in (segs, segs[::-1]):  # (whichever segment builds the shared tree first)
        pr = [params[segs.index(s)] for s in order]
        st = FS.operator_trees(q, order, pr, {})[2]
        assert [t == L.PA_STATS_NON_SCAN for t in st] == [s.name == "dict" for s in order]
        for s, t in zip(order, st):
            masks = leaf_masks(q, s)
            exp = FS.server_stats(q, [s], lambda _: masks)
            assert (exp == (0, 0)) == (t == L.PA_STATS_NON_SCAN)
