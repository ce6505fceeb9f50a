"""Server execution statistics (the DataTable metadata the broker sums: numDocsScanned, numEntriesScannedInFilter,
numEntriesScannedPostFilter, numTotalDocs), restated from the reference's operators.

numEntriesScannedInFilter is the number of forward-index entries the reference's filter operators read. The GPU
evaluates every predicate on every doc (whole staged tiles), so the count is NOT a property of the GPU scan: it
follows the reference's operator tree and iterator protocol, which depend on each predicate's matching docs and on
the segment's indexes (sorted column, inverted index, range index). This module rebuilds that tree per segment
(FilterOperatorUtils.java:74-265: leaf operator choice, AND/OR simplification, AND child priorities) and drives the
reference's iterators over per-leaf doc bitmaps that the GPU computes (pa_query_leaf_bitmaps):
  * SVScanDocIdIterator.java:76-142 — next() reads 256-doc batches, advance(t) reads doc by doc from t to the next
    match, applyAnd(ids) reads every candidate doc; MVScanDocIdIterator.java:61-110 reads every value of a doc;
  * AndDocIdSet.java:72-186 — index-based iterators merged into one bitmap, scan iterators applied to it in order
    (applyAnd), the rest leap-frogged by AndDocIdIterator.java:39-73 (advance);
  * OrDocIdSet.java:63-127 (bitmap-based children are not collected into the merged bitmap: only sorted ones are),
    OrDocIdIterator.java:50-109; NotDocIdIterator.java:36-66 (NOT = NotDocIdSet over the child's doc set:
    BaseFilterOperator.getFalses, AndFilterOperator/OrFilterOperator.getFalses);
  * the projection drives the top iterator with next() until EOF (DocIdSetOperator), except for the plans that never
    iterate the filter (NonScanBasedAggregationOperator, FastFilteredCountOperator: AggregationPlanNode.java:97-115).
numEntriesScannedPostFilter = numDocsScanned x projected columns (ProjectionOperator: the group-by and aggregation
argument columns), 0 for the non-scan plans.

The executor hands this module the filter after the reference's compile-time rewrites (optimizer.py: AND/OR
flattening, merged ranges and IN lists, constant predicates, numeric literals against the column type), so the
operator tree is the one the reference's FilterPlanNode builds. Parity is pinned by the reference's golden statistics
(InterSegmentAggregationSingleValueQueriesTest, InterSegmentGroupBySingleValueQueriesTest: tests/golden/sv_queries.json)
and its rewrite fixtures (QueryOptimizerTest: tests/golden/query_optimizer.json)."""
import ctypes

import numpy as np

from . import _lib as L
from . import query as Q
from .predicate import DictLeaf, dictionary_leaf

EOF = -1
BATCH = 256  # BlockDocIdIterator.OPTIMAL_ITERATOR_BATCH_SIZE

HIGH, MEDIUM, LOW, AND_P, OR_P, SCAN_P = 0, 100, 200, 300, 400, 500  # PrioritizedFilterOperator


# ------------------------------------------------------------------ iterators (BlockDocIdIterator)
class _DocsIt:
    """Index-based iterators over a sorted doc list: SortedDocIdIterator, BitmapDocIdIterator,
    RangelessBitmapDocIdIterator (no entries scanned)."""

    def __init__(self, docs, kind):
        self.docs = docs
        self.kind = kind  # "sorted" | "bitmap"
        self.i = 0

    def next(self):
        if self.i < len(self.docs):
            self.i += 1
            return int(self.docs[self.i - 1])
        return EOF

    def advance(self, target):
        j = int(np.searchsorted(self.docs, target))
        if j < len(self.docs):
            self.i = j + 1
            return int(self.docs[j])
        self.i = len(self.docs)
        return EOF


class _MatchAllIt:
    def __init__(self, n):
        self.n, self.nxt = n, 0

    def next(self):
        if self.nxt < self.n:
            self.nxt += 1
            return self.nxt - 1
        return EOF

    def advance(self, target):
        self.nxt = target
        return self.next()


class _EmptyIt:
    def next(self):
        return EOF

    def advance(self, target):
        return EOF


class _ScanIt:
    """SVScanDocIdIterator (weights None) / MVScanDocIdIterator (weights = values per doc)."""

    def __init__(self, match, weights=None):
        self.match = match
        self.pos = np.flatnonzero(match)
        self.n = len(match)
        self.cum = None if weights is None else np.concatenate([[0], np.cumsum(weights, dtype=np.int64)])
        self.nxt = 0
        self.entries = 0
        self.batch = np.empty(0, dtype=np.int64)
        self.cursor = 0

    def _read(self, a, b):  # docs [a, b) read from the forward index
        self.entries += (b - a) if self.cum is None else int(self.cum[b] - self.cum[a])

    def _scan_from(self, start):
        j = int(np.searchsorted(self.pos, start))
        if j < len(self.pos):
            x = int(self.pos[j])
            self._read(start, x + 1)
            self.nxt = x + 1
            return x
        if start < self.n:
            self._read(start, self.n)
        self.nxt = max(start, self.n)
        return EOF

    def next(self):
        if self.cum is not None:  # MV: doc by doc
            return self._scan_from(self.nxt)
        if self.cursor >= len(self.batch):
            while True:
                limit = min(self.n - self.nxt, BATCH)
                if limit <= 0:
                    self.batch = np.empty(0, dtype=np.int64)
                    self.cursor = 0
                    return EOF
                b = np.arange(self.nxt, self.nxt + limit)
                self.batch = b[self.match[b]]
                self.nxt += limit
                self._read(0, limit)
                if len(self.batch):
                    break
            self.cursor = 0
        self.cursor += 1
        return int(self.batch[self.cursor - 1])

    def advance(self, target):
        self.batch = np.empty(0, dtype=np.int64)  # _firstMismatch = 0
        self.cursor = 0
        return self._scan_from(target)

    def apply_and(self, docs):
        if self.cum is None:
            self.entries += len(docs)
        else:
            self.entries += int((self.cum[docs + 1] - self.cum[docs]).sum())
        return docs[self.match[docs]]


class _AndIt:
    def __init__(self, its):
        self.its, self.nxt = its, 0

    def next(self):
        mx, mi, idx = self.nxt, -1, 0
        while idx < len(self.its):
            if idx == mi:
                idx += 1
                continue
            d = self.its[idx].advance(mx)
            if d == EOF:
                return EOF
            if d == mx:
                idx += 1
            else:
                mx, mi, idx = d, idx, 0
        self.nxt = mx + 1
        return mx

    def advance(self, target):
        self.nxt = target
        return self.next()


class _OrIt:
    def __init__(self, its):
        self.its = list(its)
        self.nd = [-1] * len(its)
        self.prev = -1

    def _finish(self, best):
        keep = [i for i, d in enumerate(self.nd) if d != EOF]
        self.its = [self.its[i] for i in keep]
        self.nd = [self.nd[i] for i in keep]
        if best is None:
            return EOF
        self.prev = best
        return best

    def next(self):
        best = None
        for i, it in enumerate(self.its):
            d = self.nd[i]
            if d == self.prev:
                d = it.next()
                self.nd[i] = d
                if d == EOF:
                    continue
            best = d if best is None else min(best, d)
        return self._finish(best)

    def advance(self, target):
        best = None
        for i, it in enumerate(self.its):
            d = self.nd[i]
            if d < target:
                d = it.advance(target)
                self.nd[i] = d
                if d == EOF:
                    continue
            best = d if best is None else min(best, d)
        return self._finish(best)


class _NotIt:
    def __init__(self, child, n):
        self.child, self.n, self.nxt = child, n, 0
        c = child.next()
        self.nnm = n if c == EOF else c

    def next(self):
        while self.nxt == self.nnm:
            self.nxt += 1
            c = self.child.next()
            self.nnm = self.n if c == EOF else c
        if self.nxt >= self.n:
            return EOF
        self.nxt += 1
        return self.nxt - 1

    def advance(self, target):
        self.nxt = target
        if target > self.nnm:
            c = self.child.advance(target)
            self.nnm = self.n if c == EOF else c
        return self.next()


# ------------------------------------------------------------------ filter operators (FilterOperatorUtils)
class _Op:
    def __init__(self, kind, prio=0, mask=None, children=(), weights=None):
        self.kind = kind  # empty | all | sorted | bitmap | scan | and | or | not
        self.prio = prio
        self.mask = mask
        self.children = list(children)
        self.weights = weights


def _flatten(f):
    """FlattenAndOrFilterOptimizer: AND(AND(a, b), c) -> AND(a, b, c) (and the same for OR)."""
    if isinstance(f, (Q.And, Q.Or)):
        kids = []
        for c in f.children:
            c = _flatten(c)
            if type(c) is type(f):
                kids.extend(c.children)
            else:
                kids.append(c)
        return type(f)(tuple(kids))
    if isinstance(f, Q.Not):
        return Q.Not(_flatten(f.child))
    return f


def _count_leaves(f):
    if isinstance(f, (Q.And, Q.Or)):
        return sum(_count_leaves(c) for c in f.children)
    if isinstance(f, Q.Not):
        return _count_leaves(f.child)
    return 1


def _eval(f, bitmaps, start):
    """Doc mask of an expanded (engine-side) predicate subtree over its leaves' bitmaps [start, ...)."""
    if isinstance(f, (Q.And, Q.Or)):
        out, k = None, start
        for c in f.children:
            m = _eval(c, bitmaps, k)
            k += _count_leaves(c)
            out = m if out is None else (out & m if isinstance(f, Q.And) else out | m)
        return out
    if isinstance(f, Q.Not):
        return ~_eval(f.child, bitmaps, start)
    return bitmaps[start]


class _LeafCursor:
    """Walks the reference's predicates in the engine's leaf order (one leaf per predicate: a raw IN / NOT IN is one
    RAW_SET leaf)."""

    def __init__(self, bitmaps, segment):
        self.bitmaps, self.segment, self.k = bitmaps, segment, 0

    def take(self, pred):
        m = self.bitmaps[self.k]
        self.k += 1
        return m

    def param(self):
        return None


def _leaf_op(pred, seg, mask, index_info, lf=None):
    """FilterOperatorUtils.getLeafFilterOperator (no null handling). lf: the leaf's dictionary_leaf when the caller
    has it already (the executor's bound leaf parameters)."""
    col = seg.column(pred.column)
    sv = col.single_value
    if isinstance(pred, Q.RegexpLikePredicate):
        # DictionaryBasedRegexpLikePredicateEvaluator never sets _alwaysTrue / _alwaysFalse, and without an FST index
        # FilterOperatorUtils.java:108-117 picks the scan whatever the column's sorted / inverted index
        weights = None if sv else col.mv_lengths(seg.num_docs)
        op = _Op("scan", SCAN_P + (0 if sv else 50), mask, weights=weights)
        op.column = pred.column
        return op
    if col.has_dictionary:
        # dictionary-based predicate evaluators: always false with no matching dictId, always true with all of them
        if lf is None:
            lf = dictionary_leaf(pred, col)
        n = (lf.hi - lf.lo) if lf.ids is None else len(np.unique(lf.ids))
        n = max(0, n)
        if lf.negate:
            n = col.cardinality - n
        if n == 0:
            return _Op("empty")
        if n == col.cardinality:
            return _Op("all")
    sorted_col = col.has_dictionary and sv and bool(col.is_sorted)
    inverted, ranged, exact = index_info(pred.column)
    if sorted_col:
        return _Op("sorted", HIGH, mask)
    if isinstance(pred, Q.RangePredicate):
        if ranged:
            if not exact:  # RangeIndexBasedFilterOperator scans the index's partial matches (bucket bounds of a v1
                # index): not restated
                raise _Unsupported("RANGE predicate on an inexact (v1) range index")
            return _Op("bitmap", LOW, mask)
    elif inverted:
        return _Op("bitmap", MEDIUM, mask)
    elif ranged and exact and isinstance(pred, Q.EqPredicate):
        # RangeIndexBasedFilterOperator.canEvaluate: EQ on an exact range index (the bit-sliced v2 index every
        # segment here is taken to have; FilterOperatorUtils.java:127-130)
        return _Op("bitmap", LOW, mask)
    weights = None if sv else col.mv_lengths(seg.num_docs)
    op = _Op("scan", SCAN_P + (0 if sv else 50), mask, weights=weights)
    op.column = pred.column
    return op


def _build(f, seg, cursor, index_info):
    if isinstance(f, Q.And):
        kids = [_build(c, seg, cursor, index_info) for c in f.children]
        if any(k.kind == "empty" for k in kids):
            return _Op("empty")
        kids = [k for k in kids if k.kind != "all"]
        if not kids:
            return _Op("all")
        if len(kids) == 1:
            return kids[0]
        kids.sort(key=lambda k: k.prio)  # reorderAndFilterChildOperators (stable)
        return _Op("and", AND_P, children=kids)
    if isinstance(f, Q.Or):
        kids = [_build(c, seg, cursor, index_info) for c in f.children]
        if any(k.kind == "all" for k in kids):
            return _Op("all")
        kids = [k for k in kids if k.kind != "empty"]
        if not kids:
            return _Op("empty")
        if len(kids) == 1:
            return kids[0]
        return _Op("or", OR_P, children=kids)
    if isinstance(f, Q.Not):
        c = _build(f.child, seg, cursor, index_info)
        if c.kind == "all":
            return _Op("empty")
        if c.kind == "empty":
            return _Op("all")
        return _Op("not", c.prio, children=[c])
    mask = cursor.take(f)
    return _leaf_op(f, seg, mask, index_info, cursor.param())


def _iterator(op, n, scans):
    """BlockDocIdSet.iterator() of the operator's doc set; every scan iterator is appended to `scans`."""
    if op.kind == "empty":
        return _EmptyIt()
    if op.kind == "all":
        return _MatchAllIt(n)
    if op.kind in ("sorted", "bitmap"):
        return _DocsIt(np.flatnonzero(op.mask), op.kind)
    if op.kind == "scan":
        it = _ScanIt(op.mask, op.weights)
        scans.append(it)
        return it
    if op.kind == "not":
        return _NotIt(_iterator(op.children[0], n, scans), n)
    its = [_iterator(c, n, scans) for c in op.children]
    if op.kind == "or":
        sorted_its = [i for i in its if isinstance(i, _DocsIt) and i.kind == "sorted"]
        if len(sorted_its) > 1:  # (bitmap-based children are not collected: OrDocIdSet.java:79-80)
            docs = np.unique(np.concatenate([i.docs for i in sorted_its]))
            rest = [i for i in its if not isinstance(i, _DocsIt)]
            merged = _DocsIt(docs, "bitmap")
            return merged if not rest else _OrIt([merged] + rest)
        return _OrIt(its)
    # AND
    sorted_its = [i for i in its if isinstance(i, _DocsIt) and i.kind == "sorted"]
    bitmap_its = [i for i in its if isinstance(i, _DocsIt) and i.kind == "bitmap"]
    scan_its = [i for i in its if isinstance(i, _ScanIt)]
    rest = [i for i in its if not isinstance(i, (_DocsIt, _ScanIt))]
    bitmap_its.sort(key=lambda i: len(i.docs))
    n_index = len(sorted_its) + len(bitmap_its)
    if (n_index > 0 and scan_its) or n_index > 1:
        docs = None
        for i in sorted_its + bitmap_its:
            docs = i.docs if docs is None else np.intersect1d(docs, i.docs, assume_unique=True)
        for s in scan_its:
            docs = s.apply_and(docs)
        merged = _DocsIt(docs, "bitmap")
        return merged if not rest else _AndIt([merged] + rest)
    return _AndIt(its)


def segment_index_info(segment):
    """index_info callback from the segment's column metadata: (inverted index, range index, range index exact)."""
    return lambda name: (bool(getattr(segment.column(name), "inverted_index", False)),
                         bool(getattr(segment.column(name), "range_index", False)),
                         bool(getattr(segment.column(name), "range_index_exact", True)))


def entries_scanned_in_filter(filt, segment, bitmaps, index_info=None):
    """numEntriesScannedInFilter of one segment when the projection iterates the filter to the end.
    filt: the query's filter tree (None = no filter); bitmaps: bool[leaves, num_docs] in the engine's leaf order
    (the engine's flattening); index_info(column) -> (inverted index, range index, range index
    exact)."""
    if filt is None:
        return 0
    index_info = index_info or segment_index_info(segment)
    op = _build(_flatten(filt), segment, _LeafCursor(bitmaps, segment), index_info)
    scans = []
    it = _iterator(op, segment.num_docs, scans)
    if op.kind in ("empty", "all"):
        return 0
    while it.next() != EOF:
        pass
    return sum(s.entries for s in scans)


def filter_mask(filt, segment, bitmaps):
    """The filter's doc mask of one segment from the leaf bitmaps (numDocsScanned per segment)."""
    return _eval(filt, bitmaps, 0)


def filter_is_match_all(filt, segment, bitmaps, index_info=None):
    if filt is None:
        return True
    index_info = index_info or segment_index_info(segment)
    return _build(_flatten(filt), segment, _LeafCursor(bitmaps, segment), index_info).kind == "all"


# AggregationPlanNode.java:49-53
DICTIONARY_BASED = {"MIN", "MINMV", "MAX", "MAXMV", "MINMAXRANGE", "MINMAXRANGEMV", "DISTINCTCOUNT", "DISTINCTCOUNTMV",
                    "DISTINCTCOUNTHLL", "DISTINCTCOUNTHLLMV", "DISTINCTCOUNTRAWHLL", "DISTINCTCOUNTRAWHLLMV", "DISTINCTSUM", "DISTINCTAVG", "DISTINCTSUMMV",
                    "DISTINCTAVGMV"}
METADATA_BASED = {"COUNT", "MIN", "MINMV", "MAX", "MAXMV", "MINMAXRANGE", "MINMAXRANGEMV"}


def non_scan_plan(query, segment, match_all):
    """AggregationPlanNode.isFitForNonScanBasedPlan with a match-all filter: every aggregation answered from the
    dictionary or the column metadata (the filter is never iterated and no column is projected)."""
    if query.group_by or not match_all:
        return False
    for a in query.aggregations:
        if a.function == "COUNT":
            continue
        col = segment.column(a.column)
        if a.function in DICTIONARY_BASED and col.has_dictionary:
            continue
        if a.function in METADATA_BASED and col.is_numeric:  # (min/max values are in the segment metadata)
            continue
        return False
    return True


def projected_columns(query):
    """Columns the ProjectionOperator reads: group-by columns and aggregation arguments (COUNT(*) reads none)."""
    cols = list(query.group_by)
    for a in query.aggregations:
        if a.column is not None and a.column not in cols:
            cols.append(a.column)
    return len(cols)


def server_stats(query, segments, leaf_bitmaps):
    """(numEntriesScannedInFilter, numEntriesScannedPostFilter) of one server's segments. leaf_bitmaps(i) -> bool[leaves,
    num_docs] of segment i in the engine's leaf order (GpuQueryExecutor.leaf_bitmaps)."""
    ncols = projected_columns(query)
    in_filter = post = 0
    for si, seg in enumerate(segments):
        bitmaps = leaf_bitmaps(si) if query.filter is not None else None
        if non_scan_plan(query, seg, filter_is_match_all(query.filter, seg, bitmaps)):
            continue  # NonScanBasedAggregationOperator: neither the filter nor a column is read
        in_filter += entries_scanned_in_filter(query.filter, seg, bitmaps)
        docs = seg.num_docs if query.filter is None else int(filter_mask(query.filter, seg, bitmaps).sum())
        post += docs * ncols
    return in_filter, post


# ------------------------------------------------------------------ device path: pa_query_execution_stats
# The replay above is O(matching docs) on the host. The library counts the same entries on the GPU from the operator
# trees this host builds (pa_query_execution_stats: constants for scans driven to EOF, popcounts of AndDocIdSet's
# applyAnd chains, AndDocIdIterator leap-frogs simulated per 2048-doc chunk and chained per segment, NotDocIdIterator's
# re-run of a leap-frog's last chain; pa_stats.hip). The replay stays for the shapes outside that engine: a NOT child of
# a leap-frogging AND (NotDocIdIterator mixes next() batches and advance() on its child), an AND or NOT child of an OR
# child of one, a NOT over a leap-frog with an OR child (the re-run after the end starts from the OR children's cached
# answers), and inexact (v1) range indexes.
class _Unsupported(Exception):
    pass


def _rpn(f, start):
    """Postfix program (pa_bitmap_counts tokens) of an expanded predicate subtree over the leaves [start, ...)."""
    if isinstance(f, (Q.And, Q.Or)):
        out, k = [], start
        for i, c in enumerate(f.children):
            out += _rpn(c, k)
            k += _count_leaves(c)
            if i:
                out.append(L.PA_BIT_AND if isinstance(f, Q.And) else L.PA_BIT_OR)
        return out
    if isinstance(f, Q.Not):
        return _rpn(f.child, start) + [L.PA_BIT_NOT]
    return [start]


class _RpnCursor(_LeafCursor):
    """_LeafCursor whose masks are postfix programs instead of host bitmaps."""

    def __init__(self, segment, params=None):
        super().__init__(None, segment)
        self.params, self.last = params, None

    def take(self, pred):
        p = [self.k]
        self.last = self.k
        self.k += 1
        return p

    def param(self):
        """The bound leaf parameters of the last single-leaf predicate (DictLeaf for a dictionary column)."""
        if self.params is None or self.last is None:
            return None
        lf = self.params[self.last]
        return lf if isinstance(lf, DictLeaf) else None


def _filter_columns(f):
    if isinstance(f, (Q.And, Q.Or)):
        return set().union(*[_filter_columns(c) for c in f.children])
    if isinstance(f, Q.Not):
        return _filter_columns(f.child)
    return {f.column}


def _tree_signature(seg, fcols, params):
    """Everything _build reads from a segment (the bound leaf parameters, each filter column's dictionary size,
    sortedness, indexes and single-/multi-value), or None when the tree must be built per segment (no bound
    parameters). Segments with equal signatures share one operator tree, so this key must list EVERY segment attribute
    _build / _leaf_op read (index_info included): a new per-segment input of the leaf operator choice goes here too, or
    trees leak across segments."""
    if params is None:
        return None
    cols = []
    for name in fcols:
        c = seg.column(name)
        cols.append((bool(c.single_value), c.has_dictionary, c.cardinality if c.has_dictionary else 0,
                     bool(c.is_sorted), bool(getattr(c, "inverted_index", False)),
                     bool(getattr(c, "range_index", False)), bool(getattr(c, "range_index_exact", True))))
    leaves = tuple((p.kind, p.lo, p.hi, bool(p.negate), None if p.ids is None else len(np.unique(p.ids)))
                   if isinstance(p, DictLeaf) else None for p in params)
    return leaves, tuple(cols)


OP_WORDS = 4 + L.PA_BIT_PROG_MAX  # int32 words of one pa_filter_op
_FOP = {"empty": L.PA_FOP_EMPTY, "all": L.PA_FOP_MATCH_ALL, "sorted": L.PA_FOP_SORTED, "bitmap": L.PA_FOP_BITMAP,
        "scan": L.PA_FOP_SCAN, "and": L.PA_FOP_AND, "or": L.PA_FOP_OR, "not": L.PA_FOP_NOT}


def _encode(op, rows, column_ids):
    """op in pre-order as pa_filter_op rows (int32[OP_WORDS] each)."""
    r = np.zeros(OP_WORDS, dtype=np.int32)
    r[0] = _FOP[op.kind]
    r[1] = len(op.children)
    r[2] = -1
    if op.kind == "scan" and op.weights is not None:
        r[2] = column_ids[op.column]
    if op.kind in ("sorted", "bitmap", "scan"):
        if len(op.mask) > L.PA_BIT_PROG_MAX:
            raise _Unsupported("doc-set program too long")
        r[3] = len(op.mask)
        r[4:4 + len(op.mask)] = op.mask
    rows.append(r)
    for c in op.children:
        _encode(c, rows, column_ids)


def operator_trees(query, segments, leaf_params=None, column_ids=None):
    """The reference's filter operator tree of every segment (FilterPlanNode + FilterOperatorUtils: _build), encoded for
    pa_query_execution_stats: (ops int32[num_ops, OP_WORDS], tree_root int32[trees], segment_tree int32[segments]) —
    segment_tree[i] a tree index, PA_STATS_NON_SCAN (AggregationPlanNode's non-scan plans) or PA_STATS_HOST (a leaf the
    engine cannot express: the host replays that segment). Segments with equal trees share one."""
    filt = query.filter
    flat = _flatten(filt) if filt is not None else None
    fcols = sorted(_filter_columns(filt)) if filt is not None else []
    rows, roots, seg_tree = [], [], []
    by_bytes, by_sig = {}, {}

    def add(op):
        enc = []
        _encode(op, enc, column_ids or {})
        key = np.stack(enc).tobytes()
        if key not in by_bytes:
            by_bytes[key] = len(roots)
            roots.append(len(rows))
            rows.extend(enc)
        return by_bytes[key]

    for si, seg in enumerate(segments):
        try:
            if filt is None:
                seg_tree.append(L.PA_STATS_NON_SCAN if non_scan_plan(query, seg, True) else add(_Op("all")))
                continue
            params = None if leaf_params is None else leaf_params[si]
            sig = _tree_signature(seg, fcols, params)
            # the tree (and its encoded index) is shared per filter signature; the non-scan plan choice is made per
            # segment, as AggregationPlanNode.isFitForNonScanBasedPlan is per IndexSegment (it reads the aggregation
            # columns, which the signature does not cover)
            entry = by_sig.get(sig) if sig is not None else None
            if entry is None:
                entry = [_build(flat, seg, _RpnCursor(seg, params), segment_index_info(seg)), None]
                if sig is not None:
                    by_sig[sig] = entry
            if non_scan_plan(query, seg, entry[0].kind == "all"):
                seg_tree.append(L.PA_STATS_NON_SCAN)
                continue
            if entry[1] is None:
                entry[1] = add(entry[0])
            seg_tree.append(entry[1])
        except _Unsupported:
            seg_tree.append(L.PA_STATS_HOST)
    ops = np.stack(rows) if rows else np.zeros((1, OP_WORDS), dtype=np.int32)
    return (np.ascontiguousarray(ops, dtype=np.int32), np.asarray(roots, dtype=np.int32),
            np.asarray(seg_tree, dtype=np.int32))
