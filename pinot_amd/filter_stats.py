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
from .predicate import DictLeaf, dictionary_leaf, expand_raw_in

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
    """Walks the reference's (unexpanded) predicates in the engine's leaf order: a raw IN / NOT IN became an OR of
    equality leaves on the GPU (predicate.expand_raw_in); its doc mask is rebuilt from those leaves."""

    def __init__(self, bitmaps, segment):
        self.bitmaps, self.segment, self.k = bitmaps, segment, 0

    def take(self, pred):
        sub = expand_raw_in(pred, self.segment)
        m = _eval(sub, self.bitmaps, self.k)
        self.k += _count_leaves(sub)
        return m

    def param(self):
        return None


def _leaf_op(pred, seg, mask, index_info, lf=None):
    """FilterOperatorUtils.getLeafFilterOperator (no null handling). lf: the leaf's dictionary_leaf when the caller
    has it already (the executor's bound leaf parameters)."""
    col = seg.column(pred.column)
    sv = col.single_value
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
    return _Op("scan", SCAN_P + (0 if sv else 50), mask, weights=weights)


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
    (predicate.expand_raw_in + the engine's flattening); index_info(column) -> (inverted index, range index, range index
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
    return _eval(expand_raw_in(filt, segment), bitmaps, 0)


def filter_is_match_all(filt, segment, bitmaps, index_info=None):
    if filt is None:
        return True
    index_info = index_info or segment_index_info(segment)
    return _build(_flatten(filt), segment, _LeafCursor(bitmaps, segment), index_info).kind == "all"


# AggregationPlanNode.java:49-53
DICTIONARY_BASED = {"MIN", "MINMV", "MAX", "MAXMV", "MINMAXRANGE", "MINMAXRANGEMV", "DISTINCTCOUNT", "DISTINCTCOUNTMV",
                    "DISTINCTCOUNTHLL", "DISTINCTCOUNTHLLMV", "DISTINCTSUM", "DISTINCTAVG", "DISTINCTSUMMV",
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


# ------------------------------------------------------------------ device path: closed forms over GPU counts
# The iterator replay above is O(matching docs) on the host. The projection's iteration has closed forms for the
# operator trees queries usually have, whose inputs are counts over the leaf bitmaps that the GPU computes without
# moving the bitmaps (pa_bitmap_counts):
#   * a scan iterator driven by next() to EOF reads every entry: num_docs (SV), the column's value count (MV);
#     OR / NOT children are driven by next() to EOF too, so their costs add (NOT calls its child's next() once past
#     EOF: free for every iterator but a leap-frogging AND);
#   * AND with index-based children (AndDocIdSet.java:92-140): each SV scan child's applyAnd reads the docs that survive
#     the index children and the scan children before it: popcounts of AND chains;
#   * AND of two SV scan iterators leap-frogged by AndDocIdIterator: every advance(t) reads [t, next match of the
#     advancing iterator], so the reads telescope to num_docs - matches + advance calls - 1, and the advance calls are
#     2 per match + 1 + the leaps (pa_bitmap_counts): num_docs + popcount(A & B) + leaps.
# Other shapes (an AND leap-frogging an OR / NOT / a third iterator, MV applyAnd) keep the host replay.
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
        sub = expand_raw_in(pred, self.segment)
        p = _rpn(sub, self.k)
        n = _count_leaves(sub)
        self.last = self.k if n == 1 else None
        self.k += n
        return p

    def param(self):
        """The bound leaf parameters of the last single-leaf predicate (DictLeaf for a dictionary column)."""
        if self.params is None or self.last is None:
            return None
        lf = self.params[self.last]
        return lf if isinstance(lf, DictLeaf) else None


def _and_prog(progs):
    out = list(progs[0])
    for p in progs[1:]:
        out += list(p) + [L.PA_BIT_AND]
    return out


class _Terms:
    """A count as constant + sum of coef * (request field); requests are (program A, program B) of one segment."""

    def __init__(self, const=0):
        self.const, self.terms = const, []

    def add(self, other):
        self.const += other.const
        self.terms += other.terms
        return self

    def request(self, reqs, si, a, b, field, coef=1):
        if len(a) > L.PA_BIT_PROG_MAX or len(b) > L.PA_BIT_PROG_MAX:
            raise _Unsupported("bitmap program too long")
        key = (si, tuple(a), tuple(b))
        if key not in reqs:
            reqs[key] = len(reqs)
        self.terms.append((reqs[key], field, coef))
        return self

    def value(self, counts):
        v = self.const
        for r, f, c in self.terms:
            x = int(counts[r, f])
            if x < 0:
                raise RuntimeError("internal: count field %d of request %d not computed" % (f, r))
            v += x * c
        return v


def _cost_next(op, seg, si, reqs):
    """numEntriesScannedInFilter of op's iterator driven by next() to EOF, as _Terms."""
    n = seg.num_docs
    if op.kind in ("empty", "all", "sorted", "bitmap"):
        return _Terms(0)
    if op.kind == "scan":
        return _Terms(n if op.weights is None else int(np.sum(op.weights, dtype=np.int64)))
    if op.kind == "not":
        c = op.children[0]
        if c.kind == "and" and not any(k.kind in ("sorted", "bitmap") for k in c.children):
            # NotDocIdIterator.next() calls its child's next() once more after EOF: an AndDocIdIterator re-runs its
            # last leap-frog chain then (no closed form kept for that tail)
            raise _Unsupported("NOT over a leap-frogging AND")
        return _cost_next(c, seg, si, reqs)
    if op.kind == "or":
        t = _Terms(0)
        for c in op.children:
            t.add(_cost_next(c, seg, si, reqs))
        return t
    # AND: the iterator construction of _iterator / AndDocIdSet
    kids = op.children
    index = [c for c in kids if c.kind == "sorted"] + [c for c in kids if c.kind == "bitmap"]
    scans = [c for c in kids if c.kind == "scan"]
    rest = [c for c in kids if c.kind not in ("sorted", "bitmap", "scan")]
    if (index and scans) or len(index) > 1:
        if rest:
            raise _Unsupported("AND leap-frogs a merged index set with other iterators")
        t = _Terms(0)
        docs = _and_prog([c.mask for c in index])
        for s in scans:
            if s.weights is not None:
                raise _Unsupported("MV applyAnd")
            t.request(reqs, si, docs, [], 0)
            docs = _and_prog([docs, s.mask])
        return t
    if len(kids) == 2 and all(c.kind == "scan" and c.weights is None for c in kids):
        return _Terms(n).request(reqs, si, kids[0].mask, kids[1].mask, 2).request(reqs, si, kids[0].mask,
                                                                                    kids[1].mask, 3)
    raise _Unsupported("AND leap-frogging other than two SV scans")


def _filter_columns(f):
    if isinstance(f, (Q.And, Q.Or)):
        return set().union(*[_filter_columns(c) for c in f.children])
    if isinstance(f, Q.Not):
        return _filter_columns(f.child)
    return {f.column}


def _tree_signature(seg, fcols, params):
    """Everything _build reads from a segment (the bound leaf parameters, each filter column's dictionary size,
    sortedness and indexes), or None when the tree must be built per segment (no bound parameters; MV columns, whose
    scan costs are per-doc value counts). Segments with equal signatures share one operator tree, so this key must list
    EVERY segment attribute _build / _leaf_op read (index_info included): a new per-segment input of the leaf operator
    choice goes here too, or trees leak across segments."""
    if params is None:
        return None
    cols = []
    for name in fcols:
        c = seg.column(name)
        if not c.single_value:
            return None
        cols.append((c.has_dictionary, c.cardinality if c.has_dictionary else 0, bool(c.is_sorted),
                     bool(getattr(c, "inverted_index", False)), bool(getattr(c, "range_index", False)),
                     bool(getattr(c, "range_index_exact", True))))
    leaves = tuple((p.kind, p.lo, p.hi, bool(p.negate), None if p.ids is None else len(np.unique(p.ids)))
                   if isinstance(p, DictLeaf) else None for p in params)
    return leaves, tuple(cols)


class _StatsPlan:
    """The per-segment operator trees of one query over one segment set, reduced to what the statistics need: per
    segment None (non-scan plan), "host" (replay) or (in-filter _Terms, docs program, constant docs _Terms), the
    requests of the in-filter terms, and — built on first use — the full request set with the docs requests and the
    terms as flat arrays (one numpy gather evaluates every segment). GpuQueryExecutor keeps it across executions of
    its prepared query (the trees depend on the query and the segments, not on a scan's results)."""

    def __init__(self, ncols, plans, reqs):
        self.ncols, self.plans, self.reqs = ncols, plans, reqs
        self.full = None
        self.fused_cache = {}  # fused_counts' classification of the full request set

    def constant_value(self):
        """in-filter entries when every segment's filter cost is a constant (no request at all), else None."""
        if self.reqs or not all(p is not None and p != "host" for p in self.plans):
            return None
        return sum(p[0].value(None) for p in self.plans)

    def flat(self):
        if self.full is None:
            reqs = dict(self.reqs)
            plans = list(self.plans)
            for si, p in enumerate(plans):
                if isinstance(p, tuple):
                    try:
                        plans[si] = (p[0], p[2] if p[1] is None else _Terms(0).request(reqs, si, p[1], [], 0))
                    except _Unsupported:
                        plans[si] = "host"
            const_in = const_docs = 0
            ti, td = [], []
            for p in plans:
                if p is None or p == "host":
                    continue
                const_in += p[0].const
                const_docs += p[1].const
                ti += p[0].terms
                td += p[1].terms
            arr = lambda t: (np.array([x[0] for x in t], dtype=np.int64), np.array([x[1] for x in t], dtype=np.int64),
                             np.array([x[2] for x in t], dtype=np.int64))
            host = [si for si, p in enumerate(plans) if p == "host"]
            self.full = (reqs, const_in, arr(ti), const_docs, arr(td), host)
        return self.full

    def fused_form(self, e, z, nseg):
        """The statistics as linear forms of the counts the scan took itself (fused_counts' per-segment matched docs m
        and leaps l): in_filter = const_in + A.m + B.l, post = (const_docs + C.m) x ncols — or None when some request
        is not one the scan covers (then fused_counts + the closed forms run). Cached per (E leaf, Z leaf)."""
        key = ("form", e, z)
        if key not in self.fused_cache:
            reqs, const_in, (ri, fi, ci), const_docs, (rd, fd, cd), host = self.flat()
            form = None
            if not host and self.reqs:  # (no request: a constant-cost filter, server_stats_closed_form's shortcut)
                row = {}  # request row -> (segment, kind): 0 the AND request, 1 the whole-filter request
                ok = True
                for (si, a, b), r in reqs.items():
                    if a == (z,) and b == (e,):
                        row[r] = (si, 0)
                    elif not b and a in ((z, e, L.PA_BIT_AND), (e, z, L.PA_BIT_AND)):
                        row[r] = (si, 1)
                    else:
                        ok = False
                A, B, C = (np.zeros(nseg, dtype=np.int64) for _ in range(3))
                for rows, fields, coef, dst in ((ri, fi, ci, "in"), (rd, fd, cd, "docs")):
                    for r, f, c in zip(rows.tolist(), fields.tolist(), coef.tolist()):
                        si, kind = row.get(r, (None, None))
                        if si is None:
                            ok = False
                        elif kind == 0 and f == 2:  # popcount(A & B) = the segment's matched docs
                            (A if dst == "in" else C)[si] += c
                        elif kind == 0 and f == 3 and dst == "in":  # leaps
                            B[si] += c
                        elif kind == 1 and f == 0:  # the whole filter's popcount = matched docs
                            (A if dst == "in" else C)[si] += c
                        else:
                            ok = False
                if ok:
                    form = (int(const_in), A, B, int(const_docs), C)
            self.fused_cache[key] = form
        return self.fused_cache[key]


def plan_stats(query, segments, leaf_params=None):
    """_StatsPlan of `query` over `segments` (server_stats_closed_form's planning half)."""
    ncols = projected_columns(query)
    filt = query.filter
    reqs = {}
    plans = []  # per segment: None (non-scan plan), "host", or (in_filter _Terms, docs program, constant docs _Terms)
    flat = _flatten(filt) if filt is not None else None
    fcols = sorted(_filter_columns(filt)) if filt is not None else []
    trees = {}  # operator tree + docs program per segment signature (segments of a table usually share one)
    for si, seg in enumerate(segments):
        if filt is None:
            plans.append(None if non_scan_plan(query, seg, True) else (_Terms(0), None, _Terms(seg.num_docs)))
            continue
        try:
            params = None if leaf_params is None else leaf_params[si]
            key = _tree_signature(seg, fcols, params)
            if key is None or key not in trees:
                tree = (_build(flat, seg, _RpnCursor(seg, params), segment_index_info(seg)),
                        _rpn(expand_raw_in(filt, seg), 0))
                if key is not None:
                    trees[key] = tree
            else:
                tree = trees[key]
            op, docs_prog = tree
            if non_scan_plan(query, seg, op.kind == "all"):
                plans.append(None)
                continue
            cost = _Terms(0) if op.kind in ("empty", "all") else _cost_next(op, seg, si, reqs)
            plans.append((cost, docs_prog, None))
        except _Unsupported:
            plans.append("host")
    return _StatsPlan(ncols, plans, reqs)


def server_stats_closed_form(query, segments, counts_fn, leaf_bitmaps, leaf_params=None, docs_total=None, plan=None):
    """server_stats through the closed forms above. counts_fn(reqs) -> int64[len(reqs), 4]: for every request
    (segment index, program A, program B) -> row, pa_bitmap_counts' four counts. Segments without a closed form replay
    the iterators over leaf_bitmaps(i) (host bitmaps, as server_stats). leaf_params[i]: segment i's bound leaf
    parameters in leaf order (GpuQueryExecutor.leaf_params), reused instead of re-matching the dictionaries.
    docs_total: the scan's numDocsScanned over these segments, if known. When every segment's filter cost is a constant
    (a scan driven to EOF reads every entry; OR / NOT of scans; index-served operators read none) the post-filter count
    is docs_total x projected columns and counts_fn is never called: no pass over the filter columns.
    plan: a _StatsPlan of this query and these segments (plan_stats) to reuse; built here when None."""
    if plan is None:
        plan = plan_stats(query, segments, leaf_params)
    if docs_total is not None:
        c = plan.constant_value()
        if c is not None:
            return c, int(docs_total) * plan.ncols
    reqs, const_in, (ri, fi, ci), const_docs, (rd, fd, cd), host = plan.flat()
    counts = counts_fn(reqs) if reqs else np.zeros((0, 4), dtype=np.int64)
    vi, vd = counts[ri, fi], counts[rd, fd]
    if (vi < 0).any() or (vd < 0).any():
        raise RuntimeError("internal: a count the closed forms need was not computed")
    in_filter = const_in + _exact_dot(vi, ci)
    post = (const_docs + _exact_dot(vd, cd)) * plan.ncols
    if host:
        hi, hp = server_stats(query, [segments[si] for si in host], lambda i: leaf_bitmaps(host[i]))
        in_filter += hi
        post += hp
    return in_filter, post


def _exact_dot(v, c):
    """sum(v * c) as a Python int: int64 arithmetic when the magnitude bound keeps it exact, else object arithmetic."""
    if not len(v):
        return 0
    if float(np.abs(v).max()) * float(np.abs(c).sum()) < 2.0 ** 62:
        return int(np.dot(v.astype(np.int64), c.astype(np.int64)))
    return int(np.dot(v.astype(object), c.astype(object)))


def device_counts(executor, segments, reqs, stream=None):
    """pa_bitmap_counts' four counts for every request (segment index, program A, program B): one
    pa_query_filter_counts call (leaf bitmaps of every requested segment, then the count kernels, one launch each)."""
    n = len(reqs)
    pm = L.PA_BIT_PROG_MAX
    segs = np.zeros(n, dtype=np.int32)
    progs = np.zeros((n, 2, pm), dtype=np.int32)
    lens = np.zeros((n, 2), dtype=np.int32)
    for (si, a, b), r in reqs.items():
        segs[r] = si
        progs[r, 0, :len(a)] = a
        progs[r, 1, :len(b)] = b
        lens[r] = (len(a), len(b))
    out = np.zeros((n, 4), dtype=np.int64)
    L.check(L.lib().pa_query_filter_counts(executor.handle, n, segs.ctypes.data, progs.ctypes.data, lens.ctypes.data,
                                           out.ctypes.data, stream), "pa_query_filter_counts")
    return out


def fused_counts(reqs, fused, fallback, cache=None):
    """counts_fn rows from the counts the scan took itself (GpuQueryExecutor.fused_leap_counts: E leaf, Z leaf, per
    segment matched docs / leaps / gave-up): the AND request (A = [Z], B = [E]) gets popcount(A & B) = the segment's
    matched docs and the leaps, the post-filter request (the whole filter, no B) its popcount = the matched docs. Other
    requests, and segments whose fused count gave up, go to fallback(reqs) (device_counts). Unknown fields are -1.
    cache: a dict kept with the requests (their classification is the same for every execution)."""
    e, z, arr = fused
    cls = None if cache is None else cache.get((e, z))
    if cls is None:
        rows = {0: [], 1: []}  # 0: AND requests, 1: whole-filter requests -> (row, segment)
        other = []
        for key, r in reqs.items():
            si, a, b = key
            if a == (z,) and b == (e,):
                rows[0].append((r, si))
            elif not b and a in ((z, e, L.PA_BIT_AND), (e, z, L.PA_BIT_AND)):
                rows[1].append((r, si))
            else:
                other.append(key)
        cls = tuple(np.array(rows[k], dtype=np.int64).reshape(-1, 2) for k in (0, 1)) + (other,)
        if cache is not None:
            cache[(e, z)] = cls
    and_rs, doc_rs, other = cls
    out = np.full((len(reqs), 4), -1, dtype=np.int64)
    rest = list(other)
    inv = None
    for rs, fields in ((and_rs, (2, 3)), (doc_rs, (0,))):
        if not len(rs):
            continue
        ok = arr[rs[:, 1], 2] == 0
        r, sg = rs[ok, 0], rs[ok, 1]
        if fields == (2, 3):
            out[r, 2], out[r, 3] = arr[sg, 0], arr[sg, 1]
        else:
            out[r, 0] = arr[sg, 0]
        if not ok.all():  # (gave-up segments: from leaf bitmaps)
            if inv is None:
                inv = {v: k for k, v in reqs.items()}
            rest += [inv[int(x)] for x in rs[~ok, 0]]
    if rest:
        sub_reqs = {key: i for i, key in enumerate(rest)}
        sub = fallback(sub_reqs)
        for key, r2 in sub_reqs.items():
            out[reqs[key]] = sub[r2]
    return out


def server_stats_device(query, segments, executor, stream=None, docs_total=None, plan=None):
    """server_stats with the counts computed on the GPU (device_counts); same results. docs_total: the executor's
    numDocsScanned of its last scan (server_stats_closed_form: constant-cost filters then need no GPU pass). When the
    scan counted the statistics of its two-leaf AND itself (PA_QF_FILTER_STATS: fused_counts), no extra GPU pass runs
    for the segments it covered."""
    fz = executor.fused_leap_counts(stream) if hasattr(executor, "fused_leap_counts") else None
    if fz is not None and plan is not None:
        # every request covered by the scan's own counts: two dot products (no request table, no gathers)
        e, z, arr = fz
        form = plan.fused_form(e, z, len(segments))
        if form is not None and not arr[:, 2].any():
            const_in, A, B, const_docs, C = form
            m, lp = arr[:, 0], arr[:, 1]
            return const_in + int(A @ m + B @ lp), (const_docs + int(C @ m)) * plan.ncols

    def counts(reqs):
        dev = lambda rq: device_counts(executor, segments, rq, stream)
        return dev(reqs) if fz is None else fused_counts(reqs, fz, dev, None if plan is None else plan.fused_cache)
    return server_stats_closed_form(query, segments, counts, lambda si: executor.leaf_bitmaps(si, stream),
                                    getattr(executor, "leaf_params", None), docs_total, plan)
