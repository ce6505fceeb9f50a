"""CPU model of pa_query_execution_stats (pa_stats_host.hip `stats` + pa_stats.hip), for tests: the same reduction of an
encoded operator tree (filter_stats.operator_trees rows) to constants, applyAnd counts and leap-frogs, and the same
chunked leap-frog (per chunk and entry state, then chained per segment) with a small chunk size, so the algorithm is
checked against the iterator replay (filter_stats.server_stats) on the CPU. Not product code."""
import numpy as np

from pinot_amd import _lib as L

LF_DOCS, LF_SCAN, LF_OR = 0, 1, 2


class Unsupported(Exception):
    pass


def _prog(row):
    return [int(t) for t in row[4:4 + row[3]]]


def _join(a, b, op):
    return list(b) if not a else list(a) + list(b) + [op]


def _extent(ops, i):
    j = i + 1
    for _ in range(ops[i][1]):
        j = _extent(ops, j)
    return j


def _children(ops, i):
    out, j = [], i + 1
    for _ in range(ops[i][1]):
        out.append(j)
        j = _extent(ops, j)
    return out


def eval_prog(prog, leaves, n):
    st = []
    for t in prog:
        if t >= 0:
            st.append(leaves[t][:n].copy())
        elif t == L.PA_BIT_NOT:
            st[-1] = ~st[-1]
        else:
            y, x = st.pop(), st.pop()
            st.append(x & y if t == L.PA_BIT_AND else x | y)
    assert len(st) == 1
    return st[0]


class Seg:
    """One segment: n docs, leaf masks bool[leaves, n], mv weights {column id: values per doc}."""

    def __init__(self, n, leaves, weights=None):
        self.n, self.leaves, self.weights = n, leaves, weights or {}


def _mv(seg, col):
    if col not in seg.weights:
        raise Unsupported("not a multi-value column")
    return col


def _or_elem(ops, i, seg, counts):
    kids = _children(ops, i)
    nsorted = sum(ops[k][0] == L.PA_FOP_SORTED for k in kids)
    subs, merged = [], []
    for k in kids:
        o = ops[k]
        if o[0] == L.PA_FOP_SORTED and nsorted > 1:
            merged = _join(merged, _prog(o), L.PA_BIT_OR)
            continue
        if o[0] in (L.PA_FOP_SORTED, L.PA_FOP_BITMAP):
            subs.append((LF_DOCS, _prog(o), -1))
        elif o[0] == L.PA_FOP_SCAN:
            subs.append((LF_SCAN, _prog(o), _mv(seg, o[2]) if o[2] >= 0 else -1))
        elif o[0] == L.PA_FOP_AND:
            saved = list(counts)
            el, d = _and_build(ops, k, seg, counts)
            if el:
                counts[:] = saved
                raise Unsupported("leap-frogging AND under an OR under a leap-frog")
            subs.append((LF_DOCS, d, -1))
        else:
            raise Unsupported("NOT under an OR under a leap-frog")
    if merged:
        subs.insert(0, (LF_DOCS, merged, -1))
    prog = []
    for s in subs:
        prog = _join(prog, s[1], L.PA_BIT_OR)
    if len(kids) == nsorted:
        return (LF_DOCS, prog, -1, [])
    return (LF_OR, prog, -1, subs)


def _and_build(ops, i, seg, counts):
    kids = _children(ops, i)
    sorted_, bitmaps, scans, rest = [], [], [], []
    for k in kids:
        kd = ops[k][0]
        if kd == L.PA_FOP_SORTED:
            sorted_.append(k)
        elif kd == L.PA_FOP_BITMAP:
            bitmaps.append(k)
        elif kd == L.PA_FOP_SCAN:
            scans.append(k)
        elif kd == L.PA_FOP_OR and all(ops[c][0] == L.PA_FOP_SORTED for c in _children(ops, k)):
            bitmaps.append(k)
        else:
            rest.append(k)

    def doc_prog(k):
        if ops[k][0] != L.PA_FOP_OR:
            return _prog(ops[k])
        p = []
        for c in _children(ops, k):
            p = _join(p, _prog(ops[c]), L.PA_BIT_OR)
        return p

    out = []
    if (sorted_ or bitmaps) and scans or len(sorted_) + len(bitmaps) > 1:
        D = []
        for k in sorted_ + bitmaps:
            D = _join(D, doc_prog(k), L.PA_BIT_AND)
        for k in scans:
            o = ops[k]
            counts.append((D, _mv(seg, o[2]) if o[2] >= 0 else -1))
            D = _join(D, _prog(o), L.PA_BIT_AND)
        if not rest:
            return [], D
        out.append((LF_DOCS, D, -1, []))
        kids = rest
    for k in kids:
        o = ops[k]
        if o[0] in (L.PA_FOP_SORTED, L.PA_FOP_BITMAP):
            out.append((LF_DOCS, _prog(o), -1, []))
        elif o[0] == L.PA_FOP_SCAN:
            out.append((LF_SCAN, _prog(o), _mv(seg, o[2]) if o[2] >= 0 else -1, []))
        elif o[0] == L.PA_FOP_OR:
            out.append(_or_elem(ops, k, seg, counts))
        else:
            raise Unsupported("NOT leap-frogged")
    docs = []
    for e in out:
        docs = _join(docs, e[1], L.PA_BIT_AND)
    return out, docs


def _cost_next(ops, i, seg, counts, leaps, tail):
    o = ops[i]
    if o[0] in (L.PA_FOP_EMPTY, L.PA_FOP_MATCH_ALL, L.PA_FOP_SORTED, L.PA_FOP_BITMAP):
        return 0
    if o[0] == L.PA_FOP_SCAN:
        return int(seg.weights[_mv(seg, o[2])].sum()) if o[2] >= 0 else seg.n
    if o[0] == L.PA_FOP_OR:
        return sum(_cost_next(ops, k, seg, counts, leaps, False) for k in _children(ops, i))
    if o[0] == L.PA_FOP_NOT:
        return _cost_next(ops, i + 1, seg, counts, leaps, True)
    el, _ = _and_build(ops, i, seg, counts)
    if el:
        if len(el) > 8 or sum(len(e[3]) for e in el) > 8:
            raise Unsupported("too many children")
        if tail and any(e[3] for e in el):
            raise Unsupported("NOT over a leap-frog with an OR child")
        leaps.append((el, tail))
    return 0


# ------------------------------------------------------------------ chunked leap-frog (pa_stats.hip restated)
def _next(mask, t, c1):
    nz = np.flatnonzero(mask[t:c1])
    return t + int(nz[0]) if len(nz) else c1


def _reads(wt, t, d, c1):
    e = d + 1 if d < c1 else c1
    return int(wt[e] - wt[t]) if wt is not None else e - t


def _chunk(el, subs, masks, wts, smasks, swts, n, c0, c1, s):
    K = len(el)
    S = len(subs)
    direct = tail = matches = has = 0
    sc = [[0] * S, [0] * S]
    reach = [[c0 - 1] * S, [c0 - 1] * S]
    for j in range(S):
        if subs[j][0] != LF_DOCS:
            d = _next(smasks[j], c0, c1)
            reach[1][j] = d
            sc[1][j] = _reads(swts[j], c0, d, c1)
    idx, mi, ex = 0, -1, K
    if s < K:
        mx = _next(masks[s], c0, c1)
        if el[s][0] == LF_SCAN:
            direct += _reads(wts[s], c0, mx, c1)
        mi = s
        if mx >= c1:
            ex = s
    else:
        mx = c0
    if mx < c1:
        while True:
            left = False
            while idx < K:
                if idx == mi:
                    idx += 1
                    continue
                e = idx
                d = _next(masks[e], mx, c1)
                if el[e][0] == LF_SCAN:
                    r = _reads(wts[e], mx, d, c1)
                    direct += r
                    tail += r
                elif el[e][0] == LF_OR:
                    for j in range(S):
                        if subs[j][3] != e or subs[j][0] == LF_DOCS:
                            continue
                        v0, v1 = mx > reach[0][j], mx > reach[1][j]
                        if not (v0 or v1):
                            continue
                        dj = _next(smasks[j], mx, c1)
                        r = _reads(swts[j], mx, dj, c1)
                        if v0:
                            sc[0][j] += r
                            reach[0][j] = dj
                        if v1:
                            sc[1][j] += r
                            reach[1][j] = dj
                if d == mx:
                    idx += 1
                else:
                    mx, mi, idx = d, e, 0
                    if mx >= c1:
                        ex, left = e, True
                        break
            if left:
                break
            matches += 1
            has = 1
            tail = 0
            mx += 1
            idx, mi = 0, -1
            if mx >= c1:
                ex = K
                break
    p0 = sum(1 << j for j in range(S) if reach[0][j] >= c1)
    p1 = sum(1 << j for j in range(S) if reach[1][j] >= c1)
    return ex, has, p0, p1, matches, direct, (tail if has else direct), sc


def leapfrog(el, tail_wanted, seg, chunk=64):
    """(entries read, entries read after the last match, matches) of AndDocIdIterator over the elements, by chunks."""
    n = seg.n
    masks = [eval_prog(e[1], seg.leaves, n) for e in el]
    wts = [np.concatenate([[0], np.cumsum(seg.weights[e[2]])]) if e[2] >= 0 else None for e in el]
    subs = [(s[0], s[1], s[2], ei) for ei, e in enumerate(el) for s in e[3]]
    smasks = [eval_prog(s[1], seg.leaves, n) for s in subs]
    swts = [np.concatenate([[0], np.cumsum(seg.weights[s[2]])]) if s[2] >= 0 else None for s in subs]
    K, S = len(el), len(subs)
    nch = (n + chunk - 1) // chunk
    cells = [[_chunk(el, subs, masks, wts, smasks, swts, n, c * chunk, min(n, (c + 1) * chunk), s)
              for s in range(K + 1)] for c in range(nch)]
    st, P = K, 0
    cost = matched = 0
    tl = 0
    for c in range(nch):
        ex, has, p0, p1, m, direct, t, sc = cells[c][st]
        cost += direct + sum(sc[(P >> j) & 1][j] for j in range(S))
        matched += m
        tl = t if has else tl + direct
        P = (P & p1) | (~P & p0)
        st = ex
    return cost, tl, matched


# ------------------------------------------------------------------ iterator replay (pa_stats.hip stat_replay_kernel)
RP_EMPTY, RP_ALL, RP_DOCS, RP_SCAN, RP_AND, RP_OR, RP_NOT = range(7)
RP_MAX_NODES, RP_MAX_DEPTH = 24, 6
EOF_ = -1


def replay_build(ops, i, seg, counts, nodes):
    """pa_stats_host.hip replay_build: the iterator tree BlockDocIdSet.iterator() builds, applyAnd reads into counts.
    nodes: list of [kind, sorted, prog, mv, kids]; returns the node index."""
    o = ops[i]
    kd = o[0]

    def add(n):
        if len(nodes) >= 4 * RP_MAX_NODES:
            raise Unsupported("replay tree too large")
        nodes.append(n)
        return len(nodes) - 1
    if kd == L.PA_FOP_EMPTY:
        return add([RP_EMPTY, False, [], -1, []])
    if kd == L.PA_FOP_MATCH_ALL:
        return add([RP_ALL, False, [], -1, []])
    if kd in (L.PA_FOP_SORTED, L.PA_FOP_BITMAP):
        return add([RP_DOCS, kd == L.PA_FOP_SORTED, _prog(o), -1, []])
    if kd == L.PA_FOP_SCAN:
        return add([RP_SCAN, False, _prog(o), _mv(seg, o[2]) if o[2] >= 0 else -1, []])
    if kd == L.PA_FOP_NOT:
        c = replay_build(ops, i + 1, seg, counts, nodes)
        return add([RP_NOT, False, [], -1, [c]])
    its = [replay_build(ops, k, seg, counts, nodes) for k in _children(ops, i)]
    docs = [k for k in its if nodes[k][0] == RP_DOCS]
    if kd == L.PA_FOP_OR:
        srt = [k for k in docs if nodes[k][1]]
        rest = [k for k in its if nodes[k][0] != RP_DOCS]
        if len(srt) > 1:  # (OrDocIdSet: bitmap-based children neither merged nor kept, as the reference)
            prog = []
            for k in srt:
                prog = _join(prog, nodes[k][2], L.PA_BIT_OR)
            m = add([RP_DOCS, False, prog, -1, []])
            return m if not rest else add([RP_OR, False, [], -1, [m] + rest])
        return add([RP_OR, False, [], -1, its])
    scans = [k for k in its if nodes[k][0] == RP_SCAN]
    rest = [k for k in its if nodes[k][0] not in (RP_DOCS, RP_SCAN)]
    if (docs and scans) or len(docs) > 1:
        D = []
        for k in docs:
            D = _join(D, nodes[k][2], L.PA_BIT_AND)
        for k in scans:
            counts.append((D, nodes[k][3]))
            D = _join(D, nodes[k][2], L.PA_BIT_AND)
        m = add([RP_DOCS, False, D, -1, []])
        return m if not rest else add([RP_AND, False, [], -1, [m] + rest])
    return add([RP_AND, False, [], -1, its])


def replay_flatten(nodes, root):
    """Pre-order reachable tree, depth- and size-limited as the kernel's job."""
    out, depth = [], []

    def emit(r, d):
        if d >= RP_MAX_DEPTH or len(out) >= RP_MAX_NODES:
            raise Unsupported("replay tree too deep / large")
        me = len(out)
        out.append(list(nodes[r]))
        depth.append(d)
        out[me][4] = [emit(c, d + 1) for c in nodes[r][4]]
        return me
    emit(root, 0)
    return out, depth


def replay(flat, depth, seg):
    """stat_replay_kernel restated: the projection's next() until EOF over the node machine; entries read."""
    n = seg.n
    masks = [eval_prog(nd[2], seg.leaves, n) if nd[0] in (RP_DOCS, RP_SCAN) else None for nd in flat]
    wts = [np.concatenate([[0], np.cumsum(seg.weights[nd[3]])]) if nd[0] == RP_SCAN and nd[3] >= 0 else None
           for nd in flat]
    N = len(flat)
    a, b, c = [0] * N, [0] * N, [0] * N
    nd_, live = [-1] * N, [True] * N
    ent = [0]

    def next_set(m, t, e):
        if t >= e:
            return e
        z = np.flatnonzero(m[t:e])
        return t + int(z[0]) if len(z) else e

    def read(i, lo, hi):
        ent[0] += int(wts[i][hi] - wts[i][lo]) if wts[i] is not None else hi - lo

    def scan_from(i, start):
        d = next_set(masks[i], start, n)
        if d < n:
            read(i, start, d + 1)
            a[i] = d + 1
            return d
        if start < n:
            read(i, start, n)
        a[i] = max(start, n)
        return EOF_

    def nxt(i):
        k = flat[i][0]
        if k == RP_DOCS:
            d = next_set(masks[i], a[i], n)
            a[i] = d + 1 if d < n else n
            return d if d < n else EOF_
        if k == RP_ALL:
            if a[i] < n:
                a[i] += 1
                return a[i] - 1
            return EOF_
        if k == RP_SCAN:
            if wts[i] is not None:
                return scan_from(i, a[i])
            while True:
                if b[i] < c[i]:
                    d = next_set(masks[i], b[i], c[i])
                    if d < c[i]:
                        b[i] = d + 1
                        return d
                    b[i] = c[i]
                limit = min(n - a[i], 256)
                if limit <= 0:
                    return EOF_
                ent[0] += limit
                b[i], c[i] = a[i], a[i] + limit
                a[i] += limit
        if k == RP_AND:
            kids = flat[i][4]
            mx, mi, idx = a[i], -1, 0
            while idx < len(kids):
                if idx == mi:
                    idx += 1
                    continue
                d = adv(kids[idx], mx)
                if d == EOF_:
                    return EOF_
                if d == mx:
                    idx += 1
                else:
                    mx, mi, idx = d, idx, 0
            a[i] = mx + 1
            return mx
        if k == RP_OR:
            best = EOF_
            for kk in flat[i][4]:
                if not live[kk]:
                    continue
                d = nd_[kk]
                if d == a[i]:
                    d = nxt(kk)
                    nd_[kk] = d
                    if d == EOF_:
                        live[kk] = False
                        continue
                best = d if best == EOF_ or d < best else best
            if best != EOF_:
                a[i] = best
            return best
        if k == RP_NOT:
            kk = flat[i][4][0]
            while a[i] == b[i]:
                a[i] += 1
                d = nxt(kk)
                b[i] = n if d == EOF_ else d
            if a[i] >= n:
                return EOF_
            a[i] += 1
            return a[i] - 1
        return EOF_

    def adv(i, t):
        k = flat[i][0]
        if k == RP_DOCS:
            d = next_set(masks[i], t, n)
            a[i] = d + 1 if d < n else n
            return d if d < n else EOF_
        if k in (RP_ALL, RP_AND):
            a[i] = t
            return nxt(i)
        if k == RP_SCAN:
            b[i] = c[i] = 0
            return scan_from(i, t)
        if k == RP_OR:
            best = EOF_
            for kk in flat[i][4]:
                if not live[kk]:
                    continue
                d = nd_[kk]
                if d < t:
                    d = adv(kk, t)
                    nd_[kk] = d
                    if d == EOF_:
                        live[kk] = False
                        continue
                best = d if best == EOF_ or d < best else best
            if best != EOF_:
                a[i] = best
            return best
        if k == RP_NOT:
            a[i] = t
            if t > b[i]:
                d = adv(flat[i][4][0], t)
                b[i] = n if d == EOF_ else d
            return nxt(i)
        return EOF_

    for i in range(N):
        if flat[i][0] == RP_OR:
            a[i] = -1
    for i in reversed(range(N)):
        if flat[i][0] == RP_NOT:
            d = nxt(flat[i][4][0])
            a[i], b[i] = 0, n if d == EOF_ else d
    while nxt(0) != EOF_:
        pass
    return ent[0]


def execution_stats(ops, roots, seg_tree, segs, ncols, docs_scanned, chunk=64, replayed=None):
    """(in filter, post filter, per-segment in filter with -1 for host-replayed segments). Segments outside the
    reduction are replayed iterator by iterator (stat_replay_kernel); replayed (a list) collects their indices."""
    per = []
    non_scan = 0
    for si, seg in enumerate(segs):
        t = int(seg_tree[si])
        if t == L.PA_STATS_NON_SCAN:
            non_scan += seg.n
            per.append(0)
            continue
        if t == L.PA_STATS_HOST:
            per.append(-1)
            continue
        counts, leaps = [], []
        try:
            v = _cost_next(ops, int(roots[t]), seg, counts, leaps, False)
        except Unsupported:
            counts, leaps = [], []
            try:
                nodes = []
                root = replay_build(ops, int(roots[t]), seg, counts, nodes)
                flat, depth = replay_flatten(nodes, root)
                v = replay(flat, depth, seg)
            except Unsupported:
                per.append(-1)
                continue
            if replayed is not None:
                replayed.append(si)
        for prog, mv in counts:
            m = eval_prog(prog, seg.leaves, seg.n)
            v += int(seg.weights[mv][m].sum()) if mv >= 0 else int(m.sum())
        for el, tail in leaps:
            c, tl, _ = leapfrog(el, tail, seg, chunk)
            v += c + (tl if tail else 0)
        per.append(v)
    return sum(x for x in per if x >= 0), (docs_scanned - non_scan) * ncols, per
