// Query-shape specialised kernels compiled by hiprtc at pa_query_prepare: gdl_jit.hip (dense GROUP BY with packed
// accumulation) and pve_jit.hip (count-free partitioned emit).
#include "pa_host.h"

// ---------------------------------------------------------------- query-shape specialisation (gdl_jit.hip)
// The lane-major dense kernel with packed accumulation, compiled per query shape by hiprtc: every column width, image
// offset, leaf kind and field offset becomes a constant (no bit-width switch, no parameter reads, no DMA loop in the
// tile loop). Compiled once per shape and device and cached for the process; the generic kernel runs when the shape
// is outside the specialised form (or PA_QF_NO_JIT / PA_NO_JIT), or hiprtc fails.
static const char* kGdlJitSrc =
#include "gdl_jit_src.inc"
    ;

namespace {
std::mutex g_jit_mu;
struct JitEntry {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
};
std::map<std::string, JitEntry> g_jit_cache;  // (device, compile options) -> loaded kernel

std::string int_list(const std::vector<int>& v) {
  std::string r = "{";
  for (size_t i = 0; i < v.size(); ++i) r += (i ? "," : "") + std::to_string(v[i]);
  return r + "}";
}

hipFunction_t jit_compile(const std::vector<std::string>& defs, const char* src = kGdlJitSrc,
                          const char* name = "gdl_jit") {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::string key = std::to_string(dev) + " " + name;
  for (const std::string& d : defs) key += " " + d;
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto it = g_jit_cache.find(key);
  if (it != g_jit_cache.end()) return it->second.fn;
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src, name, 0, nullptr, nullptr) != HIPRTC_SUCCESS) return nullptr;
  std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  for (const std::string& d : defs) opts.push_back(d);
  std::vector<const char*> o;
  for (const std::string& x : opts) o.push_back(x.c_str());
  hipFunction_t fn = nullptr;
  if (hiprtcCompileProgram(prog, (int)o.size(), o.data()) == HIPRTC_SUCCESS) {
    size_t n = 0;
    if (hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n) {
      std::vector<char> code(n);
      JitEntry e;
      if (hiprtcGetCode(prog, code.data()) == HIPRTC_SUCCESS && hipModuleLoadData(&e.mod, code.data()) == hipSuccess &&
          hipModuleGetFunction(&e.fn, e.mod, name) == hipSuccess) {
        fn = e.fn;
        g_jit_cache[key] = e;
      }
    }
  } else if (std::getenv("PA_JIT_LOG")) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::vector<char> log(n + 1, 0);
    hiprtcGetProgramLog(prog, log.data());
    std::fprintf(stderr, "pinot_amd: %s compile failed:\n%s\n", name, log.data());
  }
  hiprtcDestroyProgram(&prog);
  return fn;
}
}  // namespace

// The JIT args' accumulator pointers (the block can move: pa_query_set_accumulator_buffer)
void jit_fill_pointers(pa_query* q, JitArgs& a) {
  const pa_query_spec& s = q->spec;
  a.matched = q->hq.matched_docs;
  a.count = q->hq.count;
  int k = 0;
  for (int i = 0; i < s.num_aggs; ++i) {
    if (s.aggs[i].type == PA_AGG_COUNT) continue;
    a.sum[k] = (long long*)q->hq.aggs[i].acc_i64;
    a.sum_long[k] = q->hq.aggs[i].src == SRC_LONG ? 1 : 0;
    ++k;
  }
}

namespace {
// bits that hold every value 0..v
int bits_for(uint64_t v) {
  int w = 0;
  while (w < 64 && (v >> w) != 0) ++w;
  return w;
}
size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// One SUM of the specialised kernel: its per-doc term and where the values come from
struct JitSum {
  int col = 0;          // JIT column
  int w = 0;            // term bits
  bool table = false;   // term = value table[dictId] (value - base); else dictId (+ the segment's offset)
  bool shared = true;   // (table) one dictionary for every segment: the shared LDS area, else the slots
  bool offs = false;    // (dictId) per-segment offsets
  int64_t base = 0, step = 1;
  std::vector<int64_t> aoff;  // per included segment
  int max_card = 0;
};
}  // namespace

// Query-shape specialisation of the dense GROUP BY (gdl_jit.hip), over segments that share their dictionaries or build
// their own (SegmentDictionaryCreator.java:104: per segment). Takes a query whose key box the dense planner found
// (P.gd_box_ok) with one dictionary group-by column, COUNT / integer SUMs over dictionary columns and eager dictionary
// leaves; every staged column 1..31 bits. Leaves q->jit_fn null (the generic plan runs) otherwise.
int jit_plan(pa_query* q, const Prep& P, int cus) {
  q->jit_fn = nullptr;
  q->jit_cols.clear();
  const pa_query_spec& s = q->spec;
  if (q->nseg == 0 || s.num_group_by != 1 || !P.gd_box_ok || P.gd_box || q->hq.leap_mode || q->partitioned ||
      q->limit_mode || q->limit_walk || q->hashed)
    return PA_OK;
  if ((s.flags & PA_QF_NO_JIT) || std::getenv("PA_NO_JIT") || std::getenv("PA_DEBUG_EMIT")) return PA_OK;
  // flags that pin a generic plan (tests and measurement) keep it
  if (s.flags & (PA_QF_NO_DENSE_GROUP | PA_QF_FORCE_GLOBAL | PA_QF_FORCE_LDS | PA_QF_LAZY_POST | PA_QF_NO_LANE_MAJOR |
                 PA_QF_STEPS16 | PA_QF_DEBUG_STREAM_ONLY | PA_QF_NO_GDENSE_LM | PA_QF_NO_GD_PACK))
    return PA_OK;
  const int nl_all = (int)q->literals.size();
  if (q->num_eager != nl_all) return PA_OK;
  for (int li = 0; li < nl_all; ++li) {
    const int kind = s.leaves[q->literals[li].leaf].kind;
    if (kind != PA_LEAF_DICT_RANGE && kind != PA_LEAF_DICT_SET) return PA_OK;
  }
  // a literal's standing in one segment: 1 = every doc matches (the range covers the segment's dictionary, the set holds
  // every dictId, or the negation of an empty one), -1 = no doc matches, 0 = depends on the doc
  auto literal_in = [&](int si, int li) {
    const Literal lit = q->literals[li];
    const pa_leaf_params& p = q->leaf_params[si][lit.leaf];
    const bool neg = (p.negate != 0) != lit.neg;
    const int64_t card = q->segs[si]->cols.at(s.leaves[lit.leaf].column_id)->cardinality;
    bool all = false, none = false;
    if (s.leaves[lit.leaf].kind == PA_LEAF_DICT_RANGE) {
      const int64_t lo = std::max<int64_t>(0, p.lo), hi = std::min<int64_t>(p.hi, card);
      none = hi <= lo;
      all = lo == 0 && hi >= card;
    } else {
      const std::vector<uint32_t>& lut = q->luts[si][lit.leaf];
      int64_t n = 0;
      for (int64_t w = 0; w < (card + 31) / 32 && (size_t)w < lut.size(); ++w) {
        const int64_t left = card - 32 * w;
        n += __builtin_popcount(lut[w] & (left >= 32 ? 0xffffffffu : ((1u << left) - 1u)));
      }
      none = n == 0;
      all = n == card;
    }
    if (neg) std::swap(all, none);
    return all ? 1 : (none ? -1 : 0);
  };
  // segments a unit clause provably empties (a day range outside a time partition, an IN list none of whose values the
  // segment holds) match no doc: they stay out of the kernel's tiles (numDocsScanned 0 there)
  std::vector<int> inc;  // included segments
  for (int si = 0; si < q->nseg; ++si) {
    bool empty = false;
    for (int li = 0; li < nl_all && !empty; ++li)
      empty = q->clause_end[li] && (li == 0 || q->clause_end[li - 1]) && literal_in(si, li) < 0;
    if (!empty) inc.push_back(si);
  }
  if (inc.empty()) return PA_OK;  // (nothing to scan: the generic plan's launch finds no match either)
  const int ni = (int)inc.size();
  // clauses every included segment satisfies whatever the doc (a literal of it matching every doc there: a day range
  // covering each time partition) are left out of the kernel: they cannot filter, and their unpack and compares cost
  // VALU per doc
  std::vector<int> lit;  // the kernel's leaves: indices into q->literals
  for (int c0 = 0; c0 < nl_all;) {
    int c1 = c0;
    while (!q->clause_end[c1]) ++c1;
    bool always = true;
    for (int k = 0; k < ni && always; ++k) {
      bool sat = false;
      for (int li = c0; li <= c1 && !sat; ++li) sat = literal_in(inc[k], li) > 0;
      always = sat;
    }
    if (!always)
      for (int li = c0; li <= c1; ++li) lit.push_back(li);
    c0 = c1 + 1;
  }
  const int nl = (int)lit.size();
  if (nl > kJitMax) return PA_OK;
  // the kernel's columns: the leaves', the group-by column, the SUMs'
  std::vector<int> cols;
  auto col_of = [&](int slot) {
    for (size_t k = 0; k < cols.size(); ++k)
      if (cols[k] == slot) return (int)k;
    cols.push_back(slot);
    return (int)cols.size() - 1;
  };
  std::vector<int> lk(nl), lc(nl), le(nl);
  for (int li = 0; li < nl; ++li) {
    const Literal& L = q->literals[lit[li]];
    lk[li] = s.leaves[L.leaf].kind == PA_LEAF_DICT_SET ? 1 : 0;
    lc[li] = col_of(P.leaf_slot[L.leaf]);
    le[li] = q->clause_end[lit[li]] ? 1 : 0;
  }
  const int kc = col_of(P.gb_slot[0]);
  std::vector<int> sum_aggs;
  for (int a = 0; a < s.num_aggs; ++a) {
    if (s.aggs[a].type == PA_AGG_COUNT) continue;
    if (s.aggs[a].type != PA_AGG_SUM) return PA_OK;
    sum_aggs.push_back(a);
  }
  const int na = (int)sum_aggs.size();
  if (na > kJitMax) return PA_OK;
  std::vector<JitSum> sums(na);
  for (int k = 0; k < na; ++k) sums[k].col = col_of(P.agg_slot[sum_aggs[k]]);
  const int nc = (int)cols.size();
  if (nc > kJitMax) return PA_OK;
  for (int si = 0; si < q->nseg; ++si)
    for (int c = 0; c < nc; ++c) {
      const DevCol& dc = q->hsegs[si].cols[cols[c]];
      if (dc.kind != COL_SV_DICT || !dc.words || dc.nbits < 1 || dc.nbits > 31) return PA_OK;
    }
  for (int k = 0; k < na; ++k)
    for (int si = 0; si < q->nseg; ++si) {
      const Column* c = q->segs[si]->cols.at(s.aggs[sum_aggs[k]].column_id);
      if ((c->vtype != PA_INT && c->vtype != PA_LONG) || c->hvals.size() != (size_t)c->cardinality || !c->dict.p)
        return PA_OK;
    }
  // leaves: negation per segment, DICT_SET bitmaps shared or per segment
  std::vector<int> ln(nl, 0), luts_slot(nl, 0), lut_words(nl, 0);
  std::vector<uint32_t> negmask(ni, 0);
  for (int li = 0; li < nl; ++li) {
    bool any = false, all = true;
    for (int k = 0; k < ni; ++k) {
      const bool n = q->hsegs[inc[k]].leaves[lit[li]].negate != 0;
      any |= n;
      all &= n;
      if (n) negmask[k] |= 1u << li;
    }
    ln[li] = all ? 1 : (any ? 2 : 0);
    if (lk[li]) {
      const int leaf = q->literals[lit[li]].leaf;
      for (int k = 0; k < ni; ++k) {
        lut_words[li] = std::max(lut_words[li], (int)q->luts[inc[k]][leaf].size());
        if (q->luts[inc[k]][leaf] != q->luts[inc[0]][leaf]) luts_slot[li] = 1;
      }
    }
  }
  // group key: a contiguous run of the table dictionary per segment (affine: key = dictId + offset) or a remap table
  const int64_t klo = P.gd_lo[0], kspan = P.gd_span[0];
  std::vector<int64_t> koff(ni, 0);
  bool ktab = false;
  int kcard = 0;
  for (int k = 0; k < ni; ++k) {
    const int si = inc[k];
    kcard = std::max(kcard, (int)q->hsegs[si].cols[cols[kc]].card);
    if (!q->has_remap[si][0]) continue;
    const std::vector<int32_t>& rm = q->remaps[si][0];
    for (size_t i = 0; i < rm.size() && !ktab; ++i) ktab = rm[i] != rm[0] + (int32_t)i;
    koff[k] = rm.empty() ? 0 : rm[0];
  }
  // the group key from a DICT_RANGE leaf's unpack; the box check implied in a segment when that leaf is a unit clause
  // whose range, shifted into the table's key ids, lies inside the box, or when the segment's whole dictionary does (a
  // matching doc's key is then in the box) — in every segment
  int kl = -1;
  for (int li = 0; li < nl; ++li)
    if (lk[li] == 0 && lc[li] == kc) {
      kl = li;
      break;
    }
  const bool kl_unit = kl >= 0 && ln[kl] == 0 && q->clause_end[lit[kl]] && (kl == 0 || q->clause_end[lit[kl] - 1]);
  bool kib = !ktab;
  for (int k = 0; k < ni && kib; ++k) {
    const int64_t card = q->hsegs[inc[k]].cols[cols[kc]].card;
    int64_t rlo = 0, rhi = card;
    if (kl_unit) {
      const pa_leaf_params& p = q->leaf_params[inc[k]][q->literals[lit[kl]].leaf];
      rlo = std::max<int64_t>(0, p.lo);
      rhi = std::min<int64_t>(p.hi, card);
    }
    kib = (rhi > rlo && rlo + koff[k] >= klo && rhi + koff[k] <= klo + kspan) || (koff[k] >= klo && card + koff[k] <= klo + kspan);
  }
  // SUM terms: dictIds of arithmetic dictionaries with one common step (each segment's offset into the term space), else
  // value tables (values - the smallest value)
  for (int k = 0; k < na; ++k) {
    JitSum& J = sums[k];
    const int32_t cid = s.aggs[sum_aggs[k]].column_id;
    const Column* c0 = q->segs[inc[0]]->cols.at(cid);
    bool affine = true;
    int64_t step = 0;
    std::vector<int64_t> b(ni, 0);
    __int128 gmin = 0, gmax = 0;
    bool seen = false;
    for (int i = 0; i < ni; ++i) {
      const Column* c = q->segs[inc[i]]->cols.at(cid);
      J.max_card = std::max(J.max_card, c->cardinality);
      J.shared = J.shared && (c == c0 || (c->dict_hash == c0->dict_hash && c->hvals == c0->hvals));
      for (uint64_t x : c->hvals) {
        const __int128 v = (int64_t)x;
        if (!seen) gmin = gmax = v;
        seen = true;
        gmin = std::min(gmin, v);
        gmax = std::max(gmax, v);
      }
      int64_t bs = 0, st = 0;
      if (affine && affine_dictionary(c->hvals, c->vtype, &bs, &st) && st >= 0) {
        b[i] = bs;
        if (st > 0 && step > 0 && st != step) affine = false;
        if (st > 0) step = st;
      } else {
        affine = false;
      }
    }
    if (affine) {
      if (step == 0) step = 1;
      __int128 mn = b[0];
      for (int i = 0; i < ni; ++i) mn = std::min(mn, (__int128)b[i]);
      __int128 top = 0;
      J.aoff.assign(ni, 0);
      for (int i = 0; i < ni && affine; ++i) {
        const __int128 d = (__int128)b[i] - mn;
        if (d % step != 0) affine = false;
        J.aoff[i] = (int64_t)(d / step);
        top = std::max(top, d / step + q->segs[inc[i]]->cols.at(cid)->cardinality - 1);
      }
      if (affine && top < ((__int128)1 << 32)) {
        J.table = false;
        J.base = (int64_t)mn;
        J.step = step;
        for (int64_t o : J.aoff) J.offs |= o != 0;
        // (per-segment offsets are folded in at the drain: the rows pack bare dictIds)
        J.w = J.offs ? bits_for((uint64_t)std::max(1, J.max_card) - 1) : bits_for((uint64_t)top);
        continue;
      }
    }
    if (gmax - gmin >= ((__int128)1 << 32)) return PA_OK;
    J.table = true;
    J.base = (int64_t)gmin;
    J.step = 1;
    J.w = bits_for((uint64_t)(gmax - gmin));
  }
  int wsum = 0;
  for (const JitSum& J : sums) wsum += J.w;
  const int cbits = std::min(31, (64 - wsum) / (1 + na));
  if (cbits < 11) return PA_OK;
  // width classes: each distinct tuple of the columns' bit widths
  std::vector<std::vector<int>> classes;
  std::vector<int> seg_cls(ni, 0);
  for (int k = 0; k < ni; ++k) {
    std::vector<int> t(nc);
    for (int c = 0; c < nc; ++c) t[c] = q->hsegs[inc[k]].cols[cols[c]].nbits;
    auto it = std::find(classes.begin(), classes.end(), t);
    if (it == classes.end()) {
      if (classes.size() == 4) return PA_OK;
      classes.push_back(t);
      it = classes.end() - 1;
    }
    seg_cls[k] = (int)(it - classes.begin());
  }
  // LDS: counts, sums, shared tables, the slots' tables, then (per wave count) rows and ring
  const int nkeys = P.gd_nkeys;
  size_t off = al16((size_t)nkeys * 4);
  std::vector<int> lsum(na), lut(nl, 0), at(na, -1), ats(na, 0);
  for (int k = 0; k < na; ++k) {
    lsum[k] = (int)off;
    off += al16((size_t)nkeys * 8);
  }
  size_t so = 0;  // slot layout
  for (int li = 0; li < nl; ++li) {
    if (!lk[li]) continue;
    size_t& o = luts_slot[li] ? so : off;
    lut[li] = (int)o;
    o += al16((size_t)lut_words[li] * 4);
  }
  for (int k = 0; k < na; ++k) {
    if (!sums[k].table) continue;
    ats[k] = sums[k].shared ? 0 : 1;
    size_t& o = ats[k] ? so : off;
    at[k] = (int)o;
    o += al16((size_t)sums[k].max_card * 4);
  }
  int ktab_off = -1;
  if (ktab) {
    ktab_off = (int)so;
    so += al16((size_t)kcard * 4);
  }
  const size_t l_slot = off, slot_b = al16(so);
  // waves, docs per lane and waves per set of packed rows: the most resident waves, then the larger tile, then private
  // rows (PA_GDL_W / PA_GDL_ND / PA_GDL_RS: measurement)
  struct Cand {
    int w, nd, rs;
  };
  // (12 waves of 1024-doc tiles beat 16 of 512-doc tiles: own-dictionary secondary lines 1.130 / 1.159 vs 1.158 / 1.206
  // ms; 8 waves of 1024-doc tiles beat 12 of 512: shared 1.391 vs 1.425 ms; 12 of 512 beat 8 of 512: 1.425 vs 1.594 ms)
  std::vector<Cand> cands = {{16, 16, 1}, {12, 16, 1}, {16, 8, 1}, {8, 16, 1}, {12, 8, 1}, {8, 8, 1}, {16, 16, 2},
                             {16, 8, 2}};
  auto keep_only = [&](const char* env, int Cand::*f) {
    if (const char* e = std::getenv(env)) {
      const int v = std::atoi(e);
      cands.erase(std::remove_if(cands.begin(), cands.end(), [&](const Cand& c) { return c.*f != v; }), cands.end());
    }
  };
  keep_only("PA_GDL_W", &Cand::w);
  keep_only("PA_GDL_ND", &Cand::nd);
  keep_only("PA_GDL_RS", &Cand::rs);
  bool any_offs = false;  // (per-segment SUM offsets are folded in at the drain: one segment per private row set)
  for (const JitSum& J : sums) any_offs |= !J.table && J.offs;
  // the packed rows are indexed by each segment's local keys: its keys inside the box, [lbase, lbase + lspan) of its
  // own dictIds (affine keys) or of the table keys (remap table); box index = local key + gofs
  std::vector<int> lbase(ni), lspan(ni), gofs(ni);
  int lmax = 1;
  bool segdrain = any_offs;
  for (int k = 0; k < ni; ++k) {
    if (ktab) {
      lbase[k] = (int)klo;
      lspan[k] = (int)kspan;
      gofs[k] = 0;
    } else {
      const int64_t card = q->hsegs[inc[k]].cols[cols[kc]].card;
      const int64_t lo = std::max<int64_t>(0, klo - koff[k]), hi = std::min<int64_t>(card, klo + kspan - koff[k]);
      lbase[k] = (int)lo;
      lspan[k] = (int)std::max<int64_t>(1, hi - lo);
      gofs[k] = (int)(lo + koff[k] - klo);
    }
    lmax = std::max(lmax, lspan[k]);
    segdrain |= lbase[k] != lbase[0] || gofs[k] != gofs[0];
  }
  if (any_offs || segdrain)
    cands.erase(std::remove_if(cands.begin(), cands.end(), [](const Cand& c) { return c.rs != 1; }), cands.end());
  // tile images per wave (PA_GDL_RING: measurement): RING - 1 tiles in flight while one is walked
  int ring_n = 2;
  if (const char* e = std::getenv("PA_GDL_RING")) ring_n = std::max(2, std::min(4, std::atoi(e)));
  int W = 0, ND = 0, RS = 1, RR = 1, nslot = 0, G = 0, img_dw = 0;
  size_t lds = 0, l_rows = 0, l_ring = 0;
  std::vector<int64_t> first(ni + 1, 0);
  std::vector<std::vector<int>> coff;
  for (const Cand& cd : cands) {
    const int w = cd.w, nd = cd.nd, td = 64 * nd;
    std::vector<int64_t> f(ni + 1, 0);
    for (int k = 0; k < ni; ++k) f[k + 1] = f[k] + (q->hsegs[inc[k]].num_docs + td - 1) / td;
    const int64_t T = f[ni];
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (T + w - 1) / w));
    int ns = 0;
    if (slot_b) {  // the most segments one workgroup's tiles [lb T / G, (lb + 1) T / G) cover
      int seg = 0;
      for (int64_t lb = 0; lb < g; ++lb) {
        const int64_t t0 = lb * T / g, t1 = (lb + 1) * T / g;
        if (t0 >= t1) continue;
        while (f[seg + 1] <= t0) ++seg;
        int e = seg;
        while (e + 1 < ni && f[e + 1] < t1) ++e;
        ns = std::max(ns, e - seg + 1);
      }
    }
    std::vector<std::vector<int>> co(classes.size());
    int idw = 0;
    for (size_t ci = 0; ci < classes.size(); ++ci) {
      size_t b = 16;  // a 16-byte guard in front of every region and after the last
      for (int c = 0; c < nc; ++c) {
        co[ci].push_back((int)b);
        b += (size_t)8 * nd * classes[ci][c] + 16;
      }
      idw = std::max(idw, (int)(al16(b) / 4));
    }
    const size_t rows = al16(l_slot + (size_t)ns * slot_b);
    const size_t ring_img = (size_t)w * ring_n * idw * 4;
    // row replicas: as many as fit (up to one per lane), so the lanes of a wave hitting a segment's few keys update
    // different words (PA_GDL_RR: measurement)
    int rr = 64;
    if (const char* e = std::getenv("PA_GDL_RR")) rr = std::max(1, std::min(64, std::atoi(e)));
    while (rr > 1 && al16(rows + (size_t)(w / cd.rs) * lmax * rr * 8) + ring_img > kLdsBudget) rr >>= 1;
    while (rr > 1 && (rr & (rr - 1))) rr &= rr - 1;
    const size_t ring = al16(rows + (size_t)(w / cd.rs) * lmax * rr * 8);
    const size_t total = ring + ring_img;
    if (total > kLdsBudget) continue;
    RR = rr;
    W = w;
    ND = nd;
    RS = cd.rs;
    nslot = ns;
    G = g;
    img_dw = idw;
    lds = total;
    l_rows = rows;
    l_ring = ring;
    first = f;
    coff = co;
    break;
  }
  if (!W) return PA_OK;
  // packed fields: each SUM's term + cbits, COUNT cbits at the top; drained before a field can overflow
  std::vector<int> as(na);
  int oc = 0;
  for (int k = 0; k < na; ++k) {
    as[k] = oc;
    oc += sums[k].w + cbits;
  }
  // (a row replica takes the docs of 64 / RR lanes, ND each per tile; rows shared by RS waves: between two drains of a
  // set, each of its waves ran at most its own drain period)
  int drain = (int)std::max<uint64_t>(
      1, ((uint64_t(1) << cbits) - 1) / (uint64_t)((64 / RR) * ND) / (uint64_t)RS);
  if (s.flags & PA_QF_GD_DRAIN_EACH_TILE) drain = 1;
  auto list = [](const std::vector<int>& v) {
    std::string r = "{";
    for (size_t i = 0; i < v.size(); ++i) r += (i ? "," : "") + std::to_string(v[i]);
    return r + (v.empty() ? "0}" : "}");
  };
  std::string nbs = "{", offs = "{";
  for (size_t ci = 0; ci < classes.size(); ++ci) {
    nbs += (ci ? "," : "") + list(classes[ci]);
    offs += (ci ? "," : "") + list(coff[ci]);
  }
  nbs += "}";
  offs += "}";
  std::vector<int> ac(na), ao(na);
  for (int k = 0; k < na; ++k) {
    ac[k] = sums[k].col;
    ao[k] = (!sums[k].table && sums[k].offs) ? 1 : 0;
  }
  std::vector<std::string> defs = {
      "-DJIT_W=" + std::to_string(W), "-DJIT_ND=" + std::to_string(ND), "-DJIT_IMG=" + std::to_string(img_dw),
      "-DJIT_NC=" + std::to_string(nc), "-DJIT_NCLS=" + std::to_string(classes.size()), "-DJIT_NB=" + nbs,
      "-DJIT_OFF=" + offs, "-DJIT_NL=" + std::to_string(nl), "-DJIT_LK=" + list(lk), "-DJIT_LC=" + list(lc),
      "-DJIT_LN=" + list(ln), "-DJIT_LE=" + list(le), "-DJIT_LUT=" + list(lut), "-DJIT_LUTS=" + list(luts_slot),
      "-DJIT_KC=" + std::to_string(kc), "-DJIT_KL=" + std::to_string(kl), "-DJIT_KIB=" + std::to_string(kib ? 1 : 0),
      "-DJIT_KTAB=" + std::to_string(ktab_off), "-DJIT_NA=" + std::to_string(na), "-DJIT_AC=" + list(ac),
      "-DJIT_AT=" + list(at), "-DJIT_ATS=" + list(ats), "-DJIT_AO=" + list(ao), "-DJIT_AS=" + list(as),
      "-DJIT_OC=" + std::to_string(oc), "-DJIT_DRAIN=" + std::to_string(drain), "-DJIT_L_SUM=" + list(lsum),
      "-DJIT_L_SLOT=" + std::to_string(l_slot), "-DJIT_SLOT_B=" + std::to_string(slot_b),
      "-DJIT_NSLOT=" + std::to_string(nslot), "-DJIT_L_ROWS=" + std::to_string(l_rows),
      "-DJIT_L_RING=" + std::to_string(l_ring), "-DJIT_RS=" + std::to_string(RS), "-DJIT_RR=" + std::to_string(RR),
      "-DJIT_LMAX=" + std::to_string(lmax), "-DJIT_SEGDRAIN=" + std::to_string(segdrain ? 1 : 0),
      "-DJIT_RING=" + std::to_string(ring_n)};
  if (const char* dbg = std::getenv("PA_GDL_DBG")) defs.push_back(std::string("-DJIT_DBG=") + dbg);  // (measurement)
  hipFunction_t fn = jit_compile(defs);
  if (!fn) return PA_OK;
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  // descriptors
  JitArgs a;
  std::memset(&a, 0, sizeof(a));
  a.total_tiles = first[ni];
  a.nseg = ni;
  a.nkeys = nkeys;
  a.key_lo = (int)klo;
  a.key_span = (int)kspan;
  a.xcd_major = 1;
  a.key_stride = q->hq.gb_stride[0];
  for (int k = 0; k < na; ++k) {
    a.base[k] = sums[k].base;
    a.step[k] = sums[k].step;
  }
  jit_fill_pointers(q, a);
  std::vector<JitSeg> js(ni);
  for (int k = 0; k < ni; ++k) {
    const int si = inc[k];
    const DevSeg& d = q->hsegs[si];
    JitSeg& j = js[k];
    std::memset(&j, 0, sizeof(j));
    for (int c = 0; c < nc; ++c) j.src[c] = (unsigned long long)(uintptr_t)d.cols[cols[c]].words;
    j.first_tile = first[k];
    j.num_docs = d.num_docs;
    j.num_tiles = (int)(first[k + 1] - first[k]);
    for (int li = 0; li < nl; ++li) {
      j.lo_t[li] = (uint32_t)d.leaves[lit[li]].lo;
      j.hi_t[li] = (uint32_t)d.leaves[lit[li]].span;
      if (lk[li]) {
        j.lut[li] = (unsigned long long)(uintptr_t)d.leaves[lit[li]].lut;
        j.lut_words[li] = (int)q->luts[si][q->literals[lit[li]].leaf].size();
      }
    }
    j.neg = negmask[k];
    j.cls = seg_cls[k];
    j.lbase = lbase[k];
    j.lspan = lspan[k];
    j.gofs = gofs[k];
    if (ktab) {
      const int card = (int)d.cols[cols[kc]].card;
      if (d.remap[0]) {
        j.ktab = (unsigned long long)(uintptr_t)d.remap[0];
      } else {  // (a segment on the table dictionary itself: the identity)
        std::vector<int32_t> id(card);
        for (int i = 0; i < card; ++i) id[i] = i;
        void* dp = nullptr;
        int rc = upload_owned(q, id.data(), id.size() * 4, &dp);
        if (rc) return rc;
        j.ktab = (unsigned long long)(uintptr_t)dp;
      }
      j.ktab_n = card;
    }
    for (int m = 0; m < na; ++m) {
      const Column* c = q->segs[si]->cols.at(s.aggs[sum_aggs[m]].column_id);
      if (sums[m].table) {
        j.tab[m] = (unsigned long long)(uintptr_t)c->dict.p;
        j.tab_n[m] = c->cardinality;
      } else {
        j.aoff[m] = (int)sums[m].aoff[k];
      }
    }
  }
  int rc = dev_alloc(q->jit_args, sizeof(JitArgs));
  if (!rc) rc = dev_alloc(q->jit_segs, sizeof(JitSeg) * js.size());
  if (rc) return rc;
  PA_HIP(hipMemcpy(q->jit_args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(q->jit_segs.p, js.data(), sizeof(JitSeg) * js.size(), hipMemcpyHostToDevice));
  q->jit_fn = fn;
  q->jit_waves = W;
  q->jit_nd = ND;
  q->jit_lds = (int)lds;
  q->jit_grid = G;
  q->jit_nseg = ni;
  q->jit_classes = (int)classes.size();
  q->jit_slots = nslot;
  q->jit_cols = cols;
  PLAN_LOG("gdl_jit: W %d ND %d RS %d RR %d ring %d lmax %d segdrain %d classes %zu slots %d (%zu B) segments %d/%d "
           "ktab %d kib %d lds %zu drain %d",
           W, ND, RS, RR, ring_n, lmax, (int)segdrain, classes.size(), nslot, slot_b, ni, q->nseg, (int)ktab, (int)kib,
           lds, drain);
  return PA_OK;
}

// ---------------------------------------------------------------- count-free partitioned V emit (pve_jit.hip)
// The emit pass of a V-only partitioned plan with one-word records (V_FMT_ID / V_FMT_KEY), dictionary group-by and
// value columns whose segments share the table-wide dictionaries (no remaps), DICT_RANGE filter leaves on staged
// columns and pass C's specialised variant: compiled per shape by hiprtc; each workgroup writes whole chunks of BS
// records into its own region, so no count pass runs (pa_query_scan: pve kernel, chunk lists, pass C).
static const char* kPveJitSrc =
#include "pve_jit_src.inc"
    ;


void pve_fill_pointers(const pa_query::PveStream& st, unsigned long long* matched, PveArgs& a) {
  char* b = (char*)st.buf.p;
  a.recs = (uint32_t*)b;
  a.table = (uint32_t*)(b + st.o_table);
  a.hist = (uint32_t*)(b + st.o_hist);
  a.used = (uint32_t*)(b + st.o_used);
  a.matched = matched;
}

// One record stream's kernel and buffers. V (hmode false): a record per matching doc, rw words (1: key offset | value
// id, 2 / 3: key offset + the raw 32 / 64-bit value staged from a raw column of rawb bytes per doc). H: a record per
// value of the DISTINCTCOUNTHLLMV column. base_parts: partitions the V stream's base array holds room for (Pv + 1 +
// Ph + 1 when both streams run: pass C reads the H bases at base[pv + 1 ..]). Leaves S.fn null when the shape does not
// fit (the count + emit passes run).
static int pve_stream(pa_query* q, const Prep& P, int cus, bool hmode, int rw, int rawb, int64_t base_entries,
                      pa_query::PveStream& S) {
  S.fn = nullptr;
  const pa_query_spec& s = q->spec;
  const DevQuery& h = q->hq;
  // the columns the kernel stages (its own tile image, whatever the planner staged for the count + emit passes): the
  // filter leaves', the group-by columns, the V stream's value-id column — dictionary-encoded SV in every segment
  std::vector<int> slots;
  auto col_of = [&](int slot) {
    for (size_t k = 0; k < slots.size(); ++k)
      if (slots[k] == slot) return (int)k;
    slots.push_back(slot);
    return (int)slots.size() - 1;
  };
  const DevSeg& d0 = q->hsegs[0];
  std::vector<int> lc, ln, le, gc, gs;
  for (int li = 0; li < q->num_eager; ++li) {
    const DevLeaf& L = d0.leaves[li];
    for (const DevSeg& d : q->hsegs)
      if (d.leaves[li].negate != L.negate || d.leaves[li].kind != L.kind || d.leaves[li].slot != L.slot) return PA_OK;
    if (L.kind != PA_LEAF_DICT_RANGE) return PA_OK;
    lc.push_back(col_of(L.slot));
    ln.push_back(L.negate ? 1 : 0);
    le.push_back(L.clause_end ? 1 : 0);
  }
  for (int j = 0; j < s.num_group_by; ++j) {
    if (h.gb_stride[j] <= 0 || h.gb_stride[j] > 0xffffffffll) return PA_OK;
    gc.push_back(col_of(P.gb_slot[j]));
    gs.push_back((int)(uint32_t)h.gb_stride[j]);
  }
  int vc = -1, rslot = -1, mslot = -1, hnb = 1, lg = 0;
  if (!hmode && h.v_fmt == V_FMT_ID) {
    if (h.emit_val_agg < 0) return PA_OK;
    vc = col_of(P.agg_slot[h.emit_val_agg]);
  }
  if (!hmode && rawb) {
    if (h.emit_val_agg < 0) return PA_OK;
    rslot = P.agg_slot[h.emit_val_agg];
  }
  if (hmode) {
    mslot = P.agg_slot[h.hll_agg];
    hnb = d0.cols[mslot].nbits;
    lg = h.aggs[h.hll_agg].log2m;
  }
  const int nc = (int)slots.size();
  if (nc < 1 || nc > 6) return PA_OK;
  int max_values = 1;
  // segments with their own dictionaries: each group-by column's and the value column's dictionary must be a contiguous
  // run of the table-wide one (time partitions, shifted windows), so one offset per segment maps its dictIds
  std::vector<std::array<int32_t, kJitMaxGb>> koff(q->nseg);
  std::vector<int32_t> voff(q->nseg, 0);
  bool any_koff = false, any_voff = false;
  auto run_start = [](const std::vector<int32_t>& rm, int32_t* start) {
    for (size_t i = 0; i < rm.size(); ++i)
      if (rm[i] != rm[0] + (int32_t)i) return false;
    *start = rm.empty() ? 0 : rm[0];
    return true;
  };
  for (int si = 0; si < q->nseg; ++si) {
    const DevSeg& d = q->hsegs[si];
    koff[si].fill(0);
    for (int j = 0; j < s.num_group_by; ++j) {
      if (!d.remap[j]) continue;
      if (!q->has_remap[si][j] || !run_start(q->remaps[si][j], &koff[si][j])) return PA_OK;
      any_koff |= koff[si][j] != 0;
    }
    if (d.vremap && vc >= 0) {  // (the value ids of the V records; the H stream carries none)
      if (si >= (int)q->vremap_host.size() || !run_start(q->vremap_host[si], &voff[si])) return PA_OK;
      any_voff |= voff[si] != 0;
    }
    for (int k = 0; k < nc; ++k) {
      const DevCol& c = d.cols[slots[k]];
      if (c.kind != COL_SV_DICT || !c.words || c.nbits < 1 || c.nbits > 31 || c.nbits != d0.cols[slots[k]].nbits)
        return PA_OK;
    }
    if (rslot >= 0) {
      const DevCol& c = d.cols[rslot];
      if (c.kind != COL_SV_RAW || !c.raw) return PA_OK;
      if (rawb == 4 ? c.vtype != PA_INT : (c.vtype != PA_LONG && c.vtype != PA_DOUBLE)) return PA_OK;
    }
    if (hmode) {
      const DevCol& c = d.cols[mslot];
      if (c.kind != COL_MV_DICT || !c.words || !c.mv_off || c.nbits != hnb || hnb < 1 || hnb > 31 ||
          !d.hll_lut[h.hll_agg])
        return PA_OK;
      max_values = std::max(max_values, q->segs[si]->cols.at(s.aggs[h.hll_agg].column_id)->max_values);
    }
  }
  if ((uint64_t)q->num_keys > 0xffffffffull) return PA_OK;
  const int Pn = hmode ? h.num_parts - h.pv : h.pv;
  const int ks = hmode ? h.kshift_h : h.kshift_v;
  if (Pn < 1 || Pn > 4096 || ks < 1) return PA_OK;
  // tile image of nd docs per lane (64 nd per tile): a 16-byte guard, then per column its tile's bits (8 nd nb bytes)
  // and a 16-byte guard, then the raw values (64 nd rawb bytes). 16 docs per lane unless 8 leave room for more
  // resident waves (PA_PVE_ND: measurement); 32-record bins unless 16 do (H: many partitions)
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  auto image_bytes = [&](int nd) {
    size_t b = 16;
    for (int k = 0; k < nc; ++k) b += (size_t)8 * nd * d0.cols[slots[k]].nbits + 16;
    return b + (size_t)64 * nd * rawb;
  };
  auto lds_ring = [&](int bs) { return al16(al16((size_t)(5 * Pn + 1) * 4) + (size_t)Pn * bs * rw * 4); };
  // H: a wave's buffer for one tile's MV value words (stage_values: at most max_values values per doc, whole 16-byte
  // chunks from a 16-byte aligned start, one word of look-ahead; the run rounds read a window of up to 9 words)
  auto val_bytes = [&](int nd) {
    return hmode ? (size_t)16 * (((size_t)max_values * 64 * nd * hnb / 32 + 17 + 3) / 4) : (size_t)0;
  };
  // H run rounds: one claim per run of up to hb values of one doc (its values share the doc's key); hb = the column's
  // most values per doc up to 8, so a run is normally a whole doc. PA_PVE_HRUN=0 keeps one claim per value
  // (measurement), PA_PVE_HB sets the run length
  bool hrun = true;
  if (const char* e = std::getenv("PA_PVE_HRUN")) hrun = std::atoi(e) != 0;
  int hb = (int)std::max<int64_t>(1, std::min<int64_t>(8, max_values));
  if (const char* e = std::getenv("PA_PVE_HB")) hb = std::max(1, std::min(8, std::atoi(e)));
  // tile images per wave (PA_PVE_RING: measurement; the H stream and admission loads keep two)
  int rn = 2;
  if (const char* e = std::getenv("PA_PVE_RING")) rn = std::max(2, std::min(4, std::atoi(e)));
  if (hmode || q->limit_walk) rn = 2;
  // compacted put rounds: a queue of 512 records (partition + record words) per wave, for a V stream whose filter is
  // expected to keep less than half the docs (configs[2] 10 %: 0.409 vs 0.496 ms per 200M docs; on every doc it costs
  // resident waves: 1.38 vs 1.20 ms, and the H stream's uneven MV runs gain nothing: 5.26 vs 3.89 ms). PA_PVE_Q=0 / 1
  // forces it (measurement)
  bool pq = !hmode && P.has_filter && P.post_density < 0.5 * (double)kWTileDocs;
  if (const char* e = std::getenv("PA_PVE_Q")) pq = std::atoi(e) != 0;
  const size_t qbytes = pq ? (size_t)4 * 512 * (rw + 1) : 0;
  auto waves_for = [&](int nd, int bs) {
    for (int cand : {16, 12, 8, 4})
      if (lds_ring(bs) + (size_t)cand * (rn * image_bytes(nd) + val_bytes(nd) + qbytes) <= kLdsBudget) return cand;
    return 0;
  };
  // H: 8 docs per lane (a lane's run of MV values is half as long: measured 3.97 vs 4.8 ms on configs[4]); 32-record
  // bins (16-record bins for more resident waves measured slower on both streams: V 1.70 vs 1.33 ms at 12 vs 8 waves,
  // H 4.37 vs 3.97 ms at 16 vs 12 waves), 16 only when 32 leave fewer than 8 waves
  int bs = 32;
  if (waves_for(8, 32) < 8 && waves_for(8, 16) > waves_for(8, 32)) bs = 16;
  int nd = hmode ? 8 : (waves_for(8, bs) > waves_for(16, bs) ? 8 : 16);
  if (const char* e = std::getenv("PA_PVE_ND")) nd = std::atoi(e) == 8 ? 8 : 16;
  if (const char* e = std::getenv("PA_PVE_BS")) bs = std::atoi(e) == 16 ? 16 : 32;  // (measurement)
  const int w = waves_for(nd, bs);
  if (!w) return PA_OK;
  std::vector<int> nb, coff;
  size_t img_bytes = 16;
  for (int k = 0; k < nc; ++k) {
    nb.push_back(d0.cols[slots[k]].nbits);
    coff.push_back((int)img_bytes);
    img_bytes += (size_t)8 * nd * nb.back() + 16;
  }
  const size_t raw_off = img_bytes;
  img_bytes += (size_t)64 * nd * rawb;
  const int img_dw = (int)(img_bytes / 4);
  const int td = 64 * nd;
  const size_t l_bins = al16((size_t)(5 * Pn + 1) * 4);
  const size_t l_ring = lds_ring(bs);
  const size_t l_val = l_ring + (size_t)w * rn * img_bytes;
  const size_t vbytes = val_bytes(nd);
  const size_t l_q = l_val + (size_t)w * vbytes;
  const size_t lds = l_q + (size_t)w * qbytes;
  // one workgroup per CU; a workgroup's region holds its docs' records (H: at most max_values per doc) in whole chunks
  // plus one partial chunk per partition; chunks of sc bins, more when the region would need 2^16 chunks
  std::vector<int64_t> first(q->nseg + 1, 0);  // the kernel's own tiles of td docs
  for (int si = 0; si < q->nseg; ++si) first[si + 1] = first[si] + (q->hsegs[si].num_docs + td - 1) / td;
  const int64_t T = first[q->nseg];
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (T + w - 1) / w));
  const int64_t recs_per_wg = (T + G - 1) / G * td * (int64_t)max_values;
  // chunks of 8 bins (4: configs[2] 1.215 vs 1.192 ms, configs[4] 7.49 vs 7.40 ms; PA_PVE_SC: measurement)
  int sc = std::getenv("PA_PVE_SC") ? std::atoi(std::getenv("PA_PVE_SC")) : 8;
  if (sc < 1 || sc > 16 || (sc & (sc - 1))) return PA_OK;  // (bins - 1 of a chunk: 4 bits of its list entry)
  auto chunks_for = [&](int c) { return (recs_per_wg + (int64_t)bs * c - 1) / ((int64_t)bs * c) + Pn; };
  while (sc < 16 && chunks_for(sc) >= (int64_t(1) << 16)) sc *= 2;
  const int64_t cr = (int64_t)bs * sc;  // records per chunk
  if (cr < 64) return PA_OK;             // (pass C: a wave's 64 records of one slot lie in one chunk)
  const int64_t C = chunks_for(sc);
  if (C >= (int64_t(1) << 16) || (int64_t)G * C >= (int64_t(1) << 28)) return PA_OK;  // (table ranks, chunk ids)
  auto pad1 = [](std::vector<int> v) {
    if (v.empty()) v.push_back(0);
    return v;
  };
  std::string gss = "{";
  for (size_t j = 0; j < gs.size(); ++j) gss += (j ? "," : "") + std::to_string((uint32_t)gs[j]) + "u";
  gss += "}";
  std::vector<std::string> defs = {
      "-DPVE_W=" + std::to_string(w), "-DPVE_IMG=" + std::to_string(img_dw), "-DPVE_ND=" + std::to_string(nd),
      "-DPVE_NC=" + std::to_string(nc), "-DPVE_NB=" + int_list(nb), "-DPVE_OFF=" + int_list(coff),
      "-DPVE_NL=" + std::to_string(q->num_eager), "-DPVE_LC=" + int_list(pad1(lc)), "-DPVE_LN=" + int_list(pad1(ln)),
      "-DPVE_LE=" + int_list(pad1(le)), "-DPVE_NG=" + std::to_string(s.num_group_by), "-DPVE_GC=" + int_list(gc),
      "-DPVE_GS=" + gss, "-DPVE_VC=" + std::to_string(vc), "-DPVE_KS=" + std::to_string(ks),
      "-DPVE_P=" + std::to_string(Pn), "-DPVE_BS=" + std::to_string(bs), "-DPVE_SC=" + std::to_string(sc),
      "-DPVE_L_BINS=" + std::to_string(l_bins), "-DPVE_ADMIT=" + std::to_string(q->limit_walk ? 1 : 0),
      "-DPVE_L_RING=" + std::to_string(l_ring), "-DPVE_RW=" + std::to_string(rw),
      "-DPVE_RAWB=" + std::to_string(rawb), "-DPVE_RAWOFF=" + std::to_string(raw_off),
      "-DPVE_H=" + std::to_string(hmode ? 1 : 0), "-DPVE_HNB=" + std::to_string(hnb), "-DPVE_LG=" + std::to_string(lg),
      "-DPVE_L_VAL=" + std::to_string(l_val), "-DPVE_VAL_B=" + std::to_string(vbytes),
      "-DPVE_KOFF=" + std::to_string(any_koff ? 1 : 0), "-DPVE_VOFF=" + std::to_string(any_voff ? 1 : 0),
      "-DPVE_KR=" + std::to_string(hmode ? 0 : h.part_kr_v), "-DPVE_RING=" + std::to_string(rn), "-DPVE_Q=" + std::to_string(pq ? 1 : 0),
      "-DPVE_L_Q=" + std::to_string(l_q), "-DPVE_HRUN=" + std::to_string(hmode && hrun ? 1 : 0),
      "-DPVE_HB=" + std::to_string(hb)};
  if (const char* dbg = std::getenv("PA_PVE_DBG")) defs.push_back(std::string("-DPVE_DBG=") + dbg);  // (measurement)
  if (const char* pb = std::getenv("PA_PVE_PB")) defs.push_back(std::string("-DPVE_PB=") + pb);      // (measurement)
  if (std::getenv("PA_PVE_DONE_RTN")) defs.push_back("-DPVE_DONE_RTN=1");                            // (measurement)
  hipFunction_t fn = jit_compile(defs, kPveJitSrc, "pve_jit");
  if (!fn) return PA_OK;
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const size_t o_table = al16((size_t)G * C * cr * rw * 4);
  const size_t o_hist = al16(o_table + (size_t)G * C * 4);
  const size_t o_used = al16(o_hist + (size_t)G * Pn * 4);
  const size_t o_off = al16(o_used + (size_t)G * 4);
  const size_t o_base = al16(o_off + (size_t)G * Pn * 4);
  const size_t o_index = al16(o_base + (size_t)std::max<int64_t>(base_entries, Pn + 1) * 8);
  const size_t o_tot = al16(o_index + (size_t)G * C * 4);
  const size_t total = o_tot + (size_t)Pn * 4;
  int rc = dev_alloc(S.buf, total);
  if (rc) return rc;
  S.o_table = o_table;
  S.o_hist = o_hist;
  S.o_used = o_used;
  S.o_off = o_off;
  S.o_base = o_base;
  S.o_index = o_index;
  S.o_tot = o_tot;
  PveArgs a;
  std::memset(&a, 0, sizeof(a));
  a.total_tiles = T;
  a.nseg = q->nseg;
  a.xcd_major = 1;
  a.chunks_per_wg = C;
  pve_fill_pointers(S, q->hq.matched_docs, a);
  std::vector<PveSeg> js(q->nseg);
  for (int si = 0; si < q->nseg; ++si) {
    const DevSeg& d = q->hsegs[si];
    PveSeg& j = js[si];
    std::memset(&j, 0, sizeof(j));
    for (int c = 0; c < nc; ++c) j.src[c] = (uint64_t)(uintptr_t)d.cols[slots[c]].words;
    j.first_tile = first[si];
    j.num_docs = d.num_docs;
    j.num_tiles = (int32_t)(first[si + 1] - first[si]);
    for (int li = 0; li < q->num_eager; ++li) {
      j.lo_t[li] = (uint32_t)d.leaves[li].lo;
      j.hi_t[li] = (uint32_t)d.leaves[li].span;
    }
    j.admit = (uint64_t)(uintptr_t)d.admit;
    for (int g = 0; g < s.num_group_by; ++g) j.koff[g] = koff[si][g];
    j.voff = voff[si];
    if (rslot >= 0) j.raw = (uint64_t)(uintptr_t)d.cols[rslot].raw;
    if (hmode) {
      j.mv_off = (uint64_t)(uintptr_t)d.cols[mslot].mv_off;
      j.mv_words = (uint64_t)(uintptr_t)d.cols[mslot].words;
      j.hlut = (uint64_t)(uintptr_t)d.hll_lut[h.hll_agg];
    }
  }
  rc = dev_alloc(S.args, sizeof(PveArgs));
  if (!rc) rc = dev_alloc(S.segs, sizeof(PveSeg) * js.size());
  if (rc) return rc;
  PA_HIP(hipMemcpy(S.args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(S.segs.p, js.data(), sizeof(PveSeg) * js.size(), hipMemcpyHostToDevice));
  S.fn = fn;
  S.waves = w;
  S.grid = G;
  S.lds = (int)lds;
  S.cr = (int)cr;
  S.parts = Pn;
  S.bin_shift = __builtin_ctz((unsigned)bs);
  S.chunks = C;
  PLAN_LOG("pve %s: W %d nd %d bs %d sc %d queue %d runs %d grid %d lds %zu C %lld P %d", hmode ? "H" : "V", w, nd, bs,
           sc, (int)pq, hmode && hrun ? hb : 0, G, lds,
           (long long)C, Pn);
  return PA_OK;
}

// Pass C runs one workgroup per V partition, one per CU (its LDS accumulators): a partition count just past a whole
// number of rounds leaves a round of a few full partitions at the end (configs[2] over segments with their own
// dictionaries: 1031 x 1025 keys, 259 partitions of 4096 keys on 256 CUs, pass C 839 vs 488 us for 256). The count-free
// emit divides a key by a constant, so its partitions need not hold a power of two keys: ceil(K / (rounds x CUs)) keys
// each, in as few rounds as pass C's LDS allows. The record keeps the key offset in ceil(log2) bits. Returns whether
// the V partitions changed (q->hq and pass C's LDS layout rewritten).
static bool pve_repartition(pa_query* q, const Prep& P, int cus) {
  DevQuery& h = q->hq;
  const pa_query_spec& s = q->spec;
  if (h.hll_agg >= 0 || h.pv <= cus || std::getenv("PA_PVE_POW2")) return false;  // (PA_PVE_POW2: measurement)
  size_t per_key = 4;  // pass C's LDS per key: u32 count, then each aggregation's slot
  for (int a = 0; a < s.num_aggs; ++a) {
    const int t = s.aggs[a].type;
    if (t == PA_AGG_COUNT || t == PA_AGG_DISTINCTCOUNTHLL) continue;
    per_key += (t == PA_AGG_SUM && P.agg_src[a] == SRC_LONG) ? 16 : 8;
  }
  // (the whole LDS unless the query asked for a smaller pass C, PA_QF_PART_SHIFT)
  const int choice = (s.flags >> PA_QF_PART_SHIFT) & 3;
  const size_t budget = choice ? kPartLdsChoices[choice] : kLdsBudget;
  const int64_t K = q->num_keys, rounds = (h.pv + cus - 1) / cus;
  for (int64_t r = 1; r < rounds; ++r) {
    const int64_t kr = (K + r * cus - 1) / (r * cus);
    if (kr < 2 || kr >= (int64_t(1) << 30) || (size_t)kr * per_key + 16 > budget) continue;
    const int ks = 64 - __builtin_clzll((unsigned long long)(kr - 1));
    if (h.v_fmt == V_FMT_ID && q->v_id_bits + ks > 31) continue;
    const int32_t pv = (int32_t)((K + kr - 1) / kr);
    h.pv = h.num_parts = h.part_hi = pv;
    h.kshift_v = ks;
    h.part_kr_v = (int32_t)kr;
    size_t lv = ((size_t)kr * 4 + 15) & ~(size_t)15;  // (as plan_partitioned: counts, then the accumulators)
    for (int a = 0; a < s.num_aggs; ++a) {
      const int t = s.aggs[a].type;
      if (t == PA_AGG_COUNT || t == PA_AGG_DISTINCTCOUNTHLL) continue;
      h.aggs[a].lds_off = (int32_t)lv;
      lv += (size_t)kr * ((t == PA_AGG_SUM && P.agg_src[a] == SRC_LONG) ? 16 : 8);
    }
    q->part_lds_c = (int)lv;
    PLAN_LOG("pve: V partitions of %lld keys (%d partitions, pass C lds %zu)", (long long)kr, pv, lv);
    return true;
  }
  return false;
}

int pve_plan(pa_query* q, const Prep& P, int cus) {
  q->pve.fn = q->pvh.fn = nullptr;
  const pa_query_spec& s = q->spec;
  const DevQuery& h = q->hq;
  if (!q->partitioned || q->limit_mode || q->hashed) return PA_OK;
  if (q->limit_walk && h.gb_mv >= 0) return PA_OK;
  if ((s.flags & PA_QF_NO_JIT) || (s.flags2 & PA_QF2_NO_COUNT_FREE) || std::getenv("PA_NO_JIT") ||
      (std::getenv("PA_DEBUG_EMIT") && !std::getenv("PA_PVE_DBG")))
    return PA_OK;
  // both streams (DISTINCTCOUNTHLLMV next to a V stream): two launches, COUNT from the V records
  const bool hstream = h.hll_agg >= 0;
  if (hstream && (!q->split_emit || h.h_first || h.gb_mv >= 0)) return PA_OK;
  if (!hstream && q->split_emit) return PA_OK;
  int rw = 1, rawb = 0;
  if (h.v_fmt == V_FMT_32 || h.v_fmt == V_FMT_64) {  // raw value columns only (dictionary values: V_FMT_ID)
    rw = h.v_fmt == V_FMT_32 ? 2 : 3;
    rawb = h.v_fmt == V_FMT_32 ? 4 : 8;
  } else if (h.v_fmt != V_FMT_ID && h.v_fmt != V_FMT_KEY) {
    return PA_OK;
  }
  if (h.rec_words_v != rw || q->part_vk == kVkGeneric) return PA_OK;
  if (q->nseg == 0 || s.num_group_by < 1 || s.num_group_by > 4 || q->num_eager != (int)q->literals.size() ||
      q->num_eager > 6 || h.pv > 4096 || h.kshift_v < 1)
    return PA_OK;
  const DevQuery saved = q->hq;
  const int saved_lds_c = q->part_lds_c;
  const bool repart = !hstream && pve_repartition(q, P, cus);
  const int64_t base_entries = (int64_t)h.pv + 1 + (hstream ? (int64_t)(h.num_parts - h.pv) + 1 : 0);
  int rc = pve_stream(q, P, cus, false, rw, rawb, base_entries, q->pve);
  if (repart) {
    if (rc || !q->pve.fn) {  // (the generic emit runs power-of-two partitions)
      q->hq = saved;
      q->part_lds_c = saved_lds_c;
    } else {
      PA_HIP(hipMemcpy(q->dq.p, &q->hq, sizeof(DevQuery), hipMemcpyHostToDevice));
      PA_HIP(set_part_agg_lds_limit(q->part_vk, q->part_lds_c));
    }
  }
  if (rc || !q->pve.fn || !hstream) return rc;
  rc = pve_stream(q, P, cus, true, 1, 0, 0, q->pvh);
  if (rc || !q->pvh.fn) q->pve.fn = nullptr;  // (both streams or neither: the count pass serves both)
  return rc;
}
