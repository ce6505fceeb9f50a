// Query planning, second half: tile geometry, partitions, the kernel variant and occupancy, the scan descriptors,
// scratch, numGroupsLimit buffers and the fused statistics' buffers.
#include "pa_host.h"


TilePlan plan_tiles(const pa_query* q, const std::vector<DevSeg>& segs, int strat, bool use_lm, size_t acc_b,
                    bool only16) {
  const int wpw = scan_waves(strat);  // waves per workgroup of this kernel variant
  const pa_query_spec& s = q->spec;
  const int force_ring = (s.flags >> PA_QF_RING_SHIFT) & 15;
  const int force_wg = (s.flags >> PA_QF_WG_SHIFT) & 7;
  TilePlan best;
  for (int steps : {32, 16}) {
    if (use_lm && steps != 32) continue;
    if (only16 && steps != 16) continue;
    if ((s.flags & PA_QF_STEPS16) && steps != 16) continue;
    if ((s.flags & PA_QF_STEPS32) && steps != 32) continue;
    int img_dw = kGuardWords, dma = 0;
    for (const DevSeg& d : segs) {
      int dw = kGuardWords, n = 0;
      for (int k = 0; k < d.num_staged; ++k) {
        const int nb = d.stage[k].nbits;
        dw += 2 * steps * nb + kGuardWords;
        n += ((steps / 2) * nb + 63) / 64;
      }
      img_dw = std::max(img_dw, dw);
      dma = std::max(dma, n);
    }
    const size_t img_bytes = (size_t)img_dw * 4;
    for (int wg : {4, 3, 2, 1}) {
      if (force_wg && wg != force_wg) continue;
      const size_t per_wg = kLdsBudget / wg;
      if (per_wg <= acc_b) continue;
      int ring = (int)((per_wg - acc_b) / (wpw * img_bytes));
      ring = std::min(ring, 8);
      if (force_ring) {
        if (force_ring > ring) continue;
        ring = force_ring;
      }
      if (ring < 2) continue;
      const size_t lds = acc_b + (size_t)wpw * ring * img_bytes;
      int resident = 0;
      if (set_scan_lds_limit(strat, steps, use_lm, (int)kLdsBudget) != hipSuccess ||
          scan_occupancy(strat, steps, use_lm, (int)lds, &resident) != hipSuccess)
        resident = wg;  // no device to ask (planning only): trust the LDS arithmetic
      if (resident < wg) continue;
      const double inflight = (double)wg * wpw * (ring - 1) * img_bytes;
      const double score = 1e7 * wg * wpw / kWavesPerWG + (steps == 32 ? 1e6 : 0) + std::min(inflight, 128.0 * 1024);
      if (score > best.score) best = TilePlan{steps, dma, ring, wg, img_dw, lds, score};
    }
  }
  return best;
}

// Table-wide dictionary of an aggregation's value column (V_FMT_ID records carry a value id): segment 0's device
// dictionary when every segment holds the same dictionary, else the sorted union with per-segment dictId remaps.
// Returns the value-id bits, or -1 when the column is not dictionary-encoded everywhere.
// An INT/LONG dictionary whose values are base + step * id (an arithmetic progression, e.g. a dense range): pass C then
// computes a value from its id instead of gathering it.
uint64_t max_abs_value(const std::vector<uint64_t>& v, int32_t vtype) {
  if (vtype != PA_INT && vtype != PA_LONG) return 0;
  uint64_t m = 0;
  for (uint64_t x : v) {
    const int64_t y = (int64_t)x;
    if (y == INT64_MIN) return 0;
    m = std::max<uint64_t>(m, (uint64_t)(y < 0 ? -y : y));
  }
  return m;
}

bool affine_dictionary(const std::vector<uint64_t>& v, int32_t vtype, int64_t* base, int64_t* step) {
  if (v.empty() || (vtype != PA_INT && vtype != PA_LONG)) return false;
  const int64_t b = (int64_t)v[0];
  const int64_t st = v.size() > 1 ? (int64_t)(v[1] - v[0]) : 0;
  for (size_t i = 1; i < v.size(); ++i)
    if ((uint64_t)v[i] - (uint64_t)v[i - 1] != (uint64_t)st) return false;
  *base = b;
  *step = st;
  return true;
}

int value_dictionary(pa_query* q, const Prep& P, int a, const uint64_t** vdict) {
  const pa_query_spec& s = q->spec;
  const int32_t cid = s.aggs[a].column_id;
  const Column* c0 = q->segs[0]->cols.at(cid);
  if (c0->kind != COL_SV_DICT || c0->hvals.empty()) return -1;
  bool same = true;
  for (int si = 0; si < q->nseg; ++si) {
    const Column* c = q->segs[si]->cols.at(cid);
    if (c->kind != COL_SV_DICT || c->hvals.empty() || c->vtype != c0->vtype) return -1;
    same = same && (c == c0 || (c->dict_hash == c0->dict_hash && c->hvals == c0->hvals));
  }
  for (int si = 0; si < q->nseg; ++si) q->hsegs[si].vremap = nullptr;
  q->vremap_host.assign(q->nseg, {});
  q->hq.v_affine = 0;
  q->hq.v_maxabs = 0;
  if (same) {
    *vdict = (const uint64_t*)c0->dict.p;
    q->hq.v_maxabs = max_abs_value(c0->hvals, c0->vtype);
    int64_t b = 0, st = 0;
    if (affine_dictionary(c0->hvals, c0->vtype, &b, &st)) {
      q->hq.v_affine = 1;
      q->hq.v_base = b;
      q->hq.v_step = st;
    }
    return std::max(1, 32 - __builtin_clz((uint32_t)std::max(1, c0->cardinality - 1)));
  }
  const int32_t vt = c0->vtype;
  std::vector<std::pair<int64_t, uint64_t>> all;  // (order key, value bits)
  for (int si = 0; si < q->nseg; ++si)
    for (uint64_t v : q->segs[si]->cols.at(cid)->hvals) all.push_back({value_order_key(v, vt), v});
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end(), [](const auto& x, const auto& y) { return x.first == y.first; }),
            all.end());
  if (all.size() > (size_t)INT32_MAX) return -1;
  std::vector<uint64_t> uni(all.size());
  std::vector<int64_t> keys(all.size());
  for (size_t i = 0; i < all.size(); ++i) {
    keys[i] = all[i].first;
    uni[i] = all[i].second;
  }
  void* dp = nullptr;
  if (upload_owned(q, uni.data(), uni.size() * 8, &dp)) return -2;
  *vdict = (const uint64_t*)dp;
  q->hq.v_maxabs = max_abs_value(uni, vt);
  {
    int64_t b = 0, st = 0;
    if (affine_dictionary(uni, vt, &b, &st)) {
      q->hq.v_affine = 1;
      q->hq.v_base = b;
      q->hq.v_step = st;
    }
  }
  for (int si = 0; si < q->nseg; ++si) {
    const Column* c = q->segs[si]->cols.at(cid);
    std::vector<int32_t> rm(c->hvals.size());
    for (size_t i = 0; i < rm.size(); ++i)
      rm[i] = (int32_t)(std::lower_bound(keys.begin(), keys.end(), value_order_key(c->hvals[i], vt)) - keys.begin());
    void* rp = nullptr;
    if (upload_owned(q, rm.data(), rm.size() * 4, &rp)) return -2;
    q->hsegs[si].vremap = (const int32_t*)rp;
    q->vremap_host[si] = std::move(rm);
  }
  (void)P;
  return std::max(1, 64 - __builtin_clzll((unsigned long long)std::max<size_t>(1, uni.size() - 1)));
}

// The staging of the count pass: the main pass's staged filter columns plus the group-by columns — no value columns.
std::vector<DevSeg> count_pass_segments(const pa_query* q, const Prep& P) {
  std::vector<DevSeg> out = q->hsegs;
  const int nslots = (int)q->slot_cols.size();
  for (DevSeg& d : out) {
    d.num_staged = 0;
    for (int sl = 0; sl < nslots; ++sl) {
      DevCol& dc = d.cols[sl];
      if (dc.lds_off < 0) continue;
      bool filter_col = false;
      for (size_t li = 0; li < q->literals.size(); ++li) filter_col |= d.leaves[li].slot == sl;
      bool gb_col = false;  // a group-by column the count pass decodes
      for (int j = 0; j < q->spec.num_group_by; ++j) gb_col |= P.gb_slot[j] == sl && j != q->count_skip;
      if (gb_col || filter_col) {
        d.stage[d.num_staged++] = StageDesc{dc.words, dc.nbits, 0};
      } else {
        dc.lds_off = -1;
      }
    }
    for (size_t li = 0; li < q->literals.size(); ++li) d.leaves[li].lds_off = d.cols[d.leaves[li].slot].lds_off;
  }
  return out;
}

// Partitioned aggregation plan (BASELINE configs[2] / configs[4]): streams, record formats, key partitioning, bins,
// LDS of the three kernels. Returns false when the query does not fit it (the per-doc global-atomic path runs).
bool plan_partitions(pa_query* q, Prep& P, TilePlan& emit_plan, TilePlan& count_plan) {
  const pa_query_spec& s = q->spec;
  const int64_t K = q->num_keys;
  DevQuery& h = q->hq;
  int hll = -1;
  int nv = 0;
  size_t per_key_v = 4;  // u32 count
  for (int a = 0; a < s.num_aggs; ++a) {
    const int t = s.aggs[a].type;
    if (t == PA_AGG_COUNT) continue;
    if (t == PA_AGG_COUNT_MV || t == PA_AGG_DISTINCTCOUNT) { PLAN_LOG("partitioned: no (exit 1)"); return false; }
    if (t == PA_AGG_DISTINCTCOUNTHLL) {
      if (hll >= 0) { PLAN_LOG("partitioned: no (exit 2)"); return false; }  // one H stream per query
      hll = a;
      continue;
    }
    if (P.agg_mv[a]) { PLAN_LOG("partitioned: no (exit 3)"); return false; }
    per_key_v += (t == PA_AGG_SUM && P.agg_src[a] == SRC_LONG) ? 16 : 8;
    ++nv;
  }
  const bool vstream = nv > 0 || hll < 0;
  // a multi-value group-by column: one V record per (doc, value) pair (V stream only; one such column, multi-value in
  // every segment)
  const int mvc = mv_group_component(q);
  if (mvc == -2 || (mvc >= 0 && hll >= 0)) { PLAN_LOG("partitioned: no (exit 10)"); return false; }
  // V record format: one payload slot per distinct (column, value source); SUM/MIN/MAX of one column share it
  std::vector<int> pay(s.num_aggs, 0);
  int words = 1, slots = 0, va = -1;
  for (int a = 0; a < s.num_aggs; ++a) {
    const int t = s.aggs[a].type;
    if (t == PA_AGG_COUNT || t == PA_AGG_DISTINCTCOUNTHLL) continue;
    int shared = -1;
    for (int b = 0; b < a; ++b)
      if (s.aggs[b].type != PA_AGG_COUNT && s.aggs[b].type != PA_AGG_DISTINCTCOUNTHLL && P.agg_slot[b] == P.agg_slot[a] &&
          P.agg_src[b] == P.agg_src[a])
        shared = pay[b];
    if (shared >= 0) {
      pay[a] = shared;
    } else {
      pay[a] = words;
      words += P.agg_src[a] == SRC_INT ? 1 : 2;
      ++slots;
      if (va < 0) va = a;
    }
  }
  const uint64_t* vdict = nullptr;
  const int vbits = (slots == 1 && P.val_fast[va]) ? value_dictionary(q, P, va, &vdict) : -1;
  if (vbits == -2) { PLAN_LOG("partitioned: no (exit 6)"); return false; }  // (allocation failure: reported by pa_last_error)
  // specialised V pass C: one payload, at most one SUM / MIN / MAX
  h.vop_sum = h.vop_min = h.vop_max = -1;
  bool vk_fast = vstream && slots <= 1;
  for (int a = 0; a < s.num_aggs && vk_fast; ++a) {
    const int t = s.aggs[a].type;
    int32_t* slot = t == PA_AGG_SUM ? &h.vop_sum : (t == PA_AGG_MIN ? &h.vop_min : (t == PA_AGG_MAX ? &h.vop_max : nullptr));
    if (t == PA_AGG_COUNT || t == PA_AGG_DISTINCTCOUNTHLL) continue;
    if (!slot || *slot >= 0) vk_fast = false;
    else *slot = a;
  }
  // value ids in value order: the table-wide union is sorted; a shared segment dictionary is checked
  bool sorted_ids = false;
  if (vbits > 0) {
    sorted_ids = true;
    const Column* c0 = q->segs[0]->cols.at(s.aggs[va].column_id);
    if (q->hsegs[0].vremap == nullptr)
      for (size_t i = 1; i < c0->hvals.size() && sorted_ids; ++i)
        sorted_ids = value_order_key(c0->hvals[i - 1], c0->vtype) < value_order_key(c0->hvals[i], c0->vtype);
  }
  // (pass C's MIN/MAX slots stay 8 bytes even when they hold 4-byte value ids: sizing them at 4 bytes doubles the keys
  // per partition and halves pass C's workgroups, measured slower on configs[2] with 64-bit values, r02_v6)
  const size_t part_lds = kPartLdsChoices[(s.flags >> PA_QF_PART_SHIFT) & 3];
  auto max_keys = [&](size_t per_key) {  // largest power-of-two key range whose accumulators fit pass C's LDS
    int64_t kr = 1;
    while ((size_t)(kr * 2) * per_key <= part_lds && kr < K) kr *= 2;
    return kr;
  };
  // records each stream carries when every doc matches (dense plans): one per doc (V), one per HLL value (H)
  uint64_t hrecs = 0;
  if (hll >= 0)
    for (const pa_segment* seg : q->segs) {
      const Column* c = seg->cols.at(s.aggs[hll].column_id);
      hrecs += c->kind == COL_MV_DICT ? (uint64_t)c->total_values : (uint64_t)seg->num_docs;
    }
  int64_t kr_v = 0, kr_h = 0, Pv = 0, Ph = 0;
  if (hll >= 0) {
    const int lg = s.aggs[hll].log2m;
    kr_h = max_keys(((size_t)1 << lg) + (vstream ? 0 : 4));
    Ph = (K + kr_h - 1) / kr_h;
    const int ksh = __builtin_ctzll((uint64_t)kr_h);
    if (ksh + lg + 6 > 32) { PLAN_LOG("partitioned: no (exit 4)"); return false; }  // H record: key offset | register | rank | first in 32 bits
  }
  if (vstream) {
    kr_v = max_keys(per_key_v);
    if (hll >= 0) {
      // as many records per V partition as per H partition (pass C's workgroups take about equally long)
      const double want = std::max(1.0, (double)Ph * (double)q->num_docs / (double)std::max<uint64_t>(1, hrecs));
      while (kr_v > 1 && (double)((K + kr_v - 1) / kr_v) < want / 1.5) kr_v /= 2;
    } else {
      // at least kMinParts partitions (pass C runs one workgroup each) unless that takes them below 256 keys
      while (kr_v > 256 && (K + kr_v - 1) / kr_v < kMinParts) kr_v /= 2;
    }
    Pv = (K + kr_v - 1) / kr_v;
  }
  if (Pv + Ph < 2 || Pv + Ph > kMaxParts) { PLAN_LOG("partitioned: no (exit 5)"); return false; }
  const int ksv = vstream ? __builtin_ctzll((uint64_t)kr_v) : 0;
  int fmt = V_FMT_KEY, W = 1;
  if (slots == 1) {
    if (vbits > 0 && vbits + ksv <= 31) {
      fmt = V_FMT_ID;
      W = 1;
    } else if (!P.val_fast[va]) {
      fmt = V_FMT_GEN;
      W = words;
    } else {
      fmt = P.agg_src[va] == SRC_INT ? V_FMT_32 : V_FMT_64;
      W = fmt == V_FMT_32 ? 2 : 3;
    }
    if (fmt != V_FMT_ID)
      for (int si = 0; si < q->nseg; ++si) q->hsegs[si].vremap = nullptr;
  } else if (slots > 1) {
    fmt = V_FMT_GEN;
    W = words;
  }
  if (W > kMaxVWords) { PLAN_LOG("partitioned: no (exit 7)"); return false; }
  if (mvc >= 0 && fmt == V_FMT_GEN) { PLAN_LOG("partitioned: no (exit 12)"); return false; }
  // bins: a full bin is whole 128-byte lines (V: BS * W * 4 bytes; H: 32 four-byte records)
  int bs_v = vstream ? 128 / std::gcd(128, 4 * W) : 0;
  int bs_h = hll >= 0 ? 32 : 0;
  const int Ptot = (int)(Pv + Ph);
  auto emit_state = [&](int bv, int bh) {
    size_t b = (size_t)Ptot * 16 + (size_t)Ph * 4 + (size_t)Ptot * 8;  // cnt, done, front, back, H slack + start
    b = (b + 15) & ~(size_t)15;
    b += (size_t)Pv * bv * W * 4 + (size_t)Ph * (bh ? bh + kDocVals : 0) * 4;  // H bins: + a crossing doc's tail
    return (b + 15) & ~(size_t)15;
  };
  // the emit pass stages its columns in a ring next to the bins: halve the bins (down to 64-byte bursts) while they
  // do not fit or cost resident waves (at least two workgroups per CU hide the per-record gathers)
  // both streams: two emit launches (V, then H), each holding only its own stream's bins
  const bool split = vstream && hll >= 0 && !(s.flags & PA_QF_NO_SPLIT_EMIT);
  q->split_emit = split;
  // Each launch: 4-wave or 16-wave workgroups (the bins are per workgroup: shared by 16 waves they leave LDS for more
  // resident waves when the tile images are small), whichever keeps more waves resident; bins halve (down to 64-byte
  // bursts) while they do not fit or cost resident waves (at least 8 waves per CU hide the per-record gathers).
  // resident waves per CU the emit plan wants before it keeps larger bins (PA_EMIT_MIN_WAVES: measurement override)
  static const int emit_min_waves = std::getenv("PA_EMIT_MIN_WAVES") ? std::atoi(std::getenv("PA_EMIT_MIN_WAVES"))
                                                                      : 2 * kWavesPerWG;
  auto plan_emit = [&](int vf, int hh, bool with_v, bool with_h, int& bv, int& bh, int& strat) {
    auto lds_of = [&](int v, int h2) { return emit_state(with_v ? v : 0, with_h ? h2 : 0); };
    TilePlan best;
    int best_bv = bv, best_bh = bh;
    static const int force_big = std::getenv("PA_EMIT_BIG") ? std::atoi(std::getenv("PA_EMIT_BIG")) : -1;  // (measurement)
    for (int big : {0, 1}) {
      if (force_big >= 0 && big != force_big) continue;
      const int es = pemit_strat(vf, hh, big, mvc >= 0 ? 1 : 0);
      const int wpw = scan_waves(es);
      int v = bv, h2 = bh;
      TilePlan e = plan_tiles(q, q->hsegs, es, false, lds_of(v, h2), true);
      // while below emit_min_waves: try every smaller bin size (down to 64-byte bursts) and keep the one with the most
      // resident waves (ties: the larger bursts). A halving step alone may not add a workgroup (the tile plan spends
      // the freed LDS on a deeper ring) while the next one does.
      int cv = v, ch = h2;
      while ((e.score < 0 || e.wg_per_cu * wpw < emit_min_waves) &&
             ((with_h && ch > 16) || (with_v && cv * W > 16 && cv % 8 == 0))) {
        cv = (with_v && cv * W > 16 && cv % 8 == 0) ? cv / 2 : cv;
        ch = (with_h && ch > 16) ? ch / 2 : ch;
        TilePlan t = plan_tiles(q, q->hsegs, es, false, lds_of(cv, ch), true);
        if (t.score >= 0 && (e.score < 0 || t.wg_per_cu > e.wg_per_cu)) {
          v = cv;
          h2 = ch;
          e = t;
        }
      }
      if (e.score > best.score) {
        best = e;
        best_bv = v;
        best_bh = h2;
        strat = es;
      }
    }
    bv = best_bv;
    bh = best_bh;
    return best;
  };
  if (split) {
    emit_plan = plan_emit(fmt, 0, true, false, bs_v, bs_h, q->emit_strat);
    TilePlan eh = plan_emit(-1, 1, false, true, bs_v, bs_h, q->emit_h_strat);
    if (eh.score < 0) { PLAN_LOG("partitioned: no (exit 8h)"); return false; }
    q->emit_h_lds = (int)eh.lds;
    q->emit_h_ring = eh.ring;
    q->emit_h_wg = eh.wg_per_cu;
  } else {
    emit_plan = plan_emit(vstream ? fmt : -1, hll >= 0 ? 1 : 0, vstream, hll >= 0, bs_v, bs_h, q->emit_strat);
  }
  if (emit_plan.score < 0) { PLAN_LOG("partitioned: no (exit 8)"); return false; }
  // The count pass needs only a key's partition (key >> shift). Component 0 of a direct key space with a power-of-two
  // cardinality no larger than the partition's key range never changes it: every other stride is a multiple of that
  // cardinality, so the rest of the key is a multiple of it below the shift and component 0 cannot carry into the
  // partition bits (configs[2]: d1 of GROUP BY d1, d2 — the count pass reads d2 only).
  q->count_skip = -1;
  {
    const int64_t c0 = s.num_group_by > 0 ? s.group_by_cardinality[0] : 0;
    const int sh = std::min(vstream ? ksv : 63, hll >= 0 ? (int)__builtin_ctzll((uint64_t)kr_h) : 63);
    bool ok = s.num_group_by > 1 && !q->hashed && !q->limit_walk && P.stride[0] == 1 && c0 > 0 &&
              (c0 & (c0 - 1)) == 0 && c0 <= (int64_t(1) << std::min(sh, 62));
    for (size_t li = 0; li < q->literals.size() && ok; ++li) ok = P.leaf_slot[q->literals[li].leaf] != P.gb_slot[0];
    for (int j = 1; j < s.num_group_by && ok; ++j) ok = P.gb_slot[j] != P.gb_slot[0];
    if (ok) q->count_skip = 0;
  }
  q->hsegs_count = count_pass_segments(q, P);
  q->count_strat = mvc >= 0 ? STRAT_PCOUNT_MV : STRAT_PCOUNT;
  count_plan = plan_tiles(q, q->hsegs_count, q->count_strat, false, ((size_t)Ptot * 4 + 15) & ~(size_t)15, true);
  if (count_plan.score < 0) { PLAN_LOG("partitioned: no (exit 9)"); return false; }

  // descriptors (the rest of hq is filled by fill_devquery)
  h.num_parts = Ptot;
  h.pv = (int32_t)Pv;
  h.kshift_v = ksv;
  h.kshift_h = hll >= 0 ? __builtin_ctzll((uint64_t)kr_h) : 0;
  h.v_fmt = fmt;
  h.rec_words_v = W;
  h.bs_v = bs_v;
  h.bs_h = bs_h;
  h.h_first = (hll >= 0 && !vstream) ? 1 : 0;
  h.hll_agg = hll;
  h.emit_val_agg = slots == 1 ? va : -1;
  q->part_vk = (vk_fast && fmt != V_FMT_GEN)
                   ? vk_code(h.vop_sum >= 0 ? 1 + P.agg_src[h.vop_sum] : 0, h.vop_min >= 0, h.vop_max >= 0)
                   : kVkGeneric;
  h.v_id_order = (fmt == V_FMT_ID && sorted_ids) ? 1 : 0;
  h.part_kr_v = 0;
  q->v_id_bits = fmt == V_FMT_ID ? vbits : 0;

  h.vdict = vdict;
  size_t o = 0;
  h.lds_cnt = (uint32_t)o; o += (size_t)Ptot * 4;
  h.lds_done = (uint32_t)o; o += (size_t)Ptot * 4;
  h.lds_front = (uint32_t)o; o += (size_t)Ptot * 4;
  h.lds_back = (uint32_t)o; o += (size_t)Ptot * 4;
  h.lds_slack = (uint32_t)o; o += (size_t)Ph * 4;
  o = (o + 7) & ~(size_t)7;
  h.lds_start = (uint32_t)o; o += (size_t)Ptot * 8;
  o = (o + 15) & ~(size_t)15;
  h.lds_bins_v = (uint32_t)o;
  if (!split) o += (size_t)Pv * bs_v * W * 4;  // (split: each launch's bins start right after the state)
  o = (o + 15) & ~(size_t)15;
  h.lds_bins_h = (uint32_t)o;
  h.part_lo = 0;
  h.part_hi = split ? (int32_t)Pv : Ptot;
  // pass C LDS: V: u32 count[kr_v], then every aggregation's accumulators (8-byte aligned); H: u8 registers (+ counts)
  size_t lv = 0;
  std::vector<int> agg_lds(s.num_aggs, 0);
  if (vstream) {
    lv = ((size_t)kr_v * 4 + 15) & ~(size_t)15;
    for (int a = 0; a < s.num_aggs; ++a) {
      const int t = s.aggs[a].type;
      if (t == PA_AGG_COUNT || t == PA_AGG_DISTINCTCOUNTHLL) continue;
      agg_lds[a] = (int)lv;
      lv += (size_t)kr_v * ((t == PA_AGG_SUM && P.agg_src[a] == SRC_LONG) ? 16 : 8);
    }
  }
  size_t lh = hll >= 0 ? ((size_t)kr_h << s.aggs[hll].log2m) + (vstream ? 0 : (size_t)kr_h * 4) : 0;
  q->part_lds_c = (int)std::max(lv, lh);
  for (int a = 0; a < s.num_aggs; ++a) {
    h.aggs[a].lds_off = agg_lds[a];
    h.aggs[a].pay_off = pay[a];
  }
  q->partitioned = true;
  PLAN_LOG("partitioned: K=%lld Pv=%lld (kr %lld, fmt %d, W %d, bs %d) Ph=%lld (kr %lld, bs %d) emit lds %zu wg %d ring %d; "
           "split %d strat %d/%d (H lds %d wg %d ring %d); count lds %zu wg %d", (long long)K, (long long)Pv, (long long)kr_v, fmt,
           W, bs_v, (long long)Ph, (long long)kr_h, bs_h, emit_plan.lds, emit_plan.wg_per_cu, emit_plan.ring,
           (int)split, q->emit_strat, q->emit_h_strat, q->emit_h_lds, q->emit_h_wg, q->emit_h_ring, count_plan.lds, count_plan.wg_per_cu);
  return true;
}

// Strategy + tile plan of the main pass.
int plan_kernels(pa_query* q, Prep& P, TilePlan& plan, TilePlan& count_plan) {
  const pa_query_spec& s = q->spec;
  const int64_t K = q->num_keys;
  // Lane-major kernel: every eager literal is a dictionary leaf on a staged column and the per-segment plan table
  // has room for the staged columns and eager literals (otherwise the step-major kernel runs the query).
  bool lm = !(s.flags & (PA_QF_NO_LANE_MAJOR | PA_QF_STEPS16)) && q->num_eager <= kLmEager;
  for (int li = 0; li < q->num_eager && lm; ++li) {
    const int k = s.leaves[q->literals[li].leaf].kind;
    if (k != PA_LEAF_DICT_RANGE && k != PA_LEAF_DICT_SET) lm = false;
  }
  for (int si = 0; si < q->nseg && lm; ++si)
    if (q->hsegs[si].num_staged > kLmStaged) lm = false;
  // Tile layout: lane-major when it applies, except for dense queries on global accumulators, whose per-doc atomics
  // want the most resident waves (measured, tools/bench_configs.py highcard): there the step-major plan wins when it
  // fits more workgroups per CU.
  auto plan_pick = [&](int strat, size_t acc_b) {
    if (!lm) return plan_tiles(q, q->hsegs, strat, false, acc_b, false);
    TilePlan a = plan_tiles(q, q->hsegs, strat, true, acc_b, false);
    if (strat == STRAT_GLOBAL && P.dense) {
      TilePlan b = plan_tiles(q, q->hsegs, strat, false, acc_b, false);
      if (b.score >= 0 && b.wg_per_cu > a.wg_per_cu) {
        lm = false;
        return b;
      }
    }
    return a;
  };
  // LDS-privatised accumulators when many docs are expected to reach them (and the key space fits); otherwise the
  // LDS goes to tile rings (more resident waves) and the rare survivors update global accumulators directly.
  q->strategy = STRAT_GLOBAL;
  // Dense filter + GROUP BY over a small key box, every column staged (plan_gdense decided the staging)
  // (4- or 8-wave workgroups, lane-major 2048-doc or step-major 1024-doc tiles: the most resident waves, then the
  // larger tile: plan_tiles' score)
  if (P.gdense) {
    TilePlan best;
    bool best_lm = false;
    int best_strat = STRAT_GDENSE;
    for (int st : {STRAT_GDENSE12, STRAT_GDENSE8, STRAT_GDENSE})
      for (int use_lm : {1, 0}) {
        if (use_lm && (!lm || st == STRAT_GDENSE12)) continue;
        const TilePlan t = plan_tiles(q, q->hsegs, st, use_lm != 0, P.gd_lds, use_lm == 0);
        if (t.score > best.score) {
          best = t;
          best_lm = use_lm != 0;
          best_strat = st;
        }
      }
    // lane-major walk over the LDS-DMA ring (gdl_tile) whenever its ring of two 1024-doc images per wave fits: the most
    // resident waves (16- or 8-wave workgroups); every staged dictionary column has 1..31 bits (the unpacker switch)
    // (and every DICT_SET bitmap in LDS: gdl_leaf reads no HBM in the tile loop)
    bool lm_walk = !(s.flags & (PA_QF_NO_GDENSE_LM | PA_QF_NO_LANE_MAJOR)) && q->num_eager <= kGdLmLeaves;
    for (const DevSeg& d : q->hsegs) lm_walk = lm_walk && d.num_staged <= kGdlMaxCols;
    for (int li = 0; li < q->num_eager && lm_walk; ++li)
      if (s.leaves[q->literals[li].leaf].kind == PA_LEAF_DICT_SET && (li >= (int)P.gd_lut.size() || P.gd_lut[li] < 0))
        lm_walk = false;
    for (const DevSeg& d : q->hsegs)
      for (int k = 0; k < d.num_staged && lm_walk; ++k) {
        const int nb = d.stage[k].nbits;
        lm_walk = (nb >= 1 && nb <= 31) || nb == 32 || nb == 64;
      }
    size_t lm_acc = P.gd_lds;
    bool lm_pk = false;
    if (lm_walk) {
      TilePlan lmb;
      int lm_strat = -1;
      double lm_score = -1;
      for (int st : {STRAT_GDENSE_LM16, STRAT_GDENSE_LM8})
        for (int pk : {1, 0}) {
          if (pk && !P.gd_pk_ok) continue;
          // packed accumulation: the waves' private rows (nkeys u64 each) follow the accumulators and tables; worth
          // more than twice the resident waves (one atomic per matching doc instead of one per aggregation)
          const size_t acc_b = (P.gd_lds + (pk ? (size_t)scan_waves(st) * (size_t)P.gd_nkeys * 8 : 0) + 15) & ~(size_t)15;
          const TilePlan t = plan_tiles(q, q->hsegs, st, false, acc_b, true);
          if (t.score < 0) continue;
          const double sc = t.score + (pk ? 2.5e7 : 0.0);
          if (sc > lm_score) {
            lm_score = sc;
            lmb = t;
            lm_strat = st;
            lm_acc = acc_b;
            lm_pk = pk != 0;
          }
        }
      if (lmb.score >= 0) {
        best = lmb;
        best_lm = false;
        best_strat = lm_strat;
      } else {
        lm_walk = false;
      }
    }
    // register-staged tiles (more bytes in flight than the LDS ring beside large tables) when every segment shares the
    // LDS tables and a tile's load instructions fit a variant's register ring
    bool shared = !lm_walk;
    for (int si = 1; si < q->nseg && shared; ++si) {
      for (int j = 0; j < s.num_group_by; ++j)
        shared = shared && (P.gd_tab[j] < 0 || q->hsegs[si].remap[j] == q->hsegs[0].remap[j]);
      for (int a = 0; a < s.num_aggs; ++a)
        shared = shared && (P.gd_tab_a[a] < 0 || P.gd_src[si][a] == P.gd_src[0][a]);
    }
    if (shared && !(s.flags & ((15u << PA_QF_RING_SHIFT) | (7u << PA_QF_WG_SHIFT) | PA_QF_NO_REG_STAGE))) {
      int ins = 0, img_dw = kGuardWords;
      for (const DevSeg& d : q->hsegs) {
        int n = 0, dw = kGuardWords;
        for (int k = 0; k < d.num_staged; ++k) {
          n += ((kGdSmSteps / 2) * d.stage[k].nbits + 63) / 64;
          dw += 2 * kGdSmSteps * d.stage[k].nbits + kGuardWords;
        }
        ins = std::max(ins, n);
        img_dw = std::max(img_dw, dw);
      }
      int nvalue = 0;
      for (int a = 0; a < s.num_aggs; ++a) nvalue += s.aggs[a].type != PA_AGG_COUNT;
      for (int st : {STRAT_GDENSE_RS12, STRAT_GDENSE_RS8}) {
        if (ins > gd_rs_dmax(st)) continue;
        if (st == STRAT_GDENSE_RS12 && (s.num_group_by > kGdRs12MaxGb || nvalue > kGdRs12MaxAgg)) continue;
        const size_t lds = P.gd_lds + (size_t)scan_waves(st) * img_dw * 4;
        if (lds > kLdsBudget) continue;
        int resident = 0;
        if (set_scan_lds_limit(st, kGdSmSteps, 0, (int)kLdsBudget) != hipSuccess ||
            scan_occupancy(st, kGdSmSteps, 0, (int)lds, &resident) != hipSuccess)
          resident = 1;
        if (resident < 1) continue;
        best = TilePlan{kGdSmSteps, ins, 1, 1, img_dw, lds, 1e9};
        best_lm = false;
        best_strat = st;
        break;
      }
    }
    if (best.score >= 0) {
      lm = best_lm;
      plan = best;
      q->strategy = best_strat;
      P.lds_acc = P.gd_lds;
      if (is_gdense_lm(best_strat)) {
        P.lds_acc = lm_acc;
        if (lm_pk) {  // packed: tables of values become offsets from the values' minimum
          P.gd_packed = true;
          for (int a = 0; a < s.num_aggs; ++a)
            if (P.gd_pk_t32u[a]) {
              P.gd_vs[a] = GVS_T32U;
              P.gd_base[a] = P.gd_pk_base[a];
              P.gd_step[a] = 1;
            }
        }
      }
    }
  }
  // Aggregation-only over single-value columns (configs[0]'s COUNT(*), SUM(m) WHERE ...): running totals in every lane's
  // registers, reduced once per wave at the end of the kernel (STRAT_LANE)
  bool lane_acc = q->strategy == STRAT_GLOBAL && s.num_group_by == 0 && !q->has_mv && !q->limit_mode && !q->hashed && s.num_aggs <= kLaneAggs &&
                  !(s.flags & (PA_QF_NO_LANE_ACC | PA_QF_FORCE_GLOBAL | PA_QF_FORCE_LDS));
  for (int a = 0; a < s.num_aggs && lane_acc; ++a) {
    const int t = s.aggs[a].type;
    lane_acc = t == PA_AGG_COUNT || t == PA_AGG_SUM || t == PA_AGG_MIN || t == PA_AGG_MAX;
  }
  if (lane_acc) {
    // lane-major tiles run the kernel variant of the aggregation columns' kind (raw / dictionary / none) when every
    // bound segment agrees on it
    int lane_strat = STRAT_LANE;
    if (lm) {
      bool any_raw = false, any_dict = false, other = false;
      for (int a = 0; a < s.num_aggs; ++a) {
        if (s.aggs[a].type == PA_AGG_COUNT) continue;
        for (int si = 0; si < q->nseg; ++si) {
          auto it = q->segs[si]->cols.find(s.aggs[a].column_id);
          const int k = it == q->segs[si]->cols.end() ? COL_NONE : it->second->kind;
          any_raw |= k == COL_SV_RAW;
          any_dict |= k == COL_SV_DICT;
          other |= k != COL_SV_RAW && k != COL_SV_DICT;
        }
      }
      if (!other && !any_raw && !any_dict) lane_strat = STRAT_LANE_CNT;
      else if (!other && any_raw && !any_dict) lane_strat = STRAT_LANE_RAW;
      else if (!other && any_dict && !any_raw) lane_strat = STRAT_LANE_DICT;
    }
    // the lane accumulators' LDS slots (kLaneAccBytes per thread and aggregation; none for COUNT only)
    size_t lane_b = lane_strat == STRAT_LANE_CNT ? 0 : (size_t)s.num_aggs * kWGSize * kLaneAccBytes;
    // dictionary kernel: a SUM over a column whose dictionary every bound segment shares (same values) counts dictIds in
    // an LDS histogram instead of gathering a value per doc, when the histogram fits (kLaneHistMax ids) and most docs
    // match: the histogram's LDS costs resident workgroups (configs[0], 1B docs: 100 % 3.68 -> 2.74 ms, 50 % 2.36 ->
    // 2.27 ms, 10 % 1.15 -> 1.41 ms, r03_hist2)
    const bool hist_dense = P.post_density > 0.75 * kWTileDocs;
    for (int a = 0; a < s.num_aggs; ++a) {
      q->hq.aggs[a].hist_card = 0;
      q->hq.aggs[a].hist_off = 0;
      if (lane_strat != STRAT_LANE_DICT || s.aggs[a].type != PA_AGG_SUM || q->nseg == 0 || !hist_dense) continue;
      const Column* c0 = q->segs[0]->cols.at(s.aggs[a].column_id);
      if (c0->cardinality > kLaneHistMax || c0->hvals.size() != (size_t)c0->cardinality) continue;
      bool shared = true;
      for (int si = 1; si < q->nseg && shared; ++si) {
        const Column* c = q->segs[si]->cols.at(s.aggs[a].column_id);
        shared = c->cardinality == c0->cardinality && c->vtype == c0->vtype && c->dict_hash == c0->dict_hash &&
                 c->hvals == c0->hvals;
      }
      if (!shared || (s.flags & PA_QF_NO_LANE_HIST)) continue;
      lane_b = (lane_b + 15) & ~(size_t)15;
      q->hq.aggs[a].hist_card = c0->cardinality;
      q->hq.aggs[a].hist_off = (int32_t)lane_b;
      lane_b += (size_t)c0->cardinality * 4;
    }
    plan = plan_pick(lane_strat, lane_b);
    if (plan.score < 0 && lane_b > (size_t)s.num_aggs * kWGSize * kLaneAccBytes) {
      // the histograms leave no room for a tile ring: gather per doc instead
      for (int a = 0; a < s.num_aggs; ++a) q->hq.aggs[a].hist_card = 0;
      lane_b = (size_t)s.num_aggs * kWGSize * kLaneAccBytes;
      plan = plan_pick(lane_strat, lane_b);
    }
    if (plan.score >= 0) {
      q->strategy = lane_strat;
      P.lds_acc = lane_b;
    }
  }
  if (q->strategy == STRAT_GLOBAL && !(s.flags & PA_QF_FORCE_GLOBAL) && !q->limit_mode && !q->hashed &&
      P.lds_acc <= 64 * 1024 && (P.dense || (s.flags & PA_QF_FORCE_LDS))) {
    plan = plan_pick(STRAT_LDS, P.lds_acc);
    if (plan.score >= 0) q->strategy = STRAT_LDS;
  }
  // Partitioned aggregation for dense queries whose key space does not fit LDS (BASELINE configs[2], configs[4]):
  // count pass + emit pass into key partitions + one LDS aggregation per partition, instead of ~(1 + aggregations)
  // device-scope atomics per matching doc on random keys.
  q->partitioned = false;
  PLAN_LOG("K=%lld strategy=%d dense=%d (post density %.3g) gb_mv=%d hashed=%d limit=%d", (long long)K, q->strategy,
           (int)P.dense, P.post_density, (int)P.gb_mv, (int)q->hashed, (int)q->limit_mode);
  if (q->strategy == STRAT_GLOBAL && P.dense && !q->hashed && !q->limit_mode &&
      !(s.flags & (PA_QF_NO_PARTITION | PA_QF_FORCE_GLOBAL)) && K < (int64_t(1) << 32)) {
    TilePlan e;
    if (plan_partitions(q, P, e, count_plan)) {
      plan = e;
      lm = false;
    }
  }
  if (q->strategy == STRAT_GLOBAL && !q->partitioned) plan = plan_pick(STRAT_GLOBAL, 0);
  if (plan.score < 0) return fail(PA_EUNSUPPORTED, "staged columns too wide for the LDS tile ring");
  P.lm = lm;
  q->lds_bytes = (int)plan.lds;
  q->steps = plan.steps;
  q->dma_slots = plan.dma;
  return PA_OK;
}

// Tiles per segment, LDS regions of the staged columns, staged bytes.
void apply_layout(std::vector<DevSeg>& segs, int steps, int nslots, int nleaves, const void* dummy,
                  uint64_t* staged_bytes, int64_t* total_tiles) {
  int64_t first = 0;
  uint64_t staged = 0;
  for (DevSeg& d : segs) {
    const int64_t tile_docs = (int64_t)steps * kWave;
    d.num_wtiles = (int32_t)((d.num_docs + tile_docs - 1) / tile_docs);
    d.first_wtile = first;
    first += d.num_wtiles;
    d.dummy_src = (const uint32_t*)dummy;
    int off = kGuardWords;
    for (int k = 0; k < d.num_staged; ++k) {
      d.stage[k].lds_off = off;
      for (int sl = 0; sl < nslots; ++sl)
        if (d.cols[sl].lds_off >= 0 &&
            (d.cols[sl].kind == COL_SV_RAW ? (const uint32_t*)d.cols[sl].raw : d.cols[sl].words) == d.stage[k].words)
          d.cols[sl].lds_off = off;
      staged += (uint64_t)d.num_wtiles * 2 * steps * d.stage[k].nbits * 4;
      off += 2 * steps * d.stage[k].nbits + kGuardWords;
    }
    d.image_dwords = off;
    for (int li = 0; li < nleaves; ++li) d.leaves[li].lds_off = d.cols[d.leaves[li].slot].lds_off;
  }
  if (staged_bytes) *staged_bytes = staged;
  if (total_tiles) *total_tiles = first;
}

// The scan descriptor of the main pass (and of the count pass, derived from it).
void fill_devquery(pa_query* q, const Prep& P, const TilePlan& plan, int64_t total_tiles) {
  const pa_query_spec& s = q->spec;
  const int nslots = (int)q->slot_cols.size();
  DevQuery& h = q->hq;  // partition fields were set by plan_partitions; everything else here
  h.num_segments = q->nseg;
  h.num_slots = nslots;
  h.num_leaves = (int32_t)q->literals.size();
  h.num_gb = s.num_group_by;
  h.num_aggs = s.num_aggs;
  h.strategy = q->partitioned ? STRAT_PEMIT : q->strategy;
  h.image_dwords_max = plan.img_dw;
  h.num_staged = 0;
  for (int sl = 0; sl < nslots; ++sl) {
    bool st = false;
    for (const DevSeg& d : q->hsegs) st |= d.cols[sl].lds_off >= 0;
    if (st) h.staged_slots[h.num_staged++] = sl;
  }
  for (int j = 0; j < s.num_group_by; ++j) {
    h.gb_slot[j] = P.gb_slot[j];
    h.gb_stride[j] = P.stride[j];
  }
  h.num_keys = q->num_keys;
  h.num_groups_limit = s.num_groups_limit;
  h.total_wtiles = total_tiles;
  h.ring = plan.ring;
  h.num_eager = q->num_eager;
  h.dma_per_tile = plan.dma;
  h.steps = plan.steps;
  h.debug_stream_only = (s.flags & PA_QF_DEBUG_STREAM_ONLY) ? 1 : 0;
  {
    const char* e = std::getenv("PA_DEBUG_EMIT");  // measurement only (see DevQuery::debug_emit)
    h.debug_emit = e ? std::atoi(e) : 0;
  }
  h.lane_major = P.lm ? 1 : 0;
  h.count = (unsigned long long*)q->sections[0].ptr;
  h.matched_docs = (unsigned long long*)q->sections.back().ptr;
  h.hashed = q->hashed ? 1 : 0;
  h.key_words = q->key_words;
  for (int j = 0; j < s.num_group_by; ++j) h.gb_word[j] = q->hashed ? P.gb_word[j] : 0;
  if (q->hashed) {
    h.ht_mask = q->ht_slots - 1;
    h.ht_keys = (long long*)q->sections[q->keys_section].ptr;
  }
  h.has_mv = q->has_mv;
  h.gb_mv = std::max(-1, mv_group_component(q));
  h.count_skip_gb = -1;
  for (int li = 0; li < PA_MAX_LEAVES; ++li) h.gd_lut[li] = -1;
  h.xcd_major = (P.dense || is_gdense(q->strategy)) ? 1 : 0;
  h.lds_count_off = 0;
  h.lds_acc_bytes = (q->strategy == STRAT_LDS || is_gdense(q->strategy) || is_lane(q->strategy))
                        ? (uint32_t)P.lds_acc : 0;
  if (is_gdense(q->strategy)) {
    // per-segment parameter tables (GdSegPlan): the query's key box and LDS layout + the segment's staged regions
    q->gdplans.assign((size_t)std::max(1, q->nseg) * kGdPlanDw, 0u);
    for (int si = 0; si < q->nseg; ++si) {
      GdSegPlan& g = *(GdSegPlan*)&q->gdplans[(size_t)si * kGdPlanDw];
      const DevSeg& d = q->hsegs[si];
      // register-staged variants: the tile's load instructions (stage_tile's order: columns, then 64-chunk groups)
      GdRsPlan& rp = *(GdRsPlan*)&q->gdplans[(size_t)si * kGdPlanDw + 64];
      if (is_gdense_lm(q->strategy)) {  // the lane-major walk's DMA issue table takes the same dwords
        GdLmIssue& li = *(GdLmIssue*)&q->gdplans[(size_t)si * kGdPlanDw + 64];
        li.ncols = d.num_staged;
        for (int k = 0; k < d.num_staged; ++k) {
          const int nb = d.stage[k].nbits;
          const uint64_t src = (uint64_t)(uintptr_t)d.stage[k].words;
          li.col[k].src_lo = (uint32_t)src;
          li.col[k].src_hi = (uint32_t)(src >> 32);
          li.col[k].stride = (uint32_t)(2 * kGdSmSteps * nb * 4);
          li.col[k].chunks = (uint32_t)((kGdSmSteps / 2) * nb);
          li.col[k].dst = (uint32_t)(4 * d.stage[k].lds_off);
        }
      }
      for (int k = 0; k < d.num_staged && !is_gdense_lm(q->strategy); ++k) {
        const int nb = d.stage[k].nbits;
        const int chunks = (kGdSmSteps / 2) * nb;
        for (int c0 = 0; c0 < chunks && rp.ins < kGdRsMaxIns; c0 += 64) {
          const uint64_t src = (uint64_t)(uintptr_t)d.stage[k].words + 16ull * (uint64_t)c0;
          rp.in[rp.ins].src_lo = (uint32_t)src;
          rp.in[rp.ins].src_hi = (uint32_t)(src >> 32);
          rp.in[rp.ins].stride = (uint32_t)(2 * kGdSmSteps * nb * 4);
          rp.in[rp.ins].lanes = (uint32_t)std::min(64, chunks - c0);
          rp.in[rp.ins].dst = (uint32_t)(4 * d.stage[k].lds_off + 16 * c0);
          ++rp.ins;
        }
      }
      g.ngb = s.num_group_by;
      g.rpl = P.gd_rp_log2;
      g.box = P.gd_box ? 1 : 0;
      {
        const char* e = std::getenv("PA_DEBUG_EMIT");  // measurement only (pa_gdense.h knobs; results invalid)
        g.pad = e ? std::atoi(e) : 0;
      }
      for (int j = 0; j < s.num_group_by; ++j) {
        g.gb[j].reg = d.cols[P.gb_slot[j]].lds_off;
        g.gb[j].nbits = d.cols[P.gb_slot[j]].nbits;
        g.gb[j].tab = P.gd_tab[j];
        g.gb[j].lo = P.gd_lo[j];
        g.gb[j].span = P.gd_span[j];
        g.gb[j].ls = P.gd_ls[j];
      }
      int k = 0;
      for (int a = 0; a < s.num_aggs; ++a) {
        if (s.aggs[a].type == PA_AGG_COUNT) continue;
        g.ag[k].vs = P.gd_vs[a];
        g.ag[k].op = P.gd_op[a];
        g.ag[k].reg = d.cols[P.agg_slot[a]].lds_off;
        g.ag[k].nbits = d.cols[P.agg_slot[a]].nbits;
        g.ag[k].acc = P.gd_acc[a];
        g.ag[k].tab = P.gd_tab_a[a];
        ++k;
      }
      g.nagg = k;
      if (is_gdense_lm(q->strategy)) {
        GdLmPlan& lp = *(GdLmPlan*)&q->gdplans[(size_t)si * kGdPlanDw + 128];
        lp.nleaves = q->num_eager;
        lp.num_docs = d.num_docs;
        // the group key from the filter's unpack: one group-by column, read by a DICT_RANGE leaf
        lp.key_leaf = -1;
        for (int li = 0; li < q->num_eager && li < kGdLmLeaves && s.num_group_by == 1; ++li)
          if (d.leaves[li].kind == PA_LEAF_DICT_RANGE && s.leaves[q->literals[li].leaf].column_id == s.group_by_columns[0] &&
              d.leaves[li].lds_off == d.cols[P.gb_slot[0]].lds_off) {
            lp.key_leaf = li;
            // the box check is implied when this leaf is a unit clause (not negated) whose dictId range, without a
            // remap, is exactly the box's component
            const bool unit = q->clause_end[li] && (li == 0 || q->clause_end[li - 1]);
            const pa_leaf_params& pr = q->leaf_params[si][q->literals[li].leaf];
            const int64_t card = d.cols[P.gb_slot[0]].card;
            const int64_t rlo = std::max<int64_t>(0, pr.lo), rhi = std::min<int64_t>(pr.hi, card);
            lp.key_in_box = unit && !d.leaves[li].negate && P.gd_tab[0] < 0 && rlo == P.gd_lo[0] &&
                            rhi - rlo == P.gd_span[0];
            break;
          }
        for (int li = 0; li < q->num_eager && li < kGdLmLeaves; ++li) {
          const DevLeaf& L = d.leaves[li];
          lp.lf[li].code = (uint32_t)L.kind | (L.negate ? 0x100u : 0u) | (L.clause_end ? 0x200u : 0u) |
                           ((uint32_t)L.nbits << 16);
          lp.lf[li].region = (uint32_t)(4 * L.lds_off);
          lp.lf[li].lo_t = (uint32_t)L.lo;
          lp.lf[li].hi_t = (uint32_t)L.span;
          lp.lf[li].lut_lds = li < (int)P.gd_lut.size() ? P.gd_lut[li] : -1;
          const uint64_t lut = (uint64_t)(uintptr_t)L.lut;
          lp.lf[li].lut_lo = (uint32_t)lut;
          lp.lf[li].lut_hi = (uint32_t)(lut >> 32);
        }
        if (P.gd_packed) {
          lp.packed = 1;
          int off = 0, kk = 0;
          for (int a = 0; a < s.num_aggs; ++a) {
            if (s.aggs[a].type == PA_AGG_COUNT) continue;
            lp.pk_off[kk++] = off;
            off += P.gd_pk_w[a] + P.gd_pk_c;
          }
          lp.pk_cnt = off;
          lp.pk_drain = (int32_t)(((uint64_t(1) << P.gd_pk_c) - 1) >> 10);  // tiles of <= 1024 docs each
          if (s.flags & PA_QF_GD_DRAIN_EACH_TILE) lp.pk_drain = 1;
          lp.pk_base = (int32_t)P.gd_lds;  // (the waves' rows follow the accumulators and tables)
        }
      }
    }
    h.gd_rp_log2 = P.gd_rp_log2;
    h.gd_nkeys = P.gd_nkeys;
    h.gd_pk_base = P.gd_packed ? (int32_t)P.gd_lds : 0;
    h.gd_tables = P.gd_tables;
    for (size_t li = 0; li < q->literals.size() && li < (size_t)PA_MAX_LEAVES; ++li) {
      h.gd_lut[li] = li < P.gd_lut.size() ? P.gd_lut[li] : -1;
      h.gd_lut_words[li] = li < P.gd_lut_words.size() ? P.gd_lut_words[li] : 0;
    }
    for (int j = 0; j < s.num_group_by; ++j) {
      h.gd_lo[j] = P.gd_lo[j];
      h.gd_span[j] = P.gd_span[j];
      h.gd_ls[j] = P.gd_ls[j];
      h.gd_tab[j] = P.gd_tab[j];
      h.gd_tab_n[j] = P.gd_tab_n[j];
    }
  }
  // LDS strategy: the one column every non-COUNT aggregation (SUM / MIN / MAX only) reads, if raw in segment 0 (the
  // kernel checks each segment's column kind): dense lane-major tiles then load its values coalesced
  h.lds_raw_slot = -1;
  if (q->strategy == STRAT_LDS && q->nseg > 0) {
    int slot = -1;
    bool ok = true;
    for (int a = 0; a < s.num_aggs && ok; ++a) {
      const int t = s.aggs[a].type;
      if (t == PA_AGG_COUNT) continue;
      ok = (t == PA_AGG_SUM || t == PA_AGG_MIN || t == PA_AGG_MAX) && (slot < 0 || slot == P.agg_slot[a]);
      slot = P.agg_slot[a];
    }
    if (ok && slot >= 0) {
      auto it = q->segs[0]->cols.find(q->slot_cols[slot]);
      if (it != q->segs[0]->cols.end() && it->second->kind == COL_SV_RAW) h.lds_raw_slot = slot;
    }
  }
  if (!q->partitioned) {
    h.hll_agg = -1;
    h.pv = 0;
    h.num_parts = 0;
  }
  for (int a = 0; a < s.num_aggs; ++a) {
    DevAgg& A = h.aggs[a];
    A.type = s.aggs[a].type;
    A.slot = P.agg_slot[a];
    A.log2m = s.aggs[a].log2m;
    A.src = P.agg_src[a];
    A.nvals = s.aggs[a].type == PA_AGG_DISTINCTCOUNT ? presence_stride(s.aggs[a]) : 0;
    if (is_gdense(q->strategy)) {
      A.gd_vs = P.gd_vs[a];
      A.gd_op = P.gd_op[a];
      A.gd_acc = P.gd_acc[a];
      A.gd_tab = P.gd_tab_a[a];
      A.gd_tab_n = P.gd_tab_an[a];
      A.gd_base = P.gd_base[a];
      A.gd_step = P.gd_step[a];
    }
    if (!q->partitioned) {
      A.lds_off = (int32_t)P.agg_lds[a];
      A.pay_off = 0;
    }
    if (q->agg_section[a] >= 0) {
      void* p = q->sections[q->agg_section[a]].ptr;
      A.acc_i64 = (int64_t*)p;
      A.acc_f64 = (double*)p;
      A.acc_hll = (uint8_t*)p;
    }
  }
}

// Scratch of a partitioned query (offsets into the device arena) and the arena's size for it.
int plan_scratch(pa_query* q, const Prep& P) {
  const DevQuery& h = q->hq;
  const size_t G = (size_t)q->grid, Pn = (size_t)h.num_parts;
  uint64_t vrecs = 0, hrecs = 0;
  if (h.pv > 0) {
    vrecs = q->num_docs;
    if (mv_group_component(q) >= 0) {  // one record per (doc, value) pair
      vrecs = 0;
      for (const pa_segment* seg : q->segs)
        vrecs += (uint64_t)seg->cols.at(q->spec.group_by_columns[mv_group_component(q)])->total_values;
    }
    vrecs += (uint64_t)G * h.pv * (h.bs_v - 1);
  }
  if (h.hll_agg >= 0) {
    const int32_t cid = q->spec.aggs[h.hll_agg].column_id;
    for (const pa_segment* seg : q->segs) {
      const Column* c = seg->cols.at(cid);
      hrecs += c->kind == COL_MV_DICT ? (uint64_t)c->total_values : (uint64_t)seg->num_docs;
    }
    hrecs += (uint64_t)G * (Pn - h.pv) * (h.bs_h - 1);
  }
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  q->sc_hist = o; o += al(G * (size_t)q->count_k * Pn * 4);  // count-pass rows (k per emit workgroup)
  q->sc_off = o; o += al(G * Pn * 4);
  q->sc_base = o; o += al((Pn + 2) * 8);
  q->sc_recs_v = o; o += al((size_t)vrecs * h.rec_words_v * 4);
  q->sc_recs_h = o; o += al((size_t)hrecs * 4);
  q->sc_bytes = std::max<size_t>(o, 256);
  (void)P;
  if (hipGetDevice(&q->scratch_dev) != hipSuccess) q->scratch_dev = 0;
  ScratchArena* a = arena_for(q->scratch_dev);
  std::lock_guard<std::mutex> g(a->mu);
  return arena_grow(a, q->sc_bytes);
}

// Walk form of numGroupsLimit: one admitted-key bitmap per segment where the limit can bind (DevSeg::admit).
int plan_walk(pa_query* q, const Prep& P) {
  if (!q->limit_walk) return PA_OK;
  int64_t n = 0;
  for (int si = 0; si < q->nseg; ++si) n += P.limit_bind[si] ? 1 : 0;
  int rc = dev_alloc(q->lim_admit, (size_t)std::max<int64_t>(1, n) * (size_t)q->walk_words * 4);
  if (rc) return rc;
  int64_t k = 0;
  for (int si = 0; si < q->nseg; ++si)
    q->hsegs[si].admit = P.limit_bind[si] ? (const uint32_t*)q->lim_admit.p + (k++) * q->walk_words : nullptr;
  return PA_OK;
}

int plan_limit_buffers(pa_query* q, const Prep& P, int cus, int64_t total_tiles) {
  const pa_query_spec& s = q->spec;
  // first-seen table: twice the (segment, key) pairs that can exist, a power of two
  uint64_t H = 1024;
  while (H < 2 * P.limit_pairs && H <= (uint64_t(1) << 30)) H <<= 1;
  if (H > (uint64_t(1) << 30))
    return fail(PA_EUNSUPPORTED, "numGroupsLimit trimming: more than 2^29 distinct (segment, group) pairs possible");
  const size_t hb = (size_t)H * 8;
  int rc = dev_alloc(q->lim_keys, hb);
  if (!rc) rc = dev_alloc(q->lim_pos, hb);
  const size_t ns = (size_t)std::max(1, q->nseg);
  if (!rc) rc = dev_alloc(q->lim_hist, ns * 256 * 4);
  if (!rc) rc = dev_alloc(q->lim_sel, ns * 16);
  if (!rc) rc = dev_alloc(q->lim_thresh, ns * 8);
  if (rc) return rc;
  LimitDesc& F = q->limit;
  F.fkeys = (long long*)q->lim_keys.p;
  F.fpos = (unsigned long long*)q->lim_pos.p;
  F.fmask = (int64_t)H - 1;
  F.hist = (uint32_t*)q->lim_hist.p;
  F.prefix = (unsigned long long*)q->lim_sel.p;
  F.rank = (long long*)q->lim_sel.p + ns;
  F.nseg = q->nseg;
  {  // first positions doc << eb | expansion index are below 2^(bits(max docs) + eb)
    int64_t maxd = 1;
    for (int si = 0; si < q->nseg; ++si) maxd = std::max<int64_t>(maxd, q->segs[si]->num_docs);
    int b = 0;
    while (b < 63 && (int64_t(1) << b) < maxd) ++b;
    F.pos_bits = std::max(8, b + P.limit_eb);
  }
  F.thresh = (unsigned long long*)q->lim_thresh.p;
  F.reached = q->hq.matched_docs + 2;
  F.limit = s.num_groups_limit;
  F.eb = P.limit_eb;
  q->limit_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 16, total_tiles));
  return PA_OK;
}

// Device copies of the descriptors (+ the lane-major plan tables).
int upload_descriptors(pa_query* q) {
  int rc;
  if (is_gdense(q->strategy)) {
    rc = dev_alloc(q->dgdplans, sizeof(uint32_t) * q->gdplans.size());
    if (rc) return rc;
    PA_HIP(hipMemcpy(q->dgdplans.p, q->gdplans.data(), sizeof(uint32_t) * q->gdplans.size(), hipMemcpyHostToDevice));
    q->hq.gd_plans = (const uint32_t*)q->dgdplans.p;
  }
  rc = dev_alloc(q->dq, sizeof(DevQuery));
  if (rc) return rc;
  rc = dev_alloc(q->dsegs, sizeof(DevSeg) * std::max(1, q->nseg));
  if (rc) return rc;
  PA_HIP(hipMemcpy(q->dq.p, &q->hq, sizeof(DevQuery), hipMemcpyHostToDevice));
  if (q->nseg) PA_HIP(hipMemcpy(q->dsegs.p, q->hsegs.data(), sizeof(DevSeg) * q->nseg, hipMemcpyHostToDevice));
  if (q->partitioned) {
    rc = dev_alloc(q->dq_count, sizeof(DevQuery));
    if (!rc) rc = dev_alloc(q->dsegs_count, sizeof(DevSeg) * std::max(1, q->nseg));
    if (rc) return rc;
    PA_HIP(hipMemcpy(q->dq_count.p, &q->hq_count, sizeof(DevQuery), hipMemcpyHostToDevice));
    if (q->split_emit) {
      rc = dev_alloc(q->dq_h, sizeof(DevQuery));
      if (rc) return rc;
      PA_HIP(hipMemcpy(q->dq_h.p, &q->hq_h, sizeof(DevQuery), hipMemcpyHostToDevice));
    }
    if (q->nseg)
      PA_HIP(hipMemcpy(q->dsegs_count.p, q->hsegs_count.data(), sizeof(DevSeg) * q->nseg, hipMemcpyHostToDevice));
  }
  q->hplans.assign(std::max(1, q->nseg), LmSegPlan{});
  if (q->lane_major) {
    for (int si = 0; si < q->nseg; ++si) {
      const DevSeg& d = q->hsegs[si];
      LmSegPlan& P = q->hplans[si];
      std::memset(&P, 0, sizeof(P));
      P.nstaged = d.num_staged;
      P.neager = q->num_eager;
      P.num_docs = d.num_docs;
      P.num_wtiles = d.num_wtiles;
      P.dummy_lo = (uint32_t)(uintptr_t)d.dummy_src;
      P.dummy_hi = (uint32_t)((uint64_t)(uintptr_t)d.dummy_src >> 32);
      for (int k = 0; k < d.num_staged; ++k) {
        P.st[k].lo = (uint32_t)(uintptr_t)d.stage[k].words;
        P.st[k].hi = (uint32_t)((uint64_t)(uintptr_t)d.stage[k].words >> 32);
        P.st[k].nbits = d.stage[k].nbits;
        P.st[k].lds_off = d.stage[k].lds_off;
      }
      for (int li = 0; li < q->num_eager; ++li) {
        const DevLeaf& L = d.leaves[li];
        if (L.lds_off < 0) return fail(PA_EINVAL, "internal: eager literal on an unstaged column");
        P.lf[li].kind = L.kind;
        P.lf[li].nbits = L.nbits;
        P.lf[li].lds_off = L.lds_off;
        P.lf[li].lo = (uint32_t)L.lo;
        P.lf[li].span = (uint32_t)L.span;
        P.lf[li].flags = (L.negate ? 1 : 0) | (L.clause_end ? 2 : 0);
        P.lf[li].lut_lo = (uint32_t)(uintptr_t)L.lut;
        P.lf[li].lut_hi = (uint32_t)((uint64_t)(uintptr_t)L.lut >> 32);
      }
    }
  }
  rc = dev_alloc(q->dplans, sizeof(LmSegPlan) * q->hplans.size());
  if (rc) return rc;
  PA_HIP(hipMemcpy(q->dplans.p, q->hplans.data(), sizeof(LmSegPlan) * q->hplans.size(), hipMemcpyHostToDevice));
  if (q->partitioned) {
    PA_HIP(set_scan_lds_limit(q->emit_strat, q->steps, 0, q->lds_bytes));
    if (q->split_emit) PA_HIP(set_scan_lds_limit(q->emit_h_strat, q->steps, 0, q->emit_h_lds));
    PA_HIP(set_scan_lds_limit(q->count_strat, q->steps, 0, q->count_lds));
    PA_HIP(set_part_agg_lds_limit(q->part_vk, q->part_lds_c));
  } else {
    PA_HIP(set_scan_lds_limit(q->strategy, q->steps, q->lane_major, q->lds_bytes));
  }
  return PA_OK;
}

PartScratch scratch_of(const pa_query* q, void* base) {
  char* b = (char*)base;
  return PartScratch{(uint32_t*)(b + q->sc_hist), (uint32_t*)(b + q->sc_off), (uint64_t*)(b + q->sc_base),
                     (uint32_t*)(b + q->sc_recs_v), (uint32_t*)(b + q->sc_recs_h)};
}


// counters + list length + overflow flag of the fused statistics (pa_scan.h "fused execution statistics")
size_t leap_header_bytes(const pa_query* q) {
  return ((size_t)std::max(1, q->nseg) * 3 + 1 + (size_t)q->leap_slices) * sizeof(unsigned long long);
}

// Fused statistics (unless PA_QF_NO_FILTER_STATS): the scan counts the leap-frog statistics itself (leap_tile) when the filter is an AND of two
// single-value leaves whose first (eager) clause is sparse — each of its docs costs two short neighbour searches — and
// the scan is one pass (the partitioned and numGroupsLimit plans run the tile loop more than once).
int plan_leaps(pa_query* q, const Prep& P) {
  const pa_query_spec& s = q->spec;
  q->leap_leaf = -1;
  q->hq.leap_mode = 0;
  q->hq.leap_out = nullptr;
  if ((s.flags & PA_QF_NO_FILTER_STATS) || q->literals.size() != 2 || q->num_eager != 1) return PA_OK;
  if (!q->clause_end[0] || !q->clause_end[1] || q->literals[0].neg || q->literals[1].neg) return PA_OK;
  for (const Literal& lit : q->literals) {
    const int k = s.leaves[lit.leaf].kind;
    if (k == PA_LEAF_MV_DICT_RANGE || k == PA_LEAF_MV_DICT_SET) return PA_OK;
  }
  if (q->partitioned || q->limit_mode || q->limit_walk || is_gdense(q->strategy)) return PA_OK;
  if (P.first_clause_sel > 1.0 / 256.0) return PA_OK;
  q->hq.leap_mode = 1;
  q->leap_leaf = q->literals[0].leaf;
  return PA_OK;
}

// The fused statistics' buffer (layout: pa_scan.h "fused execution statistics"), once the grid is known: one list
// slice per scan wave, each 16 x the E docs the planner's estimate gives a wave (a slice that overflows only costs
// the bitmap fallback).
int alloc_leaps(pa_query* q, const Prep& P) {
  if (!q->hq.leap_mode) return PA_OK;
  const int64_t slices = (int64_t)q->grid * scan_waves(q->strategy);
  const int64_t cap = (int64_t)(16.0 * P.first_clause_sel * (double)q->num_docs / (double)slices) + 256;
  q->leap_slices = slices;
  if (slices > kLeapMaxSlices) {  // (the search kernel keeps the slices' prefix sums in LDS): the bitmap path instead
    q->hq.leap_mode = 0;
    q->leap_leaf = -1;
    return PA_OK;
  }
  // a wave keeps its first entries in LDS past its tile ring when the workgroups per CU still fit
  q->hq.leap_lds_cap = 0;
  {
    const int wpw = scan_waves(q->strategy);
    const int want = (int)std::min<int64_t>(cap, 128);
    const size_t extra = (size_t)wpw * want * 8;
    if (q->plan_wg > 0 && ((size_t)q->lds_bytes + extra) * (size_t)q->plan_wg <= kLdsBudget) {
      q->hq.leap_lds_cap = want;
      q->lds_bytes += (int)extra;
    }
  }
  const size_t words = (size_t)std::max(1, q->nseg) * 3 + 1 + (size_t)slices + (size_t)slices * (size_t)cap;
  int rc = dev_alloc(q->leap_buf, words * sizeof(unsigned long long));
  if (rc) return rc;
  PA_HIP(hipMemset(q->leap_buf.p, 0, leap_header_bytes(q)));
  q->hq.leap_out = (unsigned long long*)q->leap_buf.p;
  q->hq.leap_cap = cap;
  q->hq.leap_slices = slices;
  return PA_OK;
}
