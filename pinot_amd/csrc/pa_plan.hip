// Query planning, first half: filter CNF and clause order, column slots, key space, numGroupsLimit, the dense
// GROUP BY plan (STRAT_GDENSE), per-segment descriptors and the accumulator layout (pa_query_prepare's units).
#include "pa_host.h"

struct Node {
  int op;    // PA_OP_*
  int leaf;  // for LEAF
  int a = -1, b = -1;
};

// Postfix program -> CNF (list of clauses, each a disjunction of possibly negated leaves).
int to_cnf(const pa_query_spec& spec, std::vector<Clause>& out) {
  out.clear();
  if (spec.num_ops == 0) return PA_OK;
  std::vector<Node> nodes;
  std::vector<int> st;
  for (int i = 0; i < spec.num_ops; ++i) {
    const int op = spec.ops[i] & 0xff;
    if (op == PA_OP_LEAF) {
      const int leaf = (spec.ops[i] >> 8) & 0xff;
      if (leaf >= spec.num_leaves) return fail(PA_EINVAL, "filter program references a missing leaf");
      nodes.push_back({PA_OP_LEAF, leaf});
      st.push_back((int)nodes.size() - 1);
    } else if (op == PA_OP_NOT) {
      if (st.empty()) return fail(PA_EINVAL, "malformed filter program");
      Node n{PA_OP_NOT, -1};
      n.a = st.back();
      st.pop_back();
      nodes.push_back(n);
      st.push_back((int)nodes.size() - 1);
    } else if (op == PA_OP_AND || op == PA_OP_OR) {
      if (st.size() < 2) return fail(PA_EINVAL, "malformed filter program");
      Node n{op, -1};
      n.b = st.back();
      st.pop_back();
      n.a = st.back();
      st.pop_back();
      nodes.push_back(n);
      st.push_back((int)nodes.size() - 1);
    } else {
      return fail(PA_EINVAL, "unknown filter opcode");
    }
  }
  if (st.size() != 1) return fail(PA_EINVAL, "malformed filter program");
  // recursive CNF with negation pushed to the leaves (De Morgan)
  std::function<int(int, bool, std::vector<Clause>&)> rec = [&](int ni, bool neg, std::vector<Clause>& cl) -> int {
    const Node& n = nodes[ni];
    if (n.op == PA_OP_LEAF) {
      cl = {Clause{Literal{n.leaf, neg}}};
      return PA_OK;
    }
    if (n.op == PA_OP_NOT) return rec(n.a, !neg, cl);
    const bool is_and = (n.op == PA_OP_AND) != neg;
    std::vector<Clause> ca, cb;
    int rc = rec(n.a, neg, ca);
    if (rc) return rc;
    rc = rec(n.b, neg, cb);
    if (rc) return rc;
    if (is_and) {
      cl = ca;
      cl.insert(cl.end(), cb.begin(), cb.end());
    } else {
      cl.clear();
      for (auto& x : ca)
        for (auto& y : cb) {
          Clause c = x;
          c.insert(c.end(), y.begin(), y.end());
          cl.push_back(c);
        }
    }
    size_t lits = 0;
    for (auto& c : cl) lits += c.size();
    if (lits > PA_MAX_LEAVES) return fail(PA_EUNSUPPORTED, "filter expands to more than PA_MAX_LEAVES CNF literals");
    return PA_OK;
  };
  return rec(st.back(), false, out);
}


int slot_of(pa_query* q, int32_t col) {
  for (size_t i = 0; i < q->slot_cols.size(); ++i)
    if (q->slot_cols[i] == col) return (int)i;
  if ((int)q->slot_cols.size() >= kMaxSlots) return -1;
  q->slot_cols.push_back(col);
  return (int)q->slot_cols.size() - 1;
}

// Estimated fraction of a segment's docs a literal matches: the matching-dictId fraction of the dictionary (dictIds
// assumed equally frequent), 1/2 for raw-value leaves. Planning input only: results never depend on it.
double leaf_selectivity(const pa_query* q, int si, int leaf, bool neg_literal) {
  const pa_query_spec& s = q->spec;
  const pa_leaf_params& p = q->leaf_params[si][leaf];
  const int kind = s.leaves[leaf].kind;
  auto it = q->segs[si]->cols.find(s.leaves[leaf].column_id);
  if (it == q->segs[si]->cols.end() || (kind != PA_LEAF_DICT_RANGE && kind != PA_LEAF_DICT_SET)) return 0.5;
  // (MV leaves: 0.5 — they are always evaluated lazily, after every single-value clause)
  const int64_t card = std::max<int32_t>(1, it->second->cardinality);
  double sel;
  if (kind == PA_LEAF_DICT_RANGE) {
    const int64_t lo = std::max<int64_t>(0, p.lo), hi = std::min<int64_t>(p.hi, card);
    sel = hi > lo ? (double)(hi - lo) / (double)card : 0.0;
  } else {
    const std::vector<uint32_t>& lut = q->luts[si][leaf];
    int64_t n = 0;
    for (int64_t id = 0; id < card && (size_t)(id >> 5) < lut.size(); ++id) n += (lut[id >> 5] >> (id & 31)) & 1u;
    sel = (double)n / (double)card;
  }
  return ((p.negate != 0) != neg_literal) ? 1.0 - sel : sel;
}

int upload_owned(pa_query* q, const void* host, size_t bytes, void** dev) {
  DevBuf b;
  int rc = dev_alloc(b, bytes);
  if (rc) return rc;
  q->owned.push_back(b);
  if (bytes) PA_HIP(hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice));
  *dev = b.p;
  return PA_OK;
}


// Filter: CNF, clause order (most selective first), eager/lazy split, column slots of the leaves.
int plan_filter(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  std::vector<Clause> cnf;
  int rc = to_cnf(s, cnf);
  if (rc) return rc;
  auto is_mv_leaf = [&](int leaf) {
    const int k = s.leaves[leaf].kind;
    return k == PA_LEAF_MV_DICT_RANGE || k == PA_LEAF_MV_DICT_SET;
  };
  P.clause_mv.assign(cnf.size(), 0);  // clauses with an MV literal are evaluated per doc (lazily), last
  for (size_t c = 0; c < cnf.size(); ++c)
    for (const Literal& lit : cnf[c]) P.clause_mv[c] |= is_mv_leaf(lit.leaf);
  // Clause order and late materialisation. Clauses are evaluated most selective first (estimated from the
  // matching-dictId fraction, i.e. assuming dictIds are equally frequent; only speed depends on the estimate).
  // The leading clauses whose expected survivors per wave tile exceed kLazyDensity run on whole staged tiles
  // ("eager"); the rest only on surviving docs, from HBM ("lazy") — the reference's AndDocIdIterator likewise
  // advances later iterators only to candidate docs (operator/dociditerators/AndDocIdIterator.java).
  const double kLazyDensity = 0.25;
  std::vector<double> csel(cnf.size(), 1.0);
  for (size_t c = 0; c < cnf.size(); ++c) {
    double worst = q->nseg ? 0.0 : 1.0;
    for (int si = 0; si < q->nseg; ++si) {
      double sum = 0.0;
      for (const Literal& lit : cnf[c]) sum += leaf_selectivity(q, si, lit.leaf, lit.neg);
      worst = std::max(worst, std::min(1.0, sum));
    }
    csel[c] = worst;
  }
  std::vector<size_t> order(cnf.size());
  for (size_t c = 0; c < cnf.size(); ++c) order[c] = c;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    if (P.clause_mv[a] != P.clause_mv[b]) return P.clause_mv[a] < P.clause_mv[b];
    return csel[a] < csel[b];
  });
  const bool no_lazy = (s.flags & (PA_QF_STAGE_ALL | PA_QF_NO_LAZY)) != 0;
  size_t eager_clauses = 0;
  double density = (double)kWTileDocs;  // expected surviving docs per wave tile
  while (eager_clauses < cnf.size() && !P.clause_mv[order[eager_clauses]] &&
         (no_lazy || eager_clauses == 0 || density > kLazyDensity))
    density *= csel[order[eager_clauses++]];
  P.post_density = density;
  P.first_clause_sel = cnf.empty() ? 1.0 : csel[order[0]];
  for (size_t c = eager_clauses; c < cnf.size(); ++c) P.post_density *= csel[order[c]];
  q->literals.clear();
  q->clause_end.clear();
  q->num_eager = 0;
  for (size_t oc = 0; oc < cnf.size(); ++oc) {
    const Clause& c = cnf[order[oc]];
    for (size_t i = 0; i < c.size(); ++i) {
      q->literals.push_back(c[i]);
      q->clause_end.push_back(i + 1 == c.size());
    }
    if (oc < eager_clauses) q->num_eager = (int)q->literals.size();
  }
  P.slot_eager.assign(kMaxSlots, 0);
  P.leaf_slot.assign(s.num_leaves, -1);
  for (int l = 0; l < s.num_leaves; ++l) {
    const int sl = slot_of(q, s.leaves[l].column_id);
    if (sl < 0) return fail(PA_EUNSUPPORTED, "too many distinct columns in one query");
    P.leaf_slot[l] = sl;
  }
  for (int li = 0; li < q->num_eager; ++li) P.slot_eager[P.leaf_slot[q->literals[li].leaf]] = 1;
  P.has_filter = !q->literals.empty();
  P.dense = !P.has_filter || P.post_density >= 1.0;
  return PA_OK;
}

// Column slots of the group-by columns and aggregations; which slots are staged with the filter columns.
int plan_slots(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  P.gb_slot.assign(s.num_group_by, 0);
  P.slot_gb.assign(kMaxSlots, 0);
  for (int j = 0; j < s.num_group_by; ++j) {
    P.gb_slot[j] = slot_of(q, s.group_by_columns[j]);
    if (P.gb_slot[j] < 0) return fail(PA_EUNSUPPORTED, "too many distinct columns in one query");
    P.slot_gb[P.gb_slot[j]] = 1;
  }
  P.agg_slot.assign(s.num_aggs, 0);
  for (int a = 0; a < s.num_aggs; ++a) {
    const int t = s.aggs[a].type;
    if (t < PA_AGG_COUNT || t > PA_AGG_DISTINCTCOUNT) return fail(PA_EINVAL, "bad aggregation type");
    if (t == PA_AGG_COUNT) continue;
    P.agg_slot[a] = slot_of(q, s.aggs[a].column_id);
    if (P.agg_slot[a] < 0) return fail(PA_EUNSUPPORTED, "too many distinct columns in one query");
    if (t == PA_AGG_DISTINCTCOUNTHLL && (s.aggs[a].log2m < 4 || s.aggs[a].log2m > 16))
      return fail(PA_EINVAL, "log2m must be 4..16");
    if (t == PA_AGG_DISTINCTCOUNT && (s.aggs[a].num_values < 1 || s.aggs[a].num_values > INT32_MAX))
      return fail(PA_EINVAL, "DISTINCTCOUNT needs the table-wide value count (1..2^31-1)");
  }
  // Post-filter columns (group-by keys, aggregated values) are staged with the filter columns when the filter lets
  // enough docs per wave tile through; below that each surviving doc reads them from HBM. Staging costs the columns'
  // whole tile (256 * nb bytes per nb-bit column); a lazy doc costs about one 64-byte sector per column, and its reads
  // sit on the doc's dependency chain, so lazy is chosen below half the byte break-even: 2 * sum(nb) docs per tile (and
  // never below the old fixed floor of a quarter doc).
  P.slot_post.assign(kMaxSlots, 0);
  for (int j = 0; j < s.num_group_by; ++j) P.slot_post[P.gb_slot[j]] = 1;
  for (int a = 0; a < s.num_aggs; ++a)
    if (s.aggs[a].type != PA_AGG_COUNT) P.slot_post[P.agg_slot[a]] = 1;
  int post_bits = 0;
  for (int sl = 0; sl < kMaxSlots; ++sl) {
    if (!P.slot_post[sl] || sl >= (int)q->slot_cols.size() || !q->nseg) continue;
    auto it = q->segs[0]->cols.find(q->slot_cols[sl]);
    if (it != q->segs[0]->cols.end() && it->second->kind == COL_SV_DICT) post_bits += it->second->nbits;
  }
  // GROUP BY queries read their post-filter columns lazily up to half a tile of matching docs: staging them deepens
  // every ring slot, and the LDS / partitioned strategies (accumulators or bins next to the ring) then lose resident
  // workgroups — measured at 1B docs, GROUP BY day SUM(dictionary metric): 10 % 3.78 -> 2.97 ms, 50 % 6.88 -> 6.71 ms;
  // configs[2] with a 10 % filter 1.63 -> 1.38 ms. Aggregation-only queries (per-lane accumulators, no LDS tables)
  // keep the byte rule: lazy there measured slower (dictionary SUM at 50 %: 0.49 -> 0.68 ms per 200M docs).
  const double kLazyPost = std::max(0.25, 2.0 * post_bits);
  const double lazy_up_to = s.num_group_by > 0 ? std::max(kLazyPost, 0.5 * kWTileDocs) : kLazyPost;
  P.stage_all = !P.has_filter || (s.flags & PA_QF_STAGE_ALL);
  P.stage_post = P.stage_all || (P.post_density > lazy_up_to && !(s.flags & PA_QF_LAZY_POST));
  return PA_OK;
}

// Key space. Direct: table-wide key id = sum_j id_j * prod_{k<j} card_k (DictionaryBasedGroupKeyGenerator raw key)
// indexes the accumulators, when every group-by column has a dictionary and the product fits kDirectMaxKeys. Hashed:
// the components (dictionary key ids, raw value bits for no-dictionary columns) are packed side by side into one
// 64-bit key, mapped to an accumulator slot by a global open-addressing table (the IntMap / LongMap /
// NoDictionary*GroupKeyGenerator holders of the reference).
int plan_key_space(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  q->hashed = false;
  q->key_words = 1;
  P.gb_word.assign(s.num_group_by, 0);
  std::vector<int> gb_bits(s.num_group_by, 0);
  P.gb_raw.assign(s.num_group_by, 0);
  bool direct_ok = true;
  int64_t K = 1;
  P.stride.assign(s.num_group_by, 0);
  for (int j = 0; j < s.num_group_by; ++j) {
    auto it = q->segs[0]->cols.find(s.group_by_columns[j]);
    if (it == q->segs[0]->cols.end()) return fail(PA_EINVAL, "group-by column missing in segment 0");
    if (it->second->kind == COL_SV_RAW) {
      P.gb_raw[j] = 1;
      const int vt = it->second->vtype;
      gb_bits[j] = (vt == PA_INT || vt == PA_FLOAT) ? 32 : 64;
      direct_ok = false;
      continue;
    }
    const int64_t card = s.group_by_cardinality[j];
    if (card < 1) return fail(PA_EINVAL, "group_by_cardinality < 1 for a dictionary column");
    gb_bits[j] = std::max(1, 64 - __builtin_clzll((unsigned long long)std::max<int64_t>(card - 1, 1)));
    P.stride[j] = K;
    if (K > kDirectMaxKeys / card) direct_ok = false;
    else K *= card;
  }
  if (!direct_ok) {
    // components side by side in one 64-bit word; wider together, in two words (a component never straddles them:
    // first fit in column order), the table then keeping [k0, k1, state] per slot (pa_keys.h ht_slot2)
    int total_bits = 0;
    for (int j = 0; j < s.num_group_by; ++j) total_bits += gb_bits[j];
    q->key_words = total_bits > 64 ? 2 : 1;
    int used[2] = {0, 0};
    for (int j = 0; j < s.num_group_by; ++j) {
      int w = 0;
      if (used[0] + gb_bits[j] > 64) w = 1;
      if (q->key_words == 1 ? w != 0 : used[w] + gb_bits[j] > 64)
        return fail(PA_EUNSUPPORTED, "packed group key wider than 128 bits");
      P.gb_word[j] = w;
      P.stride[j] = used[w] < 64 ? (int64_t)(uint64_t(1) << used[w]) : 0;
      q->key_shift[j] = 64 * w + used[w];
      used[w] += gb_bits[j];
    }
    // slots: twice the keys that can exist (docs, or docs x values for MV group-by), at least 1024, a power of two
    uint64_t bound = 0;
    for (int si = 0; si < q->nseg; ++si) {
      uint64_t n = (uint64_t)q->segs[si]->num_docs;
      for (int j = 0; j < s.num_group_by; ++j) {
        auto it = q->segs[si]->cols.find(s.group_by_columns[j]);
        if (it != q->segs[si]->cols.end() && it->second->kind == COL_MV_DICT)
          n = std::max<uint64_t>(n, (uint64_t)it->second->total_values) * 2;
      }
      bound += n;
    }
    if (s.hash_keys_bound > 0) bound = std::max<uint64_t>(bound, (uint64_t)s.hash_keys_bound);
    uint64_t H = 1024;
    while (H < 2 * bound && H < kMaxHashSlots) H <<= 1;
    q->hashed = true;
    q->ht_slots = (int64_t)H;
    K = (int64_t)H + 1;  // + the reserved slot of the key INT64_MAX (the table's empty marker)
  }
  q->num_keys = K;
  return PA_OK;
}

// The one multi-value group-by component (multi-value in every segment) of a query that partitions or walks its
// (doc, value) pairs: its index, -1 when no group-by column is multi-value anywhere, -2 when several are or one is
// multi-value in some segments only (the per-doc expansion paths run those).
int mv_group_component(const pa_query* q) {
  const pa_query_spec& s = q->spec;
  int comp = -1;
  for (int j = 0; j < s.num_group_by; ++j) {
    int nmv = 0;
    for (int si = 0; si < q->nseg; ++si) {
      auto it = q->segs[si]->cols.find(s.group_by_columns[j]);
      nmv += it != q->segs[si]->cols.end() && it->second->kind == COL_MV_DICT;
    }
    if (nmv == 0) continue;
    if (nmv != q->nseg || comp >= 0) return -2;
    comp = j;
  }
  return comp;
}

// numGroupsLimit. The reference caps each segment's group table at numGroupsLimit first-seen groups
// (DictionaryBasedGroupKeyGenerator._globalGroupIdUpperBound, NoDictionary*GroupKeyGenerator). It can only bind when a
// segment can hold that many distinct keys: min(product of its key cardinalities (a raw column: its docs), its
// expanded (doc, key) pairs). Then the first-seen trimming passes run instead of the fused scan.
int plan_limit(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  q->limit_mode = false;
  q->limit_walk = false;
  P.limit_pairs = 0;
  P.limit_eb = 0;
  P.limit_bind.assign(q->nseg, 0);
  if (s.num_group_by == 0 || s.num_groups_limit <= 0) return PA_OK;
  auto sat_mul = [](uint64_t a, uint64_t b) { return (b != 0 && a > UINT64_MAX / b) ? UINT64_MAX : a * b; };
  uint64_t max_exp = 1;
  for (int si = 0; si < q->nseg; ++si) {
    const pa_segment* seg = q->segs[si];
    uint64_t distinct = 1, per_doc = 1;
    int nmv = 0;
    int64_t mv_total = 0;
    for (int j = 0; j < s.num_group_by; ++j) {
      auto it = seg->cols.find(s.group_by_columns[j]);
      if (it == seg->cols.end()) return fail(PA_EINVAL, "group-by column missing in segment " + std::to_string(si));
      const Column* c = it->second;
      distinct = sat_mul(distinct, c->kind == COL_SV_RAW ? (uint64_t)seg->num_docs : (uint64_t)c->cardinality);
      if (c->kind == COL_MV_DICT) {
        per_doc = sat_mul(per_doc, (uint64_t)c->max_values);
        mv_total = c->total_values;
        ++nmv;
      }
    }
    const uint64_t pairs = nmv == 1 ? (uint64_t)mv_total : sat_mul((uint64_t)seg->num_docs, per_doc);
    const uint64_t bound = std::min(distinct, pairs);
    if (bound >= (uint64_t)s.num_groups_limit) q->limit_mode = true;
    P.limit_bind[si] = bound >= (uint64_t)s.num_groups_limit;
    P.limit_pairs = std::min<uint64_t>(UINT64_MAX / 4, P.limit_pairs + bound);
    max_exp = std::max(max_exp, per_doc);
  }
  while (P.limit_eb < 63 && (uint64_t(1) << P.limit_eb) < max_exp) ++P.limit_eb;
  // Walk form: one key per doc (no MV group-by) in a direct key space; its bitmaps (LDS while they fit, else HBM)
  // take at most kWalkMaxBitmapBytes. One MV group-by column (keys per (doc, value) pair): the bitmap and its round
  // snapshot in LDS.
  int64_t nbind = 0;
  for (int si = 0; si < q->nseg; ++si) nbind += P.limit_bind[si] ? 1 : 0;
  const int64_t words = (q->num_keys + 31) / 32;
  const int mvc = mv_group_component(q);
  const bool walk_ok = (mvc == -1 && max_exp == 1) || (mvc >= 0 && 2 * words <= kWalkMaxWords);
  if (q->limit_mode && !q->hashed && walk_ok &&
      (uint64_t)nbind * (uint64_t)words * 4 <= kWalkMaxBitmapBytes && !(s.flags & PA_QF_NO_LIMIT_WALK)) {
    q->limit_mode = false;
    q->limit_walk = true;
    q->walk_words = (q->num_keys + 31) / 32;
  }
  if (q->limit_mode) {
    if (P.limit_eb > 21) return fail(PA_EUNSUPPORTED, "numGroupsLimit trimming: more than 2^21 group keys in one doc");
    if (q->nseg >= 4095) return fail(PA_EUNSUPPORTED, "numGroupsLimit trimming: more than 4094 segments in one query");
  }
  return PA_OK;
}


// STRAT_GDENSE (pa_gdense.h): a filter + GROUP BY whose matching docs are dense enough to stage every column the query
// reads, over a small box of group keys, with COUNT / SUM / MIN / MAX over single-value columns. Decides eligibility, the
// key box, each aggregation's value source and LDS operation, and the LDS layout (accumulators with per-lane replicas,
// per-segment tables). Runs before build_segments, which stages the columns it asks for.
int plan_gdense(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  P.gdense = false;
  if (s.num_group_by < 1 || s.num_group_by > kGdMaxGb || q->nseg == 0 || q->hashed || q->limit_mode || q->limit_walk)
    return PA_OK;
  {
    int nvalue = 0;
    for (int a = 0; a < s.num_aggs; ++a) nvalue += s.aggs[a].type != PA_AGG_COUNT;
    if (nvalue > kGdMaxAgg) return PA_OK;
  }
  if (s.flags & (PA_QF_NO_DENSE_GROUP | PA_QF_FORCE_GLOBAL | PA_QF_FORCE_LDS | PA_QF_LAZY_POST | PA_QF_NO_LANE_MAJOR |
                 PA_QF_STEPS16 | PA_QF_DEBUG_STREAM_ONLY))
    return PA_OK;
  // every filter literal eager and a dictionary leaf on a staged column (no per-doc HBM reads in the tile loop)
  if (q->num_eager != (int)q->literals.size()) return PA_OK;
  for (const Literal& lit : q->literals) {
    const int k = s.leaves[lit.leaf].kind;
    if (k != PA_LEAF_DICT_RANGE && k != PA_LEAF_DICT_SET) return PA_OK;
  }
  // columns: group-by columns dictionary-encoded; aggregations COUNT / SUM / MIN / MAX over single-value columns of one
  // kind in every segment
  for (int si = 0; si < q->nseg; ++si)
    for (int j = 0; j < s.num_group_by; ++j) {
      auto it = q->segs[si]->cols.find(s.group_by_columns[j]);
      if (it == q->segs[si]->cols.end() || it->second->kind != COL_SV_DICT) return PA_OK;
    }
  const int na = s.num_aggs;
  std::vector<int> kind(na, COL_NONE);
  for (int a = 0; a < na; ++a) {
    const int t = s.aggs[a].type;
    if (t == PA_AGG_COUNT) continue;
    if (t != PA_AGG_SUM && t != PA_AGG_MIN && t != PA_AGG_MAX) return PA_OK;
    for (int si = 0; si < q->nseg; ++si) {
      auto it = q->segs[si]->cols.find(s.aggs[a].column_id);
      if (it == q->segs[si]->cols.end()) return PA_OK;
      const Column* c = it->second;
      if (si == 0) kind[a] = c->kind;
      if (c->kind != kind[a] || (c->kind != COL_SV_DICT && c->kind != COL_SV_RAW)) return PA_OK;
      if (c->vtype != q->segs[0]->cols.at(s.aggs[a].column_id)->vtype) return PA_OK;
      if (c->vtype != PA_INT && c->vtype != PA_LONG && c->vtype != PA_FLOAT && c->vtype != PA_DOUBLE) return PA_OK;
      if (c->kind == COL_SV_DICT && c->hvals.size() != (size_t)c->cardinality) return PA_OK;
    }
  }
  // staged columns (filter + post-filter, raw ones as 32/64-bit columns); tile images of the lane-major 2048-doc layout
  // (at most kLmStaged columns and kLmEager literals) and of the step-major 1024-doc one (wide images)
  std::vector<char> st(kMaxSlots, 0);
  for (int li = 0; li < q->num_eager; ++li) st[P.leaf_slot[q->literals[li].leaf]] = 1;
  for (int sl = 0; sl < kMaxSlots; ++sl) st[sl] |= P.slot_post[sl];
  int nst = 0, post_bits = 0;
  int img32 = kGuardWords, img16 = kGuardWords;
  for (int si = 0; si < q->nseg; ++si) {
    int n = 0, dw32 = kGuardWords, dw16 = kGuardWords, pb = 0;
    for (int sl = 0; sl < (int)q->slot_cols.size(); ++sl) {
      if (!st[sl]) continue;
      const Column* c = q->segs[si]->cols.at(q->slot_cols[sl]);
      const int nb = c->kind == COL_SV_RAW ? ((c->vtype == PA_INT || c->vtype == PA_FLOAT) ? 32 : 64) : c->nbits;
      ++n;
      dw32 += 2 * 32 * nb + kGuardWords;
      dw16 += 2 * 16 * nb + kGuardWords;
      if (P.slot_post[sl]) pb += nb;
    }
    nst = std::max(nst, n);
    img32 = std::max(img32, dw32);
    img16 = std::max(img16, dw16);
    post_bits = std::max(post_bits, pb);
  }
  const bool lm_ok = nst <= kLmStaged && q->num_eager <= kLmEager;
  const int max_img_dw = lm_ok ? std::min(img32, img16) : img16;  // (the smaller image decides whether it fits at all)
  // density: staging the post-filter columns costs 256 nb bytes per tile and column; reading them per matching doc costs
  // about a 64-byte sector each (and waits behind the ring): stage above half the byte break-even, like plan_slots
  if (P.has_filter && P.post_density <= std::max(0.25, 2.0 * post_bits)) return PA_OK;
  // key box: a CNF unit clause on a group-by column (DICT_RANGE / DICT_SET, not negated) bounds the table key ids of
  // the docs that can match; union over segments (through their remaps), intersection over clauses
  int64_t lo[PA_MAX_GROUP_BY], hi[PA_MAX_GROUP_BY];
  for (int j = 0; j < s.num_group_by; ++j) {
    lo[j] = 0;
    hi[j] = s.group_by_cardinality[j];
  }
  // The box IS the filter when every literal is a unit DICT_RANGE clause on a group-by column, not negated, with a
  // non-empty hull: dictionaries are sorted, so the table key ids of a value range form one run, and a doc's key lies
  // in the box iff its value lies in every range (the kernel then box-checks every doc instead of evaluating the filter
  // and walking its matches)
  bool box_exact = !q->literals.empty();
  for (size_t i = 0; i < q->literals.size(); ++i) {
    const bool unit = q->clause_end[i] && (i == 0 || q->clause_end[i - 1]);
    const Literal lit = q->literals[i];
    bool on_gb = false;
    for (int j = 0; j < s.num_group_by; ++j) on_gb |= s.leaves[lit.leaf].column_id == s.group_by_columns[j];
    if (!unit || !on_gb || s.leaves[lit.leaf].kind != PA_LEAF_DICT_RANGE) box_exact = false;
    if (!unit) continue;
    for (int j = 0; j < s.num_group_by; ++j) {
      if (s.leaves[lit.leaf].column_id != s.group_by_columns[j]) continue;
      int64_t ulo = INT64_MAX, uhi = INT64_MIN;
      bool bounded = true;
      for (int si = 0; si < q->nseg && bounded; ++si) {
        const pa_leaf_params& p = q->leaf_params[si][lit.leaf];
        if ((p.negate != 0) != lit.neg) {
          bounded = false;
          break;
        }
        const Column* c = q->segs[si]->cols.at(s.group_by_columns[j]);
        const std::vector<int32_t>* rm = q->has_remap[si][j] ? &q->remaps[si][j] : nullptr;
        auto take = [&](int64_t id) {
          const int64_t k = rm ? (int64_t)(*rm)[id] : id;
          ulo = std::min(ulo, k);
          uhi = std::max(uhi, k + 1);
        };
        if (s.leaves[lit.leaf].kind == PA_LEAF_DICT_RANGE) {
          const int64_t a = std::max<int64_t>(0, p.lo), b = std::min<int64_t>(p.hi, c->cardinality);
          if (rm) {
            for (int64_t id = a; id < b; ++id) take(id);
          } else if (b > a) {
            take(a);
            take(b - 1);
          }
        } else {
          const std::vector<uint32_t>& lut = q->luts[si][lit.leaf];
          for (int64_t id = 0; id < c->cardinality && (size_t)(id >> 5) < lut.size(); ++id)
            if ((lut[id >> 5] >> (id & 31)) & 1u) take(id);
        }
      }
      if (!bounded) {
        box_exact = false;
        continue;
      }
      if (ulo == INT64_MAX) {  // no segment can match: an empty box (a span of one key keeps it simple)
        ulo = uhi = 0;
        box_exact = false;
      }
      lo[j] = std::max(lo[j], ulo);
      hi[j] = std::max(lo[j], std::min(hi[j], uhi));
    }
  }
  int64_t nkeys = 1;
  for (int j = 0; j < s.num_group_by; ++j) {
    if (hi[j] <= lo[j]) {  // (disjoint ranges: nothing matches)
      hi[j] = lo[j] + 1;
      box_exact = false;
    }
    P.gd_lo[j] = (int)lo[j];
    P.gd_span[j] = (int)(hi[j] - lo[j]);
    P.gd_ls[j] = (int)nkeys;
    nkeys *= hi[j] - lo[j];
    if (nkeys > kGdMaxKeys) return PA_OK;
  }
  P.gd_nkeys = (int)nkeys;
  P.gd_box_ok = true;
  // the box as the filter from 30 % selectivity up (below it the filter + walk over the matches costs less VALU)
  // (opt-in: measured slower than filter + walk on configs[0]'s GROUP BY day at 50 %, r04_d10)
  P.gd_box = box_exact && !(s.flags & PA_QF_NO_BOX_FILTER) && (s.flags & PA_QF_BOX_FILTER);
  // per-segment key tables where some segment remaps the column
  size_t tab_bytes = 0;
  P.gd_tables = 0;
  std::vector<size_t> gtab(s.num_group_by, 0), atab(na, 0);
  for (int j = 0; j < s.num_group_by; ++j) {
    P.gd_tab[j] = -1;
    P.gd_tab_n[j] = 0;
    bool any = false;
    int32_t n = 0;
    for (int si = 0; si < q->nseg; ++si) {
      any |= q->has_remap[si][j] != 0;
      n = std::max(n, q->segs[si]->cols.at(s.group_by_columns[j])->cardinality);
    }
    if (!any) continue;
    P.gd_tab_n[j] = n;
    gtab[j] = ((size_t)n * 4 + 15) & ~(size_t)15;
    tab_bytes += gtab[j];
    P.gd_tables = 1;
  }
  // aggregations: value source and LDS operation
  P.gd_vs.assign(na, 0);
  P.gd_op.assign(na, 0);
  P.gd_acc.assign(na, 0);
  P.gd_tab_a.assign(na, -1);
  P.gd_tab_an.assign(na, 0);
  P.gd_base.assign(na, 0);
  P.gd_step.assign(na, 0);
  P.gd_stage_raw.assign(kMaxSlots, 0);
  P.gd_src.assign(q->nseg, std::vector<const void*>(na, nullptr));
  std::vector<size_t> row(na, 0);  // accumulator bytes per key replica
  for (int a = 0; a < na; ++a) {
    const int t = s.aggs[a].type;
    if (t == PA_AGG_COUNT) continue;
    const Column* c0 = q->segs[0]->cols.at(s.aggs[a].column_id);
    const int vt = c0->vtype;
    const bool fl = vt == PA_FLOAT || vt == PA_DOUBLE;
    bool fits = true, shared = true;
    int32_t card = 0;
    for (int si = 0; si < q->nseg; ++si) {
      const Column* c = q->segs[si]->cols.at(s.aggs[a].column_id);
      fits = fits && c->fits_int32;
      shared = shared && (c == c0 || (c->dict_hash == c0->dict_hash && c->hvals == c0->hvals));
      card = std::max(card, c->cardinality);
    }
    int vs, op;
    if (kind[a] == COL_SV_RAW) {
      P.gd_stage_raw[P.agg_slot[a]] = 1;
      vs = vt == PA_INT ? GVS_RI32 : vt == PA_FLOAT ? GVS_RF32 : vt == PA_LONG ? GVS_RI64 : GVS_RF64;
      op = t == PA_AGG_SUM ? (fl ? GOP_SUM_F : (fits ? GOP_SUM_I : GOP_SUM_L)) : (t == PA_AGG_MIN ? GOP_MIN_I : GOP_MAX_I);
    } else {
      int64_t b = 0, stp = 0;
      if (t == PA_AGG_SUM && !fl && shared && affine_dictionary(c0->hvals, vt, &b, &stp)) {
        vs = GVS_ID;
        op = GOP_SUM_I;
        P.gd_base[a] = b;
        P.gd_step[a] = stp;
      } else if (t != PA_AGG_SUM && shared && c0->dict_sorted) {
        vs = GVS_ID;
        op = t == PA_AGG_MIN ? GOP_MIN_U : GOP_MAX_U;
      } else {
        vs = fl ? GVS_TF : (fits ? GVS_T32 : GVS_T64);
        op = t == PA_AGG_SUM ? (fl ? GOP_SUM_F : (fits ? GOP_SUM_I : GOP_SUM_L)) : (t == PA_AGG_MIN ? GOP_MIN_I : GOP_MAX_I);
        P.gd_tab_an[a] = card;
        atab[a] = ((size_t)card * (vs == GVS_T32 ? 4 : 8) + 15) & ~(size_t)15;
        tab_bytes += atab[a];
        P.gd_tables = 1;
        // identical dictionaries share one device pointer: the workgroup loads the table once
        std::map<uint64_t, std::vector<int>> first;  // dict hash -> segments holding a distinct dictionary with it
        for (int si = 0; si < q->nseg; ++si) {
          const Column* c = q->segs[si]->cols.at(s.aggs[a].column_id);
          const void* src = c->dict.p;
          for (int sj : first[c->dict_hash]) {
            const Column* d = q->segs[sj]->cols.at(s.aggs[a].column_id);
            if (d->hvals == c->hvals) {
              src = d->dict.p;
              break;
            }
          }
          if (src == c->dict.p) first[c->dict_hash].push_back(si);
          P.gd_src[si][a] = src;
        }
      }
    }
    P.gd_vs[a] = vs;
    P.gd_op[a] = op;
    row[a] = op == GOP_SUM_L ? 16 : (op == GOP_MIN_U || op == GOP_MAX_U) ? 4 : 8;
  }
  // Packed accumulation for the lane-major walk: COUNT and every aggregation a SUM whose per-doc term is a small
  // non-negative integer — the dictId of an affine dictionary (GVS_ID), or the value minus the smallest value of every
  // segment's dictionary (a value table of uint32 offsets, GVS_T32U). Fields: each term w_a + c bits, COUNT c bits
  // (the top), c as large as 64 bits allow; a field then holds 2^c - 1 docs' terms, so the waves drain every
  // (2^c - 1) / 1024 tiles (c >= 11).
  P.gd_pk_ok = false;
  P.gd_pk_w.assign(na, 0);
  P.gd_pk_t32u.assign(na, 0);
  P.gd_pk_base.assign(na, 0);
  if (!(s.flags & PA_QF_NO_GD_PACK)) {
    bool ok = true;
    int wsum = 0, nsum = 0;
    for (int a = 0; a < na && ok; ++a) {
      const int t = s.aggs[a].type;
      if (t == PA_AGG_COUNT) continue;
      if (t != PA_AGG_SUM || P.gd_op[a] != GOP_SUM_I || kind[a] != COL_SV_DICT) {
        ok = false;
        break;
      }
      int w = 0;
      if (P.gd_vs[a] == GVS_ID) {
        int32_t card = 1;
        for (int si = 0; si < q->nseg; ++si) card = std::max(card, q->segs[si]->cols.at(s.aggs[a].column_id)->cardinality);
        while (w < 32 && (int64_t(1) << w) < (int64_t)card) ++w;
      } else if (P.gd_vs[a] == GVS_T32 || P.gd_vs[a] == GVS_T64) {
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int si = 0; si < q->nseg; ++si)
          for (uint64_t x : q->segs[si]->cols.at(s.aggs[a].column_id)->hvals) {
            lo = std::min(lo, (int64_t)x);
            hi = std::max(hi, (int64_t)x);
          }
        if (lo > hi || (__int128)hi - (__int128)lo >= ((__int128)1 << 32)) {
          ok = false;
          break;
        }
        const uint64_t span = (uint64_t)(hi - lo);
        while (w < 32 && (span >> w) != 0) ++w;
        P.gd_pk_t32u[a] = 1;
        P.gd_pk_base[a] = lo;
      } else {
        ok = false;
        break;
      }
      P.gd_pk_w[a] = w;
      wsum += w;
      ++nsum;
    }
    const int c = (64 - wsum) / (1 + nsum);
    if (ok && c >= 11) {
      P.gd_pk_ok = true;
      P.gd_pk_c = std::min(c, 31);
    }
  }
  // DICT_SET bitmaps identical in every segment go to LDS too (their per-doc reads would otherwise be global loads
  // in the tile loop, each waiting for every tile in flight: vmcnt counts in order), when they fit
  P.gd_lut.assign(q->literals.size(), -1);
  P.gd_lut_words.assign(q->literals.size(), 0);
  std::vector<size_t> lutb(q->literals.size(), 0);
  size_t lut_bytes = 0;
  for (size_t li = 0; li < q->literals.size(); ++li) {
    const int leaf = q->literals[li].leaf;
    if (s.leaves[leaf].kind != PA_LEAF_DICT_SET) continue;
    bool same = true;
    for (int si = 1; si < q->nseg && same; ++si) same = q->luts[si][leaf] == q->luts[0][leaf];
    if (!same || q->luts[0][leaf].empty()) continue;
    P.gd_lut_words[li] = (int)q->luts[0][leaf].size();
    lutb[li] = ((size_t)P.gd_lut_words[li] * 4 + 15) & ~(size_t)15;
    lut_bytes += lutb[li];
  }
  // LDS: replicated accumulators + tables + a ring of at least 2 tile images per wave (kGdWaves waves); replicas
  // 256 / keys (a wave's 64 lanes spread over >= 4 addresses per key), fewer while that does not fit
  auto acc_bytes = [&](int rpl) {
    const size_t e = (size_t)nkeys << rpl;
    size_t b = (e * 4 + 15) & ~(size_t)15;
    for (int a = 0; a < na; ++a) b += (e * row[a] + 15) & ~(size_t)15;
    return b;
  };
  const size_t ring_min = (size_t)kGdWaves * 2 * (size_t)max_img_dw * 4;
  int rpl = 0;
  // (4096 slots instead of 256 — 8 replicas for 512 keys — measured no faster: 2.09 -> 2.04 ms at 50 %, r04_f1)
  while (rpl < 5 && ((int64_t)1 << (rpl + 1)) * nkeys <= 256) ++rpl;
  while (rpl > 0 && acc_bytes(rpl) + tab_bytes + lut_bytes + ring_min > kLdsBudget) --rpl;
  if (lut_bytes && acc_bytes(rpl) + tab_bytes + lut_bytes + ring_min > kLdsBudget) {  // (the bitmaps stay in HBM)
    lut_bytes = 0;
    std::fill(lutb.begin(), lutb.end(), 0);
    std::fill(P.gd_lut_words.begin(), P.gd_lut_words.end(), 0);
    while (rpl < 5 && ((int64_t)1 << (rpl + 1)) * nkeys <= 256 && acc_bytes(rpl + 1) + tab_bytes + ring_min <= kLdsBudget)
      ++rpl;
  }
  if (acc_bytes(rpl) + tab_bytes + ring_min > kLdsBudget) return PA_OK;
  P.gd_rp_log2 = rpl;
  // layout: counts, per-aggregation accumulators, key tables, value tables
  const size_t e = (size_t)nkeys << rpl;
  size_t off = (e * 4 + 15) & ~(size_t)15;
  for (int a = 0; a < na; ++a) {
    if (s.aggs[a].type == PA_AGG_COUNT) continue;
    P.gd_acc[a] = (int)off;
    off += (e * row[a] + 15) & ~(size_t)15;
  }
  for (int j = 0; j < s.num_group_by; ++j) {
    if (!gtab[j]) continue;
    P.gd_tab[j] = (int)off;
    off += gtab[j];
  }
  for (int a = 0; a < na; ++a) {
    if (!atab[a]) continue;
    P.gd_tab_a[a] = (int)off;
    off += atab[a];
  }
  for (size_t li = 0; li < q->literals.size(); ++li) {
    if (!lutb[li]) continue;
    P.gd_lut[li] = (int)off;
    off += lutb[li];
    P.gd_tables = 1;
  }
  P.gd_lds = off;
  P.gdense = true;
  P.stage_post = true;  // every post-filter dictionary column with the filter columns (build_segments)
  PLAN_LOG("gdense: keys %d (replicas %d), LDS acc+tables %zu, staged %d, img %d / %d dw", P.gd_nkeys, 1 << rpl, off,
           nst, img32, img16);
  return PA_OK;
}

// Per-segment descriptors: columns (the staged set of the main scan pass), filter literals in the segment's dictId
// space, group-by remaps, aggregation value sources, HLL lookup tables.
int build_segments(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  const int nslots = (int)q->slot_cols.size();
  q->hsegs.assign(q->nseg, DevSeg{});
  P.agg_src.assign(s.num_aggs, SRC_INT);
  P.val_fast.assign(s.num_aggs, 1);  // emit fast path: the value is a dictionary or raw INT/LONG/DOUBLE column
  P.agg_mv.assign(s.num_aggs, 0);    // the aggregation column is multi-value in some segment
  P.gb_mv = false;                   // some group-by column is multi-value in some segment
  q->num_docs = 0;
  int rc;
  for (int si = 0; si < q->nseg; ++si) {
    const pa_segment* seg = q->segs[si];
    DevSeg& d = q->hsegs[si];
    std::memset(&d, 0, sizeof(d));
    d.num_docs = seg->num_docs;
    d.index = si;
    q->num_docs += (uint64_t)seg->num_docs;
    for (int sl = 0; sl < nslots; ++sl) {
      auto it = seg->cols.find(q->slot_cols[sl]);
      if (it == seg->cols.end())
        return fail(PA_EINVAL, "column " + std::to_string(q->slot_cols[sl]) + " missing in segment " + std::to_string(si));
      const Column* c = it->second;
      DevCol& dc = d.cols[sl];
      dc.kind = c->kind;
      dc.nbits = c->nbits;
      dc.vtype = c->vtype;
      dc.words = c->words.p ? (const uint32_t*)c->words.p + kGuardWords : nullptr;
      dc.raw = c->raw.p;
      dc.mv_off = (const int32_t*)c->mv_off.p;
      dc.dict_i64 = (c->vtype == PA_INT || c->vtype == PA_LONG) ? (const int64_t*)c->dict.p : nullptr;
      dc.dict_f64 = (c->vtype == PA_FLOAT || c->vtype == PA_DOUBLE) ? (const double*)c->dict.p : nullptr;
      dc.lds_off = -1;
      dc.card = c->cardinality;
      dc.flags = c->dict_sorted ? COLF_DICT_SORTED : 0;
      if (c->kind == COL_SV_DICT && (P.slot_eager[sl] || P.stage_all || (P.stage_post && P.slot_post[sl]))) {
        dc.lds_off = 0;  // staged; the region offset depends on the tile size (apply_layout)
        d.stage[d.num_staged++] = StageDesc{dc.words, dc.nbits, 0};
      } else if (c->kind == COL_SV_RAW && P.gdense && P.gd_stage_raw[sl]) {
        // STRAT_GDENSE: a raw column staged as a 32/64-bit column (a wave tile = 2048 values, 8 or 16 KiB)
        dc.lds_off = 0;
        d.stage[d.num_staged++] = StageDesc{(const uint32_t*)dc.raw, (c->vtype == PA_INT || c->vtype == PA_FLOAT) ? 32 : 64, 0};
      }
    }
    if (P.gdense)
      for (int a = 0; a < s.num_aggs; ++a) d.gd_src[a] = P.gd_src[si][a];
    // filter literals
    for (size_t li = 0; li < q->literals.size(); ++li) {
      const Literal lit = q->literals[li];
      const pa_leaf_params& p = q->leaf_params[si][lit.leaf];
      DevLeaf& L = d.leaves[li];
      L.kind = s.leaves[lit.leaf].kind;
      L.slot = P.leaf_slot[lit.leaf];
      L.negate = (p.negate != 0) != lit.neg;
      L.clause_end = q->clause_end[li];
      const DevCol& dc = d.cols[L.slot];
      L.nbits = dc.nbits;
      L.lds_off = dc.lds_off;
      L.words = dc.words;
      L.raw = dc.raw;
      L.vtype = dc.vtype;
      L.mv_off = dc.mv_off;
      if (L.kind == PA_LEAF_DICT_RANGE || L.kind == PA_LEAF_DICT_SET) {
        if (dc.kind != COL_SV_DICT) return fail(PA_EINVAL, "dictionary leaf on a non-dictionary column");
      } else if (L.kind == PA_LEAF_MV_DICT_RANGE || L.kind == PA_LEAF_MV_DICT_SET) {
        if (dc.kind != COL_MV_DICT) return fail(PA_EINVAL, "multi-value leaf on a single-value column");
      } else if (L.kind == PA_LEAF_RAW_RANGE || L.kind == PA_LEAF_RAW_SET) {
        if (dc.kind != COL_SV_RAW) return fail(PA_EINVAL, "raw leaf on a non-raw column");
      }
      if (L.kind == PA_LEAF_DICT_RANGE) {
        // kernel form (leaf_bits): MSB-aligned bounds lo' = lo << (32-nb), hi' = span << (32-nb) - 1;
        // an empty range becomes NOT(full range)
        const int nb = dc.nbits;
        int64_t lo = std::max<int64_t>(0, p.lo);
        int64_t span = (int64_t)p.hi - lo;
        if (span <= 0) {
          lo = 0;
          span = int64_t(1) << nb;
          L.negate = !L.negate;
        }
        if (lo + span > (int64_t(1) << nb)) span = (int64_t(1) << nb) - lo;
        L.lo = (int32_t)(uint32_t)((uint64_t)lo << (32 - nb));
        L.span = (int32_t)(uint32_t)(((uint64_t)span << (32 - nb)) - 1);
      } else if (L.kind == PA_LEAF_MV_DICT_RANGE) {  // plain bounds: lo <= id < lo + span
        const int64_t card = (int64_t)seg->cols.at(s.leaves[lit.leaf].column_id)->cardinality;
        const int64_t lo = std::max<int64_t>(0, p.lo), hi = std::min<int64_t>(p.hi, card);
        L.lo = (int32_t)lo;
        L.span = (int32_t)std::max<int64_t>(0, hi - lo);
      } else if (L.kind == PA_LEAF_DICT_SET || L.kind == PA_LEAF_MV_DICT_SET) {
        const auto& lut = q->luts[si][lit.leaf];
        void* dp = nullptr;
        rc = upload_owned(q, lut.data(), lut.size() * 4, &dp);
        if (rc) return rc;
        L.lut = (const uint32_t*)dp;
      } else if (L.kind == PA_LEAF_RAW_SET) {
        // the sorted values (binary search per doc); the first and last bound the search. An empty set matches no
        // doc: an empty range
        const auto& w = q->luts[si][lit.leaf];
        const int64_t n = (int64_t)w.size() / 2;
        void* dp = nullptr;
        rc = upload_owned(q, w.data(), std::max<size_t>(w.size(), 2) * 4, &dp);
        if (rc) return rc;
        L.lut = (const uint32_t*)dp;
        L.span = (int32_t)n;
        const int64_t* vi = (const int64_t*)w.data();
        const double* vd = (const double*)w.data();
        L.ilo = n ? vi[0] : 1;
        L.ihi = n ? vi[n - 1] : 0;
        L.dlo = n ? vd[0] : 1.0;
        L.dhi = n ? vd[n - 1] : 0.0;
      } else {
        L.ilo = p.ilo;
        L.ihi = p.ihi;
        L.dlo = p.dlo;
        L.dhi = p.dhi;
      }
    }
    // group-by remaps
    for (int j = 0; j < s.num_group_by; ++j) {
      const DevCol& dc = d.cols[P.gb_slot[j]];
      if (P.gb_raw[j]) {
        if (dc.kind != COL_SV_RAW || dc.vtype != q->segs[0]->cols.at(s.group_by_columns[j])->vtype)
          return fail(PA_EINVAL, "a raw group-by column must be raw with the same type in every segment");
        continue;
      }
      if (dc.kind != COL_SV_DICT && dc.kind != COL_MV_DICT)
        return fail(PA_EINVAL, "group-by column is dictionary-encoded in segment 0 but not here");
      if (dc.kind == COL_MV_DICT) {
        q->has_mv = 1;
        P.gb_mv = true;
      }
      if (q->has_remap[si][j]) {
        void* dp = nullptr;
        rc = upload_owned(q, q->remaps[si][j].data(), q->remaps[si][j].size() * 4, &dp);
        if (rc) return rc;
        d.remap[j] = (const int32_t*)dp;
      } else {
        const Column* c = seg->cols.at(s.group_by_columns[j]);
        if (c->cardinality > s.group_by_cardinality[j])
          return fail(PA_EINVAL, "segment cardinality exceeds the key space without a remap");
      }
    }
    // aggregations: value source + HLL lookup tables
    for (int a = 0; a < s.num_aggs; ++a) {
      const pa_agg_spec& A = s.aggs[a];
      if (A.type == PA_AGG_COUNT) continue;
      const Column* c = seg->cols.at(A.column_id);
      if (c->kind == COL_MV_DICT) {
        q->has_mv = 1;
        P.agg_mv[a] = 1;
      }
      if (A.type == PA_AGG_COUNT_MV) {
        if (c->kind != COL_MV_DICT) return fail(PA_EINVAL, "COUNT_MV on a single-value column");
        P.agg_src[a] = SRC_INT;
        continue;
      }
      if (A.type == PA_AGG_DISTINCTCOUNT) {
        if (c->kind != COL_SV_DICT && c->kind != COL_MV_DICT)
          return fail(PA_EUNSUPPORTED, "DISTINCTCOUNT needs a dictionary-encoded column");
        const std::vector<int32_t>& rm = q->vremaps[si][a];
        if (!rm.empty()) {
          void* dp = nullptr;
          rc = upload_owned(q, rm.data(), rm.size() * 4, &dp);
          if (rc) return rc;
          d.hll_lut[a] = (const uint32_t*)dp;
        } else if (c->cardinality > A.num_values) {
          return fail(PA_EINVAL, "segment dictionary larger than the DISTINCTCOUNT value space without a remap");
        }
        P.agg_src[a] = SRC_INT;
        P.val_fast[a] = 0;
        continue;
      }
      const bool wide = (A.flags & PA_AGGF_WIDE_SUM) && A.type == PA_AGG_SUM;  // layout agreed across ranks
      const int src = (c->vtype == PA_FLOAT || c->vtype == PA_DOUBLE) ? SRC_DOUBLE
                                                                     : ((c->fits_int32 && !wide) ? SRC_INT : SRC_LONG);
      if (!(c->kind == COL_SV_DICT ||
            (c->kind == COL_SV_RAW && (c->vtype == PA_INT || c->vtype == PA_LONG || c->vtype == PA_DOUBLE))))
        P.val_fast[a] = 0;
      if (A.type != PA_AGG_DISTINCTCOUNTHLL) {
        if (c->vtype == PA_STRING || c->vtype == PA_BYTES) return fail(PA_EINVAL, "numeric aggregation on a non-numeric column");
        if (c->kind == COL_SV_DICT && !c->dict.p) return fail(PA_EINVAL, "dictionary values missing");
      }
      if (si == 0) {
        P.agg_src[a] = src;
      } else if (P.agg_src[a] != src) {
        if (P.agg_src[a] == SRC_DOUBLE || src == SRC_DOUBLE)
          return fail(PA_EINVAL, "aggregation column type differs across segments");
        P.agg_src[a] = SRC_LONG;  // widen: some segment has values outside int32
      }
      if (A.type == PA_AGG_DISTINCTCOUNTHLL && (c->kind == COL_SV_DICT || c->kind == COL_MV_DICT)) {
        DevBuf b;
        rc = dev_alloc(b, (size_t)c->cardinality * 4);
        if (rc) return rc;
        q->owned.push_back(b);
        hipError_t e;
        if (c->vtype == PA_STRING || c->vtype == PA_BYTES) {
          if (!c->hashes.p) return fail(PA_EINVAL, "DISTINCTCOUNTHLL on a STRING/BYTES dictionary needs dict_hashes");
          e = launch_hll_lut_hashes((const int32_t*)c->hashes.p, c->cardinality, A.log2m, (uint32_t*)b.p, nullptr);
        } else {
          e = launch_hll_lut_numeric((const int64_t*)c->dict.p, (const double*)c->dict.p, c->vtype, c->cardinality,
                                     A.log2m, (uint32_t*)b.p, nullptr);
        }
        if (e != hipSuccess) return fail(PA_EHIP, std::string("hll lut: ") + hipGetErrorString(e));
        d.hll_lut[a] = (const uint32_t*)b.p;
      }
    }
  }
  return PA_OK;
}

// Accumulators: one device block, sections 256-byte aligned.
int plan_accumulators(pa_query* q, Prep& P) {
  const pa_query_spec& s = q->spec;
  const int64_t K = q->num_keys;
  q->sections.clear();
  q->agg_section.assign(s.num_aggs, -1);
  std::vector<std::pair<int32_t, int64_t>> sec;  // kind, elements
  sec.push_back({PA_ACC_COUNT_U64, K});
  for (int a = 0; a < s.num_aggs; ++a) {
    const pa_agg_spec& A = s.aggs[a];
    switch (A.type) {
      case PA_AGG_COUNT: continue;
      case PA_AGG_SUM:
        if (P.agg_src[a] == SRC_LONG) sec.push_back({PA_ACC_SUM_I64X2, 2 * K});
        else sec.push_back({P.agg_src[a] == SRC_INT ? PA_ACC_SUM_I64 : PA_ACC_SUM_F64, K});
        break;
      case PA_AGG_MIN: sec.push_back({PA_ACC_MIN_I64, K}); break;
      case PA_AGG_MAX: sec.push_back({PA_ACC_MAX_I64, K}); break;
      case PA_AGG_DISTINCTCOUNTHLL: sec.push_back({PA_ACC_HLL_U8, K << A.log2m}); break;
      case PA_AGG_COUNT_MV: sec.push_back({PA_ACC_SUM_I64, K}); break;
      case PA_AGG_DISTINCTCOUNT: sec.push_back({PA_ACC_PRESENCE_U8, K * presence_stride(A)}); break;
    }
    q->agg_section[a] = (int)sec.size() - 1;
  }
  q->keys_section = -1;
  if (q->hashed) {
    // slot -> packed key (INT64_MAX = empty), or [k0, k1, state] for two-word keys (state INT64_MAX = empty)
    sec.push_back({PA_ACC_KEYS_I64, K * (q->key_words == 2 ? 3 : 1)});
    q->keys_section = (int)sec.size() - 1;
  }
  sec.push_back({PA_ACC_DOCS_U64, 4});  // [0] numDocsScanned, [1] group-table overflows, [2] limit reached, [3] errors
  size_t total = 0;
  std::vector<size_t> offs;
  for (auto& x : sec) {
    offs.push_back(total);
    total += ((size_t)x.second * section_es(x.first) + 255) & ~(size_t)255;
  }
  int rc = dev_alloc(q->acc, total);
  if (rc) return rc;
  for (size_t i = 0; i < sec.size(); ++i)
    q->sections.push_back({sec[i].first, (char*)q->acc.p + offs[i], sec[i].second});
  // LDS strategy layout: u32 counts, then every aggregation's WG-private accumulators
  P.lds_acc = ((size_t)K * 4 + 15) & ~(size_t)15;
  P.agg_lds.assign(s.num_aggs, 0);
  for (int a = 0; a < s.num_aggs; ++a) {
    const pa_agg_spec& A = s.aggs[a];
    if (A.type == PA_AGG_COUNT) continue;
    P.agg_lds[a] = P.lds_acc;
    const size_t bytes = A.type == PA_AGG_DISTINCTCOUNTHLL ? ((size_t)K << A.log2m) * 4
                         : A.type == PA_AGG_DISTINCTCOUNT ? (size_t)K * presence_stride(A)
                         : (size_t)K * 8 * ((A.type == PA_AGG_SUM && P.agg_src[a] == SRC_LONG) ? 2 : 1);
    P.lds_acc += (bytes + 15) & ~(size_t)15;
  }
  return PA_OK;
}

