/*
 * pinot_oracle.c — CPU ORACLE for parity tests. TEST INFRASTRUCTURE ONLY: imported solely by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker. Never on the product path.
 *
 * Plain-C restatement of the reference's scalar segment-scan algorithm, one doc at a time in docId order:
 *  - oracle_read_int:   PinotDataBitSet.readInt            (pinot-segment-local/.../io/util/PinotDataBitSet.java:80-102)
 *  - filter evaluation:  per-doc evaluation of the filter tree with each leaf's applySV(dictId) / raw compare
 *                        (pinot-core/.../dociditerators/SVScanDocIdIterator.java:203-214 DictIdMatcher,
 *                         And/Or/NotFilterOperator semantics)
 *  - group ids:          DictionaryBasedGroupKeyGenerator raw key  rawKey = sum_j dictId_j * prod_{k<j} card_k
 *                        (query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:266-292, 396-405) and
 *                        IntGroupIdMap.getGroupId first-seen ids capped at numGroupsLimit (:992-1017)
 *  - aggregation:        DefaultGroupByExecutor.process (:140) -> Sum/Min/Max/Count aggregateGroupBySV:
 *                        double accumulation in docId order (SumAggregationFunction.java:230-234,
 *                        MinAggregationFunction.java:241-248), COUNT += 1 (CountAggregationFunction.java:113-117)
 *  - DISTINCTCOUNTHLL:   stream-lib 2.9.8 MurmurHash.hashLong / hash(byte[]) + HyperLogLog.offerHashed
 *                        (offering every doc's value; register max is idempotent, so this equals the reference's
 *                        dictId-bitmap-then-offer of DistinctCountHLLAggregationFunction.java:176-183)
 *  - DISTINCTCOUNT:      per group the set of dictIds seen (DistinctCountAggregationFunction /
 *                        BaseDistinctAggregateAggregationFunction: a dictId bitmap per group, values at extraction)
 *  - multi-value:        FixedBitMVForwardIndexReader.getDictIdMV in docId order (readers/forward/
 *                        FixedBitMVForwardIndexReader.java:106-146: start = previous end, end = next set bit of the
 *                        row-start bitmap, numValues for the last doc), MV leaves via
 *                        BaseDictionaryBasedPredicateEvaluator.applyMV (:164-179: ANY value for inclusive predicates,
 *                        ALL values for exclusive ones), MV group keys via DictionaryBasedGroupKeyGenerator.getIntRawKeys
 *                        (:473-540, cartesian expansion in the reference's order), *MV aggregations
 *                        (SumMVAggregationFunction.java:42-82 etc.: every value of the doc, for every group key)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ PinotDataBitSet.readInt */
int32_t oracle_read_int(const uint8_t* buf, int64_t index, int32_t num_bits) {
  const int64_t bit_offset = index * (int64_t)num_bits;
  int64_t byte_offset = bit_offset / 8;
  const int bit_offset_in_first_byte = (int)(bit_offset % 8);
  int32_t current = buf[byte_offset] & (0xFF >> bit_offset_in_first_byte);
  int num_bits_left = num_bits - (8 - bit_offset_in_first_byte);
  if (num_bits_left <= 0) return (int32_t)((uint32_t)current >> (-num_bits_left));
  while (num_bits_left > 8) {
    byte_offset++;
    current = (int32_t)(((uint32_t)current << 8) | buf[byte_offset]);
    num_bits_left -= 8;
  }
  return (int32_t)(((uint32_t)current << num_bits_left) | ((uint32_t)buf[byte_offset + 1] >> (8 - num_bits_left)));
}

void oracle_read_ints(const uint8_t* buf, int64_t start, int64_t n, int32_t num_bits, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = oracle_read_int(buf, start + i, num_bits);
}

/* PinotDataBitSet.writeInt (PinotDataBitSet.java:143-170), to cross-check the segment creator's packing. */
void oracle_write_int(uint8_t* buf, int64_t index, int32_t num_bits, int32_t value) {
  const int64_t bit_offset = index * (int64_t)num_bits;
  int64_t byte_offset = bit_offset / 8;
  const int bit_in_first = (int)(bit_offset % 8);
  int first = buf[byte_offset];
  int first_mask = 0xFF >> bit_in_first;
  int left = num_bits - (8 - bit_in_first);
  if (left <= 0) {
    first_mask &= (0xFF << (-left)) & 0xFF;
    buf[byte_offset] = (uint8_t)((first & ~first_mask) | (value << (-left)));
  } else {
    buf[byte_offset] = (uint8_t)((first & ~first_mask) | (((uint32_t)value >> left) & first_mask));
    while (left > 8) {
      left -= 8;
      byte_offset++;
      buf[byte_offset] = (uint8_t)(value >> left);
    }
    byte_offset++;
    const int last = buf[byte_offset];
    buf[byte_offset] = (uint8_t)((last & (0xFF >> left)) | (value << (8 - left)));
  }
}

/* ------------------------------------------------------------------ stream-lib 2.9.8 MurmurHash */
int32_t oracle_hash_long(int64_t data) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0;
  uint32_t k = (uint32_t)(int32_t)data * m;
  k ^= k >> 24;
  h ^= k * m;
  k = (uint32_t)(int32_t)(data >> 32) * m;
  k ^= k >> 24;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

int32_t oracle_hash_bytes(const uint8_t* data, int32_t length, int32_t seed) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = (uint32_t)(seed ^ length);
  const int len4 = length >> 2;
  for (int i = 0; i < len4; ++i) {
    const int i4 = i << 2;
    uint32_t k = (uint32_t)(int32_t)(int8_t)data[i4 + 3];
    k = (k << 8) | data[i4 + 2];
    k = (k << 8) | data[i4 + 1];
    k = (k << 8) | data[i4 + 0];
    k *= m;
    k ^= k >> 24;
    k *= m;
    h *= m;
    h ^= k;
  }
  const int left = length - (len4 << 2);
  if (left != 0) {
    if (left >= 3) h ^= (uint32_t)((int32_t)(int8_t)data[length - 3] << 16);
    if (left >= 2) h ^= (uint32_t)((int32_t)(int8_t)data[length - 2] << 8);
    if (left >= 1) h ^= (uint32_t)(int32_t)(int8_t)data[length - 1];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

static void hll_offer(uint8_t* regs, int32_t log2m, int32_t hashed) {
  const uint32_t h = (uint32_t)hashed;
  const uint32_t j = h >> (32 - log2m);
  const uint32_t x = (h << log2m) | ((1u << (log2m - 1)) + 1u);
  const uint32_t r = (uint32_t)__builtin_clz(x) + 1u;
  if (r > regs[j]) regs[j] = (uint8_t)r;
}

/* ------------------------------------------------------------------ query */
enum { OC_DICT = 0, OC_RAW_I32 = 1, OC_RAW_I64 = 2, OC_RAW_F32 = 3, OC_RAW_F64 = 4, OC_MV_DICT = 5 };
enum { OQ_LEAF = 0, OQ_AND = 1, OQ_OR = 2, OQ_NOT = 3 };
enum { OA_COUNT = 0, OA_SUM = 1, OA_MIN = 2, OA_MAX = 3, OA_HLL = 4, OA_COUNTMV = 5, OA_DISTINCT = 6 };

typedef struct {
  int32_t kind;
  int32_t num_bits;
  int32_t cardinality;
  int32_t reserved;
  const uint8_t* fwd;       /* dictionary-encoded forward index bytes */
  const void* raw;          /* raw values */
  const double* dict_f64;   /* dictionary values as double (getDoubleValue) */
  const int32_t* dict_hash; /* MurmurHash.hash(Dictionary.get(dictId)) */
  const uint8_t* mv_bitmap; /* MV: row-start bitmap section (one bit per value, MSB-first) */
  int64_t mv_num_values;    /* MV: total number of values */
} oracle_col;

typedef struct {
  int32_t col;
  int32_t kind;             /* 0 = dictionary leaf (match[]), 1 = raw compare */
  const uint8_t* match;     /* dict leaf: applySV(dictId) for every dictId */
  double dlo, dhi;          /* raw FLOAT/DOUBLE */
  int64_t ilo, ihi;         /* raw INT/LONG */
  int32_t lo_unbounded, hi_unbounded, lo_incl, hi_incl;
  int32_t exclusive;        /* NOT_EQ / NOT_IN: an MV doc matches when ALL its values pass applySV */
  int32_t reserved;
} oracle_leaf;

typedef struct {
  int32_t num_ops;
  const int32_t* ops;       /* postfix, OQ_LEAF | leaf << 8 (leaf index: the upper 24 bits) */
  int32_t num_leaves;
  const oracle_leaf* leaves;
  int32_t num_gb;
  const int32_t* gb_col;
  int64_t num_groups_limit;
  int32_t num_aggs;
  const int32_t* agg_type;
  const int32_t* agg_col;
  const int32_t* agg_log2m;
} oracle_query;

static int32_t dict_id(const oracle_col* c, int64_t doc) { return oracle_read_int(c->fwd, doc, c->num_bits); }

/* PinotDataBitSet.getNextSetBitOffset: first set bit at index >= from (MSB-first within each byte), or -1 */
static int64_t next_set_bit(const uint8_t* bits, int64_t from, int64_t nbits) {
  for (int64_t i = from; i < nbits; ++i)
    if (bits[i >> 3] & (0x80 >> (i & 7))) return i;
  return -1;
}

/* value range [start, end) of the current doc of every MV column: the sequential-docId reader context
 * (FixedBitMVForwardIndexReader's ChunkReaderContext), one per oracle_run_segment call so concurrent calls from
 * several threads (bench.py's cpu_baseline) never share it */
#define OMAX_COLS 32
typedef struct {
  int64_t start[OMAX_COLS], end[OMAX_COLS];
} mv_cursor;

static void mv_advance(mv_cursor* mc, const oracle_col* cols, int ncols, int64_t doc, int64_t num_docs) {
  for (int c = 0; c < ncols && c < OMAX_COLS; ++c) {
    if (cols[c].kind != OC_MV_DICT) continue;
    const int64_t start = doc == 0 ? 0 : mc->end[c];
    int64_t end = doc == num_docs - 1 ? cols[c].mv_num_values
                                      : next_set_bit(cols[c].mv_bitmap, start + 1, cols[c].mv_num_values);
    if (end < 0) end = cols[c].mv_num_values;
    mc->start[c] = start;
    mc->end[c] = end;
  }
}

static double raw_double(const oracle_col* c, int64_t doc) {
  switch (c->kind) {
    case OC_RAW_I32: return (double)((const int32_t*)c->raw)[doc];
    case OC_RAW_I64: return (double)((const int64_t*)c->raw)[doc];
    case OC_RAW_F32: return (double)((const float*)c->raw)[doc];
    default: return ((const double*)c->raw)[doc];
  }
}

static int leaf_match(const mv_cursor* mc, const oracle_leaf* L, const oracle_col* cols, int64_t doc) {
  const oracle_col* c = &cols[L->col];
  if (L->kind == 0 && c->kind == OC_MV_DICT) {
    for (int64_t v = mc->start[L->col]; v < mc->end[L->col]; ++v) {
      const int m = L->match[oracle_read_int(c->fwd, v, c->num_bits)];
      if (L->exclusive && !m) return 0;
      if (!L->exclusive && m) return 1;
    }
    return L->exclusive ? 1 : 0;
  }
  if (L->kind == 0) return L->match[dict_id(c, doc)];
  if (c->kind == OC_RAW_I32 || c->kind == OC_RAW_I64) {
    const int64_t v = c->kind == OC_RAW_I32 ? ((const int32_t*)c->raw)[doc] : ((const int64_t*)c->raw)[doc];
    if (!L->lo_unbounded && (L->lo_incl ? v < L->ilo : v <= L->ilo)) return 0;
    if (!L->hi_unbounded && (L->hi_incl ? v > L->ihi : v >= L->ihi)) return 0;
    return 1;
  }
  if (c->kind == OC_RAW_F32) { /* FloatRawValueBasedRangePredicateEvaluator compares floats */
    const float v = ((const float*)c->raw)[doc];
    if (!L->lo_unbounded && (L->lo_incl ? v < (float)L->dlo : v <= (float)L->dlo)) return 0;
    if (!L->hi_unbounded && (L->hi_incl ? v > (float)L->dhi : v >= (float)L->dhi)) return 0;
    return 1;
  }
  const double v = ((const double*)c->raw)[doc];
  if (!L->lo_unbounded && (L->lo_incl ? v < L->dlo : v <= L->dlo)) return 0;
  if (!L->hi_unbounded && (L->hi_incl ? v > L->dhi : v >= L->dhi)) return 0;
  return 1;
}

static int filter_match(const mv_cursor* mc, const oracle_query* q, const oracle_col* cols, int64_t doc) {
  if (q->num_ops == 0) return 1;
  int st[64];
  int sp = 0;
  for (int i = 0; i < q->num_ops; ++i) {
    const int op = q->ops[i] & 0xff;
    if (op == OQ_LEAF) st[sp++] = leaf_match(mc, &q->leaves[((uint32_t)q->ops[i] >> 8) & 0xffffffu], cols, doc);
    else if (op == OQ_NOT) st[sp - 1] = !st[sp - 1];
    else {
      const int b = st[--sp];
      const int a = st[--sp];
      st[sp++] = op == OQ_AND ? (a && b) : (a || b);
    }
  }
  return st[0];
}

/* open-addressing map rawKey -> groupId (first-seen ids, IntGroupIdMap semantics incl. the limit) */
typedef struct {
  int64_t* keys;
  int32_t* vals;
  int64_t cap;
  int64_t size;
} gmap;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

static int gmap_init(gmap* m, int64_t cap) {
  m->cap = 1024;
  while (m->cap < cap * 2) m->cap <<= 1;
  m->keys = (int64_t*)malloc(sizeof(int64_t) * m->cap);
  m->vals = (int32_t*)malloc(sizeof(int32_t) * m->cap);
  if (!m->keys || !m->vals) return -1;
  for (int64_t i = 0; i < m->cap; ++i) m->keys[i] = -1;
  m->size = 0;
  return 0;
}

static int32_t gmap_get(gmap* m, int64_t key, int64_t limit) {
  uint64_t i = mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
  while (m->keys[i] != -1) {
    if (m->keys[i] == key) return m->vals[i];
    i = (i + 1) & (uint64_t)(m->cap - 1);
  }
  if (m->size >= limit) return -1; /* INVALID_ID once numGroupsLimit groups exist */
  m->keys[i] = key;
  m->vals[i] = (int32_t)m->size;
  return (int32_t)m->size++;
}

/*
 * Runs one segment. Outputs, in group-id (first-seen) order, up to `capacity` groups:
 *   out_keys[g] (raw key), out_counts[g], out_vals[a*capacity + g] (double accumulators of SUM/MIN/MAX;
 *   COUNT/HLL slots unused), out_hll[(a*capacity + g) << 16 ...] registers (u8, stride 1<<log2m per group,
 *   per-agg block of capacity << log2m).
 * Returns the number of groups (aggregation-only queries: always 1), or -1 on allocation failure.
 */
int64_t oracle_run_segment(const oracle_col* cols, int64_t num_docs, const oracle_query* q, int64_t capacity,
                           int64_t* out_keys, int64_t* out_counts, double* out_vals, uint8_t* const* out_hll,
                           int64_t* out_num_matched) {
  gmap map;
  memset(&map, 0, sizeof(map));
  const int grouped = q->num_gb > 0;
  if (grouped && gmap_init(&map, capacity < 1 ? 1 : capacity) != 0) return -1;
  int64_t ngroups = grouped ? 0 : 1;
  if (!grouped) {
    out_keys[0] = 0;
    out_counts[0] = 0;
  }
  for (int a = 0; a < q->num_aggs; ++a) {
    const double init = q->agg_type[a] == OA_MIN ? INFINITY : (q->agg_type[a] == OA_MAX ? -INFINITY : 0.0);
    for (int64_t g = 0; g < capacity; ++g) out_vals[a * capacity + g] = init;
    if (q->agg_type[a] == OA_HLL) memset(out_hll[a], 0, (size_t)capacity << q->agg_log2m[a]);
    if (q->agg_type[a] == OA_DISTINCT) memset(out_hll[a], 0, (size_t)capacity * (size_t)cols[q->agg_col[a]].cardinality);
  }
  int64_t matched = 0;
  int ncols = 0;
  for (int j = 0; j < q->num_gb; ++j) if (q->gb_col[j] + 1 > ncols) ncols = q->gb_col[j] + 1;
  for (int a = 0; a < q->num_aggs; ++a) if (q->agg_col[a] + 1 > ncols) ncols = q->agg_col[a] + 1;
  for (int l = 0; l < q->num_leaves; ++l) if (q->leaves[l].col + 1 > ncols) ncols = q->leaves[l].col + 1;
  int64_t* raw_keys = NULL;
  int64_t raw_cap = 0;
  mv_cursor mc;
  memset(&mc, 0, sizeof(mc));
  for (int64_t doc = 0; doc < num_docs; ++doc) {
    mv_advance(&mc, cols, ncols, doc, num_docs);
    if (!filter_match(&mc, q, cols, doc)) continue;
    matched++;
    /* group keys of this doc: getIntRawKeys (one key for SV-only group-by) */
    int64_t nkeys = 1;
    int64_t rawkey = 0;
    if (grouped) {
      int have_array = 0;
      for (int j = q->num_gb - 1; j >= 0; --j) {
        const oracle_col* gc = &cols[q->gb_col[j]];
        const int64_t card = gc->cardinality;
        if (gc->kind != OC_MV_DICT || mc.end[q->gb_col[j]] - mc.start[q->gb_col[j]] == 1) {
          const int32_t id = gc->kind == OC_MV_DICT ? oracle_read_int(gc->fwd, mc.start[q->gb_col[j]], gc->num_bits)
                                                    : dict_id(gc, doc);
          if (!have_array) rawkey = rawkey * card + id;
          else for (int64_t k = 0; k < nkeys; ++k) raw_keys[k] = raw_keys[k] * card + id;
        } else {
          const int64_t s0 = mc.start[q->gb_col[j]], nv = mc.end[q->gb_col[j]] - s0;
          const int64_t cur = have_array ? nkeys : 1;
          if (cur * nv > raw_cap) {
            raw_cap = cur * nv * 2;
            raw_keys = (int64_t*)realloc(raw_keys, sizeof(int64_t) * raw_cap);
            if (!raw_keys) return -1;
          }
          if (!have_array) {
            for (int64_t v = 0; v < nv; ++v) raw_keys[v] = rawkey * card + oracle_read_int(gc->fwd, s0 + v, gc->num_bits);
            have_array = 1;
          } else {
            /* newRawKeys[v*cur + k] = rawKeys[k] * card + dictId_v, built back to front so it can run in place */
            for (int64_t v = nv - 1; v >= 0; --v) {
              const int32_t id = oracle_read_int(gc->fwd, s0 + v, gc->num_bits);
              for (int64_t k = cur - 1; k >= 0; --k) raw_keys[v * cur + k] = raw_keys[k] * card + id;
            }
          }
          nkeys = cur * nv;
        }
      }
      if (!have_array) {
        if (raw_cap < 1) {
          raw_cap = 16;
          raw_keys = (int64_t*)realloc(raw_keys, sizeof(int64_t) * raw_cap);
          if (!raw_keys) return -1;
        }
        raw_keys[0] = rawkey;
        nkeys = 1;
      }
    }
    for (int64_t kk = 0; kk < nkeys; ++kk) {
      int64_t g = 0;
      if (grouped) {
        const int64_t key = raw_keys[kk];
        const int32_t gid = gmap_get(&map, key, q->num_groups_limit);
        if (gid < 0) continue; /* group limit reached: the doc is not aggregated into this key */
        g = gid;
        if (g >= capacity) continue;
        if (g + 1 > ngroups) {
          ngroups = g + 1;
          out_keys[g] = key;
          out_counts[g] = 0;
        }
      }
      out_counts[g]++;
      for (int a = 0; a < q->num_aggs; ++a) {
        const int t = q->agg_type[a];
        if (t == OA_COUNT) continue;
        const oracle_col* c = &cols[q->agg_col[a]];
        const int mv = c->kind == OC_MV_DICT;
        const int64_t v0 = mv ? mc.start[q->agg_col[a]] : doc;
        const int64_t v1 = mv ? mc.end[q->agg_col[a]] : doc + 1;
        for (int64_t vi = v0; vi < v1; ++vi) {
          if (t == OA_COUNTMV) {
            out_vals[a * capacity + g] += 1.0;
            continue;
          }
          if (t == OA_DISTINCT) { /* the group's value set, as dictId presence (DistinctCountAggregationFunction) */
            out_hll[a][(size_t)g * (size_t)c->cardinality + (size_t)oracle_read_int(c->fwd, vi, c->num_bits)] = 1;
            continue;
          }
          if (t == OA_HLL) {
            int32_t h;
            if (c->kind == OC_DICT || mv) {
              h = c->dict_hash[oracle_read_int(c->fwd, vi, c->num_bits)];
            } else if (c->kind == OC_RAW_I32) {
              h = oracle_hash_long(((const int32_t*)c->raw)[vi]);
            } else if (c->kind == OC_RAW_I64) {
              h = oracle_hash_long(((const int64_t*)c->raw)[vi]);
            } else if (c->kind == OC_RAW_F32) {
              int32_t bits;
              memcpy(&bits, (const float*)c->raw + vi, 4);
              h = oracle_hash_long(bits);
            } else {
              int64_t bits;
              memcpy(&bits, (const double*)c->raw + vi, 8);
              h = oracle_hash_long(bits);
            }
            hll_offer(out_hll[a] + ((size_t)g << q->agg_log2m[a]), q->agg_log2m[a], h);
            continue;
          }
          const double v = (c->kind == OC_DICT || mv) ? c->dict_f64[oracle_read_int(c->fwd, vi, c->num_bits)]
                                                      : raw_double(c, vi);
          double* acc = &out_vals[a * capacity + g];
          if (t == OA_SUM) *acc += v;
          else if (t == OA_MIN) { if (v < *acc) *acc = v; }
          else if (t == OA_MAX) { if (v > *acc) *acc = v; }
        }
      }
    }
  }
  free(raw_keys);
  if (grouped) {
    free(map.keys);
    free(map.vals);
    ngroups = map.size;
  }
  if (out_num_matched) *out_num_matched = matched;
  return ngroups;
}
