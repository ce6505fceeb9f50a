// Host side of the C-ABI (include/pinot_amd.h): segment residency, query planning (CNF filter, column
// slots, staging, accumulator layout, strategy) and result fetch. No CPU fallback: every query runs the
// HIP kernels; errors surface as negative return codes + pa_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "pa_device.h"
#include "pa_launch.h"

using namespace pa;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define PA_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) return fail(PA_EHIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)

#define PA_HIP_NULL(call)                                                             \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) { fail(PA_EHIP, std::string(#call ": ") + hipGetErrorString(e_)); return nullptr; } \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
};

int dev_alloc(DevBuf& b, size_t bytes) {
  b.n = bytes;
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) return fail(PA_ENOMEM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
  return PA_OK;
}

void dev_free(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
}

int64_t wtiles_for(int64_t num_docs) { return (num_docs + kWTileDocs - 1) / kWTileDocs; }

struct Column {
  int32_t kind = COL_NONE;
  int32_t vtype = PA_INT;
  int32_t nbits = 0;
  int32_t cardinality = 0;
  int64_t total_values = 0;
  int32_t max_values = 1;   // MV: most values in one row
  bool fits_int32 = false;  // every dictionary value (INT/LONG) fits in int32
  DevBuf words;   // guard + stream + pad (SV dict)
  DevBuf raw;     // raw values (SV raw)
  DevBuf dict;    // int64 or double
  DevBuf hashes;  // int32 murmur hashes (STRING/BYTES dictionaries)
  DevBuf mv_off;  // MV: int32[num_docs + 1] value offset of every doc's first value
  ~Column() {
    dev_free(mv_off);
    dev_free(words);
    dev_free(raw);
    dev_free(dict);
    dev_free(hashes);
  }
};

}  // namespace

struct pa_segment {
  int32_t num_docs = 0;
  std::map<int32_t, Column*> cols;
  uint64_t bytes = 0;
  ~pa_segment() {
    for (auto& kv : cols) delete kv.second;
  }
};

namespace {

int upload_dict(Column* c, int32_t vtype, int32_t card, const void* dict_values, const int32_t* dict_hashes) {
  c->vtype = vtype;
  c->cardinality = card;
  if (dict_values != nullptr && (vtype == PA_INT || vtype == PA_LONG || vtype == PA_FLOAT || vtype == PA_DOUBLE)) {
    int rc = dev_alloc(c->dict, (size_t)card * 8);
    if (rc) return rc;
    PA_HIP(hipMemcpy(c->dict.p, dict_values, (size_t)card * 8, hipMemcpyHostToDevice));
    if (vtype == PA_INT || vtype == PA_LONG) {
      const int64_t* v = (const int64_t*)dict_values;
      c->fits_int32 = true;
      for (int32_t i = 0; i < card && c->fits_int32; ++i) c->fits_int32 = v[i] >= INT32_MIN && v[i] <= INT32_MAX;
    }
  }
  if (dict_hashes != nullptr) {
    int rc = dev_alloc(c->hashes, (size_t)card * 4);
    if (rc) return rc;
    PA_HIP(hipMemcpy(c->hashes.p, dict_hashes, (size_t)card * 4, hipMemcpyHostToDevice));
  }
  return PA_OK;
}

}  // namespace

extern "C" {

int pa_abi_version(void) { return PA_ABI_VERSION; }

int pa_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pa_set_device(int device) {
  PA_HIP(hipSetDevice(device));
  return PA_OK;
}

const char* pa_last_error(void) { return g_err.c_str(); }

pa_segment* pa_segment_create(int32_t num_docs) {
  if (num_docs < 0) {
    fail(PA_EINVAL, "num_docs < 0");
    return nullptr;
  }
  pa_segment* s = new pa_segment();
  s->num_docs = num_docs;
  return s;
}

int pa_segment_add_sv_dict_column(pa_segment* seg, int32_t column_id, const uint8_t* fwd_index,
                                  uint64_t fwd_index_bytes, int32_t num_bits_per_value, int32_t cardinality,
                                  int32_t value_type, const void* dict_values, const int32_t* dict_hashes) {
  if (!seg) return fail(PA_EINVAL, "null segment");
  if (num_bits_per_value < 1 || num_bits_per_value > 31) return fail(PA_EINVAL, "num_bits_per_value must be 1..31");
  if (cardinality < 1) return fail(PA_EINVAL, "cardinality < 1");
  if (value_type < PA_INT || value_type > PA_BYTES) return fail(PA_EINVAL, "bad value_type");
  const uint64_t need = ((uint64_t)seg->num_docs * (uint64_t)num_bits_per_value + 7) / 8;
  if (fwd_index_bytes < need) return fail(PA_EINVAL, "forward index shorter than ceil(numDocs*numBits/8)");
  if (seg->cols.count(column_id)) return fail(PA_EINVAL, "duplicate column id");
  Column* c = new Column();
  c->kind = COL_SV_DICT;
  c->nbits = num_bits_per_value;
  // guard words | whole wave tiles of 64*nb words | guard words
  const int64_t stream_words = wtiles_for(seg->num_docs) * 64 * num_bits_per_value;
  const int64_t total_words = kGuardWords + stream_words + kGuardWords;
  int rc = dev_alloc(c->words, (size_t)total_words * 4);
  if (rc) { delete c; return rc; }
  uint32_t* w = (uint32_t*)c->words.p;
  if (hipMemset(w, 0, (size_t)total_words * 4) != hipSuccess ||
      hipMemcpy(w + kGuardWords, fwd_index, need, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "forward index upload failed");
  }
  if (launch_bswap_words(w + kGuardWords, (int64_t)((need + 3) / 4), nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "bswap kernel failed");
  }
  rc = upload_dict(c, value_type, cardinality, dict_values, dict_hashes);
  if (rc) { delete c; return rc; }
  seg->bytes += c->words.n + c->dict.n + c->hashes.n;
  seg->cols[column_id] = c;
  return PA_OK;
}

int pa_segment_add_mv_dict_column(pa_segment* seg, int32_t column_id, const uint8_t* fwd_index,
                                  uint64_t fwd_index_bytes, int32_t num_bits_per_value, int32_t cardinality,
                                  int64_t total_num_values, int32_t value_type, const void* dict_values,
                                  const int32_t* dict_hashes) {
  if (!seg) return fail(PA_EINVAL, "null segment");
  if (num_bits_per_value < 1 || num_bits_per_value > 31) return fail(PA_EINVAL, "num_bits_per_value must be 1..31");
  if (cardinality < 1) return fail(PA_EINVAL, "cardinality < 1");
  if (value_type < PA_INT || value_type > PA_BYTES) return fail(PA_EINVAL, "bad value_type");
  if (seg->cols.count(column_id)) return fail(PA_EINVAL, "duplicate column id");
  const int64_t nd = seg->num_docs;
  if (total_num_values < nd || total_num_values > INT32_MAX)
    return fail(PA_EINVAL, "total_num_values must be in [num_docs, 2^31) (every MV row holds at least one value)");
  // FixedBitMVForwardIndexReader.java:66-79 section sizes: chunk offsets | row-start bitmap | bit-packed values
  int64_t num_chunks = 0, docs_per_chunk = 1;
  if (nd > 0) {
    const float avg = (float)(total_num_values / nd);  // Java: int / int, then widened
    docs_per_chunk = (int64_t)std::ceil((double)(2048.0f / avg));
    num_chunks = (nd + docs_per_chunk - 1) / docs_per_chunk;
  }
  const uint64_t bitmap_bytes = (uint64_t)(total_num_values + 7) / 8;
  const uint64_t raw_bytes = ((uint64_t)total_num_values * (uint64_t)num_bits_per_value + 7) / 8;
  const uint64_t header = (uint64_t)num_chunks * 4;
  if (fwd_index_bytes < header + bitmap_bytes + raw_bytes)
    return fail(PA_EINVAL, "MV forward index shorter than its chunk-offset, bitmap and value sections");
  const uint8_t* bitmap = fwd_index + header;
  const uint8_t* raw = bitmap + bitmap_bytes;
  // row starts: the set bits of the bitmap, in order (the reader's getNextSetBitOffset walk, done once at load)
  std::vector<int32_t> off((size_t)nd + 1);
  int64_t d = 0;
  for (int64_t v = 0; v < total_num_values; ++v) {
    if (bitmap[v >> 3] & (0x80 >> (v & 7))) {
      if (d >= nd) return fail(PA_EINVAL, "MV bitmap has more row starts than documents");
      off[d++] = (int32_t)v;
    }
  }
  if (d != nd || (nd > 0 && off[0] != 0)) return fail(PA_EINVAL, "MV bitmap row starts do not match num_docs");
  off[nd] = (int32_t)total_num_values;
  int32_t max_values = 1;
  for (int64_t i = 0; i < nd; ++i) max_values = std::max(max_values, off[i + 1] - off[i]);
  for (int64_t ch = 0; ch < num_chunks; ++ch) {  // chunk offsets (big-endian int32) must agree with the bitmap
    const uint8_t* p = fwd_index + 4 * ch;
    const int64_t co = ((int64_t)p[0] << 24) | ((int64_t)p[1] << 16) | ((int64_t)p[2] << 8) | (int64_t)p[3];
    if (co != off[ch * docs_per_chunk]) return fail(PA_EINVAL, "MV chunk offsets disagree with the row-start bitmap");
  }
  Column* c = new Column();
  c->kind = COL_MV_DICT;
  c->nbits = num_bits_per_value;
  c->total_values = total_num_values;
  c->max_values = max_values;
  // guard words | value stream padded to whole 64-value steps | guard words (reads stay in bounds)
  const int64_t stream_words = ((total_num_values + 2047) / 2048) * 64 * num_bits_per_value;
  const int64_t total_words = kGuardWords + stream_words + kGuardWords;
  int rc = dev_alloc(c->words, (size_t)total_words * 4);
  if (!rc) rc = dev_alloc(c->mv_off, off.size() * 4);
  if (rc) { delete c; return rc; }
  uint32_t* w = (uint32_t*)c->words.p;
  if (hipMemset(w, 0, (size_t)total_words * 4) != hipSuccess ||
      hipMemcpy(w + kGuardWords, raw, raw_bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->mv_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "MV forward index upload failed");
  }
  if (launch_bswap_words(w + kGuardWords, (int64_t)((raw_bytes + 3) / 4), nullptr) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "bswap kernel failed");
  }
  rc = upload_dict(c, value_type, cardinality, dict_values, dict_hashes);
  if (rc) { delete c; return rc; }
  seg->bytes += c->words.n + c->mv_off.n + c->dict.n + c->hashes.n;
  seg->cols[column_id] = c;
  return PA_OK;
}

int pa_segment_add_raw_column(pa_segment* seg, int32_t column_id, int32_t value_type, const void* values) {
  if (!seg) return fail(PA_EINVAL, "null segment");
  if (value_type < PA_INT || value_type > PA_DOUBLE) return fail(PA_EINVAL, "raw columns must be INT/LONG/FLOAT/DOUBLE");
  if (seg->cols.count(column_id)) return fail(PA_EINVAL, "duplicate column id");
  const size_t esz = (value_type == PA_INT || value_type == PA_FLOAT) ? 4 : 8;
  Column* c = new Column();
  c->kind = COL_SV_RAW;
  c->vtype = value_type;
  c->fits_int32 = value_type == PA_INT;
  const size_t padded = (size_t)wtiles_for(seg->num_docs) * kWTileDocs;
  int rc = dev_alloc(c->raw, padded * esz + 16);
  if (rc) { delete c; return rc; }
  if (hipMemset(c->raw.p, 0, padded * esz + 16) != hipSuccess ||
      hipMemcpy(c->raw.p, values, (size_t)seg->num_docs * esz, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return fail(PA_EHIP, "raw column upload failed");
  }
  seg->bytes += c->raw.n;
  seg->cols[column_id] = c;
  return PA_OK;
}

int32_t pa_segment_num_docs(const pa_segment* seg) { return seg ? seg->num_docs : -1; }
uint64_t pa_segment_device_bytes(const pa_segment* seg) { return seg ? seg->bytes : 0; }
void pa_segment_destroy(pa_segment* seg) { delete seg; }

}  // extern "C"

// ====================================================================== queries

namespace {

struct Literal {
  int leaf;
  bool neg;
};
using Clause = std::vector<Literal>;

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

constexpr size_t kFetchWholeBlockBytes = 1 << 20;
constexpr size_t kPartLdsChoices[4] = {144 * 1024, 64 * 1024, 96 * 1024, 144 * 1024};  // PA_QF_PART_SHIFT
constexpr int64_t kMinParts = 256;          // pass C parallelism: one workgroup per partition, >= one per CU
constexpr int64_t kMaxParts = 4096;          // partition counters of the scan passes: 16 KiB of LDS
constexpr size_t kPartBinLdsBytes = 152 * 1024;  // part_bin_kernel: bins + counters (one 1024-thread workgroup per CU)
constexpr int64_t kDirectMaxKeys = int64_t(1) << 27;  // direct-indexed key space limit (beyond: hashed keys)
constexpr uint64_t kMaxHashSlots = uint64_t(1) << 28;

struct Section {
  int32_t kind;
  void* ptr;
  int64_t n;
};

}  // namespace

struct pa_query {
  pa_query_spec spec;
  int32_t nseg = 0;
  std::vector<const pa_segment*> segs;
  std::vector<std::vector<pa_leaf_params>> leaf_params;
  std::vector<std::vector<std::vector<uint32_t>>> luts;        // [seg][leaf]
  std::vector<std::vector<std::vector<int32_t>>> remaps;       // [seg][gb]
  std::vector<std::vector<char>> has_remap;
  bool prepared = false;

  // plan
  std::vector<int32_t> slot_cols;
  std::vector<Literal> literals;
  std::vector<int> clause_end;
  int64_t num_keys = 1;
  int strategy = STRAT_GLOBAL;
  int grid = 0;
  int steps = 32;
  int dma_slots = 8;
  int num_eager = 0;
  int plan_ring = 2;
  int plan_wg = 1;
  int lds_bytes = 0;
  uint64_t staged_bytes = 0;
  uint64_t num_docs = 0;
  uint64_t num_tiles = 0;

  DevQuery hq;
  std::vector<DevSeg> hsegs;
  DevBuf dq, dsegs, dplans;
  void* host_acc = nullptr;  // pinned copy of the accumulator block (small-block fetch path)
  DevBuf fetch_blocks, fetch_stage;  // large-key fetch: per-block counts / compacted rows
  void* fetch_host = nullptr;        // pinned copy of the compacted rows
  int lane_major = 0;
  int has_mv = 0;
  bool hashed = false;           // packed 64-bit keys through a global open-addressing table
  int64_t ht_slots = 0;
  int key_shift[PA_MAX_GROUP_BY] = {0};
  int keys_section = -1;
  bool partitioned = false;      // partitioned aggregation (STRAT_PEMIT scan + part_bin_kernel + part_agg_kernel)
  int part_P = 0, part_shift = 0, rec_words = 0, part_lds_c = 0, bin_slots = 0, bin_iter = 0, bin_parts = 0, emit_val_agg = -1;
  int hll_agg = -1, hll_key_shift = 0;
  bool emit_fast = false;
  std::vector<int> pay_off, part_agg_lds;
  DevBuf part_hist, part_off, part_base, recs, emit, wave_cnt, tile_rec;
  int bin_lds = 0;
  int64_t last_matched = -1;  // numDocsScanned read by the last fetch
  int64_t last_reached = -1;  // segments that reached numGroupsLimit, read by the last fetch
  // numGroupsLimit first-seen trimming (launch_limit_passes): on when some segment can hold numGroupsLimit groups
  bool limit_mode = false;
  LimitDesc limit{};
  int limit_grid = 0;
  DevBuf lim_keys, lim_pos, lim_sk, lim_sorted, lim_thresh, lim_temp;
  size_t lim_temp_bytes = 0;
  std::vector<LmSegPlan> hplans;
  std::vector<DevBuf> owned;  // LUTs, remaps, HLL LUTs
  DevBuf acc;                 // all accumulator sections (unless the caller provided the block)
  void* external_acc = nullptr;
  std::vector<Section> sections;
  std::vector<int> agg_section;  // agg -> section index (-1 for COUNT)

  ~pa_query() {
    dev_free(dq);
    dev_free(dsegs);
    dev_free(dplans);
    dev_free(part_hist);
    dev_free(part_off);
    dev_free(part_base);
    dev_free(recs);
    dev_free(emit);
    dev_free(wave_cnt);
    dev_free(tile_rec);
    dev_free(lim_keys);
    dev_free(lim_pos);
    dev_free(lim_sk);
    dev_free(lim_sorted);
    dev_free(lim_thresh);
    dev_free(lim_temp);
    if (host_acc) (void)hipHostFree(host_acc);
    dev_free(fetch_blocks);
    dev_free(fetch_stage);
    if (fetch_host) (void)hipHostFree(fetch_host);
    dev_free(acc);
    for (auto& b : owned) dev_free(b);
  }
};

namespace {

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

}  // namespace

extern "C" {

pa_query* pa_query_create(const pa_query_spec* spec, int32_t num_segments) {
  if (!spec || num_segments < 0) {
    fail(PA_EINVAL, "bad query spec");
    return nullptr;
  }
  if (spec->num_leaves < 0 || spec->num_leaves > PA_MAX_LEAVES || spec->num_ops < 0 || spec->num_ops > PA_MAX_OPS ||
      spec->num_group_by < 0 || spec->num_group_by > PA_MAX_GROUP_BY || spec->num_aggs < 0 ||
      spec->num_aggs > PA_MAX_AGGS) {
    fail(PA_EINVAL, "query spec counts out of range");
    return nullptr;
  }
  pa_query* q = new pa_query();
  q->spec = *spec;
  q->nseg = num_segments;
  q->segs.assign(num_segments, nullptr);
  q->leaf_params.resize(num_segments);
  q->luts.resize(num_segments);
  q->remaps.resize(num_segments);
  q->has_remap.resize(num_segments);
  return q;
}

int pa_query_bind_segment(pa_query* q, int32_t index, const pa_segment* seg, const pa_leaf_params* leaf_params,
                          const int32_t* const* group_remaps) {
  if (!q || !seg || index < 0 || index >= q->nseg) return fail(PA_EINVAL, "bad bind arguments");
  if (q->prepared) return fail(PA_EINVAL, "query already prepared");
  const pa_query_spec& s = q->spec;
  q->segs[index] = seg;
  q->leaf_params[index].assign(leaf_params, leaf_params + s.num_leaves);
  q->luts[index].assign(s.num_leaves, {});
  for (int l = 0; l < s.num_leaves; ++l) {
    const int kind = s.leaves[l].kind;
    if (kind == PA_LEAF_DICT_SET || kind == PA_LEAF_MV_DICT_SET) {
      auto it = seg->cols.find(s.leaves[l].column_id);
      if (it == seg->cols.end()) return fail(PA_EINVAL, "leaf column missing in segment");
      if (!leaf_params[l].lut) return fail(PA_EINVAL, "DICT_SET leaf without lut");
      const size_t words = ((size_t)it->second->cardinality + 31) / 32;
      q->luts[index][l].assign(leaf_params[l].lut, leaf_params[l].lut + words);
    }
  }
  q->remaps[index].assign(s.num_group_by, {});
  q->has_remap[index].assign(s.num_group_by, 0);
  for (int j = 0; j < s.num_group_by; ++j) {
    if (group_remaps && group_remaps[j]) {
      auto it = seg->cols.find(s.group_by_columns[j]);
      if (it == seg->cols.end()) return fail(PA_EINVAL, "group-by column missing in segment");
      const int32_t card = it->second->cardinality;
      q->remaps[index][j].assign(group_remaps[j], group_remaps[j] + card);
      for (int32_t v : q->remaps[index][j])
        if (v < 0 || v >= s.group_by_cardinality[j]) return fail(PA_EINVAL, "group remap id outside the key space");
      q->has_remap[index][j] = 1;
    }
  }
  return PA_OK;
}

int pa_query_prepare(pa_query* q) {
  if (!q) return fail(PA_EINVAL, "null query");
  if (q->prepared) return PA_OK;
  const pa_query_spec& s = q->spec;
  for (int i = 0; i < q->nseg; ++i)
    if (!q->segs[i]) return fail(PA_EINVAL, "segment " + std::to_string(i) + " not bound");

  // ---- CNF + slots
  std::vector<Clause> cnf;
  int rc = to_cnf(s, cnf);
  if (rc) return rc;
  auto is_mv_leaf = [&](int leaf) {
    const int k = s.leaves[leaf].kind;
    return k == PA_LEAF_MV_DICT_RANGE || k == PA_LEAF_MV_DICT_SET;
  };
  std::vector<char> clause_mv(cnf.size(), 0);  // clauses with an MV literal are evaluated per doc (lazily), last
  for (size_t c = 0; c < cnf.size(); ++c)
    for (const Literal& lit : cnf[c]) clause_mv[c] |= is_mv_leaf(lit.leaf);
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
    if (clause_mv[a] != clause_mv[b]) return clause_mv[a] < clause_mv[b];
    return csel[a] < csel[b];
  });
  const bool no_lazy = (s.flags & (PA_QF_STAGE_ALL | PA_QF_NO_LAZY)) != 0;
  size_t eager_clauses = 0;
  double density = (double)kWTileDocs;  // expected surviving docs per wave tile
  while (eager_clauses < cnf.size() && !clause_mv[order[eager_clauses]] &&
         (no_lazy || eager_clauses == 0 || density > kLazyDensity))
    density *= csel[order[eager_clauses++]];
  double post_density = density;
  for (size_t c = eager_clauses; c < cnf.size(); ++c) post_density *= csel[order[c]];
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
  std::vector<char> slot_eager(kMaxSlots, 0);
  std::vector<int> leaf_slot(s.num_leaves, -1);
  for (int l = 0; l < s.num_leaves; ++l) {
    const int sl = slot_of(q, s.leaves[l].column_id);
    if (sl < 0) return fail(PA_EUNSUPPORTED, "too many distinct columns in one query");
    leaf_slot[l] = sl;
  }
  for (int li = 0; li < q->num_eager; ++li) slot_eager[leaf_slot[q->literals[li].leaf]] = 1;
  std::vector<int> gb_slot(s.num_group_by);
  for (int j = 0; j < s.num_group_by; ++j) {
    gb_slot[j] = slot_of(q, s.group_by_columns[j]);
    if (gb_slot[j] < 0) return fail(PA_EUNSUPPORTED, "too many distinct columns in one query");
  }
  std::vector<int> agg_slot(s.num_aggs, 0);
  for (int a = 0; a < s.num_aggs; ++a) {
    const int t = s.aggs[a].type;
    if (t < PA_AGG_COUNT || t > PA_AGG_COUNT_MV) return fail(PA_EINVAL, "bad aggregation type");
    if (t == PA_AGG_COUNT) continue;
    agg_slot[a] = slot_of(q, s.aggs[a].column_id);
    if (agg_slot[a] < 0) return fail(PA_EUNSUPPORTED, "too many distinct columns in one query");
    if (t == PA_AGG_DISTINCTCOUNTHLL && (s.aggs[a].log2m < 4 || s.aggs[a].log2m > 16))
      return fail(PA_EINVAL, "log2m must be 4..16");
  }
  const int nslots = (int)q->slot_cols.size();
  const bool has_filter = !q->literals.empty();
  // Post-filter columns (group-by keys, aggregated values) are staged with the filter columns when the filter lets
  // more than kLazyPost docs per wave tile through; below that each surviving doc reads them from HBM.
  const double kLazyPost = 0.25;
  const bool stage_all = !has_filter || (s.flags & PA_QF_STAGE_ALL);
  const bool stage_post = stage_all || post_density > kLazyPost;
  std::vector<char> slot_post(kMaxSlots, 0);
  for (int j = 0; j < s.num_group_by; ++j) slot_post[gb_slot[j]] = 1;
  for (int a = 0; a < s.num_aggs; ++a)
    if (s.aggs[a].type != PA_AGG_COUNT) slot_post[agg_slot[a]] = 1;

  // ---- key space. Direct: table-wide key id = sum_j id_j * prod_{k<j} card_k (DictionaryBasedGroupKeyGenerator raw
  // key) indexes the accumulators, when every group-by column has a dictionary and the product fits kDirectMaxKeys.
  // Hashed: the components (dictionary key ids, raw value bits for no-dictionary columns) are packed side by side into
  // one 64-bit key, mapped to an accumulator slot by a global open-addressing table (the IntMap / LongMap /
  // NoDictionary*GroupKeyGenerator holders of the reference).
  q->hashed = false;
  std::vector<int> gb_bits(s.num_group_by, 0);
  std::vector<char> gb_raw(s.num_group_by, 0);
  bool direct_ok = true;
  int64_t K = 1;
  std::vector<int64_t> stride(s.num_group_by);
  for (int j = 0; j < s.num_group_by; ++j) {
    auto it = q->segs[0]->cols.find(s.group_by_columns[j]);
    if (it == q->segs[0]->cols.end()) return fail(PA_EINVAL, "group-by column missing in segment 0");
    if (it->second->kind == COL_SV_RAW) {
      gb_raw[j] = 1;
      const int vt = it->second->vtype;
      gb_bits[j] = (vt == PA_INT || vt == PA_FLOAT) ? 32 : 64;
      direct_ok = false;
      continue;
    }
    const int64_t card = s.group_by_cardinality[j];
    if (card < 1) return fail(PA_EINVAL, "group_by_cardinality < 1 for a dictionary column");
    gb_bits[j] = std::max(1, 64 - __builtin_clzll((unsigned long long)std::max<int64_t>(card - 1, 1)));
    stride[j] = K;
    if (K > kDirectMaxKeys / card) direct_ok = false;
    else K *= card;
  }
  if (!direct_ok) {
    int total_bits = 0;
    for (int j = 0; j < s.num_group_by; ++j) {
      if (total_bits + gb_bits[j] > 64) return fail(PA_EUNSUPPORTED, "packed group key wider than 64 bits");
      stride[j] = total_bits < 64 ? (int64_t)(uint64_t(1) << total_bits) : 0;
      q->key_shift[j] = total_bits;
      total_bits += gb_bits[j];
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
    uint64_t H = 1024;
    while (H < 2 * bound && H < kMaxHashSlots) H <<= 1;
    q->hashed = true;
    q->ht_slots = (int64_t)H;
    K = (int64_t)H + 1;  // + the reserved slot of the key INT64_MAX (the table's empty marker)
  }
  q->num_keys = K;

  // ---- numGroupsLimit. The reference caps each segment's group table at numGroupsLimit first-seen groups
  // (DictionaryBasedGroupKeyGenerator._globalGroupIdUpperBound, NoDictionary*GroupKeyGenerator). It can only bind
  // when a segment can hold that many distinct keys: min(product of its key cardinalities (a raw column: its docs),
  // its expanded (doc, key) pairs). Then the first-seen trimming passes run instead of the fused scan.
  q->limit_mode = false;
  uint64_t limit_pairs = 0;  // bound on distinct (segment, key) pairs
  int limit_eb = 0;
  if (s.num_group_by > 0 && s.num_groups_limit > 0) {
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
      limit_pairs = std::min<uint64_t>(UINT64_MAX / 4, limit_pairs + bound);
      max_exp = std::max(max_exp, per_doc);
    }
    while (limit_eb < 63 && (uint64_t(1) << limit_eb) < max_exp) ++limit_eb;
    if (q->limit_mode) {
      if (limit_eb > 21) return fail(PA_EUNSUPPORTED, "numGroupsLimit trimming: more than 2^21 group keys in one doc");
      if (q->nseg >= 4095) return fail(PA_EUNSUPPORTED, "numGroupsLimit trimming: more than 4094 segments in one query");
    }
  }

  // ---- per-segment descriptors
  q->hsegs.assign(q->nseg, DevSeg{});
  std::vector<char> staged(nslots, 0);
  std::vector<int> agg_src(s.num_aggs, SRC_INT);
  std::vector<char> val_fast(s.num_aggs, 1);
  std::vector<char> agg_mv(s.num_aggs, 0);  // the aggregation column is multi-value in some segment
  bool gb_mv = false;                        // some group-by column is multi-value in some segment  // emit fast path: the value is a dictionary or raw INT/LONG/DOUBLE column
  
  
  
  q->num_docs = 0;
  for (int si = 0; si < q->nseg; ++si) {
    const pa_segment* seg = q->segs[si];
    DevSeg& d = q->hsegs[si];
    std::memset(&d, 0, sizeof(d));
    d.num_docs = seg->num_docs;
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
      if (c->kind == COL_SV_DICT && (slot_eager[sl] || stage_all || (stage_post && slot_post[sl]))) {
        staged[sl] = 1;
        dc.lds_off = 0;  // staged; the region offset depends on the tile size (apply_layout below)
        d.stage[d.num_staged++] = StageDesc{dc.words, dc.nbits, 0};
      }
    }
    // filter literals
    for (size_t li = 0; li < q->literals.size(); ++li) {
      const Literal lit = q->literals[li];
      const pa_leaf_params& p = q->leaf_params[si][lit.leaf];
      DevLeaf& L = d.leaves[li];
      L.kind = s.leaves[lit.leaf].kind;
      L.slot = leaf_slot[lit.leaf];
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
      } else if (L.kind == PA_LEAF_RAW_RANGE) {
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
      } else {
        L.ilo = p.ilo;
        L.ihi = p.ihi;
        L.dlo = p.dlo;
        L.dhi = p.dhi;
      }
    }
    // group-by remaps
    for (int j = 0; j < s.num_group_by; ++j) {
      const DevCol& dc = d.cols[gb_slot[j]];
      if (gb_raw[j]) {
        if (dc.kind != COL_SV_RAW || dc.vtype != q->segs[0]->cols.at(s.group_by_columns[j])->vtype)
          return fail(PA_EINVAL, "a raw group-by column must be raw with the same type in every segment");
        continue;
      }
      if (dc.kind != COL_SV_DICT && dc.kind != COL_MV_DICT)
        return fail(PA_EINVAL, "group-by column is dictionary-encoded in segment 0 but not here");
      if (dc.kind == COL_MV_DICT) {
        q->has_mv = 1;
        gb_mv = true;
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
        agg_mv[a] = 1;
      }
      if (A.type == PA_AGG_COUNT_MV) {
        if (c->kind != COL_MV_DICT) return fail(PA_EINVAL, "COUNT_MV on a single-value column");
        agg_src[a] = SRC_INT;
        continue;
      }
      const bool wide = (A.flags & PA_AGGF_WIDE_SUM) && A.type == PA_AGG_SUM;  // layout agreed across ranks
      const int src = (c->vtype == PA_FLOAT || c->vtype == PA_DOUBLE) ? SRC_DOUBLE
                                                                     : ((c->fits_int32 && !wide) ? SRC_INT : SRC_LONG);
      if (!(c->kind == COL_SV_DICT ||
            (c->kind == COL_SV_RAW && (c->vtype == PA_INT || c->vtype == PA_LONG || c->vtype == PA_DOUBLE))))
        val_fast[a] = 0;
      if (A.type != PA_AGG_DISTINCTCOUNTHLL) {
        if (c->vtype == PA_STRING || c->vtype == PA_BYTES) return fail(PA_EINVAL, "numeric aggregation on a non-numeric column");
        if (c->kind == COL_SV_DICT && !c->dict.p) return fail(PA_EINVAL, "dictionary values missing");
      }
      if (si == 0) {
        agg_src[a] = src;
      } else if (agg_src[a] != src) {
        if (agg_src[a] == SRC_DOUBLE || src == SRC_DOUBLE)
          return fail(PA_EINVAL, "aggregation column type differs across segments");
        agg_src[a] = SRC_LONG;  // widen: some segment has values outside int32
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
  

  // ---- accumulators (one device block, sections 256-byte aligned)
  q->sections.clear();
  q->agg_section.assign(s.num_aggs, -1);
  std::vector<std::pair<int32_t, int64_t>> sec;  // kind, elements
  sec.push_back({PA_ACC_COUNT_U64, K});
  for (int a = 0; a < s.num_aggs; ++a) {
    const pa_agg_spec& A = s.aggs[a];
    switch (A.type) {
      case PA_AGG_COUNT: continue;
      case PA_AGG_SUM:
        if (agg_src[a] == SRC_LONG) sec.push_back({PA_ACC_SUM_I64X2, 2 * K});
        else sec.push_back({agg_src[a] == SRC_INT ? PA_ACC_SUM_I64 : PA_ACC_SUM_F64, K});
        break;
      case PA_AGG_MIN: sec.push_back({PA_ACC_MIN_I64, K}); break;
      case PA_AGG_MAX: sec.push_back({PA_ACC_MAX_I64, K}); break;
      case PA_AGG_DISTINCTCOUNTHLL: sec.push_back({PA_ACC_HLL_U32, K << A.log2m}); break;
      case PA_AGG_COUNT_MV: sec.push_back({PA_ACC_SUM_I64, K}); break;
    }
    q->agg_section[a] = (int)sec.size() - 1;
  }
  q->keys_section = -1;
  if (q->hashed) {
    sec.push_back({PA_ACC_KEYS_I64, K});  // slot -> packed key (INT64_MAX = empty)
    q->keys_section = (int)sec.size() - 1;
  }
  sec.push_back({PA_ACC_DOCS_U64, 3});  // [0] numDocsScanned, [1] group-table overflows, [2] limit reached (last)
  size_t total = 0;
  std::vector<size_t> offs;
  for (auto& x : sec) {
    offs.push_back(total);
    const size_t es = x.first == PA_ACC_HLL_U32 ? 4 : 8;
    total += ((size_t)x.second * es + 255) & ~(size_t)255;
  }
  rc = dev_alloc(q->acc, total);
  if (rc) return rc;
  for (size_t i = 0; i < sec.size(); ++i)
    q->sections.push_back({sec[i].first, (char*)q->acc.p + offs[i], sec[i].second});

  // ---- strategy + LDS layout
  size_t lds_acc = ((size_t)K * 4 + 15) & ~(size_t)15;  // u32 counts
  std::vector<size_t> agg_lds(s.num_aggs, 0);
  for (int a = 0; a < s.num_aggs; ++a) {
    const pa_agg_spec& A = s.aggs[a];
    if (A.type == PA_AGG_COUNT) continue;
    agg_lds[a] = lds_acc;
    const size_t bytes = A.type == PA_AGG_DISTINCTCOUNTHLL ? ((size_t)K << A.log2m) * 4
                         : (size_t)K * 8 * ((A.type == PA_AGG_SUM && agg_src[a] == SRC_LONG) ? 2 : 1);
    lds_acc += (bytes + 15) & ~(size_t)15;
  }
  // ---- tile geometry: wave tile of 1024 or 2048 docs, D DMA instructions per tile, a ring of R tile images per
  // wave (R-1 tiles in flight). Measured on MI355X (tools/sweep.py): the decode, not the DMA, is what needs
  // hiding, so the plan maximises resident waves per CU (workgroups per CU, checked against the occupancy the
  // compiled kernel really has), then prefers 2048-doc tiles, then bytes in flight (capped at 128 KiB per CU).
  const size_t kLdsBudget = 160 * 1024;
  struct Plan {
    int steps = 0, dma = 0, ring = 0, wg_per_cu = 0, img_dw = 0;
    size_t lds = 0;
    double score = -1;
  };
  const int force_ring = (s.flags >> PA_QF_RING_SHIFT) & 15;
  const int force_wg = (s.flags >> PA_QF_WG_SHIFT) & 7;
  // Lane-major kernel: every eager literal is a dictionary leaf on a staged column and the per-segment plan table
  // has room for the staged columns and eager literals (otherwise the step-major kernel runs the query).
  bool lm = !(s.flags & (PA_QF_NO_LANE_MAJOR | PA_QF_STEPS16)) && q->num_eager <= kLmEager;
  for (int li = 0; li < q->num_eager && lm; ++li) {
    const int k = s.leaves[q->literals[li].leaf].kind;
    if (k != PA_LEAF_DICT_RANGE && k != PA_LEAF_DICT_SET) lm = false;
  }
  for (int si = 0; si < q->nseg && lm; ++si)
    if (q->hsegs[si].num_staged > kLmStaged) lm = false;
  size_t part_hist_bytes = 0;  // partitioned aggregation: the per-partition LDS counters of the scan passes
  auto plan_for = [&](int strat, bool use_lm, bool only16 = false) {
    const bool lds_strategy = strat == STRAT_LDS;
    Plan best;
    for (int steps : {32, 16}) {
      if (use_lm && steps != 32) continue;
      if (only16 && steps != 16) continue;
      if ((s.flags & PA_QF_STEPS16) && steps != 16) continue;
      if ((s.flags & PA_QF_STEPS32) && steps != 32) continue;
      int img_dw = kGuardWords, dma = 0;
      for (int si = 0; si < q->nseg; ++si) {
        int dw = kGuardWords, n = 0;
        for (int k = 0; k < q->hsegs[si].num_staged; ++k) {
          const int nb = q->hsegs[si].stage[k].nbits;
          dw += 2 * steps * nb + kGuardWords;
          n += ((steps / 2) * nb + 63) / 64;
        }
        img_dw = std::max(img_dw, dw);
        dma = std::max(dma, n);
      }
      const size_t img_bytes = (size_t)img_dw * 4;
      const size_t acc_b = lds_strategy ? lds_acc : (strat == STRAT_PEMIT ? part_hist_bytes : 0);
      for (int wg : {4, 3, 2, 1}) {
        if (force_wg && wg != force_wg) continue;
        const size_t per_wg = kLdsBudget / wg;
        if (per_wg <= acc_b) continue;
        int ring = (int)((per_wg - acc_b) / (kWavesPerWG * img_bytes));
        ring = std::min(ring, 8);
        if (force_ring) {
          if (force_ring > ring) continue;
          ring = force_ring;
        }
        if (ring < 2) continue;
        const size_t lds = acc_b + (size_t)kWavesPerWG * ring * img_bytes;
        int resident = 0;
        if (set_scan_lds_limit(strat, steps, use_lm, (int)kLdsBudget) != hipSuccess ||
            scan_occupancy(strat, steps, use_lm, (int)lds, &resident) != hipSuccess)
          resident = wg;  // no device to ask (planning only): trust the LDS arithmetic
        if (resident < wg) continue;
        const double inflight = (double)wg * kWavesPerWG * (ring - 1) * img_bytes;
        const double score = 1e7 * wg + (steps == 32 ? 1e6 : 0) + std::min(inflight, 128.0 * 1024);
        if (score > best.score) best = Plan{steps, dma, ring, wg, img_dw, lds, score};
      }
    }
    return best;
  };
  // LDS-privatised accumulators when many docs are expected to reach them (and the key space fits); otherwise the
  // LDS goes to tile rings (more resident waves) and the rare survivors update global accumulators directly.
  const bool dense = !has_filter || post_density >= 1.0;
  // Tile layout: lane-major when it applies, except for dense queries on global accumulators, whose per-doc atomics
  // want the most resident waves (measured, tools/bench_configs.py highcard): there the step-major plan wins when it
  // fits more workgroups per CU.
  auto plan_pick = [&](int strat) {
    if (strat == STRAT_PEMIT) {  // the emit pass runs 1024-doc step-major tiles only (register budget of its batches)
      lm = false;
      return plan_for(strat, false, true);
    }
    if (!lm) return plan_for(strat, false);
    Plan a = plan_for(strat, true);
    if ((strat == STRAT_GLOBAL || strat == STRAT_PEMIT) && dense) {
      Plan b = plan_for(strat, false);
      if (b.score >= 0 && b.wg_per_cu > a.wg_per_cu) {
        lm = false;
        return b;
      }
    }
    return a;
  };
  Plan plan;
  q->strategy = STRAT_GLOBAL;
  if (!(s.flags & PA_QF_FORCE_GLOBAL) && !q->limit_mode && !q->hashed && lds_acc <= 64 * 1024 &&
      (dense || (s.flags & PA_QF_FORCE_LDS))) {
    plan = plan_pick(STRAT_LDS);
    if (plan.score >= 0) q->strategy = STRAT_LDS;
  }
  // Partitioned aggregation for dense queries whose key space does not fit LDS (BASELINE configs[2]): two scan passes
  // (count per (workgroup, partition); write one record per matching doc into its partition) + one LDS aggregation
  // per partition, instead of ~(1 + aggregations) device-scope atomics per matching doc on random keys.
  q->partitioned = false;
  // A DISTINCTCOUNTHLL(MV) joins as one record per value (u8 registers per key in pass C); other multi-value columns
  // keep the per-doc atomic paths.
  q->hll_agg = -1;
  q->hll_key_shift = 0;
  if (q->strategy == STRAT_GLOBAL && dense && !gb_mv && !q->hashed && !q->limit_mode &&
      !(s.flags & (PA_QF_NO_PARTITION | PA_QF_FORCE_GLOBAL)) &&
      K < (int64_t(1) << 32) && q->num_docs < (uint64_t(1) << 30)) {
    bool ok = true;
    size_t per_key = 4;  // u32 count
    int words = 1;       // key
    std::vector<int> pay(s.num_aggs, 0);
    for (int a = 0; a < s.num_aggs && ok; ++a) {
      const int t = s.aggs[a].type;
      if (t == PA_AGG_COUNT) continue;
      if (t == PA_AGG_COUNT_MV) { ok = false; break; }
      if (t == PA_AGG_DISTINCTCOUNTHLL) {
        // one per query; word 0 = key << (log2m + 6) | register << 6 | rank << 1 | first must fit 32 bits
        const int lg = s.aggs[a].log2m;
        if (q->hll_agg >= 0 || lg + 6 >= 32 || K > (int64_t(1) << (32 - (lg + 6)))) { ok = false; break; }
        q->hll_agg = a;
        q->hll_key_shift = lg + 6;
        per_key += (size_t)1 << lg;  // u8 registers
        continue;
      }
      if (agg_mv[a]) { ok = false; break; }
      per_key += (t == PA_AGG_SUM && agg_src[a] == SRC_LONG) ? 16 : 8;
      // one payload per distinct (column, value source): SUM/MIN/MAX of one column share it
      int shared = -1;
      for (int b = 0; b < a; ++b)
        if (s.aggs[b].type != PA_AGG_COUNT && s.aggs[b].type != PA_AGG_DISTINCTCOUNTHLL && agg_slot[b] == agg_slot[a] &&
            agg_src[b] == agg_src[a])
          shared = pay[b];
      if (shared >= 0) {
        pay[a] = shared;
      } else {
        pay[a] = words;
        words += agg_src[a] == SRC_INT ? 1 : 2;
      }
    }
    words = std::max(words, 2);  // COUNT-only records carry an unused value word: records are >= 8 bytes
    int64_t kr = 1;
    const size_t part_lds = kPartLdsChoices[(s.flags >> PA_QF_PART_SHIFT) & 3];
    // largest partitions that fit pass C's LDS, but at least kMinParts of them (pass C runs one workgroup each) unless
    // that would take them below 256 keys
    while (ok && (size_t)(kr * 2) * per_key <= part_lds && ((K + 2 * kr - 1) / (2 * kr) >= kMinParts || kr < 256))
      kr *= 2;
    const int64_t P = ok ? (K + kr - 1) / kr : 0;
    // part_bin_kernel: per-partition LDS bins of kPartGroup..64 records within kPartBinLdsBytes; when even one-group
    // bins of all P partitions do not fit, groups of bin_parts partitions are binned one read of the records each
    int bin_slots = 0, bin_parts = 0;
    if (ok && P > 0) {
      const size_t per_slot = (size_t)words * 4;
      bin_slots = kPartGroup;
      while ((size_t)P * (2 * bin_slots * per_slot + 8) <= kPartBinLdsBytes && bin_slots < 64) bin_slots *= 2;
      bin_parts = (int)std::min<int64_t>(P, (int64_t)(kPartBinLdsBytes / (bin_slots * per_slot + 8)));
      if (bin_parts < 1) ok = false;
    }
    if (ok && kr >= 256 && P >= 2 && P <= kMaxParts) {
      part_hist_bytes = ((size_t)P * 4 + 4 * kWavesPerWG + 15) & ~(size_t)15;  // counters + wave record cursors
      Plan pp = plan_pick(STRAT_PEMIT);
      if (pp.score >= 0) {
        plan = pp;
        q->partitioned = true;
        q->part_P = (int)P;
        q->part_shift = __builtin_ctzll((uint64_t)kr);
        q->rec_words = words;
        q->pay_off = pay;
        // emit fast path: one payload (or none) from a dictionary / raw INT, LONG, DOUBLE column
        q->emit_val_agg = -1;
        q->emit_fast = words <= 3 && q->hll_agg < 0;
        for (int a = 0; a < s.num_aggs; ++a) {
          if (s.aggs[a].type == PA_AGG_COUNT || s.aggs[a].type == PA_AGG_DISTINCTCOUNTHLL) continue;
          if (q->emit_val_agg < 0) q->emit_val_agg = a;
          if (pay[a] != 1 || !val_fast[a]) q->emit_fast = false;
        }
        q->bin_slots = bin_slots;
        // records per thread per fill round: about a quarter of a bin per partition on uniform keys
        q->bin_parts = bin_parts;
        q->bin_iter = (int)std::max<int64_t>(1, std::min<int64_t>(4, (int64_t)bin_parts * bin_slots / (4 * kPartBinThreads)));
        q->bin_lds = (int)(8 * (size_t)bin_parts + (size_t)bin_parts * bin_slots * words * 4);
        // pass C LDS layout: u32 count[kr], then every aggregation's accumulators for kr keys (8-byte aligned)
        size_t off = ((size_t)kr * 4 + 15) & ~(size_t)15;
        q->part_agg_lds.assign(s.num_aggs, 0);
        for (int a = 0; a < s.num_aggs; ++a) {
          const int t = s.aggs[a].type;
          if (t == PA_AGG_COUNT) continue;
          q->part_agg_lds[a] = (int)off;
          if (t == PA_AGG_DISTINCTCOUNTHLL) off += (((size_t)kr << s.aggs[a].log2m) + 15) & ~(size_t)15;
          else off += (size_t)kr * ((t == PA_AGG_SUM && agg_src[a] == SRC_LONG) ? 16 : 8);
        }
        q->part_lds_c = (int)off;
      }
    }
  }
  if (!q->partitioned) {
    q->hll_agg = -1;
    q->hll_key_shift = 0;
  }
  if (q->strategy == STRAT_GLOBAL && !q->partitioned) plan = plan_pick(STRAT_GLOBAL);
  if (plan.score < 0) return fail(PA_EUNSUPPORTED, "staged columns too wide for the LDS tile ring");
  q->lds_bytes = (int)plan.lds;
  q->steps = plan.steps;
  q->dma_slots = plan.dma;

  // ---- apply the layout: tiles per segment, LDS regions, staged bytes
  int64_t first = 0;
  q->staged_bytes = 0;
  void* dummy = nullptr;  // 256 readable bytes: source of the DMA padding instructions
  {
    std::vector<char> z(256, 0);
    rc = upload_owned(q, z.data(), z.size(), &dummy);
    if (rc) return rc;
  }
  for (int si = 0; si < q->nseg; ++si) {
    DevSeg& d = q->hsegs[si];
    const int64_t tile_docs = (int64_t)plan.steps * kWave;
    d.num_wtiles = (int32_t)((d.num_docs + tile_docs - 1) / tile_docs);
    d.first_wtile = first;
    first += d.num_wtiles;
    d.dummy_src = (const uint32_t*)dummy;
    int off = kGuardWords;
    for (int k = 0; k < d.num_staged; ++k) {
      d.stage[k].lds_off = off;
      for (int sl = 0; sl < nslots; ++sl)
        if (d.cols[sl].lds_off >= 0 && d.cols[sl].words == d.stage[k].words) d.cols[sl].lds_off = off;
      q->staged_bytes += (uint64_t)d.num_wtiles * 2 * plan.steps * d.stage[k].nbits * 4;
      off += 2 * plan.steps * d.stage[k].nbits + kGuardWords;
    }
    d.image_dwords = off;
    for (size_t li = 0; li < q->literals.size(); ++li) d.leaves[li].lds_off = d.cols[d.leaves[li].slot].lds_off;
  }
  const int image_max = plan.img_dw;

  DevQuery& h = q->hq;
  std::memset(&h, 0, sizeof(h));
  h.num_segments = q->nseg;
  h.num_slots = nslots;
  h.num_leaves = (int32_t)q->literals.size();
  h.num_gb = s.num_group_by;
  h.num_aggs = s.num_aggs;
  h.strategy = q->strategy;
  h.image_dwords_max = image_max;
  h.num_staged = 0;
  for (int sl = 0; sl < nslots; ++sl)
    if (staged[sl]) h.staged_slots[h.num_staged++] = sl;
  for (int j = 0; j < s.num_group_by; ++j) {
    h.gb_slot[j] = gb_slot[j];
    h.gb_stride[j] = stride[j];
  }
  h.num_keys = K;
  h.total_wtiles = first;
  h.ring = plan.ring;
  h.num_eager = q->num_eager;
  h.dma_per_tile = plan.dma;
  h.steps = plan.steps;
  h.debug_stream_only = (s.flags & PA_QF_DEBUG_STREAM_ONLY) ? 1 : 0;
  h.lane_major = lm ? 1 : 0;
  q->lane_major = lm ? 1 : 0;
  q->plan_ring = plan.ring;
  q->plan_wg = plan.wg_per_cu;
  q->num_tiles = (uint64_t)first;
  h.count = (unsigned long long*)q->sections[0].ptr;
  h.matched_docs = (unsigned long long*)q->sections.back().ptr;
  h.hashed = q->hashed ? 1 : 0;
  if (q->hashed) {
    h.ht_mask = q->ht_slots - 1;
    h.ht_keys = (long long*)q->sections[q->keys_section].ptr;
  }
  h.has_mv = q->has_mv;
  h.xcd_major = dense ? 1 : 0;
  h.lds_count_off = 0;
  h.lds_acc_bytes = q->strategy == STRAT_LDS ? (uint32_t)lds_acc : (q->partitioned ? (uint32_t)part_hist_bytes : 0);
  for (int a = 0; a < s.num_aggs; ++a) {
    DevAgg& A = h.aggs[a];
    A.type = s.aggs[a].type;
    A.slot = agg_slot[a];
    A.log2m = s.aggs[a].log2m;
    A.src = agg_src[a];
    A.lds_off = q->partitioned ? q->part_agg_lds[a] : (int32_t)agg_lds[a];
    A.pay_off = q->partitioned ? q->pay_off[a] : 0;
    if (q->agg_section[a] >= 0) {
      void* p = q->sections[q->agg_section[a]].ptr;
      A.acc_i64 = (int64_t*)p;
      A.acc_f64 = (double*)p;
      A.acc_hll = (uint32_t*)p;
    }
  }

  // ---- grid: persistent waves, enough workgroups to cover the CUs several times over
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
  }
  int wg_per_cu = plan.wg_per_cu;
  if (wg_per_cu < 1) wg_per_cu = 1;
  const int64_t max_wg = (int64_t)cus * wg_per_cu;
  const int64_t want = (first + kWavesPerWG - 1) / kWavesPerWG;
  q->grid = (int)std::max<int64_t>(1, std::min(max_wg, want));
  if (q->partitioned) {
    // records: at most one per doc (every bound doc may match); hist: [grid][P]; base: [P + 1]
    dev_free(q->part_hist);
    dev_free(q->part_off);
    dev_free(q->part_base);
    dev_free(q->recs);
    dev_free(q->emit);
    dev_free(q->wave_cnt);
    // emit buffer: every wave's range holds all docs of its tiles; partitions: every doc plus each (workgroup,
    // partition) range's padding
    size_t emit_recs = (size_t)q->num_tiles * (size_t)q->steps * kWave;
    size_t doc_recs = (size_t)q->num_docs;
    dev_free(q->tile_rec);
    h.tile_rec_base = nullptr;
    if (q->hll_agg >= 0) {
      // one record per value of the HLL column: every wave tile's first record from a scan of per-tile counts
      rc = dev_alloc(q->tile_rec, ((size_t)q->num_tiles + 1) * 4);
      if (rc) return rc;
      for (int si = 0; si < q->nseg; ++si) {
        const DevSeg& hs = q->hsegs[si];
        const DevCol& dc = hs.cols[agg_slot[q->hll_agg]];
        PA_HIP(launch_tile_records(dc.kind == COL_MV_DICT ? dc.mv_off : nullptr, hs.num_docs, q->steps * kWave,
                                   hs.num_wtiles, (uint32_t*)q->tile_rec.p + hs.first_wtile, nullptr));
      }
      PA_HIP(launch_exclusive_scan_u32((uint32_t*)q->tile_rec.p, (int64_t)q->num_tiles, nullptr));
      uint32_t total = 0;
      PA_HIP(hipMemcpy(&total, (uint32_t*)q->tile_rec.p + q->num_tiles, 4, hipMemcpyDeviceToHost));
      if (total >= (1u << 31)) return fail(PA_EUNSUPPORTED, "more than 2^31 HLL values in one partitioned query");
      emit_recs = total;
      doc_recs = total;
      h.tile_rec_base = (const uint32_t*)q->tile_rec.p;
    }
    const size_t part_recs = doc_recs + (size_t)q->grid * q->part_P * (kPartGroup - 1);
    rc = dev_alloc(q->part_hist, (size_t)q->grid * q->part_P * 4);
    if (!rc) rc = dev_alloc(q->part_off, (size_t)q->grid * q->part_P * 4);
    if (!rc) rc = dev_alloc(q->part_base, (size_t)(q->part_P + 1) * 4);
    if (!rc) rc = dev_alloc(q->recs, std::max<size_t>(16, part_recs * q->rec_words * 4));
    if (!rc) rc = dev_alloc(q->emit, std::max<size_t>(16, emit_recs * q->rec_words * 4));
    if (!rc) rc = dev_alloc(q->wave_cnt, (size_t)q->grid * kWavesPerWG * 4);
    if (rc) return rc;
    h.part_shift = q->part_shift;
    h.num_parts = q->part_P;
    h.rec_words = q->rec_words;
    h.part_lds_bytes = (uint32_t)q->part_lds_c;
    h.part_hist = (uint32_t*)q->part_hist.p;
    h.part_off = (uint32_t*)q->part_off.p;
    h.part_base = (uint32_t*)q->part_base.p;
    h.recs = (uint32_t*)q->recs.p;
    h.emit = (uint32_t*)q->emit.p;
    h.wave_cnt = (uint32_t*)q->wave_cnt.p;
    h.bin_slots = q->bin_slots;
    h.bin_iter = q->bin_iter;
    h.bin_parts = q->bin_parts;
    h.emit_fast = q->emit_fast ? 1 : 0;
    h.emit_val_agg = q->emit_val_agg;
    h.hll_agg = q->hll_agg;
    h.key_shift = q->hll_key_shift;
  }

  if (q->limit_mode) {
    // first-seen table: twice the (segment, key) pairs that can exist, a power of two
    uint64_t H = 1024;
    while (H < 2 * limit_pairs && H <= (uint64_t(1) << 30)) H <<= 1;
    if (H > (uint64_t(1) << 30))
      return fail(PA_EUNSUPPORTED, "numGroupsLimit trimming: more than 2^29 distinct (segment, group) pairs possible");
    const size_t hb = (size_t)H * 8;
    rc = dev_alloc(q->lim_keys, hb);
    if (!rc) rc = dev_alloc(q->lim_pos, hb);
    if (!rc) rc = dev_alloc(q->lim_sk, hb);
    if (!rc) rc = dev_alloc(q->lim_sorted, hb);
    if (!rc) rc = dev_alloc(q->lim_thresh, (size_t)std::max(1, q->nseg) * 8);
    if (rc) return rc;
    q->lim_temp_bytes = 0;
    PA_HIP(sort_u64(nullptr, &q->lim_temp_bytes, nullptr, nullptr, (int64_t)H, nullptr));
    rc = dev_alloc(q->lim_temp, std::max<size_t>(q->lim_temp_bytes, 16));
    if (rc) return rc;
    LimitDesc& F = q->limit;
    F.fkeys = (long long*)q->lim_keys.p;
    F.fpos = (unsigned long long*)q->lim_pos.p;
    F.fmask = (int64_t)H - 1;
    F.sk = (unsigned long long*)q->lim_sk.p;
    F.sorted = (unsigned long long*)q->lim_sorted.p;
    F.thresh = (unsigned long long*)q->lim_thresh.p;
    F.reached = h.matched_docs + 2;
    F.limit = s.num_groups_limit;
    F.eb = limit_eb;
    q->limit_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 16, first));
  }

  // ---- upload descriptors
  rc = dev_alloc(q->dq, sizeof(DevQuery));
  if (rc) return rc;
  rc = dev_alloc(q->dsegs, sizeof(DevSeg) * std::max(1, q->nseg));
  if (rc) return rc;
  PA_HIP(hipMemcpy(q->dq.p, &h, sizeof(DevQuery), hipMemcpyHostToDevice));
  if (q->nseg) PA_HIP(hipMemcpy(q->dsegs.p, q->hsegs.data(), sizeof(DevSeg) * q->nseg, hipMemcpyHostToDevice));
  q->hplans.assign(std::max(1, q->nseg), LmSegPlan{});
  if (lm) {
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
    PA_HIP(set_scan_lds_limit(STRAT_PEMIT, q->steps, q->lane_major, q->lds_bytes));
    PA_HIP(set_part_bin_lds_limit(q->bin_lds));
    PA_HIP(set_part_agg_lds_limit(q->part_lds_c));
  } else {
    PA_HIP(set_scan_lds_limit(q->strategy, q->steps, q->lane_major, q->lds_bytes));
  }
  PA_HIP(hipDeviceSynchronize());
  q->prepared = true;
  return PA_OK;
}

int64_t pa_query_num_keys(const pa_query* q) { return q ? q->num_keys : -1; }

int pa_query_reset(pa_query* q, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  hipStream_t st = (hipStream_t)stream;
  // one memset of the whole accumulator block, then the MIN/MAX sections to their identities
  PA_HIP(hipMemsetAsync(q->external_acc ? q->external_acc : q->acc.p, 0, q->acc.n, st));
  for (const Section& sc : q->sections) {
    if (sc.kind == PA_ACC_MIN_I64 || sc.kind == PA_ACC_KEYS_I64) PA_HIP(launch_fill_i64((int64_t*)sc.ptr, sc.n, INT64_MAX, st));
    else if (sc.kind == PA_ACC_MAX_I64) PA_HIP(launch_fill_i64((int64_t*)sc.ptr, sc.n, INT64_MIN, st));
  }
  return PA_OK;
}

int pa_query_scan(pa_query* q, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (q->num_tiles == 0) return PA_OK;
  if (q->limit_mode) {  // first-seen positions, sort, thresholds, admitted aggregation
    hipStream_t st = (hipStream_t)stream;
    const DevQuery* dq = (const DevQuery*)q->dq.p;
    const DevSeg* ds = (const DevSeg*)q->dsegs.p;
    const LimitDesc& F = q->limit;
    const int64_t H = F.fmask + 1;
    PA_HIP(launch_fill_i64((int64_t*)F.fkeys, H, INT64_MAX, st));
    PA_HIP(launch_fill_i64((int64_t*)F.fpos, H, -1, st));
    PA_HIP(launch_fill_i64((int64_t*)F.thresh, std::max(1, q->nseg), -1, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 0, st));
    size_t tb = q->lim_temp_bytes;
    PA_HIP(sort_u64(q->lim_temp.p, &tb, F.sk, F.sorted, H, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 1, st));
    return PA_OK;
  }
  if (q->partitioned) {  // emit scan, per-partition offsets, binning into partitions, per-partition aggregation
    hipStream_t st = (hipStream_t)stream;
    const DevQuery* dq = (const DevQuery*)q->dq.p;
    PA_HIP(launch_scan(STRAT_PEMIT, q->steps, q->lane_major, q->grid, q->lds_bytes, dq, (const DevSeg*)q->dsegs.p,
                       (const LmSegPlan*)q->dplans.p, st));
    PA_HIP(launch_part_offsets((const uint32_t*)q->part_hist.p, (uint32_t*)q->part_off.p, q->grid, q->part_P,
                               (uint32_t*)q->part_base.p, st));
    PA_HIP(launch_part_bin(dq, q->grid, q->bin_lds, st));
    PA_HIP(launch_part_agg(dq, q->part_P, q->part_lds_c, st));
    return PA_OK;
  }
  PA_HIP(launch_scan(q->strategy, q->steps, q->lane_major, q->grid, q->lds_bytes, (const DevQuery*)q->dq.p,
                     (const DevSeg*)q->dsegs.p, (const LmSegPlan*)q->dplans.p, (hipStream_t)stream));
  return PA_OK;
}

int pa_query_execute(pa_query* q, void* stream) {
  const int rc = pa_query_reset(q, stream);
  return rc ? rc : pa_query_scan(q, stream);
}

uint64_t pa_query_accumulator_bytes(const pa_query* q) { return q ? (uint64_t)q->acc.n : 0; }

int pa_query_set_accumulator_buffer(pa_query* q, void* device_buffer, uint64_t bytes) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (!device_buffer || bytes < q->acc.n) return fail(PA_EINVAL, "accumulator buffer too small");
  if (((uintptr_t)device_buffer & 255) != 0) return fail(PA_EINVAL, "accumulator buffer must be 256-byte aligned");
  char* old = (char*)(q->external_acc ? q->external_acc : q->acc.p);
  char* nb = (char*)device_buffer;
  for (Section& s : q->sections) s.ptr = nb + ((char*)s.ptr - old);
  DevQuery& h = q->hq;
  h.count = (unsigned long long*)(nb + ((char*)h.count - old));
  h.matched_docs = (unsigned long long*)(nb + ((char*)h.matched_docs - old));
  if (q->limit_mode) q->limit.reached = h.matched_docs + 2;
  if (q->hashed) h.ht_keys = (long long*)(nb + ((char*)h.ht_keys - old));
  for (int a = 0; a < h.num_aggs; ++a) {
    if (q->agg_section[a] < 0) continue;
    void* p = q->sections[q->agg_section[a]].ptr;
    h.aggs[a].acc_i64 = (int64_t*)p;
    h.aggs[a].acc_f64 = (double*)p;
    h.aggs[a].acc_hll = (uint32_t*)p;
  }
  PA_HIP(hipMemcpy(q->dq.p, &h, sizeof(DevQuery), hipMemcpyHostToDevice));
  if (!q->external_acc) {
    const size_t n = q->acc.n;
    dev_free(q->acc);
    q->acc.n = n;
  }
  q->external_acc = device_buffer;
  return PA_OK;
}

int32_t pa_query_num_sections(const pa_query* q) { return q ? (int32_t)q->sections.size() : -1; }

void* pa_query_section(const pa_query* q, int32_t section, int32_t* kind, int64_t* num_elements) {
  if (!q || section < 0 || section >= (int32_t)q->sections.size()) {
    fail(PA_EINVAL, "bad section");
    return nullptr;
  }
  if (kind) *kind = q->sections[section].kind;
  if (num_elements) *num_elements = q->sections[section].n;
  return q->sections[section].ptr;
}

int64_t pa_query_fetch(pa_query* q, void* stream, int64_t capacity, int64_t* out_keys, int64_t* out_counts,
                       void* const* out_aggs) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  hipStream_t st = (hipStream_t)stream;
  const pa_query_spec& s = q->spec;
  const int64_t K = q->num_keys;
  const bool grouped = s.num_group_by != 0;
  char* dbase = (char*)(q->external_acc ? q->external_acc : q->acc.p);

  // Decodes `nrows` host rows into the caller's arrays: row r has key key_of(r), count hc[r] and the aggregation
  // section rows at sec(section)[r * per]. Rows with a zero count are skipped when `skip_empty`.
  // `order` (optional) lists the rows to emit, in output order (hashed key spaces: sorted by packed key).
  // `hll_u8`: HLL register rows arrive already narrowed to one byte per register (GPU compaction path).
  auto decode = [&](int64_t nrows, const uint64_t* hc, const std::function<const char*(int)>& sec,
                    const std::function<int64_t(int64_t)>& key_of, bool skip_empty,
                    const std::vector<int64_t>* order, bool hll_u8) -> int64_t {
    const char* asec[PA_MAX_AGGS];  // section base per aggregation, resolved once (not per row)
    for (int a = 0; a < s.num_aggs; ++a) asec[a] = q->agg_section[a] >= 0 ? sec(q->agg_section[a]) : nullptr;
    int64_t n = 0;
    const int64_t total = order ? (int64_t)order->size() : nrows;
    for (int64_t oi = 0; oi < total; ++oi) {
      const int64_t r = order ? (*order)[oi] : oi;
      if (skip_empty && hc[r] == 0) continue;
      if (n < capacity) {
        if (out_keys) out_keys[n] = key_of(r);
        if (out_counts) out_counts[n] = (int64_t)hc[r];
        for (int a = 0; a < s.num_aggs; ++a) {
          if (!out_aggs || !out_aggs[a]) continue;
          const pa_agg_spec& A = s.aggs[a];
          double* outd = (double*)out_aggs[a];
          if (A.type == PA_AGG_COUNT) {
            outd[n] = (double)hc[r];
            continue;
          }
          const char* sp = asec[a];
          const int src = q->hq.aggs[a].src;
          if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
            const int64_t per = int64_t(1) << A.log2m;
            uint8_t* o = (uint8_t*)out_aggs[a] + n * per;
            if (hll_u8) {
              std::memcpy(o, (const uint8_t*)sp + r * per, (size_t)per);
            } else {
              const uint32_t* rg = (const uint32_t*)sp + r * per;
              for (int64_t j = 0; j < per; ++j) o[j] = (uint8_t)rg[j];
            }
          } else if (A.type == PA_AGG_SUM || A.type == PA_AGG_COUNT_MV) {
            const int64_t* hv = (const int64_t*)sp;
            // SRC_LONG: exact 96-bit total, rounded once (the reference's double of the exact sum)
            if (src == SRC_LONG) outd[n] = (double)(((__int128)hv[2 * r + 1] << 32) + (__int128)(uint64_t)hv[2 * r]);
            else outd[n] = src == SRC_INT ? (double)hv[r] : ((const double*)sp)[r];
          } else {  // MIN / MAX; empty aggregation-only result -> +/-inf (Min/MaxAggregationFunction DEFAULT_VALUE)
            const int64_t e8 = ((const int64_t*)sp)[r];
            if (hc[r] == 0) outd[n] = A.type == PA_AGG_MIN ? __builtin_inf() : -__builtin_inf();
            else outd[n] = src != SRC_DOUBLE ? (double)e8 : f64_order_decode(e8);
          }
        }
      }
      ++n;
    }
    return n;
  };

  // Small accumulator blocks (the common case: a few thousand keys): ONE device-to-host copy of the whole block into
  // pinned memory and one synchronisation, then compaction + decode on the host.
  if (q->acc.n <= kFetchWholeBlockBytes) {
    if (!q->host_acc) {
      if (hipHostMalloc(&q->host_acc, std::max<size_t>(q->acc.n, 16), hipHostMallocDefault) != hipSuccess) {
        q->host_acc = nullptr;
        return fail(PA_ENOMEM, "hipHostMalloc for the accumulator copy failed");
      }
    }
    PA_HIP(hipMemcpyAsync(q->host_acc, dbase, q->acc.n, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    const char* hb = (const char*)q->host_acc;
    auto hsec = [&](int sec) { return hb + ((char*)q->sections[sec].ptr - dbase); };
    const uint64_t* docs = (const uint64_t*)hsec((int)q->sections.size() - 1);
    q->last_matched = (int64_t)docs[0];
    q->last_reached = (int64_t)docs[2];
    if (docs[1]) return fail(PA_EUNSUPPORTED, "group-key table overflow (more distinct groups than slots)");
    const uint64_t* hc = (const uint64_t*)hsec(0);
    if (q->hashed) {
      const int64_t* hk = (const int64_t*)hsec(q->keys_section);
      std::vector<int64_t> order;
      for (int64_t r = 0; r < K; ++r)
        if (hc[r]) order.push_back(r);
      std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return hk[a] < hk[b]; });
      return decode(K, hc, hsec, [&](int64_t r) { return hk[r]; }, false, &order, false);
    }
    return decode(K, hc, hsec, [](int64_t r) { return r; }, grouped, nullptr, false);
  }

  // Large key spaces: ordered compaction of the non-empty keys on the GPU (count + scan, then key ids and every
  // section's rows gathered into a staging block), one copy of the compacted rows, decode on the host.
  const int64_t nb = (K + 2047) / 2048;
  if ((int64_t)q->fetch_blocks.n < (nb + 1) * 4) {
    dev_free(q->fetch_blocks);
    int rc = dev_alloc(q->fetch_blocks, (size_t)(nb + 1) * 4);
    if (rc) return rc;
  }
  const int all = grouped ? 0 : 1;
  uint32_t total = 0;
  uint64_t md[3] = {0, 0, 0};
  PA_HIP(launch_compact((const unsigned long long*)q->sections[0].ptr, K, all, (uint32_t*)q->fetch_blocks.p, 0,
                        nullptr, 0, st));
  PA_HIP(hipMemcpyAsync(&total, (uint32_t*)q->fetch_blocks.p + nb, 4, hipMemcpyDeviceToHost, st));
  PA_HIP(hipMemcpyAsync(md, q->sections.back().ptr, 24, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  q->last_matched = (int64_t)md[0];
  q->last_reached = (int64_t)md[2];
  if (md[1]) return fail(PA_EUNSUPPORTED, "group-key table overflow (more distinct groups than slots)");
  const int64_t m = (int64_t)total;
  const int64_t rows_cap = std::min<int64_t>(m, std::max<int64_t>(capacity, 0));
  if (rows_cap == 0) return m;
  // staging: keys | count | one block per aggregation section (rows x per x es), 256-byte aligned pieces
  CompactDesc d;
  std::memset(&d, 0, sizeof(d));
  std::vector<int> secs = {0};
  for (int a = 0; a < s.num_aggs; ++a)
    if (q->agg_section[a] >= 0) secs.push_back(q->agg_section[a]);
  if (q->hashed) secs.push_back(q->keys_section);
  // hashed key spaces: every non-empty slot is needed to sort by packed key before the capacity cut
  const int64_t rows_needed = q->hashed ? m : std::min<int64_t>(m, std::max<int64_t>(capacity, 0));
  std::vector<size_t> offs;
  const int64_t rows = rows_needed;
  size_t bytes = ((size_t)rows * 8 + 255) & ~(size_t)255;
  for (int sec : secs) {
    const Section& sc = q->sections[sec];
    const int es = sc.kind == PA_ACC_HLL_U32 ? 1 : 8;  // HLL registers (< 64) narrowed to bytes by the gather
    const int64_t per = sc.n / K;
    offs.push_back(bytes);
    bytes += ((size_t)rows * per * es + 255) & ~(size_t)255;
  }
  if (q->fetch_stage.n < bytes) {
    dev_free(q->fetch_stage);
    int rc = dev_alloc(q->fetch_stage, bytes);
    if (rc) return rc;
    if (q->fetch_host) (void)hipHostFree(q->fetch_host);
    if (hipHostMalloc(&q->fetch_host, bytes, hipHostMallocDefault) != hipSuccess) {
      q->fetch_host = nullptr;
      return fail(PA_ENOMEM, "hipHostMalloc for the fetch staging failed");
    }
  }
  char* dstage = (char*)q->fetch_stage.p;
  d.nsec = (int32_t)secs.size();
  d.keys = (int64_t*)dstage;
  for (size_t i = 0; i < secs.size(); ++i) {
    const Section& sc = q->sections[secs[i]];
    d.es[i] = sc.kind == PA_ACC_HLL_U32 ? 4 : 8;
    d.oes[i] = sc.kind == PA_ACC_HLL_U32 ? 1 : d.es[i];
    d.per[i] = sc.n / K;
    d.src[i] = sc.ptr;
    d.dst[i] = dstage + offs[i];
  }
  PA_HIP(launch_compact((const unsigned long long*)q->sections[0].ptr, K, all, (uint32_t*)q->fetch_blocks.p, rows,
                        &d, 1, st));
  PA_HIP(hipMemcpyAsync(q->fetch_host, dstage, bytes, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  const char* hb = (const char*)q->fetch_host;
  const int64_t* hkeys = (const int64_t*)hb;
  std::map<int, const char*> hsec;
  for (size_t i = 0; i < secs.size(); ++i) hsec[secs[i]] = hb + offs[i];
  if (q->hashed) {  // rows are slots: emit them in packed-key order
    const int64_t* pk = (const int64_t*)hsec[q->keys_section];
    std::vector<int64_t> order(rows);
    for (int64_t r = 0; r < rows; ++r) order[r] = r;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return pk[a] < pk[b]; });
    order.resize(rows_cap);
    decode(rows, (const uint64_t*)hsec[0], [&](int sec) { return hsec[sec]; }, [&](int64_t r) { return pk[r]; },
           false, &order, true);
    return m;
  }
  decode(rows, (const uint64_t*)hsec[0], [&](int sec) { return hsec[sec]; }, [&](int64_t r) { return hkeys[r]; },
         false, nullptr, true);
  return m;
}

int pa_query_stats(const pa_query* q, uint64_t* staged_bytes, uint64_t* num_docs, uint64_t* num_tiles) {
  if (!q) return fail(PA_EINVAL, "null query");
  if (staged_bytes) *staged_bytes = q->staged_bytes;
  if (num_docs) *num_docs = q->num_docs;
  if (num_tiles) *num_tiles = q->num_tiles;
  return PA_OK;
}

int pa_query_plan(const pa_query* q, int32_t* strategy, int32_t* steps, int32_t* dma_slots, int32_t* ring,
                  int32_t* wg_per_cu, int32_t* grid, int32_t* lds_bytes) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (strategy) *strategy = q->partitioned ? STRAT_PEMIT : q->strategy;
  if (steps) *steps = q->steps;
  if (dma_slots) *dma_slots = q->dma_slots;
  if (ring) *ring = q->plan_ring;
  if (wg_per_cu) *wg_per_cu = q->plan_wg;
  if (grid) *grid = q->grid;
  if (lds_bytes) *lds_bytes = q->lds_bytes;
  return PA_OK;
}

int32_t pa_query_num_eager_literals(const pa_query* q) { return q && q->prepared ? q->num_eager : -1; }

int32_t pa_query_lane_major(const pa_query* q) { return q && q->prepared ? q->lane_major : -1; }

int64_t pa_query_matched_docs(const pa_query* q) { return q && q->prepared ? q->last_matched : -1; }

int32_t pa_query_limit_trimming(const pa_query* q) { return q && q->prepared ? (q->limit_mode ? 1 : 0) : -1; }

int64_t pa_query_num_groups_limit_reached(const pa_query* q) { return q && q->prepared ? q->last_reached : -1; }

int pa_query_key_layout(const pa_query* q, int32_t* hashed, int32_t* shifts) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (hashed) *hashed = q->hashed ? 1 : 0;
  if (shifts)
    for (int j = 0; j < q->spec.num_group_by; ++j) shifts[j] = q->hashed ? q->key_shift[j] : 0;
  return PA_OK;
}

void pa_query_destroy(pa_query* q) { delete q; }

}  // extern "C"
