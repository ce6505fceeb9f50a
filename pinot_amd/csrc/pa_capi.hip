// Host side of the C-ABI (include/pinot_amd.h): segment residency, query planning (CNF filter, column
// slots, staging, accumulator layout, strategy) and result fetch. No CPU fallback: every query runs the
// HIP kernels; errors surface as negative return codes + pa_last_error().
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <numeric>
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

// PA_DEBUG_PLAN=1: the planner's decisions on stderr (why a query takes a strategy)
bool plan_debug() {
  static const bool on = std::getenv("PA_DEBUG_PLAN") != nullptr;
  return on;
}
#define PLAN_LOG(...)                                  \
  do {                                                 \
    if (plan_debug()) {                                \
      std::fprintf(stderr, "[pa plan] " __VA_ARGS__); \
      std::fputc('\n', stderr);                       \
    }                                                  \
  } while (0)

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
  bool fits_int32 = false;  // every value (dictionary or raw, INT/LONG) fits in int32
  bool dict_sorted = false; // dictionary values strictly ascending (COLF_DICT_SORTED)
  std::vector<uint64_t> hvals;  // host copy of the dictionary values (8-byte bits): table-wide value dictionaries
  uint64_t dict_hash = 0;       // FNV-1a of hvals: identical dictionaries across segments are found without a compare
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

// Order key of an 8-byte dictionary value: the value itself (INT/LONG) or its order-preserving image (FLOAT/DOUBLE,
// Double.compare order: -0.0 < 0.0), so distinct values get distinct keys in value order.
inline int64_t value_order_key(uint64_t bits, int32_t vtype) {
  return (vtype == PA_FLOAT || vtype == PA_DOUBLE) ? f64_order_encode(__builtin_bit_cast(double, bits))
                                                    : (int64_t)bits;
}

int upload_dict(Column* c, int32_t vtype, int32_t card, const void* dict_values, const int32_t* dict_hashes) {
  c->vtype = vtype;
  c->cardinality = card;
  if (dict_values != nullptr && (vtype == PA_INT || vtype == PA_LONG || vtype == PA_FLOAT || vtype == PA_DOUBLE)) {
    int rc = dev_alloc(c->dict, (size_t)card * 8);
    if (rc) return rc;
    PA_HIP(hipMemcpy(c->dict.p, dict_values, (size_t)card * 8, hipMemcpyHostToDevice));
    c->hvals.assign((const uint64_t*)dict_values, (const uint64_t*)dict_values + card);
    uint64_t hsh = 1469598103934665603ull ^ (uint64_t)card;
    for (uint64_t v : c->hvals) hsh = (hsh ^ v) * 1099511628211ull;
    c->dict_hash = hsh;
    if (vtype == PA_INT || vtype == PA_LONG) {
      const int64_t* v = (const int64_t*)dict_values;
      c->fits_int32 = true;
      for (int32_t i = 0; i < card && c->fits_int32; ++i) c->fits_int32 = v[i] >= INT32_MIN && v[i] <= INT32_MAX;
    }
    // sorted dictionary (the reference's dictionaries always are: SegmentDictionaryCreator sorts the unique values)
    c->dict_sorted = true;
    for (int32_t i = 1; i < card && c->dict_sorted; ++i)
      c->dict_sorted = value_order_key(c->hvals[i - 1], vtype) < value_order_key(c->hvals[i], vtype);
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

void* pa_host_alloc(uint64_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, std::max<uint64_t>(bytes, 16), hipHostMallocDefault) != hipSuccess) {
    fail(PA_ENOMEM, "hipHostMalloc failed");
    return nullptr;
  }
  return p;
}

void pa_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

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
  if (value_type == PA_LONG) {  // (Pinot's column metadata min/max): int32-range LONG metrics sum in one int64 slot
    const int64_t* v = (const int64_t*)values;
    bool fits = true;
    for (int32_t i = 0; i < seg->num_docs; ++i) fits &= v[i] >= INT32_MIN && v[i] <= INT32_MAX;
    c->fits_int32 = fits;
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
constexpr int64_t kMaxParts = 4096;          // partitions of one query (both streams)
constexpr int64_t kDirectMaxKeys = int64_t(1) << 27;  // direct-indexed key space limit (beyond: hashed keys)
constexpr uint64_t kMaxHashSlots = uint64_t(1) << 28;
constexpr uint64_t kWalkMaxBitmapBytes = uint64_t(4) << 30;  // numGroupsLimit walk: admitted-key bitmaps of a query
constexpr size_t kLdsBudget = 160 * 1024;

struct Section {
  int32_t kind;
  void* ptr;
  int64_t n;
};

// Per-device pooled scratch of the partitioned queries (histograms, range offsets, partition bases, records): sized by
// the largest query prepared on the device and shared by all of them, so a query costs no allocation. Stream-ordered
// hand-off: a scan enqueues its kernels behind the previous user's (hipStreamWaitEvent when that was another stream)
// and records its own completion event; growing waits for that event before the old block is freed.
struct ScratchArena {
  std::mutex mu;
  void* p = nullptr;
  size_t n = 0;
  hipEvent_t last = nullptr;
  hipStream_t last_stream = nullptr;
  bool used = false;
};

ScratchArena* arena_for(int dev) {
  static std::mutex m;
  static std::map<int, ScratchArena*> arenas;
  std::lock_guard<std::mutex> g(m);
  ScratchArena*& a = arenas[dev];
  if (!a) a = new ScratchArena();  // lives for the process (freed with it)
  return a;
}

// Grows the arena to at least `bytes` (caller holds a->mu).
int arena_grow(ScratchArena* a, size_t bytes) {
  if (a->n >= bytes) return PA_OK;
  if (a->used) PA_HIP(hipEventSynchronize(a->last));
  if (a->p) PA_HIP(hipFree(a->p));
  a->p = nullptr;
  a->n = 0;
  hipError_t e = hipMalloc(&a->p, bytes);
  if (e != hipSuccess) {
    a->p = nullptr;
    return fail(PA_ENOMEM, "scratch arena hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
  }
  a->n = bytes;
  if (!a->last) PA_HIP(hipEventCreateWithFlags(&a->last, hipEventDisableTiming));
  return PA_OK;
}

// DISTINCTCOUNT presence bytes per key: the table-wide value count rounded up to whole 16-byte units
inline int64_t presence_stride(const pa_agg_spec& A) { return (A.num_values + 15) & ~int64_t(15); }
// element bytes of an accumulator section
inline size_t section_es(int32_t kind) { return (kind == PA_ACC_HLL_U8 || kind == PA_ACC_PRESENCE_U8) ? 1 : 8; }


}  // namespace

struct pa_query {
  pa_query_spec spec;
  int32_t nseg = 0;
  std::vector<const pa_segment*> segs;
  std::vector<std::vector<pa_leaf_params>> leaf_params;
  std::vector<std::vector<std::vector<uint32_t>>> luts;        // [seg][leaf]
  std::vector<std::vector<std::vector<int32_t>>> remaps;       // [seg][gb]
  std::vector<std::vector<char>> has_remap;
  std::vector<std::vector<std::vector<int32_t>>> vremaps;      // [seg][agg] DISTINCTCOUNT value remaps (empty = identity)
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
  int dense_packed = 0;  // STRAT_GDENSE_LM*: packed accumulation (GdLmPlan)
  // the dense kernel specialised to this query's shape (gdl_jit.hip, compiled by hiprtc): null = the generic kernel
  hipFunction_t jit_fn = nullptr;
  int jit_waves = 0, jit_grid = 0, jit_lds = 0;
  DevBuf jit_args, jit_segs;
  // the partitioned path's V emit without a count pass (pve_jit.hip + pa_pve.hip): null = count + emit passes
  // one per record stream: pve (V), pvh (H records of a DISTINCTCOUNTHLLMV next to a V stream)
  struct PveStream {
    hipFunction_t fn = nullptr;
    int waves = 0, grid = 0, lds = 0, cr = 0, parts = 0, bin_shift = 5;  // cr: records per chunk (pass C's unit)
    int64_t chunks = 0;                                                  // chunk slots per workgroup
    DevBuf args, segs, buf;
    size_t o_table = 0, o_hist = 0, o_used = 0, o_off = 0, o_base = 0, o_index = 0, o_tot = 0;
  } pve, pvh;
  int has_mv = 0;
  bool hashed = false;           // packed 64-bit keys through a global open-addressing table
  int key_words = 1;             // hashed: 2 = two-word keys ([k0, k1, state] per slot)
  int64_t ht_slots = 0;
  int key_shift[PA_MAX_GROUP_BY] = {0};
  int keys_section = -1;
  // partitioned aggregation: count pass (own descriptors: it stages only the filter and group-by columns), range
  // offsets, emit pass (hq / hsegs), pass C; scratch in the device arena at these offsets
  bool partitioned = false;
  DevQuery hq_count;
  std::vector<DevSeg> hsegs_count;
  DevBuf dq_count, dsegs_count;
  int count_lds = 0, count_ring = 0, part_lds_c = 0;
  int part_vk = -1;     // part_agg_kernel variant (vk_code, kVkGeneric)
  int emit_strat = 0;   // the emit kernel variant (pemit_strat)
  // both streams: the emit pass runs as two launches (V records, then H records), each with only its own bins in LDS
  // (more resident workgroups than one kernel holding both): the H launch's descriptor, variant and plan
  bool split_emit = false;
  DevQuery hq_h;
  DevBuf dq_h;
  int emit_h_strat = 0, emit_h_lds = 0, emit_h_ring = 0, emit_h_wg = 0;
  int count_k = 1;      // count-pass workgroups per emit workgroup
  int count_skip = -1;  // count pass: the group-by component it neither stages nor decodes (plan_partitions)
  int count_strat = STRAT_PCOUNT;  // STRAT_PCOUNT, or STRAT_PCOUNT_MV for a multi-value group-by
  size_t sc_hist = 0, sc_off = 0, sc_base = 0, sc_recs_v = 0, sc_recs_h = 0, sc_bytes = 0;
  int scratch_dev = 0;
  int64_t last_matched = -1;  // numDocsScanned read by the last fetch
  int64_t last_reached = -1;  // segments that reached numGroupsLimit, read by the last fetch
  // numGroupsLimit first-seen trimming (launch_limit_passes): on when some segment can hold numGroupsLimit groups
  bool limit_mode = false;
  LimitDesc limit{};
  // numGroupsLimit, walk form (limit_walk_kernel + admission inside the scan): admitted-key bitmaps of the segments
  // where the limit can bind (walk_words words each)
  bool limit_walk = false;
  int64_t walk_words = 0;
  DevBuf lim_admit;
  int limit_grid = 0;
  DevBuf lim_keys, lim_pos, lim_hist, lim_sel, lim_thresh;
  DevBuf stat_buf;  // pa_query_filter_counts: leaf bitmaps, scratch, counts, jobs (grown on demand)
  DevBuf merge_buf;  // pa_query_pack_rows / pa_query_merge_rows: row -> slot map and counters (grown on demand)
  DevBuf leap_buf;  // fused statistics (default; PA_QF_NO_FILTER_STATS turns them off): per segment (matched docs, leaps, gave up)
  int leap_leaf = -1;  // the eager leaf (spec order) when the scan counts the leaps
  bool leap_searched = true;  // the last scan's E-doc list has been searched (leap_search_kernel)
  bool scanned_since_fetch = false;  // last_matched predates the last scan
  int64_t leap_slices = 0;
  std::vector<LmSegPlan> hplans;
  std::vector<uint32_t> gdplans;  // STRAT_GDENSE: per-segment parameter tables (GdSegPlan + GdRsPlan, 128 dwords)
  DevBuf dgdplans;
  std::vector<DevBuf> owned;  // LUTs, remaps, HLL LUTs, value dictionaries
  DevBuf acc;                 // all accumulator sections (unless the caller provided the block)
  void* external_acc = nullptr;
  std::vector<Section> sections;
  std::vector<int> agg_section;  // agg -> section index (-1 for COUNT)

  ~pa_query() {
    dev_free(dq);
    dev_free(dsegs);
    dev_free(dplans);
    dev_free(dq_count);
    dev_free(dq_h);
    dev_free(dsegs_count);
    dev_free(lim_keys);
    dev_free(lim_pos);
    dev_free(lim_hist);
    dev_free(lim_sel);
    dev_free(lim_thresh);
    dev_free(stat_buf);
    dev_free(leap_buf);
    dev_free(merge_buf);
    dev_free(lim_admit);
    dev_free(dgdplans);
    dev_free(jit_args);
    dev_free(jit_segs);
    for (PveStream* p : {&pve, &pvh}) {
      dev_free(p->args);
      dev_free(p->segs);
      dev_free(p->buf);
    }
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

// ---------------------------------------------------------------- planning units of pa_query_prepare
// State handed from one unit to the next.
struct Prep {
  std::vector<char> clause_mv;
  double post_density = 1.0;
  double first_clause_sel = 1.0;  // estimated selectivity of the first (eager) clause
  bool has_filter = false;
  bool dense = true;
  bool stage_all = false, stage_post = false;
  std::vector<int> leaf_slot, gb_slot, agg_slot;
  std::vector<char> slot_eager, slot_post, slot_gb;
  std::vector<int64_t> stride;
  std::vector<int> gb_word;  // hashed, two-word keys: the word of each group-by component
  std::vector<char> gb_raw;
  uint64_t limit_pairs = 0;
  int limit_eb = 0;
  std::vector<char> limit_bind;  // per segment: the limit can bind there
  std::vector<int> agg_src;
  std::vector<char> val_fast, agg_mv;
  bool gb_mv = false;
  bool lm = false;
  size_t lds_acc = 0;  // LDS strategy: accumulator bytes
  std::vector<size_t> agg_lds;
  // STRAT_GDENSE (plan_gdense)
  bool gdense = false;
  std::vector<char> gd_stage_raw;          // per slot: raw aggregation column staged as a 32/64-bit "bit column"
  size_t gd_lds = 0;                       // LDS bytes of the accumulators + tables (the ring follows)
  int gd_rp_log2 = 0, gd_nkeys = 0, gd_tables = 0;
  bool gd_box = false;                     // the key box is exactly the filter (pa_gdense.h gd_box_tile)
  std::vector<int> gd_lut, gd_lut_words;   // per literal: LDS byte offset of its shared DICT_SET bitmap (-1: HBM)
  int gd_lo[PA_MAX_GROUP_BY] = {0}, gd_span[PA_MAX_GROUP_BY] = {0}, gd_ls[PA_MAX_GROUP_BY] = {0};
  int gd_tab[PA_MAX_GROUP_BY] = {0}, gd_tab_n[PA_MAX_GROUP_BY] = {0};
  std::vector<int> gd_vs, gd_op, gd_acc, gd_tab_a, gd_tab_an;
  std::vector<int64_t> gd_base, gd_step;
  std::vector<std::vector<const void*>> gd_src;  // [seg][agg] device dictionary behind the LDS value table
  // lane-major walk, packed accumulation (GdLmPlan): possible (COUNT + SUM terms fit), the term bits and, for a value
  // table turned into offsets (GVS_T32U), the offsets' base; chosen when the lane-major variant is
  bool gd_pk_ok = false, gd_packed = false;
  int gd_pk_c = 0;                         // bits of each field beyond its term (the drain bound)
  std::vector<int> gd_pk_w;                // per aggregation: term bits
  std::vector<char> gd_pk_t32u;            // per aggregation: the value table becomes uint32 offsets from gd_pk_base
  std::vector<int64_t> gd_pk_base;
};

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

bool affine_dictionary(const std::vector<uint64_t>& v, int32_t vtype, int64_t* base, int64_t* step);

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

// Tile geometry of one scan pass: wave tile of 1024 or 2048 docs, D DMA instructions per tile, a ring of R tile images
// per wave (R-1 tiles in flight). Measured on MI355X (tools/sweep.py): the decode, not the DMA, is what needs hiding,
// so the plan maximises resident waves per CU (workgroups per CU, checked against the occupancy the compiled kernel
// really has), then prefers 2048-doc tiles, then bytes in flight (capped at 128 KiB per CU).
struct TilePlan {
  int steps = 0, dma = 0, ring = 0, wg_per_cu = 0, img_dw = 0;
  size_t lds = 0;
  double score = -1;
};

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
          lp.pk_drain = ((1 << P.gd_pk_c) - 1) >> 10;  // tiles of <= 1024 docs each
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
  q->vremaps.assign(num_segments, std::vector<std::vector<int32_t>>(spec->num_aggs));
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

int pa_query_bind_value_remap(pa_query* q, int32_t index, int32_t agg, const int32_t* remap) {
  if (!q || index < 0 || index >= q->nseg || agg < 0 || agg >= q->spec.num_aggs) return fail(PA_EINVAL, "bad remap arguments");
  if (q->prepared) return fail(PA_EINVAL, "query already prepared");
  if (!q->segs[index]) return fail(PA_EINVAL, "bind the segment before its value remaps");
  const pa_agg_spec& A = q->spec.aggs[agg];
  if (A.type != PA_AGG_DISTINCTCOUNT) return fail(PA_EINVAL, "value remaps belong to DISTINCTCOUNT aggregations");
  auto it = q->segs[index]->cols.find(A.column_id);
  if (it == q->segs[index]->cols.end()) return fail(PA_EINVAL, "aggregation column missing in segment");
  q->vremaps[index][agg].clear();
  if (!remap) return PA_OK;
  const int32_t card = it->second->cardinality;
  q->vremaps[index][agg].assign(remap, remap + card);
  for (int32_t v : q->vremaps[index][agg])
    if (v < 0 || v >= A.num_values) return fail(PA_EINVAL, "value remap id outside the table-wide value dictionary");
  return PA_OK;
}

// counters + list length + overflow flag of the fused statistics (pa_scan.h "fused execution statistics")
static size_t leap_header_bytes(const pa_query* q) {
  return ((size_t)std::max(1, q->nseg) * 3 + 1 + (size_t)q->leap_slices) * sizeof(unsigned long long);
}

// Fused statistics (unless PA_QF_NO_FILTER_STATS): the scan counts the leap-frog statistics itself (leap_tile) when the filter is an AND of two
// single-value leaves whose first (eager) clause is sparse — each of its docs costs two short neighbour searches — and
// the scan is one pass (the partitioned and numGroupsLimit plans run the tile loop more than once).
static int plan_leaps(pa_query* q, const Prep& P) {
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
static int alloc_leaps(pa_query* q, const Prep& P) {
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

// ---------------------------------------------------------------- query-shape specialisation (gdl_jit.hip)
// The lane-major dense kernel with packed accumulation, compiled per query shape by hiprtc: every column width, image
// offset, leaf kind and field offset becomes a constant (no bit-width switch, no parameter reads, no DMA loop in the
// tile loop). Compiled once per shape and device and cached for the process; the generic kernel runs when the shape
// is outside the specialised form (or PA_QF_NO_JIT / PA_NO_JIT), or hiprtc fails.
static const char* kGdlJitSrc =
#include "gdl_jit_src.inc"
    ;

struct JitSegH {  // == gdl_jit.hip JitSeg
  uint64_t src[6];
  int64_t first_tile;
  int32_t num_docs, num_tiles;
  uint32_t lo_t[6], hi_t[6];
};
struct JitArgsH {  // == gdl_jit.hip JitArgs
  int64_t total_tiles;
  int32_t nseg, nkeys, key_lo, key_span, xcd_major, pad;
  int64_t key_stride;
  unsigned long long* matched;
  unsigned long long* count;
  int64_t* sum[6];
  int32_t sum_long[6];
  int64_t base[6], step[6];
  const uint32_t* lut[6];
  int32_t lut_words[6];
  const int64_t* tab[6];
  int32_t tab_n[6];
};

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
void jit_fill_pointers(pa_query* q, JitArgsH& a) {
  const pa_query_spec& s = q->spec;
  a.matched = q->hq.matched_docs;
  a.count = q->hq.count;
  int k = 0;
  for (int i = 0; i < s.num_aggs; ++i) {
    if (s.aggs[i].type == PA_AGG_COUNT) continue;
    a.sum[k] = q->hq.aggs[i].acc_i64;
    a.sum_long[k] = q->hq.aggs[i].src == SRC_LONG ? 1 : 0;
    ++k;
  }
}

int jit_plan(pa_query* q, const Prep& P, int cus) {
  q->jit_fn = nullptr;
  const pa_query_spec& s = q->spec;
  if (!is_gdense_lm(q->strategy) || !P.gd_packed || P.gd_box || q->hq.leap_mode || q->nseg == 0) return PA_OK;
  if ((s.flags & PA_QF_NO_JIT) || std::getenv("PA_NO_JIT") || std::getenv("PA_DEBUG_EMIT")) return PA_OK;
  if (s.num_group_by != 1 || P.gd_tab[0] >= 0 || q->num_eager > 6) return PA_OK;
  const DevSeg& d0 = q->hsegs[0];
  const int nc = d0.num_staged;
  if (nc < 1 || nc > 6) return PA_OK;
  for (const DevSeg& d : q->hsegs) {
    if (d.num_staged != nc) return PA_OK;
    for (int k = 0; k < nc; ++k)
      if (d.stage[k].nbits != d0.stage[k].nbits || d.stage[k].lds_off != d0.stage[k].lds_off || d.stage[k].nbits < 1 ||
          d.stage[k].nbits > 31)
        return PA_OK;
  }
  auto col_of = [&](int lds_off) {
    for (int k = 0; k < nc; ++k)
      if (d0.stage[k].lds_off == lds_off) return k;
    return -1;
  };
  auto lmp = [&](int si) -> const GdLmPlan& { return *(const GdLmPlan*)&q->gdplans[(size_t)si * kGdPlanDw + 128]; };
  for (int si = 1; si < q->nseg; ++si)
    if (lmp(si).key_leaf != lmp(0).key_leaf || lmp(si).key_in_box != lmp(0).key_in_box) return PA_OK;
  const int nkeys = P.gd_nkeys;
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  // LDS: counts, sums, bitmaps, tables, then (per wave count) rows and ring
  size_t off = al16((size_t)nkeys * 4);
  std::vector<int> lsum;
  std::vector<int> ac, at, as;
  JitArgsH a;
  std::memset(&a, 0, sizeof(a));
  int k = 0;
  for (int i = 0; i < s.num_aggs; ++i) {
    if (s.aggs[i].type == PA_AGG_COUNT) continue;
    if (P.gd_op[i] != GOP_SUM_I || (P.gd_vs[i] != GVS_ID && P.gd_vs[i] != GVS_T32U)) return PA_OK;
    for (int si = 1; si < q->nseg; ++si)
      if (P.gd_vs[i] == GVS_T32U && P.gd_src[si][i] != P.gd_src[0][i]) return PA_OK;
    const int c = col_of(d0.cols[P.agg_slot[i]].lds_off);
    if (c < 0) return PA_OK;
    lsum.push_back((int)off);
    off += al16((size_t)nkeys * 8);
    ac.push_back(c);
    as.push_back(lmp(0).pk_off[k]);
    a.base[k] = P.gd_base[i];
    a.step[k] = P.gd_step[i];
    ++k;
  }
  const int na = k;
  std::vector<int> lk, lc, ln, le, lut;
  for (int li = 0; li < q->num_eager; ++li) {
    const DevLeaf& L = d0.leaves[li];
    for (const DevSeg& d : q->hsegs)
      if (d.leaves[li].negate != L.negate || d.leaves[li].kind != L.kind) return PA_OK;
    if (L.kind != PA_LEAF_DICT_RANGE && L.kind != PA_LEAF_DICT_SET) return PA_OK;
    const int c = col_of(L.lds_off);
    if (c < 0) return PA_OK;
    lk.push_back(L.kind == PA_LEAF_DICT_SET ? 1 : 0);
    lc.push_back(c);
    ln.push_back(L.negate ? 1 : 0);
    le.push_back(L.clause_end ? 1 : 0);
    if (L.kind == PA_LEAF_DICT_SET) {
      if (li >= (int)P.gd_lut.size() || P.gd_lut[li] < 0) return PA_OK;
      lut.push_back((int)off);
      a.lut[li] = L.lut;
      a.lut_words[li] = P.gd_lut_words[li];
      off += al16((size_t)P.gd_lut_words[li] * 4);
    } else {
      lut.push_back(0);
    }
  }
  k = 0;
  for (int i = 0; i < s.num_aggs; ++i) {
    if (s.aggs[i].type == PA_AGG_COUNT) continue;
    if (P.gd_vs[i] == GVS_T32U) {
      at.push_back((int)off);
      a.tab[k] = (const int64_t*)P.gd_src[0][i];
      a.tab_n[k] = P.gd_tab_an[i];
      off += al16((size_t)P.gd_tab_an[i] * 4);
    } else {
      at.push_back(-1);
    }
    ++k;
  }
  const int kc = col_of(d0.cols[P.gb_slot[0]].lds_off);
  if (kc < 0) return PA_OK;
  const size_t img_b = (size_t)q->hq.image_dwords_max * 4;
  int w = 0;
  for (int cand : {16, 8})
    if (al16(off + (size_t)cand * nkeys * 8) + (size_t)cand * 2 * img_b <= kLdsBudget) {
      w = cand;
      break;
    }
  if (!w) return PA_OK;
  const size_t rows = off;
  const size_t ring = al16(off + (size_t)w * nkeys * 8);
  const size_t lds = ring + (size_t)w * 2 * img_b;
  auto pad6 = [](std::vector<int> v) {
    if (v.empty()) v.push_back(0);
    return v;
  };
  std::vector<int> nb, coff;
  for (int c = 0; c < nc; ++c) {
    nb.push_back(d0.stage[c].nbits);
    coff.push_back(4 * d0.stage[c].lds_off);
  }
  const GdLmPlan& L0 = lmp(0);
  std::vector<std::string> defs = {
      "-DJIT_W=" + std::to_string(w), "-DJIT_IMG=" + std::to_string(q->hq.image_dwords_max),
      "-DJIT_NC=" + std::to_string(nc), "-DJIT_NB=" + int_list(nb), "-DJIT_OFF=" + int_list(coff),
      "-DJIT_NL=" + std::to_string(q->num_eager), "-DJIT_LK=" + int_list(pad6(lk)), "-DJIT_LC=" + int_list(pad6(lc)),
      "-DJIT_LN=" + int_list(pad6(ln)), "-DJIT_LE=" + int_list(pad6(le)), "-DJIT_LUT=" + int_list(pad6(lut)),
      "-DJIT_KC=" + std::to_string(kc), "-DJIT_KL=" + std::to_string(L0.key_leaf),
      "-DJIT_KIB=" + std::to_string(L0.key_in_box ? 1 : 0), "-DJIT_NA=" + std::to_string(na),
      "-DJIT_AC=" + int_list(pad6(ac)), "-DJIT_AT=" + int_list(pad6(at)), "-DJIT_AS=" + int_list(pad6(as)),
      "-DJIT_OC=" + std::to_string(L0.pk_cnt), "-DJIT_DRAIN=" + std::to_string(std::max(1, L0.pk_drain)),
      "-DJIT_L_SUM=" + int_list(pad6(lsum)), "-DJIT_L_ROWS=" + std::to_string(rows),
      "-DJIT_L_RING=" + std::to_string(ring)};
  hipFunction_t fn = jit_compile(defs);
  if (!fn) return PA_OK;
  (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  // descriptors
  a.total_tiles = q->hq.total_wtiles;
  a.nseg = q->nseg;
  a.nkeys = nkeys;
  a.key_lo = P.gd_lo[0];
  a.key_span = P.gd_span[0];
  a.xcd_major = 1;
  a.key_stride = q->hq.gb_stride[0];
  jit_fill_pointers(q, a);
  std::vector<JitSegH> js(q->nseg);
  for (int si = 0; si < q->nseg; ++si) {
    const DevSeg& d = q->hsegs[si];
    JitSegH& j = js[si];
    std::memset(&j, 0, sizeof(j));
    for (int c = 0; c < nc; ++c) j.src[c] = (uint64_t)(uintptr_t)d.stage[c].words;
    j.first_tile = d.first_wtile;
    j.num_docs = d.num_docs;
    j.num_tiles = d.num_wtiles;
    for (int li = 0; li < q->num_eager; ++li) {
      j.lo_t[li] = (uint32_t)d.leaves[li].lo;
      j.hi_t[li] = (uint32_t)d.leaves[li].span;
    }
  }
  int rc = dev_alloc(q->jit_args, sizeof(JitArgsH));
  if (!rc) rc = dev_alloc(q->jit_segs, sizeof(JitSegH) * js.size());
  if (rc) return rc;
  PA_HIP(hipMemcpy(q->jit_args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(q->jit_segs.p, js.data(), sizeof(JitSegH) * js.size(), hipMemcpyHostToDevice));
  q->jit_fn = fn;
  q->jit_waves = w;
  q->jit_lds = (int)lds;
  q->jit_grid = (int)std::max<int64_t>(1, std::min<int64_t>(cus, (q->hq.total_wtiles + w - 1) / w));
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

struct PveSegH {  // == pve_jit.hip PveSeg
  uint64_t src[6];
  int64_t first_tile;
  int32_t num_docs, num_tiles;
  uint32_t lo_t[6], hi_t[6];
  uint64_t admit;
  uint64_t raw, mv_off, mv_words, hlut;
};
struct PveArgsH {  // == pve_jit.hip PveArgs
  int64_t total_tiles;
  int32_t nseg, xcd_major;
  int64_t chunks_per_wg;
  uint32_t* recs;
  uint32_t* table;
  uint32_t* hist;
  uint32_t* used;
  unsigned long long* matched;
};

static void pve_fill_pointers(const pa_query::PveStream& st, unsigned long long* matched, PveArgsH& a) {
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
  for (int si = 0; si < q->nseg; ++si) {
    const DevSeg& d = q->hsegs[si];
    if (d.vremap) return PA_OK;
    for (int j = 0; j < s.num_group_by; ++j)
      if (d.remap[j]) return PA_OK;
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
  // chunks from a 16-byte aligned start, one word of look-ahead)
  auto val_bytes = [&](int nd) {
    return hmode ? (size_t)16 * (((size_t)max_values * 64 * nd * hnb / 32 + 9 + 3) / 4) : (size_t)0;
  };
  auto waves_for = [&](int nd, int bs) {
    for (int cand : {16, 12, 8, 4})
      if (lds_ring(bs) + (size_t)cand * (2 * image_bytes(nd) + val_bytes(nd)) <= kLdsBudget) return cand;
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
  const size_t l_val = l_ring + (size_t)w * 2 * img_bytes;
  const size_t vbytes = val_bytes(nd);
  const size_t lds = l_val + (size_t)w * vbytes;
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
      "-DPVE_L_VAL=" + std::to_string(l_val), "-DPVE_VAL_B=" + std::to_string(vbytes)};
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
  PveArgsH a;
  std::memset(&a, 0, sizeof(a));
  a.total_tiles = T;
  a.nseg = q->nseg;
  a.xcd_major = 1;
  a.chunks_per_wg = C;
  pve_fill_pointers(S, q->hq.matched_docs, a);
  std::vector<PveSegH> js(q->nseg);
  for (int si = 0; si < q->nseg; ++si) {
    const DevSeg& d = q->hsegs[si];
    PveSegH& j = js[si];
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
    if (rslot >= 0) j.raw = (uint64_t)(uintptr_t)d.cols[rslot].raw;
    if (hmode) {
      j.mv_off = (uint64_t)(uintptr_t)d.cols[mslot].mv_off;
      j.mv_words = (uint64_t)(uintptr_t)d.cols[mslot].words;
      j.hlut = (uint64_t)(uintptr_t)d.hll_lut[h.hll_agg];
    }
  }
  rc = dev_alloc(S.args, sizeof(PveArgsH));
  if (!rc) rc = dev_alloc(S.segs, sizeof(PveSegH) * js.size());
  if (rc) return rc;
  PA_HIP(hipMemcpy(S.args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(S.segs.p, js.data(), sizeof(PveSegH) * js.size(), hipMemcpyHostToDevice));
  S.fn = fn;
  S.waves = w;
  S.grid = G;
  S.lds = (int)lds;
  S.cr = (int)cr;
  S.parts = Pn;
  S.bin_shift = __builtin_ctz((unsigned)bs);
  S.chunks = C;
  PLAN_LOG("pve %s: W %d nd %d bs %d sc %d grid %d lds %zu C %lld P %d", hmode ? "H" : "V", w, nd, bs, sc, G, lds,
           (long long)C, Pn);
  return PA_OK;
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
  const int64_t base_entries = (int64_t)h.pv + 1 + (hstream ? (int64_t)(h.num_parts - h.pv) + 1 : 0);
  int rc = pve_stream(q, P, cus, false, rw, rawb, base_entries, q->pve);
  if (rc || !q->pve.fn || !hstream) return rc;
  rc = pve_stream(q, P, cus, true, 1, 0, 0, q->pvh);
  if (rc || !q->pvh.fn) q->pve.fn = nullptr;  // (both streams or neither: the count pass serves both)
  return rc;
}

int pa_query_prepare(pa_query* q) {
  if (!q) return fail(PA_EINVAL, "null query");
  if (q->prepared) return PA_OK;
  for (int i = 0; i < q->nseg; ++i)
    if (!q->segs[i]) return fail(PA_EINVAL, "segment " + std::to_string(i) + " not bound");
  Prep P;
  std::memset(&q->hq, 0, sizeof(q->hq));
  int rc = plan_filter(q, P);
  if (!rc) rc = plan_slots(q, P);
  if (!rc) rc = plan_key_space(q, P);
  if (!rc) rc = plan_limit(q, P);
  if (!rc) rc = plan_gdense(q, P);
  if (!rc) rc = build_segments(q, P);
  if (!rc) rc = plan_walk(q, P);
  if (!rc) rc = plan_accumulators(q, P);
  TilePlan plan, count_plan;
  if (!rc) rc = plan_kernels(q, P, plan, count_plan);
  if (rc) return rc;

  // layout: tiles per segment, LDS regions (the count pass has its own staging), staged bytes
  void* dummy = nullptr;  // 256 readable bytes: source of the DMA padding instructions
  {
    std::vector<char> z(256, 0);
    rc = upload_owned(q, z.data(), z.size(), &dummy);
    if (rc) return rc;
  }
  const int nslots = (int)q->slot_cols.size();
  int64_t total_tiles = 0;
  apply_layout(q->hsegs, plan.steps, nslots, (int)q->literals.size(), dummy, &q->staged_bytes, &total_tiles);
  q->num_tiles = (uint64_t)total_tiles;
  q->lane_major = P.lm ? 1 : 0;
  q->dense_packed = P.gd_packed ? 1 : 0;
  q->plan_ring = plan.ring;
  q->plan_wg = plan.wg_per_cu;
  fill_devquery(q, P, plan, total_tiles);
  rc = plan_leaps(q, P);
  if (rc) return rc;

  // grid: persistent waves, enough workgroups to cover the CUs several times over
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
  }
  const int wg_cu = q->split_emit ? std::min(plan.wg_per_cu, q->emit_h_wg) : plan.wg_per_cu;
  const int64_t max_wg = (int64_t)cus * std::max(1, wg_cu);
  const int wpw = q->partitioned ? scan_waves(q->emit_strat) : scan_waves(q->strategy);
  const int64_t want = (total_tiles + wpw - 1) / wpw;
  q->grid = (int)std::max<int64_t>(1, std::min(max_wg, want));

  if (q->partitioned) {
    // the count pass: the same tiles, waves and grid; only the group-by and filter columns staged
    int64_t ct = 0;
    apply_layout(q->hsegs_count, plan.steps, nslots, (int)q->literals.size(), dummy, nullptr, &ct);
    if (ct != total_tiles) return fail(PA_EINVAL, "internal: count pass tiles differ");
    DevQuery& c = q->hq_count;
    c = q->hq;
    c.strategy = q->count_strat;
    c.count_skip_gb = q->count_skip;
    c.image_dwords_max = count_plan.img_dw;
    c.ring = count_plan.ring;
    c.dma_per_tile = count_plan.dma;
    c.num_staged = 0;
    for (int sl = 0; sl < nslots; ++sl) {
      bool st = false;
      for (const DevSeg& d : q->hsegs_count) st |= d.cols[sl].lds_off >= 0;
      if (st) c.staged_slots[c.num_staged++] = sl;
    }
    c.lds_acc_bytes = (uint32_t)(((size_t)q->hq.num_parts * 4 + 15) & ~(size_t)15);
    q->count_lds = (int)count_plan.lds;
    q->count_ring = count_plan.ring;
    // the count pass stages fewer columns, so more of its workgroups fit a CU: k per emit workgroup (each walks 1/k of
    // that workgroup's tiles; part_scan_kernel sums their rows), as many as are resident at once
    q->count_k = std::max(1, count_plan.wg_per_cu / std::max(1, wg_cu));
    while (q->count_k > 1 && (int64_t)q->grid * q->count_k * kWavesPerWG > total_tiles) --q->count_k;
    // the emit pass's LDS: partition bin state + bins in front of the ring
    q->hq.lds_acc_bytes = (uint32_t)(plan.lds - (size_t)wpw * plan.ring * plan.img_dw * 4);
    if (q->split_emit) {  // the H launch: same tiles and staging, its own ring depth, bins and partitions
      DevQuery& e = q->hq_h;
      e = q->hq;
      e.strategy = STRAT_PEMIT;
      e.ring = q->emit_h_ring;
      e.lds_acc_bytes = (uint32_t)((size_t)q->emit_h_lds -
                                   (size_t)scan_waves(q->emit_h_strat) * q->emit_h_ring * plan.img_dw * 4);
      e.part_lo = q->hq.pv;
      e.part_hi = q->hq.num_parts;
    }
    rc = plan_scratch(q, P);
    if (rc) return rc;
  }
  if (q->limit_mode) {
    rc = plan_limit_buffers(q, P, cus, total_tiles);
    if (rc) return rc;
  }
  rc = alloc_leaps(q, P);
  if (rc) return rc;
  rc = upload_descriptors(q);
  if (rc) return rc;
  rc = jit_plan(q, P, cus);
  if (rc) return rc;
  rc = pve_plan(q, P, cus);
  if (rc) return rc;
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
  if (q->hq.leap_mode) PA_HIP(hipMemsetAsync(q->leap_buf.p, 0, leap_header_bytes(q), st));
  for (const Section& sc : q->sections) {
    if (sc.kind == PA_ACC_MIN_I64 || sc.kind == PA_ACC_KEYS_I64) PA_HIP(launch_fill_i64((int64_t*)sc.ptr, sc.n, INT64_MAX, st));
    else if (sc.kind == PA_ACC_MAX_I64) PA_HIP(launch_fill_i64((int64_t*)sc.ptr, sc.n, INT64_MIN, st));
  }
  return PA_OK;
}

int pa_query_scan(pa_query* q, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  q->scanned_since_fetch = true;
  if (q->num_tiles == 0) return PA_OK;
  hipStream_t st = (hipStream_t)stream;
  if (q->limit_walk) {  // admitted keys of every segment where the limit can bind, before any pass tests them
    if (q->walk_words > kWalkMaxWords) PA_HIP(hipMemsetAsync(q->lim_admit.p, 0, q->lim_admit.n, st));
    PA_HIP(launch_limit_walk((const DevQuery*)q->dq.p, (const DevSeg*)q->dsegs.p, q->nseg, q->walk_words,
                             q->hq.gb_mv >= 0, st));
  }
  if (q->limit_mode) {  // first-seen positions, per-segment selection of the threshold, admitted aggregation
    const DevQuery* dq = (const DevQuery*)q->dq.p;
    const DevSeg* ds = (const DevSeg*)q->dsegs.p;
    const LimitDesc& F = q->limit;
    const int64_t H = F.fmask + 1;
    PA_HIP(launch_fill_i64((int64_t*)F.fkeys, H, INT64_MAX, st));
    PA_HIP(launch_fill_i64((int64_t*)F.fpos, H, -1, st));
    PA_HIP(launch_fill_i64((int64_t*)F.thresh, std::max(1, q->nseg), -1, st));
    PA_HIP(launch_fill_i64((int64_t*)F.hist, std::max(1, q->nseg) * 128, 0, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 0, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 1, st));
    PA_HIP(launch_limit_passes(dq, ds, F, q->limit_grid, 2, st));
    return PA_OK;
  }
  if (q->pve.fn) {  // the count-free emit: records in per-workgroup chunks, the partitions' chunk lists, pass C
    PartScratch ps{};
    char* vb = (char*)q->pve.buf.p;
    ps.base = (uint64_t*)(vb + q->pve.o_base);
    for (pa_query::PveStream* S : {&q->pve, &q->pvh}) {
      if (!S->fn) continue;
      void* pa = S->args.p;
      void* psg = S->segs.p;
      void* params[] = {&pa, &psg};
      PA_HIP(hipModuleLaunchKernel(S->fn, S->grid, 1, 1, S->waves * kWave, 1, 1, S->lds, st, params, nullptr));
      char* b = (char*)S->buf.p;
      // (the H partitions' bases follow the V partitions' in the V buffer's base array: base[pv + 1 ..])
      uint64_t* base = S == &q->pve ? ps.base : ps.base + q->hq.pv + 1;
      PA_HIP(launch_pve_lists((const uint32_t*)(b + S->o_hist), (uint32_t*)(b + S->o_off), base,
                              (const uint32_t*)(b + S->o_table), (const uint32_t*)(b + S->o_used),
                              (uint32_t*)(b + S->o_index), (uint32_t*)(b + S->o_tot), S->grid, S->parts, S->chunks,
                              S->cr, st));
      if (S == &q->pve) {
        ps.recs_v = (uint32_t*)b;
        ps.chunk_index = (const uint32_t*)(b + S->o_index);
        ps.chunk_shift = __builtin_ctz((unsigned)S->cr);
        ps.chunk_bin_shift = S->bin_shift;
      } else {
        ps.recs_h = (uint32_t*)b;
        ps.chunk_index_h = (const uint32_t*)(b + S->o_index);
        ps.chunk_shift_h = __builtin_ctz((unsigned)S->cr);
        ps.chunk_bin_shift_h = S->bin_shift;
      }
    }
    PA_HIP(launch_part_agg(q->part_vk, (const DevQuery*)q->dq.p, ps, q->pvh.fn ? q->hq.num_parts : q->hq.pv,
                           q->part_lds_c, st));
    return PA_OK;
  }
  if (q->partitioned) {  // count pass, range offsets, emit pass into the partitions, per-partition aggregation
    ScratchArena* a = arena_for(q->scratch_dev);
    std::lock_guard<std::mutex> g(a->mu);
    int rc = arena_grow(a, q->sc_bytes);
    if (rc) return rc;
    if (a->used && a->last_stream != st) PA_HIP(hipStreamWaitEvent(st, a->last, 0));
    const PartScratch ps = scratch_of(q, a->p);
    const LmSegPlan* plans = (const LmSegPlan*)q->dplans.p;
    PA_HIP(launch_scan(q->count_strat, q->steps, 0, q->grid * q->count_k, q->count_lds, (const DevQuery*)q->dq_count.p,
                       (const DevSeg*)q->dsegs_count.p, plans, ps, st));
    PA_HIP(launch_part_offsets(&q->hq, ps, q->grid, q->count_k, st));
    PA_HIP(launch_scan(q->emit_strat, q->steps, 0, q->grid, q->lds_bytes, (const DevQuery*)q->dq.p,
                       (const DevSeg*)q->dsegs.p, plans, ps, st));
    if (q->split_emit)
      PA_HIP(launch_scan(q->emit_h_strat, q->steps, 0, q->grid, q->emit_h_lds, (const DevQuery*)q->dq_h.p,
                         (const DevSeg*)q->dsegs.p, plans, ps, st));
    PA_HIP(launch_part_agg(q->part_vk, (const DevQuery*)q->dq.p, ps, q->hq.num_parts, q->part_lds_c, st));
    PA_HIP(hipEventRecord(a->last, st));
    a->last_stream = st;
    a->used = true;
    return PA_OK;
  }
  if (q->jit_fn) {  // the query-shape specialised dense kernel
    void* pa = q->jit_args.p;
    void* ps = q->jit_segs.p;
    void* params[] = {&pa, &ps};
    PA_HIP(hipModuleLaunchKernel(q->jit_fn, q->jit_grid, 1, 1, q->jit_waves * kWave, 1, 1, q->jit_lds, st, params,
                                 nullptr));
    return PA_OK;
  }
  PartScratch none{};
  PA_HIP(launch_scan(q->strategy, q->steps, q->lane_major, q->grid, q->lds_bytes, (const DevQuery*)q->dq.p,
                     (const DevSeg*)q->dsegs.p, (const LmSegPlan*)q->dplans.p, none, st));
  q->leap_searched = false;  // (the neighbour searches of the listed E docs run when the statistics are asked for)
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
  // every scan descriptor of the query (the partitioned count pass has its own) points into the new block
  auto relocate = [&](DevQuery& h) {
    h.count = (unsigned long long*)(nb + ((char*)h.count - old));
    h.matched_docs = (unsigned long long*)(nb + ((char*)h.matched_docs - old));
    if (q->hashed) h.ht_keys = (long long*)(nb + ((char*)h.ht_keys - old));
    for (int a = 0; a < h.num_aggs; ++a) {
      if (q->agg_section[a] < 0) continue;
      void* p = q->sections[q->agg_section[a]].ptr;
      h.aggs[a].acc_i64 = (int64_t*)p;
      h.aggs[a].acc_f64 = (double*)p;
      h.aggs[a].acc_hll = (uint8_t*)p;
    }
  };
  relocate(q->hq);
  if (q->limit_mode) q->limit.reached = q->hq.matched_docs + 2;
  PA_HIP(hipMemcpy(q->dq.p, &q->hq, sizeof(DevQuery), hipMemcpyHostToDevice));
  if (q->jit_fn) {
    JitArgsH a;
    PA_HIP(hipMemcpy(&a, q->jit_args.p, sizeof(a), hipMemcpyDeviceToHost));
    jit_fill_pointers(q, a);
    PA_HIP(hipMemcpy(q->jit_args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  }
  for (pa_query::PveStream* S : {&q->pve, &q->pvh}) {
    if (!S->fn) continue;
    PveArgsH a;
    PA_HIP(hipMemcpy(&a, S->args.p, sizeof(a), hipMemcpyDeviceToHost));
    pve_fill_pointers(*S, q->hq.matched_docs, a);
    PA_HIP(hipMemcpy(S->args.p, &a, sizeof(a), hipMemcpyHostToDevice));
  }
  if (q->partitioned) {
    relocate(q->hq_count);
    PA_HIP(hipMemcpy(q->dq_count.p, &q->hq_count, sizeof(DevQuery), hipMemcpyHostToDevice));
    if (q->split_emit) {
      relocate(q->hq_h);
      PA_HIP(hipMemcpy(q->dq_h.p, &q->hq_h, sizeof(DevQuery), hipMemcpyHostToDevice));
    }
  }
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

  // Decodes `nrows` host rows into the caller's arrays: row r has key key_of(r, w) (word w < kw: two-word hashed keys
  // fill out_keys[2 n], out_keys[2 n + 1]), count hc[r] and the aggregation section rows at sec(section)[r * per]. Rows
  // with a zero count are skipped when `skip_empty`. `order` (optional) lists the rows to emit, in output order (hashed
  // key spaces: sorted by packed key).
  const int kw = q->hashed ? q->key_words : 1;
  auto decode = [&](int64_t nrows, const uint64_t* hc, const std::function<const char*(int)>& sec,
                    const std::function<int64_t(int64_t, int)>& key_of, bool skip_empty,
                    const std::vector<int64_t>* order) -> int64_t {
    const char* asec[PA_MAX_AGGS];  // section base per aggregation, resolved once (not per row)
    for (int a = 0; a < s.num_aggs; ++a) asec[a] = q->agg_section[a] >= 0 ? sec(q->agg_section[a]) : nullptr;
    int64_t n = 0;
    const int64_t total = order ? (int64_t)order->size() : nrows;
    for (int64_t oi = 0; oi < total; ++oi) {
      const int64_t r = order ? (*order)[oi] : oi;
      if (skip_empty && hc[r] == 0) continue;
      if (n < capacity) {
        if (out_keys)
          for (int w = 0; w < kw; ++w) out_keys[kw * n + w] = key_of(r, w);
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
          if (A.type == PA_AGG_DISTINCTCOUNTHLL || A.type == PA_AGG_DISTINCTCOUNT) {
            const int64_t per = A.type == PA_AGG_DISTINCTCOUNT ? presence_stride(A) : int64_t(1) << A.log2m;
            uint8_t* o = (uint8_t*)out_aggs[a] + n * per;
            std::memcpy(o, (const uint8_t*)sp + r * per, (size_t)per);
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
    q->scanned_since_fetch = false;
    if (docs[1]) return fail(PA_EUNSUPPORTED, "group-key table overflow (more distinct groups than slots)");
    if (docs[3]) return fail(PA_EHIP, "internal: partitioned passes disagree on record counts");
    const uint64_t* hc = (const uint64_t*)hsec(0);
    if (q->hashed) {
      const int64_t* hk = (const int64_t*)hsec(q->keys_section);
      const int ks = kw == 2 ? 3 : 1;  // key-section words per slot
      std::vector<int64_t> order;
      for (int64_t r = 0; r < K; ++r)
        if (hc[r]) order.push_back(r);
      std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return hk[ks * a] != hk[ks * b] ? hk[ks * a] < hk[ks * b] : (kw == 2 && hk[ks * a + 1] < hk[ks * b + 1]);
      });
      return decode(K, hc, hsec, [&](int64_t r, int w) { return hk[ks * r + w]; }, false, &order);
    }
    return decode(K, hc, hsec, [](int64_t r, int) { return r; }, grouped, nullptr);
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
  uint64_t md[4] = {0, 0, 0, 0};
  PA_HIP(launch_compact((const unsigned long long*)q->sections[0].ptr, K, all, (uint32_t*)q->fetch_blocks.p, 0,
                        nullptr, 0, st));
  PA_HIP(hipMemcpyAsync(&total, (uint32_t*)q->fetch_blocks.p + nb, 4, hipMemcpyDeviceToHost, st));
  PA_HIP(hipMemcpyAsync(md, q->sections.back().ptr, 32, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  q->last_matched = (int64_t)md[0];
  q->last_reached = (int64_t)md[2];
  q->scanned_since_fetch = false;
  if (md[1]) return fail(PA_EUNSUPPORTED, "group-key table overflow (more distinct groups than slots)");
  if (md[3]) return fail(PA_EHIP, "internal: partitioned passes disagree on record counts");
  const int64_t m = (int64_t)total;
  const int64_t rows_cap = std::min<int64_t>(m, std::max<int64_t>(capacity, 0));
  if (rows_cap == 0) return m;
  if (!q->hashed) {
    // Direct key space: the compaction writes the caller's representation (key ids, counts, doubles / register bytes)
    // into staging columns on the GPU, and each column goes to the caller's array in one copy (a DMA straight into
    // pinned memory when the caller's arrays are pinned: engine.py keeps a reused pinned output pool). No host decode.
    FinalDesc f;
    std::memset(&f, 0, sizeof(f));
    f.nagg = s.num_aggs;
    std::vector<size_t> off(s.num_aggs, 0);
    size_t bytes = ((size_t)rows_cap * 16 + 255) & ~(size_t)255;  // keys | counts
    for (int a = 0; a < s.num_aggs; ++a) {
      const pa_agg_spec& A = s.aggs[a];
      f.type[a] = A.type;
      f.src[a] = q->hq.aggs[a].src;
      f.sec[a] = q->agg_section[a] >= 0 ? q->sections[q->agg_section[a]].ptr : nullptr;
      f.per[a] = A.type == PA_AGG_DISTINCTCOUNT ? presence_stride(A)
                                                : (A.type == PA_AGG_DISTINCTCOUNTHLL ? (int64_t(1) << A.log2m) : 8);
      off[a] = bytes;
      bytes += ((size_t)rows_cap * (size_t)f.per[a] + 255) & ~(size_t)255;
    }
    if (q->fetch_stage.n < bytes) {
      dev_free(q->fetch_stage);
      int rc = dev_alloc(q->fetch_stage, bytes);
      if (rc) return rc;
    }
    char* ds = (char*)q->fetch_stage.p;
    f.keys = (int64_t*)ds;
    f.counts = (int64_t*)(ds + (size_t)rows_cap * 8);
    for (int a = 0; a < s.num_aggs; ++a) f.out[a] = ds + off[a];
    PA_HIP(launch_compact_final((const unsigned long long*)q->sections[0].ptr, K, all,
                                (const uint32_t*)q->fetch_blocks.p, rows_cap, &f, st));
    if (out_keys) PA_HIP(hipMemcpyAsync(out_keys, f.keys, (size_t)rows_cap * 8, hipMemcpyDeviceToHost, st));
    if (out_counts) PA_HIP(hipMemcpyAsync(out_counts, f.counts, (size_t)rows_cap * 8, hipMemcpyDeviceToHost, st));
    for (int a = 0; a < s.num_aggs; ++a)
      if (out_aggs && out_aggs[a])
        PA_HIP(hipMemcpyAsync(out_aggs[a], f.out[a], (size_t)rows_cap * (size_t)f.per[a], hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    return m;
  }
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
    const int es = (int)section_es(sc.kind);  // HLL registers / presence: one byte each
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
    d.es[i] = (int32_t)section_es(sc.kind);
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
    const int ks = kw == 2 ? 3 : 1;
    std::vector<int64_t> order(rows);
    for (int64_t r = 0; r < rows; ++r) order[r] = r;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
      return pk[ks * a] != pk[ks * b] ? pk[ks * a] < pk[ks * b] : (kw == 2 && pk[ks * a + 1] < pk[ks * b + 1]);
    });
    order.resize(rows_cap);
    decode(rows, (const uint64_t*)hsec[0], [&](int sec) { return hsec[sec]; },
           [&](int64_t r, int w) { return pk[ks * r + w]; }, false, &order);
    return m;
  }
  decode(rows, (const uint64_t*)hsec[0], [&](int sec) { return hsec[sec]; }, [&](int64_t r, int) { return hkeys[r]; },
         false, nullptr);
  return m;
}

// words per leaf bitmap: whole 64-doc steps, rounded up to 4 words (the count kernels read 16-byte groups)
int64_t leaf_words(int64_t num_docs) { return (num_docs + 127) / 128 * 4; }

int64_t pa_query_leaf_bitmap_words(const pa_query* q, int32_t segment) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (segment < 0 || segment >= q->nseg) return fail(PA_EINVAL, "segment index out of range");
  return leaf_words((int64_t)q->segs[segment]->num_docs);
}

int pa_query_leaf_bitmaps(pa_query* q, int32_t segment, uint32_t* device_out, void* stream) {
  const int64_t words = pa_query_leaf_bitmap_words(q, segment);
  if (words < 0) return (int)words;
  if (!device_out) return fail(PA_EINVAL, "null bitmap buffer");
  hipStream_t st = (hipStream_t)stream;
  const DevSeg* ds = (const DevSeg*)q->dsegs.p + segment;
  for (int l = 0; l < q->spec.num_leaves; ++l) {
    // the leaf's first CNF literal: literal value = leaf value XOR the literal's negation
    int li = -1;
    for (size_t i = 0; i < q->literals.size() && li < 0; ++i)
      if (q->literals[i].leaf == l) li = (int)i;
    if (li < 0) return fail(PA_EUNSUPPORTED, "filter leaf " + std::to_string(l) + " has no literal in the plan");
    PA_HIP(launch_leaf_bitmap(ds, li, q->literals[li].neg ? 1 : 0, q->segs[segment]->num_docs,
                              device_out + (size_t)l * words, st));
  }
  return PA_OK;
}

// Validated postfix program of pa_bitmap_counts / pa_query_filter_counts into tok[0..len).
int check_bit_prog(const int32_t* prog, int32_t len, int32_t num_leaves, bool required, int32_t* tok) {
  if (len < 0 || len > kBitProgMax || (required && len == 0) || (len > 0 && !prog))
    return fail(PA_EINVAL, "bitmap program length out of range");
  int depth = 0;
  for (int i = 0; i < len; ++i) {
    const int32_t t = prog[i];
    if (t >= 0) {
      if (t >= num_leaves) return fail(PA_EINVAL, "bitmap program names a leaf out of range");
      if (++depth > kBitProgStack) return fail(PA_EINVAL, "bitmap program too deep");
    } else if (t == PA_BIT_NOT) {
      if (depth < 1) return fail(PA_EINVAL, "bitmap program: NOT on an empty stack");
    } else if (t == PA_BIT_AND || t == PA_BIT_OR) {
      if (depth < 2) return fail(PA_EINVAL, "bitmap program: AND/OR needs two masks");
      --depth;
    } else {
      return fail(PA_EINVAL, "bitmap program: unknown token");
    }
    tok[i] = t;
  }
  if (len > 0 && depth != 1) return fail(PA_EINVAL, "bitmap program must leave exactly one mask");
  return PA_OK;
}

constexpr size_t kBitTokBytes = 2 * kBitProgMax * 4;

// The count kernels keep up to 4 leaves' words in registers: renumber the programs' leaf tokens to positions in
// job.uleaf when they use at most 4 distinct leaves (else nu = 0: leaf ids, loaded in program order).
void renumber_leaves(BitJob& job, int32_t* tok) {
  int32_t u[4];
  int nu = 0;
  const int lens[2] = {job.len_a, job.len_b};
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < lens[k]; ++i) {
      const int32_t t = tok[k * kBitProgMax + i];
      if (t < 0) continue;
      int p = 0;
      while (p < nu && u[p] != t) ++p;
      if (p == nu) {
        if (nu == 4) {
          job.nu = 0;
          return;
        }
        u[nu++] = t;
      }
    }
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < lens[k]; ++i) {
      int32_t& t = tok[k * kBitProgMax + i];
      if (t < 0) continue;
      int p = 0;
      while (u[p] != t) ++p;
      t = p;
    }
  job.nu = nu;
  for (int p = 0; p < 4; ++p) job.uleaf[p] = p < nu ? u[p] : 0;
}

BitJob make_bit_job(const uint32_t* bm, int64_t words, int64_t num_docs, int64_t first_block, const int32_t* tok,
                    int32_t len_a, int32_t len_b, uint32_t* scratch, int64_t* out) {
  BitJob j{};
  j.bm = bm;
  j.words = words;
  j.num_docs = num_docs;
  j.first_block = first_block;
  j.nb = bit_count_blocks(num_docs);
  j.tok = tok;
  j.len_a = len_a;
  j.len_b = len_b;
  j.scratch = scratch;
  // the partial counts after block_last / block_in, 8-byte aligned (bit_count_scratch_words: 10 words per workgroup)
  j.part = scratch ? (unsigned long long*)(((uintptr_t)(scratch + 2 * j.nb) + 7) & ~(uintptr_t)7) : nullptr;
  j.out = (unsigned long long*)out;
  return j;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int64_t pa_bitmap_counts_scratch_bytes(int64_t words) {
  if (words < 0) return fail(PA_EINVAL, "negative word count");
  return (int64_t)(align256(4 * (size_t)bit_count_scratch_words(words)) + align256(4 * (size_t)bit_count_blocks(32 * words)) +
                   align256(sizeof(BitJob)) + kBitTokBytes);
}

int pa_bitmap_counts(const uint32_t* device_bitmaps, int64_t words, int32_t num_leaves, int64_t num_docs,
                     const int32_t* prog_a, int32_t len_a, const int32_t* prog_b, int32_t len_b, void* device_scratch,
                     int64_t* device_out, void* stream) {
  if (!device_out || num_docs < 0 || words < (num_docs + 31) / 32 || words % 4 != 0)
    return fail(PA_EINVAL, "bad bitmap counts arguments (words: a multiple of 4 covering num_docs)");
  if (num_docs > 0 && !device_bitmaps) return fail(PA_EINVAL, "null bitmaps");
  struct {
    BitJob job;
    int32_t tok[2 * kBitProgMax];
  } h{};
  int rc = check_bit_prog(prog_a, len_a, num_leaves, true, h.tok);
  if (!rc) rc = check_bit_prog(prog_b, len_b, num_leaves, false, h.tok + kBitProgMax);
  if (rc) return rc;
  if (num_docs == 0) return PA_OK;
  if (!device_scratch) return fail(PA_EINVAL, "null scratch");
  char* sc = (char*)device_scratch;
  const size_t off_table = align256(4 * (size_t)bit_count_scratch_words(words));
  const size_t off_job = off_table + align256(4 * (size_t)bit_count_blocks(32 * words));
  const size_t off_tok = off_job + align256(sizeof(BitJob));
  h.job = make_bit_job(device_bitmaps, words, num_docs, 0, (const int32_t*)(sc + off_tok), len_a, len_b,
                       (uint32_t*)sc, device_out);
  renumber_leaves(h.job, h.tok);
  hipStream_t st = (hipStream_t)stream;
  PA_HIP(hipMemcpyAsync(sc + off_job, &h.job, sizeof(BitJob), hipMemcpyHostToDevice, st));
  PA_HIP(hipMemcpyAsync(sc + off_tok, h.tok, kBitTokBytes, hipMemcpyHostToDevice, st));
  PA_HIP(launch_bit_counts_batch((const BitJob*)(sc + off_job), 1, h.job.nb, len_b > 0, (int32_t*)(sc + off_table), st));
  PA_HIP(hipStreamSynchronize(st));  // (the host staging above is on this stack frame)
  return PA_OK;
}

int pa_query_filter_counts(pa_query* q, int32_t num_requests, const int32_t* segments, const int32_t* programs,
                           const int32_t* lengths, int64_t* out, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (num_requests < 0 || (num_requests > 0 && (!segments || !programs || !lengths || !out)))
    return fail(PA_EINVAL, "bad filter counts arguments");
  if (num_requests == 0) return PA_OK;
  const int nl = q->spec.num_leaves;
  std::vector<int> leaf_lit(nl, -1);
  for (int l = 0; l < nl; ++l) {
    for (size_t i = 0; i < q->literals.size() && leaf_lit[l] < 0; ++i)
      if (q->literals[i].leaf == l) leaf_lit[l] = (int)i;
    if (leaf_lit[l] < 0) return fail(PA_EUNSUPPORTED, "filter leaf " + std::to_string(l) + " has no literal in the plan");
  }
  // device layout: leaf bitmaps of every requested segment | per-request scratch | counts | jobs | leaf jobs | tokens
  std::vector<int64_t> bm_off(q->nseg, -1);
  size_t bm_words = 0;
  for (int r = 0; r < num_requests; ++r) {
    const int si = segments[r];
    if (si < 0 || si >= q->nseg) return fail(PA_EINVAL, "request names a segment out of range");
    if (bm_off[si] < 0) {
      bm_off[si] = (int64_t)bm_words;
      bm_words += (size_t)nl * (size_t)leaf_words(q->segs[si]->num_docs);
    }
  }
  std::vector<int64_t> sc_off(num_requests);
  size_t sc_words = 0;
  std::vector<BitJob> jobs(num_requests);
  std::vector<int32_t> tok((size_t)num_requests * 2 * kBitProgMax, 0);
  bool any_b = false;
  int64_t blocks = 0;
  for (int r = 0; r < num_requests; ++r) {
    int32_t* t = tok.data() + (size_t)r * 2 * kBitProgMax;
    const int la = lengths[2 * r], lb = lengths[2 * r + 1];
    int rc = check_bit_prog(programs + (size_t)r * 2 * kBitProgMax, la, nl, true, t);
    if (!rc) rc = check_bit_prog(programs + (size_t)r * 2 * kBitProgMax + kBitProgMax, lb, nl, false, t + kBitProgMax);
    if (rc) return rc;
    any_b |= lb > 0;
    const int64_t n = q->segs[segments[r]]->num_docs;
    const int64_t words = leaf_words(n);
    sc_off[r] = (int64_t)sc_words;
    sc_words += (size_t)bit_count_scratch_words(words);
    jobs[r] = make_bit_job(nullptr, words, n, blocks, nullptr, la, lb, nullptr, nullptr);
    renumber_leaves(jobs[r], t);
    blocks += jobs[r].nb;
  }
  std::vector<LeafJob> ljobs;
  int64_t lblocks = 0;
  for (int si = 0; si < q->nseg; ++si) {
    if (bm_off[si] < 0 || q->segs[si]->num_docs == 0) continue;
    const int64_t n = q->segs[si]->num_docs, words = leaf_words(n);
    for (int l = 0; l < nl; ++l) {
      ljobs.push_back(LeafJob{(const DevSeg*)q->dsegs.p + si, nullptr, n, lblocks, leaf_lit[l],
                              q->literals[leaf_lit[l]].neg ? 1 : 0});
      ljobs.back().out = (uint32_t*)(intptr_t)(bm_off[si] + (int64_t)l * words);  // (word offset; rebased below)
      lblocks += leaf_bitmap_blocks(n);
    }
  }
  const size_t o_bm = 0, o_sc = align256(4 * bm_words), o_out = o_sc + align256(4 * sc_words),
               o_jobs = o_out + align256(32 * (size_t)num_requests),
               o_ljobs = o_jobs + align256(sizeof(BitJob) * num_requests),
               o_tok = o_ljobs + align256(sizeof(LeafJob) * std::max<size_t>(1, ljobs.size())),
               o_table = o_tok + align256(4 * tok.size()), total = o_table + 4 * (size_t)std::max<int64_t>(1, blocks);
  if (q->stat_buf.n < total) {
    dev_free(q->stat_buf);
    int rc = dev_alloc(q->stat_buf, total);
    if (rc) return rc;
  }
  char* base = (char*)q->stat_buf.p;
  for (int r = 0; r < num_requests; ++r) {
    jobs[r].bm = (const uint32_t*)(base + o_bm) + bm_off[segments[r]];
    jobs[r].tok = (const int32_t*)(base + o_tok) + (size_t)r * 2 * kBitProgMax;
    jobs[r].scratch = (uint32_t*)(base + o_sc) + sc_off[r];
    jobs[r].part = (unsigned long long*)(((uintptr_t)(jobs[r].scratch + 2 * jobs[r].nb) + 7) & ~(uintptr_t)7);
    jobs[r].out = (unsigned long long*)(base + o_out) + 4 * (size_t)r;
  }
  for (LeafJob& lj : ljobs) lj.out = (uint32_t*)(base + o_bm) + (intptr_t)lj.out;
  hipStream_t st = (hipStream_t)stream;
  PA_HIP(hipMemcpyAsync(base + o_jobs, jobs.data(), sizeof(BitJob) * num_requests, hipMemcpyHostToDevice, st));
  if (!ljobs.empty())
    PA_HIP(hipMemcpyAsync(base + o_ljobs, ljobs.data(), sizeof(LeafJob) * ljobs.size(), hipMemcpyHostToDevice, st));
  PA_HIP(hipMemcpyAsync(base + o_tok, tok.data(), 4 * tok.size(), hipMemcpyHostToDevice, st));
  PA_HIP(hipMemsetAsync(base + o_out, 0, 32 * (size_t)num_requests, st));
  PA_HIP(launch_leaf_bitmaps_batch((const LeafJob*)(base + o_ljobs), (int)ljobs.size(), lblocks, st));
  PA_HIP(launch_bit_counts_batch((const BitJob*)(base + o_jobs), num_requests, blocks, any_b,
                                 (int32_t*)(base + o_table), st));
  PA_HIP(hipMemcpyAsync(out, base + o_out, 32 * (size_t)num_requests, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  return PA_OK;
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
int32_t pa_query_count_free_emit(const pa_query* q) { return q && q->prepared ? (q->pve.fn ? (q->pvh.fn ? 2 : 1) : 0) : -1; }
int32_t pa_query_dense_packed(const pa_query* q) {
  return q && q->prepared ? (q->dense_packed ? (q->jit_fn ? 2 : 1) : 0) : -1;
}

int32_t pa_query_column_staged(const pa_query* q, int32_t column_id) {
  if (!q || !q->prepared || q->nseg == 0) return -1;
  for (size_t sl = 0; sl < q->slot_cols.size(); ++sl)
    if (q->slot_cols[sl] == column_id) return q->hsegs[0].cols[sl].lds_off >= 0 ? 1 : 0;
  return -1;
}

int64_t pa_query_matched_docs(const pa_query* q) { return q && q->prepared ? q->last_matched : -1; }

// ---------------------------------------------------------------- cross-GPU merge of hashed key spaces
// The row layout of a hashed block: every per-key section (numDocsScanned counters excluded) in section order.
static int row_desc(const pa_query* q, RowDesc& d) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (!q->hashed || q->keys_section < 0) return fail(PA_EINVAL, "row merge needs a hashed key space");
  std::memset(&d, 0, sizeof(d));
  int64_t off = 0;
  for (const Section& sc : q->sections) {
    if (sc.kind == PA_ACC_DOCS_U64) continue;
    if (d.nsec >= kMaxRowSecs) return fail(PA_EINVAL, "internal: too many sections for a row");
    RowSec& r = d.sec[d.nsec++];
    switch (sc.kind) {
      case PA_ACC_SUM_F64: r.op = ROW_ADD_F64; break;
      case PA_ACC_MIN_I64: r.op = ROW_MIN_I64; break;
      case PA_ACC_MAX_I64: r.op = ROW_MAX_I64; break;
      case PA_ACC_HLL_U8: case PA_ACC_PRESENCE_U8: r.op = ROW_MAX_U8; break;
      case PA_ACC_KEYS_I64: r.op = ROW_KEY; break;
      default: r.op = ROW_ADD_U64; break;  // COUNT, SUM (int64 and the exact lo / hi pair)
    }
    r.slot_bytes = sc.n / q->num_keys * (int64_t)section_es(sc.kind);
    if (r.slot_bytes % 8) return fail(PA_EINVAL, "internal: row section not a multiple of 8 bytes");
    r.row_off = off;
    r.base = sc.ptr;
    if (sc.kind == PA_ACC_KEYS_I64) {
      d.key_off = off;
      d.keys = (long long*)sc.ptr;
    }
    if (sc.kind == PA_ACC_COUNT_U64) d.count = (const unsigned long long*)sc.ptr;
    off += r.slot_bytes;
  }
  d.row_bytes = off;
  d.num_slots = q->num_keys;
  d.ht_mask = q->ht_slots - 1;
  d.key_words = q->key_words;
  return PA_OK;
}

static int merge_scratch(pa_query* q, size_t bytes) {
  if (q->merge_buf.n >= bytes) return PA_OK;
  dev_free(q->merge_buf);
  return dev_alloc(q->merge_buf, bytes);
}

int64_t pa_query_row_bytes(const pa_query* q) {
  RowDesc d;
  const int rc = row_desc(q, d);
  return rc ? rc : d.row_bytes;
}

int pa_query_pack_rows(pa_query* q, int32_t world, void* device_rows, int64_t* counts, void* stream) {
  RowDesc d;
  int rc = row_desc(q, d);
  if (rc) return rc;
  if (world < 1 || world > 1024 || !counts) return fail(PA_EINVAL, "pack rows: bad world size or null counts");
  hipStream_t st = (hipStream_t)stream;
  // scratch: counts[world], cursor[world], row_slot[num_slots]
  rc = merge_scratch(q, (size_t)(2 * world + d.num_slots) * 8);
  if (rc) return rc;
  unsigned long long* cnt = (unsigned long long*)q->merge_buf.p;
  unsigned long long* cur = cnt + world;
  int64_t* row_slot = (int64_t*)(cur + world);
  PA_HIP(hipMemsetAsync(cnt, 0, (size_t)world * 8, st));
  PA_HIP(launch_pack_index(d, world, 0, cnt, nullptr, nullptr, st));
  std::vector<unsigned long long> h(world);
  PA_HIP(hipMemcpyAsync(h.data(), cnt, (size_t)world * 8, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  int64_t total = 0;
  std::vector<unsigned long long> start(world);
  for (int r = 0; r < world; ++r) {
    counts[r] = (int64_t)h[r];
    start[r] = (unsigned long long)total;
    total += (int64_t)h[r];
  }
  if (!device_rows || total == 0) return PA_OK;
  PA_HIP(hipMemcpyAsync(cur, start.data(), (size_t)world * 8, hipMemcpyHostToDevice, st));
  PA_HIP(launch_pack_index(d, world, 1, nullptr, cur, row_slot, st));
  PA_HIP(launch_pack_copy(d, row_slot, total, (unsigned char*)device_rows, st));
  PA_HIP(hipStreamSynchronize(st));
  return PA_OK;
}

int pa_query_merge_rows(pa_query* q, const void* device_rows, int64_t num_rows, int64_t* groups, int64_t* overflow,
                        void* stream) {
  RowDesc d;
  int rc = row_desc(q, d);
  if (rc) return rc;
  if (num_rows < 0 || (num_rows > 0 && !device_rows)) return fail(PA_EINVAL, "merge rows: bad rows");
  hipStream_t st = (hipStream_t)stream;
  rc = merge_scratch(q, (size_t)(8 + std::max<int64_t>(num_rows, d.num_slots)) * 8);
  if (rc) return rc;
  unsigned long long* ctr = (unsigned long long*)q->merge_buf.p;
  int64_t* row_slot = (int64_t*)(ctr + 8);
  // the block is reset except its numDocsScanned counters, which stay this rank's (the broker sums them)
  void* docs = q->sections.back().ptr;
  PA_HIP(hipMemcpyAsync(ctr + 4, docs, 32, hipMemcpyDeviceToDevice, st));
  rc = pa_query_reset(q, stream);
  if (rc) return rc;
  PA_HIP(hipMemcpyAsync(docs, ctr + 4, 32, hipMemcpyDeviceToDevice, st));
  PA_HIP(hipMemsetAsync(ctr, 0, 32, st));
  PA_HIP(launch_merge_rows(d, (const unsigned char*)device_rows, num_rows, row_slot, ctr, st));
  unsigned long long h[4];
  PA_HIP(hipMemcpyAsync(h, ctr, 32, hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  if (groups) *groups = (int64_t)h[0];
  if (overflow) *overflow = (int64_t)h[1];
  return PA_OK;
}

int32_t pa_query_leap_leaf(const pa_query* q) { return q && q->prepared ? q->leap_leaf : -1; }

// the neighbour searches of the E docs the last scan listed (once per scan)
static int leap_search_pending(pa_query* q, hipStream_t st) {
  if (q->hq.leap_mode && !q->leap_searched) {
    PA_HIP(launch_leap_search((const DevQuery*)q->dq.p, (const DevSeg*)q->dsegs.p, q->leap_slices, st));
    q->leap_searched = true;
  }
  return PA_OK;
}

int pa_query_leap_counts(pa_query* q, int64_t* out, void* stream) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (q->leap_leaf < 0) return fail(PA_EINVAL, "the scan does not count the filter statistics (pa_query_leap_leaf)");
  if (!out) return fail(PA_EINVAL, "null output");
  hipStream_t st = (hipStream_t)stream;
  int rc = leap_search_pending(q, st);
  if (rc) return rc;
  std::vector<int64_t> h((size_t)q->nseg * 3 + 1);
  PA_HIP(hipMemcpyAsync(h.data(), q->leap_buf.p, h.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  PA_HIP(hipStreamSynchronize(st));
  const bool overflow = h[(size_t)q->nseg * 3] != 0;  // (a wave's E-doc slice was full: no segment's leaps are known)
  for (int si = 0; si < q->nseg; ++si) {
    out[3 * si] = h[3 * si];
    out[3 * si + 1] = h[3 * si + 1];
    out[3 * si + 2] = (h[3 * si + 2] || overflow) ? 1 : 0;
  }
  return PA_OK;
}

// ---------------------------------------------------------------- execution statistics (pa_query_execution_stats)
// The host's per-segment filter operator trees, reduced as the reference's iterators read them when the projection
// drives the tree's iterator to the end (BlockDocIdSet.iterator() construction + next() until EOF):
//   * a scan driven by next() reads every entry: num_docs, or a multi-value column's values;
//   * OR: OrDocIdIterator drives every child with next() to its end: the children's costs add;
//   * NOT: NotDocIdIterator drives its child with next() to the end and once more: for a leap-frogging AND that call
//     re-runs the chain after its last match (pa_stats.hip "tail");
//   * AND (AndDocIdSet.java:72-186): with index children (sorted / bitmap doc sets) and scan children, or several index
//     children, the index doc sets intersect and each scan's applyAnd reads the docs surviving so far (a popcount of the
//     chain, a value count for a multi-value column); what is left (OR / NOT children) leap-frogs with that doc set
//     first; otherwise every child leap-frogs (AndDocIdIterator), counted on the GPU (pa_stats.hip).
}  // extern "C"

namespace stats {
struct Elem {  // one child iterator of a leap-frog
  int32_t kind = LF_DOCS;
  std::vector<int32_t> prog;
  int32_t mv = -1;
  std::vector<Elem> subs;  // LF_OR: its children (LF_DOCS / LF_SCAN)
};
struct Leap {
  std::vector<Elem> el;
  bool tail = false;
};
struct Plan {
  int64_t cnst = 0;
  std::vector<std::pair<std::vector<int32_t>, int32_t>> counts;  // (doc set, multi-value column or -1)
  std::vector<Leap> leaps;
};
struct Unsupported {};
struct Ctx {
  const pa_query* q;
  int si;
  const pa_filter_op* ops;
  int nops;
  Plan* P;
};

std::vector<int32_t> prog_of(const pa_filter_op& o) { return std::vector<int32_t>(o.prog, o.prog + o.prog_len); }
std::vector<int32_t> prog_join(const std::vector<int32_t>& a, const std::vector<int32_t>& b, int32_t op) {
  if (a.empty()) return b;
  std::vector<int32_t> r(a);
  r.insert(r.end(), b.begin(), b.end());
  r.push_back(op);
  return r;
}

// index after the subtree at i (pre-order), or -1 when malformed
int extent(const pa_filter_op* ops, int nops, int i, int depth = 0) {
  if (i < 0 || i >= nops || depth > 64) return -1;
  int j = i + 1;
  for (int c = 0; c < ops[i].num_children; ++c) {
    j = extent(ops, nops, j, depth + 1);
    if (j < 0) return -1;
  }
  return j;
}
std::vector<int> children(const Ctx& x, int i) {
  std::vector<int> r;
  int j = i + 1;
  for (int c = 0; c < x.ops[i].num_children; ++c) {
    r.push_back(j);
    j = extent(x.ops, x.nops, j);
  }
  return r;
}

const Column* mv_col(const Ctx& x, int32_t col) {
  auto it = x.q->segs[x.si]->cols.find(col);
  if (it == x.q->segs[x.si]->cols.end() || it->second->kind != COL_MV_DICT) throw Unsupported{};
  return it->second;
}

int64_t cost_next(const Ctx& x, int i, bool tail);

// an OR's iterator (OrDocIdSet.java:63-127): more than one sorted child merge into one doc set; nullptr-like result
// (kind LF_DOCS) when that is all of it
bool and_docs_form(const Ctx& x, int i, std::vector<int32_t>* docs);
Elem or_elem(const Ctx& x, int i) {
  Elem e;
  e.kind = LF_OR;
  std::vector<int> kids = children(x, i);
  int nsorted = 0;
  for (int k : kids) nsorted += x.ops[k].kind == PA_FOP_SORTED;
  std::vector<int32_t> merged;
  for (int k : kids) {
    const pa_filter_op& o = x.ops[k];
    if (o.kind == PA_FOP_SORTED && nsorted > 1) {
      merged = prog_join(merged, prog_of(o), PA_BIT_OR);
      continue;
    }
    Elem s;
    std::vector<int32_t> d;
    if (o.kind == PA_FOP_SORTED || o.kind == PA_FOP_BITMAP) {
      s.kind = LF_DOCS;
      s.prog = prog_of(o);
    } else if (o.kind == PA_FOP_SCAN) {
      s.kind = LF_SCAN;
      s.prog = prog_of(o);
      if (o.mv_column >= 0) {
        mv_col(x, o.mv_column);
        s.mv = o.mv_column;
      }
    } else if (o.kind == PA_FOP_AND && and_docs_form(x, k, &d)) {
      s.kind = LF_DOCS;  // (its applyAnd reads are counted at construction)
      s.prog = d;
    } else {
      throw Unsupported{};  // an AND / NOT iterator advanced inside an OR inside a leap-frog
    }
    e.subs.push_back(s);
  }
  if (!merged.empty()) {
    Elem s;
    s.kind = LF_DOCS;
    s.prog = merged;
    e.subs.insert(e.subs.begin(), s);
  }
  for (const Elem& s : e.subs) e.prog = prog_join(e.prog, s.prog, PA_BIT_OR);
  if (kids.size() == (size_t)nsorted) {  // every child sorted: one merged doc set
    e.kind = LF_DOCS;
    e.subs.clear();
  }
  return e;
}

// the AND's iterator construction (AndDocIdSet.iterator): applyAnd counts into the plan; returns the leap-frog list
// (empty when the iterator is the merged doc set) and the AND's doc set in *docs
std::vector<Elem> and_build(const Ctx& x, int i, std::vector<int32_t>* docs) {
  std::vector<int> kids = children(x, i);
  std::vector<int> sorted, bitmaps, scans, rest;
  for (int k : kids) {
    const int kd = x.ops[k].kind;
    if (kd == PA_FOP_SORTED) sorted.push_back(k);
    else if (kd == PA_FOP_BITMAP) bitmaps.push_back(k);
    else if (kd == PA_FOP_SCAN) scans.push_back(k);
    else if (kd == PA_FOP_OR) {
      // an OR of sorted children only is one merged (bitmap) doc set
      bool all_sorted = true;
      for (int c : children(x, k)) all_sorted &= x.ops[c].kind == PA_FOP_SORTED;
      if (all_sorted) bitmaps.push_back(k);
      else rest.push_back(k);
    } else {
      rest.push_back(k);
    }
  }
  auto doc_prog = [&](int k) {
    if (x.ops[k].kind != PA_FOP_OR) return prog_of(x.ops[k]);
    std::vector<int32_t> p;
    for (int c : children(x, k)) p = prog_join(p, prog_of(x.ops[c]), PA_BIT_OR);
    return p;
  };
  std::vector<Elem> out;
  docs->clear();
  const size_t nindex = sorted.size() + bitmaps.size();
  if ((nindex > 0 && !scans.empty()) || nindex > 1) {
    std::vector<int32_t> D;
    for (int k : sorted) D = prog_join(D, doc_prog(k), PA_BIT_AND);
    for (int k : bitmaps) D = prog_join(D, doc_prog(k), PA_BIT_AND);
    for (int k : scans) {
      const pa_filter_op& o = x.ops[k];
      if (o.mv_column >= 0) mv_col(x, o.mv_column);
      x.P->counts.push_back({D, o.mv_column});
      D = prog_join(D, prog_of(o), PA_BIT_AND);
    }
    if (rest.empty()) {
      *docs = D;
      return out;
    }
    Elem m;
    m.kind = LF_DOCS;
    m.prog = D;
    out.push_back(m);
    kids = rest;
  }
  for (int k : kids) {
    const pa_filter_op& o = x.ops[k];
    Elem e;
    if (o.kind == PA_FOP_SORTED || o.kind == PA_FOP_BITMAP) {
      e.kind = LF_DOCS;
      e.prog = prog_of(o);
    } else if (o.kind == PA_FOP_SCAN) {
      e.kind = LF_SCAN;
      e.prog = prog_of(o);
      if (o.mv_column >= 0) {
        mv_col(x, o.mv_column);
        e.mv = o.mv_column;
      }
    } else if (o.kind == PA_FOP_OR) {
      e = or_elem(x, k);  // (an AND child's iterator is built there: its applyAnd reads)
    } else {
      throw Unsupported{};  // a NOT iterator leap-frogged (next() and advance() mixed on its child)
    }
    out.push_back(e);
  }
  for (const Elem& e : out) *docs = prog_join(*docs, e.prog, PA_BIT_AND);
  return out;
}

bool and_docs_form(const Ctx& x, int i, std::vector<int32_t>* docs) {
  Plan saved = *x.P;
  std::vector<Elem> el = and_build(x, i, docs);
  if (!el.empty()) {
    *x.P = saved;
    return false;
  }
  return true;
}

int64_t cost_next(const Ctx& x, int i, bool tail) {
  const pa_filter_op& o = x.ops[i];
  switch (o.kind) {
    case PA_FOP_EMPTY: case PA_FOP_MATCH_ALL: case PA_FOP_SORTED: case PA_FOP_BITMAP:
      return 0;
    case PA_FOP_SCAN:
      return o.mv_column >= 0 ? mv_col(x, o.mv_column)->total_values : (int64_t)x.q->segs[x.si]->num_docs;
    case PA_FOP_OR: {
      int64_t c = 0;
      for (int k : children(x, i)) c += cost_next(x, k, false);
      return c;
    }
    case PA_FOP_NOT:
      return cost_next(x, i + 1, true);
    case PA_FOP_AND: {
      std::vector<int32_t> d;
      std::vector<Elem> el = and_build(x, i, &d);
      if (el.empty()) return 0;
      size_t nsub = 0;
      for (const Elem& e : el) nsub += e.subs.size();
      if (el.size() > (size_t)kLfMaxK || nsub > (size_t)kLfMaxSub) throw Unsupported{};
      // NotDocIdIterator's extra next(): with an OR child the re-run starts from the OR children's cached answers (a
      // different chain from the first run's last one): not counted here
      if (tail && nsub > 0) throw Unsupported{};
      x.P->leaps.push_back(Leap{el, tail});
      return 0;
    }
  }
  throw Unsupported{};
}

int check_tree(const pa_filter_op* ops, int nops, int root, int num_leaves) {
  const int end = extent(ops, nops, root);
  if (end < 0) return fail(PA_EINVAL, "execution stats: malformed operator tree");
  for (int i = root; i < end; ++i) {
    const pa_filter_op& o = ops[i];
    const bool leaf = o.kind == PA_FOP_SORTED || o.kind == PA_FOP_BITMAP || o.kind == PA_FOP_SCAN;
    if (o.kind < PA_FOP_EMPTY || o.kind > PA_FOP_NOT) return fail(PA_EINVAL, "execution stats: unknown operator kind");
    if ((o.kind == PA_FOP_AND || o.kind == PA_FOP_OR) && o.num_children < 2)
      return fail(PA_EINVAL, "execution stats: AND / OR needs two children");
    if (o.kind == PA_FOP_NOT && o.num_children != 1) return fail(PA_EINVAL, "execution stats: NOT needs one child");
    if ((leaf || o.kind == PA_FOP_EMPTY || o.kind == PA_FOP_MATCH_ALL) && o.num_children != 0)
      return fail(PA_EINVAL, "execution stats: a leaf operator has children");
    if (leaf) {
      int32_t tok[kBitProgMax];
      int rc = check_bit_prog(o.prog, o.prog_len, num_leaves, true, tok);
      if (rc) return rc;
    }
  }
  return PA_OK;
}
}  // namespace stats

extern "C" {

int pa_query_execution_stats(pa_query* q, int32_t num_ops, const pa_filter_op* ops, int32_t num_trees,
                             const int32_t* tree_root, const int32_t* segment_tree, int32_t projected_columns,
                             int64_t docs_scanned, int64_t* out, int64_t* segment_in_filter, void* stream) {
  using namespace stats;
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (!out || num_ops < 0 || num_trees < 0 || projected_columns < 0 || (num_ops > 0 && !ops) ||
      (num_trees > 0 && !tree_root) || (q->nseg > 0 && !segment_tree))
    return fail(PA_EINVAL, "bad execution stats arguments");
  const int nl = q->spec.num_leaves;
  for (int t = 0; t < num_trees; ++t) {
    int rc = check_tree(ops, num_ops, tree_root[t], nl);
    if (rc) return rc;
  }
  hipStream_t st = (hipStream_t)stream;
  if (docs_scanned < 0 && !q->scanned_since_fetch) docs_scanned = q->last_matched;
  if (docs_scanned < 0) {  // numDocsScanned of the last scan, from its counter (no fetch since the scan)
    unsigned long long d = 0;
    PA_HIP(hipMemcpyAsync(&d, q->sections.back().ptr, 8, hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    docs_scanned = (int64_t)d;
  }
  // the scan's own counts of a two-scan AND (fused statistics)
  std::vector<int64_t> fused;
  if (q->leap_leaf >= 0) {
    fused.resize((size_t)q->nseg * 3);
    int rc = pa_query_leap_counts(q, fused.data(), stream);
    if (rc) return rc;
  }
  std::vector<Plan> plans(q->nseg);
  std::vector<int> state(q->nseg, 0);  // 0: plan, 1: constant known (fused / non-scan), -1: host
  std::vector<int64_t> seg_in(q->nseg, 0);
  int64_t non_scan_docs = 0;
  for (int si = 0; si < q->nseg; ++si) {
    const int t = segment_tree[si];
    const int64_t n = q->segs[si]->num_docs;
    if (t == PA_STATS_NON_SCAN) {
      non_scan_docs += n;
      state[si] = 1;
      continue;
    }
    if (t == PA_STATS_HOST) {
      state[si] = -1;
      continue;
    }
    if (t < 0 || t >= num_trees) return fail(PA_EINVAL, "execution stats: segment tree index out of range");
    const int root = tree_root[t];
    const pa_filter_op& r = ops[root];
    if (!fused.empty() && !fused[3 * si + 2] && r.kind == PA_FOP_AND && r.num_children == 2) {
      // AND(Z scan, E scan) counted by the scan: n + |Z & E| + leaps (the leap-frog's reads telescope)
      const pa_filter_op& a = ops[root + 1];
      const pa_filter_op& b = ops[root + 2];
      if (a.kind == PA_FOP_SCAN && b.kind == PA_FOP_SCAN && a.mv_column < 0 && b.mv_column < 0 && a.prog_len == 1 &&
          b.prog_len == 1 && b.prog[0] == q->leap_leaf && a.prog[0] == 1 - q->leap_leaf) {
        seg_in[si] = n + fused[3 * si] + fused[3 * si + 1];
        state[si] = 1;
        continue;
      }
    }
    Ctx x{q, si, ops, num_ops, &plans[si]};
    try {
      seg_in[si] = cost_next(x, root, false);
    } catch (const Unsupported&) {
      plans[si] = Plan{};
      state[si] = -1;
    }
  }
  // GPU work: leaf bitmaps of the segments with counts or leap-frogs, their element masks, the counts, the leap-frogs
  std::vector<int> leaf_lit(nl, -1);
  for (int l = 0; l < nl; ++l) {
    for (size_t i = 0; i < q->literals.size() && leaf_lit[l] < 0; ++i)
      if (q->literals[i].leaf == l) leaf_lit[l] = (int)i;
  }
  std::map<std::pair<int, std::vector<int32_t>>, int> mask_id;
  std::vector<std::pair<int, std::vector<int32_t>>> masks;
  auto mask_of = [&](int si, const std::vector<int32_t>& p) {
    auto key = std::make_pair(si, p);
    auto it = mask_id.find(key);
    if (it != mask_id.end()) return it->second;
    const int id = (int)masks.size();
    mask_id.emplace(key, id);
    masks.push_back(key);
    return id;
  };
  struct CountReq { int si, mask; int32_t mv; };
  struct LeapReq { int si; const Leap* lp; };
  std::vector<CountReq> creq;
  std::vector<LeapReq> lreq, breq;  // breq: two single-value scans leap-frogged (closed form over label counts)
  std::vector<char> seg_bm(q->nseg, 0);
  for (int si = 0; si < q->nseg; ++si) {
    if (state[si] != 0) continue;
    for (const auto& c : plans[si].counts) creq.push_back(CountReq{si, mask_of(si, c.first), c.second});
    for (const Leap& lp : plans[si].leaps) {
      if (lp.el.size() == 2 && !lp.tail && lp.el[0].kind == LF_SCAN && lp.el[1].kind == LF_SCAN && lp.el[0].mv < 0 &&
          lp.el[1].mv < 0 && (int)lp.el[0].prog.size() <= kBitProgMax && (int)lp.el[1].prog.size() <= kBitProgMax) {
        // AndDocIdIterator over two SVScanDocIdIterators reads num_docs + |A & B| + leaps (pa_kernels.hip word_leaps)
        breq.push_back(LeapReq{si, &lp});
        seg_bm[si] = 1;
        continue;
      }
      for (const Elem& e : lp.el) {
        mask_of(si, e.prog);
        for (const Elem& s : e.subs) mask_of(si, s.prog);
      }
      lreq.push_back(LeapReq{si, &lp});
    }
  }
  for (const auto& m : masks) seg_bm[m.first] = 1;
  int gpu_segs = 0;
  if (!masks.empty() || !breq.empty()) {
    for (int l = 0; l < nl; ++l)
      if (leaf_lit[l] < 0) return fail(PA_EUNSUPPORTED, "filter leaf " + std::to_string(l) + " has no literal in the plan");
    std::vector<int64_t> bm_off(q->nseg, -1);
    size_t bm_words = 0;
    for (int si = 0; si < q->nseg; ++si)
      if (seg_bm[si]) {
        bm_off[si] = (int64_t)bm_words;
        bm_words += (size_t)nl * (size_t)leaf_words(q->segs[si]->num_docs);
        ++gpu_segs;
      }
    // the two-scan leap-frogs: pa_bitmap_counts' jobs (programs A, B over the segment's leaf bitmaps)
    std::vector<BitJob> bjobs(breq.size());
    std::vector<int32_t> btok(breq.size() * 2 * kBitProgMax, 0);
    std::vector<size_t> bsc(breq.size());
    size_t bsc_words = 0;
    int64_t bblocks = 0;
    for (size_t r = 0; r < breq.size(); ++r) {
      const Leap& lp = *breq[r].lp;
      const int64_t n = q->segs[breq[r].si]->num_docs, words = leaf_words(n);
      int32_t* t = btok.data() + r * 2 * kBitProgMax;
      const int la = (int)lp.el[0].prog.size(), lb = (int)lp.el[1].prog.size();
      std::copy(lp.el[0].prog.begin(), lp.el[0].prog.end(), t);
      std::copy(lp.el[1].prog.begin(), lp.el[1].prog.end(), t + kBitProgMax);
      bsc[r] = bsc_words;
      bsc_words += (size_t)bit_count_scratch_words(words) + 2;
      bjobs[r] = make_bit_job(nullptr, words, n, bblocks, nullptr, la, lb, nullptr, nullptr);
      renumber_leaves(bjobs[r], t);
      bblocks += bjobs[r].nb;
    }
    std::vector<int64_t> mk_off(masks.size());
    size_t mk_words = 0;
    std::vector<int32_t> toks;
    std::vector<StatMaskJob> mjobs(masks.size());
    int64_t mblocks = 0;
    for (size_t m = 0; m < masks.size(); ++m) {
      const int si = masks[m].first;
      const int64_t words = leaf_words(q->segs[si]->num_docs);
      mk_off[m] = (int64_t)mk_words;
      mk_words += (size_t)words;
      int depth = 0, maxd = 0;
      for (int32_t t : masks[m].second) {
        if (t >= 0) maxd = std::max(maxd, ++depth);
        else if (t != PA_BIT_NOT) --depth;
      }
      if (maxd > kBitProgStack) return fail(PA_EUNSUPPORTED, "execution stats: doc-set program too deep");
      StatMaskJob& j = mjobs[m];
      j = StatMaskJob{};
      j.words = words;
      j.num_docs = q->segs[si]->num_docs;
      j.first_block = mblocks;
      j.tok_off = (int32_t)toks.size();
      j.len = (int32_t)masks[m].second.size();
      toks.insert(toks.end(), masks[m].second.begin(), masks[m].second.end());
      mblocks += stat_mask_blocks(words);
    }
    std::vector<StatCountJob> cjobs(creq.size());
    int64_t cblocks = 0;
    for (size_t r = 0; r < creq.size(); ++r) {
      const int64_t words = leaf_words(q->segs[creq[r].si]->num_docs);
      cjobs[r] = StatCountJob{};
      cjobs[r].words = words;
      cjobs[r].first_block = cblocks;
      cblocks += stat_mask_blocks(words);
    }
    std::vector<LfJob> ljobs(lreq.size());
    int64_t lanes = 0;
    size_t cell_words = 0;
    for (size_t r = 0; r < lreq.size(); ++r) {
      LfJob& j = ljobs[r];
      j = LfJob{};
      const Leap& lp = *lreq[r].lp;
      j.K = (int32_t)lp.el.size();
      j.num_docs = q->segs[lreq[r].si]->num_docs;
      j.nchunks = (j.num_docs + kLfChunkDocs - 1) / kLfChunkDocs;
      int ns = 0;
      for (int e = 0; e < j.K; ++e) {
        j.kind[e] = lp.el[e].kind;
        j.sub_first[e] = ns;
        j.sub_count[e] = (int32_t)lp.el[e].subs.size();
        for (const Elem& s : lp.el[e].subs) j.sub_kind[ns++] = s.kind;
      }
      j.nsub = ns;
      j.cell_words = 4 + 2 * ns;
      j.first_lane = lanes;
      lanes += j.nchunks * (j.K + 1);
      cell_words += (size_t)(j.nchunks * (j.K + 1) * j.cell_words);
    }
    std::vector<LeafJob> leafjobs;
    int64_t lblocks = 0;
    for (int si = 0; si < q->nseg; ++si) {
      if (bm_off[si] < 0 || q->segs[si]->num_docs == 0) continue;
      const int64_t n = q->segs[si]->num_docs, words = leaf_words(n);
      for (int l = 0; l < nl; ++l) {
        leafjobs.push_back(LeafJob{(const DevSeg*)q->dsegs.p + si, nullptr, n, lblocks, leaf_lit[l],
                                   q->literals[leaf_lit[l]].neg ? 1 : 0});
        leafjobs.back().out = (uint32_t*)(intptr_t)(bm_off[si] + (int64_t)l * words);  // (word offset; rebased below)
        lblocks += leaf_bitmap_blocks(n);
      }
    }
    const size_t nres = creq.size() + 3 * lreq.size() + 4 * breq.size();
    const size_t o_bm = 0, o_mk = align256(4 * bm_words), o_cells = o_mk + align256(4 * mk_words),
                 o_res = o_cells + align256(4 * std::max<size_t>(1, cell_words)),
                 o_bsc = o_res + align256(8 * std::max<size_t>(1, nres)),
                 o_bj = o_bsc + align256(4 * std::max<size_t>(1, bsc_words)),
                 o_btok = o_bj + align256(sizeof(BitJob) * std::max<size_t>(1, bjobs.size())),
                 o_btab = o_btok + align256(4 * std::max<size_t>(1, btok.size())),
                 o_mj = o_btab + align256(4 * (size_t)std::max<int64_t>(1, bblocks)),
                 o_cj = o_mj + align256(sizeof(StatMaskJob) * std::max<size_t>(1, mjobs.size())),
                 o_lj = o_cj + align256(sizeof(StatCountJob) * std::max<size_t>(1, cjobs.size())),
                 o_fj = o_lj + align256(sizeof(LfJob) * std::max<size_t>(1, ljobs.size())),
                 o_tok = o_fj + align256(sizeof(LeafJob) * std::max<size_t>(1, leafjobs.size())),
                 total = o_tok + 4 * std::max<size_t>(1, toks.size());
    if (q->stat_buf.n < total) {
      dev_free(q->stat_buf);
      int rc = dev_alloc(q->stat_buf, total);
      if (rc) return rc;
    }
    char* base = (char*)q->stat_buf.p;
    const uint32_t* bm = (const uint32_t*)(base + o_bm);
    uint32_t* mk = (uint32_t*)(base + o_mk);
    unsigned long long* res = (unsigned long long*)(base + o_res);
    for (size_t m = 0; m < masks.size(); ++m) {
      mjobs[m].bm = bm + bm_off[masks[m].first];
      mjobs[m].out = mk + mk_off[m];
    }
    for (size_t r = 0; r < creq.size(); ++r) {
      cjobs[r].mask = mk + mk_off[creq[r].mask];
      cjobs[r].wt = creq[r].mv >= 0 ? (const int32_t*)q->segs[creq[r].si]->cols.at(creq[r].mv)->mv_off.p : nullptr;
      cjobs[r].out = res + r;
    }
    size_t cell_at = 0;
    for (size_t r = 0; r < lreq.size(); ++r) {
      LfJob& j = ljobs[r];
      const int si = lreq[r].si;
      const Leap& lp = *lreq[r].lp;
      int ns = 0;
      for (int e = 0; e < j.K; ++e) {
        const Elem& el = lp.el[e];
        j.emask[e] = mk + mk_off[mask_id.at(std::make_pair(si, el.prog))];
        j.ewt[e] = el.mv >= 0 ? (const int32_t*)q->segs[si]->cols.at(el.mv)->mv_off.p : nullptr;
        for (const Elem& s : el.subs) {
          j.smask[ns] = mk + mk_off[mask_id.at(std::make_pair(si, s.prog))];
          j.swt[ns] = s.mv >= 0 ? (const int32_t*)q->segs[si]->cols.at(s.mv)->mv_off.p : nullptr;
          ++ns;
        }
      }
      j.cells = (uint32_t*)(base + o_cells) + cell_at;
      cell_at += (size_t)(j.nchunks * (j.K + 1) * j.cell_words);
      j.out = res + creq.size() + 3 * r;
    }
    for (LeafJob& lj : leafjobs) lj.out = (uint32_t*)(base + o_bm) + (intptr_t)lj.out;
    const size_t bres = creq.size() + 3 * lreq.size();
    for (size_t r = 0; r < breq.size(); ++r) {
      BitJob& j = bjobs[r];
      j.bm = bm + bm_off[breq[r].si];
      j.tok = (const int32_t*)(base + o_btok) + r * 2 * kBitProgMax;
      j.scratch = (uint32_t*)(base + o_bsc) + bsc[r];
      j.part = (unsigned long long*)(((uintptr_t)(j.scratch + 2 * j.nb) + 7) & ~(uintptr_t)7);
      j.out = res + bres + 4 * r;
    }
    if (!mjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_mj, mjobs.data(), sizeof(StatMaskJob) * mjobs.size(), hipMemcpyHostToDevice, st));
    if (!bjobs.empty()) {
      PA_HIP(hipMemcpyAsync(base + o_bj, bjobs.data(), sizeof(BitJob) * bjobs.size(), hipMemcpyHostToDevice, st));
      PA_HIP(hipMemcpyAsync(base + o_btok, btok.data(), 4 * btok.size(), hipMemcpyHostToDevice, st));
    }
    if (!cjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_cj, cjobs.data(), sizeof(StatCountJob) * cjobs.size(), hipMemcpyHostToDevice, st));
    if (!ljobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_lj, ljobs.data(), sizeof(LfJob) * ljobs.size(), hipMemcpyHostToDevice, st));
    if (!leafjobs.empty())
      PA_HIP(hipMemcpyAsync(base + o_fj, leafjobs.data(), sizeof(LeafJob) * leafjobs.size(), hipMemcpyHostToDevice, st));
    if (!toks.empty()) PA_HIP(hipMemcpyAsync(base + o_tok, toks.data(), 4 * toks.size(), hipMemcpyHostToDevice, st));
    PA_HIP(hipMemsetAsync(res, 0, 8 * std::max<size_t>(1, nres), st));
    if (!leafjobs.empty())
      PA_HIP(launch_leaf_bitmaps_batch((const LeafJob*)(base + o_fj), (int)leafjobs.size(), lblocks, st));
    PA_HIP(launch_stat_masks((const StatMaskJob*)(base + o_mj), (int)mjobs.size(), mblocks,
                             (const int32_t*)(base + o_tok), st));
    PA_HIP(launch_stat_counts((const StatCountJob*)(base + o_cj), (int)cjobs.size(), cblocks, st));
    PA_HIP(launch_leapfrogs((const LfJob*)(base + o_lj), (int)ljobs.size(), lanes, st));
    PA_HIP(launch_bit_counts_batch((const BitJob*)(base + o_bj), (int)bjobs.size(), bblocks, true,
                                   (int32_t*)(base + o_btab), st));
    std::vector<int64_t> h(std::max<size_t>(1, nres));
    PA_HIP(hipMemcpyAsync(h.data(), res, 8 * h.size(), hipMemcpyDeviceToHost, st));
    PA_HIP(hipStreamSynchronize(st));
    for (size_t r = 0; r < creq.size(); ++r) seg_in[creq[r].si] += h[r];
    for (size_t r = 0; r < lreq.size(); ++r)
      seg_in[lreq[r].si] += h[creq.size() + 3 * r] + (lreq[r].lp->tail ? h[creq.size() + 3 * r + 1] : 0);
    for (size_t r = 0; r < breq.size(); ++r)
      seg_in[breq[r].si] += (int64_t)q->segs[breq[r].si]->num_docs + h[bres + 4 * r + 2] + h[bres + 4 * r + 3];
  }
  int64_t in_filter = 0;
  for (int si = 0; si < q->nseg; ++si) {
    if (state[si] < 0) seg_in[si] = -1;
    else if (segment_tree[si] == PA_STATS_NON_SCAN) seg_in[si] = 0;
    else in_filter += seg_in[si];
    if (segment_in_filter) segment_in_filter[si] = seg_in[si];
  }
  out[0] = in_filter;
  out[1] = (docs_scanned - non_scan_docs) * (int64_t)projected_columns;
  out[2] = gpu_segs;
  return PA_OK;
}

int32_t pa_query_limit_trimming(const pa_query* q) {
  return q && q->prepared ? (q->limit_mode ? 1 : (q->limit_walk ? 2 : 0)) : -1;
}

int64_t pa_query_num_groups_limit_reached(const pa_query* q) { return q && q->prepared ? q->last_reached : -1; }

int pa_query_key_layout(const pa_query* q, int32_t* hashed, int32_t* shifts) {
  if (!q || !q->prepared) return fail(PA_EINVAL, "query not prepared");
  if (hashed) *hashed = q->hashed ? 1 : 0;
  if (shifts)
    for (int j = 0; j < q->spec.num_group_by; ++j) shifts[j] = q->hashed ? q->key_shift[j] : 0;
  return PA_OK;
}

int32_t pa_query_key_words(const pa_query* q) { return q && q->prepared ? (q->hashed ? q->key_words : 1) : -1; }

void pa_query_destroy(pa_query* q) { delete q; }

}  // extern "C"
