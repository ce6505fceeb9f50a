// Internal header of the host side of the C-ABI (include/pinot_amd.h): the types every host translation unit
// shares (segments, the prepared query, planner state) and the entry points one unit calls in another.
// pa_segment.hip: segment residency; pa_plan.hip / pa_plan_kernels.hip: the planner; pa_jit.hip: the hiprtc
// query-shape kernels; pa_capi.hip: query life cycle and scan; pa_fetch.hip: results and hashed-row merge;
// pa_stats_host.hip: leaf bitmaps, filter counts and the execution-statistics engine.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <array>
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
#include "pa_jit_abi.h"

using namespace pa;


inline thread_local std::string g_err;

inline int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// PA_DEBUG_PLAN=1: the planner's decisions on stderr (why a query takes a strategy)
inline bool plan_debug() {
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

inline int dev_alloc(DevBuf& b, size_t bytes) {
  b.n = bytes;
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) return fail(PA_ENOMEM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
  return PA_OK;
}

inline void dev_free(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
}

inline int64_t wtiles_for(int64_t num_docs) { return (num_docs + kWTileDocs - 1) / kWTileDocs; }

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


struct pa_segment {
  int32_t num_docs = 0;
  std::map<int32_t, Column*> cols;
  uint64_t bytes = 0;
  ~pa_segment() {
    for (auto& kv : cols) delete kv.second;
  }
};

// Order key of an 8-byte dictionary value: the value itself (INT/LONG) or its order-preserving image (FLOAT/DOUBLE,
// Double.compare order: -0.0 < 0.0), so distinct values get distinct keys in value order.
inline int64_t value_order_key(uint64_t bits, int32_t vtype) {
  return (vtype == PA_FLOAT || vtype == PA_DOUBLE) ? f64_order_encode(__builtin_bit_cast(double, bits))
                                                    : (int64_t)bits;
}

struct Literal {
  int leaf;
  bool neg;
};
using Clause = std::vector<Literal>;

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

inline ScratchArena* arena_for(int dev) {
  static std::mutex m;
  static std::map<int, ScratchArena*> arenas;
  std::lock_guard<std::mutex> g(m);
  ScratchArena*& a = arenas[dev];
  if (!a) a = new ScratchArena();  // lives for the process (freed with it)
  return a;
}

// Grows the arena to at least `bytes` (caller holds a->mu).
inline int arena_grow(ScratchArena* a, size_t bytes) {
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

struct pa_query {
  pa_query_spec spec;
  int32_t nseg = 0;
  std::vector<const pa_segment*> segs;
  std::vector<std::vector<pa_leaf_params>> leaf_params;
  std::vector<std::vector<std::vector<uint32_t>>> luts;        // [seg][leaf]
  std::vector<std::vector<std::vector<int32_t>>> remaps;       // [seg][gb]
  std::vector<std::vector<char>> has_remap;
  std::vector<std::vector<std::vector<int32_t>>> vremaps;      // [seg][agg] DISTINCTCOUNT value remaps (empty = identity)
  std::vector<std::vector<int32_t>> vremap_host;               // [seg] host copy of DevSeg::vremap (value_dictionary)
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
  int jit_waves = 0, jit_grid = 0, jit_lds = 0, jit_nd = 16, jit_nseg = 0, jit_classes = 0, jit_slots = 0;
  std::vector<int> jit_cols;  // the column slots the specialised kernel stages (pa_query_column_staged)
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
  int v_id_bits = 0;    // V_FMT_ID: bits of a table-wide value id (a record holds it above the key offset)
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
  bool gd_box_ok = false;                  // gd_lo / gd_span / gd_nkeys hold the key box (the JIT's input too)
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

// Tile geometry of one scan pass: wave tile of 1024 or 2048 docs, D DMA instructions per tile, a ring of R tile images
// per wave (R-1 tiles in flight). Measured on MI355X (tools/sweep.py): the decode, not the DMA, is what needs hiding,
// so the plan maximises resident waves per CU (workgroups per CU, checked against the occupancy the compiled kernel
// really has), then prefers 2048-doc tiles, then bytes in flight (capped at 128 KiB per CU).
struct TilePlan {
  int steps = 0, dma = 0, ring = 0, wg_per_cu = 0, img_dw = 0;
  size_t lds = 0;
  double score = -1;
};

// ---------------------------------------------------------------- cross-unit entry points
// pa_plan.hip
int upload_owned(pa_query* q, const void* host, size_t bytes, void** dev);
int mv_group_component(const pa_query* q);
int plan_filter(pa_query* q, Prep& P);
int plan_slots(pa_query* q, Prep& P);
int plan_key_space(pa_query* q, Prep& P);
int plan_limit(pa_query* q, Prep& P);
int plan_gdense(pa_query* q, Prep& P);
int build_segments(pa_query* q, Prep& P);
int plan_accumulators(pa_query* q, Prep& P);
// pa_plan_kernels.hip
bool affine_dictionary(const std::vector<uint64_t>& v, int32_t vtype, int64_t* base, int64_t* step);
void apply_layout(std::vector<DevSeg>& segs, int steps, int nslots, int nleaves, const void* dummy,
                  uint64_t* staged_bytes, int64_t* total_tiles);
int plan_kernels(pa_query* q, Prep& P, TilePlan& plan, TilePlan& count_plan);
void fill_devquery(pa_query* q, const Prep& P, const TilePlan& plan, int64_t total_tiles);
int plan_scratch(pa_query* q, const Prep& P);
int plan_walk(pa_query* q, const Prep& P);
int plan_limit_buffers(pa_query* q, const Prep& P, int cus, int64_t total_tiles);
int upload_descriptors(pa_query* q);
PartScratch scratch_of(const pa_query* q, void* base);
size_t leap_header_bytes(const pa_query* q);
int plan_leaps(pa_query* q, const Prep& P);
int alloc_leaps(pa_query* q, const Prep& P);
// pa_jit.hip
int jit_plan(pa_query* q, const Prep& P, int cus);
void jit_fill_pointers(pa_query* q, JitArgs& a);
void pve_fill_pointers(const pa_query::PveStream& st, unsigned long long* matched, PveArgs& a);
int pve_plan(pa_query* q, const Prep& P, int cus);

