// Device-side descriptors shared by the scan kernels (pa_kernels.hip) and the host layer (pa_capi.hip).
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//  * SV dictionary-encoded forward index: the reference's FixedBitSVForwardIndexWriter bitstream
//    (PinotDataBitSet.java:80, value i at stream bits [i*nb, (i+1)*nb), MSB-first) with every 32-bit
//    word byte-swapped once at upload, so word w holds stream bits [32w, 32w+32) with stream bit 32w
//    in bit 31. Four guard words precede the stream and the stream is zero-padded to a whole number of
//    2048-doc wave tiles plus four words, so every staged or lazy read is in bounds.
//  * Dictionaries: int64 (INT/LONG) or double (FLOAT/DOUBLE) arrays indexed by dictId.
//  * Raw columns: native little-endian arrays of the stored type.
#pragma once
#include <stdint.h>
#include "../../include/pinot_amd.h"

namespace pa {

constexpr int kWave = 64;
constexpr int kWavesPerWG = 4;
constexpr int kWGSize = kWave * kWavesPerWG;
// waves per workgroup of a scan-kernel variant (emit variants may run 16-wave workgroups)
constexpr int kSteps = 32;                    // 64-doc steps per wave tile
constexpr int kWTileDocs = kWave * kSteps;    // 2048 docs: one wave tile; 64*nb stream words per column
constexpr int kMaxSlots = 12;                 // distinct columns referenced by one query
constexpr int kGuardWords = 4;

enum ColKind : int32_t { COL_NONE = 0, COL_SV_DICT = 1, COL_SV_RAW = 2, COL_MV_DICT = 3 };
// Partitioned aggregation (high-cardinality dense GROUP BY), three kernels over the same tile -> wave schedule:
//   STRAT_PCOUNT: the count pass — filter + group key of every doc, records per (workgroup, key partition) counted in
//                 LDS (its group-by columns only; numDocsScanned is counted here);
//   (part_scan_kernel: exclusive scans -> every (workgroup, partition) owns a padded range of its partition);
//   STRAT_PEMIT:  the emit pass — the same docs' records go into per-partition LDS bins, and a full bin leaves as one
//                 contiguous burst into the workgroup's range of its partition (each record crosses HBM once);
//   part_agg_kernel: one workgroup per partition aggregates its records in LDS and stores its key range.
// Two record streams: V (one record per matching doc: COUNT + SUM/MIN/MAX payloads) and H (one record per value of
// the DISTINCTCOUNTHLL(MV) column: key | register | rank), each with its own key partitioning.
// STRAT_LANE: aggregation-only queries (no GROUP BY) over single-value columns: every lane keeps its own running
// COUNT/SUM/MIN/MAX in registers for the whole kernel and the wave reduces them once at the end (no per-step reduction,
// no LDS or global atomics per doc).
// STRAT_LANE_CNT / _RAW / _DICT: the lane-major STRAT_LANE kernel compiled for one kind of aggregation column only (no
// value aggregation / raw columns only / dictionary columns only), so each variant holds just its own paths (the
// all-kinds kernel spills); STRAT_LANE runs mixed sets and step-major tiles.
// STRAT_GDENSE: filter + GROUP BY over a small key space whose matching docs are dense (pa_gdense.h): every column the
// query reads is staged through the tile ring (raw metrics included), value dictionaries and group-key remaps sit in
// LDS per segment, and the accumulators are LDS-privatised with per-lane replicas, so a matching doc costs LDS
// operations only (no per-doc HBM access, which would wait behind the ring's in-flight DMA: vmcnt counts in order).
enum Strategy : int32_t {
  STRAT_LDS = 0, STRAT_GLOBAL = 1, STRAT_PEMIT = 2, STRAT_PCOUNT = 3, STRAT_LANE = 4,
  STRAT_LANE_CNT = 5, STRAT_LANE_RAW = 6, STRAT_LANE_DICT = 7, STRAT_GDENSE = 8, STRAT_GDENSE8 = 9,
  STRAT_GDENSE12 = 10,
  // STRAT_GDENSE with register-staged tiles (gdense_rs_kernel): 12 waves, 4 tiles of <= 4 instructions in VGPRs; 8 waves,
  // 3 tiles of <= 12 instructions
  STRAT_GDENSE_RS12 = 11, STRAT_GDENSE_RS8 = 12,
  // the count pass of a query grouping by a multi-value column (one record per (doc, value) pair)
  STRAT_PCOUNT_MV = 13,
  // STRAT_GDENSE over the LDS-DMA ring with the lane-major walk (gdl_tile): 8- / 16-wave workgroups
  STRAT_GDENSE_LM8 = 14, STRAT_GDENSE_LM16 = 15
};
__host__ __device__ constexpr bool is_pcount(int s) { return s == STRAT_PCOUNT || s == STRAT_PCOUNT_MV; }
// STRAT_GDENSE: 4-wave workgroups; STRAT_GDENSE8 / STRAT_GDENSE12: the same kernel with 8- / 12-wave workgroups (2 / 3
// waves per SIMD when one workgroup fits a CU, e.g. beside a 64 KiB value table: the walk's LDS round trips and VALU
// issue overlap across waves; 12 waves: step-major tiles only)
__host__ __device__ constexpr bool is_gdense(int s) {
  return s == STRAT_GDENSE || s == STRAT_GDENSE8 || s == STRAT_GDENSE12 || s == STRAT_GDENSE_RS12 || s == STRAT_GDENSE_RS8 ||
         s == STRAT_GDENSE_LM8 || s == STRAT_GDENSE_LM16;
}
__host__ __device__ constexpr bool is_gdense_lm(int s) { return s == STRAT_GDENSE_LM8 || s == STRAT_GDENSE_LM16; }
__host__ __device__ constexpr bool is_gdense_rs(int s) { return s == STRAT_GDENSE_RS12 || s == STRAT_GDENSE_RS8; }
// register ring of the register-staged variants: tiles in flight + 1, wave instructions per tile at most
__host__ __device__ constexpr int gd_rs_ring(int s) { return s == STRAT_GDENSE_RS12 ? 4 : 3; }
__host__ __device__ constexpr int gd_rs_dmax(int s) { return s == STRAT_GDENSE_RS12 ? 4 : 12; }
// STRAT_GDENSE value sources and LDS operations of one aggregation
enum GdVs : int32_t {
  GVS_ID = 0,    // the dictId itself (SUM over an affine dictionary shared by every segment; MIN/MAX of a shared sorted one)
  GVS_T32 = 1,   // per-segment LDS table of int32 values (dictId -> value)
  GVS_T64 = 2,   // per-segment LDS table of int64 values
  GVS_TF = 3,    // per-segment LDS table of double values
  GVS_RI32 = 4,  // staged raw INT
  GVS_RF32 = 5,  // staged raw FLOAT
  GVS_RI64 = 6,  // staged raw LONG
  GVS_RF64 = 7,  // staged raw DOUBLE
  GVS_T32U = 8   // per-segment LDS table of uint32 offsets from gd_base (value = gd_base + entry; packed SUMs, GdLmPlan)
};
__host__ __device__ constexpr bool gvs_float(int vs) { return vs == GVS_TF || vs == GVS_RF32 || vs == GVS_RF64; }
enum GdOp : int32_t {
  GOP_SUM_I = 0,  // int64 sum of int32-range values (one ds_add_u64)
  GOP_SUM_L = 1,  // exact pair: low 32 bits unsigned / high 32 bits signed (two ds_add_u64)
  GOP_SUM_F = 2,  // ds_add_f64
  GOP_MIN_I = 3,  // ds_min_i64 (ordered encoding of doubles)
  GOP_MAX_I = 4,
  GOP_MIN_U = 5,  // ds_min_u32 on dictIds (shared sorted dictionary: the value is looked up once per group at the end)
  GOP_MAX_U = 6
};
constexpr int kGdWaves = 4;          // waves per STRAT_GDENSE workgroup (STRAT_GDENSE8: 8)
constexpr int kGdSmSteps = 16;        // 64-doc steps of a step-major STRAT_GDENSE tile (1024 docs)
constexpr int kGdMaxKeys = 16384;    // largest LDS key space of STRAT_GDENSE
__host__ __device__ constexpr bool is_lane(int s) { return s >= STRAT_LANE && s <= STRAT_LANE_DICT; }
constexpr int kLaneAggs = 4;  // STRAT_LANE: at most this many aggregations (COUNT included)
constexpr int kLaneAccBytes = 20;  // STRAT_LANE: LDS bytes per thread and aggregation (int64 pair + a dictId)
constexpr int kLaneHistMax = 16384;  // STRAT_LANE_DICT: largest shared dictionary counted in an LDS histogram
// The emit pass's kernel variant (launch code): the V record format (-1: no V stream) and whether there is an H stream
// are template parameters, so each variant's record loop is straight-line code (no per-record format branches).
// `big`: 16-wave workgroups (the partition bins and their state are per workgroup, so sharing them among more waves
// leaves LDS for more resident waves when the tile images are small).
constexpr int kPemitBase = 16;
constexpr int kEmitBigWaves = 16;
// `mv`: the V records of a multi-value group-by (one per (doc, value) pair; V stream only, no generic records).
__host__ __device__ constexpr int pemit_strat(int vf, int hh, int big = 0, int mv = 0) {
  return kPemitBase + 2 * (vf + 1) + (hh ? 1 : 0) + (big ? 16 : 0) + (mv ? 32 : 0);
}
__host__ __device__ constexpr bool is_pemit(int s) { return s >= kPemitBase; }
__host__ __device__ constexpr int pemit_vf(int s) { return (((s - kPemitBase) & 15) >> 1) - 1; }
__host__ __device__ constexpr bool pemit_hh(int s) { return ((s - kPemitBase) & 1) != 0; }
__host__ __device__ constexpr int pemit_big(int s) { return ((s - kPemitBase) >> 4) & 1; }
__host__ __device__ constexpr bool pemit_mv(int s) { return is_pemit(s) && (s - kPemitBase) >= 32; }
// a partitioned pass (count or emit) of a multi-value group-by
__host__ __device__ constexpr bool part_mv(int s) { return s == STRAT_PCOUNT_MV || pemit_mv(s); }
__host__ __device__ constexpr int scan_waves(int s) {
  return is_pemit(s) && pemit_big(s) ? kEmitBigWaves
                                       : (s == STRAT_GDENSE8 || s == STRAT_GDENSE_RS8 || s == STRAT_GDENSE_LM8) ? 2 * kGdWaves
                                       : (s == STRAT_GDENSE12 || s == STRAT_GDENSE_RS12) ? 3 * kGdWaves
                                       : s == STRAT_GDENSE_LM16 ? 4 * kGdWaves : kWavesPerWG;
}
// V record formats (word 0 always holds the key's offset inside its partition, key & ((1 << kshift_v) - 1)):
//   V_FMT_KEY: COUNT only, one word;  V_FMT_ID: one word, | value id << kshift_v (the value column's table-wide value
//   dictionary `vdict`);  V_FMT_32: + the int32 value;  V_FMT_64: + the 64-bit value (int64, or double bits);
//   V_FMT_GEN: + every payload at its DevAgg::pay_off (one or two words each).
enum VFormat : int32_t { V_FMT_KEY = 0, V_FMT_ID = 1, V_FMT_32 = 2, V_FMT_64 = 3, V_FMT_GEN = 4 };
constexpr int kMaxVWords = 9;       // V record words (key + at most four 64-bit payloads)
constexpr int kDocVals = 8;         // H records: docs with at most this many values take the doc-reserved emit path
constexpr uint32_t kSentinel = 0xffffffffu;  // word 0 of a padding record (never a valid V or H record)
// SUM/MIN/MAX value source. SRC_INT: every value fits int32 (one exact int64 accumulator);
// SRC_LONG: 64-bit values, SUM kept exactly as a (low 32 bits unsigned, high 32 bits signed) pair of int64
// sums = a 96-bit total for up to 2^32 docs per key; SRC_DOUBLE: FLOAT/DOUBLE.
enum AccSrc : int32_t { SRC_INT = 0, SRC_DOUBLE = 1, SRC_LONG = 2 };

struct DevCol {
  const uint32_t* words;     // SV dict: byte-swapped stream words (points past the guard words)
  const void* raw;           // SV raw: values
  const int64_t* dict_i64;   // INT/LONG dictionary
  const double* dict_f64;    // FLOAT/DOUBLE dictionary
  const int32_t* mv_off;     // MV dict: value offset of every doc's first value [num_docs + 1]
  int32_t kind;              // ColKind
  int32_t nbits;
  int32_t vtype;             // PA_INT..PA_BYTES
  int32_t lds_off;           // staged: dword offset of the column's region inside a wave image; -1 = lazy
  int32_t card;              // dictionary columns: cardinality (dictIds < card)
  int32_t flags;             // COLF_*
};
constexpr int32_t COLF_DICT_SORTED = 1;  // dictionary values strictly ascending (INT/LONG by value, FLOAT/DOUBLE in
                                         // Double.compare order): MIN/MAX of values = the values of the MIN/MAX dictId

// One CNF literal for one segment. The column fields the leaf reads are copied in, so evaluating a leaf
// costs one scalar-load round per tile (no dependent leaf -> column descriptor chain).
struct DevLeaf {
  int32_t kind;              // PA_LEAF_*
  int32_t slot;
  int32_t lo;                // DICT_RANGE: (uint)(id - lo) < (uint)span
  int32_t span;
  int32_t negate;
  int32_t clause_end;        // 1 if this literal closes a CNF clause
  int32_t nbits;             // column copy: bits per dictId
  int32_t lds_off;           // column copy: staged region offset (dwords) or -1
  const uint32_t* lut;       // DICT_SET bitmap (device)
  const uint32_t* words;     // column copy: stream words
  const void* raw;           // column copy: raw values
  const int32_t* mv_off;     // column copy: MV value offsets (MV leaves)
  int32_t vtype;             // column copy
  int32_t pad;
  int64_t ilo, ihi;
  double dlo, dhi;
};

struct StageDesc {           // one staged column of a segment
  const uint32_t* words;
  int32_t nbits;
  int32_t lds_off;
};

struct DevSeg {
  int64_t first_wtile;       // prefix sum of wave tiles over the segment list
  int32_t num_docs;
  int32_t num_wtiles;
  int32_t image_dwords;      // staged image size (dwords) of one wave tile of this segment
  int32_t num_staged;
  int32_t index;             // position in the query's segment list
  int32_t pad_index;
  const uint32_t* dummy_src;  // any readable device address: source of the DMA padding instructions
  StageDesc stage[kMaxSlots];
  DevCol cols[kMaxSlots];
  DevLeaf leaves[PA_MAX_LEAVES];
  const int32_t* remap[PA_MAX_GROUP_BY];   // dictId -> table-wide key id (nullptr = identity)
  const int32_t* vremap;                   // V_FMT_ID: dictId of the value column -> table-wide value id (nullptr = id)
  const uint32_t* hll_lut[PA_MAX_AGGS];    // HLL: dictId -> (register index << 8) | rank; DISTINCTCOUNT: dictId ->
                                           // table-wide value id (nullptr = identity)
  const uint32_t* admit;                   // numGroupsLimit walk: bitmap of the table-wide keys admitted in this
                                           // segment (limit_walk_kernel writes it); nullptr = every key admitted
  const void* gd_src[PA_MAX_AGGS];         // STRAT_GDENSE: device dictionary behind aggregation a's LDS value table
                                           // (identical dictionaries of different segments share one pointer, so the
                                           // table is loaded once per workgroup)
};

struct DevAgg {
  int32_t type;              // PA_AGG_*
  int32_t slot;
  int32_t log2m;
  int32_t src;               // AccSrc
  int64_t* acc_i64;          // SUM(int) [K], SUM(long) [2K: lo, hi], MIN / MAX (ordered encoding for doubles)
  double* acc_f64;           // SUM(double)
  uint8_t* acc_hll;          // [num_keys << log2m] one byte per register; DISTINCTCOUNT: [num_keys * nvals] presence
  int64_t nvals;             // DISTINCTCOUNT: presence bytes per key (table-wide values, rounded up to 16)
  int32_t lds_off;           // LDS strategy / partition aggregation: byte offset of the WG-private copy
  int32_t pay_off;           // partitioned aggregation, V_FMT_GEN: word offset of the value inside a V record
  // STRAT_LANE_DICT, SUM over a dictionary column that every bound segment shares: per-workgroup dictId counts in LDS
  // (u32[hist_card] at byte hist_off); the sum is sum(count[id] * dict[id]) once at the end (no per-doc gather)
  int32_t hist_card;         // 0 = the per-doc gather path
  int32_t hist_off;
  // STRAT_GDENSE (pa_gdense.h)
  int32_t gd_vs, gd_op;      // GdVs, GdOp
  int32_t gd_acc;            // LDS byte offset of the replicated accumulators (K_lds << rp_log2 elements)
  int32_t gd_tab;            // LDS byte offset of the per-segment value table (GVS_T32 / T64 / TF), else -1
  int32_t gd_tab_n;          // table entries (largest segment cardinality)
  int32_t gd_pad;
  int64_t gd_base, gd_step;  // GVS_ID + GOP_SUM_I: value = base + step * dictId (affine shared dictionary)
};

struct DevQuery {
  int32_t num_segments;
  int32_t num_slots;
  int32_t num_leaves;        // CNF literals (clause-major)
  int32_t num_gb;
  int32_t num_aggs;
  int32_t strategy;
  int32_t num_staged;
  int32_t image_dwords_max;  // max over segments
  int32_t ring;              // wave-tile images per wave (tiles in flight = ring - 1)
  int32_t steps;             // 64-doc steps per wave tile (16 or 32)
  int32_t debug_stream_only; // measurement only: skip the decode (PA_QF_DEBUG_STREAM_ONLY)
  int32_t num_eager;         // literals [0, num_eager) are evaluated on whole staged tiles; the rest (whole CNF
                             // clauses) only on docs the eager clauses matched, straight from HBM
  int32_t dma_per_tile;      // LDS-DMA wave instructions per wave tile (max over segments)
  int32_t lane_major;        // 1: scan_lm_kernel (docs 32*lane + i of a tile), 0: scan_kernel (docs 64*i + lane)
  int32_t has_mv;            // a group-by or aggregation column is multi-value: per-lane key expansion path
  int32_t xcd_major;         // tiles walked in XCD-major block order (xcd_major_block): dense queries
  unsigned long long* matched_docs;  // [0]: docs that passed the filter (numDocsScanned), [1]: group-table overflows,
                                     // [2]: segments that reached numGroupsLimit, [3]: internal consistency errors
  int32_t hashed;            // packed keys through the open-addressing table ht_keys (gb_stride = 1 << shift)
  int32_t key_words;         // hashed: 1 = one 64-bit packed key per slot, 2 = two words + state (pa_keys.h)
  int32_t gb_word[PA_MAX_GROUP_BY];  // hashed, two words: the key word group-by column j's component lands in (else 0)
  int64_t ht_mask;           // table slots - 1 (power of two); slot ht_mask + 1 is reserved for the key INT64_MAX
  long long* ht_keys;        // slot -> packed key, INT64_MAX = empty
  // partitioned aggregation (STRAT_PCOUNT / STRAT_PEMIT / part_agg_kernel)
  int32_t num_parts;         // P = pv + ph; V partitions [0, pv), H partitions [pv, P)
  int32_t pv;                // V partitions (0: no V stream)
  int32_t kshift_v;          // V partition of key k: k >> kshift_v
  int32_t kshift_h;          // H partition of key k: k >> kshift_h
  int32_t part_kr_v;         // 0, or (count-free emit) V partition p = keys [p part_kr_v, (p + 1) part_kr_v), part_kr_v
                             // <= 1 << kshift_v (the record's key offset still takes kshift_v bits)
  int32_t v_fmt;            // VFormat
  int32_t rec_words_v;       // words per V record (1..kMaxVWords)
  int32_t bs_v, bs_h;        // records per LDS bin (a full bin = one store burst of whole 16-byte units)
  int32_t h_first;           // H records carry the first-value-of-the-doc flag (no V stream: COUNT comes from H)
  int32_t hll_agg;           // the partitioned DISTINCTCOUNTHLL(MV) aggregation (-1: no H stream); H record =
                             // key offset << (log2m + 6) | register << 6 | rank << 1 | first
  int32_t emit_val_agg;      // V_FMT_ID/32/64: the aggregation whose column the value comes from (-1: COUNT only)
  int32_t gb_mv;             // the multi-value group-by component (V records: one per (doc, value) pair), -1: none
  int32_t count_skip_gb;     // count pass: a group-by component that cannot change a key's partition (not staged), -1
  int32_t part_lo, part_hi;   // emit pass: the partitions this launch emits ([0, pv) V, [pv, P) H, or all)
  int32_t debug_emit;        // measurement only (PA_DEBUG_EMIT): bit 0 skips the emit pass's record stores, bit 1 its HLL
                             // dictionary gathers, bit 2 its MV value reads (wrong results; isolates the waits)
  uint32_t lds_cnt, lds_done, lds_front, lds_back, lds_start;  // STRAT_PEMIT LDS (bytes): per-partition bin state
  uint32_t lds_slack, pad_slack;  // STRAT_PEMIT LDS (bytes): per-partition parked tail of an H bin
  // (H bins are bs_h + kDocVals records apart: the doc whose records cross the bin end parks its tail past it)
  uint32_t lds_bins_v, lds_bins_h;                            // STRAT_PEMIT LDS (bytes): the V and H bins
  const uint64_t* vdict;     // V_FMT_ID: table-wide values of the value column (int64, or double bits)
  int32_t staged_slots[kMaxSlots];
  int32_t gb_slot[PA_MAX_GROUP_BY];
  int64_t gb_stride[PA_MAX_GROUP_BY];
  int64_t num_keys;
  int64_t total_wtiles;
  unsigned long long* count; // [num_keys]
  uint32_t lds_count_off;    // LDS strategy: byte offset of u32 count[num_keys]
  uint32_t lds_acc_bytes;    // LDS bytes in front of the tile ring: LDS strategy accumulators / partition state
  DevAgg aggs[PA_MAX_AGGS];
  int64_t num_groups_limit;  // numGroupsLimit (limit_walk_kernel)
  // pass C of the V stream, specialised (part_agg_kernel<VK>): every non-COUNT aggregation reads the one payload of a
  // V_FMT_ID/32/64 record and there is at most one SUM, one MIN and one MAX: their aggregation indices (-1 = none),
  // and whether V_FMT_ID value ids are in value order (MIN/MAX then run on the 32-bit ids)
  int32_t vop_sum, vop_min, vop_max;
  int32_t v_id_order;
  // V_FMT_ID value dictionary that is an arithmetic progression (INT/LONG): value = v_base + v_step * id, no gather
  int32_t v_affine, pad_affine;
  int64_t v_base, v_step;
  // V_FMT_ID INT/LONG value dictionary: the largest |value| (0 = unknown); a 64-bit SUM whose partition's record count
  // times it stays below 2^62 accumulates in one int64 instead of the 32/32-bit split pair
  uint64_t v_maxabs;
  // STRAT_LDS, lane-major: the one raw column every non-COUNT aggregation reads (-1: none / several / not all raw)
  int32_t lds_raw_slot, pad_raw;
  // STRAT_GDENSE: the LDS key space is the box the filter leaves to the group-by columns: component j = table key id of
  // column j minus gd_lo[j] (< gd_span[j]), LDS key = sum_j component_j * gd_ls[j]; each key has 1 << gd_rp_log2
  // replicas (lane l updates replica l & (replicas - 1)), so lanes sharing a key update different LDS banks
  int32_t gd_rp_log2;
  int32_t gd_nkeys;                  // LDS keys (product of the spans)
  int32_t gd_lo[PA_MAX_GROUP_BY];
  int32_t gd_span[PA_MAX_GROUP_BY];
  int32_t gd_ls[PA_MAX_GROUP_BY];
  int32_t gd_tab[PA_MAX_GROUP_BY];   // LDS byte offset of column j's per-segment key table (dictId -> component *
                                     // gd_ls[j], -1 outside the box), or -1: component = dictId - gd_lo[j]
  int32_t gd_tab_n[PA_MAX_GROUP_BY]; // key table entries (largest segment cardinality)
  int32_t gd_tables;                 // some key or value table is loaded per segment
  int32_t gd_pk_base;                // lane-major walk, packed: LDS byte offset of the waves' packed rows (which end at
                                     // lds_acc_bytes), 0 = not packed
  // DICT_SET literals whose dictId bitmap is the same in every segment: LDS byte offset of the bitmap (-1: read from
  // HBM — a global load in the tile loop waits for every tile in flight), and its words
  int32_t gd_lut[PA_MAX_LEAVES];
  int32_t gd_lut_words[PA_MAX_LEAVES];
  const uint32_t* gd_plans;          // [num_segments][64]: GdSegPlan of every segment
  // fused execution statistics (default unless PA_QF_NO_FILTER_STATS, leap_tile + leap_search_kernel): 1 = literal 0 (eager, E) and
  // literal 1 (lazy, Z) are the two scan leaves of an AND
  int32_t leap_mode;
  int32_t leap_lds_cap;           // list entries a wave keeps in LDS (after its tile ring) before writing to leap_out
  unsigned long long* leap_out;  // (layout: pa_scan.h "fused execution statistics")
  int64_t leap_cap;              // list entries per scan wave (E docs)
  int64_t leap_slices;           // scan waves (grid x waves per workgroup): one list slice each
};
// STRAT_GDENSE per-segment parameter table: 64 dwords, loaded once per segment into ONE VGPR (lane k holds dword k)
// and read back with v_readlane at compile-time lanes, so the doc loop never issues a scalar load (an SMEM wait is an
// lgkmcnt wait, which also waits for every LDS operation in flight).
constexpr int kGdMaxGb = 3;    // group-by columns
constexpr int kGdMaxAgg = 6;   // non-COUNT aggregations
constexpr int kGdRs12MaxGb = 2, kGdRs12MaxAgg = 2;  // STRAT_GDENSE_RS12: at most this many (its VGPR budget)
// (gd_plans holds kGdPlanDw dwords per segment: the GdSegPlan, the GdRsPlan of the register-staged variants or the
// GdLmIssue of the lane-major ones, then the GdLmPlan of the lane-major ones)
constexpr int kGdPlanDw = 192;
struct GdSegPlan {
  int32_t ngb, nagg, rpl, pad;           // 0..3
  struct {                               // 4 + 6j
    int32_t reg, nbits;                  // staged region (dword offset in a tile image), bits per dictId
    int32_t tab;                         // LDS byte offset of the key table, -1: component = dictId - lo
    int32_t lo, span, ls;
  } gb[kGdMaxGb];
  struct {                               // 22 + 6k: the non-COUNT aggregations in order
    int32_t vs, op;                      // GdVs, GdOp
    int32_t reg, nbits;                  // staged region, bits per dictId (dictionary columns)
    int32_t acc, tab;                    // LDS byte offsets: replicated accumulators, value table
  } ag[kGdMaxAgg];
  int32_t box;                           // 58: the key box is exactly the filter (gd_box_tile)
  int32_t pad1[5];
};
static_assert(sizeof(GdSegPlan) == 256, "one dword per lane");
constexpr int kGdBoxDword = 58;
// Register-staged tiles (STRAT_GDENSE_RS*): the wave instructions that load one 1024-doc tile of the segment's staged
// columns into VGPRs — the same 16-byte-per-lane chunks the LDS-DMA would copy — and where each goes in the tile image.
constexpr int kGdRsMaxIns = 12;
struct GdRsPlan {
  int32_t ins, pad;                      // 0, 1: instructions per tile
  struct {                               // 2 + 5k
    uint32_t src_lo, src_hi;             // the instruction's first chunk in tile 0 of the column's stream
    uint32_t stride;                     // bytes per tile
    uint32_t lanes;                      // lanes with a chunk
    uint32_t dst;                        // byte offset of the first chunk in the tile image
  } in[kGdRsMaxIns];
  int32_t pad1[2];
};
static_assert(sizeof(GdRsPlan) == 256, "one dword per lane");
// Lane-major dense walk (STRAT_GDENSE_LM*): the LDS-DMA of one 1024-doc tile of the segment's staged columns, read
// from one VGPR (lane k holds dword k) with v_readlane, so issuing a tile needs no descriptor load (a vector load's
// vmcnt wait would wait for every DMA in flight; a scalar load's lgkmcnt wait for the LDS atomics in flight).
struct GdLmIssue {
  int32_t ncols;                         // 0
  struct {                               // 1 + 5c
    uint32_t src_lo, src_hi;             // the column's stream (tile 0's first chunk)
    uint32_t stride;                     // bytes per tile
    uint32_t chunks;                     // 16-byte chunks per tile
    uint32_t dst;                        // byte offset of the column's region in the tile image
  } col[kMaxSlots];
  int32_t pad1[3];
};
static_assert(sizeof(GdLmIssue) == 256, "one dword per lane");

// Lane-major dense walk: the per-segment parameters its tile loop reads (one VGPR, v_readlane; no scalar load, whose
// lgkmcnt wait would also wait for the LDS atomics in flight). Packed accumulation: when COUNT and every SUM's per-doc
// term (a dictId of an affine dictionary, or an offset from gd_base through a GVS_T32U table) fit one 64-bit word
// together, a matching doc is ONE ds_add_u64 into its wave's private packed row [key] (term a at bit pk_off[a], COUNT
// in the top bits from pk_cnt): a field of c bits holds 2^c - 1 docs' terms, so each wave drains its packed rows into
// the workgroup's accumulators every pk_drain tiles (at most 1024 docs each).
constexpr int kGdLmLeaves = 6;
constexpr int kGdlMaxCols = 6;  // staged columns of a lane-major walk query (its DMA descriptors live in SGPRs)
struct GdLmPlan {
  int32_t nleaves;                       // 0: eager leaves (every literal)
  int32_t num_docs;                      // 1
  int32_t packed;                        // 2: 1 = packed accumulation
  int32_t pk_cnt;                        // 3: bit offset of the COUNT field (the top field)
  int32_t pk_drain;                      // 4: tiles between drains
  int32_t pk_base;                       // 5: LDS byte offset of wave 0's packed rows (nkeys u64 per wave)
  int32_t pk_off[kGdMaxAgg];             // 6..11: bit offset of non-COUNT aggregation k's field
  int32_t key_leaf;                      // 12: the eager leaf on the (single) group-by column: its unpacked values are
                                         //     the key's (no second unpack), -1: none
  int32_t key_in_box;                    // 13: key_leaf's range is exactly the key box (the filter implies the box)
  int32_t pad0[2];                       // 14..15
  struct {                               // 16 + 7l
    uint32_t code;                       // kind | negate << 8 | clause_end << 9 | nbits << 16
    uint32_t region;                     // byte offset of the column's region in the tile image
    uint32_t lo_t, hi_t;                 // DICT_RANGE bounds, MSB-aligned (leaf_bits)
    int32_t lut_lds;                     // DICT_SET: LDS byte offset of the bitmap, -1: in HBM
    uint32_t lut_lo, lut_hi;             // DICT_SET bitmap in HBM
  } lf[kGdLmLeaves];
  int32_t pad1[6];
};
static_assert(sizeof(GdLmPlan) == 256, "one dword per lane");

// part_agg_kernel variant: -1 generic, else sum kind (0 none, 1 + AccSrc) | MIN << 2 | MAX << 3
constexpr int kVkGeneric = -1;
__host__ __device__ constexpr int vk_code(int sum_kind, bool mn, bool mx) { return sum_kind | (mn ? 4 : 0) | (mx ? 8 : 0); }

// Scratch of a partitioned query, handed to its kernels per launch (it lives in the device's pooled arena).
struct PartScratch {
  uint32_t* hist;    // [grid][P] records per (workgroup, partition): count pass
  uint32_t* off;     // [grid][P] first record of the workgroup's range, relative to its partition
  uint64_t* base;    // [P + 2] first record of every partition: V at [0, pv], H at [pv + 1, P + 1] (stream-relative)
  uint32_t* recs_v;  // V records, partition-major, rec_words_v words each
  uint32_t* recs_h;  // H records, partition-major, one word each
  // count-free emit (pve_jit.hip): V record i of the partitions' concatenation is record i & (2^chunk_shift - 1) of the
  // chunk whose entry is chunk_index[i >> chunk_shift]: chunk id (bits 0..27: records [id << chunk_shift, ..) of
  // recs_v) | (bins written - 1) << 28 (bins of 2^chunk_bin_shift records; the rest of the chunk is not read).
  // nullptr: the records are contiguous
  const uint32_t* chunk_index;
  int32_t chunk_shift, chunk_bin_shift;
  const uint32_t* chunk_index_h;  // the same for the H records (recs_h), relative to base[pv + 1]
  int32_t chunk_shift_h, chunk_bin_shift_h;
};

// Per-segment table of the lane-major scan kernel (scan_lm_kernel): 64 dwords, loaded at segment entry into ONE
// VGPR (lane k holds dword k) and read back with v_readlane — the tile loop needs no scalar-memory round trips.
// Lane-major: lane l of a wave owns docs [32l, 32l+32) of a 2048-doc wave tile, i.e. stream words [l*nb, (l+1)*nb)
// of every staged nb-bit column, so an eager filter leaf is nb ds_reads + a static unpack per lane.
constexpr int kLmStaged = 4;
constexpr int kLmEager = 4;
struct LmSegPlan {
  int32_t nstaged;           // dword 0
  int32_t neager;            // 1: leading eager literals (all DICT_RANGE / DICT_SET on staged columns)
  int32_t num_docs;          // 2
  int32_t num_wtiles;        // 3
  uint32_t dummy_lo, dummy_hi;  // 4,5: readable address for the DMA padding instructions
  int32_t pad0[2];           // 6,7
  struct {                   // 8 + 4c
    uint32_t lo, hi;         // stream words (past the guard words)
    int32_t nbits;
    int32_t lds_off;         // dword offset of the region inside the tile image
  } st[kLmStaged];
  struct {                   // 24 + 8l
    int32_t kind;            // PA_LEAF_DICT_RANGE / PA_LEAF_DICT_SET
    int32_t nbits;
    int32_t lds_off;
    uint32_t lo, span;       // DICT_RANGE, MSB-aligned (see DevLeaf)
    int32_t flags;           // bit 0: negate, bit 1: closes a CNF clause
    uint32_t lut_lo, lut_hi; // DICT_SET bitmap
  } lf[kLmEager];
  int32_t pad1[8];           // 56..63
};
static_assert(sizeof(LmSegPlan) == 256, "one dword per lane");

// Order-preserving int64 image of an IEEE double (an involution): signed int64 order == double order.
__host__ __device__ inline int64_t f64_order_encode(double d) {
  int64_t b = __builtin_bit_cast(int64_t, d);
  return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFLL);
}
__host__ __device__ inline double f64_order_decode(int64_t e) {
  int64_t b = e >= 0 ? e : (e ^ 0x7FFFFFFFFFFFFFFFLL);
  return __builtin_bit_cast(double, b);
}

// stream-lib 2.9.8 com.clearspring.analytics.hash.MurmurHash#hashLong (Pinot pom.xml:1184 pins 2.9.8).
__host__ __device__ inline int32_t murmur_hash_long(int64_t data) {
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = 0;
  uint32_t k = (uint32_t)data * m;
  k ^= k >> r;
  h ^= k * m;
  k = (uint32_t)(data >> 32) * m;
  k ^= k >> r;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

// stream-lib HyperLogLog#offerHashed: register index j and rank r for a 32-bit hash.
__host__ __device__ inline uint32_t hll_slot_rank(int32_t hashed, int32_t log2m) {
  uint32_t h = (uint32_t)hashed;
  uint32_t j = h >> (32 - log2m);
  uint32_t x = (h << log2m) | ((1u << (log2m - 1)) + 1u);
  uint32_t r = (uint32_t)__builtin_clz(x) + 1u;  // x != 0 by construction
  return (j << 8) | r;
}

}  // namespace pa
