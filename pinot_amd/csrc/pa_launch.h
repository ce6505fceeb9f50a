// Host-callable launchers of the kernels in pa_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "pa_device.h"

namespace pa {
// ordered compaction of the non-empty keys (fetch): phase 0 = per-block counts + scan (block_sums[nb] = total),
// phase 1 = write key ids + gather every section's rows into d.dst
constexpr int kMaxCompactSections = PA_MAX_AGGS + 2;
struct CompactDesc {
  int32_t nsec;
  int32_t es[kMaxCompactSections];   // element bytes (8, or 1 = HLL registers)
  int64_t per[kMaxCompactSections];
  const void* src[kMaxCompactSections];
  void* dst[kMaxCompactSections];
  int64_t* keys;
};
// Final-format compaction of a direct key space (fetch of large key spaces): the non-empty keys in key order, every
// column already in the caller's representation (key ids int64, counts int64, per aggregation double or its HLL /
// presence bytes), one output row per thread (coalesced stores), so the host only copies.
struct FinalDesc {
  int32_t nagg;
  int32_t type[PA_MAX_AGGS];   // PA_AGG_*
  int32_t src[PA_MAX_AGGS];    // AccSrc of SUM / MIN / MAX
  int64_t per[PA_MAX_AGGS];    // HLL / presence: bytes per row
  const void* sec[PA_MAX_AGGS];  // the aggregation's accumulator section (nullptr: COUNT)
  void* out[PA_MAX_AGGS];      // staging column: double[n], or per bytes x n
  int64_t* keys;               // staging: key ids
  int64_t* counts;             // staging: counts
};
hipError_t launch_compact_final(const unsigned long long* count, int64_t K, int all, const uint32_t* block_off,
                                int64_t cap, const FinalDesc* d, hipStream_t s);
// one filter literal of one segment -> doc bitmap (execution statistics)
hipError_t launch_leaf_bitmap(const DevSeg* seg, int li, int flip, int64_t num_docs, uint32_t* out, hipStream_t s);
// Execution-statistics counts over leaf bitmaps (pa_bitmap_counts, pa_query_filter_counts): per job, postfix
// programs A (tok[0..len_a)) and B (tok[kBitProgMax..+len_b)) over one segment's leaf bitmaps.
constexpr int kBitProgMax = 64;
constexpr int kBitProgStack = 16;
constexpr int kBitGroups = 2;  // 16-byte word groups per thread of the count kernels
struct BitJob {
  const uint32_t* bm;  // the segment's leaf bitmaps, leaf l at bm + l * words
  int64_t words, num_docs;
  int64_t first_block, nb;
  const int32_t* tok;  // program A at tok[0..len_a), B at tok[kBitProgMax..+len_b)
  int32_t len_a, len_b;
  int32_t nu, pad;     // nu > 0: the programs use leaves uleaf[0..nu) and their leaf tokens are positions in it
  int32_t uleaf[4];
  uint32_t* scratch;   // block_last[nb], block_in[nb]
  unsigned long long* part;  // [nb][4] per-workgroup counts
  unsigned long long* out;
};
struct LeafJob {  // leaf bitmap of one (segment, leaf): workgroups [first_block, + leaf_bitmap_blocks(num_docs))
  const DevSeg* seg;
  uint32_t* out;
  int64_t num_docs, first_block;
  int32_t li, flip;
};
int64_t leaf_bitmap_blocks(int64_t num_docs);
int64_t bit_count_blocks(int64_t num_docs);
int64_t bit_count_scratch_words(int64_t words);
hipError_t launch_bit_counts_batch(const BitJob* jobs, int nj, int64_t total_blocks, bool any_b, int32_t* table,
                                   hipStream_t s);
hipError_t launch_leaf_bitmaps_batch(const LeafJob* jobs, int nj, int64_t total_blocks, hipStream_t s);
hipError_t launch_compact(const unsigned long long* count, int64_t K, int all, uint32_t* block_sums, int64_t cap,
                          const CompactDesc* d, int phase, hipStream_t s);
// numGroupsLimit first-seen trimming (pa_kernels.hip "numGroupsLimit"): the (segment, key) first-position table,
// the sort buffers and the per-segment thresholds
struct LimitDesc {
  long long* fkeys;              // composite key: accumulator slot * num_segments + segment; INT64_MAX = empty
  unsigned long long* fpos;      // first position (doc << eb | expansion index); UINT64_MAX = none
  int64_t fmask;                 // slots - 1 (power of two)
  uint32_t* hist;                // radix select: [num_segments][256] digit counts of the current pass
  unsigned long long* prefix;    // radix select: [num_segments] the selected value's digits found so far
  long long* rank;               // radix select: [num_segments] rank still to find among the prefix's values (1-based;
                                 // < 0: the segment has fewer than `limit` groups, nothing is trimmed)
  unsigned long long* thresh;    // [num_segments]: first positions below it are admitted; UINT64_MAX = all
  unsigned long long* reached;   // segments whose distinct groups reached the limit (GroupByOperator.java:112)
  int64_t limit;                 // numGroupsLimit
  int32_t eb;                    // expansion-index bits
  int32_t pos_bits;              // first positions are < 2^pos_bits (radix select digit passes)
  int32_t nseg;                  // segments of the query
  int32_t pad;
};
// phase 0: first-seen positions; 1: per segment the numGroupsLimit-th smallest first position (radix select, 8-bit
// digits from the top) -> thresholds; 2: aggregation of the admitted (doc, key) pairs
hipError_t launch_limit_passes(const DevQuery* q, const DevSeg* segs, const LimitDesc& F, int grid, int phase,
                               hipStream_t s);
// numGroupsLimit walk form: one workgroup per segment with a non-null DevSeg::admit; `words` = bitmap words (K / 32)
constexpr int64_t kWalkMaxWords = 40000;  // LDS bitmap of at most 160000 bytes
hipError_t launch_limit_walk(const DevQuery* q, const DevSeg* segs, int nseg, int64_t words, bool mv, hipStream_t s);
hipError_t launch_bswap_words(uint32_t* w, int64_t n, hipStream_t s);
hipError_t launch_hll_lut_numeric(const int64_t* di, const double* dd, int32_t vtype, int32_t card, int32_t log2m,
                                  uint32_t* lut, hipStream_t s);
hipError_t launch_hll_lut_hashes(const int32_t* hashes, int32_t card, int32_t log2m, uint32_t* lut, hipStream_t s);
hipError_t launch_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
hipError_t launch_gather(const void* src, int esize, int64_t per, const int64_t* keys, int64_t n, void* out,
                         hipStream_t s);
// partitioned aggregation: per-(workgroup, partition) range offsets + partition bases (after the count pass, which ran
// k workgroups per emit workgroup)
hipError_t launch_part_offsets(const DevQuery* hq, const PartScratch& ps, int G, int k, hipStream_t s);
// vk: the pass-C variant of the V stream (vk_code / kVkGeneric)
hipError_t set_part_agg_lds_limit(int vk, int lds_bytes);
hipError_t launch_part_agg(int vk, const DevQuery* q, const PartScratch& ps, int P, int pv, bool one_word,
                           int lds_bytes, hipStream_t s);
// Cross-GPU merge of hashed key spaces (pa_merge.hip): a row is every per-key section's elements of one slot
enum RowOp : int32_t { ROW_ADD_U64 = 0, ROW_ADD_F64 = 1, ROW_MIN_I64 = 2, ROW_MAX_I64 = 3, ROW_MAX_U8 = 4, ROW_KEY = 5 };
constexpr int kMaxRowSecs = PA_MAX_AGGS + 2;
struct RowSec {
  int32_t op;          // RowOp
  int32_t pad;
  int64_t slot_bytes;  // bytes of one slot in the section (a multiple of 8)
  int64_t row_off;     // byte offset of the section inside a row
  void* base;          // the section in the accumulator block
};
struct RowDesc {
  int32_t nsec;
  int32_t key_words;   // 1: one packed key word per slot; 2: [k0, k1, state] (pa_keys.h)
  int64_t row_bytes;
  int64_t num_slots;   // table slots incl. the reserved one (num_keys)
  int64_t ht_mask;     // probing mask (slots - 2)
  int64_t key_off;     // byte offset of the packed key (k0[, k1, state]) inside a row
  const unsigned long long* count;
  long long* keys;
  RowSec sec[kMaxRowSecs];
};
hipError_t launch_pack_index(const RowDesc& d, int world, int phase, unsigned long long* counts,
                             unsigned long long* cursor, int64_t* row_slot, hipStream_t s);
hipError_t launch_pack_copy(const RowDesc& d, const int64_t* row_slot, int64_t rows, unsigned char* out, hipStream_t s);
// counters: [0] groups inserted, [1] rows that found no free slot, [2] reserved-slot flag
hipError_t launch_merge_rows(const RowDesc& d, const unsigned char* rows, int64_t n, int64_t* row_slot,
                             unsigned long long* counters, hipStream_t s);
// fused execution statistics: the neighbour searches of the E docs the scan listed (DevQuery::leap_mode)
hipError_t launch_leap_search(const DevQuery* q, const DevSeg* segs, int64_t slices, hipStream_t s);
constexpr int64_t kLeapMaxSlices = 16384;  // fused statistics: list slices (scan waves) the search kernel scans in LDS
// Execution statistics engine (pa_stats.hip): element masks (postfix programs over one segment's leaf bitmaps),
// popcounts / value counts of masks, and leap-frogs of AndDocIdIterator over element masks
constexpr int kStatMaskWordsPerThread = 4;
constexpr int kLfMaxK = 8;      // children of one leap-frogging AND
constexpr int kLfMaxSub = 8;    // scan / index children of its OR children, together
constexpr int64_t kLfChunkDocs = 2048;
enum : int32_t { LF_DOCS = 0, LF_SCAN = 1, LF_OR = 2 };
struct StatMaskJob {  // workgroups [first_block, + stat_mask_blocks(words))
  const uint32_t* bm;  // leaf l at bm + l * words
  uint32_t* out;
  int64_t words, num_docs, first_block;
  int32_t tok_off, len;  // the program at toks[tok_off .. + len)
};
struct StatCountJob {
  const uint32_t* mask;
  const int32_t* wt;  // multi-value column: offsets[num_docs + 1] (a doc counts its values); nullptr: docs
  unsigned long long* out;
  int64_t words, first_block;
};
struct LfJob {
  int32_t K, nsub;
  int32_t kind[kLfMaxK];                        // LF_DOCS, LF_SCAN, LF_OR
  int32_t sub_first[kLfMaxK], sub_count[kLfMaxK];  // LF_OR: its children at [sub_first, + sub_count)
  int32_t sub_kind[kLfMaxSub];                  // LF_DOCS or LF_SCAN
  int32_t cell_words, pad;                      // 4 + 2 nsub
  const uint32_t* emask[kLfMaxK];
  const int32_t* ewt[kLfMaxK];                  // multi-value scan: value offsets; nullptr: one entry per doc
  const uint32_t* smask[kLfMaxSub];
  const int32_t* swt[kLfMaxSub];
  int64_t num_docs, nchunks, first_lane;        // lanes [first_lane, + nchunks (K + 1)) of lf_chunk_kernel
  uint32_t* cells;                              // [nchunks][K + 1][cell_words]
  unsigned long long* out;                      // [0] entries read, [1] read after the last match, [2] matches
};
// The filter shapes the reduction above does not express (a NOT child of a leap-frogging AND, an AND or NOT under an
// OR inside a leap-frog, a NOT over a leap-frog with an OR child): the segment's iterator tree replayed on the GPU, one
// thread per segment, over the element masks (stat_replay_kernel): the reference's iterators restated node by node.
constexpr int kRpMaxNodes = 24;
constexpr int kRpMaxDepth = 6;
enum : int32_t { RP_EMPTY = 0, RP_ALL = 1, RP_DOCS = 2, RP_SCAN = 3, RP_AND = 4, RP_OR = 5, RP_NOT = 6 };
struct RpNode {
  int32_t kind, nchild, first, depth;  // children: RpJob::kids[first .. first + nchild), depth below the root
  const uint32_t* mask;                // RP_DOCS / RP_SCAN: the doc set
  const int32_t* wt;                   // RP_SCAN over a multi-value column: value offsets (nullptr: one entry per doc)
};
struct RpJob {
  int64_t num_docs;
  int32_t nnodes, root;
  int32_t kids[kRpMaxNodes];
  RpNode node[kRpMaxNodes];
  unsigned long long* out;             // entries the scan iterators read (UINT64_MAX: the step budget ran out)
};
hipError_t launch_stat_replay(const RpJob* jobs, int nj, hipStream_t s);
int64_t stat_mask_blocks(int64_t words);
hipError_t launch_stat_masks(const StatMaskJob* jobs, int nj, int64_t blocks, const int32_t* toks, hipStream_t s);
hipError_t launch_stat_counts(const StatCountJob* jobs, int nj, int64_t blocks, hipStream_t s);
hipError_t launch_leapfrogs(const LfJob* jobs, int nj, int64_t lanes, hipStream_t s);
// count-free partitioned emit (pa_pve.hip): per-partition chunk lists from the emit workgroups' chunk tables
hipError_t launch_pve_lists(const uint32_t* hist, uint32_t* off, uint64_t* base, const uint32_t* table,
                            const uint32_t* used, uint32_t* index, uint32_t* tot, int G, int P, int64_t C, int cr,
                            hipStream_t s);
hipError_t set_scan_lds_limit(int strategy, int steps, int lm, int bytes);
hipError_t scan_occupancy(int strategy, int steps, int lm, int lds_bytes, int* blocks_per_cu);
hipError_t launch_scan(int strategy, int steps, int lm, int grid, int lds_bytes, const DevQuery* q, const DevSeg* segs,
                       const LmSegPlan* plans, const PartScratch& ps, hipStream_t s);
}  // namespace pa
