// Descriptors the host (pa_jit.hip) writes and the hiprtc-compiled query-shape kernels (gdl_jit.hip, pve_jit.hip) read.
// One definition for both sides: pa_jit.hip includes this file, and build.py pastes it into the kernels' source
// strings in place of their #include line (hiprtc sees no include path), so the layouts cannot drift apart. Plain
// built-in types only (the hiprtc side has no <cstdint>).
#pragma once

constexpr int kJitMax = 6;   // columns, eager leaves, SUM aggregations of one specialised kernel
constexpr int kJitMaxGb = 4;  // group-by columns of the count-free emit

// ---------------------------------------------------------------- gdl_jit.hip (dense GROUP BY, packed accumulation)
// One bound segment, read with scalar loads at segment switches. The per-segment tables (group-key remap, DICT_SET
// bitmaps, value tables) are copied into the workgroup's LDS table slot of the segment when the kernel starts: a
// workgroup's tile range spans at most JIT_NSLOT segments (the planner checks it; JIT_NSLOT 1 with shared tables).
struct JitSeg {
  unsigned long long src[kJitMax];      // column streams, past the guard words
  long long first_tile;                 // first tile (JIT_ND * 64 docs) in the query's tile space
  int num_docs, num_tiles;
  unsigned int lo_t[kJitMax], hi_t[kJitMax];  // DICT_RANGE leaves: MSB-aligned bounds in this segment's dictId space
  int cls;                              // width class (the column widths of JIT_NB[cls])
  int lbase, lspan;                     // the segment's keys in the box: [lbase, lbase + lspan) in its own key space
                                        // (dictIds of an affine group key, table keys through the remap table)
  int gofs;                             // box index of local key 0 (lbase + key offset - the box start)
  int aoff[kJitMax];                    // per SUM over an affine dictionary: dictId offset into the term space
  unsigned long long ktab;              // group key remap (dictId -> table key id, int32[ktab_n]); 0: affine
  unsigned long long lut[kJitMax];      // DICT_SET bitmaps (uint32 words)
  unsigned long long tab[kJitMax];      // value tables (int64 dictionary values) of the SUMs over a value table
  int lut_words[kJitMax];
  int tab_n[kJitMax];
  int ktab_n;
  unsigned int neg;                     // leaves negated in this segment (bit L; the JIT_LN 2 leaves)
};
struct JitArgs {
  long long total_tiles;
  int nseg, nkeys, key_lo, key_span, xcd_major, pad;
  long long key_stride;                 // table-wide key of box index k: (k + key_lo) * key_stride
  unsigned long long* matched;          // [0] numDocsScanned, [3] matches outside the key box (planner error)
  unsigned long long* count;            // table-wide COUNT accumulators
  long long* sum[kJitMax];              // table-wide SUM accumulators (int64, or lo/hi pairs: sum_long)
  int sum_long[kJitMax];
  long long base[kJitMax], step[kJitMax];  // value = base + step * term
};
static_assert(sizeof(JitSeg) == 48 + 8 + 8 + 48 + 16 + 24 + 8 + 48 + 48 + 24 + 24 + 8, "JitSeg layout");
static_assert(sizeof(JitArgs) == 8 + 24 + 8 + 8 + 8 + 48 + 24 + 48 + 48, "JitArgs layout");

// ---------------------------------------------------------------- pve_jit.hip (count-free partitioned emit)
struct PveSeg {
  unsigned long long src[kJitMax];      // column streams, past the guard words
  long long first_tile;                 // first TD-doc tile in the query's tile space
  int num_docs, num_tiles;
  unsigned int lo_t[kJitMax], hi_t[kJitMax];  // DICT_RANGE leaves: MSB-aligned bounds in this segment's dictId space
  unsigned long long admit;             // PVE_ADMIT: the segment's admitted-key bitmap (limit_walk_kernel; 0 = every key)
  unsigned long long raw;               // PVE_RAWB: the raw value column (padded to whole 2048-doc tiles)
  unsigned long long mv_off;            // PVE_H: int32 value offset of every doc [num_docs + 1]
  unsigned long long mv_words;          // PVE_H: the MV column's value stream (byte-swapped words, past the guard words)
  unsigned long long hlut;              // PVE_H: dictId -> register << 8 | rank
  int koff[kJitMaxGb];                  // group-by component j: table key id = dictId + koff[j] (affine remap)
  unsigned long long ktab[kJitMaxGb];   // group-by component j: dictId -> table key id (PVE_KTAB bit j), else affine
  int voff, vtab_n;                     // value id: table-wide id = dictId + voff, or through vtab (PVE_VTAB)
  unsigned long long vtab;
};
struct PveArgs {
  long long total_tiles;
  int nseg, xcd_major;
  long long chunks_per_wg;              // C: chunk slots of a workgroup's region
  unsigned int* recs;                   // record stream: workgroup g's chunks at [g C SC BS, (g + 1) C SC BS)
  unsigned int* table;                  // [G][C]: partition | (bins - 1) << 12 | rank << 16 of every chunk
  unsigned int* hist;                   // [G][P]: chunks per (workgroup, partition)
  unsigned int* used;                   // [G]: chunks a workgroup filled
  unsigned long long* matched;          // [0] numDocsScanned, [3] region overflow (must stay 0)
};
static_assert(sizeof(PveSeg) == 48 + 8 + 8 + 48 + 40 + 16 + 32 + 8 + 8, "PveSeg layout");
static_assert(sizeof(PveArgs) == 8 + 8 + 8 + 40, "PveArgs layout");
