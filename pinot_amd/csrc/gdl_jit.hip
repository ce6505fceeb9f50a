// The lane-major dense filter + GROUP BY kernel specialised to one query shape (packed accumulation), compiled at
// pa_query_prepare by hiprtc with the shape as macros (pa_jit.hip jit_plan). Same algorithm as pa_gdense.h gdl_tile +
// gdl_packed_accumulate + gdl_drain + gd_flush, with every column width, image offset, leaf kind, field offset and
// loop bound a compile-time constant: no switch on bit widths, no parameter reads in the tile loop, the DMA of a tile
// is straight-line scalar code. Self-contained (hiprtc's built-in HIP headers; pa_jit_abi.h is pasted in by build.py).
//
// Segments with their own dictionaries (every segment builds its own: SegmentDictionaryCreator.java:104, read through
// DictionaryBasedGroupKeyGenerator.java:122) take the same kernel:
//  * column widths per segment: each distinct width tuple is a class (JIT_NCLS <= 4), the tile body and its DMA are
//    instantiated per class and a segment switch picks one (a scalar branch);
//  * the group key: a segment whose dictionary is a contiguous run of the table dictionary (time partitions) shifts its
//    box by an offset; otherwise every segment reads a dictId -> table key table (JIT_KTAB). The packed rows are
//    indexed by the segment's local keys (JitSeg lbase / lspan / gofs), replicated JIT_RR times when few keys per segment
//    leave room (a time partition's handful of days: no same-address atomics), and drained at segment switches;
//  * DICT_SET bitmaps, value tables and key tables that differ per segment live in LDS table slots: a workgroup's tile
//    range spans at most JIT_NSLOT segments, whose tables it loads when it starts; tables every segment shares sit in
//    one shared area;
//  * SUMs over per-segment arithmetic dictionaries with one common step: the rows pack bare dictIds and the drain adds
//    the segment's dictId offset x count (JitSeg.aoff; rows drained at every segment switch);
//  * a leaf negated in some segments only (an empty range becomes NOT(full range)) XORs the segment's bit (JIT_LN 2).
//
// Reference semantics: GroupByOperator -> DefaultGroupByExecutor.process (DefaultGroupByExecutor.java:131-158),
// DictionaryBasedGroupKeyGenerator (one group-by column, :254-340), SumAggregationFunction.aggregateGroupBySV (:207)
// and CountAggregationFunction, ScanBasedFilterOperator over dictId ranges / dictId sets (SVScanDocIdIterator.java:203).
//
// Shape macros (all integers; lists as {a, b, ...}):
//   JIT_W waves per workgroup, JIT_ND docs per lane (a tile is 64 JIT_ND docs), JIT_IMG dwords of one tile image,
//   JIT_NC staged columns, JIT_NCLS width classes, JIT_NB {{bits per column} per class},
//   JIT_OFF {{byte offset of each column's region in the image} per class}
//   JIT_NL eager leaves, JIT_LK {0 = DICT_RANGE, 1 = DICT_SET}, JIT_LC {column}, JIT_LN {0, 1 = negate, 2 = per segment},
//          JIT_LE {closes a CNF clause}, JIT_LUT {LDS byte offset of the DICT_SET bitmap}, JIT_LUTS {1: in the slot}
//   JIT_KC the group-by column, JIT_KL the leaf whose unpack it reuses (-1: none), JIT_KIB the filter implies the box,
//          JIT_KTAB slot byte offset of the group-key table (-1: affine keys)
//   JIT_NA SUM aggregations, JIT_AC {column}, JIT_AT {LDS byte offset of a value table, -1: the dictId itself},
//          JIT_ATS {1: table in the slot}, JIT_AO {1: + the segment's dictId offset, folded in at the drain},
//          JIT_AS {bit offset of the field},
//          JIT_OC bit offset of the COUNT field
//   JIT_DRAIN tiles between drains of a wave's packed rows, JIT_RS waves sharing one set of rows, JIT_RR replicas of
//   JIT_LMAX rows, JIT_SEGDRAIN drains at segment switches
//   JIT_L_SUM {LDS byte offset of each SUM's accumulators}, JIT_L_SLOT / JIT_SLOT_B / JIT_NSLOT the table slots,
//   JIT_L_ROWS, JIT_L_RING (LDS byte offsets)
typedef unsigned int u32;
typedef unsigned long long u64;
typedef long long i64;
typedef __attribute__((address_space(3))) u32 l32;
typedef __attribute__((address_space(3))) u64 l64;

#include "pa_jit_abi.h"

#ifndef JIT_RS
#define JIT_RS 1  // waves sharing one set of packed rows (2: half the rows' LDS, drained by atomic exchange)
#endif
#ifndef JIT_RR
#define JIT_RR 1  // replicas of each row: lane l updates replica l % JIT_RR (few keys per segment: no same-address atomics)
#endif
#ifndef JIT_LMAX
#define JIT_LMAX 1  // rows (keys) per replica: the largest number of box keys one segment holds
#endif
#ifndef JIT_SEGDRAIN
#define JIT_SEGDRAIN 0  // the rows are drained at every segment switch (their local keys / offsets change there)
#endif
#ifndef JIT_DBG
#define JIT_DBG 0  // measurement only (PA_GDL_DBG; results invalid): 1 = stream the tiles only, 2 = + the filter,
#endif             // 3 = + keys and packed terms (no row atomics)
#ifndef JIT_RING
#define JIT_RING 2  // tile images per wave: JIT_RING - 1 tiles in flight while one is walked
#endif
constexpr int W = JIT_W, NC = JIT_NC, NL = JIT_NL, NA = JIT_NA, ND = JIT_ND, IMG = JIT_IMG, NCLS = JIT_NCLS;
constexpr int R = JIT_RING;
static_assert(R >= 2 && R <= 4, "2..4 tile images per wave");
static_assert(JIT_RS == 1 || JIT_RS == 2, "rows shared by 1 or 2 waves");
static_assert(JIT_RR >= 1 && JIT_RR <= 64 && (JIT_RR & (JIT_RR - 1)) == 0, "1..64 row replicas, a power of two");
constexpr int kRRLog = JIT_RR >= 64 ? 6 : JIT_RR >= 32 ? 5 : JIT_RR >= 16 ? 4 : JIT_RR >= 8 ? 3 : JIT_RR >= 4 ? 2
                                                                                      : JIT_RR >= 2 ? 1 : 0;
constexpr int TD = 64 * ND;                // docs per tile (lane l: docs [ND l, ND l + ND))
constexpr u32 FULL = (1u << ND) - 1u;      // the lane's match word of a whole tile
static_assert(ND == 8 || ND == 16, "8 or 16 docs per lane");
static_assert(NCLS >= 1 && NCLS <= 4, "1..4 width classes");
constexpr int NLA = NL > 0 ? NL : 1, NAA = NA > 0 ? NA : 1;
constexpr int kNB[NCLS][NC] = JIT_NB;
constexpr int kOFF[NCLS][NC] = JIT_OFF;
constexpr int kLK[NLA] = JIT_LK;
constexpr int kLC[NLA] = JIT_LC;
constexpr int kLN[NLA] = JIT_LN;
constexpr int kLE[NLA] = JIT_LE;
constexpr int kLUT[NLA] = JIT_LUT;
constexpr int kLUTS[NLA] = JIT_LUTS;
constexpr int kAC[NAA] = JIT_AC;
constexpr int kAT[NAA] = JIT_AT;
constexpr int kATS[NAA] = JIT_ATS;
constexpr int kAO[NAA] = JIT_AO;
constexpr int kAS[NAA] = JIT_AS;
constexpr int kLSUM[NAA] = JIT_L_SUM;
static_assert(NC <= kJitMax && NL <= kJitMax && NA <= kJitMax, "shape beyond the JIT descriptors");

typedef const __attribute__((address_space(4))) JitArgs CA;
typedef const __attribute__((address_space(4))) JitSeg CS;

__device__ __forceinline__ u32 lds_addr(const void* p) { return (u32)(unsigned long)(const l32*)p; }
template <class T>
__device__ __forceinline__ T* at(u32 a) { return (T*)(unsigned long)a; }

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// LDS-DMA with a scalar base: lane l copies 16 bytes at sbase + voff to dst + 16 l (mask: the taking-part lanes)
__device__ __forceinline__ void dma16(u32 voff, u64 sbase, u32 dst) {
  u32 keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(dst));
}
__device__ __forceinline__ void dma16m(u32 voff, u64 sbase, u32 dst, u64 mask) {
  u32 keep;
  u64 save;
  asm volatile(
      "s_mov_b64 %1, exec\n\ts_mov_b64 exec, %5\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0\n\ts_mov_b64 exec, %1"
      : "=&s"(keep), "=&s"(save) : "v"(voff), "s"(sbase), "s"(dst), "s"(mask));
}

// tile wt of every column of class K: 8 ND nb bytes per column, as 16-byte chunks
template <int K, int C>
__device__ __forceinline__ void dma_cols(CS* sg, i64 wt, u32 img, u32 voff) {
  if constexpr (C < NC) {
    constexpr int NB = kNB[K][C];
    constexpr int CH = ND * NB / 2;  // 16-byte chunks of a tile
    const u64 src = sg->src[C] + (u64)wt * (u64)(8 * ND * NB);
    const u32 dst = img + (u32)kOFF[K][C];
#pragma unroll
    for (int k = 0; k < CH / 64; ++k) dma16(voff, src + 1024u * k, dst + 1024u * k);
    if constexpr (CH % 64) dma16m(voff, src + 1024u * (CH / 64), dst + 1024u * (CH / 64), (1ull << (CH % 64)) - 1ull);
    dma_cols<K, C + 1>(sg, wt, img, voff);
  }
}
// wave DMA instructions of one tile of class K, and the fewest over the classes (a wait for "every tile but the
// R - 2 youngest" counts that many per younger tile: a class with more only makes the wait conservative)
template <int K>
constexpr int dma_instrs() {
  int n = 0;
  for (int c = 0; c < NC; ++c) n += (ND * kNB[K][c] / 2 + 63) / 64;
  return n;
}
constexpr int dma_min() {
  int n = dma_instrs<0>();
  if (NCLS > 1 && dma_instrs<(NCLS > 1 ? 1 : 0)>() < n) n = dma_instrs<(NCLS > 1 ? 1 : 0)>();
  if (NCLS > 2 && dma_instrs<(NCLS > 2 ? 2 : 0)>() < n) n = dma_instrs<(NCLS > 2 ? 2 : 0)>();
  if (NCLS > 3 && dma_instrs<(NCLS > 3 ? 3 : 0)>() < n) n = dma_instrs<(NCLS > 3 ? 3 : 0)>();
  return n;
}
constexpr int kDmaMin = dma_min();

template <int K>
__device__ __forceinline__ void dma_tile(int cls, CS* sg, i64 wt, u32 img, u32 voff) {
  if constexpr (K + 1 < NCLS) {
    if (cls == K) dma_cols<K, 0>(sg, wt, img, voff);
    else dma_tile<K + 1>(cls, sg, wt, img, voff);
  } else {
    dma_cols<K, 0>(sg, wt, img, voff);
  }
}

// The lane's ND values of an NB-bit column from its region of the image, as whole 32-bit windows: w[j] holds the
// stream bits [bit0 + 32 j, bit0 + 32 j + 32) (MSB first), bit0 = the lane's first bit
template <int NB>
__device__ __forceinline__ void lane_words(u32 region, int lane, u32 (&w)[(ND * NB + 31) / 32 + 1]) {
  constexpr int K = (ND * NB + 31) / 32 + 1;
  const u32 bit0 = (u32)lane * (u32)(ND * NB);
  if constexpr ((ND * NB) % 32 != 0) {  // the lane starts inside a word: windows through alignbit
    const u32 sh = bit0 & 31u;
    const u32 lo_shift = (32u - sh) & 31u;  // sh 0: the word itself (alignbit by 0 of the next pair)
    const l32* p = at<const l32>(region + 4u * ((bit0 >> 5) - 1u + (sh != 0u ? 1u : 0u)));
    u32 r[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) r[j] = p[j];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = __builtin_amdgcn_alignbit(r[j], r[j + 1], lo_shift);
  } else {
    const l32* p = at<const l32>(region + 4u * (bit0 >> 5));
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = p[j];
  }
}

// The lane's ND values of column C (class K), MSB-aligned: value i in the top NB bits of v[i]
template <int K, int C>
__device__ __forceinline__ void top(u32 img, int lane, u32 (&v)[ND]) {
  constexpr int NB = kNB[K][C];
  u32 w[(ND * NB + 31) / 32 + 1];
  lane_words<NB>(img + (u32)kOFF[K][C], lane, w);
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    v[i] = (o + NB <= 32) ? (w[j] << o) : __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o);
  }
}

// dictIds of column C (one v_bfe per id, two ops when it straddles words)
template <int K, int C>
__device__ __forceinline__ void ids(u32 img, int lane, u32 (&v)[ND]) {
  constexpr int NB = kNB[K][C];
  u32 w[(ND * NB + 31) / 32 + 1];
  lane_words<NB>(img + (u32)kOFF[K][C], lane, w);
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    if (o + NB <= 32) v[i] = __builtin_amdgcn_ubfe(w[j], 32 - o - NB, NB);
    else v[i] = __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o) >> (32 - NB);
  }
}

// MSB-aligned range test of ND values: non-matches as borrow bits (lo <= v < lo + span <=> t - lo' <= hi')
__device__ __forceinline__ u32 range_nm(const u32 (&t)[ND], u32 lo_t, u32 hi_t) {
  u32 nm = 0;
#pragma unroll
  for (int i = ND - 1; i >= 0; --i) {
    u32 u;
    asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\tv_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
        "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
        : [nm] "+v"(nm), [u] "=&v"(u) : [t] "v"(t[i]), [lo] "s"(lo_t), [hi] "s"(hi_t) : "vcc");
  }
  return nm;
}

// eager leaves L.. in order (CNF clauses closed by kLE); false when no doc of the wave's tile can match any more
template <int K, int L>
__device__ __forceinline__ bool leaves(CS* sg, u32 img, int lane, u32 base, u32 tb, u32& m, u32& clause,
                                       u32 (&kt)[ND]) {
  if constexpr (L < NL) {
    u32 t[ND];
    top<K, kLC[L]>(img, lane, t);
    if constexpr (L == JIT_KL) {
#pragma unroll
      for (int i = 0; i < ND; ++i) kt[i] = t[i];
    }
    u32 bits;
    if constexpr (kLK[L] == 0) {
      bits = ~range_nm(t, sg->lo_t[L], sg->hi_t[L]) & FULL;
    } else {
      constexpr int NB = kNB[K][kLC[L]];
      const u32 lb = (kLUTS[L] ? tb : base) + (u32)kLUT[L];
      u32 id[ND], w[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        id[i] = t[i] >> (32 - NB);
        w[i] = *at<const l32>(lb + 4u * (id[i] >> 5));
      }
      bits = 0;
#pragma unroll
      for (int i = 0; i < ND; ++i) bits |= __builtin_amdgcn_ubfe(w[i], id[i], 1) << i;
    }
    if constexpr (kLN[L] == 1) bits = ~bits & FULL;
    if constexpr (kLN[L] == 2) bits ^= (0u - ((sg->neg >> L) & 1u)) & FULL;
    clause |= bits;
    if constexpr (kLE[L] != 0) {
      m &= clause;
      clause = 0;
      if (__builtin_amdgcn_ballot_w64(m != 0) == 0) return false;
    }
    return leaves<K, L + 1>(sg, img, lane, base, tb, m, clause, kt);
  }
  return true;
}

// packed words of the lane's docs: COUNT + the SUM terms, ORed into their fields 32 bits at a time
template <int K, int A>
__device__ __forceinline__ void terms(CS* sg, u32 img, int lane, u32 base, u32 tb, u32 (&plo)[ND], u32 (&phi)[ND]) {
  if constexpr (A < NA) {
    u32 id[ND];
    ids<K, kAC[A]>(img, lane, id);
    if constexpr (kAT[A] >= 0) {
      const u32 ab = (kATS[A] ? tb : base) + (u32)kAT[A];
#pragma unroll
      for (int i = 0; i < ND; ++i) id[i] = *at<const l32>(ab + 4u * id[i]);
    }
    constexpr int SH = kAS[A];
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      if constexpr (SH >= 32) {
        phi[i] |= id[i] << (SH - 32);
      } else if constexpr (SH == 0) {
        plo[i] |= id[i];
      } else {
        plo[i] |= id[i] << SH;
        phi[i] |= id[i] >> (32 - SH);
      }
    }
    terms<K, A + 1>(sg, img, lane, base, tb, plo, phi);
  }
}

// one tile of class K: returns the lane's docs counted in numDocsScanned
template <int K>
__device__ __forceinline__ u32 tile(CS* sg, i64 wt, u32 img, int lane, u32 base, u32 tb, u32 rows, u32& errs) {
  if constexpr (JIT_DBG == 1) return 0;
  const i64 rem = (i64)sg->num_docs - wt * TD;
  u32 m = FULL;
  if (rem < TD) {
    const i64 n = rem - ND * lane;
    m = n >= ND ? FULL : (n <= 0 ? 0u : ((1u << n) - 1u));
  }
  u32 clause = 0, kt[ND];
  if (!leaves<K, 0>(sg, img, lane, base, tb, m, clause, kt)) return 0;
  if (__builtin_amdgcn_ballot_w64(m != 0) == 0) return 0;
  if constexpr (JIT_DBG == 2) return (u32)__builtin_popcount(m);
  if constexpr (JIT_DBG == 3) {  // (measurement: keys and terms built and kept live, no row atomics)
    u32 id[ND], plo[ND], phi[ND];
    ids<K, JIT_KC>(img, lane, id);
#pragma unroll
    for (int i = 0; i < ND; ++i) plo[i] = phi[i] = 0u;
    terms<K, 0>(sg, img, lane, base, tb, plo, phi);
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < ND; ++i) x ^= ((m >> i) & 1u) ? id[i] + plo[i] + phi[i] : 0u;
    if (x == 0x9e3779b9u) *at<l32>(rows) = x;
    return (u32)__builtin_popcount(m);
  }
  constexpr int NBK = kNB[K][JIT_KC];
  u32 id[ND];
  if constexpr (JIT_KL >= 0) {
#pragma unroll
    for (int i = 0; i < ND; ++i) id[i] = kt[i] >> (32 - NBK);
  } else {
    ids<K, JIT_KC>(img, lane, id);
  }
  if constexpr (JIT_KTAB >= 0) {  // dictId -> table key id
#pragma unroll
    for (int i = 0; i < ND; ++i) id[i] = *at<const l32>(tb + (u32)JIT_KTAB + 4u * id[i]);
  }
  // the segment's local key = key - lbase, kept when below lspan (the box check); row entry local * JIT_RR + replica
  const u32 klo = (u32)sg->lbase, span_m1 = (u32)sg->lspan - 1u;
  u32 on = m;
  if constexpr (!JIT_KIB) {
    u32 nm = 0;
#pragma unroll
    for (int i = ND - 1; i >= 0; --i) {
      u32 u;
      asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\tv_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
          "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
          : [nm] "+v"(nm), [u] "=&v"(u) : [t] "v"(id[i]), [lo] "s"(klo), [hi] "s"(span_m1) : "vcc");
    }
    on &= ~nm;
    errs += (u32)__builtin_popcount(m & ~on);
  }
  const u32 abase = rows + 8u * ((u32)lane & (u32)(JIT_RR - 1)) - (klo << (3 + kRRLog));
  u32 plo[ND], phi[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    plo[i] = JIT_OC < 32 ? (1u << (JIT_OC & 31)) : 0u;
    phi[i] = JIT_OC < 32 ? 0u : (1u << ((JIT_OC - 32) & 31));
  }
  terms<K, 0>(sg, img, lane, base, tb, plo, phi);
#pragma unroll
  for (int i = 0; i < ND; ++i)
    if ((on >> i) & 1u)
      __hip_atomic_fetch_add(at<l64>(abase + (id[i] << (3 + kRRLog))), ((u64)phi[i] << 32) | plo[i], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  return (u32)__builtin_popcount(m);
}
template <int K>
__device__ __forceinline__ u32 tile_any(int cls, CS* sg, i64 wt, u32 img, int lane, u32 base, u32 tb, u32 rows,
                                        u32& errs) {
  if constexpr (K + 1 < NCLS) {
    if (cls == K) return tile<K>(sg, wt, img, lane, base, tb, rows, errs);
    return tile_any<K + 1>(cls, sg, wt, img, lane, base, tb, rows, errs);
  } else {
    return tile<K>(sg, wt, img, lane, base, tb, rows, errs);
  }
}

// a wave's packed rows -> the workgroup's COUNT / SUM accumulators (rows zeroed; rows shared by two waves are taken by
// atomic exchange, the other wave may be adding to them). Entry e = local key (e / JIT_RR) x replica: the replicas of a
// key lie in aligned groups of lanes, unpacked one by one (fields of different replicas cannot be added packed) and
// reduced across the group before one atomic per key goes to the box accumulators at gofs + local key. A SUM over
// per-segment arithmetic dictionaries (kAO) packs bare dictIds: the rows hold one segment's docs at a time (drained at
// every segment switch), so the segment's dictId offset enters here as offset x count.
__device__ __forceinline__ void drain(u32 rows, int lane, u32 base, CS* sg) {
  l64* row = at<l64>(rows);
  u64 ao[NAA];
#pragma unroll
  for (int a = 0; a < NA; ++a) ao[a] = kAO[a] ? (u64)(u32)sg->aoff[a] : 0ull;
  const int ne = sg->lspan << kRRLog;
  const int gofs = sg->gofs;
  for (int e0 = 0; e0 < ne; e0 += 64) {
    const int e = e0 + lane;
    u64 x = 0;
    if (e < ne) {
      x = row[e];
      if (x != 0) {
        if constexpr (JIT_RS > 1) x = __hip_atomic_exchange(row + e, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else row[e] = 0;
      }
    }
    u64 cnt = x >> JIT_OC;
    u64 f[NAA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int lo = kAS[a], hi = a + 1 < NA ? kAS[a + 1 < NA ? a + 1 : a] : JIT_OC;
      f[a] = (x >> lo) & ((hi - lo) >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull));
      if (kAO[a]) f[a] += ao[a] * cnt;
    }
#pragma unroll
    for (int o = 1; o < JIT_RR; o <<= 1) {
      cnt += __shfl_xor(cnt, o);
#pragma unroll
      for (int a = 0; a < NA; ++a) f[a] += __shfl_xor(f[a], o);
    }
    if ((lane & (JIT_RR - 1)) == 0 && cnt != 0) {
      const int k = gofs + (e >> kRRLog);
      __hip_atomic_fetch_add(at<l32>(base) + k, (u32)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int a = 0; a < NA; ++a)
        __hip_atomic_fetch_add(at<l64>(base + (u32)kLSUM[a]) + k, f[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}
constexpr bool kAnyAO = [] {
  for (int a = 0; a < NA; ++a)
    if (kAO[a]) return true;
  return false;
}();
static_assert(!kAnyAO || (JIT_RS == 1 && JIT_SEGDRAIN), "per-segment offsets need private rows drained per segment");

__device__ __forceinline__ int find_segment(CS* segs, int nseg, i64 t) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].first_tile <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// one segment's tables into an LDS area (slot = its per-segment tables, else the shared ones)
__device__ __forceinline__ void load_tables(CA* A, CS* sg, u32 dst, bool slot, int tid) {
  typedef const __attribute__((address_space(1))) u32 g32;
  typedef const __attribute__((address_space(1))) i64 g64;
#pragma unroll
  for (int l = 0; l < NL; ++l)
    if (kLK[l] == 1 && (kLUTS[l] != 0) == slot)
      for (int i = tid; i < sg->lut_words[l]; i += W * 64) at<l32>(dst + (u32)kLUT[l])[i] = ((g32*)sg->lut[l])[i];
#pragma unroll
  for (int a = 0; a < NA; ++a)
    if (kAT[a] >= 0 && (kATS[a] != 0) == slot)
      for (int i = tid; i < sg->tab_n[a]; i += W * 64)
        at<l32>(dst + (u32)kAT[a])[i] = (u32)(((g64*)sg->tab[a])[i] - A->base[a]);
  if (JIT_KTAB >= 0 && slot)
    for (int i = tid; i < sg->ktab_n; i += W * 64)
      at<l32>(dst + (u32)(JIT_KTAB >= 0 ? JIT_KTAB : 0))[i] = ((g32*)sg->ktab)[i];
}

extern "C" __global__ void __launch_bounds__(W * 64, 1) gdl_jit(const JitArgs* a_in, const JitSeg* s_in) {
  CA* A = (CA*)(unsigned long)a_in;
  CS* S = (CS*)(unsigned long)s_in;
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const u32 base = lds_addr(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkeys = A->nkeys;
  // LDS: counts, sums, shared tables, table slots, the waves' packed rows, the ring
  for (int i = tid; i < nkeys; i += W * 64) smem[i] = 0u;
#pragma unroll
  for (int a = 0; a < NA; ++a)
    for (int i = tid; i < nkeys; i += W * 64) at<l64>(base + (u32)kLSUM[a])[i] = 0ull;
  for (int i = tid; i < (W / JIT_RS) * JIT_LMAX * JIT_RR; i += W * 64) at<l64>(base + (u32)JIT_L_ROWS)[i] = 0ull;
  const i64 T = A->total_tiles, G = gridDim.x;
  const i64 b = blockIdx.x;
  const i64 lb = A->xcd_major ? (b % 8) * (G / 8) + (b % 8 < G % 8 ? b % 8 : G % 8) + b / 8 : b;
  const i64 t0 = lb * T / G, t1 = (lb + 1) * T / G;
  const int nseg = A->nseg;
  // the segments this workgroup's tiles cover: their tables into the slots (the planner sized JIT_NSLOT for them)
  const int s_first = t0 < t1 ? find_segment(S, nseg, t0) : 0;
  load_tables(A, S + s_first, base, false, tid);
#pragma unroll
  for (int k = 0; k < JIT_NSLOT; ++k) {
    const int si = s_first + k;
    if (t0 < t1 && si < nseg && S[si].first_tile < t1)
      load_tables(A, S + si, base + (u32)JIT_L_SLOT + (u32)(k * JIT_SLOT_B), true, tid);
  }
  __syncthreads();
  const u32 rows = base + (u32)JIT_L_ROWS + (u32)(wave / JIT_RS) * (u32)(JIT_LMAX * JIT_RR) * 8u;
  const u32 ring = base + (u32)JIT_L_RING + (u32)wave * (u32)R * (u32)IMG * 4u;
  const u32 voff = 16u * (u32)lane;
  u32 matched = 0, errs = 0;
  if (t0 < t1) {
    int isi = find_segment(S, nseg, t0 + wave);
    int psi = isi;
    i64 ifirst = S[isi].first_tile, iend = ifirst + S[isi].num_tiles;
    i64 pfirst = ifirst, pend = iend;
    int icls = S[isi].cls, pcls = icls;
    u32 tb = base + (u32)JIT_L_SLOT + (u32)((psi - s_first) * JIT_SLOT_B);
    i64 ti = t0 + wave;
    auto issue = [&](int to) {  // the wave's next tile into image slot `to`
      if (ti < t1) {
        while (ti >= iend) {
          ++isi;
          ifirst = S[isi].first_tile;
          iend = ifirst + S[isi].num_tiles;
          icls = S[isi].cls;
        }
        dma_tile<0>(icls, S + isi, ti - ifirst, ring + (u32)to * (u32)IMG * 4u, voff);
      }
      ti += W;
    };
#pragma unroll
    for (int k = 0; k + 1 < R; ++k) issue(k);
    int slot = 0, since = 0;
    for (i64 t = t0 + wave; t < t1; t += W) {
      // tile t has landed: the R - 2 tiles after it may stay in flight when they were all issued
      if (R > 2 && t + (i64)(R - 2) * W < t1) vm_wait<(R > 2 ? (R - 2) * kDmaMin : 0)>();
      else vm_wait<0>();
      issue(slot == 0 ? R - 1 : slot - 1);  // (the image walked last)
      while (t >= pend) {
        if constexpr (JIT_SEGDRAIN) {  // (the rows hold the segment's local keys only)
          drain(rows, lane, base, S + psi);
          since = 0;
        }
        ++psi;
        pfirst = S[psi].first_tile;
        pend = pfirst + S[psi].num_tiles;
        pcls = S[psi].cls;
        tb = base + (u32)JIT_L_SLOT + (u32)((psi - s_first) * JIT_SLOT_B);
      }
      matched += tile_any<0>(pcls, S + psi, t - pfirst, ring + (u32)slot * (u32)IMG * 4u, lane, base, tb, rows, errs);
      if (++since == JIT_DRAIN) {
        drain(rows, lane, base, S + psi);
        since = 0;
      }
      slot = slot + 1 == R ? 0 : slot + 1;
    }
    vm_wait<0>();
    drain(rows, lane, base, S + psi);
  }
  u64 wm = matched, we = errs;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    wm += __shfl_xor(wm, o);
    we += __shfl_xor(we, o);
  }
  if (lane == 0 && wm) __hip_atomic_fetch_add(A->matched, wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0 && we) __hip_atomic_fetch_add(A->matched + 3, we, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  // flush: one global update per non-empty key and aggregation (gd_flush for one group-by column)
  for (int kl = tid; kl < nkeys; kl += W * 64) {
    const u64 c = smem[kl];
    if (c == 0) continue;
    const i64 key = ((i64)kl + A->key_lo) * A->key_stride;
    __hip_atomic_fetch_add(A->count + key, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const u64 s = at<l64>(base + (u32)kLSUM[a])[kl];
      const __int128 tot = (__int128)A->base[a] * (__int128)c + (__int128)A->step[a] * (__int128)s;
      unsigned long long* acc = (unsigned long long*)A->sum[a];
      if (A->sum_long[a]) {
        __hip_atomic_fetch_add(acc + 2 * key, (u64)tot & 0xffffffffull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(acc + 2 * key + 1, (u64)(i64)(tot >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_fetch_add(acc + key, (u64)(i64)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}
