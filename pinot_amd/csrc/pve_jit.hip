// The partitioned aggregation's V emit pass without a count pass, specialised to one query shape (configs[2]-like:
// dictionary group-by columns, one dictionary value column or none, DICT_RANGE filter leaves), compiled at
// pa_query_prepare by hiprtc with the shape as macros (pa_capi.hip pve_*). Self-contained (hiprtc built-ins only).
//
// Reference semantics: DictionaryBasedGroupKeyGenerator raw keys (DictionaryBasedGroupKeyGenerator.java:254-340) over
// the table-wide key space, the records feeding pass C's SUM / MIN / MAX / COUNT (part_agg_v_fast), the filter as
// ScanBasedFilterOperator over dictId ranges (SVScanDocIdIterator.java:203).
//
// Each workgroup walks its tile range lane-major (lane l: docs [16 l, 16 l + 16) of a 1024-doc tile, unpacked from its
// own words of the tile image — no per-doc LDS gather), builds one-word records (key offset in its partition | value id
// << kshift) and puts them into per-partition LDS bins of BS records (claim a slot, write it, count it written; the lane
// that completes a bin stores it). A full bin goes to the next free BS-record chunk of the workgroup's own region in the
// record stream (an LDS counter: no count pass, no global atomic), and the chunk table records (partition, rank of the
// chunk among the workgroup's chunks of that partition). At the end the partial bins leave as chunks padded with
// sentinels, and the workgroup writes its chunks per partition; pa_pve.hip then lays out every partition's chunk list
// and pass C reads records through it.
//
// Shape macros (lists as {a, b, ...}):
//   PVE_W waves per workgroup   PVE_IMG dwords of one tile image   PVE_NC staged columns
//   PVE_NB {bits per column}    PVE_OFF {byte offset of each column's region in the image}
//   PVE_NL filter leaves (DICT_RANGE), PVE_LC {column}, PVE_LN {negate}, PVE_LE {closes a CNF clause}
//   PVE_NG group-by columns, PVE_GC {column}, PVE_GS {key stride}
//   PVE_VC the value column (-1: none)   PVE_KS key bits inside a partition   PVE_P partitions   PVE_BS bin records
//   PVE_KR keys per V partition when not 1 << PVE_KS (0: 1 << PVE_KS; else partition = key / PVE_KR, a constant divisor)
//   PVE_SC bins per chunk (a chunk is SC x BS consecutive records of one partition: pass C reads long runs)
//   PVE_L_BINS, PVE_L_RING LDS byte offsets (state at 0: cnt[P], done[P], chunks[P], cur[P], fill[P], next)
//   PVE_RW record words, PVE_RAWB / PVE_RAWOFF the staged raw value column, PVE_H the H stream (PVE_HNB, PVE_LG,
//   PVE_L_VAL / PVE_VAL_B: per-wave LDS buffers of the tile's MV value words)
//   PVE_HRUN / PVE_HB the H stream's run rounds: one claim per run of up to PVE_HB values of one doc
//   PVE_KOFF / PVE_VOFF segments with their own dictionaries, each a contiguous run of the table-wide dictionary: the
//   segment's offsets into the table key ids / value ids (PveSeg.koff, voff)
typedef unsigned int u32;
typedef unsigned long long u64;
typedef long long i64;
typedef __attribute__((address_space(3))) u32 l32;

#include "pa_jit_abi.h"  // PveSeg, PveArgs (one definition with the host)

#ifndef PVE_ND
#define PVE_ND 16
#endif
constexpr int W = PVE_W, NC = PVE_NC, NL = PVE_NL, NG = PVE_NG, ND = PVE_ND, IMG = PVE_IMG;
constexpr int TD = 64 * ND;  // docs per tile (lane l: docs [ND l, ND l + ND))
static_assert(ND == 8 || ND == 16, "8 or 16 docs per lane");
constexpr int NLA = NL > 0 ? NL : 1;
constexpr int kNB[NC] = PVE_NB;
constexpr int kOFF[NC] = PVE_OFF;
constexpr int kLC[NLA] = PVE_LC;
constexpr int kLN[NLA] = PVE_LN;
constexpr int kLE[NLA] = PVE_LE;
constexpr int kGC[NG] = PVE_GC;
constexpr u32 kGS[NG] = PVE_GS;
constexpr int VC = PVE_VC, KS = PVE_KS, P = PVE_P, BS = PVE_BS, SC = PVE_SC;
#ifndef PVE_KR
#define PVE_KR 0
#endif
constexpr u32 KR = PVE_KR, KRD = KR ? KR : 1u;
static_assert(KR <= (1u << KS), "a partition's key offsets fit KS bits");
constexpr u32 kSentinel = 0xffffffffu;
#ifndef PVE_PB
#define PVE_PB 4  // records per lane per put round
#endif
#ifndef PVE_ADMIT
#define PVE_ADMIT 0  // numGroupsLimit walk form: a record is put only when the segment's bitmap admits its key
#endif
#ifndef PVE_DBG
#define PVE_DBG 0  // measurement only (PA_PVE_DBG): 1 = records built but not put, 2 = full bins not stored
#endif
#ifndef PVE_DONE_RTN
#define PVE_DONE_RTN 0  // measurement (PA_PVE_DONE_RTN): the written count's returned value decides a bin is full
#endif
#ifndef PVE_RW
#define PVE_RW 1  // words per record: 1 (key offset | value id), 2 (+ a raw 32-bit value), 3 (+ a raw 64-bit value)
#endif
#ifndef PVE_RAWB
#define PVE_RAWB 0  // bytes per doc of the raw value column staged at PVE_RAWOFF (0: none; 4 with PVE_RW 2, 8 with 3)
#endif
#ifndef PVE_RAWOFF
#define PVE_RAWOFF 0
#endif
#ifndef PVE_H
#define PVE_H 0  // the H stream: one record per value of the DISTINCTCOUNTHLLMV column (PVE_HNB bits per dictId,
#endif           // PVE_LG = log2m): key offset << (LG + 6) | register << 6 | rank << 1
#ifndef PVE_HNB
#define PVE_HNB 1
#endif
#ifndef PVE_L_VAL
#define PVE_L_VAL 0  // H: LDS byte offset of the waves' value buffers, PVE_VAL_B bytes each
#endif
#ifndef PVE_VAL_B
#define PVE_VAL_B 0
#endif
#ifndef PVE_LG
#define PVE_LG 0
#endif
#ifndef PVE_KOFF
#define PVE_KOFF 0  // segments with their own dictionaries: table key id of component j = dictId + PveSeg.koff[j]
#endif
#ifndef PVE_VOFF
#define PVE_VOFF 0  // the value column's table-wide value id = dictId + PveSeg.voff
#endif
#ifndef PVE_Q
#define PVE_Q 0  // compacted put rounds: a wave queues its records in LDS, each put round takes 64 PB of them
#endif
#ifndef PVE_L_Q
#define PVE_L_Q 0  // LDS byte offset of the waves' queues (PVE_QB bytes each)
#endif
#ifndef PVE_HRUN
#define PVE_HRUN 0  // H: one claim per run of up to PVE_HB values of one doc (they share the doc's key, so its partition)
#endif
#ifndef PVE_HB
#define PVE_HB 4
#endif
#ifndef PVE_RING
#define PVE_RING 2  // tile images per wave (V streams without admission loads: RING - 1 tiles in flight)
#endif
constexpr int RW = PVE_RW, RAWB = PVE_RAWB, HNB = PVE_HNB, LG = PVE_LG;
// (the H stream's value words and the admission bitmap loads are waited for with the image DMA counted in: two images)
constexpr int R = (PVE_H || PVE_ADMIT) ? 2 : PVE_RING;
static_assert(R >= 2 && R <= 4, "2..4 tile images per wave");
static_assert(RW >= 1 && RW <= 3 && (RAWB == 0 || RAWB == 4 * (RW - 1)), "record words and the raw column agree");
static_assert(!PVE_H || (RW == 1 && PVE_VC < 0 && RAWB == 0), "the H stream has one-word records");

static_assert(NC <= kJitMax && NL <= kJitMax && NG <= kJitMaxGb, "shape beyond the JIT descriptors");
static_assert(BS % 4 == 0, "bins are whole 16-byte units");
typedef const __attribute__((address_space(4))) PveArgs CA;
typedef const __attribute__((address_space(4))) PveSeg CS;

__device__ __forceinline__ u32 lds_addr(const void* p) { return (u32)(unsigned long)(const l32*)p; }
template <class T>
__device__ __forceinline__ T* at(u32 a) { return (T*)(unsigned long)a; }

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

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

// wave DMA instructions of one tile image (dma_cols)
constexpr int dma_instrs() {
  int n = 0;
  for (int c = 0; c < NC; ++c) n += (ND * kNB[c] / 2 + 63) / 64;
  return n + TD * RAWB / 16 / 64;
}
constexpr int kDmaImg = dma_instrs();

template <int C>
__device__ __forceinline__ void dma_cols(CS* sg, i64 wt, u32 img, u32 voff) {
  if constexpr (C < NC) {
    constexpr int CH = ND * kNB[C] / 2;  // 16-byte chunks of a tile (TD nb / 128)
    const u64 src = sg->src[C] + (u64)wt * (u64)(8 * ND * kNB[C]);
    const u32 dst = img + (u32)kOFF[C];
#pragma unroll
    for (int k = 0; k < CH / 64; ++k) dma16(voff, src + 1024u * k, dst + 1024u * k);
    if constexpr (CH % 64) dma16m(voff, src + 1024u * (CH / 64), dst + 1024u * (CH / 64), (1ull << (CH % 64)) - 1ull);
    dma_cols<C + 1>(sg, wt, img, voff);
  } else if constexpr (RAWB > 0) {
    constexpr int CH = TD * RAWB / 16;  // (a multiple of 64: whole wave instructions)
    const u64 src = sg->raw + (u64)wt * (u64)(TD * RAWB);
    const u32 dst = img + (u32)PVE_RAWOFF;
#pragma unroll
    for (int k = 0; k < CH / 64; ++k) dma16(voff, src + 1024u * k, dst + 1024u * k);
  }
}

// the lane's ND values of column C, MSB-aligned (top) or as dictIds. The lane's bits start sh bits into a word: its
// words are read from one word earlier when sh == 0 so that alignbit by (32 - sh) & 31 realigns every case
template <int C, bool TOP>
__device__ __forceinline__ void unpack(u32 img, int lane, u32 (&v)[ND]) {
  constexpr int NB = kNB[C];
  constexpr int K = (ND * NB + 31) / 32 + 1;
  const u32 region = img + (u32)kOFF[C];
  const u32 bit0 = (u32)lane * (u32)(ND * NB);
  u32 w[K];
  if constexpr ((ND * NB) % 32 != 0) {
    const u32 sh = bit0 & 31u;
    const l32* p = at<const l32>(region + 4u * ((bit0 >> 5) - (sh == 0u ? 1u : 0u)));
    u32 r[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) r[j] = p[j];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = __builtin_amdgcn_alignbit(r[j], r[j + 1], (32u - sh) & 31u);
  } else {
    const l32* p = at<const l32>(region + 4u * (bit0 >> 5));
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = p[j];
  }
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    if constexpr (TOP) {
      v[i] = (o + NB <= 32) ? (w[j] << o) : __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o);
    } else {
      if (o + NB <= 32) v[i] = __builtin_amdgcn_ubfe(w[j], 32 - o - NB, NB);
      else v[i] = __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o) >> (32 - NB);
    }
  }
}

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

template <int L>
__device__ __forceinline__ bool leaves(CS* sg, u32 img, int lane, u32& m, u32& clause) {
  if constexpr (L < NL) {
    u32 t[ND];
    unpack<kLC[L], true>(img, lane, t);
    constexpr u32 kAll = (1u << ND) - 1u;
    u32 bits = ~range_nm(t, sg->lo_t[L], sg->hi_t[L]) & kAll;
    if constexpr (kLN[L]) bits = ~bits & kAll;
    clause |= bits;
    if constexpr (kLE[L] != 0) {
      m &= clause;
      clause = 0;
      if (__builtin_amdgcn_ballot_w64(m != 0) == 0) return false;
    }
    return leaves<L + 1>(sg, img, lane, m, clause);
  }
  return true;
}

template <int G>
__device__ __forceinline__ void keys(u32 img, int lane, u32 (&key)[ND]) {
  if constexpr (G < NG) {
    u32 id[ND];
    unpack<kGC[G], false>(img, lane, id);
#pragma unroll
    for (int i = 0; i < ND; ++i) key[i] += id[i] * kGS[G];
    keys<G + 1>(img, lane, key);
  }
}

struct Bins {
  u32 cnt, done, chunks, cur, fill, next, bins;
  u32 q;                      // PVE_Q: the wave's queue (partitions [kQN], then RW record-word arrays [kQN])
  mutable u32 qhead, qtail;   // (wave-uniform record counters of the queue)
  u32* recs;
  u32* table;
  i64 region, C;
  unsigned long long* err;
};

// the chunk slot of bin p's next flush (one lane per bin): the partition's current chunk of this workgroup, a new one
// every SC bins (its table entry = partition | its rank among the workgroup's chunks of that partition). One bin per
// partition, flushed once full: the partition's chunk state has one writer at a time. Returns the record offset.
__device__ __forceinline__ i64 bin_slot(const Bins& B, u32 p) {
  const u32 f = at<l32>(B.fill)[p];
  u32 c;
  if (f == 0) {
    c = __hip_atomic_fetch_add(at<l32>(B.next), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const u32 r = at<l32>(B.chunks)[p];
    at<l32>(B.chunks)[p] = r + 1u;
    at<l32>(B.cur)[p] = c;
    if ((i64)c < B.C)  // (written full; a partition's last chunk is rewritten with its bins at the end)
      ((__attribute__((address_space(1))) u32*)B.table)[B.region + (i64)c] = p | ((u32)(SC - 1) << 12) | (r << 16);
  } else {
    c = at<l32>(B.cur)[p];
  }
  at<l32>(B.fill)[p] = f + 1u == (u32)SC ? 0u : f + 1u;
  if ((i64)c >= B.C) {
    __hip_atomic_fetch_add(B.err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return -1;
  }
  return ((B.region + (i64)c) * SC + f) * BS;
}

typedef u32 u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPieces = BS * RW / 4;  // 16-byte pieces of a bin

// Every bin the wave completed (full[i] of its lanes) leaves together: eight lanes per bin (16 bytes each per store
// instruction: a 32-record one-word bin is one instruction for eight bins), the group's first lane takes the chunk slot
// and restarts the bin after the copy.
// keep: lanes whose record-0 bin is restarted by the lane itself (PVE_HRUN: the claim's records past the bin's end
// go into the new bin first)
__device__ __forceinline__ void flush_full(const Bins& B, const bool (&full)[PVE_PB], const u32 (&pp)[PVE_PB], int lane,
                                           u64 keep = 0) {
  u64 fm[PVE_PB];
  u64 any = 0;
#pragma unroll
  for (int i = 0; i < PVE_PB; ++i) {
    fm[i] = __builtin_amdgcn_ballot_w64(full[i]);
    any |= fm[i];
  }
  if (any == 0) return;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  const int grp = lane >> 3, sub = lane & 7;
  u32 mine = 0xffffffffu;
  bool mkeep = false;
  int g = 0;
  auto round = [&]() {
    const bool on = grp < g;
    i64 at_rec = -1;
    if (on && sub == 0) at_rec = bin_slot(B, mine);
    const int leader = lane & ~7;
    const i64 dst_rec = ((i64)__builtin_amdgcn_ds_bpermute(leader << 2, (int)(u32)at_rec) & 0xffffffffll) |
                        ((i64)__builtin_amdgcn_ds_bpermute(leader << 2, (int)(u32)((u64)at_rec >> 32)) << 32);
    if (on && dst_rec >= 0 && PVE_DBG != 2) {
#pragma unroll
      for (int k = 0; k < kPieces; k += 8) {
        if (kPieces % 8 != 0 && sub + k >= kPieces) break;
        const u32x4 v = *at<const __attribute__((address_space(3))) u32x4>(B.bins + mine * (u32)(BS * RW) * 4u +
                                                                             16u * (u32)(sub + k));
        __builtin_nontemporal_store(v, (__attribute__((address_space(1))) u32x4*)(B.recs + dst_rec * RW) + sub + k);
      }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (the bin is read before it restarts: LDS runs one wave's ops in order)
    if (on && sub == 0 && !mkeep) {
      at<l32>(B.done)[mine] = 0u;
      at<l32>(B.cnt)[mine] = 0u;
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    g = 0;
    mine = 0xffffffffu;
    mkeep = false;
  };
#pragma unroll
  for (int i = 0; i < PVE_PB; ++i) {
    u64 m = fm[i];
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const u32 p = (u32)__builtin_amdgcn_readlane((int)pp[i], l);
      if (grp == g) {
        mine = p;
        mkeep = i == 0 && ((keep >> l) & 1ull);
      }
      if (++g == 8) round();
    }
  }
  if (g) round();
}

// the end of the pass: bin p (one thread) as a chunk slot, copied by that thread
__device__ __forceinline__ void flush_one(const Bins& B, u32 p) {
  const i64 dst_rec = bin_slot(B, p);
  if (dst_rec >= 0) {
    const __attribute__((address_space(3))) u32x4* src =
        at<const __attribute__((address_space(3))) u32x4>(B.bins + p * (u32)(BS * RW) * 4u);
    __attribute__((address_space(1))) u32x4* dst = (__attribute__((address_space(1))) u32x4*)(B.recs + dst_rec * RW);
    for (int k = 0; k < kPieces; ++k) __builtin_nontemporal_store(src[k], dst + k);
  }
  at<l32>(B.done)[p] = 0u;
  at<l32>(B.cnt)[p] = 0u;
}

// PB records of the lane (pend[i]: record i exists) into their partitions' bins: claim, write, count written; a lane
// that completes a bin flushes it; a record whose bin was full claims again after the flushes
constexpr int PB = PVE_PB;
__device__ __forceinline__ void put_round(const Bins& B, bool (&pend)[PB], const u32 (&pp)[PB], const u32 (&rr)[PB][RW],
                                          int lane) {
  {
    for (int round = 0;; ++round) {
      u32 s[PB];
#pragma unroll
      for (int i = 0; i < PB; ++i)
        s[i] = pend[i] ? __hip_atomic_fetch_add(at<l32>(B.cnt) + pp[i], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                       : 0xffffffffu;
#pragma unroll
      for (int i = 0; i < PB; ++i)
        if (s[i] < (u32)BS)
#pragma unroll
          for (int k = 0; k < RW; ++k) at<l32>(B.bins)[(pp[i] * (u32)BS + s[i]) * (u32)RW + (u32)k] = rr[i][k];
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      bool full[PB];
#if PVE_DONE_RTN
#pragma unroll
      for (int i = 0; i < PB; ++i)
        full[i] = s[i] < (u32)BS &&
                  __hip_atomic_fetch_add(at<l32>(B.done) + pp[i], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                      (u32)BS - 1u;
#else
      // written counts without a returned value (no round trip per round): the lane that claimed a bin's last slot
      // waits until every slot of the bin is written (LDS runs each wave's operations in order, so a writer's count
      // follows its record), then flushes it
#pragma unroll
      for (int i = 0; i < PB; ++i)
        if (s[i] < (u32)BS)
          (void)__hip_atomic_fetch_add(at<l32>(B.done) + pp[i], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      bool anyfull = false;
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        full[i] = s[i] == (u32)BS - 1u;
        anyfull |= full[i];
      }
      if (__builtin_amdgcn_ballot_w64(anyfull) != 0) {
#pragma unroll
        for (int i = 0; i < PB; ++i)
          if (full[i])
            while (__hip_atomic_load(at<l32>(B.done) + pp[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) !=
                   (u32)BS)
              __builtin_amdgcn_s_sleep(1);
      }
#endif
      flush_full(B, full, pp, lane);
      bool any = false;
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        pend[i] = pend[i] && s[i] >= (u32)BS;
        any |= pend[i];
      }
      if (__builtin_amdgcn_ballot_w64(any) == 0) break;
      if (round > 0) __builtin_amdgcn_s_sleep(2);
    }
  }
}

// Compacted put rounds (PVE_Q): a lane's records join the wave's queue in LDS (positions by ballot prefix counts), and
// a put round runs only when the queue holds 64 PB records, every lane taking PB consecutive ones; the rest waits for
// the next tile (the wave's last records go at the end of its tiles). A put round then carries 64 PB records whatever
// the filter kept or however unevenly the lanes' MV value runs are spread.
constexpr u32 kQN = 512;  // queue entries: < 64 PB left + 64 PB pushed
static_assert(!PVE_Q || 128 * PB <= (int)kQN, "queue too small for the put round");
__device__ __forceinline__ void q_push(const Bins& B, const bool (&pend)[PB], const u32 (&pp)[PB],
                                       const u32 (&rr)[PB][RW]) {
  u32 n = B.qtail;
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const u64 b = __builtin_amdgcn_ballot_w64(pend[i]);
    if (pend[i]) {
      const u32 pos = (n + __builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u))) & (kQN - 1);
      at<l32>(B.q)[pos] = pp[i];
#pragma unroll
      for (int k = 0; k < RW; ++k) at<l32>(B.q + 4u * kQN * (u32)(k + 1))[pos] = rr[i][k];
    }
    n += (u32)__builtin_popcountll(b);
  }
  B.qtail = n;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (a wave's LDS operations run in order: the round's reads see these)
}
__device__ __forceinline__ void q_drain(const Bins& B, int lane, bool all) {
  while (B.qtail - B.qhead >= 64u * (u32)PB || (all && B.qtail != B.qhead)) {
    bool pend[PB];
    u32 pp[PB], rr[PB][RW];
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const u32 idx = B.qhead + (u32)lane * (u32)PB + (u32)i;
      pend[i] = idx - B.qhead < B.qtail - B.qhead;
      const u32 pos = idx & (kQN - 1);
      pp[i] = pend[i] ? at<const l32>(B.q)[pos] : 0u;
#pragma unroll
      for (int k = 0; k < RW; ++k) rr[i][k] = pend[i] ? at<const l32>(B.q + 4u * kQN * (u32)(k + 1))[pos] : 0u;
    }
    const u32 take = B.qtail - B.qhead < 64u * (u32)PB ? B.qtail - B.qhead : 64u * (u32)PB;
    B.qhead += take;
    put_round(B, pend, pp, rr, lane);
  }
}
__device__ __forceinline__ void put_any(const Bins& B, bool (&pend)[PB], const u32 (&pp)[PB], const u32 (&rr)[PB][RW],
                                        int lane) {
  if constexpr (PVE_Q) {
    q_push(B, pend, pp, rr);
    q_drain(B, lane, false);
  } else {
    put_round(B, pend, pp, rr, lane);
  }
}

// the V stream: the lane's matching docs (bits of m), PB at a time
__device__ __forceinline__ void put(const Bins& B, u32 m, const u32 (&key)[ND], const u32 (&val)[ND][RW], int lane) {
#pragma unroll
  for (int h = 0; h < ND; h += PB) {
    bool pend[PB];
    u32 pp[PB], rr[PB][RW];
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      pend[i] = (m >> (h + i)) & 1u;
      pp[i] = KR ? key[h + i] / KRD : key[h + i] >> KS;
      rr[i][0] = (KR ? key[h + i] - pp[i] * KR : key[h + i] & ((1u << KS) - 1u)) | (VC >= 0 ? (val[h + i][0] << KS) : 0u);
#pragma unroll
      for (int k = 1; k < RW; ++k) rr[i][k] = val[h + i][k];
    }
    put_any(B, pend, pp, rr, lane);
  }
}

// The H stream: one record per value of the lane's matching docs, PB values per round. The lane's values are one run
// [o[first match], o[last match + 1]) of the MV stream; a value's doc is the last doc whose first value is not past it
// (unrolled compares: no dynamically indexed registers); values of unmatched docs inside the run are skipped.
// H: the tile's MV value words [first value's word & ~3, last value's word + 2) into the wave's value buffer (LDS DMA,
// whole 16-byte chunks: the stream has guard words on both sides); returns the first word staged
__device__ __forceinline__ u32 stage_values(CS* sg, i64 wt, u32 vbuf, u32 voff) {
  const int* off = (const int*)sg->mv_off;
  const i64 d0 = wt * TD, nd = sg->num_docs;
  const i64 d1 = d0 + TD < nd ? d0 + TD : nd;
  const u32 S = (u32)__builtin_amdgcn_readfirstlane(off[d0]), E = (u32)__builtin_amdgcn_readfirstlane(off[d1]);
  const u32 w0 = (u32)(((u64)S * (u64)HNB) >> 5) & ~3u;
  const u32 w1 = (u32)(((u64)E * (u64)HNB) >> 5) + 2u;
  const u32 n16 = (w1 - w0 + 3u) >> 2;
  const u64 src = sg->mv_words + (u64)w0 * 4u;
  for (u32 k = 0; 64u * k < n16; ++k) {
    const u32 rem = n16 - 64u * k;
    if (rem >= 64u) dma16(voff, src + 1024u * k, vbuf + 1024u * k);
    else dma16m(voff, src + 1024u * k, vbuf + 1024u * k, (1ull << rem) - 1ull);
  }
  return w0;
}

__device__ __forceinline__ void put_values(const Bins& B, CS* sg, i64 wt, u32 m, const u32 (&key)[ND], int lane,
                                           u32 vbuf, u32 vb0, bool nxt) {
  if (__builtin_amdgcn_ballot_w64(m != 0) == 0) return;
  // the value words have landed (the next tile's image DMA, issued after them, may still be in flight)
  if (nxt) vm_wait<kDmaImg>();
  else vm_wait<0>();
  const __attribute__((address_space(1))) int* off = (const __attribute__((address_space(1))) int*)sg->mv_off;
  const l32* words = at<const l32>(vbuf);
  const __attribute__((address_space(1))) u32* lut = (const __attribute__((address_space(1))) u32*)sg->hlut;
  const i64 d0 = wt * TD + (i64)ND * lane, nd = sg->num_docs;
  int o[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; ++i) o[i] = m ? off[d0 + i < nd ? d0 + i : nd] : 0;
  int s = 0, e = 0;
  if (m) {
    const int f = __builtin_ctz(m), l = 31 - __builtin_clz(m);
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      if (i == f) s = o[i];
      if (i == l) e = o[i + 1];
    }
  }
  constexpr u32 kmask = (1u << KS) - 1u;
  for (int v0 = s;; v0 += PB) {
    bool pend[PB];
    u32 pp[PB], rr[PB][RW], k[PB], wa[PB], wb[PB], sh[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int v = v0 + j;
      u32 kk = key[0];
      bool mm = m & 1u;
#pragma unroll
      for (int i = 1; i < ND; ++i)
        if (v >= o[i]) {
          kk = key[i];
          mm = (m >> i) & 1u;
        }
      pend[j] = v < e && mm;
      k[j] = kk;
      const u64 bit = (u64)(u32)v * (u64)HNB;
      sh[j] = (u32)bit & 31u;
      wa[j] = wb[j] = 0u;
      if (pend[j]) {
        const u32 rel = (u32)(bit >> 5) - vb0;
        wa[j] = words[rel];
        wb[j] = words[rel + 1u];
      }
    }
    u32 hv[PB];
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const u32 x = sh[j] ? __builtin_amdgcn_alignbit(wa[j], wb[j], 32u - sh[j]) : wa[j];
      hv[j] = pend[j] ? lut[x >> (32 - HNB)] : 0u;
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      pp[j] = k[j] >> KS;
      rr[j][0] = ((k[j] & kmask) << (LG + 6)) | ((hv[j] >> 8) << 6) | ((hv[j] & 0xffu) << 1);
    }
    if constexpr (PVE_DBG != 1) {
      put_any(B, pend, pp, rr, lane);
    } else {  // (measurement: records built, kept live, not put)
      u32 x = 0;
#pragma unroll
      for (int j = 0; j < PB; ++j) x ^= pend[j] ? rr[j][0] + pp[j] : 0u;
      if (x == 0x9e3779b9u) *at<l32>(B.next) = x;
    }
    if (__builtin_amdgcn_ballot_w64(v0 + PB < e) == 0) break;
  }
}

// The H stream by runs (PVE_HRUN): a lane walks its values in doc order, each round taking up to HB values of its
// current doc (one partition: they share the doc's key) with ONE claim of as many slots (and one written count),
// instead of one claim per value. A claim that runs past the bin's end belongs to the lane holding the bin's last
// slot: it writes what fits, flushes the bin when every slot is written, then puts the rest into the restarted bin
// itself (slots 0.., written count and claim counter set to that many: the other lanes' claims keep failing until the
// counter drops below BS). A claim that finds the bin full is retried next round. The values' words come from one
// window of NWIN words read once per round.
constexpr int HB = PVE_HB;
constexpr int NWIN = ((31 + (HB - 1) * HNB) >> 5) + 2;
__device__ __forceinline__ void put_values_run(const Bins& B, CS* sg, i64 wt, u32 m, const u32 (&key)[ND], int lane,
                                               u32 vbuf, u32 vb0, bool nxt) {
  if (__builtin_amdgcn_ballot_w64(m != 0) == 0) return;
  if (nxt) vm_wait<kDmaImg>();
  else vm_wait<0>();
  const __attribute__((address_space(1))) int* off = (const __attribute__((address_space(1))) int*)sg->mv_off;
  const l32* words = at<const l32>(vbuf);
  const __attribute__((address_space(1))) u32* lut = (const __attribute__((address_space(1))) u32*)sg->hlut;
  const i64 d0 = wt * TD + (i64)ND * lane, nd = sg->num_docs;
  int o[ND + 1];
#pragma unroll
  for (int i = 0; i <= ND; ++i) o[i] = m ? off[d0 + i < nd ? d0 + i : nd] : 0;
  int v = 0, e = 0;
  if (m) {
    const int f = __builtin_ctz(m), l = 31 - __builtin_clz(m);
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      if (i == f) v = o[i];
      if (i == l) e = o[i + 1];
    }
  }
  constexpr u32 kmask = (1u << KS) - 1u;
  while (__builtin_amdgcn_ballot_w64(v < e) != 0) {
    // the lane's current doc: the last one whose first value is not past v
    u32 kk = key[0];
    bool mm = m & 1u;
    int end = o[1];
#pragma unroll
    for (int i = 1; i < ND; ++i)
      if (v >= o[i]) {
        kk = key[i];
        mm = (m >> i) & 1u;
        end = o[i + 1];
      }
    const int avail = v < e ? end - v : 0;
    const u32 n = mm ? (u32)(avail < HB ? avail : HB) : 0u;
    const u32 p = kk >> KS;
    u32 rec[HB];
    if (n) {
      const u64 bit0 = (u64)(u32)v * (u64)HNB;
      const u32 w0 = (u32)(bit0 >> 5) - vb0, sh = (u32)bit0 & 31u;
      u32 win[NWIN];
#pragma unroll
      for (int k = 0; k < NWIN; ++k) win[k] = words[w0 + (u32)k];
      u32 hv[HB];
#pragma unroll
      for (int j = 0; j < HB; ++j) {
        const u32 q = sh + (u32)(j * HNB), wi = q >> 5, s2 = q & 31u;
        u32 wa = win[0], wb = win[1];
#pragma unroll
        for (int k = 1; k + 1 < NWIN; ++k)
          if (wi == (u32)k) {
            wa = win[k];
            wb = win[k + 1];
          }
        const u32 x = s2 ? __builtin_amdgcn_alignbit(wa, wb, 32u - s2) : wa;
        hv[j] = (u32)j < n ? lut[x >> (32 - HNB)] : 0u;
      }
#pragma unroll
      for (int j = 0; j < HB; ++j) rec[j] = ((kk & kmask) << (LG + 6)) | ((hv[j] >> 8) << 6) | ((hv[j] & 0xffu) << 1);
    }
    if constexpr (PVE_DBG == 1) {  // (measurement: records built, kept live, not put)
      u32 x = 0;
#pragma unroll
      for (int j = 0; j < HB; ++j) x ^= (u32)j < n ? rec[j] + p : 0u;
      if (x == 0x9e3779b9u) *at<l32>(B.next) = x;
      v = n ? v + (int)n : (v < e ? end : v);
      continue;
    }
    const u32 s = n ? __hip_atomic_fetch_add(at<l32>(B.cnt) + p, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                    : 0xffffffffu;
    const u32 w = s < (u32)BS ? ((u32)BS - s < n ? (u32)BS - s : n) : 0u;
#pragma unroll
    for (int j = 0; j < HB; ++j)
      if ((u32)j < w) at<l32>(B.bins)[p * (u32)BS + s + (u32)j] = rec[j];
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (w) (void)__hip_atomic_fetch_add(at<l32>(B.done) + p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // the claimer of the bin's last slot waits until every slot is written (a writer's count follows its record)
    const bool closer = w && s + n >= (u32)BS;
    const u32 carry = closer ? s + n - (u32)BS : 0u;
    if (__builtin_amdgcn_ballot_w64(closer) != 0) {
      if (closer)
        while (__hip_atomic_load(at<l32>(B.done) + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (u32)BS)
          __builtin_amdgcn_s_sleep(1);
      bool full[PVE_PB];
      u32 pp[PVE_PB];
#pragma unroll
      for (int i = 0; i < PVE_PB; ++i) {
        full[i] = i == 0 && closer;
        pp[i] = p;
      }
      flush_full(B, full, pp, lane, __builtin_amdgcn_ballot_w64(carry != 0));
      if (carry) {  // the rest of the claim starts the restarted bin (the copy's reads came first: one wave, in order)
#pragma unroll
        for (int j = 0; j < HB; ++j)
          if ((u32)j >= w && (u32)j < n) at<l32>(B.bins)[p * (u32)BS + (u32)j - w] = rec[j];
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        at<l32>(B.done)[p] = carry;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        at<l32>(B.cnt)[p] = carry;
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    // advance: past the claimed values, past an unmatched doc, or stay (the bin was full: claim again)
    if (n) {
      if (w) v += (int)n;
    } else if (v < e) {
      v = end;
    }
  }
}

// one tile: returns the lane's docs counted in numDocsScanned. issue() sends the next tile's DMA: here, after the
// admission loads have been waited for (PVE_ADMIT: a wait for them would otherwise also wait for that DMA)
template <class Issue>
__device__ __forceinline__ u32 tile(const Bins& B, CS* sg, i64 wt, u32 img, int lane, Issue&& issue, u32 vbuf, u32 vb0,
                                    bool nxt) {
  constexpr u32 kAll = (1u << ND) - 1u;
  const i64 rem = (i64)sg->num_docs - wt * TD;
  u32 m = kAll;
  if (rem < TD) {
    const i64 n = rem - ND * lane;
    m = n >= ND ? kAll : (n <= 0 ? 0u : ((1u << n) - 1u));
  }
  u32 clause = 0;
  if (!leaves<0>(sg, img, lane, m, clause) || __builtin_amdgcn_ballot_w64(m != 0) == 0) {
    if constexpr (PVE_ADMIT) issue();
    return 0;
  }
  u32 key[ND], val[ND][RW];
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    key[i] = 0u;
#pragma unroll
    for (int k = 0; k < RW; ++k) val[i][k] = 0u;
  }
  keys<0>(img, lane, key);
  if constexpr (PVE_KOFF) {  // each component's run of the table dictionary: one offset per segment
    u32 kadd = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) kadd += (u32)sg->koff[g] * kGS[g];
#pragma unroll
    for (int i = 0; i < ND; ++i) key[i] += kadd;
  }
  if constexpr (VC >= 0) {
    u32 id[ND];
    unpack<(VC >= 0 ? VC : 0), false>(img, lane, id);
    const u32 vadd = PVE_VOFF ? (u32)sg->voff : 0u;
#pragma unroll
    for (int i = 0; i < ND; ++i) val[i][0] = id[i] + vadd;
  }
  if constexpr (RAWB > 0) {  // the lane's ND raw values: ND RAWB consecutive bytes of the staged tile
    const __attribute__((address_space(3))) u32x4* r =
        at<const __attribute__((address_space(3))) u32x4>(img + (u32)PVE_RAWOFF + (u32)lane * (u32)(ND * RAWB));
    u32 w[ND * (RAWB > 0 ? RAWB : 4) / 4];
#pragma unroll
    for (int k = 0; k < ND * RAWB / 16; ++k) {
      const u32x4 x = r[k];
      w[4 * k] = x.x;
      w[4 * k + 1] = x.y;
      w[4 * k + 2] = x.z;
      w[4 * k + 3] = x.w;
    }
#pragma unroll
    for (int i = 0; i < ND; ++i)
#pragma unroll
      for (int k = 1; k < RW; ++k) val[i][k] = w[i * (RW - 1) + k - 1];
  }
  const u32 scanned = (u32)__builtin_popcount(m);  // (numDocsScanned: every doc the filter kept, admitted or not)
  if constexpr (PVE_ADMIT) {
    const __attribute__((address_space(1))) u32* adm = (const __attribute__((address_space(1))) u32*)sg->admit;
    if (adm) {
      u32 w[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) w[i] = ((m >> i) & 1u) ? adm[key[i] >> 5] : 0u;
#pragma unroll
      for (int i = 0; i < ND; ++i)
        if (!((w[i] >> (key[i] & 31u)) & 1u)) m &= ~(1u << i);
    }
    issue();
  }
  if constexpr (PVE_DBG == 1) {
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < ND; ++i) x ^= key[i] + val[i][RW - 1];
    if (x == 0x9e3779b9u) *at<l32>(B.next) = x;  // (keeps the records live)
    return scanned;
  }
  if constexpr (PVE_H && PVE_HRUN) {
    put_values_run(B, sg, wt, m, key, lane, vbuf, vb0, nxt);
    return 0u;
  } else if constexpr (PVE_H) {
    put_values(B, sg, wt, m, key, lane, vbuf, vb0, nxt);
    return 0u;  // (numDocsScanned: counted by the V stream's launch)
  } else {
    put(B, m, key, val, lane);
  }
  return scanned;
}

__device__ __forceinline__ int find_segment(CS* segs, int nseg, i64 t) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].first_tile <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

extern "C" __global__ void __launch_bounds__(W * 64, 1) pve_jit(const PveArgs* a_in, const PveSeg* s_in) {
  CA* A = (CA*)(unsigned long)a_in;
  CS* S = (CS*)(unsigned long)s_in;
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const u32 base = lds_addr(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const i64 T = A->total_tiles, G = gridDim.x;
  const i64 b = blockIdx.x;
  const i64 lb = A->xcd_major ? (b % 8) * (G / 8) + (b % 8 < G % 8 ? b % 8 : G % 8) + b / 8 : b;
  Bins B;
  B.cnt = base;
  B.done = base + 4u * P;
  B.chunks = base + 8u * P;
  B.cur = base + 12u * P;
  B.fill = base + 16u * P;
  B.next = base + 20u * P;
  B.bins = base + (u32)PVE_L_BINS;
  B.recs = A->recs;
  B.table = A->table;
  B.C = A->chunks_per_wg;
  B.region = lb * B.C;
  B.err = A->matched + 3;
  B.q = base + (u32)PVE_L_Q + (u32)wave * 4u * kQN * (u32)(RW + 1);
  B.qhead = B.qtail = 0u;
  for (int i = tid; i < 5 * P + 1; i += W * 64) smem[i] = 0u;
  __syncthreads();
  const i64 t0 = lb * T / G, t1 = (lb + 1) * T / G;
  const u32 ring = base + (u32)PVE_L_RING + (u32)wave * (u32)R * (u32)IMG * 4u;
  const u32 voff = 16u * (u32)lane;
  const u32 vbuf = base + (u32)PVE_L_VAL + (u32)wave * (u32)PVE_VAL_B;  // H: the wave's MV value words
  u32 matched = 0;
  if (t0 < t1) {
    const int nseg = A->nseg;
    int isi = find_segment(S, nseg, t0 + wave);
    int psi = isi;
    i64 ifirst = S[isi].first_tile, iend = ifirst + S[isi].num_tiles;
    i64 pfirst = ifirst, pend = iend;
    i64 ti = t0 + wave;
    auto issue_to = [&](int to) {  // the wave's next tile into image slot `to`
      if (ti < t1) {
        while (ti >= iend) {
          ++isi;
          ifirst = S[isi].first_tile;
          iend = ifirst + S[isi].num_tiles;
        }
        dma_cols<0>(S + isi, ti - ifirst, ring + (u32)to * (u32)IMG * 4u, voff);
      }
      ti += W;
    };
#pragma unroll
    for (int k = 0; k + 1 < R; ++k) issue_to(k);
    int slot = 0;
    for (i64 t = t0 + wave; t < t1; t += W) {
      // tile t has landed (the R - 2 tiles after it may stay in flight when they were all issued; the chunk stores of
      // the tiles before it are younger than their DMA and only make the count conservative)
      if (R > 2 && t + (i64)(R - 2) * W < t1) vm_wait<(R > 2 ? (R - 2) * kDmaImg : 0)>();
      else vm_wait<0>();
      const int to = slot == 0 ? R - 1 : slot - 1;  // (the image walked last)
      auto issue = [&]() { issue_to(to); };
      while (t >= pend) {
        ++psi;
        pfirst = S[psi].first_tile;
        pend = pfirst + S[psi].num_tiles;
      }
      u32 vb0 = 0;
      if constexpr (PVE_H) vb0 = stage_values(S + psi, t - pfirst, vbuf, voff);  // (before the next image's DMA)
      const bool nxt = ti < t1;
      if constexpr (!PVE_ADMIT) issue();
      matched += tile(B, S + psi, t - pfirst, ring + (u32)slot * (u32)IMG * 4u, lane, issue, vbuf, vb0, nxt);
      slot = slot + 1 == R ? 0 : slot + 1;
    }
  }
  if constexpr (PVE_Q) q_drain(B, lane, true);  // (the wave's last queued records)
  vm_wait<0>();
  u64 wm = matched;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wm += __shfl_xor(wm, o);
  if (lane == 0 && wm) __hip_atomic_fetch_add(A->matched, wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  // the partial bins, padded with sentinels, as chunks; then this workgroup's chunks per partition
  for (int p = tid; p < P; p += W * 64) {
    const u32 n = at<l32>(B.cnt)[p];
    if (n == 0) continue;
    for (u32 k = n; k < (u32)BS; ++k) at<l32>(B.bins)[((u32)p * (u32)BS + k) * (u32)RW] = kSentinel;
    flush_one(B, (u32)p);
  }
  __syncthreads();
  // each partition's last chunk: its table entry with the bins written (pass C reads no further)
  for (int p = tid; p < P; p += W * 64) {
    const u32 f = at<l32>(B.fill)[p];
    if (f == 0) continue;
    const u32 c = at<l32>(B.cur)[p];
    if ((i64)c >= B.C) continue;
    ((__attribute__((address_space(1))) u32*)B.table)[B.region + (i64)c] =
        (u32)p | ((f - 1u) << 12) | ((at<l32>(B.chunks)[p] - 1u) << 16);
  }
  for (int p = tid; p < P; p += W * 64) A->hist[lb * P + p] = at<l32>(B.chunks)[p];
  if (tid == 0) {
    const u32 n = *at<l32>(B.next);
    A->used[lb] = (i64)n < B.C ? n : (u32)B.C;
  }
}
