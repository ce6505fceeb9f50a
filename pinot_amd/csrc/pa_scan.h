// Device code of the fused scan kernel (gfx950 / CDNA4 only): included by the translation units that instantiate its
// variants (pa_scan_std.hip, pa_scan_part_a.hip, pa_scan_part_b.hip) and by pa_kernels.hip (the other kernels).
//
// HIP kernels of the segment query hot path.
//
// One fused persistent-wave kernel per query does, for every doc of every bound segment:
//   bit-unpack the dictIds of the filter columns (FixedBitSVForwardIndexReaderV2 / PinotDataBitSet
//   semantics), evaluate the CNF filter as 64-bit wave ballots (replaces SVScanDocIdIterator /
//   BitmapBasedFilterOperator / And/Or/NotFilterOperator), build the table-wide group key
//   (DictionaryBasedGroupKeyGenerator raw key: column 0 least significant), and aggregate
//   COUNT/SUM/MIN/MAX/DISTINCTCOUNTHLL into LDS-privatised (small key spaces) or global (high
//   cardinality) accumulators (DefaultGroupByExecutor + *AggregationFunction.aggregateGroupBySV).
//
// Work decomposition: a wave owns a contiguous range of 2048-doc "wave tiles" (all segments of the
// query are concatenated); for each wave tile the forward-index words of every staged column are
// copied HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, fully coalesced)
// into a wave-private double buffer, so tile t+1 streams in while tile t is decoded. Lane l decodes
// doc 64*i + l of the tile (i = 0..31): every column of a doc lands in the same lane, and a 64-doc
// step of an nb-bit column is 2*nb consecutive LDS words (conflict-free ds_read2_b32).
#pragma once
#include <hip/hip_runtime.h>
#include "pa_device.h"
#include "pa_launch.h"
#include "pa_keys.h"

namespace pa {

typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
// Descriptors through the constant address space: read-only during every kernel, so their fields are scalar loads the
// compiler may keep in registers across LDS atomics and stores (a generic pointer is re-read after each of them, and
// every scalar load's lgkmcnt wait also waits for the LDS operations in flight).
typedef const __attribute__((address_space(4))) struct DevSeg CSegT;
typedef const __attribute__((address_space(4))) struct DevQuery CQ;

// Every HBM access goes through address-space-1 pointers: global_* instructions instead of flat_*. A flat
// access may alias LDS, which makes the compiler put vmcnt(0) in front of later LDS reads.
#define AS1 __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ AS1 T* gp(T* p) { return (AS1 T*)p; }
template <class T>
__device__ __forceinline__ const AS1 T* gp(const T* p) { return (const AS1 T*)p; }
#define RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // one 16-byte load / store

__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t nbits_mask(int nb) { return nb >= 32 ? 0xffffffffu : ((1u << nb) - 1u); }

// Value of doc `doc_local` (0..2047) from a staged wave-tile region (region[-1] is a guard word).
// Stream bits [doc*nb, doc*nb+nb): the last bit e1 = doc*nb+nb-1 lies in word e1>>5; the value is the
// nb bits ending at bit position (~e1)&31 of the 64-bit window (word[we-1], word[we]).
__device__ __forceinline__ uint32_t decode_lds(const uint32_t* region, int doc_local, int nb) {
  const uint32_t e1 = (uint32_t)doc_local * (uint32_t)nb + (uint32_t)(nb - 1);
  const int we = (int)(e1 >> 5);
  const uint32_t lo = region[we];
  const uint32_t hi = region[we - 1];
  return __builtin_amdgcn_alignbit(hi, lo, (~e1) & 31u) & nbits_mask(nb);
}

// Same, straight from the HBM-resident stream (lazy columns: read only for matching docs).
__device__ __forceinline__ uint32_t decode_global(const uint32_t* words, int64_t doc, int nb) {
  const uint64_t e1 = (uint64_t)doc * (uint64_t)nb + (uint64_t)(nb - 1);
  const int64_t we = (int64_t)(e1 >> 5);
  const uint32_t lo = gp(words)[we];
  const uint32_t hi = gp(words)[we - 1];
  return __builtin_amdgcn_alignbit(hi, lo, (~(uint32_t)e1) & 31u) & nbits_mask(nb);
}

// G: the caller has no staged tile (the per-doc kernels of the numGroupsLimit path): always decode from HBM.
template <bool G = false>
__device__ __forceinline__ uint32_t decode_dict_id(const DevCol& c, const uint32_t* img, int doc_local,
                                                   int64_t doc) {
  if constexpr (G) return decode_global(c.words, doc, c.nbits);
  return c.lds_off >= 0 ? decode_lds(img + c.lds_off, doc_local, c.nbits) : decode_global(c.words, doc, c.nbits);
}

// s_waitcnt vmcnt(N) with every other counter at its maximum (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14).
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Issue the LDS-DMA of one wave tile of every staged column of `seg` into the wave image `img`: exactly D
// wave instructions (D = the maximum over the query's segments; a segment needing fewer pads with 16-byte
// dummies into the image's guard words), so `vmcnt` counts tiles and a ring of tiles can be in flight behind
// counted waits.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

typedef __attribute__((address_space(3))) uint64_t lds_u64_t;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;
__device__ __forceinline__ lds_u32_t* lds_ptr(const void* p) { return (lds_u32_t*)(uintptr_t)lds_addr(p); }

#define WG_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP


// One LDS-DMA wave instruction (global_load_lds_dwordx4): lane l copies 16 bytes from its `src` to
// lds_base + 16*l. Issued as inline asm on purpose: the compiler's waitcnt pass cannot disambiguate LDS-DMA
// writes from later ds_reads of OTHER ring slots and would put vmcnt(0) in front of every tile's decode,
// draining the whole ring. Visibility is guaranteed by the explicit counted waits in wait_tile; vm ops the
// compiler does not know about only make its own vmcnt waits stricter, never wrong.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_base) {
  uint32_t keep;
  // wave-uniform by construction; readfirstlane keeps it in an SGPR even where the compiler computed it with VALU ops
  lds_base = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_base);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_base));
}

// dma16 for the lanes of `mask` only, with EXEC set and restored inside the asm block (no branch around a partial
// DMA instruction; the compiler's EXEC tracking is unaffected).
__device__ __forceinline__ void dma16_masked(const void* src, uint32_t lds_base, uint64_t mask) {
  uint32_t keep;
  uint64_t save;
  lds_base = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_base);
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, %4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, off\n\t"
      "s_mov_b32 m0, %0\n\t"
      "s_mov_b64 exec, %1"
      : "=&s"(keep), "=&s"(save)
      : "v"(src), "s"(lds_base), "s"(mask));
}

template <int STEPS>
__device__ __forceinline__ void stage_tile(const DevSeg* __restrict__ seg, int64_t wt, uint32_t* img, int lane,
                                           const int D) {
  const int ns = seg->num_staged;
  int issued = 0;
  for (int si = 0; si < ns; ++si) {
    const StageDesc& c = seg->stage[si];
    const int nb = c.nbits;
    const uint32_t* src = c.words + wt * (int64_t)(2 * STEPS * nb);  // 2*STEPS*nb stream words per wave tile
    const uint32_t dst = lds_addr(img + c.lds_off);
    const int chunks = (STEPS / 2) * nb;  // 16-byte chunks of this column's wave tile
    for (int c0 = 0; c0 < chunks; c0 += 64) {
      if (c0 + lane < chunks) dma16(src + 4 * (c0 + lane), dst + 16 * c0);
      ++issued;
    }
  }
  for (; issued < D; ++issued) {
    if (lane == 0) dma16(seg->dummy_src, lds_addr(img));
  }
}

// ---- wave reductions (all 64 lanes participate) ----
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const int64_t w = __shfl_xor(v, o); v = w < v ? w : v; }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const int64_t w = __shfl_xor(v, o); v = w > v ? w : v; }
  return v;
}

// Value an aggregation reads for one doc. For HLL returns (register << 8) | rank.
struct AggValue {
  int64_t i;
  double d;
};

template <bool G = false>
__device__ __forceinline__ AggValue agg_value(const DevAgg& A, int a, const DevSeg* __restrict__ seg,
                                              const uint32_t* img, int doc_local, int64_t doc) {
  AggValue out{0, 0.0};
  const DevCol& c = seg->cols[A.slot];
  if (c.kind == COL_SV_DICT) {
    const uint32_t id = decode_dict_id<G>(c, img, doc_local, doc);
    if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
      out.i = gp(seg->hll_lut[a])[id];
    } else if (A.type == PA_AGG_DISTINCTCOUNT) {
      out.i = seg->hll_lut[a] != nullptr ? gp(seg->hll_lut[a])[id] : id;  // table-wide value id
    } else if (A.src != SRC_DOUBLE) {
      out.i = gp(c.dict_i64)[id];
    } else {
      out.d = gp(c.dict_f64)[id];
    }
  } else {  // raw column
    int64_t iv = 0;
    double dv = 0.0;
    switch (c.vtype) {
      case PA_INT: iv = gp((const int32_t*)c.raw)[doc]; dv = (double)iv; break;
      case PA_LONG: iv = gp((const int64_t*)c.raw)[doc]; dv = (double)iv; break;
      case PA_FLOAT: { const float f = gp((const float*)c.raw)[doc]; dv = f; iv = __builtin_bit_cast(int32_t, f); } break;
      default: dv = gp((const double*)c.raw)[doc]; iv = __builtin_bit_cast(int64_t, dv); break;
    }
    if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
      // MurmurHash.hash(Object): Integer/Long -> hashLong(value), Float -> hashLong(floatToRawIntBits),
      // Double -> hashLong(doubleToRawLongBits); iv already holds exactly those longs.
      out.i = hll_slot_rank(murmur_hash_long(iv), A.log2m);
    } else if (A.src != SRC_DOUBLE) {
      out.i = iv;
    } else {
      out.d = dv;
    }
  }
  return out;
}

// Register max on one byte of the u8 HLL registers in HBM (there are no byte atomics: compare-and-swap on the word
// holding it; registers only grow, so the loop ends as soon as the byte is already >= v).
__device__ __forceinline__ void atomic_max_u8(uint8_t* p, uint32_t v) {
  AS1 uint32_t* w = (AS1 uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
  const uint32_t sh = ((uint32_t)(uintptr_t)p & 3u) * 8u;
  uint32_t old = __hip_atomic_load(w, RLX);
  while (((old >> sh) & 0xffu) < v) {
    const uint32_t nw = (old & ~(0xffu << sh)) | (v << sh);
    if (__hip_atomic_compare_exchange_strong(w, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      break;
  }
}

// ---- accumulator targets ----
template <int STRAT>
struct Acc {
  const DevQuery* q;
  unsigned char* lds;
  const PartScratch* ps;  // partitioned passes only

  __device__ __forceinline__ void add_count(int64_t key, uint32_t n) const {
    if (STRAT == STRAT_LDS) atomicAdd((uint32_t*)(lds + q->lds_count_off) + key, n);
    else __hip_atomic_fetch_add(gp(q->count) + key, (unsigned long long)n, RLX);
  }
  __device__ __forceinline__ void add_i64(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) atomicAdd((unsigned long long*)(lds + A.lds_off) + key, (unsigned long long)v);
    else __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + key, (unsigned long long)v, RLX);
  }
  __device__ __forceinline__ void add_f64(const DevAgg& A, int64_t key, double v) const {
    if (STRAT == STRAT_LDS) atomicAdd((double*)(lds + A.lds_off) + key, v);
    else __hip_atomic_fetch_add(gp(A.acc_f64) + key, v, RLX);
  }
  __device__ __forceinline__ void min_i64(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) atomicMin((long long*)(lds + A.lds_off) + key, (long long)v);
    else __hip_atomic_fetch_min(gp((long long*)A.acc_i64) + key, (long long)v, RLX);
  }
  __device__ __forceinline__ void max_i64(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) atomicMax((long long*)(lds + A.lds_off) + key, (long long)v);
    else __hip_atomic_fetch_max(gp((long long*)A.acc_i64) + key, (long long)v, RLX);
  }
  // DISTINCTCOUNT: the group saw value id v (an idempotent byte store: no atomic needed)
  __device__ __forceinline__ void set_presence(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) ((uint8_t*)(lds + A.lds_off))[key * A.nvals + v] = 1;
    else gp(A.acc_hll)[key * A.nvals + v] = 1;
  }
  __device__ __forceinline__ void max_hll(const DevAgg& A, int64_t key, uint32_t jr) const {
    const int64_t idx = (key << A.log2m) + (jr >> 8);
    if (STRAT == STRAT_LDS) atomicMax((uint32_t*)(lds + A.lds_off) + idx, jr & 0xffu);
    else atomic_max_u8(A.acc_hll + idx, jr & 0xffu);
  }
};

// Group-key component of one doc for group-by column j: the table-wide key id of a dictionary column (remapped), or
// the value bits of a raw column (hashed key space: INT/FLOAT 32 bits, LONG/DOUBLE 64 bits).
template <bool G = false>
__device__ __forceinline__ uint64_t gb_component(const DevCol& c, const int32_t* remap, const uint32_t* img,
                                                 int doc_local, int64_t doc) {
  if (c.kind == COL_SV_RAW) {
    switch (c.vtype) {
      case PA_INT: return (uint64_t)(uint32_t)gp((const int32_t*)c.raw)[doc];
      case PA_FLOAT: return (uint64_t)gp((const uint32_t*)c.raw)[doc];
      default: return (uint64_t)gp((const int64_t*)c.raw)[doc];
    }
  }
  uint32_t id = decode_dict_id<G>(c, img, doc_local, doc);
  if (remap != nullptr) id = (uint32_t)gp(remap)[id];
  return id;
}

// Hashed key space: the accumulator slot of a packed key (pa_keys.h: one word, or two for components wider than 64
// bits together, DevQuery::key_words; a direct key space's key is its slot). -1 if the table is full (counted as an
// overflow: the query then fails loudly at fetch).
__device__ __forceinline__ int64_t key_slot(const DevQuery* __restrict__ q, int64_t k0, int64_t k1 = 0) {
  if (!q->hashed) return k0;
  int64_t s;
  if (q->key_words == 2) {
    bool ins;
    s = ht_slot2((long long*)q->ht_keys, q->ht_mask, k0, k1, &ins);
  } else {
    s = ht_slot1((long long*)q->ht_keys, q->ht_mask, k0);
  }
  if (s < 0) __hip_atomic_fetch_add(gp(q->matched_docs) + 1, 1ull, RLX);
  return s;
}

// Accumulate the matched lanes (`matched` = wave mask) of one 64-doc step.
template <int STRAT>
__device__ __forceinline__ void accumulate_step(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                                const uint32_t* img, int doc_local, int64_t doc,
                                                uint64_t matched, int lane, const Acc<STRAT>& acc) {
  bool mine = (matched >> lane) & 1ull;
  // table-wide group key (DictionaryBasedGroupKeyGenerator: rawKey = sum dictId_j * prod_{k<j} card_k), or the packed
  // key's accumulator slot in the hashed key space
  int64_t key = 0;
  if (mine) {
    int64_t kw[2] = {0, 0};  // (two words: DevQuery::gb_word)
    for (int j = 0; j < q->num_gb; ++j)
      kw[q->gb_word[j]] += (int64_t)(gb_component(seg->cols[q->gb_slot[j]], seg->remap[j], img, doc_local, doc) *
                                     (uint64_t)q->gb_stride[j]);
    key = key_slot(q, kw[0], kw[1]);
    if (key < 0) mine = false;
  }
  matched &= __ballot(mine);

  uint64_t pending = matched;
  bool first = true;
  while (pending) {
    // Pick the group of lanes sharing the first pending lane's key; if that group is small on the first
    // pass (high-cardinality keys) give up on grouping and let every pending lane update on its own.
    const int leader = __builtin_ctzll(pending);
    const int64_t k0 = __shfl(key, leader);
    const uint64_t same = __ballot(key == k0) & pending;
    const bool grouped = !first || (__builtin_popcountll(same) * 4 >= __builtin_popcountll(pending));
    first = false;
    const uint64_t set = grouped ? same : pending;
    pending &= ~set;
    const bool in = (set >> lane) & 1ull;

    if (grouped) {
      if (lane == leader) acc.add_count(k0, (uint32_t)__builtin_popcountll(set));
    } else if (in) {
      acc.add_count(key, 1u);
    }
    for (int a = 0; a < q->num_aggs; ++a) {
      const DevAgg& A = q->aggs[a];
      if (A.type == PA_AGG_COUNT) continue;
      AggValue v{0, 0.0};
      if (in) v = agg_value(A, a, seg, img, doc_local, doc);
      if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
        if (in) acc.max_hll(A, key, (uint32_t)v.i);
      } else if (A.type == PA_AGG_DISTINCTCOUNT) {
        if (in) acc.set_presence(A, key, v.i);
      } else if (grouped) {
        if (A.type == PA_AGG_SUM) {
          if (A.src == SRC_INT) {
            const int64_t s = wave_sum_i64(in ? v.i : 0);
            if (lane == leader) acc.add_i64(A, k0, s);
          } else if (A.src == SRC_LONG) {
            const int64_t lo = wave_sum_i64(in ? (int64_t)(uint32_t)v.i : 0);
            const int64_t hi = wave_sum_i64(in ? (v.i >> 32) : 0);
            if (lane == leader) {
              acc.add_i64(A, 2 * k0, lo);
              acc.add_i64(A, 2 * k0 + 1, hi);
            }
          } else {
            const double s = wave_sum_f64(in ? v.d : 0.0);
            if (lane == leader) acc.add_f64(A, k0, s);
          }
        } else {
          const int64_t e = A.src != SRC_DOUBLE ? v.i : f64_order_encode(v.d);
          if (A.type == PA_AGG_MIN) {
            const int64_t r = wave_min_i64(in ? e : INT64_MAX);
            if (lane == leader) acc.min_i64(A, k0, r);
          } else {
            const int64_t r = wave_max_i64(in ? e : INT64_MIN);
            if (lane == leader) acc.max_i64(A, k0, r);
          }
        }
      } else if (in) {
        if (A.type == PA_AGG_SUM) {
          if (A.src == SRC_INT) {
            acc.add_i64(A, key, v.i);
          } else if (A.src == SRC_LONG) {
            acc.add_i64(A, 2 * key, (int64_t)(uint32_t)v.i);
            acc.add_i64(A, 2 * key + 1, v.i >> 32);
          } else {
            acc.add_f64(A, key, v.d);
          }
        } else {
          const int64_t e = A.src != SRC_DOUBLE ? v.i : f64_order_encode(v.d);
          if (A.type == PA_AGG_MIN) acc.min_i64(A, key, e);
          else acc.max_i64(A, key, e);
        }
      }
    }
  }
}

// Value of an aggregation at value index `vi` of an MV dictionary column (SUMMV / MINMV / MAXMV / DISTINCTCOUNTHLLMV).
__device__ __forceinline__ AggValue agg_value_mv(const DevAgg& A, int a, const DevSeg* __restrict__ seg,
                                                 const DevCol& c, int64_t vi) {
  AggValue out{0, 0.0};
  const uint32_t id = decode_global(c.words, vi, c.nbits);
  if (A.type == PA_AGG_DISTINCTCOUNTHLL) out.i = gp(seg->hll_lut[a])[id];
  else if (A.type == PA_AGG_DISTINCTCOUNT) out.i = seg->hll_lut[a] != nullptr ? gp(seg->hll_lut[a])[id] : id;
  else if (A.src != SRC_DOUBLE) out.i = gp(c.dict_i64)[id];
  else out.d = gp(c.dict_f64)[id];
  return out;
}

template <int STRAT>
__device__ __forceinline__ void update_one(const DevAgg& A, int64_t key, const AggValue& v, const Acc<STRAT>& acc) {
  if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
    acc.max_hll(A, key, (uint32_t)v.i);
  } else if (A.type == PA_AGG_DISTINCTCOUNT) {
    acc.set_presence(A, key, v.i);
  } else if (A.type == PA_AGG_SUM) {
    if (A.src == SRC_INT) {
      acc.add_i64(A, key, v.i);
    } else if (A.src == SRC_LONG) {
      acc.add_i64(A, 2 * key, (int64_t)(uint32_t)v.i);
      acc.add_i64(A, 2 * key + 1, v.i >> 32);
    } else {
      acc.add_f64(A, key, v.d);
    }
  } else {
    const int64_t e = A.src != SRC_DOUBLE ? v.i : f64_order_encode(v.d);
    if (A.type == PA_AGG_MIN) acc.min_i64(A, key, e);
    else acc.max_i64(A, key, e);
  }
}

// One aggregation update of group `key` in the workgroup's LDS accumulators (STRAT_LDS layout: DevAgg::lds_off), through
// address-space-3 pointers (ds_* atomics). v: AggValue of agg_value (HLL: register << 8 | rank; DISTINCTCOUNT: value id).
__device__ __forceinline__ void lds_update(int type, int src, int log2m, int64_t nvals, uint32_t off,
                                           unsigned char* lds, int64_t key, const AggValue& v) {
  unsigned char* b = lds + off;
  switch (type) {
    case PA_AGG_SUM:
      if (src == SRC_INT) {
        __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(b) + key, (uint64_t)v.i, WG_RLX);
      } else if (src == SRC_LONG) {
        __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(b) + 2 * key, (uint64_t)(uint32_t)v.i, WG_RLX);
        __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(b) + 2 * key + 1, (uint64_t)(v.i >> 32), WG_RLX);
      } else {
        __hip_atomic_fetch_add((__attribute__((address_space(3))) double*)lds_ptr(b) + key, v.d, WG_RLX);
      }
      break;
    case PA_AGG_COUNT_MV:
      __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(b) + key, (uint64_t)v.i, WG_RLX);
      break;
    case PA_AGG_MIN:
    case PA_AGG_MAX: {
      const int64_t e = src != SRC_DOUBLE ? v.i : f64_order_encode(v.d);
      __attribute__((address_space(3))) int64_t* t = (__attribute__((address_space(3))) int64_t*)lds_ptr(b) + key;
      if (type == PA_AGG_MIN) __hip_atomic_fetch_min(t, e, WG_RLX);
      else __hip_atomic_fetch_max(t, e, WG_RLX);
    } break;
    case PA_AGG_DISTINCTCOUNTHLL:
      __hip_atomic_fetch_max(lds_ptr(b) + ((key << log2m) + ((uint32_t)v.i >> 8)), (uint32_t)v.i & 0xffu, WG_RLX);
      break;
    case PA_AGG_DISTINCTCOUNT:
      ((__attribute__((address_space(3))) uint8_t*)lds_ptr(b))[key * nvals + v.i] = 1;
      break;
    default: break;
  }
}

// LDS-privatised accumulators, lane-major tile: each lane walks its own matching docs (doc 32 * lane + i), four per
// batch — every group-by decode of the batch, then every remap gather, then every aggregation value load, then the LDS
// updates — so a tile costs the wave max-popcount / 4 dependent round trips instead of one per 64-doc step (the
// step-major path waits on each step's value loads before its wave-level key grouping). Lanes sharing a key meet in
// the LDS atomics (DefaultGroupByExecutor.aggregateGroupBySV per doc).
template <int kB>
__device__ __forceinline__ void accumulate_lds_lm(const DevQuery* __restrict__ q_in, const DevSeg* __restrict__ seg,
                                                  const uint32_t* img, int64_t doc_base, uint32_t m, int lane,
                                                  unsigned char* lds) {
  CQ* q = (CQ*)(uintptr_t)q_in;
  CSegT* cs = (CSegT*)(uintptr_t)seg;
  const int64_t d0 = doc_base + 32 * lane;
  lds_u32_t* cnt = lds_ptr(lds + q->lds_count_off);
  const int ngb = q->num_gb, na = q->num_aggs;
  while (__ballot(m != 0) != 0) {
    bool on[kB];
    int il[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      on[k] = m != 0;
      il[k] = on[k] ? __builtin_ctz(m) : 0;
      m &= m - 1u;
    }
    int64_t key[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) key[k] = 0;
    for (int j = 0; j < ngb; ++j) {
      const int slot = q->gb_slot[j];
      const int gl = cs->cols[slot].lds_off, gn = cs->cols[slot].nbits;
      const uint32_t* gw = cs->cols[slot].words;
      const int32_t* rm = cs->remap[j];
      const int64_t st = q->gb_stride[j];
      uint32_t id[kB];
#pragma unroll
      for (int k = 0; k < kB; ++k) {
        id[k] = 0u;
        if (on[k]) id[k] = gl >= 0 ? decode_lds(img + gl, 32 * lane + il[k], gn) : decode_global(gw, d0 + il[k], gn);
      }
      if (rm != nullptr) {
#pragma unroll
        for (int k = 0; k < kB; ++k)
          if (on[k]) id[k] = (uint32_t)gp(rm)[id[k]];
      }
#pragma unroll
      for (int k = 0; k < kB; ++k) key[k] += (int64_t)id[k] * st;
    }
#pragma unroll
    for (int k = 0; k < kB; ++k)
      if (on[k]) __hip_atomic_fetch_add(cnt + key[k], 1u, WG_RLX);
    for (int a = 0; a < na; ++a) {
      const int type = q->aggs[a].type;
      if (type == PA_AGG_COUNT) continue;
      const DevAgg& A = q_in->aggs[a];
      AggValue v[kB];
#pragma unroll
      for (int k = 0; k < kB; ++k)
        v[k] = on[k] ? agg_value(A, a, seg, img, 32 * lane + il[k], d0 + il[k]) : AggValue{0, 0.0};
      const int src = q->aggs[a].src, lg = q->aggs[a].log2m;
      const int64_t nv = q->aggs[a].nvals;
      const uint32_t off = (uint32_t)q->aggs[a].lds_off;
#pragma unroll
      for (int k = 0; k < kB; ++k)
        if (on[k]) lds_update(type, src, lg, nv, off, lds, key[k], v[k]);
    }
  }
}

// accumulate_lds_lm for a dense lane-major tile whose non-COUNT aggregations (SUM / MIN / MAX) all read one raw column
// (slot q->lds_raw_slot): that column's values of the tile arrive as coalesced 16-byte loads (instruction k, lane l:
// docs VPL * (64 k + l) + j, as in lane_raw_dense) with their match bits from the lanes owning the docs (ds_bpermute);
// the lane decodes the group key of each such doc from the staged image (any doc of the tile is in it) and updates.
template <int VB>
__device__ __forceinline__ void accumulate_lds_raw_dense(const DevQuery* __restrict__ q_in,
                                                         const DevSeg* __restrict__ seg, const uint32_t* img,
                                                         int64_t doc_base, uint32_t m, int lane, unsigned char* lds) {
  CQ* q = (CQ*)(uintptr_t)q_in;
  CSegT* cs = (CSegT*)(uintptr_t)seg;
  constexpr int VPL = 16 / VB;
  constexpr int NI = 2048 * VB / 1024;
  constexpr int KB = VB == 8 ? 4 : 8;  // loads in flight per batch (16 VGPRs of values)
  const int rs = q->lds_raw_slot;
  const int vt = cs->cols[rs].vtype;
  const AS1 u32x4* p = (const AS1 u32x4*)((const char*)cs->cols[rs].raw + doc_base * VB) + lane;
  lds_u32_t* cnt = lds_ptr(lds + q->lds_count_off);
  const int ngb = q->num_gb, na = q->num_aggs;
#pragma unroll 1
  for (int k0 = 0; k0 < NI; k0 += KB) {
    u32x4 w[KB];
    uint32_t mb[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      w[k] = p[(k0 + k) * kWave];
      const int owner = 2 * VPL * (k0 + k) + ((VPL * lane) >> 5);
      mb[k] = ((uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)m) >> ((VPL * lane) & 31)) & ((1u << VPL) - 1u);
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int k1 = k0 + k;
      int64_t key[VPL];
#pragma unroll
      for (int j = 0; j < VPL; ++j) key[j] = 0;
      for (int g = 0; g < ngb; ++g) {
        const int slot = q->gb_slot[g];
        const int gl = cs->cols[slot].lds_off, gn = cs->cols[slot].nbits;
        const uint32_t* gw = cs->cols[slot].words;
        const int32_t* rm = cs->remap[g];
        const int64_t st = q->gb_stride[g];
        uint32_t id[VPL];
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
          const int dl = VPL * (64 * k1 + lane) + j;  // tile-local doc (lane-major image: any doc is decodable here)
          id[j] = 0u;
          if ((mb[k] >> j) & 1u) id[j] = gl >= 0 ? decode_lds(img + gl, dl, gn) : decode_global(gw, doc_base + dl, gn);
        }
        if (rm != nullptr) {
#pragma unroll
          for (int j = 0; j < VPL; ++j)
            if ((mb[k] >> j) & 1u) id[j] = (uint32_t)gp(rm)[id[j]];
        }
#pragma unroll
        for (int j = 0; j < VPL; ++j) key[j] += (int64_t)id[j] * st;
      }
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        if (!((mb[k] >> j) & 1u)) continue;
        const uint64_t x = VB == 8 ? ((uint64_t)w[k][2 * j + 1] << 32) | w[k][2 * j] : (uint64_t)w[k][j];
        AggValue v;
        if (vt == PA_INT) { v.i = (int64_t)(int32_t)(uint32_t)x; v.d = (double)v.i; }
        else if (vt == PA_LONG) { v.i = (int64_t)x; v.d = (double)v.i; }
        else if (vt == PA_FLOAT) { v.d = __builtin_bit_cast(float, (uint32_t)x); v.i = (int64_t)(int32_t)(uint32_t)x; }
        else { v.d = __builtin_bit_cast(double, x); v.i = (int64_t)x; }
        __hip_atomic_fetch_add(cnt + key[j], 1u, WG_RLX);
        for (int a = 0; a < na; ++a) {
          const int type = q->aggs[a].type;
          if (type == PA_AGG_COUNT) continue;
          lds_update(type, q->aggs[a].src, 0, 0, (uint32_t)q->aggs[a].lds_off, lds, key[j], v);
        }
      }
    }
  }
}

// COUNT += 1 and every aggregation of one doc into accumulator slot `key`; an MV aggregation column contributes every
// value of the doc (aggregateGroupByMV / *MVAggregationFunction).
template <int STRAT, bool G = false>
__device__ __forceinline__ void update_doc_key(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                               const uint32_t* img, int doc_local, int64_t doc, int64_t key,
                                               const Acc<STRAT>& acc) {
  acc.add_count(key, 1u);
  for (int a = 0; a < q->num_aggs; ++a) {
    const DevAgg& A = q->aggs[a];
    if (A.type == PA_AGG_COUNT) continue;
    const DevCol& c = seg->cols[A.slot];
    if (c.kind == COL_MV_DICT) {
      const int32_t v0 = gp(c.mv_off)[doc], v1 = gp(c.mv_off)[doc + 1];
      if (A.type == PA_AGG_COUNT_MV) {
        acc.add_i64(A, key, (int64_t)(v1 - v0));
        continue;
      }
      for (int32_t vi = v0; vi < v1; ++vi) update_one<STRAT>(A, key, agg_value_mv(A, a, seg, c, vi), acc);
    } else {
      update_one<STRAT>(A, key, agg_value<G>(A, a, seg, img, doc_local, doc), acc);
    }
  }
}

// One matching doc of a query with a multi-value group-by or aggregation column, on its own lane (no wave
// grouping): the doc expands into the cartesian product of its MV group-by values (DictionaryBasedGroupKeyGenerator
// .getIntRawKeys; duplicates included, like the reference), and every key receives COUNT += 1 and every aggregation
// — over all values of an MV aggregation column (aggregateGroupByMV / *MVAggregationFunction).
template <int STRAT>
__device__ void accumulate_doc_mv(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                  const uint32_t* img, int doc_local, int64_t doc, const Acc<STRAT>& acc) {
  int64_t base_key[2] = {0, 0};
  int nmv = 0;
  int mv_gb[PA_MAX_GROUP_BY];
  int32_t mv_s[PA_MAX_GROUP_BY], mv_n[PA_MAX_GROUP_BY];
  int64_t combos = 1;
  for (int j = 0; j < q->num_gb; ++j) {
    const DevCol& c = seg->cols[q->gb_slot[j]];
    if (c.kind == COL_MV_DICT) {
      const int32_t s0 = gp(c.mv_off)[doc];
      mv_gb[nmv] = j;
      mv_s[nmv] = s0;
      mv_n[nmv] = gp(c.mv_off)[doc + 1] - s0;
      combos *= mv_n[nmv];
      ++nmv;
    } else {
      base_key[q->gb_word[j]] += (int64_t)(gb_component(c, seg->remap[j], img, doc_local, doc) * (uint64_t)q->gb_stride[j]);
    }
  }
  for (int64_t cb = 0; cb < combos; ++cb) {
    int64_t kw[2] = {base_key[0], base_key[1]};
    int64_t rem = cb;
    for (int t = 0; t < nmv; ++t) {
      const int j = mv_gb[t];
      const DevCol& c = seg->cols[q->gb_slot[j]];
      const int64_t digit = rem % mv_n[t];
      rem /= mv_n[t];
      uint32_t id = decode_global(c.words, mv_s[t] + digit, c.nbits);
      const int32_t* rm = seg->remap[j];
      if (rm != nullptr) id = (uint32_t)gp(rm)[id];
      kw[q->gb_word[j]] += (int64_t)id * q->gb_stride[j];
    }
    const int64_t key = key_slot(q, kw[0], kw[1]);
    if (key < 0) continue;
    // numGroupsLimit, walk form (direct key space): only the keys the segment admitted
    if (seg->admit != nullptr && !((gp(seg->admit)[key >> 5] >> (key & 31)) & 1u)) continue;
    update_doc_key<STRAT>(q, seg, img, doc_local, doc, key, acc);
  }
}

// RAW_SET membership (RawValueBasedInPredicateEvaluatorFactory's value sets): the set's first / last value bound it,
// then a binary search of the sorted values (a few L2-resident loads per doc)
template <class LeafT>
__device__ __forceinline__ bool raw_set_has(const LeafT& L, int64_t x) {
  if (x < L.ilo || x > L.ihi) return false;
  const AS1 int64_t* v = gp((const int64_t*)L.lut);
  int32_t b = 0, n = L.span;
  while (n > 1) {
    const int32_t h = n >> 1;
    b = v[b + h] <= x ? b + h : b;
    n -= h;
  }
  return v[b] == x;
}
template <class LeafT>
__device__ __forceinline__ bool raw_set_has(const LeafT& L, double x) {
  if (!(x >= L.dlo && x <= L.dhi)) return false;
  const AS1 double* v = gp((const double*)L.lut);
  int32_t b = 0, n = L.span;
  while (n > 1) {
    const int32_t h = n >> 1;
    b = v[b + h] <= x ? b + h : b;
    n -= h;
  }
  return v[b] == x;
}

// Match word of one leaf over a whole wave tile: bit i of lane l <=> doc 64*i + l of the tile matches.
// Leaf parameters are loaded once per tile; the 32 decodes are independent, so the LDS reads pipeline.
template <int STEPS, class LeafT = DevLeaf>
__device__ __forceinline__ uint32_t leaf_bits(const LeafT& L, const uint32_t* img, int64_t doc_base, int lane) {
  uint32_t bits = 0;
  if (L.kind == PA_LEAF_DICT_RANGE || L.kind == PA_LEAF_DICT_SET) {
    const int nb = L.nbits;
    const uint32_t mask = nbits_mask(nb);
    const uint32_t e1 = (uint32_t)lane * (uint32_t)nb + (uint32_t)(nb - 1);
    const uint32_t sh = (~e1) & 31u;
    const int step = 2 * nb;  // stream words per 64-doc step
    {
      const uint32_t* p = img + L.lds_off + (int)(e1 >> 5);
      if (L.kind == PA_LEAF_DICT_RANGE) {
        // MSB-aligned decode: the window starts at the word holding the value's first bit (or the word before,
        // when that bit is bit 0 of a word), so t = alignbit(.) carries the value in its top nb bits with junk
        // below. With lo' = lo << (32-nb) and hi' = span << (32-nb) - 1 (host-side),
        //   lo <= v < lo + span  <=>  (t - lo') <= hi'   (unsigned; exact for any junk bits).
        // Non-matches accumulate as nm = 2*nm + borrow(hi' - (t - lo')): sub, sub_co, addc per 64 docs.
        const uint32_t lo_t = (uint32_t)L.lo, hi_t = (uint32_t)L.span;  // pre-shifted by the host
        const uint32_t b0 = (uint32_t)lane * (uint32_t)nb;
        const uint32_t o = b0 & 31u;
        const int ws = (int)(b0 >> 5) - (o == 0 ? 1 : 0);
        const uint32_t shr = (32u - o) & 31u;
        // every scalar parameter in SGPRs before the first LDS read: a scalar load between LDS reads forces
        // lgkmcnt(0) (SMEM returns out of order) and serialises the reads. The window pointer goes through the asm
        // as a 32-bit LDS offset and comes back as an address-space-3 pointer (ds_read; a generic pointer rebuilt
        // from 32 bits would lose the shared aperture and address global memory).
        uint32_t pw_off = lds_addr(img + L.lds_off + ws);
        asm volatile("" : "+v"(pw_off) : "s"(lo_t), "s"(hi_t), "s"(step));
        const lds_u32_t* pw = (const lds_u32_t*)(uintptr_t)pw_off;
        uint32_t w0[STEPS], w1[STEPS];
#pragma unroll
        for (int i = 0; i < STEPS; ++i) {
          w0[i] = pw[i * step];
          w1[i] = pw[i * step + 1];
        }
        uint32_t nm = 0;
#pragma unroll
        for (int i = STEPS - 1; i >= 0; --i) {
          const uint32_t t = __builtin_amdgcn_alignbit(w0[i], w1[i], shr);
          uint32_t u;
          // u = t - lo'; borrow = hi' < u (non-match); nm = 2*nm + borrow  (the compiler otherwise rewrites the
          // carry-add into cndmask + or)
          asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
              "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
              "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
              : [nm] "+v"(nm), [u] "=&v"(u)
              : [t] "v"(t), [lo] "s"(lo_t), [hi] "s"(hi_t)
              : "vcc");
        }
        bits = STEPS == 32 ? ~nm : (~nm & ((1u << STEPS) - 1u));
        (void)mask;
        (void)p;
      } else {
        const AS1 uint32_t* lut = gp(L.lut);
#pragma unroll 8
        for (int i = 0; i < STEPS; ++i) {
          const uint32_t id = __builtin_amdgcn_alignbit(p[i * step - 1], p[i * step], sh) & mask;
          bits |= ((lut[id >> 5] >> (id & 31u)) & 1u) << i;
        }
      }
    }  // filter columns are always staged (pa_query_prepare), so there is no lazy filter-decode path
  } else if (L.kind == PA_LEAF_RAW_SET) {  // coalesced loads of the raw values, a set lookup each
    const int64_t d0 = doc_base + lane;
    for (int i = 0; i < STEPS; ++i) {
      bool m;
      switch (L.vtype) {
        case PA_INT: m = raw_set_has(L, (int64_t)gp((const int32_t*)L.raw)[d0 + i * kWave]); break;
        case PA_LONG: m = raw_set_has(L, gp((const int64_t*)L.raw)[d0 + i * kWave]); break;
        case PA_FLOAT: m = raw_set_has(L, (double)gp((const float*)L.raw)[d0 + i * kWave]); break;
        default: m = raw_set_has(L, gp((const double*)L.raw)[d0 + i * kWave]); break;
      }
      bits |= (uint32_t)m << i;
    }
  } else {  // PA_LEAF_RAW_RANGE: coalesced loads of the raw values
    const int64_t d0 = doc_base + lane;
    switch (L.vtype) {
      case PA_INT: {
        const AS1 int32_t* v = gp((const int32_t*)L.raw) + d0;
#pragma unroll 8
        for (int i = 0; i < STEPS; ++i) {
          const int64_t x = v[i * kWave];
          bits |= (uint32_t)(x >= L.ilo && x <= L.ihi) << i;
        }
      } break;
      case PA_LONG: {
        const AS1 int64_t* v = gp((const int64_t*)L.raw) + d0;
#pragma unroll 8
        for (int i = 0; i < STEPS; ++i) {
          const int64_t x = v[i * kWave];
          bits |= (uint32_t)(x >= L.ilo && x <= L.ihi) << i;
        }
      } break;
      case PA_FLOAT: {
        const AS1 float* v = gp((const float*)L.raw) + d0;
#pragma unroll 8
        for (int i = 0; i < STEPS; ++i) {
          const double x = v[i * kWave];
          bits |= (uint32_t)(x >= L.dlo && x <= L.dhi) << i;
        }
      } break;
      default: {
        const AS1 double* v = gp((const double*)L.raw) + d0;
#pragma unroll 8
        for (int i = 0; i < STEPS; ++i) {
          const double x = v[i * kWave];
          bits |= (uint32_t)(x >= L.dlo && x <= L.dhi) << i;
        }
      } break;
    }
  }
  return L.negate ? ~bits : bits;
}

// A wave-uniform pointer the compiler may hold in VGPRs: readfirstlane puts it in SGPRs, so the descriptor fields
// behind it are scalar loads (vector loads of descriptors need vmcnt waits, which also wait for the in-flight DMA ring).
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (T*)(((uint64_t)hi << 32) | lo);
}

// One literal on one doc, read straight from HBM: the lazy clauses, evaluated only on docs every eager clause
// matched (the leap-frog evaluation of the reference's AndDocIdIterator: later iterators only advance to candidate
// docs). DICT_RANGE bounds are stored MSB-aligned for leaf_bits; lo = lo' >> (32-nb), span = (hi' + 1) >> (32-nb).
__device__ __forceinline__ bool leaf_match_doc(const DevLeaf& L, int64_t doc) {
  bool m;
  if (L.kind == PA_LEAF_MV_DICT_RANGE || L.kind == PA_LEAF_MV_DICT_SET) {
    // MVScanDocIdIterator + applyMV: ANY value in the leaf's set (exclusive predicates arrive negated, so that is
    // NOT ANY == ALL values outside the set). Plain (not MSB-aligned) bounds for MV ranges.
    const int32_t v0 = gp(L.mv_off)[doc], v1 = gp(L.mv_off)[doc + 1];
    m = false;
    for (int32_t v = v0; v < v1 && !m; ++v) {
      const uint32_t id = decode_global(L.words, v, L.nbits);
      m = L.kind == PA_LEAF_MV_DICT_RANGE ? (id - (uint32_t)L.lo) < (uint32_t)L.span
                                          : ((gp(L.lut)[id >> 5] >> (id & 31u)) & 1u) != 0;
    }
  } else if (L.kind == PA_LEAF_DICT_RANGE || L.kind == PA_LEAF_DICT_SET) {
    const uint32_t id = decode_global(L.words, doc, L.nbits);
    if (L.kind == PA_LEAF_DICT_RANGE) {
      const int sh = 32 - L.nbits;
      const uint32_t lo = (uint32_t)L.lo >> sh;
      const uint32_t span = (uint32_t)(((uint64_t)(uint32_t)L.span + 1u) >> sh);
      m = (id - lo) < span;
    } else {
      m = (gp(L.lut)[id >> 5] >> (id & 31u)) & 1u;
    }
  } else if (L.kind == PA_LEAF_RAW_SET) {
    switch (L.vtype) {
      case PA_INT: m = raw_set_has(L, (int64_t)gp((const int32_t*)L.raw)[doc]); break;
      case PA_LONG: m = raw_set_has(L, gp((const int64_t*)L.raw)[doc]); break;
      case PA_FLOAT: m = raw_set_has(L, (double)gp((const float*)L.raw)[doc]); break;
      default: m = raw_set_has(L, gp((const double*)L.raw)[doc]); break;
    }
  } else {
    switch (L.vtype) {
      case PA_INT: { const int64_t x = gp((const int32_t*)L.raw)[doc]; m = x >= L.ilo && x <= L.ihi; } break;
      case PA_LONG: { const int64_t x = gp((const int64_t*)L.raw)[doc]; m = x >= L.ilo && x <= L.ihi; } break;
      case PA_FLOAT: { const double x = gp((const float*)L.raw)[doc]; m = x >= L.dlo && x <= L.dhi; } break;
      default: { const double x = gp((const double*)L.raw)[doc]; m = x >= L.dlo && x <= L.dhi; } break;
    }
  }
  return m != (L.negate != 0);
}

// ---------------------------------------------------------------- fused execution statistics (DevQuery::leap_mode)
// The filter is an AND of two single-value scan leaves: literal 0 (eager, E) and literal 1 (lazy, Z). The reference's
// AndDocIdIterator leap-frogs them with A = Z and B = E (filter_stats._cost_next: numEntriesScannedInFilter = num_docs +
// |A & B| + leaps). Label every doc A-only (1), B-only (2), both (3); in doc order a leap starts at each step
// both -> A-only, start -> A-only, A-only -> B-only and B-only -> A-only between consecutive labelled docs
// (pa_kernels.hip word_leaps). Every such step but the first has an E (= B) doc at one end, so
//   leaps = [the segment's first labelled doc is A-only]
//         + sum over E docs e of ([succ(e) is A-only] + [e is B-only and pred(e) is A-only]),
// with pred / succ the nearest labelled docs before / after e. The scan knows e's label (the lazy clause runs on it) and
// appends (segment, doc, label) to a list (leap_tile); after the scan, leap_search_kernel (pa_kernels.hip) gives every
// listed doc one wave: a wave-wide search over 64 docs per step, both leaves read straight from HBM, stops at the first
// labelled doc (so never past the neighbouring E doc) — in the scan itself every search step's load would wait behind
// the tile ring's in-flight DMA. The planner enables this only for a sparse E; a search that gives up
// (kLeapSearchSteps) or a full list flags the segment(s), whose counts the host then takes from leaf bitmaps.
// leap_out: [3 s]: segment s's matched docs, leaps, gave-up flag; [3 nseg]: list overflow flag; [3 nseg + 1 + w]: the
// docs wave w of the scan listed; then the list: wave w's slice of leap_cap entries at [3 nseg + 1 + slices + w cap],
// one (segment << 40 | doc << 1 | both) per E doc (a wave appends to its own slice: no atomic, no wait).
constexpr int kLeapSearchSteps = 64;  // 4096 docs

// Label of the nearest labelled doc at or beyond `from` in direction dir (+1 / -1) inside the segment: 1, 2, 3; 0 if
// the segment ends first; 4 if the search gave up. (Four rows of 64 docs per step measured slower: 51 vs 34 us for
// configs[1]'s list, r04_d1.)
__device__ __noinline__ uint32_t leap_search(const DevSeg* seg_in, int64_t from, int dir, int lane) {
  const DevSeg* __restrict__ seg = uniform_ptr(seg_in);
  const int64_t n = seg->num_docs;
  for (int k = 0; k < kLeapSearchSteps; ++k) {
    const int64_t d = from + (int64_t)dir * (int64_t)(kWave * k + lane);
    const bool in = d >= 0 && d < n;
    uint32_t lbl = 0u;
    if (in) lbl = (leaf_match_doc(seg->leaves[1], d) ? 1u : 0u) | (leaf_match_doc(seg->leaves[0], d) ? 2u : 0u);
    const uint64_t hit = __ballot(lbl != 0u);
    if (hit) return (uint32_t)__builtin_amdgcn_readlane((int)lbl, __builtin_ctzll(hit));  // lane order = distance
    if (__ballot(in) != ~0ull) return 0u;
  }
  return 4u;
}

// One segment's counters (lane 0 adds them; nothing when all are zero).
__device__ __forceinline__ void leap_add(const DevQuery* __restrict__ q, int seg_index, uint32_t matched, uint32_t leaps,
                                         uint32_t gave_up, int lane) {
  if (lane == 0 && (matched | leaps | gave_up)) {
    unsigned long long* o = q->leap_out + 3 * (int64_t)seg_index;
    if (matched) atomicAdd(o, (unsigned long long)matched);
    if (leaps) atomicAdd(o + 1, (unsigned long long)leaps);
    if (gave_up) atomicOr(o + 2, 1ull);
  }
}

// The E docs of one tile (e: eager clause bits, f: those that also matched the lazy clause) into the list, and the
// tile's matched docs into the segment's counter. LM: doc of bit i of lane l = 32 l + i, else 64 i + l.
template <int LM>
__device__ __forceinline__ void leap_tile(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg, int64_t doc_base,
                                       uint32_t e, uint32_t f, int lane, uint32_t slice, uint32_t& listed,
                                       uint32_t lds_base) {
  const uint32_t mine = (uint32_t)__builtin_popcount(e);
  uint32_t incl = mine;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)incl, o, kWave);
    if (lane >= o) incl += t;
  }
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
  uint32_t matched = (uint32_t)__builtin_popcount(f);
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) matched += (uint32_t)__shfl_xor((int)matched, o, kWave);
  const int si = seg->index;
  const int64_t nseg = q->num_segments;
  const uint64_t cap = (uint64_t)q->leap_cap;
  if ((uint64_t)listed + total > cap) {
    if (lane == 0) atomicOr(q->leap_out + 3 * nseg, 1ull);  // (the host then takes every segment's counts from bitmaps)
  } else {
    AS1 unsigned long long* list =
        gp(q->leap_out) + 3 * nseg + 1 + (int64_t)q->leap_slices + (int64_t)slice * (int64_t)cap;
    const uint32_t lcap = (uint32_t)q->leap_lds_cap;
    lds_u64_t* lds_list = (lds_u64_t*)(uintptr_t)lds_base;
    uint32_t pos = listed + (incl - mine);
    while (e) {
      const int i = __builtin_ctz(e);
      e &= e - 1u;
      const int64_t doc = doc_base + (LM ? 32 * lane + i : kWave * i + lane);
      const uint64_t ent = ((uint64_t)si << 40) | ((uint64_t)doc << 1) | ((f >> i) & 1u);
      if (pos < lcap) lds_list[pos] = ent;
      else list[pos] = ent;
      ++pos;
    }
  }
  listed += total;
  leap_add(q, si, matched, 0u, 0u, lane);
}

// ---------------------------------------------------------------- partitioned aggregation: count + emit passes
// LDS bin state of the emit pass, per partition (V partitions first, then H): records in the bin (may pass the bin
// size while a flush is in progress: the excess goes straight to the range), records written into it, the range's next
// whole-bin slot (front) and its last free record (back), and the range's first record in the stream.
// All of it through address-space-3 pointers: ds_* instructions. A flat access could alias global memory, and waiting
// for one (flat loads count in vmcnt) would drain the tile ring's LDS-DMA.
struct BinState {
  lds_u32_t* cnt;
  lds_u32_t* done;
  lds_u32_t* front;
  lds_u32_t* back;
  lds_u64_t* start;
  lds_u32_t* slk;   // H bins: records of the doc that crossed the bin end, parked past it (<= kDocVals - 1)
};

__device__ __forceinline__ BinState bin_state(const DevQuery* __restrict__ q, unsigned char* lds) {
  return BinState{lds_ptr(lds + q->lds_cnt), lds_ptr(lds + q->lds_done), lds_ptr(lds + q->lds_front),
                  lds_ptr(lds + q->lds_back), (lds_u64_t*)lds_ptr(lds + q->lds_start),
                  lds_ptr(lds + q->lds_slack) - q->pv};  // (slack words exist for the H partitions only)
}

// Wave-level put of K records per lane: every lane calls it (uniform control flow); record k of an active lane (the
// first nw words of r[k]) goes into partition p[k]'s LDS bin of BS records (bins: the stream's partitions from p0 on,
// BS * nw words each). Phases, each a run of independent LDS operations (one wait per phase, not per record):
// claim slots (cnt), write them, count them written (done). The lane whose write completes a bin marks it, and the
// wave then stores every marked bin of the batch at its range's front slot — several bins per store instruction (L
// lanes per bin, one 16-byte unit each) — and empties it; a record whose bin was full claims again after that. Every
// (workgroup, partition) range holds exactly the records the count pass counted, so front and back meet (checked at
// the end of the pass). Without RETRY a record whose bin is full goes to the range's back end instead.
// Ordering: LDS executes the DS instructions of one wave in issue order and serialises those of different waves, so
// "write the slot, then count it done" and "read the bin, then reset the counters" need only the compiler to keep
// program order (a signal fence). Acquire/release atomics would also wait for every outstanding global load, i.e.
// drain the tile ring's LDS-DMA on every record. Only the wave that completed a bin touches its front and counters
// until it resets them (a bin fills at most once per claim round: it stays full until its flush).
template <int K, bool SL = false>
__device__ __forceinline__ void flush_full_bins(const BinState& B, const bool (&full)[K], const uint32_t (&p)[K],
                                                uint32_t p0, lds_u32_t* bins, uint32_t BS, uint32_t nw,
                                                AS1 uint32_t* recs, int lane, int dbg, uint32_t BST = 0);

template <int K, int WM, bool SL = false, bool RETRY = false>
__device__ __forceinline__ void bin_put_batch(const BinState& B, const bool (&act)[K], const uint32_t (&p)[K],
                                              uint32_t p0, lds_u32_t* bins, uint32_t BS, uint32_t nw,
                                              const uint32_t (&r)[K][WM], AS1 uint32_t* recs, int lane, int dbg,
                                              uint32_t BST = 0) {
  if (BST == 0) BST = BS;
  // RETRY (the MV group-by's V records, several per doc: their bins fill fast and the back path's 4-byte stores
  // dominated, r04_c1 -> r04_c3 emit 5.76 -> 4.86 ms) or the back path (one record per doc: the retry rounds cost
  // more than the few scattered stores, configs[2] emit 1.29 -> 1.41 ms, configs[4] V emit 1.5 -> 1.9 ms)
  if constexpr (!RETRY) {
    uint32_t s[K];
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] = act[k] ? __hip_atomic_fetch_add(B.cnt + p[k], 1u, WG_RLX) : 0xffffffffu;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (s[k] < BS) {
        lds_u32_t* slot = bins + ((p[k] - p0) * BST + s[k]) * nw;
#pragma unroll
        for (int w = 0; w < WM; ++w)
          if ((uint32_t)w < nw) slot[w] = r[k][w];
      }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    bool full[K];
#pragma unroll
    for (int k = 0; k < K; ++k) full[k] = s[k] < BS && __hip_atomic_fetch_add(B.done + p[k], 1u, WG_RLX) == BS - 1u;
    if (!(dbg & 1)) {  // a record whose bin is full goes straight to the back end of its range
      uint32_t o[K];
#pragma unroll
      for (int k = 0; k < K; ++k)
        o[k] = (act[k] && s[k] >= BS) ? __hip_atomic_fetch_sub(B.back + p[k], 1u, WG_RLX) - 1u : 0u;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (act[k] && s[k] >= BS) {
          AS1 uint32_t* d = recs + (B.start[p[k]] + o[k]) * (uint64_t)nw;
#pragma unroll
          for (int w = 0; w < WM; ++w)
            if ((uint32_t)w < nw) d[w] = r[k][w];
        }
      }
    }
    flush_full_bins<K, SL>(B, full, p, p0, bins, BS, nw, recs, lane, dbg, BST);
    return;
  }
  // A record whose bin is full (claimed past BS while its completing wave flushes it) retries after this wave has
  // flushed the bins it completed itself (so no wave waits for a bin whose flusher waits too): every record leaves
  // through a whole-bin burst, never as a scattered store (a 4-byte store costs a whole 64-byte HBM write).
  bool pend[K];
#pragma unroll
  for (int k = 0; k < K; ++k) pend[k] = act[k];
  for (int round = 0;; ++round) {
    uint32_t s[K];
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] = pend[k] ? __hip_atomic_fetch_add(B.cnt + p[k], 1u, WG_RLX) : 0xffffffffu;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (s[k] < BS) {
        lds_u32_t* slot = bins + ((p[k] - p0) * BST + s[k]) * nw;
#pragma unroll
        for (int w = 0; w < WM; ++w)
          if ((uint32_t)w < nw) slot[w] = r[k][w];
      }
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    bool full[K];
#pragma unroll
    for (int k = 0; k < K; ++k) full[k] = s[k] < BS && __hip_atomic_fetch_add(B.done + p[k], 1u, WG_RLX) == BS - 1u;
    flush_full_bins<K, SL>(B, full, p, p0, bins, BS, nw, recs, lane, dbg, BST);
    bool any = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      pend[k] = pend[k] && s[k] >= BS;
      any |= pend[k];
    }
    if (__ballot(any) == 0) break;
    if (round > 0) __builtin_amdgcn_s_sleep(2);  // (the bin's flush is a few hundred cycles away)
  }
}

// The flush half of a put: every bin some lane completed (full[k]) is stored at its range's front slot — several bins
// per store instruction (L lanes per bin, one 16-byte unit each) — and emptied.
// SL (H bins of the doc-reserved path): bins are BST records apart and may hold a crossing doc's tail past BS
// (B.slk); after the store it moves to the bin's front and the bin restarts with it.
template <int K, bool SL>
__device__ __forceinline__ void flush_full_bins(const BinState& B, const bool (&full)[K], const uint32_t (&p)[K],
                                                uint32_t p0, lds_u32_t* bins, uint32_t BS, uint32_t nw,
                                                AS1 uint32_t* recs, int lane, int dbg, uint32_t BST) {
  if (BST == 0) BST = BS;
  uint64_t fm[K];
  uint64_t any = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    fm[k] = __ballot(full[k]);
    any |= fm[k];
  }
  if (any == 0) return;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (dbg & 1) {  // (measurement only: drop the bins)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (full[k]) {
        const uint32_t r = SL ? B.slk[p[k]] : 0u;
        if (SL) B.slk[p[k]] = 0u;
        __hip_atomic_store(B.done + p[k], r, WG_RLX);
        __hip_atomic_store(B.cnt + p[k], r, WG_RLX);
      }
    }
    return;
  }
  // L lanes per bin (the bin's 16-byte units, rounded up to a power of two), G = 64 / L bins per store round
  const uint32_t n16 = (BS * nw) >> 2;
  uint32_t L = 1;
  while (L < n16 && L < (uint32_t)kWave) L <<= 1;
  const uint32_t G = (uint32_t)kWave / L;
  const uint32_t grp = (uint32_t)lane / L, c0 = (uint32_t)lane % L;
  uint32_t mine = 0xffffffffu, g = 0;
  auto store_round = [&]() {
    const bool on = grp < g;
    uint32_t o = 0, r = 0;
    if (on) {
      o = B.front[mine];
      AS1 u32x4* d = (AS1 u32x4*)(recs + (B.start[mine] + o) * (uint64_t)nw);
      const lds_u32x4_t* sb = (const lds_u32x4_t*)(bins + (mine - p0) * BST * nw);
      for (uint32_t c = c0; c < n16; c += L) d[c] = sb[c];
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (SL && on) {  // the parked tail (one record per lane, nw == 1) to the bin's front
      r = B.slk[mine];
      lds_u32_t* b1 = bins + (mine - p0) * BST;
      for (uint32_t c = c0; c < r; c += L) b1[c] = b1[BS + c];  // (r < kDocVals; L may be smaller)
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (on && c0 == 0) {
      B.front[mine] = o + BS;
      if (SL) B.slk[mine] = 0u;
      __hip_atomic_store(B.done + mine, r, WG_RLX);
      __hip_atomic_store(B.cnt + mine, r, WG_RLX);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    g = 0;
    mine = 0xffffffffu;
  };
#pragma unroll
  for (int k = 0; k < K; ++k) {
    uint64_t m = fm[k];
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const uint32_t pp = (uint32_t)__builtin_amdgcn_readlane((int)p[k], l);
      if (grp == g) mine = pp;
      if (++g == G) store_round();
    }
  }
  if (g) store_round();
}

// One record per lane (K = 1).
template <int WM>
__device__ __forceinline__ void bin_put_wave(const BinState& B, bool active, uint32_t p, uint32_t p0, lds_u32_t* bins,
                                             uint32_t BS, uint32_t nw, const uint32_t (&r)[WM], AS1 uint32_t* recs,
                                             int lane, int dbg) {
  const bool a[1] = {active};
  const uint32_t pk[1] = {p};
  uint32_t rr[1][WM];
#pragma unroll
  for (int w = 0; w < WM; ++w) rr[0][w] = r[w];
  bin_put_batch<1, WM>(B, a, pk, p0, bins, BS, nw, rr, recs, lane, dbg);
}


// Batched decodes of part_tile: every load of a batch is issued before any of their results is used. (A load whose
// result is consumed inside a per-lane branch gets its wait inside that branch: the batch's round trips serialise.)
// Packed values idx[i] of the stream `words` (nb bits each) for the lanes with on[i]; 0 elsewhere.
template <int N>
__device__ __forceinline__ void decode_global_batch(const uint32_t* words, const int64_t (&idx)[N], const bool (&on)[N],
                                                    int nb, uint32_t (&out)[N]) {
  uint32_t lo[N], hi[N], sh[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t e1 = (uint64_t)idx[i] * (uint64_t)nb + (uint64_t)(nb - 1);
    const int64_t we = (int64_t)(e1 >> 5);
    sh[i] = (~(uint32_t)e1) & 31u;
    lo[i] = hi[i] = 0u;
    if (on[i]) {
      lo[i] = gp(words)[we];
      hi[i] = gp(words)[we - 1];
    }
  }
  const uint32_t mask = nbits_mask(nb);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = on[i] ? (__builtin_amdgcn_alignbit(hi[i], lo[i], sh[i]) & mask) : 0u;
}

// dictIds of the docs of steps h .. h+N-1 (match bits m) of a column: from the staged tile image (region `loff`; every
// doc of the batch lies in the image, so all are read and the matching ones kept) or, lazily, from HBM.
template <int N, int LM>
__device__ __forceinline__ void decode_batch(int loff, int nb, const uint32_t* words, const uint32_t* img,
                                             int64_t doc_base, int h, uint32_t m, int lane, uint32_t (&id)[N]) {
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
  if (loff >= 0) {
    const uint32_t* region = img + loff;
    const uint32_t mask = nbits_mask(nb);
    uint32_t lo[N], hi[N], sh[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const uint32_t e1 = (uint32_t)local(h + i) * (uint32_t)nb + (uint32_t)(nb - 1);
      const int we = (int)(e1 >> 5);
      lo[i] = region[we];
      hi[i] = region[we - 1];
      sh[i] = (~e1) & 31u;
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
      id[i] = ((m >> (h + i)) & 1u) ? (__builtin_amdgcn_alignbit(hi[i], lo[i], sh[i]) & mask) : 0u;
  } else {
    int64_t idx[N];
    bool on[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      idx[i] = doc_base + local(h + i);
      on[i] = (m >> (h + i)) & 1u;
    }
    decode_global_batch<N>(words, idx, on, nb, id);
  }
}

// MV value range [v0, v1) of the matching docs of steps h .. h+N-1 (0, 0 elsewhere, or without an MV column); nd =
// the segment's docs (hoff holds nd + 1 offsets).
template <int N, int LM>
__device__ __forceinline__ void mv_ranges(bool hmv, const int32_t* hoff, int64_t nd, int64_t doc_base, int h, uint32_t m,
                                          int lane, int32_t (&v0)[N], int32_t (&v1)[N]) {
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
  if constexpr (!LM) {
    // step i holds docs doc_base + 64 i + lane: a doc's end offset is the next lane's start offset, so one coalesced
    // load per step (every doc of the step, clamped to nd) plus lane 63's end offset
    int32_t a[N], b[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      a[i] = b[i] = 0;
      if (hmv) {
        const int64_t doc = doc_base + local(h + i);
        a[i] = gp(hoff)[doc < nd ? doc : nd];
        if (lane == kWave - 1) b[i] = gp(hoff)[doc + 1 < nd ? doc + 1 : nd];
      }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int32_t nx = __shfl_down(a[i], 1, kWave);
      const bool on = hmv && ((m >> (h + i)) & 1u);
      v0[i] = on ? a[i] : 0;
      v1[i] = on ? (lane == kWave - 1 ? b[i] : nx) : 0;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      v0[i] = v1[i] = 0;
      if (hmv && ((m >> (h + i)) & 1u)) {
        const int64_t doc = doc_base + local(h + i);
        v0[i] = gp(hoff)[doc];
        v1[i] = gp(hoff)[doc + 1];
      }
    }
  }
}


// Table-wide keys (< 2^32 on the partitioned path) of the docs of steps h .. h+N-1 (match bits m): every group-by
// dictId decode, then every remap gather (they overlap), then the keys.
template <int N, int LM>
__device__ __forceinline__ void part_keys(const DevQuery* __restrict__ q, CSegT* cs, const uint32_t* img,
                                          int64_t doc_base, int h, uint32_t m, int lane, uint32_t (&key)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) key[i] = 0u;
  for (int j = 0; j < q->num_gb; ++j) {
    // (the multi-value component: per value, mv_key_records; the count pass's skipped component: below the partition)
    if (j == q->gb_mv || j == q->count_skip_gb) continue;
    const int slot = q->gb_slot[j];
    const int gl = cs->cols[slot].lds_off, gn = cs->cols[slot].nbits;
    const uint32_t* gw = cs->cols[slot].words;
    const int32_t* rm = cs->remap[j];
    const uint32_t st = (uint32_t)q->gb_stride[j];
    uint32_t id[N];
    decode_batch<N, LM>(gl, gn, gw, img, doc_base, h, m, lane, id);
    if (rm != nullptr) {
#pragma unroll
      for (int i = 0; i < N; ++i)
        if ((m >> (h + i)) & 1u) id[i] = (uint32_t)gp(rm)[id[i]];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) key[i] += id[i] * st;
  }
}

// Element i (wave-uniform) of a register array without dynamic register indexing.
template <int N, class T>
__device__ __forceinline__ T pick(const T (&a)[N], int i) {
  T r = a[0];
#pragma unroll
  for (int k = 1; k < N; ++k) r = i == k ? a[k] : r;
  return r;
}

// The V records of one step of a query grouping by a multi-value column (DictionaryBasedGroupKeyGenerator
// .getIntRawKeys: one key per value of the doc's MV group-by column, duplicates included; a doc without values has no
// key). Lane l holds its doc's key without the MV component (`base`), its first value's index v0 and its value count n
// (0: not matching); `adm` (numGroupsLimit walk form, else null) drops the keys the segment did not admit. Value-parallel, KB x 64 records per round: lane j takes record g = b + 64 k + j, finds the owner
// lane (the first whose inclusive prefix sum of n exceeds g) by a 6-shuffle binary search and decodes that value
// (consecutive records are consecutive values of the stream: the loads coalesce). f(act, key, owner) takes each round.
template <int KB, class F>
__device__ __forceinline__ void mv_key_records(const uint32_t* words, int nb, const int32_t* rm, uint32_t stride,
                                               const uint32_t* adm, uint32_t base, int32_t v0, uint32_t n, int lane,
                                               F&& f) {
  uint32_t incl = n;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += t;
  }
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
#pragma unroll 1
  for (uint32_t b = 0; b < total; b += KB * kWave) {
    bool act[KB];
    uint32_t key[KB], id[KB];
    int own[KB];
    int64_t vi[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const uint32_t g = b + (uint32_t)(k * kWave + lane);
      int ow = 0;
#pragma unroll
      for (int st = kWave / 2; st >= 1; st >>= 1) {
        const uint32_t v = (uint32_t)__shfl((int)incl, ow + st - 1, kWave);
        if (v <= g) ow += st;
      }
      ow = ow < kWave ? ow : kWave - 1;
      const uint32_t o_incl = (uint32_t)__shfl((int)incl, ow, kWave), o_n = (uint32_t)__shfl((int)n, ow, kWave);
      act[k] = g < total;
      own[k] = ow;
      key[k] = (uint32_t)__shfl((int)base, ow, kWave);
      vi[k] = (int64_t)__shfl(v0, ow, kWave) + (int64_t)(g - (o_incl - o_n));
    }
    decode_global_batch<KB>(words, vi, act, nb, id);
    if (rm != nullptr) {
#pragma unroll
      for (int k = 0; k < KB; ++k)
        if (act[k]) id[k] = (uint32_t)gp(rm)[id[k]];
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) key[k] += id[k] * stride;
    if (adm != nullptr) {  // numGroupsLimit, walk form: the keys the segment admitted
      uint32_t w[KB];
#pragma unroll
      for (int k = 0; k < KB; ++k) w[k] = act[k] ? gp(adm)[key[k] >> 5] : 0u;
#pragma unroll
      for (int k = 0; k < KB; ++k) act[k] = act[k] && ((w[k] >> (key[k] & 31u)) & 1u);
    }
    f(act, key, own);
  }
}

// The same records, each lane its own doc (every doc of the step has at most kDocVals values): all of a doc's values
// decoded in one batch (the step's docs are consecutive, so their values are one short stretch of the stream and the
// loads nearly coalesce), no cross-lane shuffles; f(act, key) takes all of them (act[e]: value e exists and is
// admitted).
template <class F>
__device__ __forceinline__ void mv_doc_records(const uint32_t* words, int nb, const int32_t* rm, uint32_t stride,
                                               const uint32_t* adm, uint32_t base, int32_t v0, uint32_t n,
                                               uint32_t maxn, F&& f) {
  uint32_t id[kDocVals], key[kDocVals];
  int64_t vi[kDocVals];
  bool on[kDocVals];
#pragma unroll
  for (int e = 0; e < kDocVals; ++e) {
    vi[e] = (int64_t)v0 + e;
    on[e] = (uint32_t)e < n;
  }
  decode_global_batch<kDocVals>(words, vi, on, nb, id);
  if (rm != nullptr) {
#pragma unroll
    for (int e = 0; e < kDocVals; ++e)
      if (on[e]) id[e] = (uint32_t)gp(rm)[id[e]];
  }
#pragma unroll
  for (int e = 0; e < kDocVals; ++e) key[e] = base + id[e] * stride;
  if (adm != nullptr) {
    uint32_t w[kDocVals];
#pragma unroll
    for (int e = 0; e < kDocVals; ++e) w[e] = on[e] ? gp(adm)[key[e] >> 5] : 0u;
#pragma unroll
    for (int e = 0; e < kDocVals; ++e) on[e] = on[e] && ((w[e] >> (key[e] & 31u)) & 1u);
  }
  f(on, key);
  (void)maxn;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, kWave));
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// The V payload of one value column for the docs of steps h .. h+N-1: V_FMT_ID its table-wide value id (lo), V_FMT_32 /
// V_FMT_64 its value bits (lo, hi): a dictionary gather, or the raw value (a raw DOUBLE's bits unchanged).
template <int N, int LM, int VF>
__device__ __forceinline__ void part_vvals(const DevQuery* __restrict__ q, CSegT* cs, const uint32_t* img,
                                           int64_t doc_base, int h, uint32_t m, int lane, uint32_t (&lo)[N],
                                           uint32_t (&hi)[N]) {
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
#pragma unroll
  for (int i = 0; i < N; ++i) lo[i] = hi[i] = 0u;
  if constexpr (VF == V_FMT_ID || VF == V_FMT_32 || VF == V_FMT_64) {
    const int va = q->emit_val_agg;
    const int vslot = q->aggs[va].slot;
    const int vkind = cs->cols[vslot].kind;
    const int vl = cs->cols[vslot].lds_off, vn = cs->cols[vslot].nbits, vtype = cs->cols[vslot].vtype;
    const uint32_t* vw = cs->cols[vslot].words;
    const uint64_t* vd = q->aggs[va].src == SRC_DOUBLE ? (const uint64_t*)cs->cols[vslot].dict_f64
                                                        : (const uint64_t*)cs->cols[vslot].dict_i64;
    const int32_t* vrm = cs->vremap;
    const void* vraw = cs->cols[vslot].raw;
    if (vkind == COL_SV_DICT) {
      uint32_t vid[N];
      decode_batch<N, LM>(vl, vn, vw, img, doc_base, h, m, lane, vid);
      if constexpr (VF == V_FMT_ID) {
        if (vrm != nullptr) {
#pragma unroll
          for (int i = 0; i < N; ++i)
            if ((m >> (h + i)) & 1u) vid[i] = (uint32_t)gp(vrm)[vid[i]];
        }
#pragma unroll
        for (int i = 0; i < N; ++i) lo[i] = vid[i];
      } else {
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (!((m >> (h + i)) & 1u)) continue;
          const uint64_t v = gp(vd)[vid[i]];
          lo[i] = (uint32_t)v;
          hi[i] = (uint32_t)(v >> 32);
        }
      }
    } else if (vtype == PA_INT) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        if (!((m >> (h + i)) & 1u)) continue;
        lo[i] = (uint32_t)gp((const int32_t*)vraw)[doc_base + local(h + i)];
        hi[i] = (uint32_t)((int32_t)lo[i] >> 31);
      }
    } else {  // LONG, or DOUBLE bits (a SUM/MIN/MAX over a raw DOUBLE column reads the bits unchanged)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        if (!((m >> (h + i)) & 1u)) continue;
        const uint64_t v = gp((const uint64_t*)vraw)[doc_base + local(h + i)];
        lo[i] = (uint32_t)v;
        hi[i] = (uint32_t)(v >> 32);
      }
    }
  }
}

// part_tile of a query grouping by a multi-value column (one V record per (doc, value) pair; V stream only, no
// generic records): the kernel variants STRAT_PCOUNT_MV / pemit_strat(.., mv = 1), so its expansion's registers stay out
// of the SV variants' allocation.
template <int STRAT, int STEPS, int LM>
__device__ __forceinline__ void part_tile_mv(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                          const uint32_t* img, int64_t doc_base, uint32_t m, int lane,
                                          unsigned char* lds, const PartScratch& ps) {
  CSegT* cs = (CSegT*)(uintptr_t)uniform_ptr(seg);
  const int ksv = q->kshift_v;
  const int gmv = q->gb_mv;
  const int mslot = q->gb_slot[gmv];
  const int32_t* moff = cs->cols[mslot].mv_off;
  const uint32_t* mwords = cs->cols[mslot].words;
  const int mnb = cs->cols[mslot].nbits;
  const int32_t* mrm = cs->remap[gmv];
  const uint32_t mstride = (uint32_t)q->gb_stride[gmv];
  constexpr int kEB = 8;
  if constexpr (is_pcount(STRAT) && !LM) {
    // Count pass of GROUP BY <sv>, <mv> whose SV component cannot change a partition (count_skip_gb): a record's
    // partition is (value id * stride) >> shift, so a tile whose docs all match counts its whole value range as one
    // coalesced stream (no per-doc expansion)
    if (gmv >= 0 && q->num_gb == 2 && q->count_skip_gb == 1 - gmv && cs->admit == nullptr) {
      const int64_t nd = (int64_t)cs->num_docs, rem = nd - doc_base;
      uint32_t valid = STEPS == 32 ? 0xffffffffu : ((1u << STEPS) - 1u);
      if (rem < STEPS * kWave) {
        const int64_t n = rem > lane ? (rem - lane + kWave - 1) / kWave : 0;
        valid = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
      }
      if (__ballot(m != valid) == 0) {
        const int64_t d1 = rem < STEPS * kWave ? nd : doc_base + STEPS * kWave;
        const int64_t vlo = gp(moff)[doc_base], vhi = gp(moff)[d1];
        lds_u32_t* hist = lds_ptr(lds);
        constexpr int kVB = 4;
#pragma unroll 1
        for (int64_t v = vlo; v < vhi; v += kVB * kWave) {
          int64_t vi[kVB];
          bool on[kVB];
          uint32_t id[kVB];
#pragma unroll
          for (int k = 0; k < kVB; ++k) {
            vi[k] = v + k * kWave + lane;
            on[k] = vi[k] < vhi;
          }
          decode_global_batch<kVB>(mwords, vi, on, mnb, id);
          if (mrm != nullptr) {
#pragma unroll
            for (int k = 0; k < kVB; ++k)
              if (on[k]) id[k] = (uint32_t)gp(mrm)[id[k]];
          }
#pragma unroll
          for (int k = 0; k < kVB; ++k)
            if (on[k]) __hip_atomic_fetch_add(hist + ((id[k] * mstride) >> ksv), 1u, WG_RLX);
        }
        return;
      }
    }
  }
#pragma unroll 1
  for (int h = 0; h < STEPS; h += kEB) {
    if (__ballot((m >> h) != 0) == 0) break;
    uint32_t key[kEB];
    part_keys<kEB, LM>(q, cs, img, doc_base, h, m, lane, key);  // (without the MV component)
    if constexpr (is_pcount(STRAT)) {
      lds_u32_t* hist = lds_ptr(lds);
      {  // one V record per (doc, value): count each value's partition
        int32_t v0[kEB], v1[kEB];
        mv_ranges<kEB, LM>(true, moff, (int64_t)cs->num_docs, doc_base, h, m, lane, v0, v1);
        if (q->count_skip_gb == gmv && cs->admit == nullptr) {  // the MV component cannot change the partition
#pragma unroll
          for (int i = 0; i < kEB; ++i)
            if (v1[i] > v0[i]) __hip_atomic_fetch_add(hist + (key[i] >> ksv), (uint32_t)(v1[i] - v0[i]), WG_RLX);
          continue;
        }
#pragma clang loop unroll(full)
        for (int i = 0; i < kEB; ++i) {  // (unrolled: constant register indices)
          if (__ballot((m >> (h + i)) & 1u) == 0) continue;
          const int32_t a0 = pick(v0, i), a1 = pick(v1, i);
          const uint32_t nv = (uint32_t)(a1 - a0), maxn = wave_max_u32(nv);
          if (maxn <= (uint32_t)kDocVals) {
            mv_doc_records(mwords, mnb, mrm, mstride, cs->admit, pick(key, i), a0, nv, maxn,
                           [&](const bool (&act)[kDocVals], const uint32_t (&k)[kDocVals]) {
#pragma unroll
                             for (int e = 0; e < kDocVals; ++e)
                               if (act[e]) __hip_atomic_fetch_add(hist + (k[e] >> ksv), 1u, WG_RLX);
                           });
            continue;
          }
          mv_key_records<4>(mwords, mnb, mrm, mstride, cs->admit, pick(key, i), a0, nv, lane,
                            [&](const bool (&act)[4], const uint32_t (&k)[4], const int (&)[4]) {
#pragma unroll
                              for (int kk = 0; kk < 4; ++kk)
                                if (act[kk]) __hip_atomic_fetch_add(hist + (k[kk] >> ksv), 1u, WG_RLX);
                            });
        }
        continue;
      }
    } else {
      constexpr int VF = pemit_vf(STRAT);
      constexpr int NW = VF == V_FMT_32 ? 2 : (VF == V_FMT_64 ? 3 : 1);
      const BinState B = bin_state(q, lds);
      const int dbg = q->debug_emit;
      const uint32_t W = (uint32_t)NW;
      const uint32_t BS = (uint32_t)q->bs_v;
      lds_u32_t* bins = lds_ptr(lds + q->lds_bins_v);
      const uint32_t kmask = (1u << ksv) - 1u;
      uint32_t lo[kEB], hi[kEB];
      part_vvals<kEB, LM, VF>(q, cs, img, doc_base, h, m, lane, lo, hi);
          {  // one record per (doc, value) pair, the doc's payload on each
            int32_t v0[kEB], v1[kEB];
            mv_ranges<kEB, LM>(true, moff, (int64_t)cs->num_docs, doc_base, h, m, lane, v0, v1);
#pragma clang loop unroll(full)
            for (int i = 0; i < kEB; ++i) {  // (unrolled: constant register indices)
              if (__ballot((m >> (h + i)) & 1u) == 0) continue;
              const int32_t a0 = pick(v0, i), a1 = pick(v1, i);
              const uint32_t dlo = pick(lo, i), dhi = pick(hi, i);
              const uint32_t nv = (uint32_t)(a1 - a0), maxn = wave_max_u32(nv);
              // each record: key offset (| value id), the doc's payload
              auto rec = [&](uint32_t k, uint32_t plo, uint32_t phi, uint32_t (&r)[NW]) {
                r[0] = k & kmask;
#pragma unroll
                for (int w = 1; w < NW; ++w) r[w] = 0u;
                if constexpr (VF == V_FMT_ID) {
                  r[0] |= plo << ksv;
                } else if constexpr (VF == V_FMT_32) {
                  r[1] = plo;
                } else if constexpr (VF == V_FMT_64) {
                  r[1] = plo;
                  r[2] = phi;
                }
              };
              if (maxn <= (uint32_t)kDocVals) {  // each lane its own doc's records, all in one put (one wait per phase)
                mv_doc_records(mwords, mnb, mrm, mstride, cs->admit, pick(key, i), a0, nv, maxn,
                               [&](const bool (&act)[kDocVals], const uint32_t (&k)[kDocVals]) {
                                 uint32_t pk[kDocVals], r[kDocVals][NW];
#pragma unroll
                                 for (int e = 0; e < kDocVals; ++e) {
                                   pk[e] = k[e] >> ksv;
                                   rec(k[e], dlo, dhi, r[e]);
                                 }
                                 bin_put_batch<kDocVals, NW, false, true>(B, act, pk, 0u, bins, BS, W, r, gp(ps.recs_v),
                                                                          lane, dbg);
                               });
                continue;
              }
              mv_key_records<4>(mwords, mnb, mrm, mstride, cs->admit, pick(key, i), a0, nv, lane,
                                [&](const bool (&act)[4], const uint32_t (&k)[4], const int (&own)[4]) {
                                  uint32_t pk[4], r[4][NW];
#pragma unroll
                                  for (int kk = 0; kk < 4; ++kk) {
                                    const uint32_t olo = (uint32_t)__shfl((int)dlo, own[kk], kWave);
                                    pk[kk] = k[kk] >> ksv;
                                    r[kk][0] = k[kk] & kmask;
#pragma unroll
                                    for (int w = 1; w < NW; ++w) r[kk][w] = 0u;
                                    if constexpr (VF == V_FMT_ID) {
                                      r[kk][0] |= olo << ksv;
                                    } else if constexpr (VF == V_FMT_32) {
                                      r[kk][1] = olo;
                                    } else if constexpr (VF == V_FMT_64) {
                                      r[kk][1] = olo;
                                      r[kk][2] = (uint32_t)__shfl((int)dhi, own[kk], kWave);
                                    }
                                  }
                                  bin_put_batch<4, NW, false, true>(B, act, pk, 0u, bins, BS, W, r, gp(ps.recs_v), lane,
                                                                    dbg);
                                });
            }
            continue;
          }
    }
  }
}

// The matching docs of one tile (match words m) in the count pass (STRAT_PCOUNT: per (workgroup, partition) record
// counts in LDS) or the emit pass (STRAT_PEMIT: the records into the partition bins). Per batch of 8 steps: every
// group-by dictId decode, then every remap gather (they overlap), then the table-wide keys; then per stream.
template <int STRAT, int STEPS, int LM>
__device__ __forceinline__ void part_tile(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                          const uint32_t* img, int64_t doc_base, uint32_t m, int lane,
                                          unsigned char* lds, const PartScratch& ps) {
  // Descriptors through the constant address space: the segment is read-only during the kernel and its pointer is
  // wave-uniform, so every field is a scalar load the compiler keeps across the LDS atomics and the record stores.
  CSegT* cs = (CSegT*)(uintptr_t)seg;
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
  const int pv = q->pv;
  const int ksv = q->kshift_v, ksh = q->kshift_h;
  const int ha = q->hll_agg;
  const int hslot = ha >= 0 ? q->aggs[ha].slot : 0;
  const bool hmv = ha >= 0 && cs->cols[hslot].kind == COL_MV_DICT;
  const int32_t* hoff = cs->cols[hslot].mv_off;
  // steps per batch (register budget; 4 for the H-only emit measured slower: 4.83 vs 4.65 ms). The V-only emit of
  // 4-wave workgroups runs at most 2 workgroups per CU (its LDS bins), so it has the VGPRs for a whole tile per batch.
  constexpr int kEB = (is_pemit(STRAT) && !pemit_hh(STRAT) && !pemit_big(STRAT) && pemit_vf(STRAT) != V_FMT_GEN) ? 16 : 8;
  if constexpr (part_mv(STRAT)) {
    part_tile_mv<STRAT, STEPS, LM>(q, seg, img, doc_base, m, lane, lds, ps);
    return;
  }
#pragma unroll 1
  for (int h = 0; h < STEPS; h += kEB) {
    if (__ballot((m >> h) != 0) == 0) break;  // wave-uniform: the H records below shuffle across all 64 lanes
    uint32_t key[kEB];
    part_keys<kEB, LM>(q, cs, img, doc_base, h, m, lane, key);  // table-wide key (< 2^32 on this path)
    if constexpr (is_pcount(STRAT)) {
      lds_u32_t* hist = lds_ptr(lds);
      uint32_t n[kEB];
      {
        int32_t v0[kEB], v1[kEB];
        mv_ranges<kEB, LM>(hmv, hoff, (int64_t)cs->num_docs, doc_base, h, m, lane, v0, v1);
#pragma unroll
        for (int i = 0; i < kEB; ++i) n[i] = v1[i] - v0[i] > 0 ? (uint32_t)(v1[i] - v0[i]) : 1u;
      }
#pragma unroll
      for (int i = 0; i < kEB; ++i) {
        if (!((m >> (h + i)) & 1u)) continue;
        if (pv) __hip_atomic_fetch_add(hist + (key[i] >> ksv), 1u, WG_RLX);
        if (ha >= 0) __hip_atomic_fetch_add(hist + pv + (key[i] >> ksh), n[i], WG_RLX);
      }
    } else {
      constexpr int VF = pemit_vf(STRAT);
      const BinState B = bin_state(q, lds);
      const int dbg = q->debug_emit;
      if constexpr (VF >= 0) {
        // V records: the value (or its table-wide value id) of the one payload column, batched like the keys
        constexpr int NW = VF == V_FMT_GEN ? kMaxVWords : (VF == V_FMT_32 ? 2 : (VF == V_FMT_64 ? 3 : 1));
        const uint32_t W = VF == V_FMT_GEN ? (uint32_t)q->rec_words_v : (uint32_t)NW;
        const uint32_t BS = (uint32_t)q->bs_v;
        lds_u32_t* bins = lds_ptr(lds + q->lds_bins_v);
        const uint32_t kmask = (1u << ksv) - 1u;
        uint32_t lo[kEB], hi[kEB];
        part_vvals<kEB, LM, VF>(q, cs, img, doc_base, h, m, lane, lo, hi);
        if constexpr (VF != V_FMT_GEN) {
          // the batch's records (one per matching doc of the kEB steps) in one put: every LDS phase runs once
          bool act[kEB];
          uint32_t pk[kEB], r[kEB][NW];
#pragma unroll
          for (int i = 0; i < kEB; ++i) {
            act[i] = (m >> (h + i)) & 1u;
            pk[i] = key[i] >> ksv;
            r[i][0] = key[i] & kmask;
#pragma unroll
            for (int w = 1; w < NW; ++w) r[i][w] = 0u;
            if constexpr (VF == V_FMT_ID) {
              r[i][0] |= lo[i] << ksv;
            } else if constexpr (VF == V_FMT_32) {
              r[i][1] = lo[i];
            } else if constexpr (VF == V_FMT_64) {
              r[i][1] = lo[i];
              r[i][2] = hi[i];
            }
          }
          bin_put_batch<kEB, NW>(B, act, pk, 0u, bins, BS, W, r, gp(ps.recs_v), lane, dbg);
        }
        if constexpr (VF == V_FMT_GEN) {  // every payload of the record (one put per step: up to kMaxVWords words)
#pragma unroll
        for (int i = 0; i < kEB; ++i) {
          const bool mine = (m >> (h + i)) & 1u;
          if (__ballot(mine) == 0) continue;
          const uint32_t p = key[i] >> ksv;
          uint32_t r[NW];
          r[0] = key[i] & kmask;
#pragma unroll
          for (int w = 1; w < NW; ++w) r[w] = 0u;
          {
            if (mine) {
              const int dl = local(h + i);
              const int64_t doc = doc_base + dl;
              for (int a = 0; a < q->num_aggs; ++a) {
                const DevAgg& A = q->aggs[a];
                if (A.type == PA_AGG_COUNT || a == ha) continue;
                const AggValue v = agg_value(A, a, seg, img, dl, doc);
                const int po = A.pay_off;
                if (A.src == SRC_INT) {
                  if (po < kMaxVWords) r[po] = (uint32_t)v.i;
                } else {
                  const int64_t b = A.src == SRC_DOUBLE ? __builtin_bit_cast(int64_t, v.d) : v.i;
                  if (po + 1 < kMaxVWords) {
                    r[po] = (uint32_t)b;
                    r[po + 1] = (uint32_t)(b >> 32);
                  }
                }
              }
            }
          }
          bin_put_wave<NW>(B, mine, p, 0u, bins, BS, W, r, gp(ps.recs_v), lane, dbg);
        }
        }
      }
      if constexpr (pemit_hh(STRAT)) {
        // H records, value-parallel per step: each matching lane's doc owns n = max(1, values) consecutive records of
        // the step; lane j takes record g = b + j, finds its owner by a 6-shuffle binary search over the inclusive
        // prefix sums of n, and decodes that value (coalesced MV reads, no per-lane loop over a doc's values)
        const DevAgg& H = q->aggs[ha];
        const uint32_t* hwords = cs->cols[hslot].words;
        const int hnb = cs->cols[hslot].nbits;
        const uint32_t* hlut = cs->hll_lut[ha];  // dictId -> (register << 8) | rank
        const uint32_t BS = (uint32_t)q->bs_h;
        const uint32_t BST = BS + (uint32_t)kDocVals;  // bin stride: room for a crossing doc's tail
        lds_u32_t* bins = lds_ptr(lds + q->lds_bins_h);
        const uint32_t kmask = (1u << ksh) - 1u;
        const int fsh = H.log2m + 6;
        const uint32_t first_bit = q->h_first ? 1u : 0u;
        // every step's value ranges first (one wait for the batch)
        int32_t v0s[kEB], nvs[kEB];
        mv_ranges<kEB, LM>(hmv, hoff, (int64_t)cs->num_docs, doc_base, h, m, lane, v0s, nvs);
#pragma unroll
        for (int i = 0; i < kEB; ++i) nvs[i] -= v0s[i];
        // Doc-reserved batch path (every matching doc of the batch has at most kDocVals records), kHS steps at a time
        // with every phase a run of independent operations (one wait per phase): reserve each doc's consecutive bin
        // slots (one cnt atomic per doc; records past the bin's end are reserved at the back of the range), decode
        // every value of every doc (each lane its own docs: the step's docs are consecutive, so their values are one
        // short stretch of the MV stream and the loads stay nearly coalesced), gather their (register, rank), write
        // the records, count them done (one atomic per doc), store the bins that filled.
        bool big = false;
#pragma unroll
        for (int i = 0; i < kEB; ++i) big |= ((m >> (h + i)) & 1u) && nvs[i] > kDocVals;
        if (hmv && __ballot(big) == 0) {
          constexpr int kHS = 2;
#pragma unroll
          for (int h2 = 0; h2 < kEB; h2 += kHS) {
            bool mn[kHS];
            uint32_t nn[kHS], pp[kHS], sl[kHS], inb[kHS], db[kHS];
            uint32_t maxn = 0;
#pragma unroll
            for (int j = 0; j < kHS; ++j) {
              const int i = h2 + j;
              mn[j] = (m >> (h + i)) & 1u;
              nn[j] = mn[j] ? (nvs[i] > 0 ? (uint32_t)nvs[i] : 1u) : 0u;
              maxn = max(maxn, nn[j]);
              pp[j] = (uint32_t)pv + (key[i] >> ksh);
            }
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) maxn = max(maxn, (uint32_t)__shfl_xor((int)maxn, o, kWave));
            maxn = (uint32_t)__builtin_amdgcn_readfirstlane((int)maxn);
            if (maxn == 0) continue;
#pragma unroll
            for (int j = 0; j < kHS; ++j) sl[j] = mn[j] ? __hip_atomic_fetch_add(B.cnt + pp[j], nn[j], WG_RLX) : 0u;
            // a doc whose slot lies in the bin keeps all its records there (a tail past BS parks in the slack); a doc
            // arriving while the bin is full goes to the back of the range whole
            bool bk[kHS];
#pragma unroll
            for (int j = 0; j < kHS; ++j) {
              bk[j] = mn[j] && sl[j] >= BS;
              inb[j] = (mn[j] && sl[j] < BS) ? min(nn[j], BS - sl[j]) : 0u;
              db[j] = (bk[j] && !(dbg & 1)) ? __hip_atomic_fetch_sub(B.back + pp[j], nn[j], WG_RLX) - nn[j] : 0u;
            }
            uint32_t val[kHS][kDocVals];
#pragma unroll
            for (int j = 0; j < kHS; ++j) {
              int64_t vi[kDocVals];
              bool von[kDocVals];
#pragma unroll
              for (int e = 0; e < kDocVals; ++e) {
                vi[e] = (int64_t)v0s[h2 + j] + e;
                von[e] = (uint32_t)e < maxn && e < nvs[h2 + j] && mn[j];
              }
              if (dbg & 4) {
#pragma unroll
                for (int e = 0; e < kDocVals; ++e) val[j][e] = von[e] ? (uint32_t)e : 0u;
              } else {
                decode_global_batch<kDocVals>(hwords, vi, von, hnb, val[j]);
              }
            }
#pragma unroll
            for (int j = 0; j < kHS; ++j)
#pragma unroll
              for (int e = 0; e < kDocVals; ++e)
                if ((uint32_t)e < maxn && e < nvs[h2 + j] && mn[j] && !(dbg & 2)) val[j][e] = gp(hlut)[val[j][e]];
#pragma unroll
            for (int j = 0; j < kHS; ++j) {
              const uint32_t w = (key[h2 + j] & kmask) << fsh;
              lds_u32_t* bin = bins + (pp[j] - (uint32_t)pv) * BST + sl[j];
              AS1 uint32_t* dd = gp(ps.recs_h) + (B.start[pp[j]] + db[j]);
#pragma unroll
              for (int e = 0; e < kDocVals; ++e) {
                if ((uint32_t)e >= maxn || (uint32_t)e >= nn[j]) continue;
                // (an empty doc's one record has rank 0: no register update; it carries the first-value flag)
                const uint32_t hv = e < nvs[h2 + j] ? val[j][e] : 0u;
                const uint32_t r = w | (e == 0 ? first_bit : 0u) | ((hv >> 8) << 6) | ((hv & 0xffu) << 1);
                if (!bk[j]) bin[e] = r;
                else if (!(dbg & 1)) dd[e] = r;
              }
              if (inb[j] && inb[j] < nn[j]) B.slk[pp[j]] = nn[j] - inb[j];  // the crossing doc's parked tail
            }
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            bool full[kHS];
#pragma unroll
            for (int j = 0; j < kHS; ++j)
              full[j] = inb[j] > 0 && __hip_atomic_fetch_add(B.done + pp[j], inb[j], WG_RLX) + inb[j] == BS;
            flush_full_bins<kHS, true>(B, full, pp, (uint32_t)pv, bins, BS, 1u, gp(ps.recs_h), lane, dbg, BST);
          }
          continue;  // (the batch loop `h`)
        }
#pragma unroll 1
        for (int i = 0; i < kEB; ++i) {
          const bool mine = (m >> (h + i)) & 1u;
          if (__ballot(mine) == 0) continue;
          const int dl = local(h + i);
          const int64_t doc = doc_base + dl;
          uint32_t n = 0, hv_sv = 0;
          const int32_t v0 = v0s[i], nv = nvs[i];
          if (mine) {
            if (hmv) {
              n = nv > 0 ? (uint32_t)nv : 1u;
            } else {
              n = 1u;
              hv_sv = (uint32_t)agg_value(H, ha, seg, img, dl, doc).i;
            }
          }
          if (__ballot(n > (uint32_t)kDocVals) == 0) {
            // Doc-reserved path (every doc of the step has at most kDocVals records): one slot reservation per doc
            // (its records are consecutive in its bin), each lane decodes its own doc's values (the step's docs are
            // consecutive, so their values are one short stretch of the MV stream: the loads stay nearly coalesced),
            // one done count per doc. Records past the bin's end go to the back of the range.
            uint32_t maxn = n;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) maxn = max(maxn, (uint32_t)__shfl_xor((int)maxn, o, kWave));
            maxn = (uint32_t)__builtin_amdgcn_readfirstlane((int)maxn);
            const uint32_t kk = key[i];
            const uint32_t p = (uint32_t)pv + (kk >> ksh);
            const uint32_t sl = mine ? __hip_atomic_fetch_add(B.cnt + p, n, WG_RLX) : 0u;
            const uint32_t inbin = (mine && sl < BS) ? min(n, BS - sl) : 0u;
            const bool bk = mine && sl >= BS;  // (see the batched path: a tail past BS parks in the slack)
            uint32_t db = 0;
            if (bk && !(dbg & 1)) db = __hip_atomic_fetch_sub(B.back + p, n, WG_RLX) - n;
            uint32_t hvv[kDocVals];
            if (hmv) {
              uint32_t idv[kDocVals];
              int64_t vi[kDocVals];
              bool von[kDocVals];
#pragma unroll
              for (int e = 0; e < kDocVals; ++e) {
                vi[e] = (int64_t)v0 + e;
                von[e] = (uint32_t)e < maxn && mine && e < nv;
              }
              if (dbg & 4) {
#pragma unroll
                for (int e = 0; e < kDocVals; ++e) idv[e] = von[e] ? (uint32_t)e : 0u;
              } else {
                decode_global_batch<kDocVals>(hwords, vi, von, hnb, idv);
              }
#pragma unroll
              for (int e = 0; e < kDocVals; ++e) {
                hvv[e] = 0u;  // (an empty doc's one record: rank 0, no register update)
                if ((uint32_t)e < maxn && mine && e < nv) hvv[e] = (dbg & 2) ? idv[e] : gp(hlut)[idv[e]];
              }
            } else {
#pragma unroll
              for (int e = 0; e < kDocVals; ++e) hvv[e] = hv_sv;
            }
            const uint32_t w = (kk & kmask) << fsh;
            lds_u32_t* bin = bins + (p - (uint32_t)pv) * BST + sl;
            AS1 uint32_t* dd = gp(ps.recs_h) + (B.start[p] + db);
#pragma unroll
            for (int e = 0; e < kDocVals; ++e) {
              if ((uint32_t)e >= maxn || !mine || (uint32_t)e >= n) continue;
              const uint32_t r = w | (e == 0 ? first_bit : 0u) | ((hvv[e] >> 8) << 6) | ((hvv[e] & 0xffu) << 1);
              if (!bk) bin[e] = r;
              else if (!(dbg & 1)) dd[e] = r;
            }
            if (inbin && inbin < n) B.slk[p] = n - inbin;
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            bool full[1] = {inbin > 0 && __hip_atomic_fetch_add(B.done + p, inbin, WG_RLX) + inbin == BS};
            const uint32_t pa[1] = {p};
            flush_full_bins<1, true>(B, full, pa, (uint32_t)pv, bins, BS, 1u, gp(ps.recs_h), lane, dbg, BST);
            continue;
          }
          uint32_t incl = n;
#pragma unroll
          for (int o = 1; o < kWave; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += t;
          }
          const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
          const uint32_t kk = key[i];
          constexpr int kHB = 4;  // record chunks of 64 per round: their loads overlap
          for (uint32_t b = 0; b < total; b += kHB * kWave) {
            uint32_t w0[kHB], id[kHB], pk[kHB], alt[kHB];
            int32_t ok[kHB];
            int64_t vi[kHB];
            bool von[kHB];
#pragma unroll
            for (int k = 0; k < kHB; ++k) {
              const uint32_t g = b + (uint32_t)(k * kWave + lane);
              int ow = 0;  // owner lane: the first lane whose inclusive prefix exceeds g
#pragma unroll
              for (int st = kWave / 2; st >= 1; st >>= 1) {
                const uint32_t v = (uint32_t)__shfl((int)incl, ow + st - 1, kWave);
                if (v <= g) ow += st;
              }
              ow = ow < kWave ? ow : kWave - 1;
              const uint32_t o_incl = (uint32_t)__shfl((int)incl, ow, kWave), o_n = (uint32_t)__shfl((int)n, ow, kWave);
              const uint32_t o_key = (uint32_t)__shfl((int)kk, ow, kWave);
              const int32_t o_v0 = __shfl(v0, ow, kWave), o_nv = __shfl(nv, ow, kWave);
              const uint32_t o_hv = (uint32_t)__shfl((int)hv_sv, ow, kWave);
              const uint32_t e = g - (o_incl - o_n);
              ok[k] = g < total ? (hmv ? ((int32_t)e < o_nv ? 2 : 1) : 1) : 0;  // 2: an MV value to look up
              pk[k] = o_key >> ksh;
              w0[k] = ((o_key & kmask) << fsh) | (e == 0 ? first_bit : 0u);
              vi[k] = (int64_t)o_v0 + e;
              von[k] = ok[k] == 2 && !(dbg & 4);
              alt[k] = ok[k] == 2 ? e : (hmv ? 0u : o_hv);  // (e: measurement only, PA_DEBUG_EMIT bit 2)
            }
            decode_global_batch<kHB>(hwords, vi, von, hnb, id);
#pragma unroll
            for (int k = 0; k < kHB; ++k)
              if (!von[k]) id[k] = alt[k];
            uint32_t hv[kHB];
#pragma unroll
            for (int k = 0; k < kHB; ++k) hv[k] = ok[k] == 2 && !(dbg & 2) ? gp(hlut)[id[k]] : id[k];  // (register << 8) | rank
            bool act[kHB];
            uint32_t pp[kHB], r[kHB][1];
#pragma unroll
            for (int k = 0; k < kHB; ++k) {
              act[k] = ok[k] != 0;
              pp[k] = (uint32_t)pv + pk[k];
              r[k][0] = w0[k] | ((hv[k] >> 8) << 6) | ((hv[k] & 0xffu) << 1);
            }
            bin_put_batch<kHB, 1, true>(B, act, pp, (uint32_t)pv, bins, BS, 1u, r, gp(ps.recs_h), lane, dbg, BST);
          }
        }
      }
    }
  }
}

// numGroupsLimit (walk form): the docs of match words m whose table-wide group key is admitted in this segment
// (seg->admit, written by limit_walk_kernel). Eight steps per batch: every dictId decode, then every remap gather, then
// every bitmap gather (their latencies overlap).
template <int LM, int STEPS>
__device__ __forceinline__ uint32_t admitted_docs(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                                  const uint32_t* img, int64_t doc_base, uint32_t m, int lane) {
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
  const uint32_t* adm = seg->admit;
  const int ngb = q->num_gb;
  constexpr int kB = 8;
#pragma unroll 1
  for (int h = 0; h < STEPS; h += kB) {
    if (__ballot(((m >> h) & 0xffu) != 0) == 0) continue;
    uint32_t key[kB];
#pragma unroll
    for (int i = 0; i < kB; ++i) key[i] = 0u;
    for (int j = 0; j < ngb; ++j) {
      const DevCol& c = seg->cols[q->gb_slot[j]];
      const int32_t* rm = seg->remap[j];
      const uint32_t st = (uint32_t)q->gb_stride[j];
      uint32_t id[kB];
#pragma unroll
      for (int i = 0; i < kB; ++i) {
        id[i] = 0u;
        if ((m >> (h + i)) & 1u) id[i] = decode_dict_id<false>(c, img, local(h + i), doc_base + local(h + i));
      }
      if (rm != nullptr) {
#pragma unroll
        for (int i = 0; i < kB; ++i)
          if ((m >> (h + i)) & 1u) id[i] = (uint32_t)gp(rm)[id[i]];
      }
#pragma unroll
      for (int i = 0; i < kB; ++i) key[i] += id[i] * st;  // direct key space of at most kWalkMaxKeys keys
    }
    uint32_t w[kB];
#pragma unroll
    for (int i = 0; i < kB; ++i) w[i] = ((m >> (h + i)) & 1u) ? gp(adm)[key[i] >> 5] : 0u;
#pragma unroll
    for (int i = 0; i < kB; ++i)
      if (!((w[i] >> (key[i] & 31u)) & 1u)) m &= ~(1u << (h + i));
  }
  return m;
}

// ---------------------------------------------------------------- aggregation-only queries (STRAT_LANE)
// Every lane keeps its own running SUM / MIN / MAX of aggregation a in (r0[a], r1[a]) for the whole kernel (COUNT is the
// filter's own doc count): SUM over int32 values r0 += v; over 64-bit values the exact split pair r0 += low 32 bits
// (unsigned), r1 += v >> 32 (a 96-bit total, like PA_ACC_SUM_I64X2); over FLOAT/DOUBLE r0 holds the bits of a double
// sum; MIN / MAX r0 = running min / max (doubles in the order-preserving encoding). The wave reduces them once, at the
// end of the kernel (lane_acc_flush). Reference: AggregationOperator -> SumAggregationFunction.aggregate (a running sum
// over the block's values), Min/MaxAggregationFunction.aggregate.
// MIN / MAX over a sorted dictionary run on dictIds (rid[a]: the lane's min / max dictId within the current segment),
// folded into r0 as a value at the end of every segment run (lane_acc_segment_end).
struct LaneAcc {
  // Per-thread slots in LDS (the workgroup's lane-accumulator area at the front of the dynamic LDS: kLaneAccBytes per
  // thread and aggregation), so no accumulator occupies a VGPR across the tile loop: aggregation a of thread t keeps
  // (r0, r1) at pair + 16 * (a * WGS + t) and its dictId at id + 4 * (a * WGS + t) (consecutive threads 16 / 4 bytes
  // apart: conflict-free ds_read_b128 / ds_read_b32).
  uint32_t pair;   // LDS byte address of aggregation 0's (r0, r1) slot of this thread
  uint32_t id;     // LDS byte address of aggregation 0's dictId slot of this thread
  uint32_t astr;   // bytes between aggregations' pair slots (16 * WGS); dictId slots: astr / 4
  uint32_t idm;    // bit a: aggregation a's dictId was updated in the current segment run
  // fused execution statistics: this wave's slice of the E-doc list, the entries listed so far, and the LDS byte
  // address of the wave's first leap_lds_cap entries (a global store in the tile loop would make the next tile's
  // counted DMA wait longer: vmcnt counts stores too)
  uint32_t leap_slice, leap_n, leap_lds;
};
typedef __attribute__((address_space(3))) int64_t lds_i64_t;
__device__ __forceinline__ void la_get(const LaneAcc& la, int a, int64_t& r0, int64_t& r1) {
  const lds_i64_t* p = (const lds_i64_t*)(uintptr_t)(la.pair + (uint32_t)a * la.astr);
  r0 = p[0];
  r1 = p[1];
}
__device__ __forceinline__ void la_set(const LaneAcc& la, int a, int64_t r0, int64_t r1) {
  lds_i64_t* p = (lds_i64_t*)(uintptr_t)(la.pair + (uint32_t)a * la.astr);
  p[0] = r0;
  p[1] = r1;
}
__device__ __forceinline__ uint32_t la_rid(const LaneAcc& la, int a) {
  return *(const lds_u32_t*)(uintptr_t)(la.id + (uint32_t)a * (la.astr >> 2));
}
__device__ __forceinline__ void la_set_rid(const LaneAcc& la, int a, uint32_t v) {
  *(lds_u32_t*)(uintptr_t)(la.id + (uint32_t)a * (la.astr >> 2)) = v;
}

__device__ __forceinline__ uint32_t rid_init(int t) { return t == PA_AGG_MIN ? 0xffffffffu : 0u; }

__device__ __forceinline__ void lane_acc_init(const DevQuery* __restrict__ q, LaneAcc& la, const void* lds_area,
                                              int wgs) {
  la.astr = 16u * (uint32_t)wgs;
  la.pair = lds_addr(lds_area) + 16u * threadIdx.x;
  la.id = lds_addr(lds_area) + (uint32_t)q->num_aggs * la.astr + 4u * threadIdx.x;
  la.idm = 0;
  for (int a = 0; a < q->num_aggs && a < kLaneAggs; ++a) {
    const int t = q->aggs[a].type;
    la_set(la, a, t == PA_AGG_MIN ? INT64_MAX : (t == PA_AGG_MAX ? INT64_MIN : 0), 0);
    la_set_rid(la, a, rid_init(t));
  }
}

// Lane-major fast path modes (lane_agg_lm)
enum LaneMode : int { LM_SUM_INT = 0, LM_SUM_LONG = 1, LM_SUM_DOUBLE = 2, LM_MIN_ID = 3, LM_MAX_ID = 4 };

// One aggregation over the 32 docs of this lane in a lane-major tile (docs 32*lane + i, match bit i of m) from a staged
// dictionary column of NB-bit ids: the lane's NB stream words are read once and every id is a constant-shift extract.
// SUM: the value is a buffer load of dict[id] with a buffer resource bounded by the dictionary, and a doc that does not
// match asks for index 0xffffffff (its bit of ~m spread by a signed bitfield extract, ORed into the id): out of range,
// so the load returns 0 — no per-doc branch or select. MIN_ID / MAX_ID track the smallest / largest matching dictId
// (0xffffffff is neutral under unsigned min; a non-matching id is ANDed to 0 for max).
template <int NB>
__device__ __forceinline__ void lane_agg_lm(uint32_t region_lds, int lane, uint32_t m, int mode,
                                            __amdgpu_buffer_rsrc_t dict, int64_t& r0, int64_t& r1, uint32_t& rid) {
  const lds_u32_t* p = (const lds_u32_t*)(uintptr_t)(region_lds + (uint32_t)lane * (uint32_t)(NB * 4));
  constexpr int H = NB > 16 ? 2 : 1;  // halves of 16 docs for wide columns (live stream words stay ~NB/2 + 1)
  constexpr int DPH = 32 / H;
  const uint32_t nm = ~m;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    constexpr int WMAX = (DPH * NB + 31) / 32 + 1;
    const int wlo = (h * DPH * NB) >> 5;
    uint32_t w[WMAX];
#pragma unroll
    for (int j = 0; j < WMAX; ++j) w[j] = (wlo + j < NB) ? p[wlo + j] : 0u;
    auto id_of = [&](int i) -> uint32_t {
      const int s = i * NB, j = (s >> 5) - wlo, o = s & 31;
      if (o + NB <= 32) return __builtin_amdgcn_ubfe(w[j], (uint32_t)(32 - o - NB), (uint32_t)NB);
      return __builtin_amdgcn_alignbit(w[j], w[(j + 1 < WMAX) ? j + 1 : j], 32 - o) >> (32 - NB);
    };
    if (mode <= LM_SUM_DOUBLE) {
      uint64_t v[DPH];
#pragma unroll
      for (int k = 0; k < DPH; ++k) {
        const int i = h * DPH + k;
        const uint32_t off = (id_of(i) << 3) | (uint32_t)__builtin_amdgcn_sbfe((int)nm, (uint32_t)i, 1u);
        v[k] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(dict, off, 0, 0));
      }
      if (mode == LM_SUM_INT) {
#pragma unroll
        for (int k = 0; k < DPH; ++k) r0 += (int64_t)v[k];
      } else if (mode == LM_SUM_LONG) {
#pragma unroll
        for (int k = 0; k < DPH; ++k) {
          r0 += (int64_t)(uint32_t)v[k];
          r1 += (int64_t)v[k] >> 32;
        }
      } else {
        double d = __builtin_bit_cast(double, r0);
#pragma unroll
        for (int k = 0; k < DPH; ++k) d += __builtin_bit_cast(double, v[k]);
        r0 = __builtin_bit_cast(int64_t, d);
      }
    } else if (mode == LM_MIN_ID) {
#pragma unroll
      for (int k = 0; k < DPH; ++k) {
        const int i = h * DPH + k;
        rid = min(rid, id_of(i) | (uint32_t)__builtin_amdgcn_sbfe((int)nm, (uint32_t)i, 1u));
      }
    } else {
#pragma unroll
      for (int k = 0; k < DPH; ++k) {
        const int i = h * DPH + k;
        rid = max(rid, id_of(i) & (uint32_t)__builtin_amdgcn_sbfe((int)m, (uint32_t)i, 1u));
      }
    }
  }
}

__device__ __noinline__ void lane_agg_lm_any(int nb, uint32_t region_lds, int lane, uint32_t m, int mode,
                                                __amdgpu_buffer_rsrc_t dict, int64_t& r0, int64_t& r1, uint32_t& rid) {
  switch (nb) {
#define PA_LA_CASE(N) \
  case N: lane_agg_lm<N>(region_lds, lane, m, mode, dict, r0, r1, rid); break;
    PA_LA_CASE(1) PA_LA_CASE(2) PA_LA_CASE(3) PA_LA_CASE(4) PA_LA_CASE(5) PA_LA_CASE(6) PA_LA_CASE(7) PA_LA_CASE(8)
    PA_LA_CASE(9) PA_LA_CASE(10) PA_LA_CASE(11) PA_LA_CASE(12) PA_LA_CASE(13) PA_LA_CASE(14) PA_LA_CASE(15)
    PA_LA_CASE(16) PA_LA_CASE(17) PA_LA_CASE(18) PA_LA_CASE(19) PA_LA_CASE(20) PA_LA_CASE(21) PA_LA_CASE(22)
    PA_LA_CASE(23) PA_LA_CASE(24) PA_LA_CASE(25) PA_LA_CASE(26) PA_LA_CASE(27) PA_LA_CASE(28) PA_LA_CASE(29)
    PA_LA_CASE(30) PA_LA_CASE(31)
#undef PA_LA_CASE
    default: break;
  }
}

// End of a wave's run over one segment: MIN / MAX dictIds of the segment -> values, folded into r0 (only when the
// lane kept some doc of the segment: a MAX dictId of 0 is otherwise meaningless).
__device__ __forceinline__ void lane_acc_segment_end(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                                     LaneAcc& la, bool any) {
#pragma unroll
  for (int a = 0; a < kLaneAggs; ++a) {
    if (a >= q->num_aggs) break;
    const int t = q->aggs[a].type;
    if (t != PA_AGG_MIN && t != PA_AGG_MAX) continue;
    const uint32_t id = la_rid(la, a);
    la_set_rid(la, a, rid_init(t));
    if (!((la.idm >> a) & 1u) || !any || (t == PA_AGG_MIN && id == 0xffffffffu)) continue;
    const DevCol& c = seg->cols[q->aggs[a].slot];
    const int64_t e = q->aggs[a].src == SRC_DOUBLE ? f64_order_encode(gp(c.dict_f64)[id]) : gp(c.dict_i64)[id];
    int64_t r0, r1;
    la_get(la, a, r0, r1);
    la_set(la, a, t == PA_AGG_MIN ? (e < r0 ? e : r0) : (e > r0 ? e : r0), r1);
  }
  la.idm = 0;
}

// One value (int64, or double bits for SRC_DOUBLE) into a lane accumulator pair: SUM over int32-range values r0 += v;
// 64-bit integer SUM as the exact split pair (r0 += low 32 bits unsigned, r1 += high 32 bits signed); double SUM in
// r0's bits; MIN / MAX on the order-preserving encoding.
__device__ __forceinline__ void lane_fold(int type, int src, uint64_t v, int64_t& r0, int64_t& r1) {
  if (type == PA_AGG_SUM) {
    if (src == SRC_INT) {
      r0 += (int64_t)v;
    } else if (src == SRC_LONG) {
      r0 += (int64_t)(uint32_t)v;
      r1 += (int64_t)v >> 32;
    } else {
      r0 = __builtin_bit_cast(int64_t, __builtin_bit_cast(double, r0) + __builtin_bit_cast(double, v));
    }
  } else {
    const int64_t e = src == SRC_DOUBLE ? f64_order_encode(__builtin_bit_cast(double, v)) : (int64_t)v;
    r0 = type == PA_AGG_MIN ? (e < r0 ? e : r0) : (e > r0 ? e : r0);
  }
}

// A raw value as the 64-bit pattern lane_fold takes: INT sign-extended, FLOAT widened to double bits, LONG / DOUBLE as is.
__device__ __forceinline__ uint64_t raw_bits(int vtype, uint64_t x) {
  switch (vtype) {
    case PA_INT: return (uint64_t)(int64_t)(int32_t)(uint32_t)x;
    case PA_FLOAT: return __builtin_bit_cast(uint64_t, (double)__builtin_bit_cast(float, (uint32_t)x));
    default: return x;
  }
}

// Sparse lane-major tile (few matching docs): each lane walks its own set bits of m (doc 32*lane + i), four per batch so
// their loads overlap; the wave loops max-popcount times instead of over all 32 docs. `load(i)` issues the value load of
// doc i (nothing is consumed before all four are issued).
template <class LOAD>
__device__ __forceinline__ void lane_sparse(uint32_t m, int type, int src, LOAD load, int64_t& r0, int64_t& r1) {
  while (__ballot(m != 0) != 0) {
    bool on[4];
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      on[k] = m != 0;
      const int i = on[k] ? __builtin_ctz(m) : 0;
      m &= m - 1u;
      v[k] = on[k] ? load(i) : 0ull;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (on[k]) lane_fold(type, src, v[k], r0, r1);
  }
}

// lane_sparse for a dictId histogram: every matching doc adds one to hist[dictId] (dec(i) = dictId of doc i); the
// decodes of a batch of four are issued before their (non-returning) LDS adds.
template <class DEC>
__device__ __forceinline__ void lane_sparse_hist(uint32_t m, DEC dec, lds_u32_t* hist) {
  while (__ballot(m != 0) != 0) {
    bool on[4];
    uint32_t id[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      on[k] = m != 0;
      const int i = on[k] ? __builtin_ctz(m) : 0;
      m &= m - 1u;
      id[k] = on[k] ? dec(i) : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (on[k]) __hip_atomic_fetch_add(hist + id[k], 1u, WG_RLX);
  }
}

// lane_sparse for MIN / MAX of a sorted dictionary: the smallest / largest matching dictId (dec(i) = dictId of doc i).
template <class DEC>
__device__ __forceinline__ void lane_sparse_ids(uint32_t m, bool is_min, DEC dec, uint32_t& rid) {
  while (__ballot(m != 0) != 0) {
    bool on[4];
    uint32_t id[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      on[k] = m != 0;
      const int i = on[k] ? __builtin_ctz(m) : 0;
      m &= m - 1u;
      id[k] = on[k] ? dec(i) : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (on[k]) rid = is_min ? min(rid, id[k]) : max(rid, id[k]);
  }
}

// Dense lane-major tile of a raw column of VB-byte values: the whole tile's values as coalesced 16-byte loads
// (instruction k, lane l: docs VPL*(64k + l) .. + VPL-1 of the tile, VPL = 16 / VB), every value's match bit read from
// the lane owning its doc in the lane-major layout (doc d: lane d >> 5, bit d & 31) by one ds_bpermute per
// instruction. Non-matching values are skipped by a select (no per-doc branch). Raw columns are padded to whole wave
// tiles, so the last tile's loads stay in bounds. 32 VGPRs of loads per batch, all issued before use.
template <int VB>
__device__ __forceinline__ void lane_raw_dense(const char* tile, uint32_t m, int lane, int vtype, int type, int src,
                                               int64_t& r0, int64_t& r1) {
  constexpr int VPL = 16 / VB;        // values per lane per instruction
  constexpr int NI = 2048 * VB / 1024;  // instructions per tile
  constexpr int KB = VB == 8 ? 4 : 8;
  const AS1 u32x4* p = (const AS1 u32x4*)tile + lane;
#pragma unroll
  for (int k0 = 0; k0 < NI; k0 += KB) {
    u32x4 w[KB];
    uint32_t mb[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      w[k] = p[(k0 + k) * kWave];
      // owner of doc VPL*(64k + l): lane 2*VPL*k + (VPL*l >> 5); its bits VPL*l & 31 .. + VPL-1
      const int owner = 2 * VPL * (k0 + k) + ((VPL * lane) >> 5);
      mb[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(owner << 2, (int)m) >> ((VPL * lane) & 31);
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        const uint64_t x = VB == 8 ? ((uint64_t)w[k][2 * j + 1] << 32) | w[k][2 * j] : (uint64_t)w[k][j];
        const bool on = (mb[k] >> j) & 1u;
        if (type == PA_AGG_SUM) {
          lane_fold(type, src, on ? raw_bits(vtype, x) : 0ull, r0, r1);  // (+0 / +0.0 for a doc that does not match)
        } else if (on) {
          lane_fold(type, src, raw_bits(vtype, x), r0, r1);
        }
      }
    }
  }
}

// The matching docs (match words m) of one tile into the lane accumulators: per aggregation, 8 steps per batch — every
// value load of the batch is issued before any is used (staged dictIds from the tile image, lazy ones and raw values from
// HBM, then the dictionary gathers).
template <int LM, int STEPS, int STRAT>
__device__ __forceinline__ void lane_acc_tile(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                              const uint32_t* img, int64_t doc_base, uint32_t m, int lane,
                                              LaneAcc& la, unsigned char* lds) {
  typedef const __attribute__((address_space(4))) DevSeg CSeg;
  CSeg* cs = (CSeg*)(uintptr_t)seg;
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
  constexpr int kB = 8;
  const int na = q->num_aggs;
  // matching docs of the tile: the wave's total and the largest count of one lane (sparse vs dense paths)
  uint32_t tot = 0, mx = 0;
  if constexpr (LM) {
    tot = mx = (uint32_t)__builtin_popcount(m);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      tot += (uint32_t)__shfl_xor((int)tot, o, kWave);
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, kWave));
    }
    tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)tot);
    mx = (uint32_t)__builtin_amdgcn_readfirstlane((int)mx);
  }
  // one copy of the per-aggregation code (a loop that is not unrolled; the accumulators live in LDS): the unrolled form
  // replicated every path per aggregation and spilled
#pragma unroll 1
  for (int a = 0; a < na && a < kLaneAggs; ++a) {
    const int type = q->aggs[a].type;
    if (type == PA_AGG_COUNT) continue;
    const int slot = q->aggs[a].slot, src = q->aggs[a].src;
    const int kind = cs->cols[slot].kind, vtype = cs->cols[slot].vtype;
    const int loff = cs->cols[slot].lds_off, nb = cs->cols[slot].nbits;
    const uint32_t* words = cs->cols[slot].words;
    const uint64_t* dict = src == SRC_DOUBLE ? (const uint64_t*)cs->cols[slot].dict_f64
                                             : (const uint64_t*)cs->cols[slot].dict_i64;
    const void* raw = cs->cols[slot].raw;
    int64_t r0, r1;
    la_get(la, a, r0, r1);
    uint32_t rid = la_rid(la, a);
    do {  // (break: this aggregation is done)
    if (STRAT == STRAT_LANE_DICT) {
    } else if (LM && kind == COL_SV_RAW) {
      // raw column: per-doc loads of the few matching docs, or the whole tile as coalesced 16-byte loads (a sparse
      // tile's loads touch at most `tot` lines; the dense read is 2048 * VB bytes = 16 * VB lines of 128 B)
      const int vb = (vtype == PA_INT || vtype == PA_FLOAT) ? 4 : 8;
      if (tot <= (uint32_t)(6 * vb)) {
        const int64_t d0 = doc_base + 32 * lane;
        if (vb == 4) {
          const AS1 uint32_t* rp = gp((const uint32_t*)raw) + d0;
          lane_sparse(m, type, src, [&](int i) { return raw_bits(vtype, rp[i]); }, r0, r1);
        } else {
          const AS1 uint64_t* rp = gp((const uint64_t*)raw) + d0;
          lane_sparse(m, type, src, [&](int i) { return rp[i]; }, r0, r1);
        }
      } else if (vb == 4) {
        lane_raw_dense<4>((const char*)raw + doc_base * 4, m, lane, vtype, type, src, r0, r1);
      } else {
        lane_raw_dense<8>((const char*)raw + doc_base * 8, m, lane, vtype, type, src, r0, r1);
      }
      break;
    }
    if (STRAT == STRAT_LANE_RAW) break;  // (the raw kernel's columns are all raw: handled above)
    if constexpr (STRAT == STRAT_LANE_DICT) {
      if (type == PA_AGG_SUM && q->aggs[a].hist_card > 0) {
        // shared dictionary: count the dictIds in the workgroup's LDS histogram (the values come in at the end)
        lds_u32_t* hist = lds_ptr(lds + q->aggs[a].hist_off);
        lane_sparse_hist(m, [&](int i) -> uint32_t {
          return loff >= 0 ? decode_lds(img + loff, 32 * lane + i, nb) : decode_global(words, doc_base + 32 * lane + i, nb);
        }, hist);
        break;
      }
      // dictionary kernel: every tile walks the lanes' set bits (a lane's matching docs one after another, the wave
      // max-popcount times): decode from the staged image (or HBM when lazy), then MIN / MAX of a sorted dictionary on
      // the dictIds, anything else on the gathered values. One path (no per-width unpack calls): nothing spills.
      auto dec = [&](int i) -> uint32_t {
        return loff >= 0 ? decode_lds(img + loff, 32 * lane + i, nb) : decode_global(words, doc_base + 32 * lane + i, nb);
      };
      if (type != PA_AGG_SUM && (cs->cols[slot].flags & COLF_DICT_SORTED)) {
        lane_sparse_ids(m, type == PA_AGG_MIN, dec, rid);
        la.idm |= 1u << a;
      } else {
        lane_sparse(m, type, src, [&](int i) { return gp(dict)[dec(i)]; }, r0, r1);
      }
      break;
    }
    if (LM && kind == COL_SV_DICT && mx <= 12 &&
        !(type != PA_AGG_SUM && (cs->cols[slot].flags & COLF_DICT_SORTED) && loff >= 0)) {
      // dictionary column, few matching docs per lane: decode only those (staged image or HBM) and gather their values
      if (loff >= 0) {
        const uint32_t* region = img + loff;
        lane_sparse(m, type, src, [&](int i) { return gp(dict)[decode_lds(region, 32 * lane + i, nb)]; }, r0, r1);
      } else {
        const int64_t d0 = doc_base + 32 * lane;
        lane_sparse(m, type, src, [&](int i) { return gp(dict)[decode_global(words, d0 + i, nb)]; }, r0, r1);
      }
      break;
    }
    if (LM && kind == COL_SV_DICT && loff >= 0 &&
        (type == PA_AGG_SUM || (cs->cols[slot].flags & COLF_DICT_SORTED))) {
      const int mode = type == PA_AGG_SUM ? (src == SRC_INT ? LM_SUM_INT : (src == SRC_LONG ? LM_SUM_LONG : LM_SUM_DOUBLE))
                                          : (type == PA_AGG_MIN ? LM_MIN_ID : LM_MAX_ID);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)dict, (short)0, cs->cols[slot].card * 8, 0x00020000);
      lane_agg_lm_any(nb, lds_addr(img + loff), lane, m, mode, rs, r0, r1, rid);
      if (mode >= LM_MIN_ID) la.idm |= 1u << a;
      break;
    }
#pragma unroll 1
    for (int h = 0; h < STEPS; h += kB) {
      if (__ballot(((m >> h) & 0xffu) != 0) == 0) continue;
      uint64_t v[kB];
      if (kind == COL_SV_DICT) {
        uint32_t id[kB];
        decode_batch<kB, LM>(loff, nb, words, img, doc_base, h, m, lane, id);
#pragma unroll
        for (int i = 0; i < kB; ++i) v[i] = ((m >> (h + i)) & 1u) ? gp(dict)[id[i]] : 0ull;
      } else if (vtype == PA_INT) {
#pragma unroll
        for (int i = 0; i < kB; ++i)
          v[i] = ((m >> (h + i)) & 1u) ? (uint64_t)(int64_t)gp((const int32_t*)raw)[doc_base + local(h + i)] : 0ull;
      } else if (vtype == PA_FLOAT) {
#pragma unroll
        for (int i = 0; i < kB; ++i)
          v[i] = ((m >> (h + i)) & 1u) ? __builtin_bit_cast(uint64_t, (double)gp((const float*)raw)[doc_base + local(h + i)])
                                      : 0ull;
      } else {  // LONG, DOUBLE bits
#pragma unroll
        for (int i = 0; i < kB; ++i)
          v[i] = ((m >> (h + i)) & 1u) ? gp((const uint64_t*)raw)[doc_base + local(h + i)] : 0ull;
      }
      if (type == PA_AGG_SUM) {
        if (src == SRC_INT) {
#pragma unroll
          for (int i = 0; i < kB; ++i) r0 += (int64_t)v[i];
        } else if (src == SRC_LONG) {
#pragma unroll
          for (int i = 0; i < kB; ++i) {
            r0 += (int64_t)(uint32_t)v[i];
            r1 += (int64_t)v[i] >> 32;
          }
        } else {
          double d = __builtin_bit_cast(double, r0);
#pragma unroll
          for (int i = 0; i < kB; ++i) d += __builtin_bit_cast(double, v[i]);  // (0.0 for the docs that do not match)
          r0 = __builtin_bit_cast(int64_t, d);
        }
      } else {
#pragma unroll
        for (int i = 0; i < kB; ++i) {
          if (!((m >> (h + i)) & 1u)) continue;
          const int64_t e = src == SRC_DOUBLE ? f64_order_encode(__builtin_bit_cast(double, v[i])) : (int64_t)v[i];
          r0 = type == PA_AGG_MIN ? (e < r0 ? e : r0) : (e > r0 ? e : r0);
        }
      }
    }
    } while (false);
    la_set(la, a, r0, r1);
    la_set_rid(la, a, rid);
  }
}

// End of the kernel: one wave reduction per accumulator and one device-scope atomic per wave.
__device__ __forceinline__ void lane_acc_flush(const DevQuery* __restrict__ q, const LaneAcc& la, int lane) {
#pragma unroll
  for (int a = 0; a < kLaneAggs; ++a) {
    if (a >= q->num_aggs) break;
    const DevAgg& A = q->aggs[a];
    if (A.type == PA_AGG_COUNT) continue;
    int64_t r0, r1;
    la_get(la, a, r0, r1);
    if (A.type == PA_AGG_SUM) {
      if (A.src == SRC_DOUBLE) {
        const double s = wave_sum_f64(__builtin_bit_cast(double, r0));
        if (lane == 0) __hip_atomic_fetch_add(gp(A.acc_f64), s, RLX);
      } else if (A.src == SRC_LONG) {
        const int64_t lo = wave_sum_i64(r0), hi = wave_sum_i64(r1);
        if (lane == 0) {
          __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64), (unsigned long long)lo, RLX);
          __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + 1, (unsigned long long)hi, RLX);
        }
      } else {
        const int64_t s = wave_sum_i64(r0);
        if (lane == 0) __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64), (unsigned long long)s, RLX);
      }
    } else if (A.type == PA_AGG_MIN) {
      const int64_t r = wave_min_i64(r0);
      if (lane == 0 && r != INT64_MAX) __hip_atomic_fetch_min(gp((long long*)A.acc_i64), (long long)r, RLX);
    } else {
      const int64_t r = wave_max_i64(r0);
      if (lane == 0 && r != INT64_MIN) __hip_atomic_fetch_max(gp((long long*)A.acc_i64), (long long)r, RLX);
    }
  }
}

// The rare part of a tile (some doc survived the eager clauses): lazy clauses per surviving doc, then aggregation.
// Returns the docs that matched.
// LM: doc of bit i of lane l = 32l + i (lane-major tile), else 64i + l.
template <int STRAT, int STEPS, int LM>
__device__ __forceinline__ uint32_t tile_survivors(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg_in,
                                                const uint32_t* img, int64_t doc_base, uint32_t m, int lane,
                                                unsigned char* lds, const PartScratch& ps, LaneAcc& la) {
  const DevSeg* __restrict__ seg = uniform_ptr(seg_in);
  doc_base = ((int64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)doc_base >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)doc_base);
  const Acc<STRAT> acc{q, lds, &ps};
  auto local = [&](int i) { return LM ? 32 * lane + i : i * kWave + lane; };
  const int nleaves = q->num_leaves;
  const int neager = q->num_eager;
  if (neager < nleaves) {
    const uint32_t eager = m;
    // lazy clauses: only the docs the eager clauses kept, one step at a time, straight from HBM
    for (int i = 0; i < STEPS; ++i) {
      const uint32_t bit = 1u << i;
      if (__ballot((m & bit) != 0) == 0) continue;
      const int64_t doc = doc_base + local(i);
      bool ok = (m & bit) != 0;
      bool any = false;
      for (int li = neager; li < nleaves; ++li) {
        const DevLeaf& L = seg->leaves[li];
        if (ok && !any) any = leaf_match_doc(L, doc);
        if (L.clause_end) {
          ok = ok && any;
          any = false;
        }
      }
      if (!ok) m &= ~bit;
    }
    if constexpr (!is_pcount(STRAT) && !is_pemit(STRAT))
      if (q->leap_mode) leap_tile<LM>(q, seg, doc_base, eager, m, lane, la.leap_slice, la.leap_n, la.leap_lds);
    if (__ballot(m != 0) == 0) return 0;
  }
  const uint32_t scanned = m;  // numDocsScanned counts every doc the filter kept, admitted or not
  // (an MV group-by admits (doc, value) keys one by one: accumulate_doc_mv, mv_key_records)
  if (seg->admit != nullptr && q->gb_mv < 0) {
    m = admitted_docs<LM, STEPS>(q, seg, img, doc_base, m, lane);
    if (__ballot(m != 0) == 0) return (uint32_t)__builtin_popcount(scanned);
  }
  if constexpr (is_lane(STRAT)) {
    if constexpr (STRAT != STRAT_LANE_CNT) lane_acc_tile<LM, STEPS, STRAT>(q, seg, img, doc_base, m, lane, la, lds);
  } else if constexpr (is_pcount(STRAT) || is_pemit(STRAT)) {
    part_tile<STRAT, STEPS, LM>(q, seg, img, doc_base, m, lane, lds, ps);

  } else if (q->has_mv) {
    for (int i = 0; i < STEPS; ++i)
      if ((m >> i) & 1u) accumulate_doc_mv<STRAT>(q, seg, img, local(i), doc_base + local(i), acc);
  } else if constexpr (STRAT == STRAT_LDS && LM) {
    // matches of the wave's tile: a dense tile whose aggregations all read one raw column takes that column's tile as
    // coalesced loads; else per-lane batches, 8 docs deep when most lanes have that many (more gathers in flight)
    uint32_t tot = (uint32_t)__builtin_popcount(m);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) tot += (uint32_t)__shfl_xor((int)tot, o, kWave);
    const int rs = q->hashed ? -1 : q->lds_raw_slot;
    if (tot > 256u && rs >= 0 && seg->cols[rs].kind == COL_SV_RAW) {
      const int vt = seg->cols[rs].vtype;
      if (vt == PA_INT || vt == PA_FLOAT) accumulate_lds_raw_dense<4>(q, seg, img, doc_base, m, lane, lds);
      else accumulate_lds_raw_dense<8>(q, seg, img, doc_base, m, lane, lds);
    } else if (tot > 512u) {
      accumulate_lds_lm<8>(q, seg, img, doc_base, m, lane, lds);
    } else {
      accumulate_lds_lm<4>(q, seg, img, doc_base, m, lane, lds);
    }
  } else if (q->has_mv) {
    for (int i = 0; i < STEPS; ++i)
      if ((m >> i) & 1u) accumulate_doc_mv<STRAT>(q, seg, img, local(i), doc_base + local(i), acc);
  } else {
    for (int i = 0; i < STEPS; ++i) {
      const uint64_t sm = __ballot((m >> i) & 1u);
      if (sm == 0) continue;
      accumulate_step<STRAT>(q, seg, img, local(i), doc_base + local(i), sm, lane, acc);
    }
  }
  __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));  // vmcnt(0): no compiler-visible load left pending
  return (uint32_t)__builtin_popcount(scanned);
}

template <int STRAT, int STEPS>
__device__ __forceinline__ void process_tile(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                             int64_t wt, const uint32_t* img, int lane, const Acc<STRAT>& acc,
                                             uint32_t& matched, LaneAcc& la) {
  const int64_t doc_base = wt * (STEPS * kWave);
  // docs of this tile owned by the lane: 64*i + lane < rem
  const int64_t rem = (int64_t)seg->num_docs - doc_base;
  // bit i <=> step i holds a doc of this segment (only the low STEPS bits: a negated leaf sets the others, and the
  // matched-doc count must not see them)
  constexpr uint32_t kFull = STEPS == 32 ? 0xffffffffu : ((1u << STEPS) - 1u);
  uint32_t valid;
  if (rem >= (STEPS * kWave)) {
    valid = kFull;
  } else {
    const int64_t n = rem > lane ? (rem - lane + kWave - 1) / kWave : 0;  // steps with a valid doc for this lane
    valid = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
  }
  uint32_t m = valid;
  uint32_t clause = 0;
  const int neager = q->num_eager;
  for (int li = 0; li < neager; ++li) {
    const DevLeaf& L = seg->leaves[li];
    clause |= leaf_bits<STEPS>(L, img, doc_base, lane);
    if (L.clause_end) {
      m &= clause;
      clause = 0;
      if (__ballot(m != 0) == 0) return;  // no doc of the tile can match any more
    }
  }
  if (__ballot(m != 0) == 0) return;
  matched += tile_survivors<STRAT, STEPS, 0>(q, seg, img, doc_base, m, lane, acc.lds, *acc.ps, la);
}


// ---------------------------------------------------------------- lane-major tile evaluation (scan_kernel<.., LM=1>)
//
// Lane l owns docs [32l, 32l+32) of the wave tile, i.e. the nb consecutive stream words [l*nb, (l+1)*nb) of every
// staged column: an eager leaf is nb ds_reads at immediate offsets (1x the staged bytes, against 2 dwords per doc in
// the step-major layout) plus a static unpack (nb is a template parameter: every shift is a constant).

__device__ __forceinline__ uint32_t rl(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }

// Match word of one DICT_RANGE / DICT_SET leaf: bit i <=> doc 32*lane + i of the tile matches (before negation).
template <int NB>
__device__ __forceinline__ uint32_t leaf_lm(int kind, uint32_t region_lds, int lane, uint32_t lo_t, uint32_t hi_t,
                                            const uint32_t* lut) {
  const lds_u32_t* p = (const lds_u32_t*)(uintptr_t)(region_lds + (uint32_t)lane * (uint32_t)(NB * 4));
  // Wide columns are unpacked in two halves of 16 docs, so at most ~NB/2 + 1 stream words are live at once (keeps
  // the kernel within 128 VGPRs: 4 waves per SIMD).
  constexpr int H = NB > 16 ? 2 : 1;
  constexpr int DPH = 32 / H;  // docs per half
  uint32_t nm = 0, bits = 0;
#pragma unroll
  for (int h = H - 1; h >= 0; --h) {
    constexpr int WMAX = (DPH * NB + 31) / 32 + 1;
    const int wlo = (h * DPH * NB) >> 5;  // first stream word of this half (compile-time after unrolling)
    uint32_t w[WMAX];
#pragma unroll
    for (int j = 0; j < WMAX; ++j) w[j] = (wlo + j < NB) ? p[wlo + j] : 0u;
    // MSB-aligned value of doc i: the NB bits starting at stream bit i*NB, in the top bits of t
    auto top = [&](int i) -> uint32_t {
      const int s = i * NB, j = (s >> 5) - wlo, o = s & 31;
      if (o + NB <= 32) return w[j] << o;
      return __builtin_amdgcn_alignbit(w[j], w[(j + 1 < WMAX) ? j + 1 : j], 32 - o);
    };
    if (kind == PA_LEAF_DICT_RANGE) {
      // lo <= v < lo + span  <=>  (t - lo') <= hi' (unsigned), lo' / hi' MSB-aligned by the host (see leaf_bits);
      // non-matches accumulate as nm = 2*nm + borrow: bit i of nm = doc i does not match
#pragma unroll
      for (int i = (h + 1) * DPH - 1; i >= h * DPH; --i) {
        const uint32_t t = top(i);
        uint32_t u;
        asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
            "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
            "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
            : [nm] "+v"(nm), [u] "=&v"(u)
            : [t] "v"(t), [lo] "s"(lo_t), [hi] "s"(hi_t)
            : "vcc");
      }
    } else {
      const AS1 uint32_t* lt = gp(lut);
#pragma unroll
      for (int i = h * DPH; i < (h + 1) * DPH; ++i) {
        const uint32_t id = top(i) >> (32 - NB);
        bits |= ((lt[id >> 5] >> (id & 31u)) & 1u) << i;
      }
    }
  }
  return kind == PA_LEAF_DICT_RANGE ? ~nm : bits;
}

__device__ __forceinline__ uint32_t leaf_lm_any(int nb, int kind, uint32_t region_lds, int lane, uint32_t lo_t,
                                                uint32_t hi_t, const uint32_t* lut) {
  switch (nb) {
#define PA_LM_CASE(N) \
  case N: return leaf_lm<N>(kind, region_lds, lane, lo_t, hi_t, lut);
    PA_LM_CASE(1) PA_LM_CASE(2) PA_LM_CASE(3) PA_LM_CASE(4) PA_LM_CASE(5) PA_LM_CASE(6) PA_LM_CASE(7) PA_LM_CASE(8)
    PA_LM_CASE(9) PA_LM_CASE(10) PA_LM_CASE(11) PA_LM_CASE(12) PA_LM_CASE(13) PA_LM_CASE(14) PA_LM_CASE(15)
    PA_LM_CASE(16) PA_LM_CASE(17) PA_LM_CASE(18) PA_LM_CASE(19) PA_LM_CASE(20) PA_LM_CASE(21) PA_LM_CASE(22)
    PA_LM_CASE(23) PA_LM_CASE(24) PA_LM_CASE(25) PA_LM_CASE(26) PA_LM_CASE(27) PA_LM_CASE(28) PA_LM_CASE(29)
    PA_LM_CASE(30) PA_LM_CASE(31) PA_LM_CASE(32)
#undef PA_LM_CASE
    default: return 0;
  }
}

// LDS-DMA of one wave tile of every staged column (plan table `ip`), padded to exactly D instructions.
__device__ __forceinline__ void stage_tile_lm(uint32_t ip, int64_t wt, uint32_t img_lds, int lane, const int D) {
  const int ns = (int)rl(ip, 0);
  int issued = 0;
  for (int c = 0; c < ns; ++c) {
    const uint64_t words = ((uint64_t)rl(ip, 9 + 4 * c) << 32) | rl(ip, 8 + 4 * c);
    const int nb = (int)rl(ip, 10 + 4 * c);
    const uint32_t dst = img_lds + 4u * rl(ip, 11 + 4 * c);
    const char* src = (const char*)words + wt * (int64_t)(256 * nb) + 16 * lane;  // 256*nb bytes per wave tile
    const int chunks = 16 * nb;                                                      // 16-byte chunks per wave tile
    for (int c0 = 0; c0 < chunks; c0 += 64) {
      if (c0 + lane < chunks) dma16(src + 16 * c0, dst + 16 * c0);
      ++issued;
    }
  }
  const void* dummy = (const void*)(((uint64_t)rl(ip, 5) << 32) | rl(ip, 4));
  for (; issued < D; ++issued) {
    if (lane == 0) dma16(dummy, img_lds);
  }
}

template <int STRAT>
__device__ __forceinline__ void process_tile_lm(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                                uint32_t pp, int64_t wt, const uint32_t* img, uint32_t img_lds,
                                                int lane, const Acc<STRAT>& acc, uint32_t& matched, LaneAcc& la) {
  const int64_t doc_base = wt * kWTileDocs;
  const int64_t rem = (int64_t)(int32_t)rl(pp, 2) - doc_base;
  uint32_t valid = 0xffffffffu;
  if (rem < kWTileDocs) {
    const int64_t n = rem - 32 * lane;  // docs of this lane's 32 that exist
    valid = n >= 32 ? 0xffffffffu : (n <= 0 ? 0u : ((1u << n) - 1u));
  }
  uint32_t m = valid;
  uint32_t clause = 0;
  const int neager = (int)rl(pp, 1);
  for (int l = 0; l < neager; ++l) {
    const int b = 24 + 8 * l;
    const int flags = (int)rl(pp, b + 5);
    const uint32_t* lut = (const uint32_t*)(((uint64_t)rl(pp, b + 7) << 32) | rl(pp, b + 6));
    uint32_t bits = leaf_lm_any((int)rl(pp, b + 1), (int)rl(pp, b), img_lds + 4u * rl(pp, b + 2), lane,
                                rl(pp, b + 3), rl(pp, b + 4), lut);
    if (flags & 1) bits = ~bits;
    clause |= bits;
    if (flags & 2) {
      m &= clause;
      clause = 0;
      if (__ballot(m != 0) == 0) return;
    }
  }
  if (__ballot(m != 0) == 0) return;
  matched += tile_survivors<STRAT, 32, 1>(q, seg, img, doc_base, m, lane, acc.lds, *acc.ps, la);
}

__device__ __forceinline__ int find_segment(const DevSeg* __restrict__ segs, int nseg, int64_t t) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].first_wtile <= t) lo = mid;
    else hi = mid - 1;
  }
  while (t >= segs[lo].first_wtile + segs[lo].num_wtiles) ++lo;
  return lo;
}

// s_waitcnt vmcnt(N) that also "produces" `token` (the ring slot's LDS offset): every LDS read of the slot is
// addressed through the token, so it cannot be scheduled above the wait. No "memory" clobber: a clobber would
// make the compiler re-load every query/segment descriptor field after each wait (dependent SMEM round trips per
// tile).
template <int N>
__device__ __forceinline__ void vm_wait_token(uint32_t& token) {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  token = (uint32_t)__builtin_amdgcn_readfirstlane((int)token);  // wave-uniform (see dma16)
  asm volatile("s_waitcnt vmcnt(%1)" : "+s"(token) : "n"(N));
}

// vmcnt(n) for a wave-uniform runtime n in [LO, HI]: a 6-deep binary tree of scalar branches down to the immediate.
template <int LO, int HI>
__device__ __forceinline__ void vm_wait_n(uint32_t& token, int n) {
  if constexpr (LO == HI) {
    vm_wait_token<LO>(token);
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) vm_wait_n<LO, MID>(token, n);
    else vm_wait_n<MID + 1, HI>(token, n);
  }
}

// Wait until the tile with `younger` tiles issued after it has landed (every tile is exactly D DMA instructions,
// so that is vmcnt(younger * D); above 63 — the counter's width — vmcnt(63) waits for more, never less); `token` =
// the tile's slot offset.
__device__ __forceinline__ void wait_tile(int younger, int D, uint32_t& token) {
  const int n = younger * D;
  vm_wait_n<0, 63>(token, n < 63 ? n : 63);
}

// Issue side of the lane-major steady state, hoisted per segment (see scan_kernel).
struct LmIssue {
  const char* base[kLmStaged];  // column stream (wave-uniform: the lane's 16-byte offset is added per DMA)
  int64_t stride[kLmStaged];    // bytes per wave tile
  uint32_t off[kLmStaged];      // LDS byte offset of the column region in a tile image
  int nfull[kLmStaged];         // full 64-lane DMA instructions per tile
  uint64_t tail[kLmStaged];     // lanes of the last, partial instruction (0 = none)
  int nst;
  const void* dummy;
};

// Wait for the tile in slot `slot_off`, then issue the next tile `ti` (ring slot `islot`): every instruction a full
// 64-lane DMA except a column's lane-masked tail, padded to exactly D instructions.
__device__ __forceinline__ void lm_wait_issue(const LmIssue& I, uint32_t& slot_off, int R, int D, int64_t younger,
                                              uint32_t dst0, int64_t it, uint32_t lane_off) {
  if (R == 2) vm_wait_token<0>(slot_off);  // the one tile in flight has landed
  else wait_tile((int)younger, D, slot_off);
  int issued = 0;
#pragma unroll
  for (int c = 0; c < kLmStaged; ++c) {
    if (c < I.nst) {
      const char* src = I.base[c] + it * I.stride[c] + lane_off;
      const uint32_t dst = dst0 + I.off[c];
      for (int k = 0; k < I.nfull[c]; ++k) dma16(src + 1024 * k, dst + 1024 * k);
      issued += I.nfull[c];
      if (I.tail[c]) {
        dma16_masked(src + 1024 * I.nfull[c], dst + 1024 * I.nfull[c], I.tail[c]);
        ++issued;
      }
    }
  }
  for (; issued < D; ++issued) dma16_masked(I.dummy, dst0, 1ull);
}

// Workgroups are dispatched to the 8 XCDs round-robin (block b runs on XCD b % 8). For queries that gather per matching
// doc (dense), the scan gives block b the logical index of its place in XCD-major order, so the workgroups of one XCD
// walk one contiguous eighth of the tiles: the segments (dictionaries, remaps) an XCD touches at a time are few, and
// their lines stay in that XCD's L2 (configs[2]: HBM fetch of the emit pass 8.8 GB -> 0.9 GB per launch).
__device__ __forceinline__ int64_t xcd_major_block(int64_t b, int64_t G) {
  constexpr int kXcds = 8;
  const int64_t x = b % kXcds, j = b / kXcds, per = G / kXcds, extra = G % kXcds;
  return x * per + (x < extra ? x : extra) + j;
}

// The V-only emit of 4-wave workgroups (one whole tile per batch in part_tile): compiled for 2 workgroups per CU.
__host__ __device__ constexpr bool emit_v_wide(int s) {
  return is_pemit(s) && !pemit_hh(s) && !pemit_big(s) && pemit_vf(s) != V_FMT_GEN;
}

// LM = 1: lane-major tiles (STEPS must be 32) driven by the per-segment plan tables `plans`; LM = 0: step-major.
template <int STRAT, int STEPS, int LM>
__global__ void __launch_bounds__(scan_waves(STRAT) * kWave, emit_v_wide(STRAT) ? 2 : (scan_waves(STRAT) == kWavesPerWG ? 4 : 1)) scan_kernel(const DevQuery* __restrict__ q,
                                                       const DevSeg* __restrict__ segs,
                                                       const LmSegPlan* __restrict__ plans, PartScratch ps) {
  static_assert(!LM || STEPS == 32, "lane-major tiles are 2048 docs");
  constexpr int WPW = scan_waves(STRAT);  // waves per workgroup
  constexpr int WGS = WPW * kWave;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  // wave-uniform by construction; readfirstlane makes the compiler keep the whole tile/segment cursor in SGPRs
  // (otherwise segment descriptors are read with vector loads whose vmcnt(0) waits drain the DMA ring)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned char* lds_acc = (unsigned char*)smem;
  const uint32_t acc_dwords = STRAT != STRAT_GLOBAL ? (q->lds_acc_bytes >> 2) : 0u;
  const int img_dw = q->image_dwords_max;
  uint32_t* ring = smem + acc_dwords + wave * q->ring * img_dw;
  Acc<STRAT> acc{q, lds_acc, &ps};

  if (STRAT == STRAT_LDS) {
    const int64_t K = q->num_keys;
    uint32_t* cnt = (uint32_t*)(lds_acc + q->lds_count_off);
    for (int64_t k = threadIdx.x; k < K; k += WGS) cnt[k] = 0;
    for (int a = 0; a < q->num_aggs; ++a) {
      const DevAgg& A = q->aggs[a];
      if (A.type == PA_AGG_COUNT) continue;
      if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
        uint32_t* r = (uint32_t*)(lds_acc + A.lds_off);
        for (int64_t k = threadIdx.x; k < (K << A.log2m); k += WGS) r[k] = 0;
      } else if (A.type == PA_AGG_DISTINCTCOUNT) {
        uint32_t* r = (uint32_t*)(lds_acc + A.lds_off);
        for (int64_t k = threadIdx.x; k < K * A.nvals / 4; k += WGS) r[k] = 0;
      } else {
        int64_t* r = (int64_t*)(lds_acc + A.lds_off);
        const int64_t init = A.type == PA_AGG_MIN ? INT64_MAX : (A.type == PA_AGG_MAX ? INT64_MIN : 0);  // SUM, COUNT_MV: 0
        const int64_t n = (A.type == PA_AGG_SUM && A.src == SRC_LONG) ? 2 * K : K;
        for (int64_t k = threadIdx.x; k < n; k += WGS) r[k] = init;  // SUM(double) 0.0 == all-zero bits
      }
    }
    __syncthreads();
  } else if (is_pcount(STRAT)) {
    uint32_t* hist = (uint32_t*)lds_acc;
    for (int p = threadIdx.x; p < q->num_parts; p += WGS) hist[p] = 0u;
    __syncthreads();
  } else if (is_pemit(STRAT)) {
    // every partition's bin empty; its range in the stream: the partition base + this workgroup's offset (part_scan),
    // holding exactly the records the count pass counted here
    const BinState B = bin_state(q, lds_acc);
    const int64_t lbi = q->xcd_major ? xcd_major_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int P = q->num_parts, pv = q->pv;
    for (int p = q->part_lo + threadIdx.x; p < q->part_hi; p += WGS) {
      B.cnt[p] = 0u;
      B.done[p] = 0u;
      B.front[p] = 0u;
      if (p >= pv) B.slk[p] = 0u;
      B.back[p] = gp(ps.hist)[lbi * P + p];
      B.start[p] = gp(ps.base)[p < pv ? p : p + 1] + gp(ps.off)[lbi * P + p];
    }
    __syncthreads();
  }

  uint32_t matched = 0;  // docs of this lane that passed the filter (numDocsScanned)
  LaneAcc la;
  la.leap_slice = (uint32_t)((q->xcd_major ? xcd_major_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x) * WPW + wave);
  la.leap_n = 0u;
  la.leap_lds = lds_addr(smem + acc_dwords + (uint32_t)WPW * (uint32_t)q->ring * (uint32_t)img_dw) +
                (uint32_t)wave * (uint32_t)q->leap_lds_cap * 8u;
  if constexpr (is_lane(STRAT) && STRAT != STRAT_LANE_CNT) lane_acc_init(q, la, smem, WGS);
  if constexpr (STRAT == STRAT_LANE_DICT) {  // the dictId histograms of SUMs over a shared dictionary
    for (int a = 0; a < q->num_aggs; ++a) {
      const int hc = q->aggs[a].hist_card;
      if (hc <= 0) continue;
      uint32_t* h = (uint32_t*)(lds_acc + q->aggs[a].hist_off);
      for (int i = threadIdx.x; i < hc; i += WGS) h[i] = 0u;
    }
    __syncthreads();
  }
  const int64_t T = q->total_wtiles;
  const int64_t W = (int64_t)gridDim.x * WPW;
  const int64_t lb = q->xcd_major ? xcd_major_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;  // logical block
  const int64_t gw = lb * WPW + wave;
  const int64_t t0 = gw * T / W;
  const int64_t t1 = (gw + 1) * T / W;
  if (t0 < t1) {
    // Ring of R wave-tile images: tiles t+1 .. t+R-1 stream in (LDS-DMA) while tile t is decoded; each tile is
    // exactly D DMA instructions, so "tile t landed" is vmcnt(<= (tiles issued after t) * D).
    const int R = q->ring;
    const int D = q->dma_per_tile;
    int isi = find_segment(segs, q->num_segments, t0);   // issue cursor: segment, its tile range, ring slot
    int64_t ifirst = segs[isi].first_wtile;
    int64_t iend = ifirst + segs[isi].num_wtiles;
    // LM: the issue segment's plan table, one dword per lane (its load drains the ring once per segment crossing)
    uint32_t ip = LM ? ((const uint32_t*)(plans + isi))[lane] : 0u;
    int64_t ti = t0;
    int islot = 0;
    const uint32_t ring_lds = lds_addr(ring);
    auto issue_next = [&]() {
      while (ti >= iend) {
        ++isi;
        ifirst = segs[isi].first_wtile;
        iend = ifirst + segs[isi].num_wtiles;
        if (LM) ip = ((const uint32_t*)(plans + isi))[lane];
      }
      if constexpr (LM) stage_tile_lm(ip, ti - ifirst, ring_lds + 4u * (uint32_t)(islot * img_dw), lane, D);
      else stage_tile<STEPS>(segs + isi, ti - ifirst, ring + islot * img_dw, lane, D);
      ++ti;
      islot = islot + 1 == R ? 0 : islot + 1;
    };
    for (int k = 0; k < R - 1 && ti < t1; ++k) issue_next();

    int si = find_segment(segs, q->num_segments, t0);
    int pslot = 0;
    int64_t t = t0;
    while (t < t1) {
      // segment-outer / tile-inner: `seg` is invariant in the inner loop, so its descriptors stay in SGPRs
      const DevSeg* seg = segs + si;
      const uint32_t matched_seg0 = matched;
      const int64_t seg_first = seg->first_wtile;
      const int64_t seg_end = min(t1, seg_first + (int64_t)seg->num_wtiles);
      const uint32_t pp = LM ? ((const uint32_t*)(plans + si))[lane] : 0u;  // process segment's plan table
      const bool stream_only = q->debug_stream_only != 0;
      if constexpr (LM) {
        if (!stream_only && isi == si) {
          // Steady state: the tile to issue lies in this segment too; every per-segment value of the issue side and of
          // the leaf is hoisted into registers (no segment-crossing checks, no plan-table reads per tile).
          LmIssue I;
          I.nst = (int)rl(pp, 0);
#pragma unroll
          for (int c = 0; c < kLmStaged; ++c) {
            const int nb = c < I.nst ? (int)rl(pp, 10 + 4 * c) : 0;
            I.base[c] = (const char*)(((uint64_t)rl(pp, 9 + 4 * c) << 32) | rl(pp, 8 + 4 * c));
            I.stride[c] = 256 * (int64_t)nb;  // bytes of one wave tile of an nb-bit column
            I.off[c] = 4u * rl(pp, 11 + 4 * c);
            I.nfull[c] = (16 * nb) / 64;
            const int tail = (16 * nb) % 64;
            I.tail[c] = tail ? ((1ull << tail) - 1ull) : 0ull;
          }
          I.dummy = (const void*)(((uint64_t)rl(pp, 5) << 32) | rl(pp, 4));
          const int64_t issue_end = min(iend, t1);
          const bool single_range = (int)rl(pp, 1) == 1 && (int)rl(pp, 24) == PA_LEAF_DICT_RANGE && (rl(pp, 29) & 2u);
          if (single_range) {
            // one eager DICT_RANGE literal closing its clause: the hoisted leaf on whole tiles (the ragged last tile of
            // a segment goes through process_tile_lm)
            const int nb0 = (int)rl(pp, 25);
            const uint32_t off0 = 4u * rl(pp, 26), lo0 = rl(pp, 27), hi0 = rl(pp, 28);
            const bool neg0 = (rl(pp, 29) & 1u) != 0;
            const int64_t full_tiles = (int64_t)(int32_t)rl(pp, 2) / kWTileDocs;
            while (t < seg_end && ti < issue_end) {
              uint32_t slot_off = (uint32_t)(pslot * img_dw);
              lm_wait_issue(I, slot_off, R, D, ti - (t + 1), ring_lds + 4u * (uint32_t)(islot * img_dw), ti - ifirst,
                            16u * (uint32_t)lane);
              ++ti;
              islot = islot + 1 == R ? 0 : islot + 1;
              if (t - seg_first < full_tiles) {
                uint32_t m = leaf_lm_any(nb0, PA_LEAF_DICT_RANGE, ring_lds + 4u * slot_off + off0, lane, lo0, hi0,
                                         nullptr);
                if (neg0) m = ~m;
                if (__ballot(m != 0) != 0)
                  matched += tile_survivors<STRAT, 32, 1>(q, seg, ring + slot_off, (t - seg_first) * kWTileDocs, m,
                                                          lane, acc.lds, *acc.ps, la);
              } else {
                process_tile_lm<STRAT>(q, seg, pp, t - seg_first, ring + slot_off, ring_lds + 4u * slot_off, lane, acc,
                                       matched, la);
              }
              pslot = pslot + 1 == R ? 0 : pslot + 1;
              ++t;
            }
          } else {
            while (t < seg_end && ti < issue_end) {
              uint32_t slot_off = (uint32_t)(pslot * img_dw);
              lm_wait_issue(I, slot_off, R, D, ti - (t + 1), ring_lds + 4u * (uint32_t)(islot * img_dw), ti - ifirst,
                            16u * (uint32_t)lane);
              ++ti;
              islot = islot + 1 == R ? 0 : islot + 1;
              process_tile_lm<STRAT>(q, seg, pp, t - seg_first, ring + slot_off, ring_lds + 4u * slot_off, lane, acc,
                                     matched, la);
              pslot = pslot + 1 == R ? 0 : pslot + 1;
              ++t;
            }
          }
        }
      }
      for (; t < seg_end; ++t) {
        uint32_t slot_off = (uint32_t)(pslot * img_dw);
        wait_tile((int)(ti - (t + 1)), D, slot_off);  // tile t has landed in its slot (same-wave LDS-DMA)
        if (ti < t1) issue_next();                     // refill the slot tile t-1 used
        if (!stream_only) {
          if constexpr (LM) process_tile_lm<STRAT>(q, seg, pp, t - seg_first, ring + slot_off, ring_lds + 4u * slot_off, lane, acc, matched, la);
          else process_tile<STRAT, STEPS>(q, seg, t - seg_first, ring + slot_off, lane, acc, matched, la);
        }
        pslot = pslot + 1 == R ? 0 : pslot + 1;
      }
      if constexpr (is_lane(STRAT) && STRAT != STRAT_LANE_CNT) lane_acc_segment_end(q, seg, la, matched != matched_seg0);
      if (t < t1) {
        ++si;
        while (t >= segs[si].first_wtile + segs[si].num_wtiles) ++si;
      }
    }
  }

  if constexpr (!is_pcount(STRAT) && !is_pemit(STRAT))
    if (q->leap_mode) {
      // the entries kept in LDS to the wave's slice, then its count (every wave: the search kernel reads every count)
      const uint32_t nl = min(la.leap_n, (uint32_t)q->leap_lds_cap);
      AS1 unsigned long long* list = gp(q->leap_out) + 3 * (int64_t)q->num_segments + 1 + (int64_t)q->leap_slices +
                                     (int64_t)la.leap_slice * (int64_t)q->leap_cap;
      const lds_u64_t* ll = (const lds_u64_t*)(uintptr_t)la.leap_lds;
      for (uint32_t k = (uint32_t)lane; k < nl; k += kWave) list[k] = ll[k];
      if (lane == 0) gp(q->leap_out)[3 * (int64_t)q->num_segments + 1 + la.leap_slice] = la.leap_n;
    }
  if (!is_pemit(STRAT)) {  // (the partitioned count pass counts numDocsScanned; its emit pass sees the same docs)
    const int64_t wm = wave_sum_i64((int64_t)matched);
    if (lane == 0 && wm != 0) __hip_atomic_fetch_add(gp(q->matched_docs), (unsigned long long)wm, RLX);
    if constexpr (is_lane(STRAT)) {  // COUNT(*) of an aggregation-only query = the docs the filter kept
      if (lane == 0 && wm != 0) __hip_atomic_fetch_add(gp(q->count), (unsigned long long)wm, RLX);
      if constexpr (STRAT == STRAT_LANE_DICT) {
        // each thread folds histogram entries t, t + WGS, ... : count * value into its lane accumulator (exact split
        // pair for 64-bit values: count < 2^32, so count * low32 and count * high32 fit their int64 halves)
        __syncthreads();
        for (int a = 0; a < q->num_aggs; ++a) {
          const DevAgg& A = q->aggs[a];
          if (A.hist_card <= 0) continue;
          const uint32_t* h = (const uint32_t*)(lds_acc + A.hist_off);
          const DevCol& c = segs[0].cols[A.slot];
          int64_t r0, r1;
          la_get(la, a, r0, r1);
          for (int i = threadIdx.x; i < A.hist_card; i += WGS) {
            const uint32_t n = h[i];
            if (n == 0) continue;
            if (A.src == SRC_DOUBLE) {
              r0 = __builtin_bit_cast(int64_t, __builtin_bit_cast(double, r0) + (double)n * gp(c.dict_f64)[i]);
            } else {
              const int64_t v = gp(c.dict_i64)[i];
              if (A.src == SRC_INT) {
                r0 += (int64_t)n * v;
              } else {
                r0 += (int64_t)n * (int64_t)(uint32_t)v;
                r1 += (int64_t)n * (v >> 32);
              }
            }
          }
          la_set(la, a, r0, r1);
        }
      }
      if constexpr (STRAT != STRAT_LANE_CNT) lane_acc_flush(q, la, lane);
    }
  }
  if (is_pcount(STRAT)) {
    __syncthreads();
    const uint32_t* hist = (const uint32_t*)lds_acc;
    for (int p = threadIdx.x; p < q->num_parts; p += WGS) gp(ps.hist)[lb * q->num_parts + p] = hist[p];
  }
  if (is_pemit(STRAT)) {
    // every bin's rest (< one bin) between the range's front and back, then sentinel records up to the padded end
    __syncthreads();
    const BinState B = bin_state(q, lds_acc);
    const int P = q->num_parts, pv = q->pv;
    for (int p = q->part_lo + threadIdx.x; p < q->part_hi; p += WGS) {
      const bool isv = p < pv;
      const uint32_t nw = isv ? (uint32_t)q->rec_words_v : 1u;
      const uint32_t BS = (uint32_t)(isv ? q->bs_v : q->bs_h);
      const lds_u32_t* bin = isv ? lds_ptr(lds_acc + q->lds_bins_v) + (uint32_t)p * BS * nw
                                 : lds_ptr(lds_acc + q->lds_bins_h) + (uint32_t)(p - pv) * (BS + (uint32_t)kDocVals);
      AS1 uint32_t* recs = gp(isv ? ps.recs_v : ps.recs_h);
      const uint32_t n = B.cnt[p], o = B.front[p];
      const uint32_t h = gp(ps.hist)[lb * P + p];
      if ((n >= BS || o + n != B.back[p]) && !q->debug_emit)  // the emit pass must see exactly the count pass's records
        __hip_atomic_fetch_add(gp(q->matched_docs) + 3, 1ull, RLX);
      AS1 uint32_t* d = recs + (B.start[p] + o) * (uint64_t)nw;
      const uint32_t nn = n < BS ? n : BS;
      for (uint32_t e = 0; e < nn * nw; ++e) d[e] = bin[e];
      const uint32_t padded = (h + BS - 1u) / BS * BS;
      AS1 uint32_t* z = recs + (B.start[p] + h) * (uint64_t)nw;
      for (uint32_t e = 0; e < (padded - h) * nw; ++e) z[e] = (e % nw) == 0 ? kSentinel : 0u;
    }
  }
  if (STRAT == STRAT_LDS) {
    __syncthreads();
    const int64_t K = q->num_keys;
    const uint32_t* cnt = (const uint32_t*)(lds_acc + q->lds_count_off);
    for (int64_t k = threadIdx.x; k < K; k += WGS) {
      const uint32_t c = cnt[k];
      if (c == 0) continue;
      __hip_atomic_fetch_add(gp(q->count) + k, (unsigned long long)c, RLX);
      for (int a = 0; a < q->num_aggs; ++a) {
        const DevAgg& A = q->aggs[a];
        switch (A.type) {
          case PA_AGG_SUM:
            if (A.src == SRC_INT) {
              __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + k, ((const unsigned long long*)(lds_acc + A.lds_off))[k], RLX);
            } else if (A.src == SRC_LONG) {
              const unsigned long long* r = (const unsigned long long*)(lds_acc + A.lds_off);
              __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + 2 * k, r[2 * k], RLX);
              __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + 2 * k + 1, r[2 * k + 1], RLX);
            } else {
              __hip_atomic_fetch_add(gp(A.acc_f64) + k, ((const double*)(lds_acc + A.lds_off))[k], RLX);
            }
            break;
          case PA_AGG_COUNT_MV:
            __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + k, ((const unsigned long long*)(lds_acc + A.lds_off))[k], RLX);
            break;
          case PA_AGG_MIN: __hip_atomic_fetch_min(gp((long long*)A.acc_i64) + k, ((const long long*)(lds_acc + A.lds_off))[k], RLX); break;
          case PA_AGG_MAX: __hip_atomic_fetch_max(gp((long long*)A.acc_i64) + k, ((const long long*)(lds_acc + A.lds_off))[k], RLX); break;
          case PA_AGG_DISTINCTCOUNT: {  // presence words with a value seen here -> bytes of the global block
            const uint32_t* r = (const uint32_t*)(lds_acc + A.lds_off + k * A.nvals);
            AS1 uint8_t* g = gp(A.acc_hll) + k * A.nvals;
            for (int64_t j = 0; j < A.nvals / 4; ++j) {
              const uint32_t w = r[j];
              if (w == 0) continue;
              for (int b = 0; b < 4; ++b)
                if ((w >> (8 * b)) & 0xffu) g[4 * j + b] = 1;
            }
          } break;
          case PA_AGG_DISTINCTCOUNTHLL: {
            const uint32_t* r = (const uint32_t*)(lds_acc + A.lds_off) + (k << A.log2m);
            uint8_t* g = A.acc_hll + (k << A.log2m);
            for (int j = 0; j < (1 << A.log2m); ++j)
              if (r[j] != 0) atomic_max_u8(g + j, r[j]);
          } break;
          default: break;
        }
      }
    }
  }
}

// Kernel-pointer getters of the scan variants, one translation unit per group (parallel builds): nullptr when the
// unit does not hold the strategy.
const void* scan_fn_std(int strategy, int steps, int lm);   // pa_scan_std.hip: LDS, GLOBAL (LANE via scan_fn_lane)
const void* scan_fn_lane(int strategy, int steps, int lm);  // pa_scan_lane.hip: LANE and its variants
const void* scan_fn_part_a(int strategy);                  // pa_scan_part_a.hip: PCOUNT + emit variants (one part)
const void* scan_fn_part_b(int strategy);                  // pa_scan_part_b.hip: the other emit variants
const void* scan_fn_part_mv(int strategy);                 // pa_scan_part_mv.hip: the multi-value group-by passes
const void* scan_fn_gdense(int strategy, int lm);          // pa_scan_gdense.hip: STRAT_GDENSE (pa_gdense.h)

}  // namespace pa
