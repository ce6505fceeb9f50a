// HIP kernels of the segment query hot path (gfx950 / CDNA4 only).
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
#include <hip/hip_runtime.h>
#include "pa_device.h"
#include "pa_launch.h"

namespace pa {

typedef __attribute__((address_space(3))) uint32_t lds_u32_t;

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
  const uint32_t lo = words[we];
  const uint32_t hi = words[we - 1];
  return __builtin_amdgcn_alignbit(hi, lo, (~(uint32_t)e1) & 31u) & nbits_mask(nb);
}

__device__ __forceinline__ uint32_t decode_dict_id(const DevCol& c, const uint32_t* img, int doc_local,
                                                   int64_t doc) {
  return c.lds_off >= 0 ? decode_lds(img + c.lds_off, doc_local, c.nbits) : decode_global(c.words, doc, c.nbits);
}

// Issue the LDS-DMA of one wave tile of every staged column of `seg` into the wave image `img`.
__device__ __forceinline__ void stage_tile(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                           int64_t wt, uint32_t* img, int lane) {
  for (int si = 0; si < q->num_staged; ++si) {
    const DevCol& c = seg->cols[q->staged_slots[si]];
    const int nb = c.nbits;
    const uint32_t* src = c.words + wt * (int64_t)(64 * nb);
    uint32_t* dst = img + c.lds_off;
    const int chunks = 16 * nb;  // 16-byte chunks of this column's wave tile (64*nb words)
    for (int c0 = 0; c0 < chunks; c0 += 64) {
      if (c0 + lane < chunks)
        __builtin_amdgcn_global_load_lds((const void*)(src + 4 * (c0 + lane)), (lds_u32_t*)(dst + 4 * c0), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ bool eval_leaf(const DevLeaf& L, const DevSeg* __restrict__ seg, const uint32_t* img,
                                          int doc_local, int64_t doc, bool valid) {
  const DevCol& c = seg->cols[L.slot];
  bool m = false;
  if (L.kind == PA_LEAF_DICT_RANGE) {
    const uint32_t id = decode_dict_id(c, img, doc_local, doc);
    m = (id - (uint32_t)L.lo) < (uint32_t)L.span;
  } else if (L.kind == PA_LEAF_DICT_SET) {
    const uint32_t id = decode_dict_id(c, img, doc_local, doc);
    m = (L.lut[id >> 5] >> (id & 31u)) & 1u;
  } else if (L.kind == PA_LEAF_RAW_RANGE) {
    switch (c.vtype) {
      case PA_INT: { const int64_t v = ((const int32_t*)c.raw)[doc]; m = v >= L.ilo && v <= L.ihi; } break;
      case PA_LONG: { const int64_t v = ((const int64_t*)c.raw)[doc]; m = v >= L.ilo && v <= L.ihi; } break;
      case PA_FLOAT: { const double v = ((const float*)c.raw)[doc]; m = v >= L.dlo && v <= L.dhi; } break;
      default: { const double v = ((const double*)c.raw)[doc]; m = v >= L.dlo && v <= L.dhi; } break;
    }
  }
  return valid && (m != (L.negate != 0));
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

__device__ __forceinline__ AggValue agg_value(const DevAgg& A, int a, const DevSeg* __restrict__ seg,
                                              const uint32_t* img, int doc_local, int64_t doc) {
  AggValue out{0, 0.0};
  const DevCol& c = seg->cols[A.slot];
  if (c.kind == COL_SV_DICT) {
    const uint32_t id = decode_dict_id(c, img, doc_local, doc);
    if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
      out.i = seg->hll_lut[a][id];
    } else if (A.src != SRC_DOUBLE) {
      out.i = c.dict_i64[id];
    } else {
      out.d = c.dict_f64[id];
    }
  } else {  // raw column
    int64_t iv = 0;
    double dv = 0.0;
    switch (c.vtype) {
      case PA_INT: iv = ((const int32_t*)c.raw)[doc]; dv = (double)iv; break;
      case PA_LONG: iv = ((const int64_t*)c.raw)[doc]; dv = (double)iv; break;
      case PA_FLOAT: { const float f = ((const float*)c.raw)[doc]; dv = f; iv = __builtin_bit_cast(int32_t, f); } break;
      default: dv = ((const double*)c.raw)[doc]; iv = __builtin_bit_cast(int64_t, dv); break;
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

// ---- accumulator targets ----
template <int STRAT>
struct Acc {
  const DevQuery* q;
  unsigned char* lds;

  __device__ __forceinline__ void add_count(int64_t key, uint32_t n) const {
    if (STRAT == STRAT_LDS) atomicAdd((uint32_t*)(lds + q->lds_count_off) + key, n);
    else atomicAdd(q->count + key, (unsigned long long)n);
  }
  __device__ __forceinline__ void add_i64(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) atomicAdd((unsigned long long*)(lds + A.lds_off) + key, (unsigned long long)v);
    else atomicAdd((unsigned long long*)A.acc_i64 + key, (unsigned long long)v);
  }
  __device__ __forceinline__ void add_f64(const DevAgg& A, int64_t key, double v) const {
    if (STRAT == STRAT_LDS) atomicAdd((double*)(lds + A.lds_off) + key, v);
    else atomicAdd(A.acc_f64 + key, v);
  }
  __device__ __forceinline__ void min_i64(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) atomicMin((long long*)(lds + A.lds_off) + key, (long long)v);
    else atomicMin((long long*)A.acc_i64 + key, (long long)v);
  }
  __device__ __forceinline__ void max_i64(const DevAgg& A, int64_t key, int64_t v) const {
    if (STRAT == STRAT_LDS) atomicMax((long long*)(lds + A.lds_off) + key, (long long)v);
    else atomicMax((long long*)A.acc_i64 + key, (long long)v);
  }
  __device__ __forceinline__ void max_hll(const DevAgg& A, int64_t key, uint32_t jr) const {
    const int64_t idx = (key << A.log2m) + (jr >> 8);
    if (STRAT == STRAT_LDS) atomicMax((uint32_t*)(lds + A.lds_off) + idx, jr & 0xffu);
    else atomicMax(A.acc_hll + idx, jr & 0xffu);
  }
};

// Accumulate the matched lanes (`matched` = wave mask) of one 64-doc step.
template <int STRAT>
__device__ __forceinline__ void accumulate_step(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                                const uint32_t* img, int doc_local, int64_t doc,
                                                uint64_t matched, int lane, const Acc<STRAT>& acc) {
  const bool mine = (matched >> lane) & 1ull;
  // table-wide group key (DictionaryBasedGroupKeyGenerator: rawKey = sum dictId_j * prod_{k<j} card_k)
  int64_t key = 0;
  for (int j = 0; j < q->num_gb; ++j) {
    const DevCol& c = seg->cols[q->gb_slot[j]];
    uint32_t id = 0;
    if (mine) {
      id = decode_dict_id(c, img, doc_local, doc);
      const int32_t* rm = seg->remap[j];
      if (rm != nullptr) id = (uint32_t)rm[id];
    }
    key += (int64_t)id * q->gb_stride[j];
  }

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

template <int STRAT>
__device__ __forceinline__ void process_tile(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                             int64_t wt, const uint32_t* img, int lane, const Acc<STRAT>& acc) {
  const int64_t doc_base = wt * kWTileDocs;
  const int nleaves = q->num_leaves;
  const int64_t ndocs = seg->num_docs;
  for (int i = 0; i < kSteps; ++i) {
    const int doc_local = i * kWave + lane;
    const int64_t doc = doc_base + doc_local;
    const bool valid = doc < ndocs;
    uint64_t m = __ballot(valid);
    if (m == 0) break;
    uint64_t clause = 0;
    for (int li = 0; li < nleaves; ++li) {
      if (m == 0) break;
      const DevLeaf& L = seg->leaves[li];
      clause |= __ballot(eval_leaf(L, seg, img, doc_local, doc, valid));
      if (L.clause_end) {
        m &= clause;
        clause = 0;
      }
    }
    if (m == 0) continue;
    accumulate_step<STRAT>(q, seg, img, doc_local, doc, m, lane, acc);
  }
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

template <int STRAT>
__global__ void __launch_bounds__(kWGSize) scan_kernel(const DevQuery* __restrict__ q,
                                                       const DevSeg* __restrict__ segs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  unsigned char* lds_acc = (unsigned char*)smem;
  const uint32_t acc_dwords = STRAT == STRAT_LDS ? (q->lds_acc_bytes >> 2) : 0u;
  const int img_dw = q->image_dwords_max;
  uint32_t* img0 = smem + acc_dwords + wave * 2 * img_dw;
  uint32_t* img1 = img0 + img_dw;
  Acc<STRAT> acc{q, lds_acc};

  if (STRAT == STRAT_LDS) {
    const int64_t K = q->num_keys;
    uint32_t* cnt = (uint32_t*)(lds_acc + q->lds_count_off);
    for (int64_t k = threadIdx.x; k < K; k += kWGSize) cnt[k] = 0;
    for (int a = 0; a < q->num_aggs; ++a) {
      const DevAgg& A = q->aggs[a];
      if (A.type == PA_AGG_COUNT) continue;
      if (A.type == PA_AGG_DISTINCTCOUNTHLL) {
        uint32_t* r = (uint32_t*)(lds_acc + A.lds_off);
        for (int64_t k = threadIdx.x; k < (K << A.log2m); k += kWGSize) r[k] = 0;
      } else {
        int64_t* r = (int64_t*)(lds_acc + A.lds_off);
        const int64_t init = A.type == PA_AGG_MIN ? INT64_MAX : (A.type == PA_AGG_MAX ? INT64_MIN : 0);
        const int64_t n = (A.type == PA_AGG_SUM && A.src == SRC_LONG) ? 2 * K : K;
        for (int64_t k = threadIdx.x; k < n; k += kWGSize) r[k] = init;  // SUM(double) 0.0 == all-zero bits
      }
    }
    __syncthreads();
  }

  const int64_t T = q->total_wtiles;
  const int64_t W = (int64_t)gridDim.x * kWavesPerWG;
  const int64_t gw = (int64_t)blockIdx.x * kWavesPerWG + wave;
  const int64_t t0 = gw * T / W;
  const int64_t t1 = (gw + 1) * T / W;
  if (t0 < t1) {
    const DevSeg* seg = segs + find_segment(segs, q->num_segments, t0);
    stage_tile(q, seg, t0 - seg->first_wtile, img0, lane);
    for (int64_t t = t0; t < t1; ++t) {
      const bool odd = ((t - t0) & 1) != 0;
      uint32_t* img = odd ? img1 : img0;
      uint32_t* nimg = odd ? img0 : img1;
      vm_wait_all();  // tile t has landed in `img` (same-wave LDS-DMA: vmcnt covers it)
      const DevSeg* cur = seg;
      if (t + 1 < t1) {
        while (t + 1 >= seg->first_wtile + seg->num_wtiles) ++seg;
        stage_tile(q, seg, t + 1 - seg->first_wtile, nimg, lane);
      }
      process_tile<STRAT>(q, cur, t - cur->first_wtile, img, lane, acc);
    }
  }

  if (STRAT == STRAT_LDS) {
    __syncthreads();
    const int64_t K = q->num_keys;
    const uint32_t* cnt = (const uint32_t*)(lds_acc + q->lds_count_off);
    for (int64_t k = threadIdx.x; k < K; k += kWGSize) {
      const uint32_t c = cnt[k];
      if (c == 0) continue;
      atomicAdd(q->count + k, (unsigned long long)c);
      for (int a = 0; a < q->num_aggs; ++a) {
        const DevAgg& A = q->aggs[a];
        switch (A.type) {
          case PA_AGG_SUM:
            if (A.src == SRC_INT) {
              atomicAdd((unsigned long long*)A.acc_i64 + k, ((const unsigned long long*)(lds_acc + A.lds_off))[k]);
            } else if (A.src == SRC_LONG) {
              const unsigned long long* r = (const unsigned long long*)(lds_acc + A.lds_off);
              atomicAdd((unsigned long long*)A.acc_i64 + 2 * k, r[2 * k]);
              atomicAdd((unsigned long long*)A.acc_i64 + 2 * k + 1, r[2 * k + 1]);
            } else {
              atomicAdd(A.acc_f64 + k, ((const double*)(lds_acc + A.lds_off))[k]);
            }
            break;
          case PA_AGG_MIN: atomicMin((long long*)A.acc_i64 + k, ((const long long*)(lds_acc + A.lds_off))[k]); break;
          case PA_AGG_MAX: atomicMax((long long*)A.acc_i64 + k, ((const long long*)(lds_acc + A.lds_off))[k]); break;
          case PA_AGG_DISTINCTCOUNTHLL: {
            const uint32_t* r = (const uint32_t*)(lds_acc + A.lds_off) + (k << A.log2m);
            uint32_t* g = A.acc_hll + (k << A.log2m);
            for (int j = 0; j < (1 << A.log2m); ++j)
              if (r[j] != 0) atomicMax(g + j, r[j]);
          } break;
          default: break;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- segment-load / query-prep kernels

__global__ void bswap_words_kernel(uint32_t* w, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    w[i] = __builtin_bswap32(w[i]);
}

// dictId -> (register << 8) | rank for DISTINCTCOUNTHLL over a dictionary column.
// MurmurHash.hash(Object) on the boxed dictionary value (Dictionary.get): Integer/Long -> hashLong(v),
// Float -> hashLong(Float.floatToRawIntBits(v)), Double -> hashLong(Double.doubleToRawLongBits(v)).
__global__ void hll_lut_numeric_kernel(const int64_t* di, const double* dd, int32_t vtype, int32_t card,
                                       int32_t log2m, uint32_t* lut) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < card; i += gridDim.x * blockDim.x) {
    int64_t x;
    switch (vtype) {
      case PA_INT: case PA_LONG: x = di[i]; break;
      case PA_FLOAT: x = __builtin_bit_cast(int32_t, (float)dd[i]); break;
      default: x = __builtin_bit_cast(int64_t, dd[i]); break;
    }
    lut[i] = hll_slot_rank(murmur_hash_long(x), log2m);
  }
}

__global__ void hll_lut_hashes_kernel(const int32_t* hashes, int32_t card, int32_t log2m, uint32_t* lut) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < card; i += gridDim.x * blockDim.x)
    lut[i] = hll_slot_rank(hashes[i], log2m);
}

__global__ void fill_i64_kernel(int64_t* p, int64_t n, int64_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// out[i*per + j] = src[keys[i]*per + j] for elements of `esize` bytes (4 or 8)
__global__ void gather_kernel(const void* src, int esize, int64_t per, const int64_t* keys, int64_t n, void* out) {
  const int64_t total = n * per;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per, j = i - r * per;
    const int64_t s = keys[r] * per + j;
    if (esize == 8) ((uint64_t*)out)[i] = ((const uint64_t*)src)[s];
    else ((uint32_t*)out)[i] = ((const uint32_t*)src)[s];
  }
}

static int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

// ---------------------------------------------------------------- launchers

hipError_t launch_bswap_words(uint32_t* w, int64_t n, hipStream_t s) {
  bswap_words_kernel<<<grid_for(n, 256), 256, 0, s>>>(w, n);
  return hipGetLastError();
}

hipError_t launch_hll_lut_numeric(const int64_t* di, const double* dd, int32_t vtype, int32_t card, int32_t log2m,
                                  uint32_t* lut, hipStream_t s) {
  hll_lut_numeric_kernel<<<grid_for(card, 256), 256, 0, s>>>(di, dd, vtype, card, log2m, lut);
  return hipGetLastError();
}

hipError_t launch_hll_lut_hashes(const int32_t* hashes, int32_t card, int32_t log2m, uint32_t* lut, hipStream_t s) {
  hll_lut_hashes_kernel<<<grid_for(card, 256), 256, 0, s>>>(hashes, card, log2m, lut);
  return hipGetLastError();
}

hipError_t launch_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s) {
  fill_i64_kernel<<<grid_for(n, 256), 256, 0, s>>>(p, n, v);
  return hipGetLastError();
}

hipError_t launch_gather(const void* src, int esize, int64_t per, const int64_t* keys, int64_t n, void* out,
                         hipStream_t s) {
  gather_kernel<<<grid_for(n * per, 256), 256, 0, s>>>(src, esize, per, keys, n, out);
  return hipGetLastError();
}

hipError_t set_scan_lds_limit(int strategy, int bytes) {
  if (strategy == STRAT_LDS)
    return hipFuncSetAttribute((const void*)scan_kernel<STRAT_LDS>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  return hipFuncSetAttribute((const void*)scan_kernel<STRAT_GLOBAL>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

hipError_t launch_scan(int strategy, int grid, int lds_bytes, const DevQuery* q, const DevSeg* segs, hipStream_t s) {
  if (strategy == STRAT_LDS) scan_kernel<STRAT_LDS><<<grid, kWGSize, lds_bytes, s>>>(q, segs);
  else scan_kernel<STRAT_GLOBAL><<<grid, kWGSize, lds_bytes, s>>>(q, segs);
  return hipGetLastError();
}

}  // namespace pa
