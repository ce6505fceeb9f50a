// Dense filter + GROUP BY over a small key space (STRAT_GDENSE), gfx950.
//
// Reference semantics: GroupByOperator -> DefaultGroupByExecutor.process (DefaultGroupByExecutor.java:131-158):
// DictionaryBasedGroupKeyGenerator raw keys (:254-340) and {Count,Sum,Min,Max}AggregationFunction.aggregateGroupBySV
// per matching doc, then GroupByCombineOperator's merge (one table-wide accumulator set per GPU here).
//
// Why a separate kernel: the LDS strategy of pa_scan.h reads a GROUP BY's post-filter columns per matching doc from HBM
// and gathers dictionary values from HBM. Every such load is consumed while the next tiles' LDS-DMA is in flight, and
// vmcnt counts loads, stores and LDS-DMA together in issue order: waiting for the doc's load waits for the ring too, so a
// dense filter serialises the ring (GROUP BY day SUM(dictionary m) at 50 %: 0.056 of the HBM roofline). Here:
//   * every column the query reads is staged by the wave's LDS-DMA ring: filter, group-by and aggregation columns,
//     raw metrics as 4- or 8-byte "bit columns" (a 2048-doc tile of a raw LONG is 16 KiB, 16 DMA instructions);
//   * value dictionaries (int32 / int64 / double) and group-key remaps sit in LDS, loaded once per segment by the
//     workgroup (identical dictionaries of different segments share one load);
//   * a workgroup owns one contiguous range of tiles and its waves interleave over it (wave w takes tiles t0 + w,
//     t0 + w + 4, ...), so the four waves cross segment boundaries together and the per-segment tables can be swapped
//     between two barriers;
//   * accumulators are LDS-privatised over the box of group keys the filter admits (a unit clause day BETWEEN a AND b
//     leaves b - a + 1 keys of that column), replicated so lanes sharing a key update different banks (lane l takes
//     replica l & (R - 1)); one global atomic per non-empty key and aggregation at the end;
//   * dense tiles are walked step-major (doc 64 i + lane: conflict-free LDS decodes of consecutive docs, the lane-major
//     match bit fetched by ds_bpermute), sparse tiles lane-major (each lane its own matching docs).
// A matching doc thus costs LDS operations only: decodes (ds_read2), table reads and ds_add/min/max atomics.
#pragma once
#include "pa_scan.h"

namespace pa {

typedef __attribute__((address_space(3))) int32_t lds_i32_t;
typedef __attribute__((address_space(3))) int64_t lds_i64_t;
typedef __attribute__((address_space(3))) double lds_f64_t;

template <class T>
__device__ __forceinline__ T* lds_at(uint32_t byte_addr) {
  return (T*)(uintptr_t)byte_addr;
}

// Value of doc `doc` (0..2047) of an nb-bit column region of a staged tile image (region[-1] is a guard word).
__device__ __forceinline__ uint32_t gd_decode(const lds_u32_t* region, uint32_t doc, uint32_t nb) {
  const uint32_t e1 = doc * nb + (nb - 1u);
  const uint32_t we = e1 >> 5;
  return __builtin_amdgcn_alignbit(region[we - 1], region[we], (~e1) & 31u) & nbits_mask((int)nb);
}

// Per-tile, per-lane view of the staged columns for the step-major walk: doc 64 i + lane of an nb-bit column has its
// last bit at 64 nb i + (lane nb + nb - 1), and 64 nb i is a multiple of 32: the two stream words holding the value sit
// at a lane constant plus 8 nb i bytes, and the alignbit shift is a lane constant. A decode is then one v_mad (address),
// one ds_read2_b32 and alignbit + and. Raw columns: 4 or 8 bytes per doc, stride 256 / 512 bytes per step.
// MG / MA: the group-by columns / non-COUNT aggregations a kernel variant handles at most (fewer: fewer VGPRs)
template <int MG = kGdMaxGb, int MA = kGdMaxAgg>
struct GdLane {
  uint32_t ga[MG], gs[MG];    // group-by column j: LDS address of step 0's word pair, alignbit shift
  uint32_t va[MA], vs[MA];    // aggregation k: the same for its column (raw: the value's address)
};

template <int MG, int MA>
__device__ __forceinline__ void gd_lane_setup(uint32_t gt, uint32_t img, int lane, GdLane<MG, MA>& L) {
  const int ngb = (int)rl(gt, 0), na = (int)rl(gt, 1);
#pragma unroll
  for (int j = 0; j < MG; ++j) {
    if (j >= ngb) break;
    const uint32_t nb = rl(gt, 5 + 6 * j);
    const uint32_t c = (uint32_t)lane * nb + nb - 1u;
    L.ga[j] = img + 4u * rl(gt, 4 + 6 * j) + 4u * ((c >> 5) - 1u);
    L.gs[j] = (~c) & 31u;
  }
#pragma unroll
  for (int k = 0; k < MA; ++k) {
    if (k >= na) break;
    const int vsrc = (int)rl(gt, 22 + 6 * k);
    const uint32_t reg = img + 4u * rl(gt, 24 + 6 * k);
    if (vsrc <= GVS_TF) {
      const uint32_t nb = rl(gt, 25 + 6 * k);
      const uint32_t c = (uint32_t)lane * nb + nb - 1u;
      L.va[k] = reg + 4u * ((c >> 5) - 1u);
      L.vs[k] = (~c) & 31u;
    } else {
      L.va[k] = reg + (uint32_t)lane * ((vsrc == GVS_RI32 || vsrc == GVS_RF32) ? 4u : 8u);
      L.vs[k] = 0u;
    }
  }
}

// dictId of step st[k] of a column: word pair at a + 8 nb st, shift sh
template <int N>
__device__ __forceinline__ void gd_dec(uint32_t a, uint32_t sh, uint32_t nb, const uint32_t (&st)[N], uint32_t (&id)[N]) {
  const uint32_t stride = 8u * nb, mask = nbits_mask((int)nb);
  uint32_t w0[N], w1[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const lds_u32_t* p = lds_at<const lds_u32_t>(a + st[k] * stride);
    w0[k] = p[0];
    w1[k] = p[1];
  }
#pragma unroll
  for (int k = 0; k < N; ++k) id[k] = __builtin_amdgcn_alignbit(w0[k], w1[k], sh) & mask;
}

// N docs per lane (step st[k] of the tile: doc 64 st[k] + lane; on[k]): group key, then COUNT and every aggregation into
// replica r of the key's LDS accumulators. Parameters come from the segment's GdSegPlan in the VGPR gt (v_readlane at
// compile-time lanes: no scalar loads, whose lgkmcnt waits would also wait for the LDS operations in flight); every load
// is an LDS read. errs counts matching docs whose key fell outside the LDS box (cannot happen when the planner's box is
// right; the query then reports an error).
// BOX (the key box is the filter, gd_box_tile): errs counts the docs inside the box instead (numDocsScanned).
template <int N, bool BOX = false, int MG = kGdMaxGb, int MA = kGdMaxAgg>
__device__ __forceinline__ void gd_batch(uint32_t gt, const GdLane<MG, MA>& L, const uint32_t (&st)[N], const bool (&on_in)[N],
                                         uint32_t r, uint32_t base, uint32_t& errs) {
  const int ngb = (int)rl(gt, 0), na = (int)rl(gt, 1);
  const uint32_t rpl = rl(gt, 2);
  const uint32_t dbg = rl(gt, 3);  // measurement only (PA_DEBUG_EMIT): 2 = no atomics, 4 = no value-table reads
  uint32_t key[N];
  bool on[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    key[k] = 0u;
    on[k] = on_in[k];
  }
#pragma unroll
  for (int j = 0; j < MG; ++j) {
    if (j >= ngb) break;
    const int o = 4 + 6 * j;
    uint32_t id[N];
    gd_dec<N>(L.ga[j], L.gs[j], rl(gt, o + 1), st, id);
    const int tab = (int)rl(gt, o + 2);
    if (tab >= 0) {
      const lds_i32_t* t = lds_at<const lds_i32_t>(base + (uint32_t)tab);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const int32_t e = t[id[k]];
        on[k] = on[k] && e >= 0;
        key[k] += (uint32_t)e;
      }
    } else {
      const uint32_t lo = rl(gt, o + 3), span = rl(gt, o + 4), ls = rl(gt, o + 5);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const uint32_t c0 = id[k] - lo;
        on[k] = on[k] && c0 < span;
        key[k] += c0 * ls;
      }
    }
  }
  uint32_t idx[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    errs += BOX ? (on[k] ? 1u : 0u) : ((on_in[k] && !on[k]) ? 1u : 0u);
    idx[k] = (key[k] << rpl) | r;
  }
  if (dbg & 2) {
#pragma unroll
    for (int k = 0; k < N; ++k) asm volatile("" ::"v"(idx[k]), "v"((uint32_t)on[k]));
  } else {
    lds_u32_t* cnt = lds_at<lds_u32_t>(base);
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (on[k]) __hip_atomic_fetch_add(cnt + idx[k], 1u, WG_RLX);
  }
#pragma unroll
  for (int g = 0; g < MA; ++g) {
    if (g >= na) break;
    const int o = 22 + 6 * g;
    const int vs = (int)rl(gt, o), op = (int)rl(gt, o + 1);
    const uint32_t acc = base + rl(gt, o + 4);
    int64_t vi[N];
    double vd[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      vi[k] = 0;
      vd[k] = 0.0;
    }
    if (vs <= GVS_TF) {  // dictionary column: dictId from the staged stream, value from the LDS table (or the id)
      uint32_t id[N];
      gd_dec<N>(L.va[g], L.vs[g], rl(gt, o + 3), st, id);
      const uint32_t tab = base + rl(gt, o + 5);
      if (vs == GVS_ID || (dbg & 4)) {
#pragma unroll
        for (int k = 0; k < N; ++k) vi[k] = id[k];
      } else if (vs == GVS_T32) {
#pragma unroll
        for (int k = 0; k < N; ++k) vi[k] = lds_at<const lds_i32_t>(tab)[id[k]];
      } else if (vs == GVS_T64) {
#pragma unroll
        for (int k = 0; k < N; ++k) vi[k] = lds_at<const lds_i64_t>(tab)[id[k]];
      } else {
#pragma unroll
        for (int k = 0; k < N; ++k) vd[k] = lds_at<const lds_f64_t>(tab)[id[k]];
      }
    } else if (vs == GVS_RI32) {
#pragma unroll
      for (int k = 0; k < N; ++k) vi[k] = lds_at<const lds_i32_t>(L.va[g] + 256u * st[k])[0];
    } else if (vs == GVS_RF32) {
#pragma unroll
      for (int k = 0; k < N; ++k) vd[k] = __builtin_bit_cast(float, lds_at<const lds_u32_t>(L.va[g] + 256u * st[k])[0]);
    } else if (vs == GVS_RI64) {
#pragma unroll
      for (int k = 0; k < N; ++k) vi[k] = lds_at<const lds_i64_t>(L.va[g] + 512u * st[k])[0];
    } else {
#pragma unroll
      for (int k = 0; k < N; ++k) vd[k] = lds_at<const lds_f64_t>(L.va[g] + 512u * st[k])[0];
    }
    const bool fl = gvs_float(vs);
    if (dbg & 2) {
#pragma unroll
      for (int k = 0; k < N; ++k) asm volatile("" ::"v"((uint32_t)vi[k]), "v"((uint32_t)(vi[k] >> 32)), "v"(vd[k]));
      continue;
    }
    switch (op) {
      case GOP_SUM_I:
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (on[k]) __hip_atomic_fetch_add(lds_at<lds_u64_t>(acc) + idx[k], (uint64_t)vi[k], WG_RLX);
        break;
      case GOP_SUM_L:
#pragma unroll
        for (int k = 0; k < N; ++k) {
          if (!on[k]) continue;
          __hip_atomic_fetch_add(lds_at<lds_u64_t>(acc) + 2 * idx[k], (uint64_t)(uint32_t)vi[k], WG_RLX);
          __hip_atomic_fetch_add(lds_at<lds_u64_t>(acc) + 2 * idx[k] + 1, (uint64_t)(vi[k] >> 32), WG_RLX);
        }
        break;
      case GOP_SUM_F:
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (on[k]) __hip_atomic_fetch_add(lds_at<lds_f64_t>(acc) + idx[k], vd[k], WG_RLX);
        break;
      case GOP_MIN_I:
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (on[k]) __hip_atomic_fetch_min(lds_at<lds_i64_t>(acc) + idx[k], fl ? f64_order_encode(vd[k]) : vi[k], WG_RLX);
        break;
      case GOP_MAX_I:
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (on[k]) __hip_atomic_fetch_max(lds_at<lds_i64_t>(acc) + idx[k], fl ? f64_order_encode(vd[k]) : vi[k], WG_RLX);
        break;
      case GOP_MIN_U:
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (on[k]) __hip_atomic_fetch_min(lds_at<lds_u32_t>(acc) + idx[k], (uint32_t)vi[k], WG_RLX);
        break;
      default:  // GOP_MAX_U
#pragma unroll
        for (int k = 0; k < N; ++k)
          if (on[k]) __hip_atomic_fetch_max(lds_at<lds_u32_t>(acc) + idx[k], (uint32_t)vi[k], WG_RLX);
        break;
    }
  }
}

// The matching docs of one tile, step-major match bits s (bit i <=> doc 64 i + lane): every lane walks its own set bits,
// KB per batch, so a batch is productive on every lane until the lanes run out of matches (max popcount over the
// lanes batches: ~23 of 32 steps at 50 % density, ~7 at 10 %).
template <int KB = 4, int MG = kGdMaxGb, int MA = kGdMaxAgg>
__device__ __forceinline__ void gd_walk(uint32_t gt, uint32_t img, uint32_t s, int lane, uint32_t base, uint32_t& errs) {
  GdLane<MG, MA> L;
  gd_lane_setup(gt, img, lane, L);
  const uint32_t r = (uint32_t)lane & ((1u << rl(gt, 2)) - 1u);
#pragma unroll 1
  while (__ballot(s != 0) != 0) {
    uint32_t st[KB];
    bool on[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      on[k] = s != 0;
      st[k] = on[k] ? (uint32_t)__builtin_ctz(s) : 0u;
      s &= s - 1u;
    }
    gd_batch<KB, false, MG, MA>(gt, L, st, on, r, base, errs);
  }
}

// A DICT_SET leaf whose dictId bitmap sits in LDS (gd_lut): bit i of lane l <=> doc 64 i + l of the step-major tile
// (leaf_bits' decode, the bitmap read with ds_read instead of a global load that would wait for the tile ring).
template <int STEPS, class LeafT>
__device__ __forceinline__ uint32_t gd_leaf_set_lds(const LeafT& L, uint32_t img, int lane, uint32_t lut_addr) {
  const int nb = L.nbits;
  const uint32_t mask = nbits_mask(nb);
  const uint32_t e1 = (uint32_t)lane * (uint32_t)nb + (uint32_t)(nb - 1);
  const uint32_t sh = (~e1) & 31u;
  const int step = 2 * nb;
  // (address-space-3 pointers: a generic one would be a flat load, counted in vmcnt too)
  const lds_u32_t* p = lds_at<const lds_u32_t>(img + 4u * (uint32_t)(L.lds_off + (int)(e1 >> 5)));
  const lds_u32_t* lut = lds_at<const lds_u32_t>(lut_addr);
  uint32_t id[STEPS];
#pragma unroll
  for (int i = 0; i < STEPS; ++i) id[i] = __builtin_amdgcn_alignbit(p[i * step - 1], p[i * step], sh) & mask;
  uint32_t w[STEPS];
#pragma unroll
  for (int i = 0; i < STEPS; ++i) w[i] = lut[id[i] >> 5];
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < STEPS; ++i) bits |= ((w[i] >> (id[i] & 31u)) & 1u) << i;
  return L.negate ? ~bits : bits;
}

// The filter is exactly the key box (GdSegPlan::box: unit DICT_RANGE clauses on group-by columns): every valid doc of a
// step-major tile goes through gd_batch, whose box check is the filter, KB steps per batch at compile-time step offsets
// — no filter evaluation, no walk. Returns the lane's docs inside the box.
template <int MG = kGdMaxGb, int MA = kGdMaxAgg>
__device__ __forceinline__ uint32_t gd_box_tile(uint32_t gt, uint32_t img, uint32_t valid, int lane, uint32_t base) {
  constexpr int KB = 4;
  GdLane<MG, MA> L;
  gd_lane_setup(gt, img, lane, L);
  const uint32_t r = (uint32_t)lane & ((1u << rl(gt, 2)) - 1u);
  uint32_t inbox = 0;
#pragma unroll
  for (int s0 = 0; s0 < kGdSmSteps; s0 += KB) {
    uint32_t st[KB];
    bool on[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      st[k] = (uint32_t)(s0 + k);
      on[k] = (valid >> (s0 + k)) & 1u;
    }
    gd_batch<KB, true, MG, MA>(gt, L, st, on, r, base, inbox);
  }
  return inbox;
}

// Filter of one lane-major 2048-doc tile (every literal eager: the planner's condition), then the transpose of the match
// words to step-major bits (lane l, bit i <=> doc 64 i + l lives in lane 2i + l/32, bit l % 32: one ds_bpermute per step)
// and the walk.
__device__ __forceinline__ uint32_t gd_tile(uint32_t gt, uint32_t pp, int64_t wt, uint32_t img, int lane,
                                            uint32_t base, uint32_t& errs) {
  const int64_t doc_base = wt * kWTileDocs;
  const int64_t rem = (int64_t)(int32_t)rl(pp, 2) - doc_base;
  uint32_t m = 0xffffffffu;
  if (rem < kWTileDocs) {
    const int64_t n = rem - 32 * lane;  // docs of this lane's 32 that exist
    m = n >= 32 ? 0xffffffffu : (n <= 0 ? 0u : ((1u << n) - 1u));
  }
  uint32_t clause = 0;
  const int neager = (int)rl(pp, 1);
  for (int l = 0; l < neager; ++l) {
    const int b = 24 + 8 * l;
    const int flags = (int)rl(pp, b + 5);
    const uint32_t* lut = (const uint32_t*)(((uint64_t)rl(pp, b + 7) << 32) | rl(pp, b + 6));
    uint32_t bits = leaf_lm_any((int)rl(pp, b + 1), (int)rl(pp, b), img + 4u * rl(pp, b + 2), lane, rl(pp, b + 3),
                                rl(pp, b + 4), lut);
    if (flags & 1) bits = ~bits;
    clause |= bits;
    if (flags & 2) {
      m &= clause;
      clause = 0;
      if (__ballot(m != 0) == 0) return 0;
    }
  }
  const uint32_t mine = (uint32_t)__builtin_popcount(m);
  if (__ballot(mine != 0) == 0) return 0;
  if (rl(gt, 3) & 1) return mine;  // measurement only: filter only
  uint32_t s = 0;
  const int sh = lane & 31;
#pragma unroll
  for (int i = 0; i < kSteps; ++i) {
    const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((2 * i + (lane >> 5)) << 2, (int)m);
    s |= ((w >> sh) & 1u) << i;
  }
  gd_walk(gt, img, s, lane, base, errs);
  return mine;
}

// Step-major 1024-doc tiles: filter by leaf_bits (bit i of lane l <=> doc 64 i + l) straight into the walk's order.
// KB: docs per lane per walk batch (the 12-wave register-staged variant walks 2 at a time: at 4 its tile ring no longer
// fits the 170 VGPRs of 3 waves per SIMD and a ring slot spills, each refill then waiting for its own load)
template <int KB = 4, int MG = kGdMaxGb, int MA = kGdMaxAgg>
__device__ __forceinline__ uint32_t gd_tile_sm(uint32_t gt, const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                               int64_t wt, const uint32_t* img_ptr, uint32_t img, int lane,
                                               uint32_t base, uint32_t& errs) {
  constexpr int ST = kGdSmSteps;
  // descriptors through the constant address space (scalar loads): a flat load of a descriptor field would be counted
  // in vmcnt, and waiting for it would wait for every tile in flight
  if (rl(gt, 3) & 32) return 0;  // measurement only: the tile streamed in, nothing evaluated
  CSegT* cs = (CSegT*)(uintptr_t)uniform_ptr(seg);
  CQ* cq = (CQ*)(uintptr_t)uniform_ptr(q);
  const int64_t doc_base = wt * (ST * kWave);
  const int64_t rem = (int64_t)cs->num_docs - doc_base;
  uint32_t m;
  if (rem >= ST * kWave) {
    m = (1u << ST) - 1u;
  } else {
    const int64_t n = rem > lane ? (rem - lane + kWave - 1) / kWave : 0;
    m = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
  }
  if (rl(gt, kGdBoxDword)) return gd_box_tile<MG, MA>(gt, img, m, lane, base);
  uint32_t clause = 0;
  const int neager = cq->num_eager;
  for (int li = 0; li < neager; ++li) {
    const auto& L = cs->leaves[li];
    const int lut = cq->gd_lut[li];
    if (lut >= 0) clause |= gd_leaf_set_lds<ST>(L, img, lane, base + (uint32_t)lut);
    else clause |= leaf_bits<ST>(L, img_ptr, doc_base, lane);
    if (L.clause_end) {
      m &= clause;
      clause = 0;
      if (__ballot(m != 0) == 0) return 0;
    }
  }
  const uint32_t mine = (uint32_t)__builtin_popcount(m);
  if (__ballot(mine != 0) == 0) return 0;
  if (rl(gt, 3) & 1) return mine;  // measurement only: filter only
  gd_walk<KB, MG, MA>(gt, img, m, lane, base, errs);
  return mine;
}

// ---------------------------------------------------------------- lane-major walk (STRAT_GDENSE_LM8 / LM16)
// The image of a 1024-doc tile is the step-major one (stage_tile<kGdSmSteps>: each column's 1024 nb-bit values as one
// contiguous stream), but lane l takes docs [16 l, 16 l + 16): its 16 values of an nb-bit column are the stream bits
// [16 l nb, 16 (l + 1) nb), i.e. nb / 2 + 1 words read once (ds_read_b32, conflict-free for odd nb, 2-way for nb = 2
// mod 4) and unpacked with constant shifts (a switch on nb selects the unpacker). Against the step-major walk's ds_read2
// per doc and column (plus its ds_bpermute transpose and set-bit walk), a column costs 1/32 of a read per doc, and every
// value the accumulation needs is already in the lane's registers: a matching doc costs only its LDS atomics, issued
// under a per-doc EXEC mask for docs i = 0..15 in turn.
constexpr int kGdlDocs = 16;  // docs per lane of a 1024-doc tile

// The lane's 16 values of an NB-bit column region (word 0 = the tile's first stream word), MSB-aligned: value i in
// the top NB bits of v[i] (junk below). The lane's bits start at 16 lane NB, a word boundary or (odd NB, odd lane) 16
// bits into a word: the words are read from one word earlier on word boundaries and realigned with ONE alignbit each
// (shift 0 or 16), then unpacked with constant shifts.
template <int NB>
__device__ __forceinline__ void gdl_top(uint32_t region, int lane, uint32_t (&v)[kGdlDocs]) {
  constexpr int K = (kGdlDocs * NB + 31) / 32 + 1;  // words holding the lane's 16 values (+1: the unpack's window)
  // (an opaque copy of the lane id per call: otherwise the compiler computes every unpacker case's lane offset ahead
  // of the switch, ~5 instructions per case on every tile)
  uint32_t ln = (uint32_t)lane;
  asm volatile("" : "+v"(ln));
  const uint32_t bit0 = __umul24(ln, (uint32_t)(kGdlDocs * NB));
  uint32_t w[K];
  if constexpr ((kGdlDocs * NB) % 32 != 0) {  // odd NB
    const uint32_t sh = bit0 & 16u;
    const lds_u32_t* p = lds_at<const lds_u32_t>(region + 4u * ((bit0 >> 5) - 1u + (sh >> 4)));
    uint32_t r[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) r[j] = p[j];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = __builtin_amdgcn_alignbit(r[j], r[j + 1], sh);
  } else {
    const lds_u32_t* p = lds_at<const lds_u32_t>(region + 4u * (bit0 >> 5));
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = p[j];
  }
#pragma unroll
  for (int i = 0; i < kGdlDocs; ++i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    v[i] = (o + NB <= 32) ? (w[j] << o) : __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o);
  }
}

#define PA_GDL_NB_CASES(X)                                                                                          \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)   \
  X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31)

// The lane's 16 dictIds of an NB-bit column region: gdl_top's words, each id by one v_bfe_u32 (two ops when it
// straddles two words)
template <int NB>
__device__ __forceinline__ void gdl_idv(uint32_t region, int lane, uint32_t (&v)[kGdlDocs]) {
  constexpr int K = (kGdlDocs * NB + 31) / 32 + 1;
  uint32_t ln = (uint32_t)lane;
  asm volatile("" : "+v"(ln));
  const uint32_t bit0 = __umul24(ln, (uint32_t)(kGdlDocs * NB));
  uint32_t w[K];
  if constexpr ((kGdlDocs * NB) % 32 != 0) {
    const uint32_t sh = bit0 & 16u;
    const lds_u32_t* p = lds_at<const lds_u32_t>(region + 4u * ((bit0 >> 5) - 1u + (sh >> 4)));
    uint32_t r[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) r[j] = p[j];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = __builtin_amdgcn_alignbit(r[j], r[j + 1], sh);
  } else {
    const lds_u32_t* p = lds_at<const lds_u32_t>(region + 4u * (bit0 >> 5));
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = p[j];
  }
#pragma unroll
  for (int i = 0; i < kGdlDocs; ++i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    if (o + NB <= 32) v[i] = __builtin_amdgcn_ubfe(w[j], 32 - o - NB, NB);
    else v[i] = __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o) >> (32 - NB);
  }
}

// dictIds of the lane's 16 docs (nb wave-uniform, 1..31)
__device__ __forceinline__ void gdl_ids(int nb, uint32_t region, int lane, uint32_t (&id)[kGdlDocs]) {
  switch (nb) {
#define PA_GDL_IDS(N)                                                \
  case N: {                                                          \
    gdl_idv<N>(region, lane, id);                                    \
  } break;
    PA_GDL_NB_CASES(PA_GDL_IDS)
#undef PA_GDL_IDS
    default:
#pragma unroll
      for (int i = 0; i < kGdlDocs; ++i) id[i] = 0;
      break;
  }
}

// Match bits of one DICT_RANGE / DICT_SET leaf over the lane's 16 docs (bit i <=> doc 16 lane + i), before negation.
// DICT_RANGE bounds MSB-aligned by the host (leaf_bits): 3 VALU per doc; a DICT_SET bitmap in LDS: the word by the
// dictId's high bits, the bit by v_bfe, 5 VALU + one LDS read per doc (the bitmap is always in LDS: a global load in
// the tile loop would make the compiler's vmcnt waits cover the DMA in flight — the planner keeps such queries off the
// lane-major walk). keep_it: the unpacked values also go to `keep` (the group key is this leaf's column).
template <int NB>
__device__ __forceinline__ uint32_t gdl_leaf(int kind, uint32_t region, int lane, uint32_t lo_t, uint32_t hi_t,
                                             uint32_t lut_lds, bool keep_it, uint32_t (&keep)[kGdlDocs]) {
  uint32_t t[kGdlDocs];
  gdl_top<NB>(region, lane, t);
  if (keep_it) {
#pragma unroll
    for (int i = 0; i < kGdlDocs; ++i) keep[i] = t[i];
  }
  if (kind == PA_LEAF_DICT_RANGE) {
    uint32_t nm = 0;
#pragma unroll
    for (int i = kGdlDocs - 1; i >= 0; --i) {
      uint32_t u;
      asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
          "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
          "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
          : [nm] "+v"(nm), [u] "=&v"(u)
          : [t] "v"(t[i]), [lo] "s"(lo_t), [hi] "s"(hi_t)
          : "vcc");
    }
    return ~nm & 0xffffu;
  }
  uint32_t id[kGdlDocs], w[kGdlDocs];
#pragma unroll
  for (int i = 0; i < kGdlDocs; ++i) {
    id[i] = t[i] >> (32 - NB);
    w[i] = *lds_at<const lds_u32_t>(lut_lds + 4u * (id[i] >> 5));
  }
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < kGdlDocs; ++i) bits |= __builtin_amdgcn_ubfe(w[i], id[i], 1) << i;
  return bits;
}

__device__ __forceinline__ uint32_t gdl_leaf_any(int nb, int kind, uint32_t region, int lane, uint32_t lo_t,
                                                 uint32_t hi_t, uint32_t lut_lds, bool keep_it,
                                                 uint32_t (&keep)[kGdlDocs]) {
  switch (nb) {
#define PA_GDL_LEAF(N) \
  case N: return gdl_leaf<N>(kind, region, lane, lo_t, hi_t, lut_lds, keep_it, keep);
    PA_GDL_NB_CASES(PA_GDL_LEAF)
#undef PA_GDL_LEAF
    default: return 0;
  }
}

// The lane's 16 values of a staged raw column (4 or 8 bytes each, 16-byte aligned region): 4 / 8 ds_read_b128
__device__ __forceinline__ void gdl_raw32(uint32_t region, int lane, uint32_t (&v)[kGdlDocs]) {
  const lds_u32x4_t* p = lds_at<const lds_u32x4_t>(region + 64u * (uint32_t)lane);
  u32x4 r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = p[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[4 * k] = r[k].x;
    v[4 * k + 1] = r[k].y;
    v[4 * k + 2] = r[k].z;
    v[4 * k + 3] = r[k].w;
  }
}
__device__ __forceinline__ void gdl_raw64(uint32_t region, int lane, uint64_t (&v)[kGdlDocs]) {
  const lds_u32x4_t* p = lds_at<const lds_u32x4_t>(region + 128u * (uint32_t)lane);
  u32x4 r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = p[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[2 * k] = ((uint64_t)r[k].y << 32) | r[k].x;
    v[2 * k + 1] = ((uint64_t)r[k].w << 32) | r[k].z;
  }
}

// One LDS-DMA wave instruction with a scalar base address (global_load_lds_dwordx4 vaddr = 32-bit lane offset, saddr):
// lane l copies the 16 bytes at sbase + voff_l to dst + 16 l. `mask` (a partial instruction): the lanes that take part.
__device__ __forceinline__ void dma16s(uint32_t voff, uint64_t sbase, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(dst));
}
__device__ __forceinline__ void dma16s_masked(uint32_t voff, uint64_t sbase, uint32_t dst, uint64_t mask) {
  uint32_t keep;
  uint64_t save;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, %5\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %3\n\t"
      "s_mov_b32 m0, %0\n\t"
      "s_mov_b64 exec, %1"
      : "=&s"(keep), "=&s"(save)
      : "v"(voff), "s"(sbase), "s"(dst), "s"(mask));
}

// The lane-major walk's DMA descriptors of one segment, wave-uniform (SGPRs, read once per segment from the GdLmIssue
// VGPR): per staged column the tile-0 source, bytes per tile, 16-byte chunks per tile and LDS destination. Issuing a
// tile is then scalar arithmetic and one instruction per 1 KiB, no descriptor read and no per-lane address math.
struct GdlDma {
  int nc;
  uint64_t src[kGdlMaxCols];
  uint32_t stride[kGdlMaxCols], chunks[kGdlMaxCols], dst[kGdlMaxCols];
};

__device__ __forceinline__ void gdl_dma_load(uint32_t ip, GdlDma& d) {
  d.nc = (int)rl(ip, 0);
#pragma unroll
  for (int c = 0; c < kGdlMaxCols; ++c) {
    d.src[c] = ((uint64_t)rl(ip, 2 + 5 * c) << 32) | rl(ip, 1 + 5 * c);
    d.stride[c] = rl(ip, 3 + 5 * c);
    d.chunks[c] = rl(ip, 4 + 5 * c);
    d.dst[c] = rl(ip, 5 + 5 * c);
  }
}

// One 1024-doc tile: every column's chunks, exactly D instructions (dummies re-read column 0's first chunk into the
// image's leading guard words)
__device__ __forceinline__ void gdl_dma_issue(const GdlDma& d, int64_t wt, uint32_t img, uint32_t voff, int lane,
                                              const int D) {
  int issued = 0;
#pragma unroll
  for (int c = 0; c < kGdlMaxCols; ++c) {
    if (c >= d.nc) break;
    const uint64_t base = d.src[c] + (uint64_t)wt * d.stride[c];
    const uint32_t dst = img + d.dst[c];
    const int chunks = (int)d.chunks[c];
    int c0 = 0;
    for (; c0 + 64 <= chunks; c0 += 64, ++issued) dma16s(voff, base + 16u * (uint32_t)c0, dst + 16u * (uint32_t)c0);
    if (c0 < chunks) {
      dma16s_masked(voff, base + 16u * (uint32_t)c0, dst + 16u * (uint32_t)c0, (1ull << (chunks - c0)) - 1ull);
      ++issued;
    }
  }
  for (; issued < D; ++issued) dma16s_masked(voff, d.src[0], img, 1ull);
  (void)lane;
}

// LDS-DMA of one 1024-doc tile from the segment's GdLmIssue (VGPR ip), padded to exactly D instructions (the padding
// re-reads the first column's first chunk into the image's guard words).
__device__ __forceinline__ void gdl_stage(uint32_t ip, int64_t wt, uint32_t img, int lane, const int D) {
  const int nc = (int)rl(ip, 0);
  int issued = 0;
  for (int c = 0; c < nc; ++c) {
    const uint32_t b = 1u + 5u * (uint32_t)c;
    const uint64_t src = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)ip, b + 1) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)ip, b)) +
                         (uint64_t)wt * (uint32_t)__builtin_amdgcn_readlane((int)ip, b + 2);
    const int chunks = __builtin_amdgcn_readlane((int)ip, b + 3);
    const uint32_t dst = img + (uint32_t)__builtin_amdgcn_readlane((int)ip, b + 4);
    for (int c0 = 0; c0 < chunks; c0 += 64) {
      if (c0 + lane < chunks) dma16((const void*)(src + 16ull * (uint64_t)(c0 + lane)), dst + 16u * (uint32_t)c0);
      ++issued;
    }
  }
  const uint64_t src0 = ((uint64_t)rl(ip, 2) << 32) | rl(ip, 1);
  for (; issued < D; ++issued)
    if (lane == 0) dma16((const void*)src0, img);
}

// Packed accumulation of the lane's matching docs (bits of `on`) into their rows (LDS byte addresses `addr`): one word
// per doc, COUNT + every SUM term at its field. The fields of one doc's word do not overlap, so the word is built with
// ORs, 32 bits at a time (a term below bit 32 also spills into the high word).
template <int MA>
__device__ __forceinline__ void gdl_packed_accumulate(uint32_t gt, uint32_t lp, uint32_t img, int lane, uint32_t base,
                                                      uint32_t on, const uint32_t (&addr)[kGdlDocs]) {
  constexpr int ND = kGdlDocs;
  const int na = (int)rl(gt, 1);
  uint32_t plo[ND], phi[ND];
  const uint32_t oc = rl(lp, 3);
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    plo[i] = oc < 32 ? 1u << oc : 0u;
    phi[i] = oc < 32 ? 0u : 1u << (oc - 32);
  }
#pragma unroll 1
  for (int g = 0; g < MA; ++g) {
    if (g >= na) break;
    const int o = 22 + 6 * g;
    uint32_t id[ND];
    gdl_ids((int)rl(gt, o + 3), img + 4u * rl(gt, o + 2), lane, id);
    if ((int)rl(gt, o) == GVS_T32U) {
      const lds_u32_t* t = lds_at<const lds_u32_t>(base + rl(gt, o + 5));
#pragma unroll
      for (int i = 0; i < ND; ++i) id[i] = t[id[i]];
    }
    const uint32_t sh = (uint32_t)__builtin_amdgcn_readlane((int)lp, 6 + g);
    if (sh >= 32) {
#pragma unroll
      for (int i = 0; i < ND; ++i) phi[i] |= id[i] << (sh - 32);
    } else if (sh == 0) {
#pragma unroll
      for (int i = 0; i < ND; ++i) plo[i] |= id[i];
    } else {
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        plo[i] |= id[i] << sh;
        phi[i] |= __builtin_amdgcn_alignbit(0u, id[i], 32u - sh);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < ND; ++i)
    if ((on >> i) & 1u) __hip_atomic_fetch_add(lds_at<lds_u64_t>(addr[i]), ((uint64_t)phi[i] << 32) | plo[i], WG_RLX);
}

// Drain of a wave's packed rows (GdLmPlan) into the workgroup's accumulators: every non-zero row is read, zeroed and
// split into its fields (COUNT -> the count array, SUM term a -> the aggregation's u64 sums, replica 0).
__device__ __forceinline__ void gdl_drain(uint32_t gt, uint32_t lp, uint32_t rows, int nkeys, int lane, uint32_t base) {
  const int na = (int)rl(gt, 1);
  const uint32_t rpl = rl(gt, 2), off_c = rl(lp, 3);
  lds_u64_t* row = lds_at<lds_u64_t>(rows);
  for (int k = lane; k < nkeys; k += kWave) {
    const uint64_t x = row[k];
    if (x == 0) continue;
    row[k] = 0;
    const uint32_t idx = (uint32_t)k << rpl;
    __hip_atomic_fetch_add(lds_at<lds_u32_t>(base) + idx, (uint32_t)(x >> off_c), WG_RLX);
    for (int g = 0; g < na; ++g) {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)lp, 6 + g);
      const uint32_t hi = g + 1 < na ? (uint32_t)__builtin_amdgcn_readlane((int)lp, 7 + g) : off_c;
      const uint64_t f = (x >> lo) & ((hi - lo) >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull));
      __hip_atomic_fetch_add(lds_at<lds_u64_t>(base + (uint32_t)__builtin_amdgcn_readlane((int)gt, 26 + 6 * g)) + idx, f,
                             WG_RLX);
    }
  }
}

// One 1024-doc tile, lane-major: filter (or the key box), keys, then the LDS updates of the lane's matching docs —
// packed (one ds_add_u64 per doc into the wave's row, GdLmPlan) or per aggregation (the lane's 16 values, then one
// atomic per matching doc). Every parameter comes from the segment's plan VGPRs gt (GdSegPlan) and lp (GdLmPlan).
// Returns the lane's docs counted in numDocsScanned.
template <int MG = kGdMaxGb, int MA = kGdMaxAgg>
__device__ __forceinline__ uint32_t gdl_tile(uint32_t gt, uint32_t lp, int64_t wt, uint32_t img, int lane,
                                             uint32_t base, uint32_t rows, uint32_t& errs) {
  constexpr int ND = kGdlDocs;
  const uint32_t dbg = rl(gt, 3);  // measurement only (PA_DEBUG_EMIT): 32 stream only, 1 filter only, 2 no atomics
  if (dbg & 32) return 0;
  const int64_t rem = (int64_t)(int32_t)rl(lp, 1) - wt * (kGdSmSteps * kWave);
  uint32_t m = 0xffffu;
  if (rem < kGdSmSteps * kWave) {
    const int64_t n = rem - ND * lane;
    m = n >= ND ? 0xffffu : (n <= 0 ? 0u : ((1u << n) - 1u));
  }
  const bool box = rl(gt, kGdBoxDword) != 0;
  const int key_leaf = box ? -1 : (int)rl(lp, 12);
  uint32_t kt[ND];  // key_leaf >= 0: that leaf's unpacked values (MSB-aligned) = group-by column 0's
  if (!box) {
    uint32_t clause = 0;
    const int nl = (int)rl(lp, 0);
    for (int li = 0; li < nl; ++li) {
      const uint32_t b = 16u + 7u * (uint32_t)li;
      const uint32_t code = (uint32_t)__builtin_amdgcn_readlane((int)lp, b);
      const int lut_lds = __builtin_amdgcn_readlane((int)lp, b + 4);
      uint32_t bits = gdl_leaf_any((int)(code >> 16), (int)(code & 0xffu),
                                   img + (uint32_t)__builtin_amdgcn_readlane((int)lp, b + 1), lane,
                                   (uint32_t)__builtin_amdgcn_readlane((int)lp, b + 2),
                                   (uint32_t)__builtin_amdgcn_readlane((int)lp, b + 3), base + (uint32_t)lut_lds,
                                   li == key_leaf, kt);
      if (code & 0x100u) bits = ~bits & 0xffffu;
      clause |= bits;
      if (code & 0x200u) {
        m &= clause;
        clause = 0;
        if (__ballot(m != 0) == 0) return 0;
      }
    }
  }
  if (__ballot(m != 0) == 0) return 0;
  if (dbg & 1) return (uint32_t)__builtin_popcount(m);
  const int ngb = (int)rl(gt, 0), na = (int)rl(gt, 1);
  if (rl(lp, 2) && ngb == 1 && (int)rl(gt, 6) < 0) {
    // packed, one group-by column without a key table: the doc's packed-row address straight from its dictId
    // (rows + 8 (id - lo)), the box check only where the filter does not imply it (GdLmPlan key_in_box)
    const uint32_t nb = rl(gt, 5), lo = rl(gt, 7), span = rl(gt, 8);
    uint32_t id[ND];
    if (key_leaf >= 0) {
#pragma unroll
      for (int i = 0; i < ND; ++i) id[i] = kt[i] >> (32u - nb);
    } else {
      gdl_ids((int)nb, img + 4u * rl(gt, 4), lane, id);
    }
    uint32_t on = m;
    if (!rl(lp, 13)) {
      uint32_t nm = 0;  // (not in the box: non-matches as in gdl_leaf's range, then cleared from the matches)
#pragma unroll
      for (int i = ND - 1; i >= 0; --i) {
        uint32_t u;
        asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
            "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
            "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
            : [nm] "+v"(nm), [u] "=&v"(u)
            : [t] "v"(id[i]), [lo] "s"(lo), [hi] "s"(span - 1u)
            : "vcc");
      }
      on &= ~nm;
    }
    uint32_t mine;
    if (box) {
      mine = (uint32_t)__builtin_popcount(on);
    } else {
      mine = (uint32_t)__builtin_popcount(m);
      errs += (uint32_t)__builtin_popcount(m & ~on);
    }
    if (dbg & 2) {
#pragma unroll
      for (int i = 0; i < ND; ++i) asm volatile("" ::"v"(id[i]), "v"(on));
      return mine;
    }
    const uint32_t abase = rows - 8u * lo;
#pragma unroll
    for (int i = 0; i < ND; ++i) id[i] = abase + (id[i] << 3);  // (from here on: the row's LDS address)
    gdl_packed_accumulate<MA>(gt, lp, img, lane, base, on, id);
    return mine;
  }
  // group keys: component j = key table entry (per-segment remap into the box, < 0 outside) or dictId - lo (< span)
  uint32_t key[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) key[i] = 0u;
  uint32_t on = m;
#pragma unroll
  for (int j = 0; j < MG; ++j) {
    if (j >= ngb) break;
    const int o = 4 + 6 * j;
    uint32_t id[ND];
    if (j == 0 && key_leaf >= 0) {
      const uint32_t shr = 32u - rl(gt, o + 1);
#pragma unroll
      for (int i = 0; i < ND; ++i) id[i] = kt[i] >> shr;
    } else {
      gdl_ids((int)rl(gt, o + 1), img + 4u * rl(gt, o), lane, id);
    }
    const int tab = (int)rl(gt, o + 2);
    if (tab >= 0) {
      const lds_i32_t* t = lds_at<const lds_i32_t>(base + (uint32_t)tab);
      int32_t e[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) e[i] = t[id[i]];
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        on &= ~((e[i] < 0 ? 1u : 0u) << i);
        key[i] += (uint32_t)e[i];
      }
    } else {
      const uint32_t lo = rl(gt, o + 3), span = rl(gt, o + 4), ls = rl(gt, o + 5);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const uint32_t c0 = id[i] - lo;
        on &= ~((c0 < span ? 0u : 1u) << i);
        key[i] += c0 * ls;
      }
    }
  }
  uint32_t mine;
  if (box) {
    mine = (uint32_t)__builtin_popcount(on);  // the box is the filter: numDocsScanned = the docs inside it
  } else {
    mine = (uint32_t)__builtin_popcount(m);
    errs += (uint32_t)__builtin_popcount(m & ~on);  // (the planner's box holds every match: none expected)
  }
  if (dbg & 2) {
#pragma unroll
    for (int i = 0; i < ND; ++i) asm volatile("" ::"v"(key[i]), "v"(on));
    return mine;
  }
  if (rl(lp, 2)) {
#pragma unroll
    for (int i = 0; i < ND; ++i) key[i] = rows + (key[i] << 3);
    gdl_packed_accumulate<MA>(gt, lp, img, lane, base, on, key);
    return mine;
  }
  const uint32_t rpl = rl(gt, 2);
  const uint32_t r = (uint32_t)lane & ((1u << rpl) - 1u);
#pragma unroll
  for (int i = 0; i < ND; ++i) key[i] = (key[i] << rpl) | r;  // (from here on: the accumulator index)
  {
    lds_u32_t* cnt = lds_at<lds_u32_t>(base);
#pragma unroll
    for (int i = 0; i < ND; ++i)
      if ((on >> i) & 1u) __hip_atomic_fetch_add(cnt + key[i], 1u, WG_RLX);
  }
#pragma unroll 1
  for (int g = 0; g < MA; ++g) {
    if (g >= na) break;
    const int o = 22 + 6 * g;
    const int vs = (int)rl(gt, o), op = (int)rl(gt, o + 1);
    const uint32_t reg = img + 4u * rl(gt, o + 2);
    const uint32_t acc = base + rl(gt, o + 4);
    // v[i]: the value as an int64, or a double's bits (float sources)
    uint64_t v[ND];
    if (vs <= GVS_TF || vs == GVS_T32U) {  // dictionary column: dictId from the staged stream, value from the LDS table
      uint32_t id[ND];
      gdl_ids((int)rl(gt, o + 3), reg, lane, id);
      const uint32_t tab = base + rl(gt, o + 5);
      if (vs == GVS_ID) {
#pragma unroll
        for (int i = 0; i < ND; ++i) v[i] = id[i];
      } else if (vs == GVS_T32) {
#pragma unroll
        for (int i = 0; i < ND; ++i) v[i] = (uint64_t)(int64_t)lds_at<const lds_i32_t>(tab)[id[i]];
      } else if (vs == GVS_T32U) {
#pragma unroll
        for (int i = 0; i < ND; ++i) v[i] = lds_at<const lds_u32_t>(tab)[id[i]];
      } else {  // GVS_T64 / GVS_TF: 8-byte entries
#pragma unroll
        for (int i = 0; i < ND; ++i) v[i] = lds_at<const lds_u64_t>(tab)[id[i]];
      }
    } else if (vs == GVS_RI32 || vs == GVS_RF32) {
      uint32_t w[ND];
      gdl_raw32(reg, lane, w);
#pragma unroll
      for (int i = 0; i < ND; ++i)
        v[i] = vs == GVS_RI32 ? (uint64_t)(int64_t)(int32_t)w[i]
                              : __builtin_bit_cast(uint64_t, (double)__builtin_bit_cast(float, w[i]));
    } else {
      gdl_raw64(reg, lane, v);
    }
    const bool fl = gvs_float(vs);
    switch (op) {
      case GOP_SUM_I:
#pragma unroll
        for (int i = 0; i < ND; ++i)
          if ((on >> i) & 1u) __hip_atomic_fetch_add(lds_at<lds_u64_t>(acc) + key[i], v[i], WG_RLX);
        break;
      case GOP_SUM_L:
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          if (!((on >> i) & 1u)) continue;
          __hip_atomic_fetch_add(lds_at<lds_u64_t>(acc) + 2 * key[i], (uint64_t)(uint32_t)v[i], WG_RLX);
          __hip_atomic_fetch_add(lds_at<lds_u64_t>(acc) + 2 * key[i] + 1, (uint64_t)((int64_t)v[i] >> 32), WG_RLX);
        }
        break;
      case GOP_SUM_F:
#pragma unroll
        for (int i = 0; i < ND; ++i)
          if ((on >> i) & 1u)
            __hip_atomic_fetch_add(lds_at<lds_f64_t>(acc) + key[i], __builtin_bit_cast(double, v[i]), WG_RLX);
        break;
      case GOP_MIN_I:
#pragma unroll
        for (int i = 0; i < ND; ++i)
          if ((on >> i) & 1u)
            __hip_atomic_fetch_min(lds_at<lds_i64_t>(acc) + key[i],
                                   fl ? f64_order_encode(__builtin_bit_cast(double, v[i])) : (int64_t)v[i], WG_RLX);
        break;
      case GOP_MAX_I:
#pragma unroll
        for (int i = 0; i < ND; ++i)
          if ((on >> i) & 1u)
            __hip_atomic_fetch_max(lds_at<lds_i64_t>(acc) + key[i],
                                   fl ? f64_order_encode(__builtin_bit_cast(double, v[i])) : (int64_t)v[i], WG_RLX);
        break;
      case GOP_MIN_U:
#pragma unroll
        for (int i = 0; i < ND; ++i)
          if ((on >> i) & 1u) __hip_atomic_fetch_min(lds_at<lds_u32_t>(acc) + key[i], (uint32_t)v[i], WG_RLX);
        break;
      default:  // GOP_MAX_U
#pragma unroll
        for (int i = 0; i < ND; ++i)
          if ((on >> i) & 1u) __hip_atomic_fetch_max(lds_at<lds_u32_t>(acc) + key[i], (uint32_t)v[i], WG_RLX);
        break;
    }
  }
  return mine;
}

// Per-segment LDS tables: key tables of the group-by columns that have them and value tables of the aggregations.
__device__ __forceinline__ bool gd_tables_differ(CQ* q, CSegT* a, CSegT* b) {
  for (int j = 0; j < q->num_gb; ++j)
    if (q->gd_tab[j] >= 0 && a->remap[j] != b->remap[j]) return true;
  for (int i = 0; i < q->num_aggs; ++i)
    if (q->aggs[i].gd_tab >= 0 && a->gd_src[i] != b->gd_src[i]) return true;
  return false;
}

__device__ void gd_load_tables(CQ* q, CSegT* cs, unsigned char* lds, int tid, int nthreads) {
  for (int li = 0; li < q->num_eager; ++li) {  // shared DICT_SET bitmaps (the same in every segment)
    const int off = q->gd_lut[li];
    if (off < 0) continue;
    uint32_t* t = (uint32_t*)(lds + off);
    const uint32_t* src = cs->leaves[li].lut;
    for (int i = tid; i < q->gd_lut_words[li]; i += nthreads) t[i] = gp(src)[i];
  }
  for (int j = 0; j < q->num_gb; ++j) {
    const int tab = q->gd_tab[j];
    if (tab < 0) continue;
    int32_t* t = (int32_t*)(lds + tab);
    const int32_t* rm = cs->remap[j];
    const int32_t card = cs->cols[q->gb_slot[j]].card;
    const int32_t lo = q->gd_lo[j], span = q->gd_span[j], ls = q->gd_ls[j];
    for (int i = tid; i < q->gd_tab_n[j]; i += nthreads) {
      int32_t e = -1;
      if (i < card) {
        const int32_t c = (rm != nullptr ? gp(rm)[i] : i) - lo;
        if (c >= 0 && c < span) e = c * ls;
      }
      t[i] = e;
    }
  }
  for (int a = 0; a < q->num_aggs; ++a) {
    const int tab = q->aggs[a].gd_tab;
    if (tab < 0) continue;
    const int vs = q->aggs[a].gd_vs;
    const int32_t card = cs->cols[q->aggs[a].slot].card;
    const int n = q->aggs[a].gd_tab_n;
    if (vs == GVS_TF) {
      const double* src = (const double*)cs->gd_src[a];
      double* t = (double*)(lds + tab);
      for (int i = tid; i < n; i += nthreads) t[i] = i < card ? gp(src)[i] : 0.0;
    } else {
      const int64_t* src = (const int64_t*)cs->gd_src[a];
      if (vs == GVS_T64) {
        int64_t* t = (int64_t*)(lds + tab);
        for (int i = tid; i < n; i += nthreads) t[i] = i < card ? gp(src)[i] : 0;
      } else if (vs == GVS_T32U) {  // offsets from the smallest value of every segment's dictionary
        uint32_t* t = (uint32_t*)(lds + tab);
        const int64_t b = q->aggs[a].gd_base;
        for (int i = tid; i < n; i += nthreads) t[i] = i < card ? (uint32_t)(gp(src)[i] - b) : 0u;
      } else {
        int32_t* t = (int32_t*)(lds + tab);
        for (int i = tid; i < n; i += nthreads) t[i] = i < card ? (int32_t)gp(src)[i] : 0;
      }
    }
  }
}

__device__ void gd_init(CQ* q, unsigned char* lds, int tid, int nthreads) {
  if (q->gd_pk_base > 0)  // the waves' packed rows (lane-major walk)
    for (uint32_t i = (uint32_t)q->gd_pk_base / 4u + (uint32_t)tid; i < q->lds_acc_bytes / 4u; i += (uint32_t)nthreads)
      ((uint32_t*)lds)[i] = 0u;
  const int64_t n = (int64_t)q->gd_nkeys << q->gd_rp_log2;
  uint32_t* cnt = (uint32_t*)lds;
  for (int64_t i = tid; i < n; i += nthreads) cnt[i] = 0u;
  for (int a = 0; a < q->num_aggs; ++a) {
    if (q->aggs[a].type == PA_AGG_COUNT) continue;
    const int op = q->aggs[a].gd_op;
    unsigned char* p = lds + q->aggs[a].gd_acc;
    if (op == GOP_MIN_U || op == GOP_MAX_U) {
      const uint32_t v = op == GOP_MIN_U ? 0xffffffffu : 0u;
      for (int64_t i = tid; i < n; i += nthreads) ((uint32_t*)p)[i] = v;
    } else {
      const int64_t v = op == GOP_MIN_I ? INT64_MAX : (op == GOP_MAX_I ? INT64_MIN : 0);  // sums: 0 (0.0 == 0 bits)
      const int64_t m = op == GOP_SUM_L ? 2 * n : n;
      for (int64_t i = tid; i < m; i += nthreads) ((int64_t*)p)[i] = v;
    }
  }
}

// One global update per non-empty LDS key and aggregation: replicas reduced, the LDS key mapped back to the table-wide
// key (component j + gd_lo[j] times the direct key-space stride), values in the accumulator section's representation.
__device__ void gd_flush(const DevQuery* __restrict__ q, const DevSeg* __restrict__ segs, unsigned char* lds, int tid,
                         int nthreads) {
  const int nk = q->gd_nkeys;
  const int rp = 1 << q->gd_rp_log2;
  const uint32_t* cnt = (const uint32_t*)lds;
  for (int kl = tid; kl < nk; kl += nthreads) {
    uint64_t c = 0;
    for (int r = 0; r < rp; ++r) c += cnt[kl * rp + r];
    if (c == 0) continue;
    int64_t key = 0;
    for (int j = 0; j < q->num_gb; ++j) {
      const int64_t comp = (kl / q->gd_ls[j]) % q->gd_span[j];
      key += (comp + q->gd_lo[j]) * q->gb_stride[j];
    }
    __hip_atomic_fetch_add(gp(q->count) + key, (unsigned long long)c, RLX);
    for (int a = 0; a < q->num_aggs; ++a) {
      const DevAgg& A = q->aggs[a];
      if (A.type == PA_AGG_COUNT) continue;
      const unsigned char* p = lds + A.gd_acc;
      switch (A.gd_op) {
        case GOP_SUM_I:
        case GOP_SUM_L: {
          __int128 tot = 0;
          if (A.gd_op == GOP_SUM_I) {
            int64_t s = 0;
            for (int r = 0; r < rp; ++r) s += ((const int64_t*)p)[kl * rp + r];
            tot = (A.gd_vs == GVS_ID || A.gd_vs == GVS_T32U)
                      ? (__int128)A.gd_base * (__int128)c + (__int128)A.gd_step * (__int128)s
                      : (__int128)s;
          } else {
            int64_t lo = 0, hi = 0;
            for (int r = 0; r < rp; ++r) {
              lo += ((const int64_t*)p)[2 * (kl * rp + r)];
              hi += ((const int64_t*)p)[2 * (kl * rp + r) + 1];
            }
            tot = (__int128)lo + ((__int128)hi << 32);
          }
          if (A.src == SRC_LONG) {
            const uint64_t lo = (uint64_t)tot & 0xffffffffull;
            const int64_t hi = (int64_t)(tot >> 32);
            __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + 2 * key, (unsigned long long)lo, RLX);
            __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + 2 * key + 1, (unsigned long long)hi, RLX);
          } else {
            __hip_atomic_fetch_add(gp((unsigned long long*)A.acc_i64) + key, (unsigned long long)(int64_t)tot, RLX);
          }
        } break;
        case GOP_SUM_F: {
          double s = 0.0;
          for (int r = 0; r < rp; ++r) s += ((const double*)p)[kl * rp + r];
          __hip_atomic_fetch_add(gp(A.acc_f64) + key, s, RLX);
        } break;
        case GOP_MIN_I:
        case GOP_MAX_I: {
          int64_t v = ((const int64_t*)p)[kl * rp];
          for (int r = 1; r < rp; ++r) {
            const int64_t w = ((const int64_t*)p)[kl * rp + r];
            v = A.gd_op == GOP_MIN_I ? (w < v ? w : v) : (w > v ? w : v);
          }
          if (A.gd_op == GOP_MIN_I) __hip_atomic_fetch_min(gp((long long*)A.acc_i64) + key, (long long)v, RLX);
          else __hip_atomic_fetch_max(gp((long long*)A.acc_i64) + key, (long long)v, RLX);
        } break;
        default: {  // GOP_MIN_U / GOP_MAX_U: dictId of the shared sorted dictionary -> its value
          uint32_t v = ((const uint32_t*)p)[kl * rp];
          for (int r = 1; r < rp; ++r) {
            const uint32_t w = ((const uint32_t*)p)[kl * rp + r];
            v = A.gd_op == GOP_MIN_U ? (w < v ? w : v) : (w > v ? w : v);
          }
          const DevCol& col = segs[0].cols[A.slot];
          const int64_t e = A.src == SRC_DOUBLE ? f64_order_encode(gp(col.dict_f64)[v]) : gp(col.dict_i64)[v];
          if (A.gd_op == GOP_MIN_U) __hip_atomic_fetch_min(gp((long long*)A.acc_i64) + key, (long long)e, RLX);
          else __hip_atomic_fetch_max(gp((long long*)A.acc_i64) + key, (long long)e, RLX);
        } break;
      }
    }
  }
}

// The kernel. LDS: [accumulators | tables] (q->lds_acc_bytes) then each wave's ring of q->ring tile images.
// LM = 1: lane-major 2048-doc tiles (per-segment plan tables); LM = 0: step-major 1024-doc tiles; LM = 2: the same
// 1024-doc images walked lane-major (gdl_tile).
template <int WPW, int LM>
__global__ void __launch_bounds__(WPW * kWave, 1) gdense_kernel(const DevQuery* __restrict__ q_in,
                                                                const DevSeg* __restrict__ segs,
                                                                const LmSegPlan* __restrict__ plans, PartScratch) {
  CQ* q = (CQ*)(uintptr_t)q_in;
  constexpr int WGS = WPW * kWave;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned char* lds = (unsigned char*)smem;
  const uint32_t base = lds_addr(smem);
  const int img_dw = q->image_dwords_max;
  const int R = q->ring, D = q->dma_per_tile;
  const uint32_t ring_lds = base + q->lds_acc_bytes + 4u * (uint32_t)(wave * R * img_dw);
  uint32_t* const ring = smem + (q->lds_acc_bytes >> 2) + wave * R * img_dw;
  gd_init(q, lds, tid, WGS);
  __syncthreads();
  const int64_t T = q->total_wtiles, G = gridDim.x;
  const int64_t lb = q->xcd_major ? xcd_major_block(blockIdx.x, G) : (int64_t)blockIdx.x;
  const int64_t t0 = lb * T / G, t1 = (lb + 1) * T / G;
  uint32_t matched = 0, errs = 0;
  // LM == 2: the segment's GdSegPlan / GdLmPlan, the wave's packed rows, tiles between drains (0: not packed)
  uint32_t gt_cur = 0, lp = 0, rows = 0, pk_drain = 0, since = 0;
  if (t0 < t1) {  // (workgroup-uniform)
    const int nseg = q->num_segments;
    // issue side: this wave's tiles t0 + wave + WPW k, LDS-DMA into its ring, R - 1 tiles ahead
    int64_t ti = t0 + wave;
    int isi = find_segment(segs, nseg, t0);
    int64_t ifirst = segs[isi].first_wtile, iend = ifirst + segs[isi].num_wtiles;
    uint32_t ip = LM == 1 ? ((const uint32_t*)(plans + isi))[lane] : 0u;
    GdlDma dd;  // LM == 2: the issue segment's DMA descriptors (SGPRs)
    dd.nc = 0;
    const uint32_t voff = 16u * (uint32_t)lane;
    if (LM == 2) {
      ip = gp(q->gd_plans)[(int64_t)isi * kGdPlanDw + 64 + lane];  // GdLmIssue
      // (a use right here makes the compiler wait for this load here, once per segment, and not at the next merge
      // point after a tile's DMA issue, where its vmcnt(0) would wait for the DMA too)
      asm volatile("" ::"v"(ip));
      gdl_dma_load(ip, dd);
    }
    int islot = 0;
    auto issue_next = [&]() {
      while (ti >= iend) {
        ++isi;
        ifirst = segs[isi].first_wtile;
        iend = ifirst + segs[isi].num_wtiles;
        if (LM == 1) ip = ((const uint32_t*)(plans + isi))[lane];
        if (LM == 2) {
          ip = gp(q->gd_plans)[(int64_t)isi * kGdPlanDw + 64 + lane];
          asm volatile("" ::"v"(ip));
          gdl_dma_load(ip, dd);
        }
      }
      if constexpr (LM == 1) stage_tile_lm(ip, ti - ifirst, ring_lds + 4u * (uint32_t)(islot * img_dw), lane, D);
      else if constexpr (LM == 2) gdl_dma_issue(dd, ti - ifirst, ring_lds + 4u * (uint32_t)(islot * img_dw), voff, lane, D);
      else stage_tile<kGdSmSteps>(segs + isi, ti - ifirst, ring + islot * img_dw, lane, D);
      ti += WPW;
      islot = islot + 1 == R ? 0 : islot + 1;
    };
    for (int k = 0; k < R - 1 && ti < t1; ++k) issue_next();
    const int s_first = find_segment(segs, nseg, t0), s_last = find_segment(segs, nseg, t1 - 1);
    int64_t t = t0 + wave;
    int pslot = 0;
    for (int s = s_first; s <= s_last; ++s) {  // (every wave walks the same segments: the barriers below match)
      CSegT* cs = (CSegT*)(uintptr_t)(segs + s);
      if (q->gd_tables && (s == s_first || gd_tables_differ(q, (CSegT*)(uintptr_t)(segs + s - 1), cs))) {
        __syncthreads();  // every wave is done with the previous segment's tables
        gd_load_tables(q, cs, lds, tid, WGS);
        __syncthreads();
      }
      const int64_t sfirst = cs->first_wtile;
      const int64_t send = min(t1, sfirst + (int64_t)cs->num_wtiles);
      const uint32_t pp = LM == 1 ? ((const uint32_t*)(plans + s))[lane] : 0u;
      const uint32_t gt = gp(q->gd_plans)[(int64_t)s * kGdPlanDw + lane];  // this segment's GdSegPlan, one dword per lane
      asm volatile("" ::"v"(gt));  // (waited for here, once per segment: see ip)
      gt_cur = gt;
      if (LM == 2) {
        lp = gp(q->gd_plans)[(int64_t)s * kGdPlanDw + 128 + lane];  // GdLmPlan
        asm volatile("" ::"v"(lp));
        pk_drain = rl(lp, 2) ? rl(lp, 4) : 0u;
        rows = base + rl(lp, 5) + (uint32_t)wave * (uint32_t)q->gd_nkeys * 8u;
      }
      for (; t < send; t += WPW) {
        uint32_t slot_off = (uint32_t)(pslot * img_dw);
        if (LM == 2 && (rl(gt, 3) & 64)) {  // measurement only (PA_DEBUG_EMIT 64): no DMA, compute on stale images
          ti = t1;
        } else {
          if (LM == 2 && R == 2) vm_wait<0>();  // (two images: the one tile in flight is this one)
          else wait_tile((int)((ti - t) / WPW - 1), D, slot_off);  // tile t has landed (younger tiles may still fly)
          if (ti < t1) issue_next();
        }
        if constexpr (LM == 1) matched += gd_tile(gt, pp, t - sfirst, ring_lds + 4u * slot_off, lane, base, errs);
        else if constexpr (LM == 2) {
          matched += gdl_tile(gt, lp, t - sfirst, ring_lds + 4u * slot_off, lane, base, rows, errs);
          if (pk_drain && ++since == pk_drain) {  // (packed rows: drained before a field can overflow)
            gdl_drain(gt, lp, rows, q->gd_nkeys, lane, base);
            since = 0;
          }
        }
        else matched += gd_tile_sm(gt, q_in, segs + s, t - sfirst, ring + slot_off, ring_lds + 4u * slot_off, lane, base, errs);
        pslot = pslot + 1 == R ? 0 : pslot + 1;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));  // vmcnt(0): no DMA left in flight
  if constexpr (LM == 2) {
    if (pk_drain) gdl_drain(gt_cur, lp, rows, q->gd_nkeys, lane, base);
  }
  const int64_t wm = wave_sum_i64((int64_t)matched);
  const int64_t we = wave_sum_i64((int64_t)errs);
  if (lane == 0 && wm != 0) __hip_atomic_fetch_add(gp(q->matched_docs), (unsigned long long)wm, RLX);
  if (lane == 0 && we != 0) __hip_atomic_fetch_add(gp(q->matched_docs) + 3, (unsigned long long)we, RLX);
  __syncthreads();
  gd_flush(q_in, segs, lds, tid, WGS);
}

// ---------------------------------------------------------------- register-staged tiles (STRAT_GDENSE_RS*)
// The LDS holds the accumulators, the value tables and ONE tile image per wave; the ring of tiles in flight lives in
// VGPRs: each tile's staged columns are loaded with plain 16-byte global loads — the chunks the LDS-DMA would copy —
// RS - 1 tiles ahead, and written into the wave's image just before the tile is walked. A 64 KiB value table then no
// longer limits the bytes in flight per CU (DMA ring: 12 waves x 1 tile of 3 KiB; here 12 waves x 3 tiles). The
// compiler counts the loads' vmcnt itself (ring slots are compile-time register arrays: the tile loop is unrolled by
// RS). Used when every segment shares the LDS tables (loaded once) and a tile is at most DM wave instructions.
// Every tile issues exactly DM load instructions on every lane, unconditionally (an unused instruction re-reads
// instruction 0's chunk, a lane past a column's chunks re-reads the column's last one): the compiler's in-order vmcnt
// accounting then waits for exactly the ring slot being consumed. (A predicated load may or may not count, so the
// compiler would wait for vmcnt(0) — every tile in flight — before each tile.)
template <int DM>
__device__ __forceinline__ void rs_issue(uint32_t rp, int64_t wt, int lane, u32x4 (&r)[DM]) {
  const int n = (int)rl(rp, 0);
  const uint64_t src0 = ((uint64_t)rl(rp, 3) << 32) | rl(rp, 2);
  const uint32_t stride0 = rl(rp, 4), lanes0 = rl(rp, 5);
#pragma unroll DM
  for (int k = 0; k < DM; ++k) {
    const bool use = k < n;  // (wave-uniform)
    const uint64_t src = use ? (((uint64_t)rl(rp, 3 + 5 * k) << 32) | rl(rp, 2 + 5 * k)) : src0;
    const uint32_t stride = use ? rl(rp, 4 + 5 * k) : stride0, lanes = use ? rl(rp, 5 + 5 * k) : lanes0;
    const uint32_t l = (uint32_t)lane < lanes ? (uint32_t)lane : lanes - 1u;
    r[k] = *(const AS1 u32x4*)(src + (uint64_t)wt * stride + 16u * l);
  }
}

template <int DM>
__device__ __forceinline__ void rs_store(uint32_t rp, uint32_t img, int lane, const u32x4 (&r)[DM]) {
  const int n = (int)rl(rp, 0);
#pragma unroll DM
  for (int k = 0; k < DM; ++k) {
    const uint32_t lanes = rl(rp, 5 + 5 * k), dst = rl(rp, 6 + 5 * k);
    if (k < n && (uint32_t)lane < lanes) *lds_at<lds_u32x4_t>(img + dst + 16u * (uint32_t)lane) = r[k];
  }
}

// issue cursor: the next tile this wave loads, its segment and that segment's GdRsPlan (one dword per lane)
struct RsCursor {
  int64_t ti;
  int si;
  int64_t first, end;
  uint32_t rp;
};

template <int DM>
__device__ __forceinline__ void rs_issue_next(CQ* q, const DevSeg* __restrict__ segs, RsCursor& c, int64_t t1, int wpw,
                                              int lane, u32x4 (&r)[DM]) {
  if (c.ti < t1) {
    while (c.ti >= c.end) {
      c.si = __builtin_amdgcn_readfirstlane(c.si + 1);
      CSegT* sg = (CSegT*)(uintptr_t)uniform_ptr(segs + c.si);
      c.first = sg->first_wtile;
      c.end = c.first + sg->num_wtiles;
      c.rp = gp(q->gd_plans)[(int64_t)c.si * kGdPlanDw + 64 + lane];
    }
    rs_issue<DM>(c.rp, c.ti - c.first, lane, r);
  }
  c.ti += wpw;
}

// process cursor: the next tile this wave walks, its segment and that segment's GdSegPlan / GdRsPlan
struct RsProc {
  int64_t t;
  int si;
  int64_t first, end;
  uint32_t gt, rp;
};

template <int RS, int DM>
struct RsRing {
  u32x4 s0[DM], s1[DM], s2[RS > 2 ? DM : 1], s3[RS > 3 ? DM : 1];
};

template <int J, int RS, int DM>
__device__ __forceinline__ u32x4 (&rs_slot(RsRing<RS, DM>& r))[DM] {
  if constexpr (J == 0) return r.s0;
  else if constexpr (J == 1) return r.s1;
  else if constexpr (J == 2) return r.s2;
  else return r.s3;
}

// One tile: issue the next load into slot `refill` (free: its tile was walked last), then walk the tile in `cur`.
template <int DM>
__device__ __forceinline__ void rs_step(CQ* q, const DevQuery* __restrict__ q_in, const DevSeg* __restrict__ segs,
                                        RsCursor& ic, RsProc& pc, int64_t t1, int wpw, int lane, uint32_t img,
                                        const uint32_t* img_ptr, uint32_t base, uint32_t& matched, uint32_t& errs,
                                        u32x4 (&refill)[DM], const u32x4 (&cur)[DM]) {
  rs_issue_next<DM>(q, segs, ic, t1, wpw, lane, refill);
  while (pc.t >= pc.end) {
    pc.si = __builtin_amdgcn_readfirstlane(pc.si + 1);
    CSegT* sg = (CSegT*)(uintptr_t)uniform_ptr(segs + pc.si);
    pc.first = sg->first_wtile;
    pc.end = pc.first + sg->num_wtiles;
    pc.gt = gp(q->gd_plans)[(int64_t)pc.si * kGdPlanDw + lane];
    pc.rp = gp(q->gd_plans)[(int64_t)pc.si * kGdPlanDw + 64 + lane];
  }
  rs_store<DM>(pc.rp, img, lane, cur);
  // (a wave-uniform segment pointer: its descriptor fields are scalar loads, which do not wait for the ring's loads)
  // (the 12-wave variant: at most 2 group-by columns and 2 value aggregations, so its tile ring fits the 170 VGPRs of
  // 3 waves per SIMD; with the general limits a ring slot spilled and each refill waited for its own load)
  matched += gd_tile_sm<4, (DM <= 4 ? kGdRs12MaxGb : kGdMaxGb), (DM <= 4 ? kGdRs12MaxAgg : kGdMaxAgg)>(
      pc.gt, q_in, uniform_ptr(segs + pc.si), pc.t - pc.first, img_ptr, img, lane, base, errs);
  pc.t += wpw;
}

template <int WPW, int RS, int DM>
__global__ void __launch_bounds__(WPW * kWave, 1) gdense_rs_kernel(const DevQuery* __restrict__ q_in,
                                                                   const DevSeg* __restrict__ segs,
                                                                   const LmSegPlan* __restrict__, PartScratch) {
  CQ* q = (CQ*)(uintptr_t)q_in;
  constexpr int WGS = WPW * kWave;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned char* lds = (unsigned char*)smem;
  const uint32_t base = lds_addr(smem);
  const int img_dw = q->image_dwords_max;
  uint32_t* const img_ptr = smem + (q->lds_acc_bytes >> 2) + wave * img_dw;
  const uint32_t img = base + q->lds_acc_bytes + 4u * (uint32_t)(wave * img_dw);
  gd_init(q, lds, tid, WGS);
  const int64_t T = q->total_wtiles, G = gridDim.x;
  const int64_t lb = q->xcd_major ? xcd_major_block(blockIdx.x, G) : (int64_t)blockIdx.x;
  const int64_t t0 = lb * T / G, t1 = (lb + 1) * T / G;
  const int nseg = q->num_segments;
  if (q->gd_tables && t0 < t1) gd_load_tables(q, (CSegT*)(uintptr_t)(segs + find_segment(segs, nseg, t0)), lds, tid, WGS);
  __syncthreads();
  uint32_t matched = 0, errs = 0;
  if (t0 < t1) {
    // issue cursor (segment, its plan) and process cursor
    int64_t ti = t0 + wave;
    int isi = find_segment(segs, nseg, t0);
    int64_t ifirst = segs[isi].first_wtile, iend = ifirst + segs[isi].num_wtiles;
    uint32_t rpi = gp(q->gd_plans)[(int64_t)isi * kGdPlanDw + 64 + lane];
    int64_t t = ti;
    int psi = isi;
    int64_t pfirst = ifirst, pend = iend;
    uint32_t gt = gp(q->gd_plans)[(int64_t)psi * kGdPlanDw + lane], rpp = rpi;
    RsRing<RS, DM> ring;
    RsCursor ic{ti, isi, ifirst, iend, rpi};
    RsProc pc{t, psi, pfirst, pend, gt, rpp};
    rs_issue_next<DM>(q, segs, ic, t1, WPW, lane, ring.s0);
    if constexpr (RS > 2) rs_issue_next<DM>(q, segs, ic, t1, WPW, lane, ring.s1);
    if constexpr (RS > 3) rs_issue_next<DM>(q, segs, ic, t1, WPW, lane, ring.s2);
    while (pc.t < t1) {
      // one tile per ring slot, every slot a compile-time register set: issue into the slot the last tile used, then
      // store this slot's tile into the wave's image and walk it
      rs_step<DM>(q, q_in, segs, ic, pc, t1, WPW, lane, img, img_ptr, base, matched, errs, rs_slot<RS - 1, RS, DM>(ring), ring.s0);
      if (pc.t >= t1) break;
      rs_step<DM>(q, q_in, segs, ic, pc, t1, WPW, lane, img, img_ptr, base, matched, errs, ring.s0, ring.s1);
      if (pc.t >= t1) break;
      if constexpr (RS > 2) {
        rs_step<DM>(q, q_in, segs, ic, pc, t1, WPW, lane, img, img_ptr, base, matched, errs, ring.s1, ring.s2);
        if (pc.t >= t1) break;
      }
      if constexpr (RS > 3) {
        rs_step<DM>(q, q_in, segs, ic, pc, t1, WPW, lane, img, img_ptr, base, matched, errs, ring.s2, ring.s3);
      }
    }
  }
  const int64_t wm = wave_sum_i64((int64_t)matched);
  const int64_t we = wave_sum_i64((int64_t)errs);
  if (lane == 0 && wm != 0) __hip_atomic_fetch_add(gp(q->matched_docs), (unsigned long long)wm, RLX);
  if (lane == 0 && we != 0) __hip_atomic_fetch_add(gp(q->matched_docs) + 3, (unsigned long long)we, RLX);
  __syncthreads();
  gd_flush(q_in, segs, lds, tid, WGS);
}

}  // namespace pa
