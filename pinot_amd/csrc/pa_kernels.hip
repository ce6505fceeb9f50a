// HIP kernels of the segment query hot path other than the scan kernel (gfx950 / CDNA4 only): numGroupsLimit trimming,
// segment-load and query-prep kernels, fetch compaction, partitioned pass C, and the launchers. The scan kernel's device
// code is pa_scan.h; its variants are instantiated in pa_scan_std.hip / pa_scan_part_a.hip / pa_scan_part_b.hip.
#include "pa_scan.h"

namespace pa {

// ---------------------------------------------------------------- numGroupsLimit: first-seen group trimming
// The reference's group-key generators hand out group ids per segment in first-seen order — docId order, and within a
// doc the order getIntRawKeys / getLongRawKeys expand multi-value keys in (DictionaryBasedGroupKeyGenerator.java:473,
// :668) — and once numGroupsLimit groups exist a new key gets INVALID_ID (IntGroupIdMap.getGroupId :992-1017,
// LongMapBasedHolder.getGroupId :629-637, NoDictionarySingleColumnGroupKeyGenerator :419): the result holders skip its
// docs in that segment (DoubleGroupByResultHolder.java:76). So a key is aggregated in segment s iff its first position
// there (doc << eb | expansion index) is among the numGroupsLimit smallest first positions of the segment's distinct
// keys. Three steps over all segments at once:
//   1. limit_first_kernel: atomicMin of the position of every (matching doc, expanded key) into a (segment, key) table;
//   2. per segment, select the L-th smallest first position by 8-bit digit passes from the top (limit_hist_kernel
//      counts the digits of the entries still in the running, limit_pick_kernel picks the digit holding the rank):
//      threshold T[s] = that position + 1;
//   3. limit_agg_kernel: the aggregation over matching docs, admitting (doc, key) iff first[s, key] < T[s].
// These are per-doc kernels (no staged tiles): this path only runs when the limit can bind.

__device__ __forceinline__ bool doc_passes(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg, int64_t doc) {
  bool ok = true, any = false;
  for (int li = 0; li < q->num_leaves; ++li) {
    const DevLeaf& L = seg->leaves[li];
    if (ok && !any) any = leaf_match_doc(L, doc);
    if (L.clause_end) {
      ok = ok && any;
      any = false;
    }
  }
  return ok;
}

// Calls f(e, key) for every group key of one doc, e = the key's index in the reference's expansion: the last group-by
// column is processed first, and a multi-value column with n values multiplies the keys so far by n with the column's
// value index as the MORE significant digit (newRawKeys[v * cur + k], getIntRawKeys), i.e. e = sum_t v_t * prod_{t'<t}
// n_t' over the MV columns taken from the last to the first.
template <class F>
__device__ __forceinline__ void for_each_key(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg, int64_t doc,
                                             F&& f) {
  int64_t base[2] = {0, 0};
  int nmv = 0;
  int mv_gb[PA_MAX_GROUP_BY];
  int32_t mv_s[PA_MAX_GROUP_BY], mv_n[PA_MAX_GROUP_BY];
  int64_t combos = 1;
  for (int j = q->num_gb - 1; j >= 0; --j) {
    const DevCol& c = seg->cols[q->gb_slot[j]];
    if (c.kind == COL_MV_DICT) {
      const int32_t s0 = gp(c.mv_off)[doc];
      mv_gb[nmv] = j;
      mv_s[nmv] = s0;
      mv_n[nmv] = gp(c.mv_off)[doc + 1] - s0;
      combos *= mv_n[nmv];
      ++nmv;
    } else {
      base[q->gb_word[j]] += (int64_t)(gb_component<true>(c, seg->remap[j], nullptr, 0, doc) * (uint64_t)q->gb_stride[j]);
    }
  }
  for (int64_t e = 0; e < combos; ++e) {
    int64_t kw[2] = {base[0], base[1]};
    int64_t rem = e;
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
    f(e, key_slot(q, kw[0], kw[1]));
  }
}

// Slot of composite key ck = accumulator slot * nseg + segment in the first-seen table (linear probing, CAS insert on
// the empty marker INT64_MAX); -1 when absent (lookup) or when the table is full (counted as an overflow).
__device__ __forceinline__ int64_t first_slot(const DevQuery* __restrict__ q, const LimitDesc& F, int64_t ck, bool insert) {
  AS1 long long* keys = gp(F.fkeys);
  int64_t h = (int64_t)(mix64((uint64_t)ck) & (uint64_t)F.fmask);
  for (int64_t probe = 0; probe <= F.fmask; ++probe) {
    long long cur = __hip_atomic_load(keys + h, RLX);
    if (cur == ck) return h;
    if (cur == INT64_MAX) {
      if (!insert) return -1;
      long long expected = INT64_MAX;
      if (__hip_atomic_compare_exchange_strong(keys + h, &expected, (long long)ck, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT) ||
          expected == ck)
        return h;
    }
    h = (h + 1) & F.fmask;
  }
  if (insert) __hip_atomic_fetch_add(gp(q->matched_docs) + 1, 1ull, RLX);
  return -1;
}

// Grid-stride over the scan's tiles (DevSeg::first_wtile), one doc per thread.
template <class F>
__device__ __forceinline__ void for_each_doc(const DevQuery* __restrict__ q, const DevSeg* __restrict__ segs, F&& f) {
  const int64_t tile_docs = (int64_t)q->steps * kWave;
  for (int64_t t = blockIdx.x; t < q->total_wtiles; t += gridDim.x) {
    const int si = find_segment(segs, q->num_segments, t);
    const DevSeg* seg = segs + si;
    const int64_t d0 = (t - seg->first_wtile) * tile_docs;
    const int64_t d1 = min(d0 + tile_docs, (int64_t)seg->num_docs);
    for (int64_t base = d0; base < d1; base += blockDim.x) f(si, seg, base + threadIdx.x, base + threadIdx.x < d1);
  }
}

__global__ void __launch_bounds__(256) limit_first_kernel(const DevQuery* __restrict__ q, const DevSeg* __restrict__ segs,
                                                          LimitDesc F) {
  const int nseg = q->num_segments;
  for_each_doc(q, segs, [&](int si, const DevSeg* seg, int64_t doc, bool valid) {
    if (!valid || !doc_passes(q, seg, doc)) return;
    for_each_key(q, seg, doc, [&](int64_t e, int64_t slot) {
      if (slot < 0) return;
      const int64_t fs = first_slot(q, F, slot * nseg + si, true);
      if (fs < 0) return;
      __hip_atomic_fetch_min(gp(F.fpos) + fs, ((unsigned long long)doc << F.eb) | (unsigned long long)e, RLX);
    });
  });
}

// Radix select of every segment's L-th smallest first position (L = numGroupsLimit; first positions are distinct within
// a segment: each belongs to one (doc, expansion) and so to one key). One digit pass per 8 bits from the top: count the
// digits of the entries whose higher digits equal the segment's prefix (per-workgroup LDS histograms when the segments'
// histograms fit, flushed with one global add per nonzero bucket), then per segment pick the digit holding the wanted
// rank. After the last pass the prefix is the L-th smallest value itself.
constexpr int kSelBuckets = 256;
constexpr int kSelLdsSegs = 48;  // LDS histograms up to this many segments (48 KiB)

__global__ void __launch_bounds__(256) limit_hist_kernel(LimitDesc F, int nseg, int shift, int first) {
  __shared__ uint32_t lh[kSelLdsSegs * kSelBuckets];
  const bool lds = nseg <= kSelLdsSegs;
  if (lds) {
    for (int i = threadIdx.x; i < nseg * kSelBuckets; i += 256) lh[i] = 0u;
    __syncthreads();
  }
  const int64_t n = F.fmask + 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const long long ck = F.fkeys[i];
    if (ck == INT64_MAX) continue;
    const int s = (int)(ck % nseg);
    const unsigned long long v = F.fpos[i];
    // (a rank < 0: the segment is out of the selection; the entries above the prefix's digits do not count)
    if (!first && (F.rank[s] < 0 || ((v ^ F.prefix[s]) >> (shift + 8)) != 0)) continue;
    const uint32_t d = (uint32_t)(v >> shift) & (kSelBuckets - 1);
    if (lds) atomicAdd(&lh[s * kSelBuckets + d], 1u);
    else __hip_atomic_fetch_add(&F.hist[(size_t)s * kSelBuckets + d], 1u, RLX);
  }
  if (lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < nseg * kSelBuckets; i += 256)
      if (lh[i]) __hip_atomic_fetch_add(&F.hist[i], lh[i], RLX);
  }
}

// One wave per segment: the digit whose cumulative count first reaches the wanted rank (the first pass also decides
// whether the segment holds L groups at all); the histogram is cleared for the next pass. Last pass: the threshold.
__global__ void __launch_bounds__(64) limit_pick_kernel(LimitDesc F, int shift, int first, int last) {
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  uint32_t* h = F.hist + (size_t)s * kSelBuckets;
  uint32_t c[kSelBuckets / 64];
  uint64_t tot = 0;
  for (int j = 0; j < kSelBuckets / 64; ++j) {  // lane owns buckets 4 lane .. 4 lane + 3
    c[j] = h[4 * lane + j];
    tot += c[j];
  }
  uint64_t incl = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const uint64_t all = __shfl(incl, 63, 64);
  long long r = first ? (long long)F.limit : F.rank[s];
  const bool active = first ? (int64_t)all >= F.limit : r >= 0;
  for (int j = 0; j < kSelBuckets / 64; ++j) h[4 * lane + j] = 0u;
  if (!active) {
    if (lane == 0 && first) F.rank[s] = -1;
    return;
  }
  uint64_t below = incl - tot;  // entries in lower buckets of this lane's first bucket
  for (int j = 0; j < kSelBuckets / 64; ++j) {
    if ((long long)below < r && (long long)(below + c[j]) >= r) {
      const unsigned long long p = (first ? 0ull : F.prefix[s]) | ((unsigned long long)(4 * lane + j) << shift);
      F.prefix[s] = p;
      F.rank[s] = r - (long long)below;
      if (last) {
        F.thresh[s] = p + 1;  // admit first positions up to and including the L-th
        __hip_atomic_fetch_add(F.reached, 1ull, RLX);  // this segment has >= numGroupsLimit groups
      }
    }
    below += c[j];
  }
}

__global__ void __launch_bounds__(256) limit_agg_kernel(const DevQuery* __restrict__ q, const DevSeg* __restrict__ segs,
                                                        LimitDesc F) {
  const Acc<STRAT_GLOBAL> acc{q, nullptr, nullptr};
  const int nseg = q->num_segments;
  const int lane = threadIdx.x & (kWave - 1);
  for_each_doc(q, segs, [&](int si, const DevSeg* seg, int64_t doc, bool valid) {
    const bool pass = valid && doc_passes(q, seg, doc);
    const uint64_t wm = __ballot(pass);
    if (lane == 0 && wm) __hip_atomic_fetch_add(gp(q->matched_docs), (unsigned long long)__builtin_popcountll(wm), RLX);
    if (!pass) return;
    const unsigned long long T = F.thresh[si];
    for_each_key(q, seg, doc, [&](int64_t e, int64_t slot) {
      if (slot < 0) return;
      const int64_t fs = first_slot(q, F, slot * nseg + si, false);
      if (fs < 0 || F.fpos[fs] >= T) return;  // INVALID_ID: the segment's group table was full at first sight
      update_doc_key<STRAT_GLOBAL, true>(q, seg, nullptr, 0, doc, slot, acc);
    });
  });
}

// ---- walk form (SV group-by columns over a direct key space of at most kWalkMaxKeys keys)
// A key is admitted in segment s iff it occurs among the segment's matching docs before the doc that brings its
// numGroupsLimit-th distinct key, i.e. iff it is in the set of keys seen in the docId prefix [0, T_s). With keys
// spread over a segment, that prefix is short (the first L distinct keys show up within ~L docs when keys are dense),
// so one workgroup per segment walks it in docId order with the key set as an LDS bitmap, instead of a first-position
// pass over every doc: rounds of kWalkRound docs mark their keys with LDS atomicOr (the old bit tells "new": the
// number of distinct new keys of a round is exact in any order); the round in which the count reaches L is undone and
// replayed in docId order (64 docs a step, each step by the wave whose registers hold its keys, duplicates inside a
// step resolved by lane order), stopping at the L-th distinct key. The bitmap is then the segment's admitted keys (admitted_docs tests it in the scan).
constexpr int kWalkThreads = 1024;
constexpr int kWalkPerThread = 8;
constexpr int kWalkRound = kWalkThreads * kWalkPerThread;
constexpr uint32_t kNoKey = 0xffffffffu;

// The keys of a thread's kWalkPerThread docs of a round (doc0 + k kWalkThreads): columns outer, docs inner, so a
// dictionary column's loads for every doc issue back to back (one HBM latency per column and per remap, not one per
// doc and column)
__device__ __forceinline__ void walk_keys(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg, int64_t doc0,
                                          uint32_t (&key)[kWalkPerThread]) {
  const int64_t nd = seg->num_docs;
  int64_t doc[kWalkPerThread];
  bool pass[kWalkPerThread];
#pragma unroll
  for (int k = 0; k < kWalkPerThread; ++k) {
    const int64_t d = doc0 + (int64_t)k * kWalkThreads;
    pass[k] = d < nd && doc_passes(q, seg, d);
    doc[k] = d < nd ? d : (nd > 0 ? nd - 1 : 0);  // (a doc past the end reads the last one's words: no key taken)
    key[k] = 0u;
  }
  for (int j = 0; j < q->num_gb; ++j) {
    const DevCol& c = seg->cols[q->gb_slot[j]];
    const int32_t* rm = seg->remap[j];
    const uint32_t stride = (uint32_t)q->gb_stride[j];
    if (c.kind == COL_SV_DICT) {
      uint32_t id[kWalkPerThread];
#pragma unroll
      for (int k = 0; k < kWalkPerThread; ++k) id[k] = decode_global(c.words, doc[k], c.nbits);
      if (rm != nullptr) {
#pragma unroll
        for (int k = 0; k < kWalkPerThread; ++k) id[k] = (uint32_t)gp(rm)[id[k]];
      }
#pragma unroll
      for (int k = 0; k < kWalkPerThread; ++k) key[k] += id[k] * stride;
    } else {
#pragma unroll
      for (int k = 0; k < kWalkPerThread; ++k)
        key[k] += (uint32_t)gb_component<true>(c, rm, nullptr, 0, doc[k]) * stride;
    }
  }
#pragma unroll
  for (int k = 0; k < kWalkPerThread; ++k)
    if (!pass[k]) key[k] = kNoKey;
}

// G: the bitmap is the segment's admit bitmap in HBM (zeroed by the host; key spaces beyond kWalkMaxWords * 32 keys),
// else an LDS copy written out at the end.
// tlog: log2 of the replay's first-lane table (LDS words after the bitmap; 0: none). A step's candidate lanes take
// atomicMin(lane) on their key's slot: a lane whose slot holds a lane with the same key knows the key's first lane (it
// or a lower one) with no compare against the other lanes; only when the slot's lane has another key (two keys in one
// slot) do the candidates compare against every candidate lane.
template <bool G>
__global__ void __launch_bounds__(kWalkThreads) limit_walk_kernel(const DevQuery* __restrict__ q,
                                                                   const DevSeg* __restrict__ segs, int64_t words,
                                                                   int tlog) {
  extern __shared__ uint32_t lds_seen[];
  __shared__ uint32_t round_new[2];  // by round parity: a round resets its counter while the last one may be read
  __shared__ int64_t relay_cnt;      // the replay's running count of distinct keys, step to step
  __shared__ int relay_done;
  const DevSeg* seg = segs + blockIdx.x;
  uint32_t* adm = (uint32_t*)seg->admit;
  if (adm == nullptr) return;  // (workgroup-uniform) the limit cannot bind in this segment
  uint32_t* seen = G ? adm : lds_seen;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  if (!G)
    for (int64_t w = tid; w < words; w += kWalkThreads) seen[w] = 0u;
  uint32_t* tab = lds_seen + (G ? 0 : words);
  for (int w = tid; w < (tlog ? 1 << tlog : 0); w += kWalkThreads) tab[w] = 0xffffffffu;
  const int64_t L = q->num_groups_limit;
  const int64_t nd = seg->num_docs;
  int64_t cnt = 0;  // distinct keys before the current round
  bool reached = false;
  __syncthreads();
  int par = 0;
  for (int64_t d0 = 0; d0 < nd && !reached; d0 += kWalkRound, par ^= 1) {
    if (tid == 0) round_new[par] = 0u;
    uint32_t key[kWalkPerThread];
    walk_keys(q, seg, d0 + tid, key);
    __syncthreads();
    uint32_t mine = 0;  // bit k: this thread's doc k brought a key new to the bitmap
#pragma unroll
    for (int k = 0; k < kWalkPerThread; ++k) {
      if (key[k] == kNoKey) continue;
      const uint32_t b = 1u << (key[k] & 31u);
      if (!(atomicOr(seen + (key[k] >> 5), b) & b)) mine |= 1u << k;
    }
    uint32_t n = (uint32_t)__builtin_popcount(mine);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) n += (uint32_t)__shfl_xor((int)n, o, kWave);
    if (lane == 0 && n) atomicAdd(&round_new[par], n);
    __syncthreads();
    const int64_t rn = round_new[par];  // workgroup-uniform
    if (cnt + rn < L) {
      cnt += rn;
      continue;
    }
    // the L-th distinct key appears in this round: undo its marks, replay it in docId order, 64 docs per step. The
    // round's keys stay in the registers that computed them (doc d0 + k * kWalkThreads + tid), so step s (docs
    // d0 + 64 s ..) is replayed by the wave holding them (wave s % waves, its key[s / waves]) and the running count
    // passes from step to step through LDS, one barrier per step (a single replaying wave re-read every key from HBM,
    // one dependent load per step)
#pragma unroll
    for (int k = 0; k < kWalkPerThread; ++k)
      if ((mine >> k) & 1u) atomicAnd(seen + (key[k] >> 5), ~(1u << (key[k] & 31u)));
    if (tid == 0) {
      relay_cnt = cnt;
      relay_done = 0;
    }
    __syncthreads();
    constexpr int kWaves = kWalkThreads / kWave;
    const int wave = tid / kWave;
    for (int st = 0; st < kWalkRound / kWave; ++st) {
      const int64_t b = d0 + (int64_t)st * kWave;
      if (b >= nd) break;  // (workgroup-uniform)
      if (wave == st % kWaves) {
        uint32_t k0 = kNoKey;
#pragma unroll
        for (int k = 0; k < kWalkPerThread; ++k)
          if (k == st / kWaves) k0 = key[k];
        const int64_t c0 = relay_cnt;
        // (an atomic load: in HBM the bitmap's lines may sit stale in this CU's L1 after the atomics at L2)
        bool cand = k0 != kNoKey &&
                    !((__hip_atomic_load(seen + (k0 >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (k0 & 31u)) & 1u);
        // a key new to the bitmap counts at its first lane only
        uint64_t cm = __ballot(cand);
        bool dup = false, unres = cand;
        if (tlog) {
          const uint32_t slot = (k0 * 0x9e3779b1u) >> (32 - tlog);
          if (cand) atomicMin(tab + slot, (uint32_t)lane);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (one wave: its LDS operations run in order)
          const uint32_t w = cand ? tab[slot] : 0u;
          const uint32_t kw = (uint32_t)__shfl((int)k0, (int)w, kWave);
          unres = cand && kw != k0;
          dup = cand && kw == k0 && w != (uint32_t)lane;
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          if (cand) tab[slot] = 0xffffffffu;
        }
        if (__ballot(unres) != 0) {
          bool d2 = false;
          while (cm) {
            const int j = __builtin_ctzll(cm);
            cm &= cm - 1;
            const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)k0, j);
            d2 |= j < lane && kj == k0;
          }
          if (unres) dup = d2;
        }
        const bool nw = cand && !dup;
        const uint64_t nm = __ballot(nw);
        const int64_t c = __builtin_popcountll(nm);
        uint64_t take = nm;
        if (c0 + c >= L) {  // keep the first L - c0 new keys of this step
          int64_t need = L - c0;
          uint64_t t = 0, r = nm;
          while (need-- > 0) {
            const uint64_t low = r & (~r + 1);
            t |= low;
            r &= r - 1;
          }
          take = t;
        }
        if ((take >> lane) & 1ull) atomicOr(seen + (k0 >> 5), 1u << (k0 & 31u));
        if (lane == 0) {
          relay_cnt = c0 + __builtin_popcountll(take);
          relay_done = c0 + __builtin_popcountll(take) >= L ? 1 : 0;
        }
      }
      __syncthreads();
      if (relay_done) break;  // (read after the barrier: workgroup-uniform)
    }
    cnt = relay_cnt;
    reached = true;
    __syncthreads();
  }
  __syncthreads();
  if (!G)
    for (int64_t w = tid; w < words; w += kWalkThreads) gp(adm)[w] = seen[w];
  if (reached && tid == 0) __hip_atomic_fetch_add(gp(q->matched_docs) + 2, 1ull, RLX);  // numGroupsLimitReached
}

// ---- walk form with one multi-value group-by column (q->gb_mv): a doc brings one key per value, in the reference's
// order (doc, then value index: getIntRawKeys with one MV column; a repeated value is not new the second time).
// Rounds as in limit_walk_kernel, each from a snapshot of the LDS bitmap; the round in which the count reaches L is
// rolled back to its snapshot and replayed by one wave, 64 keys at a time in (doc, value) order (each lane finds the
// doc of its key by a binary search over the inclusive prefix sums of the 64 docs' value counts).
__device__ __forceinline__ void walk_doc_mv(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg, int64_t doc,
                                            uint32_t& base, int32_t& v0, uint32_t& n) {
  base = 0u;
  v0 = 0;
  n = 0u;
  if (doc >= seg->num_docs || !doc_passes(q, seg, doc)) return;
  for (int j = 0; j < q->num_gb; ++j)
    if (j != q->gb_mv)
      base += (uint32_t)gb_component<true>(seg->cols[q->gb_slot[j]], seg->remap[j], nullptr, 0, doc) *
              (uint32_t)q->gb_stride[j];
  const int32_t* off = seg->cols[q->gb_slot[q->gb_mv]].mv_off;
  v0 = gp(off)[doc];
  n = (uint32_t)(gp(off)[doc + 1] - v0);
}

__device__ __forceinline__ uint32_t walk_mv_key(const DevQuery* __restrict__ q, const DevSeg* __restrict__ seg,
                                                uint32_t base, int64_t v) {
  const int j = q->gb_mv;
  const DevCol& c = seg->cols[q->gb_slot[j]];
  uint32_t id = decode_global(c.words, v, c.nbits);
  if (seg->remap[j] != nullptr) id = (uint32_t)gp(seg->remap[j])[id];
  return base + id * (uint32_t)q->gb_stride[j];
}

__global__ void __launch_bounds__(kWalkThreads) limit_walk_mv_kernel(const DevQuery* __restrict__ q,
                                                                      const DevSeg* __restrict__ segs, int64_t words,
                                                                      int tlog) {
  extern __shared__ uint32_t lds_walk[];
  __shared__ uint32_t round_new[2];
  uint32_t* seen = lds_walk;
  uint32_t* snap = lds_walk + words;
  uint32_t* tab = lds_walk + 2 * words;  // the replay's first-lane table (as limit_walk_kernel; tlog 0: none)
  const DevSeg* seg = segs + blockIdx.x;
  uint32_t* adm = (uint32_t*)seg->admit;
  if (adm == nullptr) return;  // (workgroup-uniform)
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  for (int64_t w = tid; w < words; w += kWalkThreads) seen[w] = 0u;
  for (int w = tid; w < (tlog ? 1 << tlog : 0); w += kWalkThreads) tab[w] = 0xffffffffu;
  const int64_t L = q->num_groups_limit;
  const int64_t nd = seg->num_docs;
  int64_t cnt = 0;
  bool reached = false;
  int par = 0;
  __syncthreads();
  for (int64_t d0 = 0; d0 < nd && !reached; d0 += kWalkRound, par ^= 1) {
    for (int64_t w = tid; w < words; w += kWalkThreads) snap[w] = seen[w];
    if (tid == 0) round_new[par] = 0u;
    __syncthreads();
    uint32_t nnew = 0;
    for (int k = 0; k < kWalkPerThread; ++k) {
      uint32_t base, n;
      int32_t v0;
      walk_doc_mv(q, seg, d0 + (int64_t)k * kWalkThreads + tid, base, v0, n);
      for (uint32_t e = 0; e < n; ++e) {
        const uint32_t key = walk_mv_key(q, seg, base, (int64_t)v0 + e);
        const uint32_t b = 1u << (key & 31u);
        if (!(atomicOr(seen + (key >> 5), b) & b)) ++nnew;
      }
    }
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) nnew += (uint32_t)__shfl_xor((int)nnew, o, kWave);
    if (lane == 0 && nnew) atomicAdd(&round_new[par], nnew);
    __syncthreads();
    const int64_t rn = round_new[par];  // workgroup-uniform
    if (cnt + rn < L) {
      cnt += rn;
      continue;
    }
    for (int64_t w = tid; w < words; w += kWalkThreads) seen[w] = snap[w];  // roll the round back
    __syncthreads();
    if (tid < kWave) {
      for (int64_t b = d0; b < d0 + kWalkRound && b < nd && cnt < L; b += kWave) {
        uint32_t base, n;
        int32_t v0;
        walk_doc_mv(q, seg, b + lane, base, v0, n);
        uint32_t incl = n;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const uint32_t t = __shfl_up(incl, o, kWave);
          if (lane >= o) incl += t;
        }
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
        for (uint32_t g0 = 0; g0 < total && cnt < L; g0 += kWave) {
          const uint32_t g = g0 + (uint32_t)lane;
          int ow = 0;
#pragma unroll
          for (int st = kWave / 2; st >= 1; st >>= 1) {
            const uint32_t v = (uint32_t)__shfl((int)incl, ow + st - 1, kWave);
            if (v <= g) ow += st;
          }
          ow = ow < kWave ? ow : kWave - 1;
          const uint32_t o_incl = (uint32_t)__shfl((int)incl, ow, kWave), o_n = (uint32_t)__shfl((int)n, ow, kWave);
          const uint32_t o_base = (uint32_t)__shfl((int)base, ow, kWave);
          const int32_t o_v0 = __shfl(v0, ow, kWave);
          const bool act = g < total;
          const uint32_t k0 = act ? walk_mv_key(q, seg, o_base, (int64_t)o_v0 + (g - (o_incl - o_n))) : kNoKey;
          const bool cand = act && !((seen[k0 >> 5] >> (k0 & 31u)) & 1u);
          // a key new to the bitmap counts at its first record only
          uint64_t cm = __ballot(cand);
          bool dup = false, unres = cand;
          if (tlog) {
            const uint32_t slot = (k0 * 0x9e3779b1u) >> (32 - tlog);
            if (cand) atomicMin(tab + slot, (uint32_t)lane);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            const uint32_t w = cand ? tab[slot] : 0u;
            const uint32_t kw = (uint32_t)__shfl((int)k0, (int)w, kWave);
            unres = cand && kw != k0;
            dup = cand && kw == k0 && w != (uint32_t)lane;
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            if (cand) tab[slot] = 0xffffffffu;
          }
          if (__ballot(unres) != 0) {
            bool d2 = false;
            while (cm) {
              const int j = __builtin_ctzll(cm);
              cm &= cm - 1;
              const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)k0, j);
              d2 |= j < lane && kj == k0;
            }
            if (unres) dup = d2;
          }
          const bool nw = cand && !dup;
          const uint64_t nm = __ballot(nw);
          uint64_t take = nm;
          if (cnt + __builtin_popcountll(nm) >= L) {  // keep the first L - cnt new keys of these records
            int64_t need = L - cnt;
            uint64_t t = 0, r = nm;
            while (need-- > 0) {
              t |= r & (~r + 1);
              r &= r - 1;
            }
            take = t;
          }
          if ((take >> lane) & 1ull) atomicOr(seen + (k0 >> 5), 1u << (k0 & 31u));
          cnt += __builtin_popcountll(take);
        }
      }
    }
    reached = true;
    __syncthreads();
  }
  __syncthreads();
  for (int64_t w = tid; w < words; w += kWalkThreads) gp(adm)[w] = seen[w];
  if (reached && tid == 0) __hip_atomic_fetch_add(gp(q->matched_docs) + 2, 1ull, RLX);  // numGroupsLimitReached
}

hipError_t launch_limit_walk(const DevQuery* q, const DevSeg* segs, int nseg, int64_t words, bool mv, hipStream_t s) {
  // the replay's first-lane table: up to 4096 words in what the bitmap leaves of the LDS (PA_WALK_TAB=0: none,
  // measurement)
  static const bool use_tab = [] {
    const char* e = std::getenv("PA_WALK_TAB");
    return e == nullptr || std::atoi(e) != 0;
  }();
  auto tlog_for = [&](size_t used) {
    int t = 0;
    if (use_tab)
      for (int l = 12; l >= 6 && !t; --l)
        if (used + ((size_t)4 << l) + 64 <= (size_t)kWalkMaxWords * 4 + 3840) t = l;
    return t;
  };
  if (mv) {  // (the planner keeps 2 * words within kWalkMaxWords)
    const int tl = tlog_for((size_t)words * 8);
    const size_t lds = (size_t)words * 8 + (tl ? (size_t)4 << tl : 0);
    hipError_t e = hipFuncSetAttribute((const void*)limit_walk_mv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    limit_walk_mv_kernel<<<nseg, kWalkThreads, lds, s>>>(q, segs, words, tl);
    return hipGetLastError();
  }
  if (words > kWalkMaxWords) {
    const int tl = tlog_for(0);
    hipError_t e = hipFuncSetAttribute((const void*)limit_walk_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)((size_t)4 << tl));
    if (e != hipSuccess) return e;
    limit_walk_kernel<true><<<nseg, kWalkThreads, tl ? (size_t)4 << tl : 0, s>>>(q, segs, words, tl);
    return hipGetLastError();
  }
  const int tl = tlog_for((size_t)words * 4);
  const size_t lds = (size_t)words * 4 + (tl ? (size_t)4 << tl : 0);
  hipError_t e = hipFuncSetAttribute((const void*)limit_walk_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  limit_walk_kernel<false><<<nseg, kWalkThreads, lds, s>>>(q, segs, words, tl);
  return hipGetLastError();
}

hipError_t launch_limit_passes(const DevQuery* q, const DevSeg* segs, const LimitDesc& F, int grid, int phase,
                               hipStream_t s) {
  const int64_t n = F.fmask + 1;
  const int g = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  switch (phase) {
    case 0:
      limit_first_kernel<<<grid, 256, 0, s>>>(q, segs, F);
      break;
    case 1: {
      const int nseg = F.nseg;
      const int passes = (F.pos_bits + 7) / 8;
      for (int p = 0; p < passes; ++p) {
        const int shift = 8 * (passes - 1 - p);
        limit_hist_kernel<<<g, 256, 0, s>>>(F, nseg, shift, p == 0);
        limit_pick_kernel<<<nseg, 64, 0, s>>>(F, shift, p == 0, p == passes - 1);
      }
    } break;
    case 2:
      limit_agg_kernel<<<grid, 256, 0, s>>>(q, segs, F);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- segment-load / query-prep kernels

// One filter literal over every doc of one segment -> a doc bitmap (execution statistics; pa_query_leaf_bitmaps):
// 64 docs per wave step, one ballot, two words.
__global__ void __launch_bounds__(256) leaf_bitmap_kernel(const DevSeg* __restrict__ seg, int li, int flip,
                                                          int64_t num_docs, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  for (int64_t c = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; c * kWave < num_docs; c += waves) {
    const int64_t doc = c * kWave + lane;
    const bool m = doc < num_docs && (leaf_match_doc(seg->leaves[li], doc) != (flip != 0));
    const uint64_t b = __ballot(m);
    if (lane < 2) gp(out)[2 * c + lane] = (uint32_t)(b >> (32 * lane));
  }
}

hipError_t launch_leaf_bitmap(const DevSeg* seg, int li, int flip, int64_t num_docs, uint32_t* out, hipStream_t s) {
  const int64_t steps = (num_docs + kWave - 1) / kWave;
  int64_t g = (steps + 3) / 4;
  g = g < 1 ? 1 : (g > 4096 ? 4096 : g);
  leaf_bitmap_kernel<<<(int)g, 256, 0, s>>>(seg, li, flip, num_docs, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- execution statistics over leaf bitmaps
// Doc masks A and B are postfix programs over the leaf bitmaps. Word w of a mask: 32 docs. The counts feed the closed
// forms of filter_stats.py: popcounts for the applyAnd chains and the post-filter docs, and for an AND of two scan
// iterators (AndDocIdIterator.java:39-73 leap-frogging SVScanDocIdIterator.advance, which reads from the target to the
// next match) the number of leaps. Labelled docs: A-only (1), B-only (2), both (3). In the sequence of labelled docs, a
// leap starts at an A-only doc preceded by a both-doc (or the segment start), and at every A-only / B-only doc preceded
// by the other of the two.
// Batched form (pa_query_filter_counts): one launch per kernel for every request of every segment; a workgroup finds
// its job by binary search over the jobs' first workgroup.
constexpr int kBitBlockWords = 256 * 4 * kBitGroups;  // words per workgroup: 256 threads x kBitGroups 16-byte groups

// Per-workgroup copy of the job and its programs, and an LDS operand stack per thread ([depth][thread]; a private
// array would live in scratch memory).
struct BitShared {
  BitJob J;
  int32_t tok[2 * kBitProgMax];
  uint32_t stk[kBitProgStack][256];
  uint32_t lds4[4];
  unsigned long long part[4][4];
};

__device__ __forceinline__ void bit_load_job(const BitJob* __restrict__ jobs, int j, BitShared& S) {
  if (threadIdx.x < sizeof(BitJob) / 4) ((uint32_t*)&S.J)[threadIdx.x] = gp((const uint32_t*)(jobs + j))[threadIdx.x];
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * kBitProgMax; i += blockDim.x) S.tok[i] = gp(S.J.tok)[i];
  __syncthreads();
}

// The thread's words of the job's leaves used by its programs (nu <= 4 distinct leaves, tokens renumbered to their
// positions by the host): one 16-byte load per leaf and group, every load of a group issued before any is used.
struct BitWords {
  u32x4 lw[kBitGroups][4];
};

__device__ __forceinline__ void bit_load_words(const BitShared& S, int64_t w0, BitWords& W) {
#pragma unroll
  for (int g = 0; g < kBitGroups; ++g) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      W.lw[g][p] = u32x4{0u, 0u, 0u, 0u};
      // (leaf bitmaps hold a multiple of 4 words covering num_docs: a group that starts before num_docs is in bounds)
      if (p < S.J.nu && 32 * (w0 + 4 * g) < S.J.num_docs)
        W.lw[g][p] = *(const AS1 u32x4*)(gp(S.J.bm) + (int64_t)S.J.uleaf[p] * S.J.words + w0 + 4 * g);
    }
  }
}

// word k of group g of one program's mask
__device__ __forceinline__ uint32_t bit_eval(BitShared& S, int base, int len, const BitWords& W, int g, int k,
                                             int64_t w, uint32_t valid) {
  const int t0 = threadIdx.x;
  int sp = 0;
  for (int i = 0; i < len; ++i) {
    const int t = S.tok[base + i];
    if (t >= 0) {
      uint32_t x;
      if (S.J.nu > 0) {
        x = t == 0 ? W.lw[g][0][k] : (t == 1 ? W.lw[g][1][k] : (t == 2 ? W.lw[g][2][k] : W.lw[g][3][k]));
      } else {
        x = gp(S.J.bm)[(int64_t)t * S.J.words + w];  // (more than 4 leaves: loads in program order)
      }
      S.stk[sp++][t0] = x & valid;
    } else if (t == PA_BIT_NOT) {
      S.stk[sp - 1][t0] = ~S.stk[sp - 1][t0] & valid;
    } else {
      --sp;
      const uint32_t x = S.stk[sp - 1][t0], y = S.stk[sp][t0];
      S.stk[sp - 1][t0] = t == PA_BIT_AND ? (x & y) : (x | y);
    }
  }
  return S.stk[0][t0];
}

// masks A and B of the thread's kBitGroups * 4 words (w0 ..)
__device__ __forceinline__ void bit_masks(BitShared& S, int64_t w0, uint32_t (&a)[kBitGroups * 4],
                                          uint32_t (&b)[kBitGroups * 4]) {
  BitWords W;
  bit_load_words(S, w0, W);
#pragma unroll
  for (int g = 0; g < kBitGroups; ++g) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t w = w0 + 4 * g + k;
      const int64_t left = S.J.num_docs - 32 * w;
      const uint32_t valid = left >= 32 ? 0xffffffffu : (left <= 0 ? 0u : ((1u << left) - 1u));
      a[4 * g + k] = b[4 * g + k] = 0u;
      if (valid == 0u) continue;
      a[4 * g + k] = bit_eval(S, 0, S.J.len_a, W, g, k, w, valid);
      if (S.J.len_b > 0) b[4 * g + k] = bit_eval(S, kBitProgMax, S.J.len_b, W, g, k, w, valid);
    }
  }
}

// Leaps of one word in constant time. Labelled docs L = a | b; for X a subset of L, the labelled docs whose predecessor
// within the word is in X are (~L + (X << 1)) & L: each X bit's carry runs through the unlabelled docs above it and
// stops at the next labelled doc (carries of different X bits never meet: each stops at a labelled doc first). The
// word's lowest labelled doc follows `prev` (the last label before the word); prev becomes the word's last label.
__device__ __forceinline__ uint32_t word_leaps(uint32_t a, uint32_t b, uint32_t& prev) {
  const uint32_t l = a | b;
  if (l == 0u) return 0u;
  const uint32_t a1 = a & ~b, b1 = b & ~a, c = a & b, z = ~l;
  const uint32_t after_c = (z + (c << 1)) & l, after_a = (z + (a1 << 1)) & l, after_b = (z + (b1 << 1)) & l;
  uint32_t n = (uint32_t)(__builtin_popcount(a1 & after_c) + __builtin_popcount(a1 & after_b) +
                          __builtin_popcount(b1 & after_a));
  const int p0 = __builtin_ctz(l);
  const uint32_t first = ((a >> p0) & 1u) | (((b >> p0) & 1u) << 1);
  n += ((first == 1u && prev == 3u) || (first != 3u && prev != 3u && first != prev)) ? 1u : 0u;
  const int p1 = 31 - __builtin_clz(l);
  prev = ((a >> p1) & 1u) | (((b >> p1) & 1u) << 1);
  return n;
}

// label of the highest labelled doc of a word (0: none)
__device__ __forceinline__ uint32_t last_label(uint32_t a, uint32_t b) {
  const uint32_t l = a | b;
  if (l == 0u) return 0u;
  const int p = 31 - __builtin_clz(l);
  return ((a >> p) & 1u) | (((b >> p) & 1u) << 1);
}

__device__ __forceinline__ uint32_t later_label(uint32_t x, uint32_t y) { return y != 0u ? y : x; }

// "last labelled" scan over the 256 threads of the workgroup (threads in doc order): the exclusive value per thread,
// and the workgroup's last label in *total
__device__ __forceinline__ uint32_t block_last_exclusive(uint32_t v, uint32_t* lds4, uint32_t* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)inc, o, kWave);
    if (lane >= o) inc = later_label(u, inc);
  }
  if (lane == kWave - 1) lds4[wv] = inc;
  __syncthreads();
  uint32_t before = 0u, all = 0u;
  for (int i = 0; i < 4; ++i) {
    if (i < wv) before = later_label(before, lds4[i]);
    all = later_label(all, lds4[i]);
  }
  uint32_t exc = (uint32_t)__shfl_up((int)inc, 1, kWave);
  exc = lane == 0 ? before : later_label(before, exc);
  *total = all;
  return exc;
}

constexpr int kBitThreadWords = 4 * kBitGroups;

__device__ __forceinline__ void bit_last_block(BitShared& S, int64_t blk) {
  const int64_t w0 = (blk * 256 + threadIdx.x) * kBitThreadWords;
  uint32_t a[kBitThreadWords], b[kBitThreadWords];
  bit_masks(S, w0, a, b);
  uint32_t last = 0u;
#pragma unroll
  for (int k = 0; k < kBitThreadWords; ++k) last = later_label(last, last_label(a[k], b[k]));
  uint32_t total;
  block_last_exclusive(last, S.lds4, &total);
  if (threadIdx.x == 0) gp(S.J.scratch)[blk] = total;
}

// 1024 threads: block_in[i] = last label of the job's workgroups < i, or 3 (segment start) when none
__device__ __forceinline__ void bit_carry_block(const BitJob& J, uint32_t* part) {
  const uint32_t* block_last = J.scratch;
  uint32_t* block_in = J.scratch + J.nb;
  const int t = threadIdx.x;
  const int64_t per = (J.nb + 1023) / 1024;
  const int64_t b0 = t * per, b1 = b0 + per < J.nb ? b0 + per : J.nb;
  uint32_t v = 0u;
  for (int64_t i = b0; i < b1; ++i) v = later_label(v, gp(block_last)[i]);
  part[t] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t u = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] = later_label(u, part[t]);
    __syncthreads();
  }
  uint32_t run = t > 0 ? part[t - 1] : 0u;
  for (int64_t i = b0; i < b1; ++i) {
    gp(block_in)[i] = run != 0u ? run : 3u;
    run = later_label(run, gp(block_last)[i]);
  }
}

__device__ __forceinline__ void bit_count_block(BitShared& S, int64_t blk) {
  const int64_t w0 = (blk * 256 + threadIdx.x) * kBitThreadWords;
  uint32_t a[kBitThreadWords], b[kBitThreadWords];
  bit_masks(S, w0, a, b);
  uint32_t last = 0u;
  unsigned long long pa = 0, pb = 0, pab = 0, leaps = 0;
#pragma unroll
  for (int k = 0; k < kBitThreadWords; ++k) {
    last = later_label(last, last_label(a[k], b[k]));
    pa += __builtin_popcount(a[k]);
    pb += __builtin_popcount(b[k]);
    pab += __builtin_popcount(a[k] & b[k]);
  }
  if (S.J.len_b > 0) {
    uint32_t total;
    uint32_t prev = block_last_exclusive(last, S.lds4, &total);
    if (prev == 0u) prev = gp(S.J.scratch + S.J.nb)[blk];
#pragma unroll
    for (int k = 0; k < kBitThreadWords; ++k) leaps += word_leaps(a[k], b[k], prev);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pa += __shfl_xor(pa, o, kWave);
    pb += __shfl_xor(pb, o, kWave);
    pab += __shfl_xor(pab, o, kWave);
    leaps += __shfl_xor(leaps, o, kWave);
  }
  // the workgroup's four counts into its partial slot (summed per job by bit_sum_batch_kernel: no atomics on one
  // address from every workgroup)
  if ((threadIdx.x & 63) == 0) {
    const int wv = threadIdx.x >> 6;
    S.part[wv][0] = pa;
    S.part[wv][1] = pb;
    S.part[wv][2] = pab;
    S.part[wv][3] = leaps;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int f = threadIdx.x;
    gp(S.J.part)[4 * blk + f] = S.part[0][f] + S.part[1][f] + S.part[2][f] + S.part[3][f];
  }
}

// 1024 threads per job: out[f] = sum over the job's workgroups of part[4 * blk + f]
__global__ void __launch_bounds__(1024) bit_sum_batch_kernel(const BitJob* __restrict__ jobs) {
  __shared__ unsigned long long red[16][4];
  const BitJob& J = jobs[blockIdx.x];
  unsigned long long v[4] = {0, 0, 0, 0};
  for (int64_t b = threadIdx.x; b < J.nb; b += 1024)
    for (int f = 0; f < 4; ++f) v[f] += gp(J.part)[4 * b + f];
  for (int f = 0; f < 4; ++f)
    for (int o = 32; o > 0; o >>= 1) v[f] += __shfl_xor(v[f], o, kWave);
  if ((threadIdx.x & 63) == 0)
    for (int f = 0; f < 4; ++f) red[threadIdx.x >> 6][f] = v[f];
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long t = 0;
    for (int w = 0; w < 16; ++w) t += red[w][threadIdx.x];
    gp(J.out)[threadIdx.x] += t;  // (the caller zeroes out; pa_bitmap_counts adds)
  }
}

// block -> job tables (one workgroup per job writes its range)
__global__ void __launch_bounds__(256) bit_block_table_kernel(const BitJob* __restrict__ jobs,
                                                              int32_t* __restrict__ table) {
  const BitJob& J = jobs[blockIdx.x];
  for (int64_t b = threadIdx.x; b < J.nb; b += blockDim.x) gp(table)[J.first_block + b] = (int32_t)blockIdx.x;
}

__global__ void __launch_bounds__(256) bit_last_batch_kernel(const BitJob* __restrict__ jobs,
                                                             const int32_t* __restrict__ table) {
  __shared__ BitShared S;
  bit_load_job(jobs, gp(table)[blockIdx.x], S);
  if (S.J.len_b > 0) bit_last_block(S, blockIdx.x - S.J.first_block);
}

__global__ void __launch_bounds__(1024) bit_carry_batch_kernel(const BitJob* __restrict__ jobs) {
  __shared__ uint32_t part[1024];
  const BitJob& J = jobs[blockIdx.x];
  if (J.len_b > 0 && J.nb > 0) bit_carry_block(J, part);
}

__global__ void __launch_bounds__(256) bit_count_batch_kernel(const BitJob* __restrict__ jobs,
                                                              const int32_t* __restrict__ table) {
  __shared__ BitShared S;
  bit_load_job(jobs, gp(table)[blockIdx.x], S);
  bit_count_block(S, blockIdx.x - S.J.first_block);
}

int64_t bit_count_blocks(int64_t num_docs) { return ((num_docs + 31) / 32 + kBitBlockWords - 1) / kBitBlockWords; }

// per workgroup: block_last, block_in (u32) and the four partial counts (u64)
int64_t bit_count_scratch_words(int64_t words) { return 10 * ((words + kBitBlockWords - 1) / kBitBlockWords); }

hipError_t launch_bit_counts_batch(const BitJob* jobs, int nj, int64_t total_blocks, bool any_b, int32_t* table,
                                   hipStream_t s) {
  if (nj == 0 || total_blocks == 0) return hipSuccess;
  if (total_blocks > INT32_MAX) return hipErrorInvalidValue;
  bit_block_table_kernel<<<nj, 256, 0, s>>>(jobs, table);
  if (any_b) {
    bit_last_batch_kernel<<<(int)total_blocks, 256, 0, s>>>(jobs, table);
    bit_carry_batch_kernel<<<nj, 1024, 0, s>>>(jobs);
  }
  bit_count_batch_kernel<<<(int)total_blocks, 256, 0, s>>>(jobs, table);
  bit_sum_batch_kernel<<<nj, 1024, 0, s>>>(jobs);
  return hipGetLastError();
}

// Leaf bitmaps of many (segment, leaf) pairs in one launch: job j covers wave steps [first_step, first_step + steps)
// of its segment (64 docs per step, one ballot, two words), as leaf_bitmap_kernel.
constexpr int kLeafStepsPerWave = 128;  // wave steps (64 docs) per wave
constexpr int kLeafBatch = 16;         // steps whose loads are in flight together

// kLeafBatch wave steps from s0 of one leaf: every load of the batch issued before any is used
__device__ __forceinline__ void leaf_bitmap_batch(const DevLeaf& L, int64_t n, int flip, uint32_t* out, int64_t s0,
                                                  int lane) {
  if (s0 * kWave >= n) return;
  if (L.kind == PA_LEAF_DICT_RANGE || L.kind == PA_LEAF_DICT_SET) {
    // (forward indexes are padded to whole wave tiles: the decodes past num_docs stay in bounds)
    uint32_t id[kLeafBatch];
#pragma unroll
    for (int k = 0; k < kLeafBatch; ++k) id[k] = decode_global(L.words, (s0 + k) * kWave + lane, L.nbits);
    bool m[kLeafBatch];
    if (L.kind == PA_LEAF_DICT_RANGE) {
      const int sh = 32 - L.nbits;
      const uint32_t lo = (uint32_t)L.lo >> sh;
      const uint32_t span = (uint32_t)(((uint64_t)(uint32_t)L.span + 1u) >> sh);
#pragma unroll
      for (int k = 0; k < kLeafBatch; ++k) m[k] = (id[k] - lo) < span;
    } else {
#pragma unroll
      for (int k = 0; k < kLeafBatch; ++k) m[k] = (gp(L.lut)[id[k] >> 5] >> (id[k] & 31u)) & 1u;
    }
#pragma unroll
    for (int k = 0; k < kLeafBatch; ++k) {
      const int64_t st = s0 + k;
      const int64_t doc = st * kWave + lane;
      const uint64_t b = __ballot(doc < n && (m[k] != ((L.negate != 0) != (flip != 0))));
      if (st * kWave < n && lane < 2) gp(out)[2 * st + lane] = (uint32_t)(b >> (32 * lane));
    }
    return;
  }
  for (int k = 0; k < kLeafBatch; ++k) {
    const int64_t st = s0 + k;
    const int64_t doc = st * kWave + lane;
    if (st * kWave >= n) break;
    const bool m = doc < n && (leaf_match_doc(L, doc) != (flip != 0));
    const uint64_t b = __ballot(m);
    if (lane < 2) gp(out)[2 * st + lane] = (uint32_t)(b >> (32 * lane));
  }
}


// Single-value dictionary leaves, lane-major: a wave takes a whole wave tile (2048 docs), lane l docs [32l, 32l + 32),
// which are exactly the lane's nb stream words (the same layout the scan stages): the tile's 64 * nb words arrive as
// coalesced 16-byte loads into the wave's LDS region, and leaf_lm decodes the lane's 32 docs into one bitmap word.
constexpr int kLeafTilesPerWave = 4;

__device__ __forceinline__ void leaf_bitmap_tiles_lm(const DevLeaf& L, int64_t n, int flip, uint32_t* out,
                                                     int64_t t0, int lane, uint32_t* region) {
  const int nb = L.nbits;
  const uint32_t region_lds = lds_addr(region);
  for (int64_t t = t0; t < t0 + kLeafTilesPerWave; ++t) {
    const int64_t base = t * kWTileDocs;
    if (base >= n) return;
    const AS1 u32x4* src = (const AS1 u32x4*)(gp(L.words) + t * (int64_t)(kWave * nb));
    for (int c = lane; c < 16 * nb; c += kWave) ((lds_u32x4_t*)lds_ptr(region))[c] = src[c];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the region written before the decode reads it
    uint32_t bits = leaf_lm_any(nb, L.kind, region_lds, lane, (uint32_t)L.lo, (uint32_t)L.span, L.lut);
    if ((L.negate != 0) != (flip != 0)) bits = ~bits;
    const int64_t left = n - (base + 32 * lane);
    bits &= left >= 32 ? 0xffffffffu : (left <= 0 ? 0u : ((1u << left) - 1u));
    // (a leaf's bitmap holds (n + 127) / 128 * 4 words, not whole tiles: the next leaf's bitmap follows it)
    if (t * kWave + lane < (n + 127) / 128 * 4) gp(out)[t * kWave + lane] = bits;
    asm volatile("" ::: "memory");  // (this tile's reads before the next tile's writes)
  }
}

__global__ void __launch_bounds__(256) leaf_bitmaps_batch_kernel(const LeafJob* __restrict__ jobs, int nj) {
  __shared__ LeafJob SJ;
  __shared__ DevLeaf SL;
  __shared__ u32x4 regions[4][kWave * 32 / 4];  // one wave tile of a <= 32-bit column per wave
  if (threadIdx.x == 0) {
    int lo = 0, hi = nj - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].first_block <= (int64_t)blockIdx.x) lo = mid;
      else hi = mid - 1;
    }
    SJ = jobs[lo];
  }
  __syncthreads();
  if (threadIdx.x < sizeof(DevLeaf) / 4)
    ((uint32_t*)&SL)[threadIdx.x] = gp((const uint32_t*)&SJ.seg->leaves[SJ.li])[threadIdx.x];
  __syncthreads();
  const DevLeaf L = SL;  // (registers)
  const int64_t n = SJ.num_docs;
  uint32_t* out = SJ.out;
  const int flip = SJ.flip;
  const int lane = threadIdx.x & 63;
  const int64_t blk = (int64_t)blockIdx.x - SJ.first_block;
  if (L.kind == PA_LEAF_DICT_RANGE || L.kind == PA_LEAF_DICT_SET) {
    leaf_bitmap_tiles_lm(L, n, flip, out, (blk * 4 + (threadIdx.x >> 6)) * kLeafTilesPerWave, lane,
                         (uint32_t*)regions[threadIdx.x >> 6]);
    return;
  }
  // MV and raw leaves: per doc (leaf_match_doc), 64 docs per step
  const int64_t sw = (blk * 4 + (threadIdx.x >> 6)) * kLeafStepsPerWave;
  for (int64_t s0 = sw; s0 < sw + kLeafStepsPerWave; s0 += kLeafBatch) leaf_bitmap_batch(L, n, flip, out, s0, lane);
}

static_assert(kLeafStepsPerWave * kWave == kLeafTilesPerWave * kWTileDocs, "one work split for both leaf paths");

int64_t leaf_bitmap_blocks(int64_t num_docs) {
  return ((num_docs + kWave - 1) / kWave + 4 * kLeafStepsPerWave - 1) / (4 * kLeafStepsPerWave);
}

hipError_t launch_leaf_bitmaps_batch(const LeafJob* jobs, int nj, int64_t total_blocks, hipStream_t s) {
  if (nj == 0 || total_blocks == 0) return hipSuccess;
  if (total_blocks > INT32_MAX) return hipErrorInvalidValue;
  leaf_bitmaps_batch_kernel<<<(int)total_blocks, 256, 0, s>>>(jobs, nj);
  return hipGetLastError();
}

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


// ---------------------------------------------------------------- fetch: ordered compaction of non-empty keys
// Block b covers keys [2048b, 2048b + 2048): thread t owns keys 8t .. 8t+7 of it.
constexpr int kCompactKeys = 2048;

__device__ __forceinline__ uint32_t block_exclusive_scan_256(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t add = t >= o ? sh[t - o] : 0u;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const uint32_t incl = sh[t];
  if (total) *total = sh[255];
  __syncthreads();
  return incl - v;
}

__global__ void __launch_bounds__(256) compact_count_kernel(const unsigned long long* count, int64_t K, int all,
                                                            uint32_t* block_sums) {
  __shared__ uint32_t sh[256];
  const int64_t k0 = (int64_t)blockIdx.x * kCompactKeys + 8 * threadIdx.x;
  uint32_t c = 0;
  for (int j = 0; j < 8; ++j) c += (k0 + j < K) && (all || count[k0 + j] != 0);
  uint32_t total;
  block_exclusive_scan_256(c, sh, &total);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

// single workgroup: in-place exclusive scan of n block sums; v[n] = total
__global__ void __launch_bounds__(256) compact_scan_kernel(uint32_t* v, int64_t n) {
  __shared__ uint32_t sh[256];
  uint32_t carry = 0;
  for (int64_t base = 0; base < n; base += 256) {
    const int64_t i = base + threadIdx.x;
    const uint32_t x = i < n ? v[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan_256(x, sh, &tot);
    if (i < n) v[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) v[n] = carry;
}

__global__ void __launch_bounds__(256) compact_gather_kernel(const unsigned long long* count, int64_t K, int all,
                                                             const uint32_t* block_off, int64_t cap,
                                                             CompactDesc d) {
  __shared__ uint32_t sh[256];
  const int64_t k0 = (int64_t)blockIdx.x * kCompactKeys + 8 * threadIdx.x;
  uint32_t c = 0;
  for (int j = 0; j < 8; ++j) c += (k0 + j < K) && (all || count[k0 + j] != 0);
  int64_t pos = (int64_t)block_off[blockIdx.x] + block_exclusive_scan_256(c, sh, nullptr);
  for (int j = 0; j < 8; ++j) {
    const int64_t k = k0 + j;
    if (k >= K || !(all || count[k] != 0)) continue;
    if (pos < cap) {
      d.keys[pos] = k;
      for (int si = 0; si < d.nsec; ++si) {
        const int64_t per = d.per[si];
        if (d.es[si] == 8) {
          const uint64_t* src = (const uint64_t*)d.src[si] + k * per;
          uint64_t* dst = (uint64_t*)d.dst[si] + pos * per;
          for (int64_t e = 0; e < per; ++e) dst[e] = src[e];
        } else if (d.es[si] == 1) {  // HLL registers, one byte each (per is a power of two >= 16)
          const u32x4* src = (const u32x4*)((const uint8_t*)d.src[si] + k * per);
          u32x4* dst = (u32x4*)((uint8_t*)d.dst[si] + pos * per);
          for (int64_t e = 0; e < per / 16; ++e) dst[e] = src[e];
        } else {
          const uint32_t* src = (const uint32_t*)d.src[si] + k * per;
          uint32_t* dst = (uint32_t*)d.dst[si] + pos * per;
          for (int64_t e = 0; e < per; ++e) dst[e] = src[e];
        }
      }
    }
    ++pos;
  }
}

// Correctly rounded (nearest, ties to even) double of the signed 128-bit integer hi:lo — the host's (double)__int128 of
// an exact 96-bit SUM (PA_ACC_SUM_I64X2), an int64 SUM or an integer MIN / MAX, computed with integer operations only.
__device__ double i128_to_double(int64_t hi, uint64_t lo) {
  const bool neg = hi < 0;
  uint64_t mh = (uint64_t)hi, ml = lo;
  if (neg) {
    ml = ~ml + 1ull;
    mh = ~mh + (ml == 0 ? 1ull : 0ull);
  }
  if (mh == 0 && ml < (1ull << 53)) return neg ? -(double)ml : (double)ml;  // (exact)
  const int msb = mh ? 127 - __builtin_clzll(mh) : 63 - __builtin_clzll(ml);
  const int s = msb - 52;  // bits below the 53-bit significand (>= 1 here)
  auto bit = [&](int i) -> uint64_t { return i >= 64 ? (mh >> (i - 64)) & 1ull : (ml >> i) & 1ull; };
  uint64_t sig = s >= 64 ? mh >> (s - 64) : ((ml >> s) | (mh << (64 - s)));
  sig &= (1ull << 53) - 1ull;
  sig |= 1ull << 52;  // (the leading bit; the masks above keep exactly 53 bits)
  const uint64_t half = bit(s - 1);
  bool sticky;
  const int t = s - 1;  // bits [0, t) below the half bit
  if (t <= 0) sticky = false;
  else if (t >= 64) sticky = ml != 0 || (t > 64 && (mh & ((1ull << (t - 64)) - 1ull)) != 0);
  else sticky = (ml & ((1ull << t) - 1ull)) != 0;
  int e = s;
  if (half && (sticky || (sig & 1ull))) {
    ++sig;
    if (sig == (1ull << 53)) {
      sig >>= 1;
      ++e;
    }
  }
  const double d = ldexp((double)sig, e);
  return neg ? -d : d;
}

// Block b covers keys [2048b, 2048b + 2048) as in compact_gather_kernel; positions first (thread t counts keys 8t..8t+7,
// scans, and records each key's position in LDS), then thread t writes the rows of keys t + 256 j: consecutive threads,
// consecutive rows, 8-byte columns stored as 512-byte wave bursts.
__global__ void __launch_bounds__(256) compact_final_kernel(const unsigned long long* count, int64_t K, int all,
                                                            const uint32_t* block_off, int64_t cap, FinalDesc d) {
  __shared__ uint32_t sh[256];
  __shared__ uint32_t pos[kCompactKeys];
  const int64_t kb = (int64_t)blockIdx.x * kCompactKeys;
  const int64_t k0 = kb + 8 * threadIdx.x;
  uint32_t c = 0;
  for (int j = 0; j < 8; ++j) c += (k0 + j < K) && (all || count[k0 + j] != 0);
  uint32_t p = block_exclusive_scan_256(c, sh, nullptr);
  for (int j = 0; j < 8; ++j) {
    const bool on = (k0 + j < K) && (all || count[k0 + j] != 0);
    pos[8 * threadIdx.x + j] = on ? p : 0xffffffffu;
    p += on ? 1u : 0u;
  }
  __syncthreads();
  const int64_t base = block_off[blockIdx.x];
  for (int j = 0; j < kCompactKeys / 256; ++j) {
    const int kl = threadIdx.x + 256 * j;
    const uint32_t pl = pos[kl];
    if (pl == 0xffffffffu) continue;
    const int64_t r = base + pl;
    if (r >= cap) continue;
    const int64_t k = kb + kl;
    const unsigned long long cnt = count[k];
    d.keys[r] = k;
    d.counts[r] = (int64_t)cnt;
    for (int a = 0; a < d.nagg; ++a) {
      const int t = d.type[a];
      if (t == PA_AGG_DISTINCTCOUNTHLL || t == PA_AGG_DISTINCTCOUNT) {
        const int64_t per = d.per[a];  // (a multiple of 16 bytes)
        const u32x4* src = (const u32x4*)((const uint8_t*)d.sec[a] + k * per);
        u32x4* dst = (u32x4*)((uint8_t*)d.out[a] + r * per);
        for (int64_t e = 0; e < per / 16; ++e) dst[e] = src[e];
        continue;
      }
      double v;
      if (t == PA_AGG_COUNT) {
        v = (double)cnt;
      } else if (t == PA_AGG_SUM || t == PA_AGG_COUNT_MV) {
        const int64_t* sv = (const int64_t*)d.sec[a];
        if (d.src[a] == SRC_LONG) {  // exact 96-bit total hi * 2^32 + lo, rounded once
          const int64_t hs = sv[2 * k + 1];
          const uint64_t ls = (uint64_t)sv[2 * k];
          const uint64_t l0 = (uint64_t)hs << 32;
          const uint64_t lo = l0 + ls;
          v = i128_to_double((hs >> 32) + (lo < l0 ? 1 : 0), lo);
        } else if (d.src[a] == SRC_INT || t == PA_AGG_COUNT_MV) {
          v = i128_to_double(sv[k] >> 63, (uint64_t)sv[k]);
        } else {
          v = ((const double*)d.sec[a])[k];
        }
      } else {  // MIN / MAX (an empty aggregation-only result: +/-inf, Min/MaxAggregationFunction DEFAULT_VALUE)
        const int64_t e8 = ((const int64_t*)d.sec[a])[k];
        if (cnt == 0) v = t == PA_AGG_MIN ? __builtin_inf() : -__builtin_inf();
        else v = d.src[a] != SRC_DOUBLE ? i128_to_double(e8 >> 63, (uint64_t)e8) : f64_order_decode(e8);
      }
      ((double*)d.out[a])[r] = v;
    }
  }
}

hipError_t launch_compact_final(const unsigned long long* count, int64_t K, int all, const uint32_t* block_off,
                                int64_t cap, const FinalDesc* d, hipStream_t s) {
  const int64_t nb = (K + kCompactKeys - 1) / kCompactKeys;
  compact_final_kernel<<<(unsigned)nb, 256, 0, s>>>(count, K, all, block_off, cap, *d);
  return hipGetLastError();
}

hipError_t launch_compact(const unsigned long long* count, int64_t K, int all, uint32_t* block_sums, int64_t cap,
                          const CompactDesc* d, int phase, hipStream_t s) {
  const int64_t nb = (K + kCompactKeys - 1) / kCompactKeys;
  if (phase == 0) {
    compact_count_kernel<<<(unsigned)nb, 256, 0, s>>>(count, K, all, block_sums);
    compact_scan_kernel<<<1, 256, 0, s>>>(block_sums, nb);
  } else {
    compact_gather_kernel<<<(unsigned)nb, 256, 0, s>>>(count, K, all, block_sums, cap, *d);
  }
  return hipGetLastError();
}


// ---------------------------------------------------------------- partitioned aggregation: offsets + pass C
__device__ __forceinline__ uint64_t block_exclusive_scan_256_u64(uint64_t v, uint64_t* sh, uint64_t* total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint64_t add = t >= o ? sh[t - o] : 0ull;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const uint64_t incl = sh[t];
  if (total) *total = sh[255];
  __syncthreads();
  return incl - v;
}

// Block p: exclusive scan over the G emit workgroups of partition p's record counts, each rounded up to whole bins of
// the partition's stream (-> off[wg][p], relative to the partition); the padded total -> the partition's base slot.
// The count pass ran k workgroups per emit workgroup (more resident waves: it stages fewer columns): emit workgroup wg
// walked exactly the tiles of count workgroups [wg*k, wg*k + k) (both split the tiles by the same formula), so its
// counts are the sum of those k rows, stored back into row wg (rows wg*k.. are read before any row is written: the
// scan's barriers separate them, and a later chunk of 256 reads only rows >= its own first row * k).
__global__ void __launch_bounds__(256) part_scan_kernel(uint32_t* hist, uint32_t* off, int G, int k, int P, int pv,
                                                        uint32_t bs_v, uint32_t bs_h, uint64_t* base) {
  __shared__ uint64_t sh[256];
  const int p = blockIdx.x;
  const uint32_t bs = p < pv ? bs_v : bs_h;
  uint64_t carry = 0;
  for (int b0 = 0; b0 < G; b0 += 256) {
    const int wg = b0 + threadIdx.x;
    uint32_t n = 0;
    if (wg < G)
      for (int j = 0; j < k; ++j) n += hist[((size_t)wg * k + j) * P + p];
    const uint64_t x = (uint64_t)((n + bs - 1u) / bs * bs);
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan_256_u64(x, sh, &tot);
    if (wg < G) {
      off[(size_t)wg * P + p] = (uint32_t)(carry + ex);
      if (k > 1) hist[(size_t)wg * P + p] = n;
    }
    carry += tot;
  }
  if (threadIdx.x == 0) base[p < pv ? p : p + 1] = carry;
}

// single workgroup: in-place exclusive scan of n 64-bit counts; v[n] = total
__global__ void __launch_bounds__(256) scan_u64_kernel(uint64_t* v, int64_t n) {
  __shared__ uint64_t sh[256];
  uint64_t carry = 0;
  for (int64_t b0 = 0; b0 < n; b0 += 256) {
    const int64_t i = b0 + threadIdx.x;
    const uint64_t x = i < n ? v[i] : 0ull;
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan_256_u64(x, sh, &tot);
    if (i < n) v[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) v[n] = carry;
}

// Pass C. One workgroup per partition: V partitions aggregate COUNT/SUM/MIN/MAX of their key range in LDS, H
// partitions the u8 HLL registers (and COUNT from first-value flags when there is no V stream); either way the
// workgroup owns its keys and stores every accumulator of its range (empty keys get the identities), so no global
// atomics and no read of the accumulators.
constexpr int kPartAggThreads = 512;

// one aggregation update of local key lk with the value bits iv (int64, or double bits)
__device__ __forceinline__ void part_apply(const DevAgg& A, unsigned char* lds, int64_t lk, int64_t iv) {
  if (A.type == PA_AGG_SUM) {
    if (A.src == SRC_INT) {
      atomicAdd((unsigned long long*)(lds + A.lds_off) + lk, (unsigned long long)iv);
    } else if (A.src == SRC_LONG) {
      atomicAdd((unsigned long long*)(lds + A.lds_off) + 2 * lk, (unsigned long long)(uint32_t)iv);
      atomicAdd((unsigned long long*)(lds + A.lds_off) + 2 * lk + 1, (unsigned long long)(iv >> 32));
    } else {
      atomicAdd((double*)(lds + A.lds_off) + lk, __builtin_bit_cast(double, iv));
    }
  } else {
    const int64_t e = A.src != SRC_DOUBLE ? iv : f64_order_encode(__builtin_bit_cast(double, iv));
    if (A.type == PA_AGG_MIN) atomicMin((long long*)(lds + A.lds_off) + lk, (long long)e);
    else atomicMax((long long*)(lds + A.lds_off) + lk, (long long)e);
  }
}

__device__ void part_agg_v(const DevQuery* __restrict__ q, const PartScratch& ps, int p, unsigned char* lds) {
  const int ks = q->kshift_v;
  const int64_t KR = int64_t(1) << ks;
  const int64_t kbase = (int64_t)p << ks;
  const int64_t nk = min(KR, q->num_keys - kbase);
  uint32_t* cnt = (uint32_t*)lds;
  for (int64_t k = threadIdx.x; k < KR; k += kPartAggThreads) cnt[k] = 0;
  for (int a = 0; a < q->num_aggs; ++a) {
    const DevAgg& A = q->aggs[a];
    if (A.type == PA_AGG_COUNT || A.type == PA_AGG_DISTINCTCOUNTHLL) continue;  // (HLL: the H partitions)
    int64_t* r = (int64_t*)(lds + A.lds_off);
    const int64_t init = A.type == PA_AGG_MIN ? INT64_MAX : (A.type == PA_AGG_MAX ? INT64_MIN : 0);
    const int64_t n = (A.type == PA_AGG_SUM && A.src == SRC_LONG) ? 2 * KR : KR;
    for (int64_t k = threadIdx.x; k < n; k += kPartAggThreads) r[k] = init;
  }
  __syncthreads();
  const uint64_t r0 = gp(ps.base)[p], r1 = gp(ps.base)[p + 1];
  const int W = q->rec_words_v;
  const int fmt = q->v_fmt;
  const uint32_t kmask = (1u << ks) - 1u;  // (the key offset's bits: KR need not be a power of two)
  const AS1 uint32_t* recs = gp((const uint32_t*)ps.recs_v);
  const AS1 uint64_t* vdict = gp(q->vdict);
  // 8 records per thread in flight: every load of the batch first, then the LDS updates
  constexpr int kB = 8;
  const uint64_t span = (uint64_t)kB * kPartAggThreads;
  for (uint64_t b0 = r0; b0 < r1; b0 += span) {
    uint32_t w0[kB], w1[kB], w2[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const uint64_t ri = b0 + (uint64_t)j * kPartAggThreads + threadIdx.x;
      w0[j] = kSentinel;
      w1[j] = w2[j] = 0u;
      if (ri < r1) {
        // (contiguous partition ranges only: the count-free emit's chunk lists feed the specialised variants, never this
        // one — pve_plan refuses kVkGeneric, so ps.chunk_index is null here)
        const AS1 uint32_t* rec = recs + ri * (uint64_t)W;
        w0[j] = __builtin_nontemporal_load(rec);
        if (fmt == V_FMT_32 || fmt == V_FMT_64) w1[j] = __builtin_nontemporal_load(rec + 1);
        if (fmt == V_FMT_64) w2[j] = __builtin_nontemporal_load(rec + 2);
      }
    }
    int64_t iv[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {  // V_FMT_ID: the table-wide value of the record's value id (L2-resident dictionary)
      iv[j] = 0;
      if (w0[j] == kSentinel) continue;
      if (fmt == V_FMT_ID) iv[j] = (int64_t)vdict[w0[j] >> ks];
      else if (fmt == V_FMT_32) iv[j] = (int64_t)(int32_t)w1[j];
      else if (fmt == V_FMT_64) iv[j] = (int64_t)(((uint64_t)w2[j] << 32) | w1[j]);
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      if (w0[j] == kSentinel) continue;
      const int64_t lk = (int64_t)(w0[j] & kmask);
      atomicAdd(cnt + lk, 1u);
      if (fmt == V_FMT_KEY) continue;
      if (fmt == V_FMT_GEN) {
        const uint64_t ri = b0 + (uint64_t)j * kPartAggThreads + threadIdx.x;
        const AS1 uint32_t* rec = recs + ri * (uint64_t)W;
        for (int a = 0; a < q->num_aggs; ++a) {
          const DevAgg& A = q->aggs[a];
          if (A.type == PA_AGG_COUNT || A.type == PA_AGG_DISTINCTCOUNTHLL) continue;
          const int64_t v = A.src == SRC_INT ? (int64_t)(int32_t)rec[A.pay_off]
                                             : (int64_t)(((uint64_t)rec[A.pay_off + 1] << 32) | rec[A.pay_off]);
          part_apply(A, lds, lk, v);
        }
      } else {
        for (int a = 0; a < q->num_aggs; ++a) {
          const DevAgg& A = q->aggs[a];
          if (A.type == PA_AGG_COUNT || A.type == PA_AGG_DISTINCTCOUNTHLL) continue;
          part_apply(A, lds, lk, iv[j]);
        }
      }
    }
  }
  __syncthreads();
  // this workgroup owns keys [kbase, kbase + nk): plain stores of every accumulator
  for (int64_t lk = threadIdx.x; lk < nk; lk += kPartAggThreads) {
    const int64_t k = kbase + lk;
    gp(q->count)[k] = cnt[lk];
    for (int a = 0; a < q->num_aggs; ++a) {
      const DevAgg& A = q->aggs[a];
      if (A.type == PA_AGG_COUNT || A.type == PA_AGG_DISTINCTCOUNTHLL) continue;
      const int64_t* r = (const int64_t*)(lds + A.lds_off);
      if (A.type == PA_AGG_SUM && A.src == SRC_LONG) {
        gp(A.acc_i64)[2 * k] = r[2 * lk];
        gp(A.acc_i64)[2 * k + 1] = r[2 * lk + 1];
      } else {
        gp(A.acc_i64)[k] = r[lk];  // SUM(int) / SUM(double) bits / MIN / MAX
      }
    }
  }
}

// Specialised V pass C (VK = vk_code): one payload per record, at most one SUM / MIN / MAX; every descriptor field is
// read once into registers, the record loop is straight-line. V_FMT_ID records with value ids in value order keep
// MIN/MAX as 32-bit ids (the value is looked up once per key at the store), so the per-record dictionary gather is
// only needed by SUM.
template <int VK, int NT = kPartAggThreads>
__device__ void part_agg_v_fast(const DevQuery* __restrict__ q, const PartScratch& ps, int p, unsigned char* lds) {
  constexpr int SK = VK & 3;
  constexpr bool MN = (VK & 4) != 0, MX = (VK & 8) != 0;
  const int ks = q->kshift_v;
  const int64_t KR = q->part_kr_v ? (int64_t)q->part_kr_v : int64_t(1) << ks;  // (part_kr_v: count-free emit)
  const int64_t kbase = (int64_t)p * KR;
  const int64_t nk = min(KR, q->num_keys - kbase);
  const int fmt = q->v_fmt;
  const bool ids = fmt == V_FMT_ID && q->v_id_order != 0;  // MIN/MAX on value ids
  const int W = q->rec_words_v;
  const int as = q->vop_sum, amn = q->vop_min, amx = q->vop_max;
  const uint32_t off_s = SK ? (uint32_t)q->aggs[as].lds_off : 0u;
  const uint32_t off_mn = MN ? (uint32_t)q->aggs[amn].lds_off : 0u;
  const uint32_t off_mx = MX ? (uint32_t)q->aggs[amx].lds_off : 0u;
  const bool dbl_mn = MN && q->aggs[amn].src == SRC_DOUBLE, dbl_mx = MX && q->aggs[amx].src == SRC_DOUBLE;
  lds_u32_t* cnt = lds_ptr(lds);
  for (int64_t k = threadIdx.x; k < KR; k += NT) {
    cnt[k] = 0u;
    if (SK) {
      ((lds_u64_t*)lds_ptr(lds + off_s))[k] = 0ull;
      if (SK == 1 + SRC_LONG) ((lds_u64_t*)lds_ptr(lds + off_s))[KR + k] = 0ull;
    }
    if (MN) {
      if (ids) lds_ptr(lds + off_mn)[k] = 0xffffffffu;
      else ((lds_u64_t*)lds_ptr(lds + off_mn))[k] = (uint64_t)INT64_MAX;
    }
    if (MX) {
      if (ids) lds_ptr(lds + off_mx)[k] = 0u;
      else ((lds_u64_t*)lds_ptr(lds + off_mx))[k] = (uint64_t)INT64_MIN;
    }
  }
  __syncthreads();
  const uint64_t r0 = gp(ps.base)[p], r1 = gp(ps.base)[p + 1];
  // 64-bit SUM in one int64 per key when this partition's records cannot overflow it
  const bool narrow = SK == 1 + SRC_LONG && fmt == V_FMT_ID && q->v_maxabs > 0 &&
                      (r1 - r0) < ((uint64_t)1 << 62) / q->v_maxabs;
  const uint32_t kmask = (1u << ks) - 1u;  // (the key offset's bits: KR need not be a power of two)
  const AS1 uint32_t* recs = gp((const uint32_t*)ps.recs_v);
  const AS1 uint64_t* vdict = gp(q->vdict);
  const bool aff = q->v_affine != 0;
  const int64_t vbase = q->v_base, vstep = q->v_step;
  constexpr int kB = 16;  // records per thread in flight
  const uint64_t span = (uint64_t)kB * NT;
  // chunked records (count-free emit): the chunk entries of a batch are loaded one batch ahead, so a record load never
  // waits for its entry load (vector loads: a scalar load's wait would also wait for the LDS atomics in flight). A
  // wave's 64 records of one slot j lie in one chunk (chunks are >= 64 records, partition bases whole chunks), so
  // lane j < kB loads slot j's entry — one load per batch, not one per record — and slot j reads it back uniform
  const AS1 uint32_t* cix = ps.chunk_index ? gp(ps.chunk_index) : nullptr;
  const int csh = (int)ps.chunk_shift;
  const uint64_t cmask = cix ? (1ull << csh) - 1ull : 0ull;
  const uint32_t ln = threadIdx.x & 63u, wofs = threadIdx.x & ~63u;
  auto load_cids = [&](uint64_t b) -> uint32_t {
    const uint64_t ri = b + (uint64_t)ln * NT + wofs;
    return (ln < (uint32_t)kB && ri < r1) ? cix[ri >> csh] : 0u;
  };
  // A batch = kB records per thread. issue(): addresses (the chunk entries were loaded a batch ago), then the loads back
  // to back without a branch per load (a branch per load makes each wait for the one before it; an absent record reads
  // record 0, always allocated, and becomes a sentinel), then the next batch's chunk entries. process(): the LDS
  // updates. Two register batches alternate, so one batch's loads are in flight while the other's updates run
  // (one batch at a time measured 2 % slower on configs[2], the same on configs[4]).
  struct Batch {
    uint32_t w0[kB], w1[kB], w2[kB];
    uint32_t okm;  // (record j exists: bit j; tested in process(), so issue() never waits for its loads)
  };
  uint32_t cidv = cix ? load_cids(r0) : 0u;
  auto issue = [&](uint64_t b0, Batch& B) {
    uint32_t cid[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) cid[j] = (uint32_t)__builtin_amdgcn_readlane((int)cidv, j);
    uint64_t pa[kB];
    bool ok[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const uint64_t ri = b0 + (uint64_t)j * NT + threadIdx.x;
      const uint64_t pi = cix ? ((uint64_t)(cid[j] & 0x0fffffffu) << csh) | (ri & cmask) : ri;
      // (a partition's last chunk per workgroup holds (cid >> 28) + 1 bins)
      ok[j] = ri < r1 && (!cix || (uint32_t)(ri & cmask) < (((cid[j] >> 28) + 1u) << ps.chunk_bin_shift));
      pa[j] = ok[j] ? pi * (uint64_t)W : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) B.w0[j] = __builtin_nontemporal_load(recs + pa[j]);
#pragma unroll
    for (int j = 0; j < kB; ++j) B.w1[j] = B.w2[j] = 0u;
    if (fmt == V_FMT_32 || fmt == V_FMT_64) {
#pragma unroll
      for (int j = 0; j < kB; ++j) B.w1[j] = __builtin_nontemporal_load(recs + pa[j] + 1);
    }
    if (fmt == V_FMT_64) {
#pragma unroll
      for (int j = 0; j < kB; ++j) B.w2[j] = __builtin_nontemporal_load(recs + pa[j] + 2);
    }
    B.okm = 0u;
#pragma unroll
    for (int j = 0; j < kB; ++j) B.okm |= ok[j] ? 1u << j : 0u;
    if (cix) cidv = load_cids(b0 + span);
  };
  auto process = [&](Batch& B) {
    int64_t iv[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j)
      if (!((B.okm >> j) & 1u)) B.w0[j] = kSentinel;
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      iv[j] = 0;
      if (B.w0[j] == kSentinel) continue;
      if (fmt == V_FMT_ID) {
        if (SK || !ids) iv[j] = aff ? vbase + vstep * (int64_t)(B.w0[j] >> ks) : (int64_t)vdict[B.w0[j] >> ks];
      } else if (fmt == V_FMT_32) {
        iv[j] = (int64_t)(int32_t)B.w1[j];
      } else if (fmt == V_FMT_64) {
        iv[j] = (int64_t)(((uint64_t)B.w2[j] << 32) | B.w1[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      if (B.w0[j] == kSentinel) continue;
      const uint32_t lk = B.w0[j] & kmask;
      __hip_atomic_fetch_add(cnt + lk, 1u, WG_RLX);
      if (SK == 1 + SRC_INT) {
        __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(lds + off_s) + lk, (uint64_t)iv[j], WG_RLX);
      } else if (SK == 1 + SRC_LONG) {
        // (low and high partial sums in two arrays of 8-byte slots: interleaved 16-byte slots left a u64 atomic's
        // 16 lanes only 8 bank pairs)
        if (narrow) {
          __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(lds + off_s) + lk, (uint64_t)iv[j], WG_RLX);
        } else {
          __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(lds + off_s) + lk, (uint64_t)(uint32_t)iv[j], WG_RLX);
          __hip_atomic_fetch_add((lds_u64_t*)lds_ptr(lds + off_s) + KR + lk, (uint64_t)(iv[j] >> 32), WG_RLX);
        }
      } else if (SK == 1 + SRC_DOUBLE) {
        atomicAdd((double*)(lds + off_s) + lk, __builtin_bit_cast(double, iv[j]));
      }
      if (ids) {
        const uint32_t id = B.w0[j] >> ks;
        if (MN) __hip_atomic_fetch_min(lds_ptr(lds + off_mn) + lk, id, WG_RLX);
        if (MX) __hip_atomic_fetch_max(lds_ptr(lds + off_mx) + lk, id, WG_RLX);
      } else {
        if (MN) {
          const int64_t e = dbl_mn ? f64_order_encode(__builtin_bit_cast(double, iv[j])) : iv[j];
          __hip_atomic_fetch_min((__attribute__((address_space(3))) int64_t*)lds_ptr(lds + off_mn) + lk, e, WG_RLX);
        }
        if (MX) {
          const int64_t e = dbl_mx ? f64_order_encode(__builtin_bit_cast(double, iv[j])) : iv[j];
          __hip_atomic_fetch_max((__attribute__((address_space(3))) int64_t*)lds_ptr(lds + off_mx) + lk, e, WG_RLX);
        }
      }
    }
  };
  Batch X, Y;
  if constexpr (NT > kPartAggThreads) {  // 16 waves hide the loads themselves: one register batch
    for (uint64_t b0 = r0; b0 < r1; b0 += span) {
      issue(b0, X);
      process(X);
    }
  } else if (r0 < r1) {
    issue(r0, X);
    for (uint64_t b0 = r0;; b0 += 2 * span) {
      const bool more = b0 + span < r1;
      if (more) issue(b0 + span, Y);
      process(X);
      if (!more) break;
      const bool more2 = b0 + 2 * span < r1;
      if (more2) issue(b0 + 2 * span, X);
      process(Y);
      if (!more2) break;
    }
  }
  __syncthreads();
  // this workgroup owns keys [kbase, kbase + nk): plain stores of every accumulator
  AS1 unsigned long long* gc = gp(q->count);
  AS1 int64_t* gs = SK ? gp(q->aggs[as].acc_i64) : nullptr;
  AS1 int64_t* gmn = MN ? gp(q->aggs[amn].acc_i64) : nullptr;
  AS1 int64_t* gmx = MX ? gp(q->aggs[amx].acc_i64) : nullptr;
  for (int64_t lk = threadIdx.x; lk < nk; lk += NT) {
    const int64_t k = kbase + lk;
    const uint32_t c = cnt[lk];
    gc[k] = c;
    if (SK == 1 + SRC_LONG) {
      const int64_t lo = (int64_t)((const lds_u64_t*)lds_ptr(lds + off_s))[lk];
      const int64_t hi = (int64_t)((const lds_u64_t*)lds_ptr(lds + off_s))[KR + lk];
      // (narrow: lo holds the whole sum S; the pair is (S mod 2^32, S >> 32), the same total)
      gs[2 * k] = narrow ? (int64_t)(uint32_t)lo : lo;
      gs[2 * k + 1] = narrow ? (lo >> 32) : hi;
    } else if (SK) {
      gs[k] = (int64_t)((const lds_u64_t*)lds_ptr(lds + off_s))[lk];  // SUM(int) / SUM(double) bits
    }
    if (ids) {
      if (MN) {
        const uint64_t v = c ? vdict[lds_ptr(lds + off_mn)[lk]] : 0ull;
        gmn[k] = c == 0 ? INT64_MAX : (dbl_mn ? f64_order_encode(__builtin_bit_cast(double, v)) : (int64_t)v);
      }
      if (MX) {
        const uint64_t v = c ? vdict[lds_ptr(lds + off_mx)[lk]] : 0ull;
        gmx[k] = c == 0 ? INT64_MIN : (dbl_mx ? f64_order_encode(__builtin_bit_cast(double, v)) : (int64_t)v);
      }
    } else {
      if (MN) gmn[k] = (int64_t)((const lds_u64_t*)lds_ptr(lds + off_mn))[lk];
      if (MX) gmx[k] = (int64_t)((const lds_u64_t*)lds_ptr(lds + off_mx))[lk];
    }
  }
}

template <int NT = kPartAggThreads, int KB = 8>
__device__ void part_agg_h(const DevQuery* __restrict__ q, const PartScratch& ps, int ph, unsigned char* lds) {
  const DevAgg& H = q->aggs[q->hll_agg];
  const int lg = H.log2m;
  const int ks = q->kshift_h;
  const int64_t KR = int64_t(1) << ks;
  const int64_t kbase = (int64_t)ph << ks;
  const int64_t nk = min(KR, q->num_keys - kbase);
  const bool first = q->h_first != 0;
  uint32_t* regw = (uint32_t*)lds;                      // KR << lg one-byte registers, as words
  uint32_t* cnt = (uint32_t*)(lds + ((size_t)KR << lg));  // first-value counts (h_first)
  for (int64_t k = threadIdx.x; k < (KR << lg) / 4; k += NT) regw[k] = 0u;
  if (first)
    for (int64_t k = threadIdx.x; k < KR; k += NT) cnt[k] = 0u;
  __syncthreads();
  const int pv = q->pv;
  const uint64_t r0 = gp(ps.base)[pv + 1 + ph], r1 = gp(ps.base)[pv + 2 + ph];
  const AS1 uint32_t* recs = gp((const uint32_t*)ps.recs_h);
  const uint32_t rmask = (1u << lg) - 1u;
  constexpr int kB = KB;
  const uint64_t span = (uint64_t)kB * NT;
  // chunked records (count-free emit): as part_agg_v_fast, the chunk entries one batch ahead
  const AS1 uint32_t* cix = ps.chunk_index_h ? gp(ps.chunk_index_h) : nullptr;
  const int csh = (int)ps.chunk_shift_h;
  const uint64_t cmask = cix ? (1ull << csh) - 1ull : 0ull;
  const uint32_t ln = threadIdx.x & 63u, wofs = threadIdx.x & ~63u;
  auto load_cids = [&](uint64_t b) -> uint32_t {
    const uint64_t ri = b + (uint64_t)ln * NT + wofs;
    return (ln < (uint32_t)kB && ri < r1) ? cix[ri >> csh] : 0u;
  };
  uint32_t cidv = cix ? load_cids(r0) : 0u;
  for (uint64_t b0 = r0; b0 < r1; b0 += span) {
    uint32_t cid[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) cid[j] = (uint32_t)__builtin_amdgcn_readlane((int)cidv, j);
    // (as part_agg_v_fast: every address, then the loads without a branch per load; an absent record reads record 0)
    uint32_t w[kB];
    uint64_t pa[kB];
    bool ok[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const uint64_t ri = b0 + (uint64_t)j * NT + threadIdx.x;
      const uint64_t pi = cix ? ((uint64_t)(cid[j] & 0x0fffffffu) << csh) | (ri & cmask) : ri;
      ok[j] = ri < r1 && (!cix || (uint32_t)(ri & cmask) < (((cid[j] >> 28) + 1u) << ps.chunk_bin_shift_h));
      pa[j] = ok[j] ? pi : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) w[j] = __builtin_nontemporal_load(recs + pa[j]);
#pragma unroll
    for (int j = 0; j < kB; ++j)
      if (!ok[j]) w[j] = kSentinel;
    if (cix) cidv = load_cids(b0 + span);
    // Byte max by compare-and-swap, in phases over the kB records (each phase one run of independent LDS operations,
    // one wait): read every target word, try every needed swap once, then retry the few that lost a race.
    uint32_t rk[kB], sh[kB], old[kB];
    uint32_t* wp[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      // (a sentinel is never a valid record: its rank field would be 31; rank 0 = an empty doc's record)
      const bool ok = w[j] != kSentinel;
      const uint32_t lk = w[j] >> (lg + 6);
      rk[j] = ok ? (w[j] >> 1) & 31u : 0u;
      const uint32_t idx = (lk << lg) | ((w[j] >> 6) & rmask);
      wp[j] = regw + (rk[j] != 0 ? (idx >> 2) : 0u);
      sh[j] = (idx & 3u) * 8u;
      if (ok && first && (w[j] & 1u)) atomicAdd(cnt + lk, 1u);
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) old[j] = rk[j] != 0 ? __hip_atomic_load(wp[j], WG_RLX) : 0u;
    bool done[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      done[j] = ((old[j] >> sh[j]) & 0xffu) >= rk[j];
      if (!done[j]) {
        const uint32_t nw = (old[j] & ~(0xffu << sh[j])) | (rk[j] << sh[j]);
        done[j] = __hip_atomic_compare_exchange_strong(wp[j], &old[j], nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      if (done[j]) continue;
      uint32_t o = old[j];  // (the value the failed swap saw)
      while (((o >> sh[j]) & 0xffu) < rk[j]) {
        const uint32_t nw = (o & ~(0xffu << sh[j])) | (rk[j] << sh[j]);
        if (__hip_atomic_compare_exchange_strong(wp[j], &o, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP))
          break;
      }
    }
  }
  __syncthreads();
  // the partition's registers (16-byte stores: 2^lg >= 16 bytes per key) and, without a V stream, its counts
  AS1 u32x4* g = (AS1 u32x4*)(H.acc_hll + ((size_t)kbase << lg));
  const u32x4* l = (const u32x4*)lds;
  for (int64_t i = threadIdx.x; i < (nk << lg) / 16; i += NT) g[i] = l[i];
  if (first)
    for (int64_t lk = threadIdx.x; lk < nk; lk += NT) gp(q->count)[kbase + lk] = cnt[lk];
}

template <int VK>
__global__ void __launch_bounds__(kPartAggThreads) part_agg_kernel(const DevQuery* __restrict__ q, PartScratch ps) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  if ((int)blockIdx.x < q->pv) {
    if constexpr (VK == kVkGeneric) part_agg_v(q, ps, (int)blockIdx.x, (unsigned char*)smem);
    else part_agg_v_fast<VK>(q, ps, (int)blockIdx.x, (unsigned char*)smem);
  } else {
    part_agg_h(q, ps, (int)blockIdx.x - q->pv, (unsigned char*)smem);
  }
}

// H partitions alone, 16 waves per workgroup: a partition's registers fill the LDS (one workgroup per CU), and with 8
// waves each wave's record loads and LDS round trips sat exposed (the V variants' registers do not fit 16 waves)
constexpr int kPartAggHThreads = 1024;
template <int KB>
__global__ void __launch_bounds__(kPartAggHThreads) part_agg_h_kernel(const DevQuery* __restrict__ q, PartScratch ps) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  part_agg_h<kPartAggHThreads, KB>(q, ps, (int)blockIdx.x, (unsigned char*)smem);
}
static const void* part_agg_h_fn() {  // 16 records per thread in flight (8: 990 vs 960 us on configs[4]; PA_PASSC_HKB)
  static const bool b16 = [] {
    const char* e = std::getenv("PA_PASSC_HKB");
    return e == nullptr || std::atoi(e) != 8;
  }();
  return b16 ? (const void*)part_agg_h_kernel<16> : (const void*)part_agg_h_kernel<8>;
}
// V partitions at 16 waves per workgroup, one register batch per wave: for one-word records (configs[2]: pass C 505 ->
// 364 us, the all-docs line 1.185 -> 1.069 ms); 3-word raw-value records stay at 8 waves with two batches (configs[4]:
// 775 vs 735 us). PA_PASSC_V16=0 / 1 forces it (measurement)
template <int VK>
__global__ void __launch_bounds__(kPartAggHThreads) part_agg_v16_kernel(const DevQuery* __restrict__ q, PartScratch ps) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  part_agg_v_fast<VK, kPartAggHThreads>(q, ps, (int)blockIdx.x, (unsigned char*)smem);
}
static bool part_agg_v16(bool one_word) {
  static const int force = [] {
    const char* e = std::getenv("PA_PASSC_V16");
    return e == nullptr ? -1 : (std::atoi(e) != 0 ? 1 : 0);
  }();
  return force < 0 ? one_word : force != 0;
}
static const void* part_agg_v16_variant(int vk) {
  switch (vk) {
#define PA_VK(c) case c: return (const void*)part_agg_v16_kernel<c>;
    PA_VK(0) PA_VK(1) PA_VK(2) PA_VK(3) PA_VK(4) PA_VK(5) PA_VK(6) PA_VK(7)
    PA_VK(8) PA_VK(9) PA_VK(10) PA_VK(11) PA_VK(12) PA_VK(13) PA_VK(14) PA_VK(15)
#undef PA_VK
    default: return nullptr;
  }
}
static bool part_agg_h_split() {
  static const bool on = [] {
    const char* e = std::getenv("PA_PASSC_H_SPLIT");  // (measurement: 0 = H partitions in the V launch, 8 waves)
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

template <int VK>
static const void* part_agg_fn() { return (const void*)part_agg_kernel<VK>; }
static const void* part_agg_variant(int vk) {
  switch (vk) {
#define PA_VK(c) case c: return part_agg_fn<c>();
    PA_VK(0) PA_VK(1) PA_VK(2) PA_VK(3) PA_VK(4) PA_VK(5) PA_VK(6) PA_VK(7)
    PA_VK(8) PA_VK(9) PA_VK(10) PA_VK(11) PA_VK(12) PA_VK(13) PA_VK(14) PA_VK(15)
#undef PA_VK
    default: return part_agg_fn<kVkGeneric>();
  }
}

hipError_t launch_part_offsets(const DevQuery* hq, const PartScratch& ps, int G, int k, hipStream_t s) {
  const int P = hq->num_parts, pv = hq->pv;
  part_scan_kernel<<<P, 256, 0, s>>>(ps.hist, ps.off, G, k, P, pv, (uint32_t)hq->bs_v, (uint32_t)hq->bs_h, ps.base);
  if (pv > 0) scan_u64_kernel<<<1, 256, 0, s>>>(ps.base, pv);
  if (P > pv) scan_u64_kernel<<<1, 256, 0, s>>>(ps.base + pv + 1, P - pv);
  return hipGetLastError();
}

hipError_t set_part_agg_lds_limit(int vk, int lds_bytes) {
  hipError_t e = hipFuncSetAttribute(part_agg_h_fn(), hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  if (e != hipSuccess) return e;
  if (const void* f = part_agg_v16_variant(vk)) {
    e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) return e;
  }
  return hipFuncSetAttribute(part_agg_variant(vk), hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

// pv: the V partitions (workgroups [0, pv) of the launch); the H partitions [pv, P) go to their own launch. one_word:
// the V records are one word (key offset | value id)
hipError_t launch_part_agg(int vk, const DevQuery* q, const PartScratch& ps, int P, int pv, bool one_word,
                           int lds_bytes, hipStream_t s) {
  void* args[] = {(void*)&q, (void*)&ps};
  const bool v16 = part_agg_v16(one_word) && part_agg_v16_variant(vk) != nullptr;
  if (!part_agg_h_split() || (pv >= P && !v16))
    return hipLaunchKernel(part_agg_variant(vk), dim3(P), dim3(kPartAggThreads), args, (size_t)lds_bytes, s);
  if (pv > 0) {
    hipError_t e = v16 ? hipLaunchKernel(part_agg_v16_variant(vk), dim3(pv), dim3(kPartAggHThreads), args,
                                         (size_t)lds_bytes, s)
                       : hipLaunchKernel(part_agg_variant(vk), dim3(pv), dim3(kPartAggThreads), args, (size_t)lds_bytes, s);
    if (e != hipSuccess) return e;
  }
  if (pv >= P) return hipSuccess;
  return hipLaunchKernel(part_agg_h_fn(), dim3(P - pv), dim3(kPartAggHThreads), args, (size_t)lds_bytes, s);
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

// Fused execution statistics after the scan (pa_scan.h "fused execution statistics"). The scan waves' list slices hold
// a few E docs each, unevenly (a Poisson spread: one wave walking its own slice's docs one search after another would
// take the longest slice's time), so every workgroup first takes the prefix sums of the slice lengths into LDS, and
// its waves then take listed docs g = w, w + waves, ... (the slice of g by a binary search in LDS): one wave per listed
// E doc (its successor's label, and for a B-only doc its predecessor's) and one per segment (its first labelled doc),
// each a wave-wide neighbour search over both leaves; the leaps go into the segments' counters.
constexpr int kLeapThreads = 1024;

__global__ void __launch_bounds__(kLeapThreads) leap_search_kernel(const DevQuery* __restrict__ q,
                                                                   const DevSeg* __restrict__ segs) {
  extern __shared__ uint32_t pre[];  // [slices + 1]: exclusive prefix sums of the slice lengths
  __shared__ uint32_t part[kLeapThreads];
  const int t = threadIdx.x, lane = t & (kWave - 1);
  const int64_t nseg = q->num_segments, S = q->leap_slices, cap = q->leap_cap;
  const AS1 unsigned long long* hdr = gp(q->leap_out) + 3 * nseg;
  if (hdr[0]) return;  // (a slice overflowed: the host takes every segment's counts from leaf bitmaps)
  const int64_t per = (S + kLeapThreads - 1) / kLeapThreads;
  const int64_t s0 = min(S, (int64_t)t * per), s1 = min(S, s0 + per);
  uint32_t sum = 0;
  for (int64_t w = s0; w < s1; ++w) sum += (uint32_t)hdr[1 + w];
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < kLeapThreads; o <<= 1) {  // inclusive scan of the partial sums
    const uint32_t v = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int64_t w = s0; w < s1; ++w) {
    pre[w] = run;
    run += (uint32_t)hdr[1 + w];
  }
  if (t == kLeapThreads - 1) pre[S] = part[t];
  __syncthreads();
  const int64_t total = pre[S];
  const AS1 unsigned long long* lists = hdr + 1 + S;
  const int64_t waves = ((int64_t)gridDim.x * kLeapThreads) >> 6;
  for (int64_t g = (int64_t)blockIdx.x * (kLeapThreads >> 6) + (t >> 6); g < total + nseg; g += waves) {
    if (g < total) {
      int64_t lo = 0, hi = S;  // the last slice whose start is <= g
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)pre[mid] <= g) lo = mid;
        else hi = mid;
      }
      const uint64_t ent = lists[lo * cap + (g - (int64_t)pre[lo])];
      const int si = (int)(ent >> 40);
      const int64_t doc = (int64_t)((ent >> 1) & ((1ull << 39) - 1ull));
      uint32_t leaps = 0u, gave = 0u;
      const uint32_t succ = leap_search(segs + si, doc + 1, 1, lane);
      leaps += succ == 1u;
      gave |= succ == 4u;
      if (!(ent & 1ull)) {
        const uint32_t pred = leap_search(segs + si, doc - 1, -1, lane);
        leaps += pred == 1u;
        gave |= pred == 4u;
      }
      leap_add(q, si, 0u, leaps, gave, lane);
    } else {
      const int si = (int)(g - total);
      const uint32_t first = leap_search(segs + si, 0, 1, lane);
      leap_add(q, si, 0u, first == 1u ? 1u : 0u, first == 4u ? 1u : 0u, lane);
    }
  }
}

hipError_t launch_leap_search(const DevQuery* q, const DevSeg* segs, int64_t slices, hipStream_t s) {
  const size_t lds = (size_t)(slices + 1) * 4;  // (alloc_leaps keeps slices within kLeapMaxSlices)
  hipError_t e = hipFuncSetAttribute((const void*)leap_search_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  // 512 workgroups of 16 waves: two per CU, 8192 waves (a listed doc's two searches are a dependent chain of loads:
  // the list is spread over as many waves as fit; 256 workgroups measured 52 us, twice the docs per wave)
  hipLaunchKernelGGL(leap_search_kernel, dim3(512), dim3(kLeapThreads), lds, s, q, segs);
  return hipGetLastError();
}

static const void* scan_fn(int strategy, int steps, int lm) {
  if (const void* f = scan_fn_std(strategy, steps, lm)) return f;
  if (const void* f = scan_fn_gdense(strategy, lm)) return f;
  if (const void* f = scan_fn_part_a(strategy)) return f;
  if (const void* f = scan_fn_part_mv(strategy)) return f;
  return scan_fn_part_b(strategy);
}

hipError_t set_scan_lds_limit(int strategy, int steps, int lm, int bytes) {
  return hipFuncSetAttribute(scan_fn(strategy, steps, lm), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

hipError_t scan_occupancy(int strategy, int steps, int lm, int lds_bytes, int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, scan_fn(strategy, steps, lm), scan_waves(strategy) * kWave,
                                                      (size_t)lds_bytes);
}

hipError_t launch_scan(int strategy, int steps, int lm, int grid, int lds_bytes, const DevQuery* q, const DevSeg* segs,
                       const LmSegPlan* plans, const PartScratch& ps, hipStream_t s) {
  PartScratch pcopy = ps;
  void* args[] = {(void*)&q, (void*)&segs, (void*)&plans, (void*)&pcopy};
  return hipLaunchKernel(scan_fn(strategy, steps, lm), dim3(grid), dim3(scan_waves(strategy) * kWave), args,
                         (size_t)lds_bytes, s);
}

}  // namespace pa
