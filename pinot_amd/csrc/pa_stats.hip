// Execution statistics engine (pa_query_execution_stats): numEntriesScannedInFilter of the reference's filter operator
// trees, computed on the GPU from per-leaf doc bitmaps.
//
// The reference counts the forward-index entries its scan iterators read while the projection drives the filter's
// iterator to the end (SVScanDocIdIterator.java:76-142, MVScanDocIdIterator.java:61-110). The host reduces an operator
// tree to constants (a scan driven by next() reads every entry), applyAnd chains (AndDocIdSet.java:92-140: each scan
// child reads the docs surviving the index children and the scans before it: a popcount, weighted by values per doc
// for a multi-value column) and leap-frogs (AndDocIdIterator.java:39-90 over a list of child iterators). This file
// holds the three kernels behind those:
//   * stat_mask_kernel: an element's doc set (a postfix program over the leaf bitmaps) materialised as a bitmap;
//   * stat_count_kernel: popcount (or value count) of a mask;
//   * leap-frog: lf_chunk_kernel + lf_compose_kernel, below.
//
// Leap-frog. AndDocIdIterator.next() advances its children in order to the candidate mx; a child answering d > mx
// makes d the candidate and restarts from the first child (skipping the one that answered). Each call is
// advance(t) -> smallest doc >= t of the child's set, and costs, for a scan child, the entries from t to the answer
// (SVScanDocIdIterator.advance reads doc by doc); for an OR child (OrDocIdIterator.java:51-110) each of its scan
// children is advanced only when t is past its cached answer, and reads from t to its own answer.
// Parallel form: the docs are cut into 2048-doc chunks. At a chunk's first doc c0 the iterator's state is one of K+1
// (K children): "child j answered a doc >= c0 that became the candidate" (then the candidate is child j's first doc >=
// c0, whatever the target was), or "fresh at c0" (a match at c0 - 1, or the segment start). One lane per (chunk,
// entry state) runs the iterator through its chunk: the exit state, the docs matched, the scan children's reads inside
// the chunk, and per scan child of an OR child the reads for both values of its "still reading from before c0" bit
// (whether an earlier call's read runs into this chunk), with that bit's value at the chunk end. lf_compose_kernel
// then chains the chunks of a segment (one wave: per lane a run of chunks composed for every entry state, the lanes'
// runs chained in order, then each run walked from its true entry), and sums the reads.
// NotDocIdIterator.java:45-70 calls its child's next() once more after the child's end: an AndDocIdIterator then
// re-runs its last chain from the last match (its scan children re-read; an OR child's scan children are all past the
// targets, so they are not advanced again): the "tail" — the direct children's reads after the segment's last match.
#include "pa_launch.h"

namespace pa {

// ---------------------------------------------------------------- element masks
__global__ void __launch_bounds__(256) stat_mask_kernel(const StatMaskJob* __restrict__ jobs, int nj,
                                                        const int32_t* __restrict__ toks) {
  __shared__ StatMaskJob SJ;
  __shared__ uint32_t stk[kBitProgStack][256];
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
  const StatMaskJob J = SJ;
  const int t0 = threadIdx.x;
  const int64_t blk = (int64_t)blockIdx.x - J.first_block;
  for (int k = 0; k < kStatMaskWordsPerThread; ++k) {
    const int64_t w = (blk * kStatMaskWordsPerThread + k) * 256 + t0;
    if (w >= J.words) break;
    const int64_t left = J.num_docs - 32 * w;
    const uint32_t valid = left >= 32 ? 0xffffffffu : (left <= 0 ? 0u : ((1u << left) - 1u));
    int sp = 0;
    for (int i = 0; i < J.len; ++i) {
      const int32_t t = toks[J.tok_off + i];
      if (t >= 0) {
        stk[sp++][t0] = J.bm[(int64_t)t * J.words + w] & valid;
      } else if (t == PA_BIT_NOT) {
        stk[sp - 1][t0] = ~stk[sp - 1][t0] & valid;
      } else {
        --sp;
        const uint32_t x = stk[sp - 1][t0], y = stk[sp][t0];
        stk[sp - 1][t0] = t == PA_BIT_AND ? (x & y) : (x | y);
      }
    }
    J.out[w] = stk[0][t0];
  }
}

// ---------------------------------------------------------------- popcounts / value counts of masks
__global__ void __launch_bounds__(256) stat_count_kernel(const StatCountJob* __restrict__ jobs, int nj) {
  __shared__ StatCountJob SJ;
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
  const StatCountJob J = SJ;
  const int64_t blk = (int64_t)blockIdx.x - J.first_block;
  unsigned long long c = 0;
  for (int k = 0; k < kStatMaskWordsPerThread; ++k) {
    const int64_t w = (blk * kStatMaskWordsPerThread + k) * 256 + threadIdx.x;
    if (w >= J.words) break;
    uint32_t b = J.mask[w];
    if (!J.wt) {
      c += (unsigned long long)__builtin_popcount(b);
    } else {
      while (b) {  // values of each set doc: offsets[d + 1] - offsets[d]
        const int64_t d = 32 * w + __builtin_ctz(b);
        b &= b - 1u;
        c += (unsigned long long)(J.wt[d + 1] - J.wt[d]);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(J.out, c);
}

// ---------------------------------------------------------------- leap-frog
// smallest set bit >= t of mask m, or c1 when none is below c1 (t < c1)
__device__ __forceinline__ int64_t lf_next(const uint32_t* __restrict__ m, int64_t t, int64_t c1) {
  int64_t w = t >> 5;
  uint32_t b = m[w] & (0xffffffffu << (t & 31));
  const int64_t wend = (c1 + 31) >> 5;
  while (b == 0u) {
    if (++w >= wend) return c1;
    b = m[w];
  }
  const int64_t d = (w << 5) + __builtin_ctz(b);
  return d < c1 ? d : c1;
}

// entries read by a scan advanced to t that answered d: docs [t, d] clipped to the chunk (d == c1: past the chunk)
__device__ __forceinline__ uint32_t lf_reads(const int32_t* __restrict__ wt, int64_t t, int64_t d, int64_t c1) {
  const int64_t e = d < c1 ? d + 1 : c1;
  return wt ? (uint32_t)(wt[e] - wt[t]) : (uint32_t)(e - t);
}

__device__ __forceinline__ const LfJob& lf_find(const LfJob* __restrict__ jobs, int nj, int64_t g) {
  int lo = 0, hi = nj - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].first_lane <= g) lo = mid;
    else hi = mid - 1;
  }
  return jobs[lo];
}

__global__ void __launch_bounds__(256) lf_chunk_kernel(const LfJob* __restrict__ jobs, int nj, int64_t lanes) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= lanes) return;
  const LfJob& J = lf_find(jobs, nj, g);
  const int K = J.K, S = J.nsub;
  const int64_t local = g - J.first_lane;
  const int64_t chunk = local / (K + 1);
  const int s = (int)(local - chunk * (K + 1));
  const int64_t c0 = chunk * kLfChunkDocs;
  const int64_t c1 = c0 + kLfChunkDocs < J.num_docs ? c0 + kLfChunkDocs : J.num_docs;
  uint32_t direct = 0, tail = 0, matches = 0, has_match = 0;
  uint32_t scost[2][kLfMaxSub];
  int64_t reach[2][kLfMaxSub];  // per OR-scan child and "reading from before c0" bit: its cached answer
  for (int j = 0; j < S; ++j) {
    scost[0][j] = scost[1][j] = 0u;
    reach[0][j] = c0 - 1;
    reach[1][j] = c0 - 1;
    if (J.sub_kind[j] != LF_DOCS) {  // bit 1: the earlier call answered the sub's first doc >= c0
      const int64_t d = lf_next(J.smask[j], c0, c1);
      reach[1][j] = d;
      scost[1][j] = lf_reads(J.swt[j], c0, d, c1);
    }
  }
  int64_t mx;
  int idx = 0, mi = -1, exit_state = K;
  if (s < K) {  // a call of child s answered its first doc >= c0: the candidate; a scan child read up to it
    mx = lf_next(J.emask[s], c0, c1);
    if (J.kind[s] == LF_SCAN) direct += lf_reads(J.ewt[s], c0, mx, c1);
    mi = s;
    if (mx >= c1) exit_state = s;
  } else {
    mx = c0;
  }
  if (mx < c1) {
    for (;;) {
      bool left = false;
      while (idx < K) {
        if (idx == mi) {
          ++idx;
          continue;
        }
        const int e = idx;
        const int64_t d = lf_next(J.emask[e], mx, c1);
        const int kd = J.kind[e];
        if (kd == LF_SCAN) {
          const uint32_t r = lf_reads(J.ewt[e], mx, d, c1);
          direct += r;
          tail += r;
        } else if (kd == LF_OR) {
          for (int j = J.sub_first[e]; j < J.sub_first[e] + J.sub_count[e]; ++j) {
            if (J.sub_kind[j] == LF_DOCS) continue;
            const bool c0v = mx > reach[0][j], c1v = mx > reach[1][j];
            if (!c0v && !c1v) continue;
            const int64_t dj = lf_next(J.smask[j], mx, c1);
            const uint32_t r = lf_reads(J.swt[j], mx, dj, c1);
            if (c0v) {
              scost[0][j] += r;
              reach[0][j] = dj;
            }
            if (c1v) {
              scost[1][j] += r;
              reach[1][j] = dj;
            }
          }
        }
        if (d == mx) {
          ++idx;
        } else {
          mx = d;
          mi = e;
          idx = 0;
          if (mx >= c1) {
            exit_state = e;
            left = true;
            break;
          }
        }
      }
      if (left) break;
      ++matches;  // every child answered mx
      has_match = 1u;
      tail = 0u;
      ++mx;
      idx = 0;
      mi = -1;
      if (mx >= c1) {
        exit_state = K;
        break;
      }
    }
  }
  uint32_t p0 = 0u, p1 = 0u;
  for (int j = 0; j < S; ++j) {
    if (reach[0][j] >= c1) p0 |= 1u << j;
    if (reach[1][j] >= c1) p1 |= 1u << j;
  }
  uint32_t* cell = J.cells + (chunk * (K + 1) + s) * (int64_t)J.cell_words;
  cell[0] = (uint32_t)exit_state | (has_match << 8) | (p0 << 16) | (p1 << 24);
  cell[1] = matches;
  cell[2] = direct;
  cell[3] = has_match ? tail : direct;
  for (int j = 0; j < S; ++j) {
    cell[4 + 2 * j] = scost[0][j];
    cell[5 + 2 * j] = scost[1][j];
  }
}

// One wave per leap-frog: lane l owns chunks [l * per, (l + 1) * per).
__global__ void __launch_bounds__(64) lf_compose_kernel(const LfJob* __restrict__ jobs) {
  const LfJob& J = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const int K = J.K, S = J.nsub;
  const int64_t nch = J.nchunks;
  const int64_t per = (nch + kWave - 1) / kWave;
  const int64_t a = (int64_t)lane * per, b = a + per < nch ? a + per : nch;
  __shared__ uint8_t ex[kWave][kLfMaxK + 1], pa[kWave][kLfMaxK + 1], pb[kWave][kLfMaxK + 1];
  __shared__ uint8_t in_s[kWave], in_p[kWave];
  __shared__ unsigned long long red[kWave][4];
  // (A) this lane's run for every entry state: exit state, and per OR-scan child the bit after the run for an entry
  // bit of 0 (pa) and of 1 (pb)
  for (int s = 0; s <= K; ++s) {
    int st = s;
    uint32_t A = 0u, B = (1u << S) - 1u;
    for (int64_t c = a; c < b; ++c) {
      const uint32_t h = J.cells[(c * (K + 1) + st) * (int64_t)J.cell_words];
      const uint32_t o0 = (h >> 16) & 0xffu, o1 = h >> 24;
      A = (A & o1) | (~A & o0);
      B = (B & o1) | (~B & o0);
      st = (int)(h & 0xffu);
    }
    ex[lane][s] = (uint8_t)st;
    pa[lane][s] = (uint8_t)A;
    pb[lane][s] = (uint8_t)B;
  }
  __syncthreads();
  // (B) the runs in order from the segment start (fresh, no read running in)
  if (lane == 0) {
    int st = K;
    uint32_t P = 0u;
    for (int l = 0; l < kWave; ++l) {
      in_s[l] = (uint8_t)st;
      in_p[l] = (uint8_t)P;
      const uint32_t A = pa[l][st], B = pb[l][st];
      P = (P & B) | (~P & A);
      st = ex[l][st];
    }
  }
  __syncthreads();
  // (C) walk the run from its true entry
  int st = in_s[lane];
  uint32_t P = in_p[lane];
  unsigned long long cost = 0, matched = 0, tl = 0;
  uint32_t any = 0u;
  for (int64_t c = a; c < b; ++c) {
    const uint32_t* cell = J.cells + (c * (K + 1) + st) * (int64_t)J.cell_words;
    const uint32_t h = cell[0];
    cost += cell[2];
    for (int j = 0; j < S; ++j) cost += cell[4 + 2 * j + ((P >> j) & 1u)];
    matched += cell[1];
    if ((h >> 8) & 1u) {
      tl = cell[3];
      any = 1u;
    } else {
      tl += cell[2];
    }
    const uint32_t o0 = (h >> 16) & 0xffu, o1 = h >> 24;
    P = (P & o1) | (~P & o0);
    st = (int)(h & 0xffu);
  }
  red[lane][0] = cost;
  red[lane][1] = matched;
  red[lane][2] = tl;
  red[lane][3] = any;
  __syncthreads();
  if (lane == 0) {
    unsigned long long C = 0, M = 0, T = 0;
    for (int l = 0; l < kWave; ++l) {
      C += red[l][0];
      M += red[l][1];
      T = red[l][3] ? red[l][2] : T + red[l][2];
    }
    J.out[0] = C;
    J.out[1] = T;
    J.out[2] = M;
  }
}

int64_t stat_mask_blocks(int64_t words) { return (words + 256 * kStatMaskWordsPerThread - 1) / (256 * kStatMaskWordsPerThread); }

hipError_t launch_stat_masks(const StatMaskJob* jobs, int nj, int64_t blocks, const int32_t* toks, hipStream_t s) {
  if (nj == 0 || blocks == 0) return hipSuccess;
  stat_mask_kernel<<<(unsigned)blocks, 256, 0, s>>>(jobs, nj, toks);
  return hipGetLastError();
}

hipError_t launch_stat_counts(const StatCountJob* jobs, int nj, int64_t blocks, hipStream_t s) {
  if (nj == 0 || blocks == 0) return hipSuccess;
  stat_count_kernel<<<(unsigned)blocks, 256, 0, s>>>(jobs, nj);
  return hipGetLastError();
}

hipError_t launch_leapfrogs(const LfJob* jobs, int nj, int64_t lanes, hipStream_t s) {
  if (nj == 0 || lanes == 0) return hipSuccess;
  lf_chunk_kernel<<<(unsigned)((lanes + 255) / 256), 256, 0, s>>>(jobs, nj, lanes);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  lf_compose_kernel<<<nj, kWave, 0, s>>>(jobs);
  return hipGetLastError();
}

// ---------------------------------------------------------------- iterator replay (the shapes the reduction leaves out)
// One thread per segment drives the reference's iterators over the element masks exactly as the projection does
// (DocIdSetOperator: next() until EOF), counting the entries the scan iterators read:
//   RP_DOCS  SortedDocIdIterator / BitmapDocIdIterator (and the merged doc sets AndDocIdSet / OrDocIdSet build): no reads
//   RP_SCAN  SVScanDocIdIterator.java:76-142: next() reads 256-doc batches, advance(t) reads from t to the next match;
//            MVScanDocIdIterator.java:61-110: doc by doc, every value of a doc
//   RP_AND   AndDocIdIterator.java:39-73   RP_OR  OrDocIdIterator.java:50-109   RP_NOT  NotDocIdIterator.java:36-66
// The host built the tree the way the reference's BlockDocIdSet.iterator() calls do (AndDocIdSet's applyAnd merges are
// counted there, as popcounts). Node state lives in the thread's private arrays; calls nest at most kRpMaxDepth deep
// (a template per depth: no recursion).
namespace {
constexpr int64_t kRpEof = -1;
constexpr int kRpBatch = 256;  // BlockDocIdIterator.OPTIMAL_ITERATOR_BATCH_SIZE

struct RpCtx {
  const RpJob* J;
  int64_t n;
  int64_t a[kRpMaxNodes], b[kRpMaxNodes], c[kRpMaxNodes];  // per-node iterator state (kind-specific)
  int64_t nd[kRpMaxNodes];                                 // an OR child's cached answer
  bool live[kRpMaxNodes];                                  // an OR child not yet exhausted
  unsigned long long ent;
};

// smallest set bit of m in [t, e), or e
__device__ __forceinline__ int64_t rp_next_set(const uint32_t* __restrict__ m, int64_t t, int64_t e) {
  if (t >= e) return e;
  int64_t w = t >> 5;
  uint32_t bits = m[w] & (0xffffffffu << (t & 31));
  const int64_t wend = (e + 31) >> 5;
  while (bits == 0u) {
    if (++w >= wend) return e;
    bits = m[w];
  }
  const int64_t d = (w << 5) + __builtin_ctz(bits);
  return d < e ? d : e;
}

__device__ __forceinline__ void rp_read(RpCtx& x, const RpNode& nd, int64_t lo, int64_t hi) {
  x.ent += nd.wt ? (unsigned long long)(nd.wt[hi] - nd.wt[lo]) : (unsigned long long)(hi - lo);
}

// SVScanDocIdIterator / MVScanDocIdIterator reading from `start` to its next match (advance; MV next)
__device__ __forceinline__ int64_t rp_scan_from(RpCtx& x, int i, int64_t start) {
  const RpNode& nd = x.J->node[i];
  const int64_t n = x.n;
  const int64_t d = rp_next_set(nd.mask, start, n);
  if (d < n) {
    rp_read(x, nd, start, d + 1);
    x.a[i] = d + 1;
    return d;
  }
  if (start < n) rp_read(x, nd, start, n);
  x.a[i] = start > n ? start : n;
  return kRpEof;
}

template <int D> __device__ int64_t rp_next(RpCtx& x, int i);
template <int D> __device__ int64_t rp_adv(RpCtx& x, int i, int64_t t);

template <int D>
__device__ __forceinline__ int64_t rp_next_child(RpCtx& x, int k) {
  if constexpr (D + 1 < kRpMaxDepth) return rp_next<D + 1>(x, k);
  else return kRpEof;  // (the host limits the depth)
}
template <int D>
__device__ __forceinline__ int64_t rp_adv_child(RpCtx& x, int k, int64_t t) {
  if constexpr (D + 1 < kRpMaxDepth) return rp_adv<D + 1>(x, k, t);
  else return kRpEof;
}

template <int D>
__device__ int64_t rp_next(RpCtx& x, int i) {
  const RpNode& nd = x.J->node[i];
  const int64_t n = x.n;
  switch (nd.kind) {
    case RP_DOCS: {
      const int64_t d = rp_next_set(nd.mask, x.a[i], n);
      x.a[i] = d < n ? d + 1 : n;
      return d < n ? d : kRpEof;
    }
    case RP_ALL:
      return x.a[i] < n ? x.a[i]++ : kRpEof;
    case RP_SCAN: {
      if (nd.wt) return rp_scan_from(x, i, x.a[i]);
      // a = next doc to read, [b, c) the current batch (its matches not yet returned from b on)
      while (true) {
        if (x.b[i] < x.c[i]) {
          const int64_t d = rp_next_set(nd.mask, x.b[i], x.c[i]);
          if (d < x.c[i]) {
            x.b[i] = d + 1;
            return d;
          }
          x.b[i] = x.c[i];
        }
        const int64_t limit = n - x.a[i] < kRpBatch ? n - x.a[i] : kRpBatch;
        if (limit <= 0) return kRpEof;
        x.ent += (unsigned long long)limit;
        x.b[i] = x.a[i];
        x.c[i] = x.a[i] + limit;
        x.a[i] += limit;
      }
    }
    case RP_AND: {
      int64_t mx = x.a[i];
      int mi = -1, idx = 0;
      while (idx < nd.nchild) {
        if (idx == mi) {
          ++idx;
          continue;
        }
        const int64_t d = rp_adv_child<D>(x, x.J->kids[nd.first + idx], mx);
        if (d == kRpEof) return kRpEof;
        if (d == mx) {
          ++idx;
        } else {
          mx = d;
          mi = idx;
          idx = 0;
        }
      }
      x.a[i] = mx + 1;
      return mx;
    }
    case RP_OR: {
      int64_t best = kRpEof;
      for (int j = 0; j < nd.nchild; ++j) {
        const int k = x.J->kids[nd.first + j];
        if (!x.live[k]) continue;
        int64_t d = x.nd[k];
        if (d == x.a[i]) {
          d = rp_next_child<D>(x, k);
          x.nd[k] = d;
          if (d == kRpEof) {
            x.live[k] = false;
            continue;
          }
        }
        best = best == kRpEof || d < best ? d : best;
      }
      if (best != kRpEof) x.a[i] = best;
      return best;
    }
    case RP_NOT: {
      const int k = x.J->kids[nd.first];
      while (x.a[i] == x.b[i]) {
        ++x.a[i];
        const int64_t c = rp_next_child<D>(x, k);
        x.b[i] = c == kRpEof ? n : c;
      }
      if (x.a[i] >= n) return kRpEof;
      return x.a[i]++;
    }
    default:
      return kRpEof;
  }
}

template <int D>
__device__ int64_t rp_adv(RpCtx& x, int i, int64_t t) {
  const RpNode& nd = x.J->node[i];
  const int64_t n = x.n;
  switch (nd.kind) {
    case RP_DOCS: {
      const int64_t d = rp_next_set(nd.mask, t, n);
      x.a[i] = d < n ? d + 1 : n;
      return d < n ? d : kRpEof;
    }
    case RP_ALL:
      x.a[i] = t;
      return rp_next<D>(x, i);
    case RP_SCAN:
      x.b[i] = x.c[i] = 0;  // (the batch is dropped)
      return rp_scan_from(x, i, t);
    case RP_AND:
      x.a[i] = t;
      return rp_next<D>(x, i);
    case RP_OR: {
      int64_t best = kRpEof;
      for (int j = 0; j < nd.nchild; ++j) {
        const int k = x.J->kids[nd.first + j];
        if (!x.live[k]) continue;
        int64_t d = x.nd[k];
        if (d < t) {
          d = rp_adv_child<D>(x, k, t);
          x.nd[k] = d;
          if (d == kRpEof) {
            x.live[k] = false;
            continue;
          }
        }
        best = best == kRpEof || d < best ? d : best;
      }
      if (best != kRpEof) x.a[i] = best;
      return best;
    }
    case RP_NOT: {
      x.a[i] = t;
      if (t > x.b[i]) {
        const int64_t c = rp_adv_child<D>(x, x.J->kids[nd.first], t);
        x.b[i] = c == kRpEof ? n : c;
      }
      return rp_next<D>(x, i);
    }
    default:
      return kRpEof;
  }
}

// NotDocIdIterator's constructor: its child's first next()
template <int D>
__device__ void rp_construct_not(RpCtx& x, int i, int depth) {
  if constexpr (D < kRpMaxDepth) {
    if (depth != D) {
      rp_construct_not<D + 1>(x, i, depth);
      return;
    }
    const int64_t c = rp_next_child<D>(x, x.J->kids[x.J->node[i].first]);
    x.a[i] = 0;
    x.b[i] = c == kRpEof ? x.n : c;
  }
}
}  // namespace

__global__ void __launch_bounds__(64) stat_replay_kernel(const RpJob* __restrict__ jobs, int nj) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nj) return;
  RpCtx x;
  x.J = jobs + j;
  x.n = x.J->num_docs;
  x.ent = 0;
  for (int i = 0; i < kRpMaxNodes; ++i) {
    x.a[i] = x.b[i] = x.c[i] = 0;
    x.nd[i] = -1;
    x.live[i] = true;
  }
  // every OR's cached answers start below doc 0 (OrDocIdIterator: _nextDocIds = -1, _previousDocId = -1)
  for (int i = 0; i < x.J->nnodes; ++i)
    if (x.J->node[i].kind == RP_OR) x.a[i] = -1;
  // iterator construction, children before parents (reverse pre-order): each NOT reads its child's first answer
  for (int i = x.J->nnodes - 1; i >= 0; --i)
    if (x.J->node[i].kind == RP_NOT) rp_construct_not<0>(x, i, x.J->node[i].depth);
  // the projection: next() until EOF; every call returns a larger doc, so n + 1 calls end it (a bound every thread
  // reaches whatever the tree)
  bool done = false;
  for (int64_t it = 0; it <= x.n + 1; ++it)
    if (rp_next<0>(x, x.J->root) == kRpEof) {
      done = true;
      break;
    }
  *x.J->out = done ? x.ent : ~0ull;
}

hipError_t launch_stat_replay(const RpJob* jobs, int nj, hipStream_t s) {
  if (nj == 0) return hipSuccess;
  stat_replay_kernel<<<(unsigned)((nj + 63) / 64), 64, 0, s>>>(jobs, nj);
  return hipGetLastError();
}

}  // namespace pa
