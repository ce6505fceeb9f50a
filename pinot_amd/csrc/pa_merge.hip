// Cross-GPU merge of hashed key spaces, the two local halves on the device (pa_query_pack_rows / pa_query_merge_rows,
// driven by parallel.merge_hashed_sections around one RCCL all-to-all):
//   pack:  the occupied slots of a rank's open-addressing table (count > 0) become byte rows grouped by the rank that
//          owns their packed key (owner_of, a multiplicative hash of the key);
//   merge: the rows a rank received (its share of every rank's groups) go into its own reset table by packed key,
//          each accumulator combined with its section's operator (GroupByCombineOperator's merge of intermediate
//          results: SUM for counts and sums, MIN, MAX, byte max for HLL registers and DISTINCTCOUNT presence).
// Row = every per-key section's elements of one slot, in section order (RowDesc). Both halves move rows with one
// thread per (row, 8-byte unit), so the copies are coalesced within a row whatever the row size.
#include <hip/hip_runtime.h>

#include "pa_keys.h"
#include "pa_launch.h"

namespace pa {

#define MRLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// Rank that owns packed key (k0, k1) among `world` ranks (one-word keys: k1 = 0 is not mixed in, so the function is
// parallel.key_owner's).
__device__ __forceinline__ int owner_of(int64_t k0, int64_t k1, int words, int world) {
  const int64_t k = words == 2 ? (int64_t)((uint64_t)k0 ^ mix64((uint64_t)k1)) : k0;
  int64_t h = k ^ (k >> 31);
  h = (int64_t)((uint64_t)h * 0x9E3779B97F4A7C15ULL);
  return (int)(((h >> 33) & 0x7FFFFFFF) % world);
}

__device__ __forceinline__ int row_section(const RowDesc& d, int64_t off) {
  int s = 0;
  while (s + 1 < d.nsec && d.sec[s + 1].row_off <= off) ++s;
  return s;
}

// phase 0: rows per owner (counts[world]); phase 1: every occupied slot's row index (grouped by owner: cursor[o]
// starts at the owner's first row), row_slot[row] = slot
__global__ void __launch_bounds__(256) pack_index_kernel(RowDesc d, int world, int phase, unsigned long long* counts,
                                                          unsigned long long* cursor, int64_t* row_slot) {
  const int lane = threadIdx.x & 63;
  for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x; s0 < d.num_slots; s0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = s0 + threadIdx.x;
    int o = -1;
    if (s < d.num_slots && __hip_atomic_load(d.count + s, MRLX) > 0ull) {
      const int ks = d.key_words == 2 ? 3 : 1;
      o = owner_of(d.keys[ks * s], d.key_words == 2 ? d.keys[ks * s + 1] : 0, d.key_words, world);
    }
    for (int r = 0; r < world; ++r) {
      const uint64_t m = __ballot(o == r);
      if (m == 0) continue;
      const int lead = __builtin_ctzll(m);
      if (phase == 0) {
        if (lane == lead) atomicAdd(counts + r, (unsigned long long)__builtin_popcountll(m));
      } else {
        unsigned long long base = 0;
        if (lane == lead) base = atomicAdd(cursor + r, (unsigned long long)__builtin_popcountll(m));
        base = (unsigned long long)__shfl((long long)base, lead, 64);
        if (o == r) row_slot[base + __builtin_popcountll(m & ((1ull << lane) - 1ull))] = s;
      }
    }
  }
}

// one thread per (row, 8-byte unit): slot row_slot[row] of every section into the row
__global__ void __launch_bounds__(256) pack_copy_kernel(RowDesc d, const int64_t* row_slot, int64_t rows,
                                                         unsigned char* out) {
  const int64_t upr = d.row_bytes >> 3;
  const int64_t total = rows * upr;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / upr, off = (t - r * upr) << 3;
    const RowSec& S = d.sec[row_section(d, off)];
    const int64_t slot = row_slot[r];
    const uint64_t v = *(const uint64_t*)((const unsigned char*)S.base + slot * S.slot_bytes + (off - S.row_off));
    *(uint64_t*)(out + r * d.row_bytes + off) = v;
  }
}

// phase A: one thread per received row: its packed key into the table (linear probing, insert by CAS on the empty
// marker INT64_MAX, which itself lives in slot num_slots - 1: the scan's reserved slot ht_mask + 1)
__global__ void __launch_bounds__(256) merge_keys_kernel(RowDesc d, const unsigned char* rows, int64_t n,
                                                          int64_t* row_slot, unsigned long long* counters) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t* kp = (const int64_t*)(rows + r * d.row_bytes + d.key_off);
    int64_t slot;
    if (d.key_words == 2) {
      bool ins;
      slot = ht_slot2(d.keys, d.ht_mask, kp[0], kp[1], &ins);
      if (ins) atomicAdd(counters, 1ull);
    } else if (kp[0] == INT64_MAX) {
      slot = d.ht_mask + 1;  // (the reserved slot is its own marker: its group is counted by the first such row)
      if (atomicCAS(counters + 2, 0ull, 1ull) == 0ull) atomicAdd(counters, 1ull);
    } else {
      // (a new group is counted by the row whose CAS claimed the slot: compare the slot's word before and after)
      const int64_t mask = d.ht_mask;
      int64_t h = (int64_t)(mix64((uint64_t)kp[0]) & (uint64_t)mask);
      slot = -1;
      for (int64_t probe = 0; probe <= mask; ++probe) {
        long long cur = __hip_atomic_load(d.keys + h, MRLX);
        if (cur == kp[0]) {
          slot = h;
          break;
        }
        if (cur == INT64_MAX) {
          long long expected = INT64_MAX;
          if (__hip_atomic_compare_exchange_strong(d.keys + h, &expected, (long long)kp[0], __ATOMIC_RELAXED,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            slot = h;
            atomicAdd(counters, 1ull);
            break;
          }
          if (expected == kp[0]) {
            slot = h;
            break;
          }
        }
        h = (h + 1) & mask;
      }
    }
    if (slot < 0) atomicAdd(counters + 1, 1ull);
    row_slot[r] = slot;
  }
}

__device__ __forceinline__ void atomic_max_bytes4(uint32_t* w, uint32_t v) {
  uint32_t old = __hip_atomic_load(w, MRLX);
  for (;;) {
    uint32_t nw = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) nw |= max((old >> (8 * b)) & 0xffu, (v >> (8 * b)) & 0xffu) << (8 * b);
    if (nw == old) return;
    if (__hip_atomic_compare_exchange_strong(w, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return;
  }
}

// phase B: one thread per (row, 8-byte unit): combine the unit into its slot with the section's operator
__global__ void __launch_bounds__(256) merge_values_kernel(RowDesc d, const unsigned char* rows, int64_t n,
                                                            const int64_t* row_slot) {
  const int64_t upr = d.row_bytes >> 3;
  const int64_t total = n * upr;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / upr, off = (t - r * upr) << 3;
    const int64_t slot = row_slot[r];
    if (slot < 0) continue;
    const RowSec& S = d.sec[row_section(d, off)];
    if (S.op == ROW_KEY) continue;
    const uint64_t v = *(const uint64_t*)(rows + r * d.row_bytes + off);
    unsigned char* dst = (unsigned char*)S.base + slot * S.slot_bytes + (off - S.row_off);
    switch (S.op) {
      case ROW_ADD_U64: __hip_atomic_fetch_add((unsigned long long*)dst, (unsigned long long)v, MRLX); break;
      case ROW_ADD_F64: __hip_atomic_fetch_add((double*)dst, __builtin_bit_cast(double, v), MRLX); break;
      case ROW_MIN_I64: __hip_atomic_fetch_min((long long*)dst, (long long)v, MRLX); break;
      case ROW_MAX_I64: __hip_atomic_fetch_max((long long*)dst, (long long)v, MRLX); break;
      default:  // ROW_MAX_U8
        atomic_max_bytes4((uint32_t*)dst, (uint32_t)v);
        atomic_max_bytes4((uint32_t*)dst + 1, (uint32_t)(v >> 32));
        break;
    }
  }
}

static int grid_for(int64_t threads) {
  const int64_t g = (threads + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

hipError_t launch_pack_index(const RowDesc& d, int world, int phase, unsigned long long* counts,
                             unsigned long long* cursor, int64_t* row_slot, hipStream_t s) {
  hipLaunchKernelGGL(pack_index_kernel, dim3(grid_for(d.num_slots)), dim3(256), 0, s, d, world, phase, counts, cursor,
                     row_slot);
  return hipGetLastError();
}

hipError_t launch_pack_copy(const RowDesc& d, const int64_t* row_slot, int64_t rows, unsigned char* out,
                            hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(pack_copy_kernel, dim3(grid_for(rows * (d.row_bytes >> 3))), dim3(256), 0, s, d, row_slot, rows,
                     out);
  return hipGetLastError();
}

hipError_t launch_merge_rows(const RowDesc& d, const unsigned char* rows, int64_t n, int64_t* row_slot,
                             unsigned long long* counters, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_keys_kernel, dim3(grid_for(n)), dim3(256), 0, s, d, rows, n, row_slot, counters);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(merge_values_kernel, dim3(grid_for(n * (d.row_bytes >> 3))), dim3(256), 0, s, d, rows, n,
                     row_slot);
  return hipGetLastError();
}

}  // namespace pa
