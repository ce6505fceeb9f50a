// Hashed group-key tables (open addressing, linear probing) shared by the scan (pa_scan.h key_slot), the numGroupsLimit
// passes and the cross-GPU row merge (pa_merge.hip). The reference's holders: IntMap / LongMap / Object2IntOpenHashMap
// of NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator.
//
// One-word keys: slot s holds the packed key itself; empty = INT64_MAX, which is also the one key that cannot be stored
// there: it lives in the reserved slot mask + 1. Insert by CAS on the empty marker. A relaxed load may return a stale
// empty marker (another XCD's CAS not yet visible in this XCD's L2): the CAS then fails and returns the real word.
//
// Two-word keys (group-by components wider than 64 bits together): slot s holds [k0, k1, state]. state = INT64_MAX when
// empty, otherwise a 60-bit fingerprint of the key with a status bit: BUSY while the claiming lane writes k0 / k1,
// READY after. A lane whose fingerprint matches a slot waits for READY, then reads k0 / k1 with read-modify-writes (they
// execute at the coherence point, so no XCD's L2 serves a stale copy) and compares; a fingerprint collision moves on to
// the next slot. The claiming lane writes k0 / k1 in the same loop iteration as its CAS, before any waiting lane of its
// wave re-reads the state (no intra-wave deadlock), and publishes READY with release order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pa {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

constexpr long long kKeyFpMask = (1LL << 60) - 1;
constexpr long long kKeyReady = 1LL << 60;
constexpr long long kKeyBusy = 1LL << 61;

#define PA_KRLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// Slot of a one-word key in a table of mask + 1 slots (+ the reserved one); -1 when the table is full.
__device__ __forceinline__ int64_t ht_slot1(long long* keys, int64_t mask, int64_t key) {
  if (key == INT64_MAX) return mask + 1;
  int64_t h = (int64_t)(mix64((uint64_t)key) & (uint64_t)mask);
  for (int64_t probe = 0; probe <= mask; ++probe) {
    long long cur = __hip_atomic_load(keys + h, PA_KRLX);
    if (cur == key) return h;
    if (cur == INT64_MAX) {
      long long expected = INT64_MAX;
      if (__hip_atomic_compare_exchange_strong(keys + h, &expected, (long long)key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT) ||
          expected == key)
        return h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

// Slot of a two-word key (k0, k1) in a table of mask + 1 slots of [k0, k1, state]; -1 when the table is full.
// *inserted = true when this call claimed the slot.
__device__ __forceinline__ int64_t ht_slot2(long long* kt, int64_t mask, int64_t k0, int64_t k1, bool* inserted) {
  const long long fp = (long long)(mix64((uint64_t)k1 ^ mix64((uint64_t)k0 + 0x9E3779B97F4A7C15ULL)) & kKeyFpMask);
  int64_t h = (int64_t)(mix64((uint64_t)k0 ^ mix64((uint64_t)k1)) & (uint64_t)mask);
  *inserted = false;
  for (int64_t probe = 0; probe <= mask; ++probe) {
    long long* st = kt + 3 * h + 2;
    long long cur = __hip_atomic_load(st, PA_KRLX);
    if (cur == INT64_MAX) {
      long long expected = INT64_MAX;
      if (__hip_atomic_compare_exchange_strong(st, &expected, fp | kKeyBusy, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_exchange(kt + 3 * h, (long long)k0, PA_KRLX);
        __hip_atomic_exchange(kt + 3 * h + 1, (long long)k1, PA_KRLX);
        __hip_atomic_exchange(st, fp | kKeyReady, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        *inserted = true;
        return h;
      }
      cur = expected;
    }
    if ((cur & kKeyFpMask) == fp) {
      while (!(cur & kKeyReady)) cur = __hip_atomic_fetch_add(st, 0LL, PA_KRLX);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const long long a = __hip_atomic_fetch_add(kt + 3 * h, 0LL, PA_KRLX);
      const long long b = __hip_atomic_fetch_add(kt + 3 * h + 1, 0LL, PA_KRLX);
      if (a == k0 && b == k1) return h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

}  // namespace pa
