// Host-callable launchers of the kernels in pa_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "pa_device.h"

namespace pa {
// ordered compaction of the non-empty keys (fetch): phase 0 = per-block counts + scan (block_sums[nb] = total),
// phase 1 = write key ids + gather every section's rows into d.dst
constexpr int kMaxCompactSections = PA_MAX_AGGS + 2;
struct CompactDesc {
  int32_t nsec;
  int32_t es[kMaxCompactSections];
  int64_t per[kMaxCompactSections];
  const void* src[kMaxCompactSections];
  void* dst[kMaxCompactSections];
  int64_t* keys;
};
hipError_t launch_compact(const unsigned long long* count, int64_t K, int all, uint32_t* block_sums, int64_t cap,
                          const CompactDesc* d, int phase, hipStream_t s);
hipError_t launch_bswap_words(uint32_t* w, int64_t n, hipStream_t s);
hipError_t launch_hll_lut_numeric(const int64_t* di, const double* dd, int32_t vtype, int32_t card, int32_t log2m,
                                  uint32_t* lut, hipStream_t s);
hipError_t launch_hll_lut_hashes(const int32_t* hashes, int32_t card, int32_t log2m, uint32_t* lut, hipStream_t s);
hipError_t launch_fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
hipError_t launch_gather(const void* src, int esize, int64_t per, const int64_t* keys, int64_t n, void* out,
                         hipStream_t s);
hipError_t launch_part_offsets(uint32_t* hist, int G, int P, uint32_t* part_base, hipStream_t s);
hipError_t set_part_agg_lds_limit(int lds_bytes);
hipError_t launch_part_agg(const DevQuery* q, int P, int lds_bytes, hipStream_t s);
hipError_t set_scan_lds_limit(int strategy, int steps, int lm, int bytes);
hipError_t scan_occupancy(int strategy, int steps, int lm, int lds_bytes, int* blocks_per_cu);
hipError_t launch_scan(int strategy, int steps, int lm, int grid, int lds_bytes, const DevQuery* q, const DevSeg* segs,
                       const LmSegPlan* plans, hipStream_t s);
}  // namespace pa
