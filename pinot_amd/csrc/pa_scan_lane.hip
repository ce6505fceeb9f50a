// Scan-kernel variants of aggregation-only queries: per-lane register accumulators (STRAT_LANE and its lane-major
// single-kind variants STRAT_LANE_CNT / _RAW / _DICT).
#include "pa_scan.h"

namespace pa {

const void* scan_fn_lane(int strategy, int steps, int lm) {
  if (lm) {
    switch (strategy) {
      case STRAT_LANE_CNT: return (const void*)scan_kernel<STRAT_LANE_CNT, 32, 1>;
      case STRAT_LANE_RAW: return (const void*)scan_kernel<STRAT_LANE_RAW, 32, 1>;
      case STRAT_LANE_DICT: return (const void*)scan_kernel<STRAT_LANE_DICT, 32, 1>;
      default: return (const void*)scan_kernel<STRAT_LANE, 32, 1>;
    }
  }
  if (strategy != STRAT_LANE) return nullptr;  // (the single-kind variants are lane-major only)
  return steps == 16 ? (const void*)scan_kernel<STRAT_LANE, 16, 0> : (const void*)scan_kernel<STRAT_LANE, 32, 0>;
}

}  // namespace pa
