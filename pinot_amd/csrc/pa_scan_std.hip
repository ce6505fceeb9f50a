// Scan-kernel variants of the direct strategies: LDS-privatised accumulators, global atomics (per-lane registers:
// pa_scan_lane.hip).
#include "pa_scan.h"

namespace pa {

template <int STRAT>
static const void* fn_s(int steps, int lm) {
  if (lm) return (const void*)scan_kernel<STRAT, 32, 1>;
  return steps == 16 ? (const void*)scan_kernel<STRAT, 16, 0> : (const void*)scan_kernel<STRAT, 32, 0>;
}

const void* scan_fn_std(int strategy, int steps, int lm) {
  switch (strategy) {
    case STRAT_LDS: return fn_s<STRAT_LDS>(steps, lm);
    case STRAT_GLOBAL: return fn_s<STRAT_GLOBAL>(steps, lm);
    case STRAT_LANE:
    case STRAT_LANE_CNT:
    case STRAT_LANE_RAW:
    case STRAT_LANE_DICT: return scan_fn_lane(strategy, steps, lm);
    default: return nullptr;
  }
}

}  // namespace pa
