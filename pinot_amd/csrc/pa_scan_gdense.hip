// The dense filter + GROUP BY kernel (STRAT_GDENSE, pa_gdense.h) in its own translation unit (parallel builds).
#include "pa_gdense.h"

namespace pa {

const void* scan_fn_gdense(int strategy, int lm) {
  if (strategy == STRAT_GDENSE)
    return lm ? (const void*)gdense_kernel<kGdWaves, 1> : (const void*)gdense_kernel<kGdWaves, 0>;
  if (strategy == STRAT_GDENSE8)
    return lm ? (const void*)gdense_kernel<2 * kGdWaves, 1> : (const void*)gdense_kernel<2 * kGdWaves, 0>;
  if (strategy == STRAT_GDENSE12 && !lm) return (const void*)gdense_kernel<3 * kGdWaves, 0>;
  if (strategy == STRAT_GDENSE_RS12 && !lm)
    return (const void*)gdense_rs_kernel<3 * kGdWaves, gd_rs_ring(STRAT_GDENSE_RS12), gd_rs_dmax(STRAT_GDENSE_RS12)>;
  if (strategy == STRAT_GDENSE_RS8 && !lm)
    return (const void*)gdense_rs_kernel<2 * kGdWaves, gd_rs_ring(STRAT_GDENSE_RS8), gd_rs_dmax(STRAT_GDENSE_RS8)>;
  if (strategy == STRAT_GDENSE_LM8 && !lm) return (const void*)gdense_kernel<2 * kGdWaves, 2>;
  if (strategy == STRAT_GDENSE_LM16 && !lm) return (const void*)gdense_kernel<4 * kGdWaves, 2>;
  return nullptr;
}

}  // namespace pa
