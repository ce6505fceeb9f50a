// Explicit instantiations of the partitioned passes of a multi-value group-by (one V record per (doc, value) pair):
// the count pass and the V-only emit variants (no generic records), in their own translation unit for parallel builds.
#include "pa_scan.h"

namespace pa {

const void* scan_fn_part_mv(int strategy) {
  switch (strategy) {
    case STRAT_PCOUNT_MV: return (const void*)scan_kernel<STRAT_PCOUNT_MV, 16, 0>;
#define PA_PEMIT_MV_CASE(VF) \
  case pemit_strat(VF, 0, 0, 1): return (const void*)scan_kernel<pemit_strat(VF, 0, 0, 1), 16, 0>; \
  case pemit_strat(VF, 0, 1, 1): return (const void*)scan_kernel<pemit_strat(VF, 0, 1, 1), 16, 0>;
    PA_PEMIT_MV_CASE(V_FMT_KEY) PA_PEMIT_MV_CASE(V_FMT_ID) PA_PEMIT_MV_CASE(V_FMT_32) PA_PEMIT_MV_CASE(V_FMT_64)
#undef PA_PEMIT_MV_CASE
    default: return nullptr;
  }
}

}  // namespace pa
