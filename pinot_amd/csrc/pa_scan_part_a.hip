// Scan-kernel variants of the partitioned aggregation, part A: the count pass and the emit variants without an H stream.
#include "pa_scan.h"

namespace pa {

const void* scan_fn_part_a(int strategy) {
  switch (strategy) {
    case STRAT_PCOUNT: return (const void*)scan_kernel<STRAT_PCOUNT, 16, 0>;  // the planner's only partitioned layout
#define PA_PEMIT_CASE(VF, HH) \
  case pemit_strat(VF, HH): return (const void*)scan_kernel<pemit_strat(VF, HH), 16, 0>; \
  case pemit_strat(VF, HH, 1): return (const void*)scan_kernel<pemit_strat(VF, HH, 1), 16, 0>;
    PA_PEMIT_CASE(V_FMT_KEY, 0) PA_PEMIT_CASE(V_FMT_ID, 0) PA_PEMIT_CASE(V_FMT_32, 0) PA_PEMIT_CASE(V_FMT_64, 0)
    PA_PEMIT_CASE(V_FMT_GEN, 0)
#undef PA_PEMIT_CASE
    default: return nullptr;
  }
}

}  // namespace pa
