// Scan-kernel variants of the partitioned aggregation, part B: the emit variants with an H (DISTINCTCOUNTHLL) stream.
#include "pa_scan.h"

namespace pa {

const void* scan_fn_part_b(int strategy) {
  switch (strategy) {
#define PA_PEMIT_CASE(VF, HH) \
  case pemit_strat(VF, HH): return (const void*)scan_kernel<pemit_strat(VF, HH), 16, 0>; \
  case pemit_strat(VF, HH, 1): return (const void*)scan_kernel<pemit_strat(VF, HH, 1), 16, 0>;
    PA_PEMIT_CASE(-1, 1)
    PA_PEMIT_CASE(V_FMT_KEY, 1) PA_PEMIT_CASE(V_FMT_ID, 1) PA_PEMIT_CASE(V_FMT_32, 1) PA_PEMIT_CASE(V_FMT_64, 1)
    PA_PEMIT_CASE(V_FMT_GEN, 1)
#undef PA_PEMIT_CASE
    default: return nullptr;
  }
}

}  // namespace pa
