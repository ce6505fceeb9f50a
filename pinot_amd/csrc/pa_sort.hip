// Device radix sort used by the numGroupsLimit path (pa_kernels.hip): kept in its own translation unit so the
// hipcub/rocPRIM templates compile once, apart from the scan kernels.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "pa_launch.h"

namespace pa {

hipError_t sort_u64(void* temp, size_t* temp_bytes, const unsigned long long* in, unsigned long long* out, int64_t n,
                    hipStream_t s) {
  if (n < 0 || n > INT32_MAX) return hipErrorInvalidValue;
  return hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, in, out, (int)n, 0, 64, s);
}

}  // namespace pa
