// Count-free partitioned emit (pve_jit.hip): the per-partition chunk lists pass C reads. Each emit workgroup g wrote
// its chunks (BS records each) into its own region with a table entry (partition | rank << 12) per chunk and its chunk
// count per partition (hist[g][p]). pve_offsets_kernel: per partition the exclusive scan over the workgroups (off) and
// the partition's first list entry (base, in records = chunks x BS, the unit pass C's ranges use); pve_scatter_kernel:
// every chunk's id into its partition's list at base + off + rank.
#include "pa_launch.h"

namespace pa {

__global__ void __launch_bounds__(1024) pve_offsets_kernel(const uint32_t* __restrict__ hist, uint32_t* __restrict__ off,
                                                           uint64_t* __restrict__ base, int G, int P, int bs) {
  __shared__ unsigned long long tot[1024];
  __shared__ unsigned long long run;
  if (threadIdx.x == 0) run = 0;
  for (int p0 = 0; p0 < P; p0 += 1024) {
    const int p = p0 + (int)threadIdx.x;
    unsigned long long t = 0;
    if (p < P) {
      for (int g = 0; g < G; ++g) {  // (consecutive threads read consecutive partitions of one workgroup's row)
        const uint32_t h = hist[(int64_t)g * P + p];
        off[(int64_t)g * P + p] = (uint32_t)t;
        t += h;
      }
    }
    tot[threadIdx.x] = t;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the partitions' totals
      const unsigned long long u = threadIdx.x >= (unsigned)o ? tot[threadIdx.x - o] : 0ull;
      __syncthreads();
      tot[threadIdx.x] += u;
      __syncthreads();
    }
    if (p < P) base[p] = (run + tot[threadIdx.x] - t) * (uint64_t)bs;
    __syncthreads();
    if (threadIdx.x == 1023) run += tot[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) base[P] = run * (uint64_t)bs;
}

__global__ void __launch_bounds__(256) pve_scatter_kernel(const uint32_t* __restrict__ table,
                                                          const uint32_t* __restrict__ used,
                                                          const uint32_t* __restrict__ off,
                                                          const uint64_t* __restrict__ base, uint32_t* __restrict__ index,
                                                          int64_t C, int P, int bs) {
  const int64_t g = blockIdx.x;
  const uint32_t n = used[g];
  for (uint32_t c = threadIdx.x; c < n; c += blockDim.x) {
    const uint32_t e = table[g * C + c];
    const uint32_t p = e & 0xfffu, r = e >> 12;
    index[base[p] / (uint64_t)bs + off[g * P + p] + r] = (uint32_t)(g * C + c);
  }
}

hipError_t launch_pve_lists(const uint32_t* hist, uint32_t* off, uint64_t* base, const uint32_t* table,
                            const uint32_t* used, uint32_t* index, int G, int P, int64_t C, int bs, hipStream_t s) {
  pve_offsets_kernel<<<1, 1024, 0, s>>>(hist, off, base, G, P, bs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  pve_scatter_kernel<<<G, 256, 0, s>>>(table, used, off, base, index, C, P, bs);
  return hipGetLastError();
}

}  // namespace pa
