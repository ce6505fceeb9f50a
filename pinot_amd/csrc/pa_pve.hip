// Count-free partitioned emit (pve_jit.hip): the per-partition chunk lists pass C reads. Each emit workgroup g wrote
// its chunks (cr records each) into its own region with a table entry (partition | (bins - 1) << 12 | rank << 16) per
// chunk and its chunk
// count per partition (hist[g][p]). pve_offsets_kernel: per partition the exclusive scan over the workgroups (off) and
// its total; pve_base_kernel: every partition's first list entry (base, in records = chunks x cr, the unit of pass C's
// ranges); pve_scatter_kernel: every chunk's id into its partition's list at base + off + rank.
#include "pa_launch.h"

namespace pa {

// block-wide exclusive scan of v over blockDim.x threads (<= 1024); *total = the sum
__device__ __forceinline__ uint32_t block_exclusive(uint32_t v, uint32_t* tmp, uint32_t* total) {
  tmp[threadIdx.x] = v;
  __syncthreads();
  for (unsigned o = 1; o < blockDim.x; o <<= 1) {
    const uint32_t u = threadIdx.x >= o ? tmp[threadIdx.x - o] : 0u;
    __syncthreads();
    tmp[threadIdx.x] += u;
    __syncthreads();
  }
  const uint32_t inc = tmp[threadIdx.x];
  *total = tmp[blockDim.x - 1];
  __syncthreads();
  return inc - v;
}

// one workgroup per partition: the workgroups' chunk counts of the partition -> their first entry in its list (off),
// the partition's chunk total (tot)
__global__ void __launch_bounds__(256) pve_offsets_kernel(const uint32_t* __restrict__ hist, uint32_t* __restrict__ off,
                                                          uint32_t* __restrict__ tot, int G, int P) {
  __shared__ uint32_t tmp[256];
  const int p = blockIdx.x;
  uint32_t run = 0;
  for (int g0 = 0; g0 < G; g0 += 256) {
    const int g = g0 + (int)threadIdx.x;
    const uint32_t h = g < G ? hist[(int64_t)g * P + p] : 0u;
    uint32_t t;
    const uint32_t e = block_exclusive(h, tmp, &t);
    if (g < G) off[(int64_t)g * P + p] = run + e;
    run += t;
  }
  if (threadIdx.x == 0) tot[p] = run;
}

// the partitions' first list entries (in records: chunk position x records per chunk, pass C's unit)
__global__ void __launch_bounds__(1024) pve_base_kernel(const uint32_t* __restrict__ tot, uint64_t* __restrict__ base,
                                                        int P, int cr) {
  __shared__ uint32_t tmp[1024];
  uint64_t run = 0;
  for (int p0 = 0; p0 < P; p0 += 1024) {
    const int p = p0 + (int)threadIdx.x;
    uint32_t t;
    const uint32_t e = block_exclusive(p < P ? tot[p] : 0u, tmp, &t);
    if (p < P) base[p] = (run + e) * (uint64_t)cr;
    run += t;
  }
  if (threadIdx.x == 0) base[P] = run * (uint64_t)cr;
}

__global__ void __launch_bounds__(1024) pve_scatter_kernel(const uint32_t* __restrict__ table,
                                                          const uint32_t* __restrict__ used,
                                                          const uint32_t* __restrict__ off,
                                                          const uint64_t* __restrict__ base, uint32_t* __restrict__ index,
                                                          int64_t C, int P, int bs) {
  const int64_t g = blockIdx.x;
  const uint32_t n = used[g];
  for (uint32_t c = threadIdx.x; c < n; c += blockDim.x) {
    const uint32_t e = table[g * C + c];
    const uint32_t p = e & 0xfffu, r = e >> 16;
    index[base[p] / (uint64_t)bs + off[g * P + p] + r] = (uint32_t)(g * C + c) | (((e >> 12) & 15u) << 28);
  }
}

hipError_t launch_pve_lists(const uint32_t* hist, uint32_t* off, uint64_t* base, const uint32_t* table,
                            const uint32_t* used, uint32_t* index, uint32_t* tot, int G, int P, int64_t C, int cr,
                            hipStream_t s) {
  pve_offsets_kernel<<<P, 256, 0, s>>>(hist, off, tot, G, P);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  pve_base_kernel<<<1, 1024, 0, s>>>(tot, base, P, cr);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  pve_scatter_kernel<<<G, 1024, 0, s>>>(table, used, off, base, index, C, P, cr);
  return hipGetLastError();
}

}  // namespace pa
