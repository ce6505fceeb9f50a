// LDS operation-rate probe for the dense GROUP BY walk (measurement tool, not product code).
//
// Every thread issues ITER batches of 4 LDS operations at random addresses (xorshift per lane) of the kind the walk
// issues per matching doc, with W waves per CU (one workgroup per CU, held there by its LDS allocation). Prints the
// CU-cycles per wave operation at 2.4 GHz:
//   read2   : ds_read2_b32 of consecutive docs (conflict-free: the step-major decode)
//   lut     : ds_read_b32 at a random word of a 16 KiB bitmap (the DICT_SET filter lookup)
//   add32   : ds_add_u32 at a random one of K slots (COUNT)
//   add64   : ds_add_u64 at a random one of K slots (a SUM)
//   add64x3 : three ds_add_u64 per doc into three K-slot arrays (COUNT + two SUMs, unpacked)
//   add64x1p: one ds_add_u64 per doc (COUNT + two id sums packed into one word)
// hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o tools/lds_probe && ./tools/lds_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) uint32_t l32;
typedef __attribute__((address_space(3))) uint64_t l64;

__device__ __forceinline__ uint32_t xs(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

template <int MODE>
__global__ void probe(int iters, uint32_t K, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int tid = threadIdx.x;
  for (int i = tid; i < 16384; i += blockDim.x) smem[i] = i * 2654435761u;
  __syncthreads();
  uint32_t s = 0x9e3779b9u * (blockIdx.x * blockDim.x + tid + 1);
  uint32_t acc = 0;
  const uint32_t base = (uint32_t)(uintptr_t)(l32*)smem;
  for (int it = 0; it < iters; ++it) {
    uint32_t r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = xs(s);
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const l32* p = (const l32*)(uintptr_t)(base + 4u * ((tid & 63) * 9u + (r[k] & 7u) * 576u));
        acc += __builtin_amdgcn_alignbit(p[0], p[1], r[k] & 31u);
      }
    } else if (MODE == 1) {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = ((const l32*)(uintptr_t)base)[r[k] & 4095u];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += w[k];
    } else if (MODE == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) __hip_atomic_fetch_add((l32*)(uintptr_t)base + (r[k] % K), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 3) {
#pragma unroll
      for (int k = 0; k < 4; ++k) __hip_atomic_fetch_add((l64*)(uintptr_t)base + (r[k] % K), (uint64_t)r[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t key = r[k] % K;
        __hip_atomic_fetch_add((l32*)(uintptr_t)base + key, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add((l64*)(uintptr_t)(base + 8192u) + key, (uint64_t)(r[k] & 1023u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add((l64*)(uintptr_t)(base + 40960u) + key, (uint64_t)(r[k] >> 18), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else if (MODE == 5) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t key = r[k] % K;
        __hip_atomic_fetch_add((l64*)(uintptr_t)base + key, ((uint64_t)1 << 51) | ((uint64_t)(r[k] & 1023u) << 27) | (r[k] >> 18), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else if (MODE == 6) {  // per-wave private slot region (K slots per wave)
      const uint32_t wb = base + (uint32_t)(tid >> 6) * K * 8u;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        __hip_atomic_fetch_add((l64*)(uintptr_t)wb + (r[k] % K), (uint64_t)r[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  if (acc == 0x12345678u || smem[tid] == 0x12345679u) out[0] = acc;
}

template <int MODE>
double run(int waves, int iters, uint32_t K, int ncu, uint32_t* out) {
  const int threads = waves * 64;
  const size_t lds = 96 * 1024;  // one workgroup per CU
  auto k = probe<MODE>;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(ncu), dim3(threads), lds, 0, iters / 10, K, out);
  CHECK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(k, dim3(ncu), dim3(threads), lds, 0, iters, K, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double per_mode = MODE == 4 ? 3.0 : 1.0;
  const double wave_ops = (double)waves * iters * 4 * per_mode;  // per CU
  return ms * 1e-3 * 2.4e9 / wave_ops;                            // CU cycles per wave op
}

int main(int argc, char** argv) {
  int ncu = 256;
  uint32_t* out;
  CHECK(hipMalloc(&out, 64));
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const char* names[] = {"read2", "lut", "add32", "add64", "add64x3", "add64x1p", "add64wave"};
  for (int waves : {4, 8, 16}) {
    for (uint32_t K : {384u, 1536u, 4096u}) {
      double c[7];
      c[0] = run<0>(waves, iters, K, ncu, out);
      c[1] = run<1>(waves, iters, K, ncu, out);
      c[2] = run<2>(waves, iters, K, ncu, out);
      c[3] = run<3>(waves, iters, K, ncu, out);
      c[4] = run<4>(waves, iters, K, ncu, out);
      c[5] = run<5>(waves, iters, K, ncu, out);
      c[6] = K * 8u * waves <= 96u * 1024u ? run<6>(waves, iters, K, ncu, out) : -1.0;
      printf("waves %2d K %5u:", waves, K);
      for (int m = 0; m < 7; ++m) printf("  %s %.2f", names[m], c[m]);
      printf("  (CU cycles per wave op)\n");
      fflush(stdout);
    }
  }
  return 0;
}
