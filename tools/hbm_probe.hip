// HBM read-ceiling probe for the scan kernel's access shape (measurement tool, not product code).
//
// Reads a B-byte buffer (default 2.125 GB = the bench's staged bytes per launch) three ways and prints GB/s:
//   reg    : grid-stride 16 B/lane global_load_dwordx4 into registers (xor-reduced), U loads in flight per lane
//   wchunk : each wave owns a contiguous range and reads it in C-KiB chunks into registers (the scan's tile order)
//   ldsdma : each wave owns a contiguous range and streams C-KiB chunks HBM->LDS with global_load_lds_dwordx4
//            into a ring of R slots behind counted vmcnt waits (the scan kernel's staging loop without the decode)
// hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe && ./tools/hbm_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U>
__global__ void __launch_bounds__(256) read_reg(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x12345678u) out[0] = acc;
}

// chunk = CK KiB = CK wave-instructions of 1 KiB
template <int CK>
__global__ void __launch_bounds__(256) read_wchunk(const uint4* __restrict__ p, int64_t nchunks, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t c0 = gw * nchunks / W, c1 = (gw + 1) * nchunks / W;
  uint32_t acc = 0;
  for (int64_t c = c0; c < c1; ++c) {
    const uint4* q = p + c * (CK * 64) + lane;
    uint4 v[CK];
#pragma unroll
    for (int u = 0; u < CK; ++u) v[u] = q[u * 64];
#pragma unroll
    for (int u = 0; u < CK; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds_base));
}
template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// RD: ds_read_b32 per lane per chunk (synthetic decode LDS load), VA: dependent VALU ops per read
template <int CK, int R, int RD = 0, int VA = 0>
__global__ void __launch_bounds__(256) read_ldsdma(const uint4* __restrict__ p, int64_t nchunks, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* ring = smem + wave * R * CK * 256;
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t c0 = gw * nchunks / W, c1 = (gw + 1) * nchunks / W;
  uint32_t acc = 0;
  int64_t ci = c0;
  int slot = 0;
  auto issue = [&](int64_t c) {
    const uint4* q = p + c * (CK * 64) + lane;
    const uint32_t dst = lds_addr(ring + slot * CK * 256);
#pragma unroll
    for (int u = 0; u < CK; ++u) dma16(q + u * 64, dst + u * 1024);
    slot = slot + 1 == R ? 0 : slot + 1;
  };
  for (int k = 0; k < R - 1; ++k) { if (ci < c1) issue(ci); ++ci; }
  int pslot = 0;
  for (int64_t c = c0; c < c1; ++c) {
    if (ci < c1) { vm_wait<(R - 2) * CK>(); } else { vm_wait<0>(); }
    if (ci < c1) issue(ci);
    if constexpr (RD == 0) {
      acc ^= ((volatile uint32_t*)(ring + pslot * CK * 256))[lane];
    } else {
      const __attribute__((address_space(3))) uint32_t* img =
          (const __attribute__((address_space(3))) uint32_t*)(uintptr_t)lds_addr(ring + pslot * CK * 256);
      uint32_t w[RD];
#pragma unroll
      for (int k = 0; k < RD; ++k) w[k] = img[(lane * 17 + k * 37) & (CK * 256 - 1)];
#pragma unroll
      for (int k = 0; k < RD; ++k) {
        uint32_t x = w[k];
#pragma unroll
        for (int v = 0; v < VA; ++v) x = __builtin_amdgcn_alignbit(x, acc, (k + v) & 31) + v;
        acc ^= x;
      }
    }
    ++ci;
    pslot = pslot + 1 == R ? 0 : pslot + 1;
  }
  vm_wait<0>();
  if (acc == 0x12345678u) out[0] = acc;
}

static float time_kernel(void (*launch)(void*), void* arg, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch(arg);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) launch(arg);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return ms / reps;
}

struct Args { const uint4* p; int64_t bytes; uint32_t* out; int grid; };
static Args g;

#define REG(U) [](void* v) { Args* a = (Args*)v; read_reg<U><<<a->grid, 256>>>(a->p, a->bytes / 16, a->out); }
#define WCH(CK) [](void* v) { Args* a = (Args*)v; read_wchunk<CK><<<a->grid, 256>>>(a->p, a->bytes / (CK * 1024), a->out); }
#define DMAX(CK, R, RD, VA) [](void* v) { Args* a = (Args*)v; read_ldsdma<CK, R, RD, VA><<<a->grid, 256, 4 * R * CK * 1024>>>(a->p, a->bytes / (CK * 1024), a->out); }
#define DMA(CK, R) [](void* v) { Args* a = (Args*)v; read_ldsdma<CK, R><<<a->grid, 256, 4 * R * CK * 1024>>>(a->p, a->bytes / (CK * 1024), a->out); }

int main(int argc, char** argv) {
  int64_t bytes = argc > 1 ? atoll(argv[1]) : 2125081600LL;
  bytes -= bytes % (64 * 1024);
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  void* p;
  CHECK(hipMalloc(&p, bytes));
  CHECK(hipMemset(p, 1, bytes));
  uint32_t* out;
  CHECK(hipMalloc(&out, 64));
  g = Args{(const uint4*)p, bytes, out, 0};
  struct V { const char* name; void (*fn)(void*); int wg_per_cu; int lds; };
  V vs[] = {
      {"reg U4", REG(4), 8, 0}, {"reg U8", REG(8), 8, 0}, {"reg U4 wg4", REG(4), 4, 0}, {"reg U8 wg16", REG(8), 16, 0},
      {"wchunk 4K", WCH(4), 8, 0}, {"wchunk 8K", WCH(8), 4, 0}, {"wchunk 8K wg8", WCH(8), 8, 0}, {"wchunk 16K", WCH(16), 2, 0},
      {"ldsdma 4K r2", DMA(4, 2), 4, 4 * 2 * 4 * 1024}, {"ldsdma 4K r3", DMA(4, 3), 4, 4 * 3 * 4 * 1024},
      {"ldsdma 4K r4", DMA(4, 4), 2, 4 * 4 * 4 * 1024}, {"ldsdma 8K r2", DMA(8, 2), 2, 4 * 2 * 8 * 1024},
      {"ldsdma 8K r3", DMA(8, 3), 1, 4 * 3 * 8 * 1024}, {"ldsdma 2K r4", DMA(2, 4), 4, 4 * 4 * 2 * 1024},
      {"ldsdma 2K r8", DMA(2, 8), 2, 4 * 8 * 2 * 1024}, {"ldsdma 4K r2 wg3", DMA(4, 2), 3, 4 * 2 * 4 * 1024},
      // synthetic decode on a 4 KiB chunk (~1900 docs of 17 bits): current scheme = 60 ds_read + 4 VALU per read pair
      {"dec 4K r2 rd60 va2", DMAX(4, 2, 60, 2), 4, 4 * 2 * 4 * 1024}, {"dec 4K r2 rd60 va0", DMAX(4, 2, 60, 0), 4, 4 * 2 * 4 * 1024},
      {"dec 4K r2 rd16 va8", DMAX(4, 2, 16, 8), 4, 4 * 2 * 4 * 1024}, {"dec 4K r2 rd16 va0", DMAX(4, 2, 16, 0), 4, 4 * 2 * 4 * 1024},
      {"dec 4K r3 rd60 va2", DMAX(4, 3, 60, 2), 4, 4 * 3 * 4 * 1024}, {"dec 4K r3 rd16 va8", DMAX(4, 3, 16, 8), 4, 4 * 3 * 4 * 1024},
      {"dec 4K r2 rd4 va30", DMAX(4, 2, 4, 30), 4, 4 * 2 * 4 * 1024}, {"dec 8K r2 rd32 va8", DMAX(8, 2, 32, 8), 2, 4 * 2 * 8 * 1024},
  };
  for (auto& v : vs) {
    if (v.lds > 65536) {
      printf("%-18s skipped (lds %d)\n", v.name, v.lds);
      continue;
    }
    g.grid = cus * v.wg_per_cu;
    float ms = time_kernel(v.fn, &g, 10);
    printf("{\"variant\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", v.name, g.grid, ms, bytes / ms / 1e6);
    fflush(stdout);
  }
  CHECK(hipFree(p));
  CHECK(hipFree(out));
  return 0;
}
