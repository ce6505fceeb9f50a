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


// Mimic of scan_kernel<GLOBAL, 32, LM> on one 17-bit column: 4352-B tiles (5 DMA instructions, the last with 16
// lanes), ring of R, lane-major decode (17 ds_read_b32 + static unpack + 3-op range compare per doc), ballot.
template <int R, int DECODE>
__global__ void __launch_bounds__(256) lm17(const uint32_t* __restrict__ words, int64_t ntiles, uint32_t lo,
                                            uint32_t hi, uint32_t* out) {
  constexpr int NB = 17;
  constexpr int TILE_DW = 64 * NB;  // 1088 dwords = 4352 B
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* ring = smem + wave * R * (TILE_DW + 16);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t t0 = gw * ntiles / W, t1 = (gw + 1) * ntiles / W;
  uint32_t found = 0;
  int64_t ti = t0;
  int islot = 0;
  auto issue = [&](int64_t t) {
    const char* src = (const char*)(words + t * TILE_DW) + 16 * lane;
    const uint32_t dst = lds_addr(ring + islot * (TILE_DW + 16));
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (k < 4 || lane < 16) dma16(src + 1024 * k, dst + 1024 * k);
    islot = islot + 1 == R ? 0 : islot + 1;
  };
  for (int k = 0; k < R - 1 && ti < t1; ++k) issue(ti++);
  int pslot = 0;
  for (int64_t t = t0; t < t1; ++t) {
    if (ti < t1) { vm_wait<(R - 2) * 5>(); } else { vm_wait<0>(); }
    if (ti < t1) issue(ti++);
    if (DECODE) {
      const __attribute__((address_space(3))) uint32_t* p =
          (const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(lds_addr(ring + pslot * (TILE_DW + 16)) + lane * NB * 4);
      uint32_t w[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) w[j] = p[j];
      uint32_t nm = 0;
#pragma unroll
      for (int i = 31; i >= 0; --i) {
        const int s = i * NB, j = s >> 5, o = s & 31;
        const uint32_t tt = (o + NB <= 32) ? (w[j] << o) : __builtin_amdgcn_alignbit(w[j], w[(j + 1 < NB) ? j + 1 : j], 32 - o);
        uint32_t u;
        asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
            "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
            "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
            : [nm] "+v"(nm), [u] "=&v"(u) : [t] "v"(tt), [lo] "s"(lo), [hi] "s"(hi) : "vcc");
      }
      const uint32_t m = ~nm;
      if (__ballot(m != 0) != 0) found += __builtin_popcount(m);
    }
    pslot = pslot + 1 == R ? 0 : pslot + 1;
  }
  vm_wait<0>();
  if (found == 0x12345678u) out[0] = found;
}


template <int NB>
__device__ __forceinline__ uint32_t probe_leaf(uint32_t region_lds, int lane, uint32_t lo, uint32_t hi) {
  const __attribute__((address_space(3))) uint32_t* p =
      (const __attribute__((address_space(3))) uint32_t*)(uintptr_t)(region_lds + lane * NB * 4);
  uint32_t w[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) w[j] = p[j];
  uint32_t nm = 0;
#pragma unroll
  for (int i = 31; i >= 0; --i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    const uint32_t tt = (o + NB <= 32) ? (w[j] << o) : __builtin_amdgcn_alignbit(w[j], w[(j + 1 < NB) ? j + 1 : j], 32 - o);
    uint32_t u;
    asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
        "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
        "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
        : [nm] "+v"(nm), [u] "=&v"(u) : [t] "v"(tt), [lo] "s"(lo), [hi] "s"(hi) : "vcc");
  }
  return ~nm;
}
__device__ __forceinline__ uint32_t probe_leaf_any(int nb, uint32_t region_lds, int lane, uint32_t lo, uint32_t hi) {
  switch (nb) {
#define PC(N) case N: return probe_leaf<N>(region_lds, lane, lo, hi);
    PC(1) PC(2) PC(3) PC(4) PC(5) PC(6) PC(7) PC(8) PC(9) PC(10) PC(11) PC(12) PC(13) PC(14) PC(15) PC(16)
    PC(17) PC(18) PC(19) PC(20) PC(21) PC(22) PC(23) PC(24) PC(25) PC(26) PC(27) PC(28) PC(29) PC(30) PC(31) PC(32)
#undef PC
    default: return 0;
  }
}
template <int LO, int HI>
__device__ __forceinline__ void vm_wait_rt(int n) {
  if constexpr (LO == HI) {
    vm_wait<LO>();
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) vm_wait_rt<LO, MID>(n);
    else vm_wait_rt<MID + 1, HI>(n);
  }
}
// SWITCH: decode through the 32-way runtime dispatch; RTWAIT: vmcnt through the runtime binary tree
template <int SWITCH, int RTWAIT>
__global__ void __launch_bounds__(256) lm17x(const uint32_t* __restrict__ words, int64_t ntiles, uint32_t lo,
                                             uint32_t hi, int nb, int D, uint32_t* out) {
  constexpr int R = 2;
  constexpr int TILE_DW = 64 * 17;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* ring = smem + wave * R * (TILE_DW + 16);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t t0 = gw * ntiles / W, t1 = (gw + 1) * ntiles / W;
  uint32_t found = 0;
  int64_t ti = t0;
  int islot = 0;
  auto issue = [&](int64_t t) {
    const char* src = (const char*)(words + t * TILE_DW) + 16 * lane;
    const uint32_t dst = lds_addr(ring + islot * (TILE_DW + 16));
    const int chunks = 16 * nb;
    int issued = 0;
    for (int c0 = 0; c0 < chunks; c0 += 64) {
      if (c0 + lane < chunks) dma16(src + 16 * c0, dst + 16 * c0);
      ++issued;
    }
    islot = islot + 1 == R ? 0 : islot + 1;
  };
  for (int k = 0; k < R - 1 && ti < t1; ++k) issue(ti++);
  int pslot = 0;
  for (int64_t t = t0; t < t1; ++t) {
    if (RTWAIT) {
      vm_wait_rt<0, 63>((int)(ti - (t + 1)) * D);
    } else {
      if (ti < t1) { vm_wait<5>(); } else { vm_wait<0>(); }
    }
    if (ti < t1) issue(ti++);
    const uint32_t region = lds_addr(ring + pslot * (TILE_DW + 16));
    const uint32_t m = SWITCH ? probe_leaf_any(nb, region, lane, lo, hi) : probe_leaf<17>(region, lane, lo, hi);
    if (__ballot(m != 0) != 0) found += __builtin_popcount(m);
    pslot = pslot + 1 == R ? 0 : pslot + 1;
  }
  vm_wait<0>();
  if (found == 0x12345678u) out[0] = found;
}

__global__ void fill_random(uint32_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    p[i] = (uint32_t)x;
  }
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
#define LM17X(SW, RT) [](void* v) { Args* a = (Args*)v; lm17x<SW, RT><<<a->grid, 256, 4 * 2 * (1088 + 16) * 4>>>((const uint32_t*)a->p, a->bytes / 4352, 0x80000000u, 0x7fffu, 17, 5, a->out); }
#define LM17(R, DEC) [](void* v) { Args* a = (Args*)v; lm17<R, DEC><<<a->grid, 256, 4 * R * (1088 + 16) * 4>>>((const uint32_t*)a->p, a->bytes / 4352, 0x80000000u, 0x7fffu, a->out); }
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
  const bool random = argc > 2 && argv[2][0] == 'r';
  if (random) {
    fill_random<<<4096, 256>>>((uint32_t*)p, bytes / 4);
    CHECK(hipDeviceSynchronize());
  }
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
      {"lm17 r2 stream", LM17(2, 0), 4, 4 * 2 * 1104 * 4}, {"lm17 r2 decode", LM17(2, 1), 4, 4 * 2 * 1104 * 4},
      {"lm17 r3 decode wg3", LM17(3, 1), 3, 4 * 3 * 1104 * 4}, {"lm17 r2 decode wg3", LM17(2, 1), 3, 4 * 2 * 1104 * 4},
      {"lm17x base", LM17X(0, 0), 4, 4 * 2 * 1104 * 4}, {"lm17x switch", LM17X(1, 0), 4, 4 * 2 * 1104 * 4},
      {"lm17x rtwait", LM17X(0, 1), 4, 4 * 2 * 1104 * 4}, {"lm17x switch+rtwait", LM17X(1, 1), 4, 4 * 2 * 1104 * 4},
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
