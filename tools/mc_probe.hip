// Prototype / probe of a lane-major dense filter + GROUP BY (measurement tool, not product code).
//
// The bench's secondary plan: 4 dictionary columns (day 9 bits, accountId 17, clicks 10, impressions 14 = 6.25 B/doc),
// WHERE day in a 384-day range AND accountId IN (an LDS bitmap) GROUP BY day SUM(clicks), SUM(impressions).
// Lane-major tiles (lane l owns TD consecutive docs of a 64*TD-doc tile), LDS-DMA ring of R images per wave, every
// column's bits unpacked from the lane's own words (static shifts: NB are template constants here), one packed u64
// LDS atomic (count | clicks id | impressions id) per matching doc into per-wave accumulators.
// MODE: 0 stream only, 1 + lane-major reads, 2 + filter, 3 + packed atomics, 4 + unpacked atomics (3 per doc),
//       5 = 3 with the key unpack but the atomics replaced by an xor
// hipcc --offload-arch=gfx950 -O3 tools/mc_probe.hip -o tools/mc_probe && ./tools/mc_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) uint32_t l32;
typedef __attribute__((address_space(3))) uint64_t l64;

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

constexpr int NB0 = 9, NB1 = 17, NB2 = 10, NB3 = 14;
constexpr int kNB[4] = {NB0, NB1, NB2, NB3};

template <int TD>
__host__ __device__ constexpr int col_dw(int nb) { return 2 * TD * nb; }  // dwords of a 64*TD-doc tile
template <int TD>
__host__ __device__ constexpr int col_ins(int nb) { return (col_dw<TD>(nb) / 4 + 63) / 64; }
template <int TD>
__host__ __device__ constexpr int tile_ins() { return col_ins<TD>(NB0) + col_ins<TD>(NB1) + col_ins<TD>(NB2) + col_ins<TD>(NB3); }
template <int TD>
__host__ __device__ constexpr int reg_off(int c) {  // dword offset of column c's region in the image (4 guard words each)
  int o = 4;
  for (int k = 0; k < c; ++k) o += col_dw<TD>(kNB[k]) + 4;
  return o;
}
template <int TD>
__host__ __device__ constexpr int img_dw() { return reg_off<TD>(4); }

// The lane's TD values of an NB-bit column, MSB-aligned (value i in the top NB bits of v[i])
template <int TD, int NB>
__device__ __forceinline__ void unpack(uint32_t region, int lane, uint32_t (&v)[TD]) {
  constexpr int K = (TD * NB + 31) / 32 + 1;
  const uint32_t bit0 = (uint32_t)lane * (uint32_t)(TD * NB);
  const l32* p = (const l32*)(uintptr_t)(region + 4u * (bit0 >> 5));
  uint32_t w[K];
#pragma unroll
  for (int j = 0; j < K; ++j) w[j] = p[j];
  if constexpr ((TD * NB) % 32 != 0) {
    const uint32_t o = bit0 & 31u;  // (TD = 16, odd NB: 0 or 16)
#pragma unroll
    for (int j = 0; j < K - 1; ++j) w[j] = o ? __builtin_amdgcn_alignbit(w[j], w[j + 1], 32u - o) : w[j];
  }
#pragma unroll
  for (int i = 0; i < TD; ++i) {
    const int s = i * NB, j = s >> 5, o = s & 31;
    v[i] = (o + NB <= 32) ? (w[j] << o) : __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - o);
  }
}

template <int TD, int W, int MODE, int ORDER = 0>
__global__ void __launch_bounds__(W * 64, 1) proto(const uint32_t* c0, const uint32_t* c1, const uint32_t* c2,
                                                   const uint32_t* c3, int64_t ntiles, uint32_t lo_t, uint32_t hi_t,
                                                   uint32_t* out) {
  constexpr int R = 2;
  constexpr int IMG = img_dw<TD>();
  constexpr int D = tile_ins<TD>();
  constexpr int NK = 384;  // day keys
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // LDS: [LUT 16 KiB][workgroup accumulators: 3 x NK u64 (packed: first NK)][ring]
  uint32_t* lut = smem;
  uint64_t* accw = (uint64_t*)(smem + 4096);
  uint32_t* ring = smem + 4096 + 2 * 3 * NK + wave * R * IMG;
  for (int i = tid; i < 4096; i += W * 64) lut[i] = (i * 2654435761u) ^ (i >> 3) * 40503u;
  for (int i = tid; i < 3 * NK; i += W * 64) accw[i] = 0;
  __syncthreads();
  const uint32_t accb = lds_addr(accw), lutb = lds_addr(lut);
  // ORDER 0: each wave its own contiguous range; 1: the workgroup's range, waves interleaved (t0 + wave + W k);
  // 2: as 1 with XCD-major workgroup ranges
  const int64_t WT = (int64_t)gridDim.x * W;
  const int64_t gw = (int64_t)blockIdx.x * W + wave;
  int64_t t0 = gw * ntiles / WT, t1 = (gw + 1) * ntiles / WT, tstep = 1;
  if (ORDER) {
    const int64_t G = gridDim.x, b = blockIdx.x;
    const int64_t lb = ORDER == 2 ? (b % 8) * (G / 8) + b / 8 : b;
    t0 = lb * ntiles / G + wave;
    t1 = (lb + 1) * ntiles / G;
    tstep = W;
  }
  const uint32_t* cols[4] = {c0, c1, c2, c3};
  uint32_t acc = 0, matched = 0;
  int64_t ti = t0;
  int islot = 0;
  auto issue = [&](int64_t t) {
    const uint32_t dst = lds_addr(ring + islot * IMG);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int nb = kNB[c];
      const char* src = (const char*)(cols[c] + t * col_dw<TD>(nb)) + 16 * lane;
      const uint32_t d = dst + 4u * reg_off<TD>(c);
      const int chunks = col_dw<TD>(nb) / 4;
#pragma unroll
      for (int k = 0; k < col_ins<TD>(nb); ++k)
        if (k * 64 + lane < chunks) dma16(src + 1024 * k, d + 1024u * k);
    }
    islot = islot + 1 == R ? 0 : islot + 1;
  };
  if (ti < t1) { issue(ti); ti += tstep; }
  int pslot = 0;
  for (int64_t t = t0; t < t1; t += tstep) {
    if (ti < t1) {
      vm_wait<0>();
      issue(ti);
      ti += tstep;
    } else {
      vm_wait<0>();
    }
    // (R = 2: the tile being processed landed, the next one is in flight)
    const uint32_t img = lds_addr(ring + pslot * IMG);
    if constexpr (MODE == 0) {
      acc ^= ((volatile uint32_t*)(ring + pslot * IMG))[lane];
    } else if constexpr (MODE == 1) {
      uint32_t v0[TD], v1[TD], v2[TD], v3[TD];
      unpack<TD, NB0>(img + 4u * reg_off<TD>(0), lane, v0);
      unpack<TD, NB1>(img + 4u * reg_off<TD>(1), lane, v1);
      unpack<TD, NB2>(img + 4u * reg_off<TD>(2), lane, v2);
      unpack<TD, NB3>(img + 4u * reg_off<TD>(3), lane, v3);
#pragma unroll
      for (int i = 0; i < TD; ++i) acc ^= v0[i] ^ v1[i] ^ v2[i] ^ v3[i];
    } else {
      uint32_t day[TD];
      unpack<TD, NB0>(img + 4u * reg_off<TD>(0), lane, day);
      uint32_t m = 0;
      {
        uint32_t nm = 0;
#pragma unroll
        for (int i = TD - 1; i >= 0; --i) {
          uint32_t u;
          asm("v_sub_u32_e64 %[u], %[t], %[lo]\n\t"
              "v_sub_co_u32_e32 %[u], vcc, %[hi], %[u]\n\t"
              "v_addc_co_u32_e32 %[nm], vcc, %[nm], %[nm], vcc"
              : [nm] "+v"(nm), [u] "=&v"(u) : [t] "v"(day[i]), [lo] "s"(lo_t), [hi] "s"(hi_t) : "vcc");
        }
        m = ~nm & (TD == 32 ? 0xffffffffu : ((1u << TD) - 1u));
      }
      {
        uint32_t a[TD];
        unpack<TD, NB1>(img + 4u * reg_off<TD>(1), lane, a);
        uint32_t wl[TD];
#pragma unroll
        for (int i = 0; i < TD; ++i) wl[i] = ((const l32*)(uintptr_t)lutb)[a[i] >> (32 - NB1 + 5)];
        uint32_t b = 0;
#pragma unroll
        for (int i = 0; i < TD; ++i) b |= ((wl[i] >> ((a[i] >> (32 - NB1)) & 31u)) & 1u) << i;
        m &= b;
      }
      matched += __builtin_popcount(m);
      if constexpr (MODE >= 3) {
        uint32_t cl[TD], im[TD];
        unpack<TD, NB2>(img + 4u * reg_off<TD>(2), lane, cl);
        unpack<TD, NB3>(img + 4u * reg_off<TD>(3), lane, im);
#pragma unroll
        for (int i = 0; i < TD; ++i) {
          if (!((m >> i) & 1u)) continue;
          const uint32_t key = (day[i] >> (32 - NB0)) - 64u;  // (the range's low id; keys 0..383)
          const uint32_t c = cl[i] >> (32 - NB2), x = im[i] >> (32 - NB3);
          if constexpr (MODE == 3) {
            const uint64_t pk = (1ull << 51) | ((uint64_t)c << 27) | x;
            __hip_atomic_fetch_add((l64*)(uintptr_t)accb + key, pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else if constexpr (MODE == 4) {
            __hip_atomic_fetch_add((l32*)(uintptr_t)accb + key, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add((l64*)(uintptr_t)accb + NK + key, (uint64_t)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add((l64*)(uintptr_t)accb + 2 * NK + key, (uint64_t)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
            acc ^= key + c + x;
          }
        }
      }
    }
    pslot = pslot + 1 == R ? 0 : pslot + 1;
  }
  vm_wait<0>();
  __syncthreads();
  if (acc == 0x12345678u || matched == 0x12345679u || ((uint32_t*)accw)[lane] == 0x1234567au) out[0] = acc + matched;
  if (lane == 0) atomicAdd(out + 1, matched);
}

template <int TD, int W, int MODE, int ORDER = 0>
void run(uint32_t* const* cols, int64_t docs, uint32_t lo_t, uint32_t hi_t, uint32_t* out, int ncu) {
  constexpr int IMG = img_dw<TD>();
  const size_t lds = 4u * (4096 + 2 * 3 * 384 + (size_t)W * 2 * IMG);
  const int64_t ntiles = docs / (64 * TD);
  auto k = proto<TD, W, MODE, ORDER>;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(ncu), dim3(W * 64), lds, 0, cols[0], cols[1], cols[2], cols[3], ntiles, lo_t, hi_t, out);
  CHECK(hipMemset(out, 0, 8));
  const int reps = 5;
  CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k, dim3(ncu), dim3(W * 64), lds, 0, cols[0], cols[1], cols[2], cols[3], ntiles, lo_t, hi_t, out);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  uint32_t h[2];
  CHECK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
  const double bytes = (double)docs * 50 / 8;
  printf("TD %2d W %d mode %d order %d: %.3f ms  %.2f TB/s  frac %.3f  matched/launch %.3f  lds %zu\n", TD, W, MODE, ORDER, ms,
         bytes / (ms * 1e-3) / 1e12, bytes / (ms * 1e-3) / 8e12, h[1] / (double)reps / docs, lds);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int64_t docs = argc > 1 ? atoll(argv[1]) : 1000000000LL;
  int dev;
  CHECK(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, dev));
  const int ncu = prop.multiProcessorCount;
  uint32_t* cols[4];
  for (int c = 0; c < 4; ++c) {
    const size_t bytes = (size_t)docs * kNB[c] / 8 + 4096;
    CHECK(hipMalloc(&cols[c], bytes));
    // pseudo-random words (a cheap device fill)
    uint32_t* h = (uint32_t*)malloc(1 << 24);
    for (int i = 0; i < (1 << 22); ++i) h[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(c * 40503u) ^ ((uint32_t)i >> 7) * 97u;
    for (size_t off = 0; off < bytes; off += (1 << 24)) CHECK(hipMemcpy((char*)cols[c] + off, h, bytes - off < (1u << 24) ? bytes - off : (1u << 24), hipMemcpyHostToDevice));
    free(h);
  }
  uint32_t* out;
  CHECK(hipMalloc(&out, 64));
  // day range: ids [64, 448) of 512, MSB-aligned compare (v - lo) <= hi - lo
  const uint32_t lo_t = 64u << (32 - NB0), hi_t = (447u << (32 - NB0)) - lo_t + ((1u << (32 - NB0)) - 1u);
  printf("ncu %d docs %lld\n", ncu, (long long)docs);
  if (argc > 2) {  // one mode only (profiling): ./mc_probe DOCS MODE
    const int m = atoi(argv[2]);
    if (m == 0) run<16, 8, 0>(cols, docs, lo_t, hi_t, out, ncu);
    if (m == 2) run<16, 8, 2>(cols, docs, lo_t, hi_t, out, ncu);
    if (m == 3) run<16, 8, 3>(cols, docs, lo_t, hi_t, out, ncu);
    if (m == 4) run<16, 8, 4>(cols, docs, lo_t, hi_t, out, ncu);
    return 0;
  }
  run<16, 8, 0>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 2>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 3>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 4>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 0, 1>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 2, 1>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 4, 1>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 0, 2>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 2, 2>(cols, docs, lo_t, hi_t, out, ncu);
  run<16, 8, 4, 2>(cols, docs, lo_t, hi_t, out, ncu);
  return 0;
}
