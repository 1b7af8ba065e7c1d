// Issue-cost probe 3: the memory instructions of one 256x256x64 GEMM K-tile (per wave of a 4-wave,
// one-wave-per-SIMD workgroup: 32 ds_read_b128 fragment reads + 16 LDS-DMA pieces) beside the
// K-tile's MFMAs, for the two bf16 MFMA shapes:
//   16x16x32: 128 MFMAs per K-tile, 16 cycles each, 8 of them free for other issue
//   32x32x16:  64 MFMAs per K-tile, 32 cycles each, 24 of them free
// and two placements: "bunched" (a slot's 3 memory instructions back to back, then its MFMAs) and
// "spread" (at most one memory instruction per MFMA gap). Probes 1 and 2 found ~15 cycles per
// ds_read_b128 and ~38 per LDS-DMA beside 16x16x32 MFMAs, the same with free-running waves as in
// lockstep: a per-wave issue cost, which a longer MFMA should hide.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/issue_probe3.hip -o scripts/probes/issue_probe3
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) char lds_char;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ unsigned lds_off(const lds_char* p) { return (unsigned)(__UINTPTR_TYPE__)p; }

enum { DSR = 1, DMA = 2 };

// SHAPE 16: acc16[64] (f32x4); SHAPE 32: acc32[16] (f32x16). 256 AGPRs either way.
template <int SHAPE>
struct Acc;
template <>
struct Acc<16> {
  f32x4 a[64];
};
template <>
struct Acc<32> {
  f32x16 a[16];
};

template <int SHAPE>
__device__ __forceinline__ void mfma(Acc<SHAPE>& acc, int i, const s16x8& fa, const s16x8& fb) {
  if constexpr (SHAPE == 16)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc.a[i & 63]) : "v"(fa), "v"(fb));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc.a[i & 15]) : "v"(fa), "v"(fb));
}

template <int SHAPE, int OPS, bool SPREAD>
__global__ __launch_bounds__(256, 1) void probe3(const char* __restrict__ src, long region, float* __restrict__ sink,
                                                 long long* __restrict__ cyc, int nit) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  constexpr int MPS = SHAPE == 16 ? 8 : 4;  // MFMAs per slot (16 slots per K-tile)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  Acc<SHAPE> acc;
  constexpr int NA = SHAPE == 16 ? 64 : 16;
#pragma unroll
  for (int i = 0; i < NA; ++i) acc.a[i] = {};
  s16x8 fa, fb;
#pragma unroll
  for (int e = 0; e < 8; ++e) { fa[e] = (short)(0x3f80 + lane + e); fb[e] = (short)(0x3f00 + lane * 3 + e); }
  s16x8 r0, r1;
  r0 = fa;
  r1 = fb;
  const unsigned lane_off = (unsigned)lane * 16u;
  const long wg_off = (long)(blockIdx.x % 64) * 65536;
  long long t0 = 0;
  if (lane == 0) t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < nit; ++it) {
    const long gbase = ((long)it * 65536 + wg_off) % region;  // one 64 KB K-tile (A + B) per iteration
    lds_char* stg = smem + (it & 1) * 65536;
    const lds_char* rdb = smem + ((it + 1) & 1) * 65536;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const long piece = (long)(s * 4 + wid) * 1024;
      const unsigned rd_a = lds_off(rdb + (2 * s) * 1024) + lane_off;
      const unsigned rd_b = lds_off(rdb + (2 * s + 1) * 1024) + lane_off;
      // memory op k of this slot goes before MFMA position pos[k]: bunched = 0,0,0; spread = 0,1,2
#pragma unroll
      for (int u = 0; u < MPS; ++u) {
        fence();
        if ((OPS & DSR) && u == 0) asm volatile("ds_read_b128 %0, %1" : "=&v"(r0) : "v"(rd_a) : "memory");
        if ((OPS & DSR) && u == (SPREAD ? 1 : 0)) asm volatile("ds_read_b128 %0, %1" : "=&v"(r1) : "v"(rd_b) : "memory");
        if ((OPS & DMA) && u == (SPREAD ? 2 : 0))
          __builtin_amdgcn_global_load_lds((const void*)(src + gbase + piece + lane_off),
                                           (__attribute__((address_space(3))) void*)(stg + piece), 16, 0, 0);
        fence();
        mfma<SHAPE>(acc, s * MPS + u, fa, fb);
      }
    }
    fence();
    if constexpr (OPS & DMA) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    if constexpr (OPS & DSR) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence();
    __builtin_amdgcn_s_barrier();
    fence();
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  long long t1 = 0;
  if (lane == 0) t1 = __builtin_amdgcn_s_memtime();
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    asm volatile("" : "+a"(acc.a[i]));
    sm += acc.a[i][0];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sm += (float)r0[e] + (float)r1[e];
  sink[blockIdx.x * blockDim.x + tid] = sm;
  if (lane == 0) cyc[blockIdx.x * 4 + wid] = t1 - t0;
}

template <int SHAPE, int OPS, bool SPREAD>
void run(const char* name, const char* src, long region, float* sink, long long* cyc, int nit) {
  auto kern = probe3<SHAPE, OPS, SPREAD>;
  const int smem = 2 * 65536;
  CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), smem, 0, src, region, sink, cyc, nit);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), smem, 0, src, region, sink, cyc, nit);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  std::vector<long long> h(1024);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  const double flops = 1024.0 * nit * (128.0 * 16 * 16 * 32 * 2);  // 128x128x64 per wave per K-tile
  printf("%2dx%2d %-26s cyc/K-tile %7.1f (MFMA floor 2048)  util %5.1f%%  wall %7.3f ms  %7.1f TF\n", SHAPE, SHAPE,
         name, (double)h[512] / nit, 100.0 * 2048.0 * nit / h[512], ms, flops / (ms * 1e-3) / 1e12);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int nit = argc > 1 ? atoi(argv[1]) : 1000;
  const long region = 64L << 20;
  char* src;
  float* sink;
  long long* cyc;
  CHECK(hipMalloc(&src, region + (8 << 20)));
  CHECK(hipMemset(src, 0x3c, region + (8 << 20)));
  CHECK(hipMalloc(&sink, 256 * 256 * 4));
  CHECK(hipMalloc(&cyc, 1024 * 8));
#define SHAPES(OPS, SP, NAME) run<16, OPS, SP>(NAME, src, region, sink, cyc, nit); run<32, OPS, SP>(NAME, src, region, sink, cyc, nit);
  SHAPES(0, false, "mfma only")
  SHAPES(DSR, false, "+32 ds_read bunched")
  SHAPES(DSR, true, "+32 ds_read spread")
  SHAPES(DMA, false, "+16 glds")
  SHAPES(DSR | DMA, false, "+32 dsr +16 glds bunched")
  SHAPES(DSR | DMA, true, "+32 dsr +16 glds spread")
  printf("done\n");
  return 0;
}
