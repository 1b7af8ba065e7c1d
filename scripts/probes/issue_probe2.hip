// Issue-cost probe 2 (branch-free): is the per-instruction cost of a memory instruction beside a
// one-wave-per-SIMD MFMA stream a per-wave cost, or queueing behind the other waves of the CU that
// issue the same instruction at the same moment (lockstep after a barrier)?
//
//   NW = 4: one 4-wave workgroup per CU, a barrier per iteration (the GEMM's lockstep shape);
//   NW = 1: four 1-wave workgroups per CU (one per SIMD), no barrier: the waves drift apart.
// Same per-wave stream in both: NIT iterations x 64 v_mfma_f32_16x16x32_bf16, with the mode's
// memory instructions one per 8 MFMAs (ds_read_b128: two). Address forms: 64-bit VGPR address
// ("vaddr") vs SGPR base + 32-bit VGPR offset ("saddr"), for LDS-DMA and register loads.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/issue_probe2.hip -o scripts/probes/issue_probe2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ unsigned lds_off(const lds_char* p) { return (unsigned)(__UINTPTR_TYPE__)p; }

enum { OP_NONE = 0, OP_DSR = 1, OP_DMA_V = 2, OP_DMA_S = 3, OP_GLD_V = 4, OP_GLD_S = 5, OP_DSW = 6 };

template <int NW, int OP>
__global__ __launch_bounds__(64 * NW, 1) void probe2(const char* __restrict__ src, long region,
                                                     float* __restrict__ sink, long long* __restrict__ cyc, int nit) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  constexpr int STAGE = NW * 8 * 1024;  // one iteration's LDS-DMA footprint of the workgroup
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 fa, fb;
#pragma unroll
  for (int e = 0; e < 8; ++e) { fa[e] = (short)(0x3f80 + lane + e); fb[e] = (short)(0x3f00 + lane * 3 + e); }
  s16x8 rd0, rd1;
  u32x4 g[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = u32x4{1u, 2u, 3u, (unsigned)lane};
  const unsigned lane_off = (unsigned)lane * 16u;
  const long wg_off = (long)(blockIdx.x % 64) * NW * 8 * 1024;  // workgroups read different lines
  long long t0 = 0;
  if (lane == 0) t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < nit; ++it) {
    const long gbase = ((long)it * NW * 8 * 1024 + wg_off) % region;
    lds_char* stg = smem + (it & 3) * STAGE;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      fence();
      const long piece = (long)(s * NW + wid) * 1024;
      const char* gp = src + gbase + piece;
      lds_char* lp = stg + piece;
      if constexpr (OP == OP_DSR) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(rd0) : "v"(lds_off(smem + ((it + 1) & 3) * STAGE + 2 * s * 1024) + lane_off) : "memory");
        asm volatile("ds_read_b128 %0, %1" : "=v"(rd1) : "v"(lds_off(smem + ((it + 1) & 3) * STAGE + (2 * s + 1) * 1024) + lane_off) : "memory");
      }
      if constexpr (OP == OP_DMA_V) {
        const char* p = gp + lane_off;
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds_off(lp)), "v"(p) : "memory");
      }
      if constexpr (OP == OP_DMA_S) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_off(lp)), "v"(lane_off), "s"(gp) : "memory");
      }
      if constexpr (OP == OP_GLD_V) {
        const char* p = gp + lane_off;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(g[s]) : "v"(p) : "memory");
      }
      if constexpr (OP == OP_GLD_S) {
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=&v"(g[s]) : "v"(lane_off), "s"(gp) : "memory");
      }
      if constexpr (OP == OP_DSW) {
        asm volatile("ds_write_b128 %0, %1" ::"v"(lds_off(lp) + lane_off), "v"(g[s]) : "memory");
      }
      fence();
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = s * 8 + u;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[idx / 8][idx % 8]) : "v"(fa), "v"(fb));
      }
      fence();
    }
    if constexpr (OP == OP_DMA_V || OP == OP_DMA_S || OP == OP_GLD_V || OP == OP_GLD_S)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    if constexpr (OP == OP_DSR || OP == OP_DSW) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence();
    if constexpr (NW > 1) __builtin_amdgcn_s_barrier();
    fence();
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  long long t1 = 0;
  if (lane == 0) t1 = __builtin_amdgcn_s_memtime();
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { asm volatile("" : "+a"(acc[i][j])); sm += acc[i][j][0] + acc[i][j][3]; }
  if constexpr (OP == OP_DSR) sm += (float)rd0[1] + (float)rd1[2];
  if constexpr (OP >= OP_GLD_V) {
#pragma unroll
    for (int e = 0; e < 8; ++e) sm += (float)(g[e][0] + g[e][1] + g[e][2] + g[e][3]);  // every dword live:
    // an asm load's destination is written asynchronously, so no part of it may be reused early
  }
  sink[blockIdx.x * blockDim.x + tid] = sm;
  if (lane == 0) cyc[blockIdx.x * NW + wid] = t1 - t0;
}

template <int NW, int OP>
void run(const char* name, const char* src, long region, float* sink, long long* cyc, int nit) {
  auto kern = probe2<NW, OP>;
  const int smem = 4 * NW * 8 * 1024;
  CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  const int nwg = 256 * 4 / NW;  // 1024 waves: one per SIMD
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * NW), smem, 0, src, region, sink, cyc, nit);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * NW), smem, 0, src, region, sink, cyc, nit);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  std::vector<long long> h(1024);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  const double per = 64.0 * nit;
  const double flops = 1024.0 * per * 16 * 16 * 32 * 2;
  printf("NW=%d %-22s cyc/MFMA %6.2f (p10 %6.2f p90 %6.2f)  wall %7.3f ms  %7.1f TF\n", NW, name, h[512] / per,
         h[102] / per, h[921] / per, ms, flops / (ms * 1e-3) / 1e12);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int nit = argc > 1 ? atoi(argv[1]) : 2000;
  const long region = 64L << 20;
  char* src;
  float* sink;
  long long* cyc;
  CHECK(hipMalloc(&src, region + (4 << 20)));
  CHECK(hipMemset(src, 0x3c, region + (4 << 20)));
  CHECK(hipMalloc(&sink, 1024 * 64 * 4));
  CHECK(hipMalloc(&cyc, 1024 * 8));
#define BOTH(OP, NAME) run<4, OP>(NAME, src, region, sink, cyc, nit); run<1, OP>(NAME, src, region, sink, cyc, nit);
  BOTH(OP_NONE, "mfma only")
  BOTH(OP_DSR, "+16 ds_read_b128")
  BOTH(OP_DMA_V, "+8 glds vaddr")
  BOTH(OP_DMA_S, "+8 glds saddr")
  BOTH(OP_GLD_V, "+8 gload vaddr")
  BOTH(OP_GLD_S, "+8 gload saddr")
  BOTH(OP_DSW, "+8 ds_write_b128")
  printf("done\n");
  return 0;
}
