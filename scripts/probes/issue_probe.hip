// Issue-cost probe: what do memory-side instructions cost a wave that is the ONLY wave feeding its
// SIMD's matrix pipe (the one-wave-per-SIMD 128x128 GEMM), and what do they cost when a PARTNER
// wave on the same SIMD issues them instead (8-wave ping-pong)?
//
// Every mode runs the same MFMA stream per compute wave: NIT iterations x 64
// v_mfma_f32_16x16x32_bf16 on 64 independent accumulators (acc[8][8], AGPRs), with 8 "slots" per
// iteration (one every 8 MFMAs) where the mode's extra instructions go. Per-iteration traffic per
// CU matches one 32-deep K-slice of a 256x256 tile (32 KB). Timing: s_memtime around the loop (wave
// 0 of each workgroup) + hipEvent wall.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/issue_probe.hip -o /tmp/issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ unsigned lds_off(const lds_char* p) { return (unsigned)(__UINTPTR_TYPE__)p; }

template <int NI, int NJ>
__device__ __forceinline__ void mfma8(f32x4 (&acc)[NI][NJ], const s16x8& a, const s16x8& b, int base) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int idx = (base + u) % (NI * NJ);
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[idx / NJ][idx % NJ]) : "v"(a), "v"(b));
  }
}

// MODE bits
enum {
  M_DMA = 1,       // 1 global_load_lds_dwordx4 per slot
  M_GLD = 2,       // 1 global_load_dwordx4 (to VGPRs) per slot
  M_DSW = 4,       // 1 ds_write_b128 per slot (data: the previous iteration's GLD registers, or constants)
  M_DSR = 8,       // 2 ds_read_b128 per slot
  M_BUF = 16,      // 1 buffer_load_dwordx4 ... lds per slot (instead of the global form)
  M_SPLIT = 32,    // 8 waves: waves 0-3 compute (acc[8][4]... same 64 MFMA/iter), waves 4-7 issue the memory ops
  M_PRIO = 64,     // compute waves at s_setprio 1 (with M_SPLIT)
  M_STAG = 128,    // wave w issues its memory ops 2*w MFMAs later than wave 0 (no two waves collide)
  M_ONE = 256,     // only memory-wave 0 issues memory ops (no contention at all)
};

// One iteration (64 MFMAs, 8 memory slots) of a wave whose memory ops are shifted by SH MFMAs.
template <int MODE, int SH, int NJ>
__device__ __forceinline__ void iteration(f32x4 (&acc)[8][NJ], const s16x8& fa, const s16x8& fb, s16x8 (&rd)[2],
                                          u32x4 (&ga)[8], u32x4 (&gb)[8], const char* src, long gbase,
                                          lds_char* smem, lds_char* stg, int it, int half, int mw, bool computer,
                                          bool memer, unsigned lane_off, __amdgpu_buffer_rsrc_t rsrc) {
#pragma unroll
  for (int u = 0; u < 64; ++u) {
    // STAG: memory-wave w's ops sit 2*w MFMAs after wave 0's; a uniform branch per op
    const bool at = (MODE & M_STAG) ? ((u & 7) % 2 == 0 && mw == (u & 7) / 2) : ((u & 7) == SH);
    if (at && memer) {
      const int s = u >> 3;
      fence();
      const char* gp = src + gbase + (long)(s * 4 + mw) * 1024;
      if constexpr (MODE & M_DMA)
        __builtin_amdgcn_global_load_lds((const void*)(gp + lane_off),
                                         (__attribute__((address_space(3))) void*)(stg + (s * 4 + mw) * 1024), 16, 0, 0);
      if constexpr (MODE & M_BUF)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(stg + (s * 4 + mw) * 1024),
                                                 16, (int)(gbase + (s * 4 + mw) * 1024) + (int)lane_off, 0, 0, 0);
      if constexpr (MODE & M_GLD) {
        u32x4& r = half ? gb[s] : ga[s];
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(lane_off), "s"(gp) : "memory");
      }
      if constexpr (MODE & M_DSW) {
        const u32x4& r = half ? ga[s] : gb[s];
        asm volatile("ds_write_b128 %0, %1" ::"v"(lds_off(stg + (s * 4 + mw) * 1024) + lane_off), "v"(r) : "memory");
      }
      if constexpr (MODE & M_DSR) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          asm volatile("ds_read_b128 %0, %1" : "=v"(rd[q]) : "v"(lds_off(smem + (((it + half + 1) & 3) * 32768) + (s * 2 + q) * 1024) + lane_off) : "memory");
      }
      fence();
    }
    if (computer) {
      const int idx = u % (8 * NJ);
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[idx / NJ][idx % NJ]) : "v"(fa), "v"(fb));
    }
  }
}

template <int MODE>
__global__ __launch_bounds__((MODE & M_SPLIT) ? 512 : 256, 1) void probe(const char* __restrict__ src, long region,
                                                                       float* __restrict__ sink,
                                                                       long long* __restrict__ cyc, int nit) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr bool split = (MODE & M_SPLIT) != 0;
  const bool computer = !split || wid < 4;
  const bool memer = !split || wid >= 4;
  const int mw = split ? wid - 4 : wid;  // memory-wave index 0..3
  constexpr int NJ = split ? 3 : 8;
  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 fa, fb;
#pragma unroll
  for (int e = 0; e < 8; ++e) { fa[e] = (short)(0x3f80 + lane + e); fb[e] = (short)(0x3f00 + lane * 3 + e); }
  s16x8 rd[2];
  u32x4 ga[8], gb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { ga[e] = u32x4{1u, 2u, 3u, (unsigned)lane}; gb[e] = ga[e]; }
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);

  long long t0 = 0;
  if (computer && lane == 0) t0 = __builtin_amdgcn_s_memtime();
  const unsigned lane_off = (unsigned)lane * 16u;
  for (int it = 0; it < nit; it += 2) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const long gbase = ((long)(it + half) * 32768L) % region;
      lds_char* stg = smem + ((it + half) & 3) * 32768;
      fence();
      if constexpr ((MODE & M_PRIO) != 0) { if (computer) __builtin_amdgcn_s_setprio(1); }
      const bool mem_here = memer && (!(MODE & M_ONE) || mw == 0);
      iteration<MODE, 0>(acc, fa, fb, rd, ga, gb, src, gbase, smem, stg, it, half, mw, computer, mem_here, lane_off, rsrc);
      fence();
      // end of iteration: keep one iteration of loads in flight, drain LDS ops, one barrier
      if (memer) {
        if constexpr ((MODE & (M_DMA | M_GLD | M_BUF)) != 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        if constexpr ((MODE & (M_DSW | M_DSR)) != 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      fence();
      __builtin_amdgcn_s_barrier();
      fence();
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  long long t1 = 0;
  if (computer && lane == 0) t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  if (computer) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) { asm volatile("" : "+a"(acc[i][j])); s += acc[i][j][0] + acc[i][j][3]; }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr ((MODE & M_GLD) != 0) s += (float)(ga[e][0] ^ gb[e][1]);
    if constexpr ((MODE & M_DSR) != 0) s += (float)rd[e & 1][e];
  }
  sink[blockIdx.x * blockDim.x + tid] = s;
  if (computer && lane == 0) cyc[blockIdx.x * 4 + wid] = t1 - t0;
}

template <int MODE>
void run(const char* name, const char* src, long region, float* sink, long long* cyc, int nwg, int nit) {
  auto kern = probe<MODE>;
  const int smem = 4 * 32768;
  CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  const int nthr = (MODE & M_SPLIT) ? 512 : 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(nwg), dim3(nthr), smem, 0, src, region, sink, cyc, nit);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(kern, dim3(nwg), dim3(nthr), smem, 0, src, region, sink, cyc, nit);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  std::vector<long long> h(nwg * 4);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  const double med = (double)h[h.size() / 2];
  const double mfma_per_wave = 64.0 * nit;
  const double flops = (double)nwg * 4 * mfma_per_wave * 16 * 16 * 32 * 2;
  printf("%-34s region %6.1f MB  cyc/MFMA %6.2f (min %6.2f max %6.2f)  wall %8.3f ms  %7.1f TF\n", name,
         region / 1048576.0, med / mfma_per_wave, h[0] / mfma_per_wave, h.back() / mfma_per_wave, ms,
         flops / (ms * 1e-3) / 1e12);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int nit = argc > 1 ? atoi(argv[1]) : 2000;
  const int nwg = 256;
  const long big = 512L << 20;
  char* src;
  float* sink;
  long long* cyc;
  CHECK(hipMalloc(&src, big + (1 << 20)));
  CHECK(hipMemset(src, 0x3c, big + (1 << 20)));
  CHECK(hipMalloc(&sink, nwg * 512 * 4));
  CHECK(hipMalloc(&cyc, nwg * 4 * 8));
  for (long region : {64L << 20}) {
    run<0>("mfma only", src, region, sink, cyc, nwg, nit);
    run<M_DSR>("+16 ds_read_b128", src, region, sink, cyc, nwg, nit);
    run<M_DSR | M_STAG>("+16 ds_read_b128 STAG", src, region, sink, cyc, nwg, nit);
    run<M_DSR | M_ONE>("+16 ds_read_b128 wave0 only", src, region, sink, cyc, nwg, nit);
    run<M_DMA>("+8 glds", src, region, sink, cyc, nwg, nit);
    run<M_DMA | M_STAG>("+8 glds STAG", src, region, sink, cyc, nwg, nit);
    run<M_DMA | M_ONE>("+8 glds wave0 only", src, region, sink, cyc, nwg, nit);
    run<M_GLD>("+8 gld", src, region, sink, cyc, nwg, nit);
    run<M_GLD | M_STAG>("+8 gld STAG", src, region, sink, cyc, nwg, nit);
    run<M_DSW>("+8 ds_write", src, region, sink, cyc, nwg, nit);
    run<M_DSW | M_STAG>("+8 ds_write STAG", src, region, sink, cyc, nwg, nit);
    run<M_DSR | M_DMA>("+16 dsr +8 glds", src, region, sink, cyc, nwg, nit);
    run<M_DSR | M_DMA | M_STAG>("+16 dsr +8 glds STAG", src, region, sink, cyc, nwg, nit);
    run<M_DSR | M_GLD | M_DSW>("+16 dsr +8 gld +8 dsw", src, region, sink, cyc, nwg, nit);
    run<M_DSR | M_GLD | M_DSW | M_STAG>("+16 dsr +8 gld +8 dsw STAG", src, region, sink, cyc, nwg, nit);
    run<M_SPLIT>("8w: mfma only", src, region, sink, cyc, nwg, nit);
    run<M_SPLIT | M_DMA>("8w: partner +8 glds", src, region, sink, cyc, nwg, nit);
    run<M_SPLIT | M_DMA | M_STAG>("8w: partner +8 glds STAG", src, region, sink, cyc, nwg, nit);
    run<M_SPLIT | M_DMA | M_ONE>("8w: partner0 only +8 glds", src, region, sink, cyc, nwg, nit);
  }
  printf("done\n");
  return 0;
}
