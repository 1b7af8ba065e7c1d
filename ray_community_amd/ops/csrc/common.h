// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of ray_community_amd.
// Wave = 64 lanes; all vector memory access is 16 B per lane (8 x bf16 or 4 x f32).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define RCA_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;  // raw bf16 bits
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

static constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((unsigned)u) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  // plain conversion: hipcc -O3 lowers this to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving)
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&b);
}

// unpack a 16-byte vector of 8 bf16 into f32
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned w = v[i];
    f[2 * i] = __uint_as_float(w << 16);
    f[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = (unsigned)f2bf(f[2 * i]) | ((unsigned)f2bf(f[2 * i + 1]) << 16);
  }
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats. Result broadcast to all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// XCD-aware bijective remap of a 1-D block id (MI355X: 8 XCDs dealt round-robin).
// Consecutive logical ids land on the same XCD so that neighbouring tiles share an L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// XCD-grouped work mapping: a grid of ngroups x per workgroups where the `per` workgroups of one
// group stream the same operand (e.g. the K/V or Q/dO of one (batch, kv-head)). When ngroups is a
// multiple of 8, every group lives on ONE XCD (hardware deals block ids round-robin over the 8
// XCDs) and its items are dispatched in item order there, so concurrently resident workgroups of a
// group read the stream through one L2 instead of eight. Otherwise falls back to xcd_remap order
// (item-major). Bijective in both cases.
__device__ __forceinline__ void xcd_group_map(int bid, int ngroups, int per, int& group, int& item) {
  if ((ngroups & 7) == 0) {
    const int gpx = ngroups >> 3, xcd = bid & 7, slot = bid >> 3;
    group = xcd * gpx + slot % gpx;
    item = slot / gpx;
  } else {
    const int lid = xcd_remap(bid, ngroups * per);
    group = lid % ngroups;
    item = lid / ngroups;
  }
}
