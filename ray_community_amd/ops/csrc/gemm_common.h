// Shared pieces of the gfx950 bf16 GEMM kernels (gemm.hip: 8-wave two-stage ring; gemm4.hip:
// 4-wave, one wave per SIMD, 128x128 per wave): operand tile staging by LDS-DMA into lane-linear
// swizzled images, MFMA fragment reads (ds_read_b128 / ds_read_b64_tr_b16), tile order.
#pragma once
#include "common.h"

namespace rca_gemm {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) s16x8 lds_s16x8;

constexpr int BM = 256, BN = 256, NTHR = 512;
constexpr int GROUP_M = 8;

__device__ __forceinline__ int kswz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// Stage one 256 x BK operand tile into a lane-linear LDS image: 256*BK*2/1024 one-KB blocks, one
// global_load_lds (64 lanes x 16 B) each, dealt round-robin over the NW waves.
template <bool KMAJ, int BK, int NW = 8>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ g, long ld, int o0, int k0, lds_char* dst,
                                           int wid, int lane) {
  constexpr int CPR = BK / 8;  // 16-B chunks per k-contiguous row
  constexpr int RSH = CPR == 8 ? 1 : 2;  // rows sharing a 256-B bank row differ in (row >> RSH)
#pragma unroll
  for (int i = 0; i < (BK / 2) / NW; ++i) {
    const int blk = i * NW + wid;         // 1 KB block of the image this wave instruction fills
    const int p = blk * 64 + lane;        // 16-B chunk index in the image
    const bf16_t* src;
    if constexpr (!KMAJ) {                // [256 outer][CPR chunks]
      const int row = p / CPR, c = (p % CPR) ^ ((row >> RSH) & (CPR - 1));
      src = g + (long)(o0 + row) * ld + k0 + c * 8;
    } else {                              // [BK k][32 chunks]
      const int kr = p >> 5, c = (p & 31) ^ kswz(kr);
      src = g + (long)(k0 + kr) * ld + o0 + c * 8;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + blk * 1024),
                                     16, 0, 0);
  }
}

// MFMA operand fragment: 16 outer indices (ob*16 + lane&15) x 8 k (kk*32 + 8*(lane>>4) + 0..7).
template <bool KMAJ, int BK>
__device__ __forceinline__ bf16x8_t load_frag(const lds_char* t, int ob, int kk, int lane) {
  constexpr int CPR = BK / 8;
  constexpr int RSH = CPR == 8 ? 1 : 2;
  if constexpr (!KMAJ) {
    const int row = ob * 16 + (lane & 15);
    const int c = (kk * 4 + (lane >> 4)) ^ ((row >> RSH) & (CPR - 1));
    s16x8 v = *(const lds_s16x8*)(t + row * (BK * 2) + c * 16);
    return __builtin_bit_cast(bf16x8_t, v);
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int k1 = kk * 32 + 8 * g + q, k2 = k1 + 4;
    const int c = ob * 2 + (p >> 1), h = (p & 1) * 8;
    s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + k1 * 512 + ((c ^ kswz(k1)) << 4) + h));
    s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + k2 * 512 + ((c ^ kswz(k2)) << 4) + h));
    s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


// Tile order: XCD-contiguous ranges (xcd_remap), then GROUP_M-row groups inside, so the ~32
// blocks co-resident on one XCD share A and B panels through that XCD's L2.
__device__ __forceinline__ void tile_origin(int bid, int M, int N, int& m0, int& n0) {
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  const int lin = xcd_remap(bid, nwg);
  const int gsz = GROUP_M * ntn, gi = lin / gsz, fm = gi * GROUP_M;
  const int gm = min(ntm - fm, GROUP_M), r = lin % gsz;
  m0 = (fm + r % gm) * BM;
  n0 = (r / gm) * BN;
}

// bf16x4 epilogue store of one accumulator (4 consecutive n of one m), optionally adding C.
template <bool ACC>
__device__ __forceinline__ void store4(bf16_t* __restrict__ C, long off, const f32x4 v) {
  unsigned long long* dst = (unsigned long long*)(C + off);
  float v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
  if constexpr (ACC) {
    const unsigned long long old = *dst;
    v0 += bf2f((bf16_t)(old & 0xffff));
    v1 += bf2f((bf16_t)((old >> 16) & 0xffff));
    v2 += bf2f((bf16_t)((old >> 32) & 0xffff));
    v3 += bf2f((bf16_t)((old >> 48) & 0xffff));
  }
  *dst = (unsigned long long)f2bf(v0) | ((unsigned long long)f2bf(v1) << 16) |
         ((unsigned long long)f2bf(v2) << 32) | ((unsigned long long)f2bf(v3) << 48);
}

}  // namespace rca_gemm
