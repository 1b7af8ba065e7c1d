// Shared device helpers of the gfx950 flash-attention kernels (attention.hip: forward, delta,
// dQ; attention_dkdv.hip: dK/dV). Everything lives in an anonymous namespace: each translation
// unit gets its own copy (the two files are compiled with different register-form flags,
// ops/build.py FILE_FLAGS).
#pragma once
#include "common.h"

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// LDS image of a [rows][D] bf16 tile (cdna_hip_programming.md T11 image (a)): 8-row x 32-column
// subtiles of 512 B, chunk XOR-swizzled inside each 64-B row piece. Both operand reads the kernels
// need are conflict-free on it and AFFINE in the loop indices, so every LDS read is one of two
// per-lane base registers plus an immediate offset:
//   row operand   (rows l32 + 32t, chunk 2kk + h):            rb[kk&1] + 4*G8*t + 512*(kk>>1)
//   transposed op (rows R0 + 4h + q (+8), cols 32db+16g+4p):  tb[rd]   + G8*(R0/8 + rd) + 512*db
template <int D>
struct Img {
  static constexpr int G8 = D * 16;  // bytes per 8-row group
  __device__ static __forceinline__ int off(int row, int ch) {
    return G8 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
  }
  __device__ static __forceinline__ int row_base(int l32, int h, int e) {
    return G8 * (l32 >> 3) + 64 * (l32 & 7) + 16 * ((2 * e + h) ^ ((l32 >> 2) & 3));
  }
  __device__ static __forceinline__ int tr_base(int lane, int rd) {
    const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    return 64 * (4 * h + q) + 16 * ((2 * g + (p >> 1)) ^ ((h + 2 * rd) & 3)) + 8 * (p & 1);
  }
};

__device__ __forceinline__ bf16x8_t lds_b128(const char* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4*>(p));
}

// transposed 8-element MFMA operand: two ds_read_b64_tr_b16 (k-steps j = 0..3 and 4..7)
__device__ __forceinline__ bf16x8_t lds_tr8(const char* p0, const char* p1) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
  s16x8 r = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, r);
}

// lds_tr8 as inline asm, for kernels that stage tiles by LDS-DMA: hipcc drains every in-flight
// DMA (vmcnt(0)) before a ds_read_tr16 builtin it cannot prove disjoint from the DMA target,
// which would serialise the next tile's prefetch with this tile's math. The asm read is invisible
// to hipcc's counters: call lds_tr_settle() on the results before they are used (it waits
// lgkmcnt(0) and redefines them, so no consumer is scheduled above the wait).
__device__ __forceinline__ bf16x8_t lds_tr8_asm(const char* p0, const char* p1) {
  s16x4 a, b;
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3"
               : "=&v"(a), "=&v"(b)
               : "v"((unsigned)(__UINTPTR_TYPE__)p0), "v"((unsigned)(__UINTPTR_TYPE__)p1));
  s16x8 r = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, r);
}

template <int N>
__device__ __forceinline__ void lds_tr_settle(bf16x8_t (&fr)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(fr[i]));
}

// registers 8s..8s+7 of an accumulator -> bf16 MFMA operand (k-step s)
__device__ __forceinline__ bf16x8_t acc_to_bf16(const f32x16& x, int s) {
  bf16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[8 * s + j];
  return r;
}

// Pin a register operand loaded from global memory: the asm "redefines" it after its load has
// landed, so hipcc's loop-merged s_waitcnt bookkeeping stops treating it as pending inside the
// main loop (otherwise every tile's first MFMAs wait vmcnt for the NEXT tile's staging loads).
__device__ __forceinline__ void settle(bf16x8_t& v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ bf16x8_t gload8(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4*>(p));
}

// store 4 consecutive fp32 as bf16 (8 bytes)
__device__ __forceinline__ void store4(bf16_t* p, float a, float b, float c, float d) {
  uint2 v;
  v.x = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
  v.y = (unsigned)f2bf(c) | ((unsigned)f2bf(d) << 16);
  *reinterpret_cast<uint2*>(p) = v;
}

// ---------------------------------------------------------------------------------------------
// [ROWS x D] tile staging HBM -> registers -> LDS. The per-lane parts of both addresses are
// computed once; per tile only a wave-uniform base changes (global) or an immediate (LDS).
template <int D, int ROWS>
struct Stage {
  static constexpr int NCH = D / 8, N = ROWS * NCH / kThreads, RPI = kThreads / NCH;
  u32x4 r[N];
  __amdgpu_buffer_rsrc_t rsrc;  // whole [rows x stride] extent of one (batch, head): wave-uniform
  int voff, loff;
  __device__ __forceinline__ void init(const bf16_t* base, long stride, int rows, int tid, int cols = D) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base), (short)0,
                                             (int)((long)(rows - 1) * stride * 2 + cols * 2), 0x00020000);
    // thread -> (row, chunk): each 8-lane group of a ds_write_b128 (the unit that conflicts,
    // bank = (a/4) mod 32) stores chunks 0-3 of TWO consecutive rows, i.e. 8 distinct 16-B slots
    // of a 128-B bank window in the image; row-major tid / NCH put chunks 0-3 and 4-7 of one row
    // in a group, which alias (512-B subtile stride) -> 2-way conflicts on every staging store.
    // Global loads stay coalesced (each wave covers whole 2*NCH*16-B row pairs).
    constexpr int LG = NCH == 16 ? 2 : (NCH == 8 ? 1 : 0);  // log2(NCH / 4)
    const int ch = (tid & 3) | (((tid >> 3) & ((NCH >> 2) - 1)) << 2);
    const int row = ((tid >> 2) & 1) | ((tid >> (3 + LG)) << 1);
    voff = (int)(row * stride * 2 + ch * 16);
    loff = Img<D>::off(row, ch);
  }
  __device__ __forceinline__ void load(int row0, long stride, int extra = 0) {
#pragma unroll
    for (int i = 0; i < N; ++i)
      r[i] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, (int)((row0 + i * RPI) * stride * 2) + extra, 0));
  }
  __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<u32x4*>(lds + loff + i * (RPI / 8) * Img<D>::G8) = r[i];
  }
};

// [ROWS x D] tile staging HBM -> LDS directly (buffer_load ... lds, no register round trip and
// no ds_write): the image above is cut into 1-KB blocks, each one 64-lane DMA whose lane l lands
// at byte 16 l of the block, so each lane fetches the (row, chunk) the image keeps there. Block b
// (of D/64 per 8-row group): group b / (D/64), subtile pair b % (D/64); lane l -> row
// 8 group + ((l >> 2) & 7), chunk 4 (2 sub + (l >> 5)) + ((l & 3) ^ ((2 group + ((l >> 4) & 1)) & 3)).
// A DMA instruction reads 8 rows x 128 contiguous bytes (whole cache lines). Wave w issues
// blocks w, w + 4, ...; the per-lane offsets depend on the block only through (group parity, sub),
// so they are computed once and every tile changes one scalar offset.
template <int D, int ROWS>
struct DmaStage {
  static constexpr int BPG = D / 64, NBLK = ROWS / 8 * BPG, NB = NBLK / 4;
  static_assert(NB >= 1 && NBLK % 4 == 0, "tile must split into 4 waves of 1-KB blocks");
  __amdgpu_buffer_rsrc_t rsrc;
  int voff[NB];
  int wave;
  __device__ __forceinline__ void init(const bf16_t* base, long stride, int rows, int tid, int cols = D) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base), (short)0,
                                             (int)((long)(rows - 1) * stride * 2 + cols * 2), 0x00020000);
    const int l = tid & 63;
    wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int b = wave + 4 * i, group = b / BPG, sub = b % BPG;
      const int row = 8 * group + ((l >> 2) & 7);
      const int ch = 4 * (2 * sub + (l >> 5)) + ((l & 3) ^ ((2 * group + ((l >> 4) & 1)) & 3));
      voff[i] = (int)(row * stride * 2 + ch * 16);
    }
  }
  // one of this wave's NB 1-KB pieces (hand-scheduled kernels spread them over MFMA phases)
  __device__ __forceinline__ void issue_one(int i, int row0, long stride, char* lds) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds + (wave + 4 * i) * 1024),
                                             16, voff[i], __builtin_amdgcn_readfirstlane((int)(row0 * stride * 2)), 0, 0);
  }
  // DMA rows row0 .. row0 + ROWS - 1 (column offset ``extra`` bytes) into the image at ``lds``
  __device__ __forceinline__ void issue(int row0, long stride, char* lds, int extra = 0) const {
    const int soff = (int)(row0 * stride * 2) + extra;
#pragma unroll
    for (int i = 0; i < NB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(lds + (wave + 4 * i) * 1024), 16, voff[i], soff, 0, 0);
  }
};

__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int V>
using IC = std::integral_constant<int, V>;

// ---------------------------------------------------------------------------------------------
// Cross-half (lane <-> lane^32) reductions on the VALU (v_permlane32_swap; no LDS round trip).
__device__ __forceinline__ float xhalf_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// max of three in plain C: hipcc emits one v_max3_f32 per call on MFMA results (no canonicalising
// v_max pairs) AND counts the MFMA -> VALU read hazard wait states. An inline-asm v_max3 here was
// issued with NO wait states behind the S^T MFMA chain (the hazard recognizer does not look into
// asm operands), so it read stale accumulator VGPRs: a timing-dependent row max, i.e. a
// run-to-run nondeterministic forward.
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

__device__ __forceinline__ float max16(const f32x16& s, float init) {
  float a = max3f(init, s[0], s[1]), b = max3f(s[2], s[3], s[4]);
  a = max3f(a, s[5], s[6]);
  b = max3f(b, s[7], s[8]);
  a = max3f(a, s[9], s[10]);
  b = max3f(b, s[11], s[12]);
  a = max3f(a, s[13], s[14]);
  return max3f(a, b, s[15]);
}

}  // namespace
