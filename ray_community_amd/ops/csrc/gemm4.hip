// bf16 GEMM for gfx950, one wave per SIMD: 256x256x64 block tile, 4 waves of 128x128 each.
//
//   C[M][N] (+)= sum_k A(m, k) * B(n, k)     (layouts as gemm.hip: row = k-contiguous, kmaj = k-outer)
//
// Why this shape (MI355X_MICROARCH.md "Register files", "Two waves per SIMD"): a 128x128 wave
// tile is 8 x 8 accumulators of v_mfma_f32_16x16x32_bf16 = 256 accumulator registers, which fit
// the AGPR half of a one-wave-per-SIMD register file (512 per lane) and leave the VGPR half for
// TWO full fragment sets (k-slices kk = 0 and 1 of a 64-deep K-tile: 2 x 16 fragments x 4 VGPRs).
// Each fragment feeds 8 MFMAs (vs 4 or 2 in the 8-wave 128x64 tiling), halving LDS read traffic
// per MFMA, and the next k-slice's fragments are read while the current one's 64 MFMAs run, so
// the matrix pipe never waits on LDS latency and there is no partner wave to share it with.
// (This file is built WITHOUT -amdgpu-mfma-vgpr-form: the accumulators must live in AGPRs.)
//
// Per K-tile t (stage s = t & 1 of a two-stage, 2 x 64 KB LDS ring; images as gemm.hip):
//   phase A: ds_read the kk=1 fragments (F1); 64 MFMAs on the kk=0 fragments (F0);
//   phase B: 32 MFMAs on F1; lgkmcnt(0) + vmcnt(0) + barrier (K-tile t+1 landed for every wave,
//            and every wave is done reading stage s); LDS-DMA of K-tile t+2 into stage s;
//            ds_read F0 of K-tile t+1; 32 more MFMAs on F1.
// One workgroup barrier per K-tile.
#include "common.h"
#include "gemm_common.h"

namespace {
using namespace rca_gemm;

constexpr int NT4 = 256;            // 4 waves
constexpr int TB = 256 * 64 * 2;    // one 256 x 64 bf16 operand tile (32 KB)
constexpr int STG = 2 * TB;         // A tile | B tile

// Stage one 256 x 64 operand tile (32 one-KB LDS-DMA blocks, 8 per wave) into the image layout of
// gemm_common.h's stage_tile, with the addressing split into a wave-uniform base (SGPRs) plus one
// per-lane 32-bit byte offset (k-outer: two, by block parity), so 16 in-flight DMAs cost two or
// three VGPRs instead of a 64-bit address each.
//   k-contiguous: block b = 4i + wid holds rows 8b .. 8b+7; the swizzle (row>>1)&7 of lane l is
//                 (4*wid + (l>>4)) & 7 for every i  ->  src = g + (o0 + 8*wid)*ld + k0 + 32*i*ld + off
//   k-outer:      block b holds k-rows 2b, 2b+1; kswz(k) depends on i only through i & 1.
template <bool KMAJ>
struct Stage4 {
  unsigned off[2];
  __device__ __forceinline__ Stage4(long ld, int wid, int lane) {
    if constexpr (!KMAJ) {
      const int c = (lane & 7) ^ ((4 * wid + (lane >> 4)) & 7);
      off[0] = off[1] = (unsigned)(((lane >> 3) * ld + c * 8) * 2);
    } else {
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const int kr = 8 * par + 2 * wid + (lane >> 5);
        const int c = (lane & 31) ^ kswz(kr);
        off[par] = (unsigned)(((lane >> 5) * ld + c * 8) * 2);
      }
    }
  }
  __device__ __forceinline__ void issue_one(int i, const bf16_t* __restrict__ g, long ld, int o0, int k0,
                                            lds_char* dst, int wid) const {
    const char* base;
    if constexpr (!KMAJ) base = (const char*)(g + (long)(o0 + 8 * wid + 32 * i) * ld + k0);
    else base = (const char*)(g + (long)(k0 + 2 * wid + 8 * i) * ld + o0);
    __builtin_amdgcn_global_load_lds((const void*)(base + off[i & 1]),
                                     (__attribute__((address_space(3))) void*)(dst + (4 * i + wid) * 1024), 16, 0, 0);
  }
  __device__ __forceinline__ void issue(const bf16_t* __restrict__ g, long ld, int o0, int k0, lds_char* dst,
                                        int wid) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) issue_one(i, g, ld, o0, k0, dst, wid);
  }
};

// Fragment reads and MFMAs are inline asm. hipcc's own handling of this loop was the limit:
// with the builtins it (a) drained every in-flight LDS-DMA (vmcnt(0)) before ds_read_b64_tr_b16
// reads it could not prove disjoint from the DMA target, and (b) shuffled the 256 loop-carried
// accumulators through spare AGPRs. Here the compiler only allocates registers: each MFMA is a
// non-volatile asm tying its accumulator ("+a"), each LDS read a volatile asm, and the kernel
// counts lgkmcnt itself at phase boundaries (the reads of a phase are consumed one phase later).
__device__ __forceinline__ unsigned lds_off(const lds_char* p) { return (unsigned)(__UINTPTR_TYPE__)p; }

template <bool KMAJ>
__device__ __forceinline__ bf16x8_t frag_asm(const lds_char* t, int ob, int kk, int lane) {
  if constexpr (!KMAJ) {
    const int row = ob * 16 + (lane & 15);
    const int c = (kk * 4 + (lane >> 4)) ^ ((row >> 1) & 7);
    s16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_off(t + row * 128 + c * 16)));
    return __builtin_bit_cast(bf16x8_t, v);
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int k1 = kk * 32 + 8 * g + q;
    const int c = ob * 2 + (p >> 1), h = (p & 1) * 8;
    // k2 = k1 + 4 has the same kswz (its bit 3 is k1's): the second read is 4 k-rows (2 KB) on
    s16x4 a, b;
    const unsigned addr = lds_off(t + k1 * 512 + ((c ^ kswz(k1)) << 4) + h);
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:2048"
                 : "=&v"(a), "=&v"(b) : "v"(addr));
    s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

template <bool AK, bool BKM>
__device__ __forceinline__ void read_frags(const lds_char* st, int kk, int wr, int wc, int lane, bf16x8_t (&af)[8],
                                           bf16x8_t (&bf)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) af[i] = frag_asm<AK>(st, wr * 8 + i, kk, lane);
#pragma unroll
  for (int j = 0; j < 8; ++j) bf[j] = frag_asm<BKM>(st + TB, wc * 8 + j, kk, lane);
}

template <int I0, int I1>
__device__ __forceinline__ void mfma_rows(f32x4 (&acc)[8][8], const bf16x8_t (&af)[8], const bf16x8_t (&bf)[8]) {
#pragma unroll
  for (int i = I0; i < I1; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(bf[j]), "v"(af[i]));
}

template <int N>
__device__ __forceinline__ void mfma_n(f32x4 (&acc)[8][8], const bf16x8_t (&af)[8], const bf16x8_t (&bf)[8], int i,
                                       int j0) {
#pragma unroll
  for (int j = j0; j < j0 + N; ++j)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(bf[j]), "v"(af[i]));
}

// The asm MFMAs are invisible to the hazard recognizer: before the epilogue reads the
// accumulators, cover the last MFMAs' write latency with s_nops, then pass every accumulator
// through an empty asm that redefines it, so no AGPR read can be scheduled ahead of the nops.
__device__ __forceinline__ void drain_acc(f32x4 (&acc)[8][8]) {
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
}

__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void fence_sched() { __builtin_amdgcn_sched_barrier(0); }

template <bool AK, bool BKM, bool ACC, int DIAG = 0>
__global__ __launch_bounds__(NT4, 1) void gemm4_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                       bf16_t* __restrict__ C, int M, int N, int K, long lda,
                                                       long ldb, long ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  tile_origin(blockIdx.x, M, N, m0, n0);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = K / 64;
  const Stage4<AK> sa(lda, wid, lane);
  const Stage4<BKM> sb(ldb, wid, lane);
  sa.issue(A, lda, m0, 0, smem, wid);
  sb.issue(B, ldb, n0, 0, smem + TB, wid);
  wait_vmcnt<0>();
  fence_sched();
  __builtin_amdgcn_s_barrier();
  fence_sched();
  {
    const int k1 = min(1, nt - 1) * 64;
    sa.issue(A, lda, m0, k1, smem + STG, wid);
    sb.issue(B, ldb, n0, k1, smem + STG + TB, wid);
  }

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
  read_frags<AK, BKM>(smem, 0, wr, wc, lane, f0a, f0b);
  wait_lgkm0();

  // The loop body is ONE basic block (no branches): past the end the DMA re-reads K-tile nt-1
  // and F0 reads the idle stage (harmless: nothing reads either afterwards). Scheduling fences
  // between every small group pin the interleave of LDS reads, LDS-DMA issue and MFMAs.
  // The DMA of K-tile t+2 goes out right after iteration t's barrier, into the stage K-tile t
  // just vacated (every wave's F0(t) and F1(t) reads were retired before that barrier), so each
  // tile is in flight for a whole iteration (~2,000 MFMA cycles) before it is waited for.
  for (int t = 0; t < nt; ++t) {
    const lds_char* st = smem + (t & 1) * STG;
    const lds_char* nx = smem + ((t + 1) & 1) * STG;
    const int k2 = min(t + 2, nt - 1) * 64;
    // ---- phase A: the 16 F1 fragment reads spread over the first 64 MFMAs (on F0), one per 4
    fence_sched();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (u < 8) f1a[u] = frag_asm<AK>(st, wr * 8 + u, 1, lane);
      else f1b[u - 8] = frag_asm<BKM>(st + TB, wc * 8 + u - 8, 1, lane);
      mfma_n<4>(acc, f0a, f0b, u >> 1, (u & 1) * 4);
      fence_sched();
    }
    wait_lgkm0();  // F1 resident
    fence_sched();
    // ---- phase B: 32 MFMAs on F1 rows 0-3; K-tile t+1 landed everywhere and stage t&1 vacated;
    //      then, beside the 32 MFMAs on rows 4-7, one F0 fragment read of K-tile t+1 and one
    //      LDS-DMA block of K-tile t+2 (into stage t&1) per 2 MFMAs
    mfma_rows<0, 4>(acc, f1a, f1b);
    fence_sched();
    if constexpr (DIAG != 2) wait_vmcnt<0>();
    fence_sched();
    __builtin_amdgcn_s_barrier();
    fence_sched();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (u < 8) {
        f0a[u] = frag_asm<AK>(nx, wr * 8 + u, 0, lane);
        if constexpr (DIAG != 1) sa.issue_one(u, A, lda, m0, k2, (lds_char*)st, wid);
      } else {
        f0b[u - 8] = frag_asm<BKM>(nx + TB, wc * 8 + u - 8, 0, lane);
        if constexpr (DIAG != 1) sb.issue_one(u - 8, B, ldb, n0, k2, (lds_char*)st + TB, wid);
      }
      mfma_n<2>(acc, f1a, f1b, 4 + (u >> 2), (u & 3) * 2);
      fence_sched();
    }
    wait_lgkm0();  // F0 of K-tile t+1 resident
    fence_sched();
  }
  wait_vmcnt<0>();
  // the asm MFMAs are invisible to the hazard recognizer: cover the last ones' write latency
  // before the epilogue reads the accumulators
  drain_acc(acc);

  // epilogue: acc[i][j] reg r = C[m0 + wr*128 + i*16 + (lane&15)][n0 + wc*128 + j*16 + 4*(lane>>4) + r]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = m0 + wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) store4<ACC>(C, m * ldc + n0 + wc * 128 + j * 16 + 4 * (lane >> 4), acc[i][j]);
  }
}

// ------------------------------------------------------------------------------------------------
// Slice-ring variant (RCA_GEMM_VARIANT=3): same 4 waves x 128x128, but K advances in 32-deep
// SLICES through a 4-stage LDS ring (4 x 32 KB). Measured on the 64-deep two-stage loop above:
// without its LDS-DMA it runs 1.39-1.82 PF, with it 1.15-1.31 -- issuing 16 DMAs per wave in
// the half-iteration between the barrier and the next tile's first read stalls the only wave
// that feeds the SIMD's matrix pipe (a DMA costs the issuing wave far more than the 2 x 16-cycle
// MFMA gap it was given). In the ring a stage frees up one slice after it was read, so the
// DMA of slice s+3 can be spread over the WHOLE of slice s: 8 DMAs beside 64 MFMAs (one per 8
// MFMAs), each in flight ~2 slices before it is waited for.
//   iteration s (stage s & 3):  vmcnt(8) [own DMA of slice s+1 landed; slice s+2 in flight]
//     + barrier [everyone's slice s+1 landed; everyone's reads of slice s-1 retired]
//     -> 16 groups of { 1 F(s+1) fragment read, [1 DMA of slice s+3 -> stage (s+3)&3], 4 MFMA on F(s) }
//     -> lgkmcnt(0) [F(s+1) resident]
// 64-B k-contiguous rows: chunk' = chunk ^ ((-(row >> 2)) & 3) makes every ds_read_b128 lane
// group of the 16x16x32 fragment read (16 rows, 2 chunks) hit 16 distinct 16-B bank slots.
constexpr int SLB = 256 * 32 * 2;  // one operand slice (16 KB)
constexpr int SST = 2 * SLB;       // stage: A slice | B slice

__device__ __forceinline__ int swz32(int row) { return (-(row >> 2)) & 3; }

template <bool KMAJ>
struct SliceStage {
  unsigned off[2];  // per-lane global byte offset from the step's wave-uniform base (by step parity)
  __device__ __forceinline__ SliceStage(long ld, int wid, int lane) {
    if constexpr (!KMAJ) {  // block b = 4i + wid: rows 16b .. 16b+15 (64-B rows, 4 chunks)
      const int row = (lane >> 2), c = (lane & 3) ^ swz32(16 * wid + row);
      off[0] = off[1] = (unsigned)((row * ld + c * 8) * 2);
    } else {  // block b = 4i + wid: k-rows 8i + 2w + (l>>5); kswz sees i only through bit 3 (i & 1)
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const int kr = 8 * par + 2 * wid + (lane >> 5), c = (lane & 31) ^ kswz(kr);
        off[par] = (unsigned)(((lane >> 5) * ld + c * 8) * 2);
      }
    }
  }
  // step i (0..3) of a 16-KB slice: LDS block 4i + wid
  __device__ __forceinline__ void issue(int i, const bf16_t* __restrict__ g, long ld, int o0, int k0, lds_char* dst,
                                        int wid) const {
    const char* base;
    if constexpr (!KMAJ) base = (const char*)(g + (long)(o0 + 16 * wid + 64 * i) * ld + k0);
    else base = (const char*)(g + (long)(k0 + 2 * wid + 8 * i) * ld + o0);
    __builtin_amdgcn_global_load_lds((const void*)(base + off[i & 1]),
                                     (__attribute__((address_space(3))) void*)(dst + (4 * i + wid) * 1024), 16, 0, 0);
  }
};

template <bool KMAJ>
__device__ __forceinline__ bf16x8_t sfrag(const lds_char* t, int ob, int lane) {
  if constexpr (!KMAJ) {
    const int row = ob * 16 + (lane & 15);
    const int c = (lane >> 4) ^ swz32(row);
    s16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_off(t + row * 64 + c * 16)));
    return __builtin_bit_cast(bf16x8_t, v);
  } else {
    return frag_asm<true>(t, ob, 0, lane);  // [32 k][256] with 512-B rows: the kk = 0 read
  }
}

// lgkmcnt(n) for a value that is a constant once the surrounding loop is unrolled (the switch
// folds away); n >= 16 needs no wait (the counter holds at most 15 pending LDS reads here).
__device__ __forceinline__ void wait_lgkm_upto(int n) {
  switch (n) {
#define RCA_W(k) case k: asm volatile("s_waitcnt lgkmcnt(" #k ")" ::: "memory"); break;
    RCA_W(0) RCA_W(1) RCA_W(2) RCA_W(3) RCA_W(4) RCA_W(5) RCA_W(6) RCA_W(7)
    RCA_W(8) RCA_W(9) RCA_W(10) RCA_W(11) RCA_W(12) RCA_W(13) RCA_W(14) RCA_W(15)
#undef RCA_W
    default: break;
  }
}

// PW (variant 5): no lgkmcnt(0) drain at the end of a slice. The next slice's fragments are read
// B first, then A, and before group u each wave waits only until the reads that group's MFMAs
// consume have landed (counted: the reads of earlier groups of this slice are younger, so they may
// stay in flight). Variant 3 drained every fragment read and then met the barrier with the matrix
// pipe idle for the LDS latency once per slice.
template <bool AK, bool BKM, bool ACC, bool PW = false>
__global__ __launch_bounds__(NT4, 1) void gemm4s_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                        bf16_t* __restrict__ C, int M, int N, int K, long lda,
                                                        long ldb, long ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  tile_origin(blockIdx.x, M, N, m0, n0);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ns = K / 32;  // even (K % 64 == 0)
  const SliceStage<AK> sa(lda, wid, lane);
  const SliceStage<BKM> sb(ldb, wid, lane);
  auto dma = [&](int sl, int i) {  // step i of slice sl (clamped: past the end re-reads the last)
    const int k0 = min(sl, ns - 1) * 32;
    lds_char* st = smem + (sl & 3) * SST;
    if (i < 4) sa.issue(i, A, lda, m0, k0, st, wid);
    else sb.issue(i - 4, B, ldb, n0, k0, st + SLB, wid);
  };
#pragma unroll
  for (int sl = 0; sl < 3; ++sl)
#pragma unroll
    for (int i = 0; i < 8; ++i) dma(sl, i);
  wait_vmcnt<16>();  // slice 0 (own part) landed
  fence_sched();
  __builtin_amdgcn_s_barrier();
  fence_sched();
  bf16x8_t xa[8], xb[8], ya[8], yb[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    xa[u] = sfrag<AK>(smem, wr * 8 + u, lane);
    xb[u] = sfrag<BKM>(smem + SLB, wc * 8 + u, lane);
  }
  wait_lgkm0();

  // LDS reads per fragment (k-outer images take two ds_read_b64_tr_b16)
  constexpr int RA = AK ? 2 : 1, RB = BKM ? 2 : 1, RTOT = 8 * RA + 8 * RB;
  // one slice: cur = F(s) (in registers), nxt <- F(s+1)
#define RCA_SLICE(S, CA, CB, NA, NB)                                                   \
  {                                                                                    \
    fence_sched();                                                                     \
    wait_vmcnt<8>();                                                                   \
    fence_sched();                                                                     \
    __builtin_amdgcn_s_barrier();                                                      \
    fence_sched();                                                                     \
    const lds_char* ns_ = smem + (((S) + 1) & 3) * SST;                                \
    _Pragma("unroll") for (int u = 0; u < 16; ++u) {                                   \
      if constexpr (PW) {                                                              \
        /* group u's MFMAs use all of B and A rows 0..u>>1 of the previous slice's */  \
        /* reads (issued B0..B7, A0..A7); this slice's u earlier reads are younger */  \
        const int need = 8 * RB + ((u >> 1) + 1) * RA;                                 \
        const int younger = (u < 8 ? u : 8) * RB + (u > 8 ? u - 8 : 0) * RA;           \
        wait_lgkm_upto(RTOT - need + younger);                                         \
        fence_sched();                                                                 \
        if (u < 8) NB[u] = sfrag<BKM>(ns_ + SLB, wc * 8 + u, lane);                    \
        else NA[u - 8] = sfrag<AK>(ns_, wr * 8 + u - 8, lane);                         \
      } else {                                                                         \
        if (u < 8) NA[u] = sfrag<AK>(ns_, wr * 8 + u, lane);                           \
        else NB[u - 8] = sfrag<BKM>(ns_ + SLB, wc * 8 + u - 8, lane);                  \
      }                                                                                \
      if ((u & 1) == 0) dma((S) + 3, u >> 1);                                          \
      mfma_n<4>(acc, CA, CB, u >> 1, (u & 1) * 4);                                     \
      fence_sched();                                                                   \
    }                                                                                  \
    if constexpr (!PW) wait_lgkm0();                                                   \
    fence_sched();                                                                     \
  }
  for (int s = 0; s < ns; s += 2) {
    RCA_SLICE(s, xa, xb, ya, yb)
    RCA_SLICE(s + 1, ya, yb, xa, xb)
  }
#undef RCA_SLICE
  wait_lgkm0();
  wait_vmcnt<0>();
  drain_acc(acc);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = m0 + wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) store4<ACC>(C, m * ldc + n0 + wc * 128 + j * 16 + 4 * (lane >> 4), acc[i][j]);
  }
}

// ---------------------------------------------------------------------------------------------
// Variant 6: variant 3's slice ring for the k-contiguous (TN) layout with no per-iteration vector
// address arithmetic. Variant 3's loop body carried ~50 VALU ops per 64-deep K-tile beside its 128
// MFMAs (a 64-bit v_lshl_add_u64 per LDS-DMA, a v_add_u32 per fragment read: the asm read took a
// materialised address); hipBLASLt's 256x256x64 kernel carries two. Here:
//   - LDS-DMA is a buffer load (`buffer_load_dwordx4 ... offen lds`): a per-wave resource
//     descriptor (SGPRs) whose base is the wave's first row, a per-lane byte offset per DMA step
//     that never changes (8 VGPRs), and the slice's k offset in the scalar soffset operand;
//   - fragment reads are `ds_read_b128 base offset:IMM`: with the 64-B-row swizzle the chunk
//     index depends on the lane only, so each of the 16 reads per slice is one of two constant
//     base VGPRs (stages 0-1 / 2-3, the immediate field is 16 bits) plus a compile-time offset;
//   - four slices per loop iteration, so every stage index is a template constant.
// Placement per 64-MFMA slice: the 16 reads of the next slice's fragments one per MFMA gap right
// after the barrier, the 8 DMAs of slice s+3 one every 6 MFMAs after that.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int OFF>
__device__ __forceinline__ bf16x8_t rd_imm(unsigned base) {
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
  return __builtin_bit_cast(bf16x8_t, v);
}

template <bool ACC>
__global__ __launch_bounds__(NT4, 1) void gemm4b_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                        bf16_t* __restrict__ C, int M, int N, int K, long lda,
                                                        long ldb, long ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  tile_origin(blockIdx.x, M, N, m0, n0);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ns = K / 32;  // multiple of 4 (host check)
  // DMA block 4i + wid of a slice = rows 16(4i + wid) .. +15 of the 256-row panel, 64 B each.
  // Wave base row 16 wid; lane row (l >> 2) + 64 i; chunk (l & 3) ^ swz32(row) = (l & 3) ^ swz32(l >> 2).
  const bf16_t* wa = A + (long)(m0 + 16 * wid) * lda;
  const bf16_t* wb = B + (long)(n0 + 16 * wid) * ldb;
  const __amdgpu_buffer_rsrc_t ra = wave_rsrc(wa, (unsigned)((long)(M - m0 - 16 * wid) * lda * 2));
  const __amdgpu_buffer_rsrc_t rb = wave_rsrc(wb, (unsigned)((long)(N - n0 - 16 * wid) * ldb * 2));
  const int lrow = lane >> 2, lch = (lane & 3) ^ swz32(lrow);
  int va[4], vb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    va[i] = (int)(((long)(lrow + 64 * i) * lda + lch * 8) * 2);
    vb[i] = (int)(((long)(lrow + 64 * i) * ldb + lch * 8) * 2);
  }
  // fragment read base: row ob*16 + (l & 15) of the stage image, chunk (l >> 4) ^ swz32(l & 15)
  const unsigned rl = (unsigned)((lane & 15) * 64 + (((lane >> 4) ^ swz32(lane & 15)) << 4));
  const unsigned sbase = lds_off(smem);
  const unsigned ba_lo = sbase + rl + wr * 8 * 1024, bb_lo = sbase + rl + SLB + wc * 8 * 1024;
  const unsigned ba_hi = ba_lo + 2 * SST, bb_hi = bb_lo + 2 * SST;

  auto dma = [&](int sl, int stage, int step) {  // step 0..7: A steps 0..3, then B steps 0..3
    const int soff = min(sl, ns - 1) * 64;
    lds_char* st = smem + stage * SST;
    if (step < 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(st + (4 * step + wid) * 1024),
                                               16, va[step], soff, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(st + SLB + (4 * (step - 4) + wid) * 1024), 16, vb[step - 4],
          soff, 0, 0);
  };
#pragma unroll
  for (int sl = 0; sl < 3; ++sl)
#pragma unroll
    for (int i = 0; i < 8; ++i) dma(sl, sl, i);
  wait_vmcnt<16>();
  fence_sched();
  __builtin_amdgcn_s_barrier();
  fence_sched();
  bf16x8_t xa[8], xb[8], ya[8], yb[8];
#define RCA_RD0(u)                                    \
  xa[u] = rd_imm<(u) * 1024>(ba_lo);                  \
  xb[u] = rd_imm<(u) * 1024>(bb_lo);
  RCA_RD0(0) RCA_RD0(1) RCA_RD0(2) RCA_RD0(3) RCA_RD0(4) RCA_RD0(5) RCA_RD0(6) RCA_RD0(7)
#undef RCA_RD0
  wait_lgkm0();

  // one MFMA of slice position p (0..63): acc[p>>3][p&7]
#define RCA_MF(CA, CB, p) \
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[(p) >> 3][(p)&7]) : "v"(CB[(p)&7]), "v"(CA[(p) >> 3]))
  // read r (0..15) of the next slice (stage NST): A fragments 0..7, then B 0..7
#define RCA_RDN(NST, NA, NB, r)                                                                    \
  {                                                                                                \
    constexpr int off_ = ((NST)&1) * SST + ((r)&7) * 1024;                                         \
    if constexpr ((r) < 8) NA[(r)&7] = rd_imm<off_>((NST) < 2 ? ba_lo : ba_hi);                   \
    else NB[(r)&7] = rd_imm<off_>((NST) < 2 ? bb_lo : bb_hi);                                      \
  }
#define RCA_P(ST, CA, CB, NA, NB, p)                                                               \
  {                                                                                                \
    fence_sched();                                                                                 \
    if constexpr ((p) < 16) RCA_RDN(((ST) + 1) & 3, NA, NB, (p));                                  \
    if constexpr ((p) >= 16 && ((p)-16) % 6 == 0 && ((p)-16) / 6 < 8)                              \
      dma(s + (ST) + 3, ((ST) + 3) & 3, ((p)-16) / 6);                                             \
    fence_sched();                                                                                 \
    RCA_MF(CA, CB, p);                                                                             \
  }
#define RCA_P8(ST, CA, CB, NA, NB, b)                                                              \
  RCA_P(ST, CA, CB, NA, NB, (b) + 0) RCA_P(ST, CA, CB, NA, NB, (b) + 1)                             \
  RCA_P(ST, CA, CB, NA, NB, (b) + 2) RCA_P(ST, CA, CB, NA, NB, (b) + 3)                             \
  RCA_P(ST, CA, CB, NA, NB, (b) + 4) RCA_P(ST, CA, CB, NA, NB, (b) + 5)                             \
  RCA_P(ST, CA, CB, NA, NB, (b) + 6) RCA_P(ST, CA, CB, NA, NB, (b) + 7)
#define RCA_SL(ST, CA, CB, NA, NB)                                                                 \
  {                                                                                                \
    fence_sched();                                                                                 \
    wait_vmcnt<8>();                                                                               \
    fence_sched();                                                                                 \
    __builtin_amdgcn_s_barrier();                                                                  \
    RCA_P8(ST, CA, CB, NA, NB, 0) RCA_P8(ST, CA, CB, NA, NB, 8)                                    \
    RCA_P8(ST, CA, CB, NA, NB, 16) RCA_P8(ST, CA, CB, NA, NB, 24)                                  \
    RCA_P8(ST, CA, CB, NA, NB, 32) RCA_P8(ST, CA, CB, NA, NB, 40)                                  \
    RCA_P8(ST, CA, CB, NA, NB, 48) RCA_P8(ST, CA, CB, NA, NB, 56)                                  \
    fence_sched();                                                                                 \
    wait_lgkm0();                                                                                  \
    fence_sched();                                                                                 \
  }
  for (int s = 0; s < ns; s += 4) {
    RCA_SL(0, xa, xb, ya, yb)
    RCA_SL(1, ya, yb, xa, xb)
    RCA_SL(2, xa, xb, ya, yb)
    RCA_SL(3, ya, yb, xa, xb)
  }
#undef RCA_SL
#undef RCA_P8
#undef RCA_P
#undef RCA_RDN
#undef RCA_MF
  wait_lgkm0();
  wait_vmcnt<0>();
  drain_acc(acc);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = m0 + wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) store4<ACC>(C, m * ldc + n0 + wc * 128 + j * 16 + 4 * (lane >> 4), acc[i][j]);
  }
}

template <bool ACC>
int launch4b(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
             hipStream_t st) {
  auto kern = gemm4b_kernel<ACC>;
  constexpr int smem = 4 * SST;
  static bool attr = [&] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess;
  }();
  if (!attr) return -3;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(NT4), smem, st, (const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K,
                     lda, ldb, ldc);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Variant 7: full-cache-line LDS-DMA. A PMC pass on the o_proj forward product
// (`profiles/gemm_r4.md`) showed variant 6's 32-deep slices costing twice hipBLASLt's L1->L2 read
// requests (TCP_TCC_READ_REQ 34.1 M vs 16.8 M) and a texture-addresser unit busy 86 % of the
// kernel (TA_TA_BUSY 86.8 M vs 40.0 M): each DMA instruction covered 16 rows x 64 B, i.e. 16 half
// cache lines. Here K-tiles are 64 deep (128-B rows: 8 rows x 128 B per DMA instruction) in two
// 64 KB LDS buffers, and a buffer is refilled while the tile it held is still being multiplied:
// both 32-deep halves of a tile's fragments are in registers by the middle of its iteration
// (F0 read during the previous iteration, F1 in the first 16 MFMAs), so after one barrier the
// DMAs of tile t+2 go into tile t's buffer, two tiles (~250 MFMAs) ahead of their use.
//   iteration t (buffer b = t & 1), 128 MFMAs: [0, 64) on F0(t), [64, 128) on F1(t)
//     M0-15   read F1(t) from b                       M24   lgkmcnt(0) + barrier (b is free)
//     M24-84  16 DMAs of tile t+2 into b               M96   vmcnt(16) + barrier (t+1 landed)
//     M96-127 read F0(t+1) from b ^ 1, one per 2 MFMAs  end   lgkmcnt(0)
// Image: row-major 256 x 128 B per operand; 16-B chunk c of row r at c ^ ((r >> 1) & 7) (the
// variant-2 image: conflict-free ds_read_b128 fragment reads).
// Fused epilogues of variant 7 (EPI): 0 = store C (+= C when ACC); 1 = SwiGLU backward (C is the
// down projection's input gradient dh = dy W_down, never stored; see swiglu_bwd_epilogue).
struct EpiArgs {
  const bf16_t* gu;  // [M][2F] gate | up (the forward's gate_up output)
  bf16_t* dgu;       // [M][2F]
  bf16_t* dgu_t;     // [2F][M]
  long ldg, ldd, ldt;
  int F;
  // EPI 2 (per-column affine epilogue): C = act(acc + shift[n] (+ res[m][n]))
  const float* shift;
  const bf16_t* res;
  long ldr;
  int relu;
};

// SwiGLU-backward epilogue (variant 7, EPI 1). The wave's 128 x 128 accumulator tile is
// dh[m][n] (token m, feature n) in fp32; with g = gu[m][n], u = gu[m][F + n]:
//   dg = dh * u * s * (1 + g (1 - s)),  du = dh * bf16(g s),  s = sigmoid(g)
// (elementwise.hip's swiglu_bwd, but from the fp32 dh instead of its bf16 rounding). dg, du go to
// dgu[m][n], dgu[m][F + n] (8-B stores of 4 consecutive n) and, through a wave-private LDS tile
// [128 n][128 m] (272-B rows: the 4 lane groups' rows land 16 banks apart), to the transposed
// copy dgu_t[n][m], dgu_t[F + n][m] that the gate_up weight gradient reads, as 16-B row stores.
// Replaces the dh store + the separate swiglu_bwd_tr pass (its dh read and write).
constexpr int kEpiRow = 272, kEpiWaveLds = 128 * kEpiRow;

__device__ __forceinline__ void epi_tile_store_t(const lds_char* tw, bf16_t* __restrict__ dst, long ldt, long row0,
                                                 long m0, int lane) {
#pragma unroll 8
  for (int q = 0; q < 32; ++q) {
    const int idx = q * 64 + lane, row = idx >> 4, ch = idx & 15;
    const u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(tw + row * kEpiRow + ch * 16);
    *reinterpret_cast<u32x4*>(dst + (row0 + row) * ldt + m0 + ch * 8) = v;
  }
}

__device__ __forceinline__ void swiglu_bwd_epilogue(f32x4 (&acc)[8][8], const EpiArgs& ep, lds_char* smem, int mw,
                                                    int nw, int wid, int lane) {
  __builtin_amdgcn_s_barrier();  // every wave has left the LDS ring (its waits came before)
  lds_char* tw = smem + wid * kEpiWaveLds;
  const int ml0 = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = mw + i * 16 + ml0;
    const bf16_t* grow = ep.gu + m * ep.ldg;
    bf16_t* drow = ep.dgu + m * ep.ldd;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int nl = j * 16 + nq, n = nw + nl;
      const unsigned long long gv = *reinterpret_cast<const unsigned long long*>(grow + n);
      const unsigned long long uv = *reinterpret_cast<const unsigned long long*>(grow + ep.F + n);
      unsigned long long og = 0, ou = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float g = bf2f((bf16_t)(gv >> (16 * r))), u = bf2f((bf16_t)(uv >> (16 * r)));
        const float d = acc[i][j][r];
        const float sg = 1.f / (1.f + __expf(-g));
        const float si = g * sg;
        const bf16_t dgb = f2bf(d * u * sg * (1.f + g * (1.f - sg)));
        const bf16_t dub = f2bf(d * bf2f(f2bf(si)));
        og |= (unsigned long long)dgb << (16 * r);
        ou |= (unsigned long long)dub << (16 * r);
        *(__attribute__((address_space(3))) bf16_t*)(tw + (nl + r) * kEpiRow + (i * 16 + ml0) * 2) = dgb;
        acc[i][j][r] = bf2f(dub);  // du kept for the second transposed pass
      }
      *reinterpret_cast<unsigned long long*>(drow + n) = og;
      *reinterpret_cast<unsigned long long*>(drow + ep.F + n) = ou;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  epi_tile_store_t(tw, ep.dgu_t, ep.ldt, nw, mw, lane);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *(__attribute__((address_space(3))) bf16_t*)(tw + (j * 16 + nq + r) * kEpiRow + (i * 16 + ml0) * 2) =
            f2bf(acc[i][j][r]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  epi_tile_store_t(tw, ep.dgu_t, ep.ldt, (long)ep.F + nw, mw, lane);
}

// Where each event of a variant-7 iteration sits (position p = index of the MFMA it precedes).
// SPLIT = 0: the knob schedule below. SPLIT = 1: the buffer is freed in two halves (variant 77):
// F1's A fragments are read first and a barrier frees the A region for the A DMAs while the B
// fragments are still being read; a second barrier frees the B region; the F0(t+1) wait comes
// after 13 of the iteration's 16 DMAs (vmcnt(13)), the last 3 B DMAs overlap the F0 reads.
template <int B1, int DS, int W2, int RD, int R1, int SPLIT>
struct Sch7 {
  static constexpr int f1(int p) {  // F1(t) read index (0-7 A, 8-15 B) or -1
    if (SPLIT) {
      if (p >= 1 && p <= 15 && (p & 1)) return (p - 1) / 2;
      constexpr int b[8] = {25, 28, 31, 34, 37, 39, 41, 43};
      for (int i = 0; i < 8; ++i)
        if (b[i] == p) return 8 + i;
      return -1;
    }
    return (p % R1 == 0 && p / R1 < 16) ? p / R1 : -1;
  }
  static constexpr int dma(int p) {  // DMA step (0-7 A, 8-15 B) or -1
    if (SPLIT) {
      constexpr int d[16] = {23, 26, 29, 32, 35, 53, 56, 59, 62, 65, 86, 88, 90, 97, 101, 125};
      for (int i = 0; i < 16; ++i)
        if (d[i] == p) return i;
      return -1;
    }
    return (p >= B1 && p <= B1 + 15 * DS && (p - B1) % DS == 0) ? (p - B1) / DS : -1;
  }
  static constexpr int wait(int p) {  // 1: lgkmcnt(0) + barrier, 2: vmcnt(VM) + barrier
    if (SPLIT) return (p == 21 || p == 51) ? 1 : (p == 92 ? 2 : 0);
    return p == B1 ? 1 : (p == W2 ? 2 : 0);
  }
  static constexpr int VM = SPLIT ? 13 : 16;
  static constexpr int f0(int p) {  // F0(t+1) read index or -1
    if (SPLIT) return (p >= 94 && p < 110) ? p - 94 : -1;
    return (p >= W2 && (p - W2) % RD == 0 && (p - W2) / RD < 16) ? (p - W2) / RD : -1;
  }
};

// Schedule knobs (positions in the iteration's 128 MFMAs): B1 = the lgkmcnt(0) + barrier that frees
// the buffer, DMAs every DS MFMAs from B1, W2 = the vmcnt(16) + barrier before the F0(t+1) reads,
// which then go one per RD MFMAs; F1 reads one per R1 MFMAs from M0; ORD 1 walks the MFMAs with
// the B-tile fragment (the MFMA's first operand) fixed over 8 consecutive MFMAs instead of the
// A-tile one. Defaults = variant 7 (= the split schedule, measured best: 24.42 vs 25.26 ms for the
// 13 TN shapes, gemm_r4.md); variants 71-78 are the timing A/Bs.
template <bool ACC, int B1 = 24, int DS = 4, int W2 = 96, int RD = 2, int R1 = 1, int ORD = 1, int SPLIT = 1, int EPI = 0,
          int AUX = 0>
__global__ __launch_bounds__(NT4, 1) void gemm4c_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                        bf16_t* __restrict__ C, int M, int N, int K, long lda,
                                                        long ldb, long ldc, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  tile_origin(blockIdx.x, M, N, m0, n0);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = K / 64;  // even (host check: K % 128 == 0)
  // DMA step i (0..7) of an operand: LDS block 4i + wid = rows 8(4i + wid) .. +7 of the panel.
  // Wave base row 8 wid, lane row (l >> 3) + 32 i; the lane's 16-B LDS slot l & 7 holds logical
  // chunk (l & 7) ^ ((row >> 1) & 7) = (l & 7) ^ ((4 wid + (l >> 4)) & 7).
  const bf16_t* wa = A + (long)(m0 + 8 * wid) * lda;
  const bf16_t* wb = B + (long)(n0 + 8 * wid) * ldb;
  const __amdgpu_buffer_rsrc_t ra = wave_rsrc(wa, (unsigned)((long)(M - m0 - 8 * wid) * lda * 2));
  const __amdgpu_buffer_rsrc_t rb = wave_rsrc(wb, (unsigned)((long)(N - n0 - 8 * wid) * ldb * 2));
  const int lch = (lane & 7) ^ ((4 * wid + (lane >> 4)) & 7);
  int va[8], vb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    va[i] = (int)(((long)((lane >> 3) + 32 * i) * lda + lch * 8) * 2);
    vb[i] = (int)(((long)((lane >> 3) + 32 * i) * ldb + lch * 8) * 2);
  }
  // fragment read of row block ob, half kk: row ob*16 + (l & 15), chunk (4 kk + (l >> 4)) ^ ((l & 15) >> 1)
  constexpr int TBK = 256 * 128;  // one operand tile (32 KB); buffer = A | B = 64 KB
  const unsigned sbase = lds_off(smem);
  unsigned rbA[2][2], rbB[2][2];  // [buffer][kk]
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const unsigned lo = (unsigned)((lane & 15) * 128 + (((4 * kk + (lane >> 4)) ^ ((lane & 15) >> 1)) << 4));
    rbA[0][kk] = sbase + lo + wr * 128 * 128;
    rbB[0][kk] = sbase + lo + TBK + wc * 128 * 128;
    rbA[1][kk] = rbA[0][kk] + 2 * TBK;
    rbB[1][kk] = rbB[0][kk] + 2 * TBK;
  }

  auto dma = [&](int t, int buf, int step) {  // step 0..7: A, 8..15: B
    const int soff = min(t, nt - 1) * 128;
    lds_char* st = smem + buf * 2 * TBK;
    if (step < 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(st + (4 * step + wid) * 1024),
                                               16, va[step], soff, 0, AUX);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(st + TBK + (4 * (step - 8) + wid) * 1024), 16, vb[step - 8],
          soff, 0, AUX);
  };
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) dma(t, t, i);
  wait_vmcnt<16>();
  fence_sched();
  __builtin_amdgcn_s_barrier();
  fence_sched();
  bf16x8_t xa[8], xb[8], ya[8], yb[8];
#define RCA_RD0(u)                                      \
  xa[u] = rd_imm<(u) * 2048>(rbA[0][0]);                \
  xb[u] = rd_imm<(u) * 2048>(rbB[0][0]);
  RCA_RD0(0) RCA_RD0(1) RCA_RD0(2) RCA_RD0(3) RCA_RD0(4) RCA_RD0(5) RCA_RD0(6) RCA_RD0(7)
#undef RCA_RD0
  wait_lgkm0();

#define RCA_MF(FA, FB, q)                                                                                  \
  {                                                                                                        \
    constexpr int i_ = ORD ? ((q)&7) : ((q) >> 3), j_ = ORD ? ((q) >> 3) : ((q)&7);                        \
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i_][j_]) : "v"(FB[j_]), "v"(FA[i_]));          \
  }
  // position p (0..127) of the iteration on buffer BUF
#define RCA_Q(BUF, p)                                                                                \
  {                                                                                                  \
    using S_ = Sch7<B1, DS, W2, RD, R1, SPLIT>;                                                      \
    fence_sched();                                                                                   \
    if constexpr (S_::f1(p) >= 0) {                                                                  \
      constexpr int f_ = S_::f1(p);                                                                  \
      if constexpr (f_ < 8) ya[f_ & 7] = rd_imm<(f_ & 7) * 2048>(rbA[BUF][1]);                       \
      else yb[f_ & 7] = rd_imm<(f_ & 7) * 2048>(rbB[BUF][1]);                                        \
    }                                                                                                \
    if constexpr (S_::wait(p) == 1) {                                                                \
      wait_lgkm0();                                                                                  \
      fence_sched();                                                                                 \
      __builtin_amdgcn_s_barrier();                                                                  \
    }                                                                                                \
    if constexpr (S_::dma(p) >= 0) dma(t + (BUF) + 2, BUF, S_::dma(p));                              \
    if constexpr (S_::wait(p) == 2) {                                                                \
      wait_vmcnt<S_::VM>();                                                                          \
      fence_sched();                                                                                 \
      __builtin_amdgcn_s_barrier();                                                                  \
    }                                                                                                \
    if constexpr (S_::f0(p) >= 0) {                                                                  \
      constexpr int r_ = S_::f0(p);                                                                  \
      if constexpr (r_ < 8) xa[r_ & 7] = rd_imm<(r_ & 7) * 2048>(rbA[(BUF) ^ 1][0]);                 \
      else xb[r_ & 7] = rd_imm<(r_ & 7) * 2048>(rbB[(BUF) ^ 1][0]);                                  \
    }                                                                                                \
    fence_sched();                                                                                   \
    if constexpr ((p) < 64) {                                                                        \
      RCA_MF(xa, xb, (p))                                                                            \
    } else {                                                                                         \
      RCA_MF(ya, yb, (p)-64)                                                                         \
    }                                                                                                \
  }
#define RCA_Q8(BUF, b)                                                                              \
  RCA_Q(BUF, (b) + 0) RCA_Q(BUF, (b) + 1) RCA_Q(BUF, (b) + 2) RCA_Q(BUF, (b) + 3) RCA_Q(BUF, (b) + 4) \
  RCA_Q(BUF, (b) + 5) RCA_Q(BUF, (b) + 6) RCA_Q(BUF, (b) + 7)
#define RCA_IT(BUF)                                                                                 \
  {                                                                                                 \
    RCA_Q8(BUF, 0) RCA_Q8(BUF, 8) RCA_Q8(BUF, 16) RCA_Q8(BUF, 24)                                   \
    RCA_Q8(BUF, 32) RCA_Q8(BUF, 40) RCA_Q8(BUF, 48) RCA_Q8(BUF, 56)                                 \
    RCA_Q8(BUF, 64) RCA_Q8(BUF, 72) RCA_Q8(BUF, 80) RCA_Q8(BUF, 88)                                 \
    RCA_Q8(BUF, 96) RCA_Q8(BUF, 104) RCA_Q8(BUF, 112) RCA_Q8(BUF, 120)                              \
    fence_sched();                                                                                  \
    wait_lgkm0();                                                                                   \
    fence_sched();                                                                                  \
  }
  for (int t = 0; t < nt; t += 2) {
    RCA_IT(0)
    RCA_IT(1)
  }
#undef RCA_IT
#undef RCA_Q8
#undef RCA_Q
#undef RCA_MF
  wait_lgkm0();
  wait_vmcnt<0>();
  drain_acc(acc);
  if constexpr (EPI == 1) {
    swiglu_bwd_epilogue(acc, ep, smem, m0 + wr * 128, n0 + wc * 128, wid, lane);
    return;
  }
  if constexpr (EPI == 2) {
    // conv-as-GEMM epilogue (1x1 NHWC convolution with the folded BatchNorm): the per-channel
    // shift, the residual and the ReLU applied to the fp32 accumulators before the one bf16 store,
    // instead of a separate read-modify-write pass over the output
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wc * 128 + j * 16 + 4 * (lane >> 4);
      const f32x4 sh = *reinterpret_cast<const f32x4*>(ep.shift + n);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const long m = m0 + wr * 128 + i * 16 + (lane & 15);
        f32x4 v = acc[i][j] + sh;
        if (ep.res) {
          const unsigned long long r = *reinterpret_cast<const unsigned long long*>(ep.res + m * ep.ldr + n);
          v[0] += bf2f((bf16_t)(r & 0xffff));
          v[1] += bf2f((bf16_t)((r >> 16) & 0xffff));
          v[2] += bf2f((bf16_t)((r >> 32) & 0xffff));
          v[3] += bf2f((bf16_t)((r >> 48) & 0xffff));
        }
        if (ep.relu) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
        }
        store4<false>(C, m * ldc + n, v);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = m0 + wr * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) store4<ACC>(C, m * ldc + n0 + wc * 128 + j * 16 + 4 * (lane >> 4), acc[i][j]);
  }
}

template <bool ACC, int B1 = 24, int DS = 4, int W2 = 96, int RD = 2, int R1 = 1, int ORD = 1, int SPLIT = 1, int EPI = 0,
          int AUX = 0>
int launch4c(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
             hipStream_t st, EpiArgs ep = EpiArgs{}) {
  static_assert(SPLIT || (B1 >= 16 * R1 && B1 + 15 * DS < W2 && W2 + 15 * RD < 128), "schedule positions");
  auto kern = gemm4c_kernel<ACC, B1, DS, W2, RD, R1, ORD, SPLIT, EPI, AUX>;
  constexpr int smem = EPI == 1 ? 4 * kEpiWaveLds : 4 * 256 * 128;
  static bool attr = [&] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess;
  }();
  if (!attr) return -3;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(NT4), smem, st, (const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K,
                     lda, ldb, ldc, ep);
  return (int)hipGetLastError();
}

template <bool AK, bool BKM, bool ACC, bool PW = false>
int launch4s(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc,
             hipStream_t st) {
  auto kern = gemm4s_kernel<AK, BKM, ACC, PW>;
  constexpr int smem = 4 * SST;
  static bool attr = [&] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess;
  }();
  if (!attr) return -3;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(NT4), smem, st, (const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K,
                     lda, ldb, ldc);
  return (int)hipGetLastError();
}

template <bool AK, bool BKM, bool ACC, int DIAG = 0>
int launch4(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc, hipStream_t st) {
  auto kern = gemm4_kernel<AK, BKM, ACC, DIAG>;
  constexpr int smem = 2 * STG;
  static bool attr = [&] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess;
  }();
  if (!attr) return -3;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(NT4), smem, st, (const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K,
                     lda, ldb, ldc);
  return (int)hipGetLastError();
}

}  // namespace

// Internal entry (dispatched from rca_gemm_bf16 in gemm.hip; shapes already checked there).
extern "C" int rca_gemm4_bf16_internal(const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                                       long long ldb, long long ldc, int a_kmaj, int b_kmaj, int accumulate,
                                       hipStream_t st, int diag) {
  // timing diagnostics (WRONG results): 1 = no LDS-DMA inside the K loop, 2 = DMA issued but
  // never waited for
  if (diag == 1 || diag == 2) {
#define RCA_G4D(D)                                                                         \
  {                                                                                        \
    if (!a_kmaj && !b_kmaj) return launch4<false, false, false, D>(A, B, C, M, N, K, lda, ldb, ldc, st); \
    if (!a_kmaj && b_kmaj) return launch4<false, true, false, D>(A, B, C, M, N, K, lda, ldb, ldc, st);   \
    return launch4<true, true, false, D>(A, B, C, M, N, K, lda, ldb, ldc, st);                           \
  }
    if (diag == 1) RCA_G4D(1)
    RCA_G4D(2)
#undef RCA_G4D
  }
  // variants 6 / 7 (71-73: variant-7 schedule A/Bs): k-contiguous A and B, K % 128 == 0, every
  // wave's buffer range < 4 GB; else 3
  if (diag == 6 || diag == 7 || (diag >= 71 && diag <= 78)) {
    if (!a_kmaj && !b_kmaj && K % 128 == 0 && (double)M * lda * 2 < 4294967296.0 &&
        (double)N * ldb * 2 < 4294967296.0) {
      if (diag >= 71 && accumulate) diag = 7;
      if (diag == 71) return launch4c<false, 20, 3, 88, 2, 1, 0, 0>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 72) return launch4c<false, 24, 4, 104, 1, 1, 0, 0>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 73) return launch4c<false, 32, 4, 100, 1, 1, 0, 0>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 74) return launch4c<false, 24, 4, 104, 1, 1, 1, 0>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 75) return launch4c<false, 36, 4, 100, 1, 2, 0, 0>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 76) return launch4c<false, 36, 4, 100, 1, 2, 1, 0>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 77) return launch4c<false, 24, 4, 96, 2, 1, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 78) return launch4c<false, 24, 4, 96, 2, 1, 1, 1>(A, B, C, M, N, K, lda, ldb, ldc, st);
      if (diag == 7) {
        if (accumulate) return launch4c<true>(A, B, C, M, N, K, lda, ldb, ldc, st);
        return launch4c<false>(A, B, C, M, N, K, lda, ldb, ldc, st);
      }
      if (accumulate) return launch4b<true>(A, B, C, M, N, K, lda, ldb, ldc, st);
      return launch4b<false>(A, B, C, M, N, K, lda, ldb, ldc, st);
    }
    diag = 3;
  }
  if (diag == 5) {
#define RCA_G4P(a, b, c) return launch4s<a, b, c, true>(A, B, C, M, N, K, lda, ldb, ldc, st)
    if (!a_kmaj && !b_kmaj) { if (accumulate) RCA_G4P(false, false, true); RCA_G4P(false, false, false); }
    if (!a_kmaj && b_kmaj) { if (accumulate) RCA_G4P(false, true, true); RCA_G4P(false, true, false); }
    if (a_kmaj && b_kmaj) { if (accumulate) RCA_G4P(true, true, true); RCA_G4P(true, true, false); }
    if (accumulate) RCA_G4P(true, false, true);
    RCA_G4P(true, false, false);
#undef RCA_G4P
  }
  if (diag == 3) {
#define RCA_G4S(a, b, c) return launch4s<a, b, c>(A, B, C, M, N, K, lda, ldb, ldc, st)
    if (!a_kmaj && !b_kmaj) { if (accumulate) RCA_G4S(false, false, true); RCA_G4S(false, false, false); }
    if (!a_kmaj && b_kmaj) { if (accumulate) RCA_G4S(false, true, true); RCA_G4S(false, true, false); }
    if (a_kmaj && b_kmaj) { if (accumulate) RCA_G4S(true, true, true); RCA_G4S(true, true, false); }
    if (accumulate) RCA_G4S(true, false, true);
    RCA_G4S(true, false, false);
#undef RCA_G4S
  }
#define RCA_G4(a, b, c) return launch4<a, b, c>(A, B, C, M, N, K, lda, ldb, ldc, st)
  if (!a_kmaj && !b_kmaj) { if (accumulate) RCA_G4(false, false, true); RCA_G4(false, false, false); }
  if (!a_kmaj && b_kmaj) { if (accumulate) RCA_G4(false, true, true); RCA_G4(false, true, false); }
  if (a_kmaj && b_kmaj) { if (accumulate) RCA_G4(true, true, true); RCA_G4(true, true, false); }
  if (accumulate) RCA_G4(true, false, true);
  RCA_G4(true, false, false);
#undef RCA_G4
}

// dgu, dgu_t = SwiGLU-backward(gu, dh) with dh = dy W_down computed in registers (variant 7's
// main loop, EPI 1): dy [T][H] (k = H contiguous, row stride ld_dy), w_t = W_down^T [F][H] (row
// stride ld_w), gu / dgu [T][2F] contiguous, dgu_t [2F][T] contiguous.
// Contract: T % 256 == 0, F % 256 == 0, H % 128 == 0, 16-B aligned rows; returns -1 otherwise.
// out[m][n] = act(sum_k x[m][k] w[n][k] + shift[n] (+ res[m][n])): a 1x1 NHWC convolution with the
// folded-BatchNorm shift, residual add and ReLU in the epilogue (variant 7's main loop, EPI 2).
// x [M][K] (row stride ldx), w [N][K] (ldw), out / res [M][N] (ldo / ldr), shift fp32 [N].
// Contract: M % 256 == 0, N % 256 == 0, K % 128 == 0, 16-B aligned rows, each operand < 4 GB;
// returns -1 otherwise.
RCA_API int rca_gemm_affine_act(const void* x, const void* w, const float* shift, const void* res, void* out, int M,
                                int N, int K, long long ldx, long long ldw, long long ldo, long long ldr, int relu,
                                hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 128 || ldx % 8 || ldw % 8 || ldo % 4 ||
      (res && ldr % 4))
    return -1;
  if ((double)M * ldx * 2 >= 4294967296.0 || (double)N * ldw * 2 >= 4294967296.0) return -1;
  EpiArgs ep{};
  ep.shift = shift;
  ep.res = (const bf16_t*)res;
  ep.ldr = (long)ldr;
  ep.relu = relu;
  return launch4c<false, 24, 4, 96, 2, 1, 1, 1, 2>(x, w, out, M, N, K, ldx, ldw, ldo, st, ep);
}

RCA_API int rca_gemm_swiglu_bwd(const void* dy, const void* w_t, const void* gu, void* dgu, void* dgu_t, int T, int F,
                                int H, long long ld_dy, long long ld_w, hipStream_t st) {
  if (T <= 0 || F <= 0 || H <= 0 || T % 256 || F % 256 || H % 128 || ld_dy % 8 || ld_w % 8) return -1;
  if ((double)T * ld_dy * 2 >= 4294967296.0 || (double)F * ld_w * 2 >= 4294967296.0) return -1;
  EpiArgs ep{(const bf16_t*)gu, (bf16_t*)dgu, (bf16_t*)dgu_t, 2L * F, 2L * F, (long)T, F};
  return launch4c<false, 24, 4, 96, 2, 1, 1, 1, 1>(dy, w_t, nullptr, T, F, H, ld_dy, ld_w, 0, st, ep);
}
