// bf16 GEMM for gfx950 (MI355X) on MFMA 16x16x32, with either operand stored k-contiguous or
// k-outer, so the training backward reads W, dY and X in their natural layouts:
//
//   C[M][N] (+)= sum_k A(m, k) * B(n, k)
//   A: "row"  = A[m][k] (k contiguous, lda = row stride)     | "kmaj" = A[k][m] (m contiguous)
//   B: "row"  = B[n][k]                                       | "kmaj" = B[k][n]
//
//   forward   y  = x W^T      A = x  [T][K] row,   B = W  [N][K] row
//   dgrad     dx = dy W       A = dy [T][N] row,   B = W  [N][K] kmaj   (k = N)
//   wgrad     dW = dy^T x     A = dy [T][N] kmaj,  B = x  [T][K] kmaj   (k = T)
//
// Structure (cdna_hip_programming.md §5): 256x256x64 block tile, 8 waves (2 M x 4 N), 128x64
// per wave = 8x4 accumulators of v_mfma_f32_16x16x32_bf16; global->LDS by global_load_lds 16 B
// per lane (no VGPR staging), two LDS stages (2 x 64 KB); the LDS images are lane-linear with
// the bank swizzle applied to the per-lane SOURCE address and undone on the read:
//   * k-contiguous tile [256][64]: 128-B rows, chunk' = chunk ^ ((row >> 1) & 7) -> the 16 rows a
//     16-lane ds_read_b128 group touches cover all 16 bank slots;
//   * k-outer tile [64][256]: 512-B k-rows read by ds_read_b64_tr_b16 (hardware transpose: lane
//     i of a 16-lane group gets column i of 4 k-rows), 16-B chunk' = chunk ^ s(k) with
//     s(k) = 2 * ((k & 3) | ((k >> 3) & 1) << 2): the 8 k-rows one 32-lane half reads land on 8
//     distinct even chunk pairs.
// The MFMA's "A" operand is the B tile and its "B" operand the A tile, so a lane's 4 accumulator
// registers are 4 CONSECUTIVE n of one m: 8-byte bf16x4 stores in the epilogue.
// Workgroup order: XCD remap (each XCD gets a contiguous range) then GROUP_M=8 grouped tiles, so
// the ~32 blocks co-resident on one XCD share A and B panels through that XCD's L2.
#include "common.h"
#include "gemm_common.h"

namespace {
using namespace rca_gemm;

// NS-stage ring of BK-deep stages; NS-1 stages in flight. One raw s_barrier per stage: the
// counted vmcnt retires exactly the stage about to be read (the later stages stay in flight
// ACROSS the barrier -- __syncthreads() would drain them), the barrier publishes every wave's
// DMA, and the stage refilled right after it was last read one stage earlier by all waves.
template <bool AK, bool BKM, bool ACC, int BK, int NS>
__global__ __launch_bounds__(NTHR) void gemm_bf16_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                         bf16_t* __restrict__ C, int M, int N, int K, long lda,
                                                         long ldb, long ldc) {
  constexpr int TILE_BYTES = 256 * BK * 2;
  constexpr int STAGE_BYTES = 2 * TILE_BYTES;
  constexpr int LOADS = 2 * (BK / 16);  // glds per thread per stage
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;

  // tile order: XCD-contiguous ranges, GROUP_M-row groups inside
  const int ntm = M / BM, ntn = N / BN, nwg = ntm * ntn;
  const int lin = xcd_remap(blockIdx.x, nwg);
  const int gsz = GROUP_M * ntn, grp = lin / gsz, fm = grp * GROUP_M;
  const int gm = min(ntm - fm, GROUP_M), r = lin % gsz;
  const int m0 = (fm + r % gm) * BM, n0 = (r / gm) * BN;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = K / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (s < nt) {
      lds_char* buf = smem + s * STAGE_BYTES;
      stage_tile<AK, BK>(A, lda, m0, s * BK, buf, wid, lane);
      stage_tile<BKM, BK>(B, ldb, n0, s * BK, buf + TILE_BYTES, wid, lane);
    }
  }

  for (int t = 0; t < nt; ++t) {
    if (t + NS - 1 <= nt) wait_vmcnt<(NS - 2) * LOADS>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nt) {
      const int s = t + NS - 1;
      lds_char* buf = smem + (s % NS) * STAGE_BYTES;
      stage_tile<AK, BK>(A, lda, m0, s * BK, buf, wid, lane);
      stage_tile<BKM, BK>(B, ldb, n0, s * BK, buf + TILE_BYTES, wid, lane);
    }
    const lds_char* ta = smem + (t % NS) * STAGE_BYTES;
    const lds_char* tb = ta + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t bf[4], af[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = load_frag<BKM, BK>(tb, wn * 4 + j, kk, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = load_frag<AK, BK>(ta, wm * 8 + i, kk, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // epilogue: acc[i][j] reg r = C[m0 + wm*128 + i*16 + (lane&15)][n0 + wn*64 + j*16 + 4*(lane>>4) + r]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = m0 + wm * 128 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      unsigned long long* dst = (unsigned long long*)(C + m * ldc + n);
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if constexpr (ACC) {
        const unsigned long long old = *dst;
        v0 += bf2f((bf16_t)(old & 0xffff));
        v1 += bf2f((bf16_t)((old >> 16) & 0xffff));
        v2 += bf2f((bf16_t)((old >> 32) & 0xffff));
        v3 += bf2f((bf16_t)((old >> 48) & 0xffff));
      }
      const unsigned long long o = (unsigned long long)f2bf(v0) | ((unsigned long long)f2bf(v1) << 16) |
                                   ((unsigned long long)f2bf(v2) << 32) | ((unsigned long long)f2bf(v3) << 48);
      *dst = o;
    }
  }
}

template <bool AK, bool BKM, bool ACC, int BK, int NS>
int launch(const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb, long ldc, hipStream_t st) {
  auto kern = gemm_bf16_kernel<AK, BKM, ACC, BK, NS>;
  constexpr int smem = NS * 2 * 256 * BK * 2;
  static bool attr = [&] {
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem) == hipSuccess;
  }();
  if (!attr) return -3;
  if (K % BK) return -1;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(NTHR), smem, st, (const bf16_t*)A, (const bf16_t*)B, (bf16_t*)C, M, N, K,
                     lda, ldb, ldc);
  return (int)hipGetLastError();
}

// Variants (RCA_GEMM_VARIANT, or rca_gemm_set_variant for same-process A/B):
//   0: this file's 8-wave two-stage ring (round 2; fwd 1.15-1.24 PF, dgrad 0.97-1.04, wgrad
//      0.82-0.98 on the 8B shapes, random operands, round-3 remeasure)
//   2: gemm4.hip, one wave per SIMD with 128x128 wave tiles (default)
template <bool AK, bool BKM, bool ACC>
int launch_variant(int variant, const void* A, const void* B, void* C, int M, int N, int K, long lda, long ldb,
                   long ldc, hipStream_t st) {
  (void)variant;
  return launch<AK, BKM, ACC, 64, 2>(A, B, C, M, N, K, lda, ldb, ldc, st);
}

}  // namespace

// Shape contract (checked here and by the Python wrapper): M % 256 == 0, N % 256 == 0,
// K % 64 == 0; leading dimensions multiples of 8 elements and 16-B aligned base pointers.
// a_kmaj / b_kmaj select the k-outer layouts; accumulate adds into C (bf16 read-modify-write).
extern "C" int rca_gemm4_bf16_internal(const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                                       long long ldb, long long ldc, int a_kmaj, int b_kmaj, int accumulate,
                                       hipStream_t st, int diag);

static int g_gemm_variant = [] {
  const char* e = getenv("RCA_GEMM_VARIANT");
  return e ? atoi(e) : 3;
}();
static int gemm_variant() { return g_gemm_variant; }

// A/B switch for benchmarks (same process, interleaved rounds); returns the previous variant.
RCA_API int rca_gemm_set_variant(int v) {
  const int old = g_gemm_variant;
  g_gemm_variant = v;
  return old;
}

RCA_API int rca_gemm_bf16(const void* A, const void* B, void* C, int M, int N, int K, long long lda, long long ldb,
                          long long ldc, int a_kmaj, int b_kmaj, int accumulate, hipStream_t st) {
  if (M % BM || N % BN || K % 64 || M <= 0 || N <= 0 || K <= 0) return -1;
  if ((lda | ldb | ldc) & 7) return -2;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return -2;
  int v = gemm_variant();
  // k-contiguous (TN) operands: variant 7 (64-deep tiles, full-line DMA) is faster than 3 on
  // every measured shape (profiles/gemm_r4.md); it falls back to 3 where its contract fails
  if (v == 3 && !a_kmaj && !b_kmaj) v = 7;
  if (v >= 90) return rca_gemm4_bf16_internal(A, B, C, M, N, K, lda, ldb, ldc, a_kmaj, b_kmaj, 0, st, v - 90);
  if (v == 3 || v == 5 || v == 6 || v == 7 || (v >= 71 && v <= 78))
    return rca_gemm4_bf16_internal(A, B, C, M, N, K, lda, ldb, ldc, a_kmaj, b_kmaj, accumulate, st, v);
  if (v != 0) return rca_gemm4_bf16_internal(A, B, C, M, N, K, lda, ldb, ldc, a_kmaj, b_kmaj, accumulate, st, 0);
#define RCA_G(a, b, c) return launch_variant<a, b, c>(v, A, B, C, M, N, K, lda, ldb, ldc, st)
  if (!a_kmaj && !b_kmaj) { if (accumulate) RCA_G(false, false, true); RCA_G(false, false, false); }
  if (!a_kmaj && b_kmaj) { if (accumulate) RCA_G(false, true, true); RCA_G(false, true, false); }
  if (a_kmaj && b_kmaj) { if (accumulate) RCA_G(true, true, true); RCA_G(true, true, false); }
  if (accumulate) RCA_G(true, false, true);
  RCA_G(true, false, false);
#undef RCA_G
}
