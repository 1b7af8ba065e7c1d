// Wide-row flash-attention forward for gfx950 (D = 128; RCA_ATTN_FWD=wide, opt-in). Same math, LDS image
// and LDS-DMA K/V staging as attn_fwd_kernel (attention.hip), but each wave owns 64 query rows
// (two 32-row groups) instead of 32: every K fragment read from LDS feeds the S^T MFMAs of both
// groups and every V^T fragment the P.V MFMAs of both, halving the LDS bytes per MFMA. The
// 32-row kernel reads 32 KB of K/V per wave per 64-key tile against 32 MFMAs, which at two
// waves per SIMD is the LDS's whole 128 B/clk at full MFMA rate; here it is half. One wave per
// SIMD (4 waves x 64 rows = 256 query rows per workgroup); the O^T accumulators of both groups
// (128 registers) sit in the accumulator file: this file is built without -amdgpu-mfma-vgpr-form.
#include "attention_common.h"

#include <cstdlib>

namespace {

template <bool CAUSAL>
__global__ __launch_bounds__(kThreads, 1) void attn_fwd_wide_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    bf16_t* __restrict__ O, float* __restrict__ LSE, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long so, float scale2) {
  constexpr int D = 128, BQ = 256, BK = 64, NKS = D / 16, NDB = D / 32, TILE = BK * D * 2, G8 = Img<D>::G8;
  constexpr float THR = 8.f;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];

  const int nqb = S / BQ, G = Hq / Hk;
  int bhk, item;
  xcd_group_map(blockIdx.x, B * Hk, G * nqb, bhk, item);
  const int qr = item / G, b = bhk / Hk, hk = bhk % Hk, hq = hk * G + item % G, bh = b * Hq + hq;
  const int qb = CAUSAL ? nqb - 1 - qr : qr;  // longest causal rows first
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int q0 = qb * BQ, qw0 = q0 + 64 * w;  // group g rows: qw0 + 32 g + l32
  const int rb0 = Img<D>::row_base(l32, h, 0), rb1 = Img<D>::row_base(l32, h, 1);
  const int tb0 = Img<D>::tr_base(lane, 0), tb1 = Img<D>::tr_base(lane, 1);

  const bf16_t* Kb = K + (long)b * S * sk + (long)hk * D;
  const bf16_t* Vb = V + (long)b * S * sv + (long)hk * D;

  bf16x8_t qf[2][NKS];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const bf16_t* Qr = Q + ((long)b * S + qw0 + 32 * g + l32) * sq + (long)hq * D;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[g][ks] = gload8(Qr + 16 * ks + 8 * h);
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) settle(qf[g][ks]);

  f32x16 o[2][NDB];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int i = 0; i < NDB; ++i) o[g][i] = zero16();
  float m[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};

  const int ntile = CAUSAL ? (q0 + BQ) / BK : S / BK;  // even
  DmaStage<D, BK> kst, vst;
  kst.init(Kb, sk, S, tid);
  vst.init(Vb, sv, S, tid);
  kst.issue(0, sk, smem);
  vst.issue(0, sv, smem + TILE);
  wait_dma();
  __syncthreads();

  auto tile = [&](auto bufc, int it) {
    constexpr int buf = decltype(bufc)::value;
    const char* Ks = smem + buf * 2 * TILE;
    const char* Vs = Ks + TILE;
    const int kb = it * BK;
    const bool more = it + 1 < ntile;
    if (more) {  // into the other buffer: every wave left it at the last barrier
      kst.issue(kb + BK, sk, smem + (buf ^ 1) * 2 * TILE);
      vst.issue(kb + BK, sv, smem + (buf ^ 1) * 2 * TILE + TILE);
    }
    if (!CAUSAL || kb <= qw0 + 63) {
      // S^T of 32-key half t for both row groups: one K fragment burst, two MFMA chains
      auto qk = [&](int t, f32x16 (&sx)[2], auto diagc) {
        constexpr bool DIAG = decltype(diagc)::value;
        bf16x8_t fr[NKS];
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) fr[kk] = lds_b128(Ks + ((kk & 1) ? rb1 : rb0) + 4 * G8 * t + 512 * (kk >> 1));
        sx[0] = zero16();
        sx[1] = zero16();
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          sx[0] = mfma32(fr[kk], qf[0][kk], sx[0]);
          sx[1] = mfma32(fr[kk], qf[1][kk], sx[1]);
        }
        if constexpr (DIAG) {
#pragma unroll
          for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int kofs = kb + 32 * t - (qw0 + 32 * g) + (r & 3) + 8 * (r >> 2) + 4 * h;
              sx[g][r] = kofs > l32 ? -INFINITY : sx[g][r];
            }
        }
      };
      auto rescale = [&](int g, float mt_raw) {
        const float mts = mt_raw * scale2;
        if (__builtin_amdgcn_ballot_w64(mts > m[g] + THR) != 0) {
          const float mn = fmaxf(m[g], mts);
          const float a = mn == -INFINITY ? 1.f : fast_exp2(m[g] - mn);
#pragma unroll
          for (int i = 0; i < NDB; ++i) o[g][i] *= a;
          lsum[g] *= a;
          m[g] = mn;
        }
      };
      auto softmax = [&](int g, f32x16& sx, bf16x8_t& p0, bf16x8_t& p1) {
        const float nm = -m[g];
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          sx[r] = fast_exp2(fmaf(sx[r], scale2, nm));
          sx[r + 1] = fast_exp2(fmaf(sx[r + 1], scale2, nm));
          a0 += sx[r];
          a1 += sx[r + 1];
        }
        lsum[g] += a0 + a1;
        p0 = acc_to_bf16(sx, 0);
        p1 = acc_to_bf16(sx, 1);
      };
      // O^T += V^T P^T for half t, both groups: one V^T burst, each fragment feeds two MFMAs. The
      // reads go out a phase ahead of their MFMAs (vread), so their latency hides under the softmax.
      auto vread = [&](int t, bf16x8_t (&fr)[2 * NDB]) {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const int ts = 2 * t + st;
            fr[st * NDB + db] = lds_tr8_asm(Vs + tb0 + G8 * (2 * ts) + 512 * db, Vs + tb1 + G8 * (2 * ts + 1) + 512 * db);
          }
      };
      auto pv = [&](bf16x8_t (&fr)[2 * NDB], const bf16x8_t (&p)[2][2]) {
        lds_tr_settle(fr);
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            o[0][db] = mfma32(fr[st * NDB + db], p[0][st], o[0][db]);
            o[1][db] = mfma32(fr[st * NDB + db], p[1][st], o[1][db]);
          }
      };
      // half 1's S^T MFMAs beside half 0's softmax, half 0's P.V beside half 1's row maxima
      auto run = [&](auto diagc) {
        f32x16 s0[2], s1[2];
        bf16x8_t v0[2 * NDB], v1[2 * NDB];
        qk(0, s0, diagc);
        vread(0, v0);
        rescale(0, xhalf_max(max16(s0[0], -INFINITY)));
        rescale(1, xhalf_max(max16(s0[1], -INFINITY)));
        qk(1, s1, diagc);
        bf16x8_t p0[2][2];
        softmax(0, s0[0], p0[0][0], p0[0][1]);
        softmax(1, s0[1], p0[1][0], p0[1][1]);
        const float mt10 = xhalf_max(max16(s1[0], -INFINITY)), mt11 = xhalf_max(max16(s1[1], -INFINITY));
        pv(v0, p0);
        vread(1, v1);
        rescale(0, mt10);
        rescale(1, mt11);
        bf16x8_t p1[2][2];
        softmax(0, s1[0], p1[0][0], p1[0][1]);
        softmax(1, s1[1], p1[1][0], p1[1][1]);
        pv(v1, p1);
      };
      if (CAUSAL && kb + BK - 1 > qw0) {
        run(std::integral_constant<bool, CAUSAL>{});
      } else {
        run(std::false_type{});
      }
    }
    if (more) wait_dma();
    __syncthreads();
  };
  for (int it = 0; it < ntile; it += 2) {
    tile(IC<0>{}, it);
    tile(IC<1>{}, it + 1);
  }

#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int qrow = qw0 + 32 * g + l32;
    const float lt = xhalf_sum(lsum[g]);
    const float inv = 1.f / lt;
    bf16_t* Or = O + ((long)b * S + qrow) * so + (long)hq * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        store4(Or + 32 * db + 8 * gg + 4 * h, o[g][db][4 * gg] * inv, o[g][db][4 * gg + 1] * inv,
               o[g][db][4 * gg + 2] * inv, o[g][db][4 * gg + 3] * inv);
      }
    }
    if (h == 0) LSE[(long)bh * S + qrow] = m[g] + __log2f(lt);
  }
}

template __global__ void attn_fwd_wide_kernel<true>(const bf16_t* __restrict__, const bf16_t* __restrict__,
                                                     const bf16_t* __restrict__, bf16_t* __restrict__,
                                                     float* __restrict__, int, int, int, int, long, long, long, long,
                                                     float);
template __global__ void attn_fwd_wide_kernel<false>(const bf16_t* __restrict__, const bf16_t* __restrict__,
                                                      const bf16_t* __restrict__, bf16_t* __restrict__,
                                                      float* __restrict__, int, int, int, int, long, long, long, long,
                                                      float);

}  // namespace

// Forward kernel choice for D = 128 (A/B): 0 = 32 rows per wave (attention.hip), 1 = this
// kernel (RCA_ATTN_FWD=wide), 2 = the hand-scheduled 64-row kernel (attention_fwd_hs.hip,
// RCA_ATTN_FWD=hs); 1 and 2 need S % 256 == 0. Also measured and dropped: the 32-row kernel with
// s_setprio(1) around its MFMA clusters, 0.296 vs 0.288 ms (profiles/attn_fwd_wide_ab_r4.log).
static int g_fwd_mode = [] {
  const char* e = getenv("RCA_ATTN_FWD");
  return !e ? 0 : e[0] == 'w' ? 1 : e[0] == 'h' ? 2 : 0;
}();
RCA_API int rca_attn_set_fwd_mode(int mode) {
  const int old = g_fwd_mode;
  g_fwd_mode = mode;
  return old;
}

bool rca_attn_launch_fwd_hs(bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse,
                            int B, int S, int Hq, int Hk, long sq, long sk, long sv, long so, float scale2,
                            hipStream_t st);

// Returns false when no 64-row kernel is selected for the shape (the caller runs the 32-row one).
bool rca_attn_launch_fwd_wide(bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse,
                              int B, int S, int Hq, int Hk, long sq, long sk, long sv, long so, float scale2,
                              hipStream_t st) {
  if (g_fwd_mode == 2) return rca_attn_launch_fwd_hs(causal, q, k, v, o, lse, B, S, Hq, Hk, sq, sk, sv, so, scale2, st);
  if (g_fwd_mode != 1 || S % 256) return false;
  const dim3 grid(B * Hq * (S / 256)), block(kThreads);
  if (causal)
    hipLaunchKernelGGL((attn_fwd_wide_kernel<true>), grid, block, 0, st, q, k, v, o, lse, B, S, Hq, Hk, sq, sk, sv, so,
                       scale2);
  else
    hipLaunchKernelGGL((attn_fwd_wide_kernel<false>), grid, block, 0, st, q, k, v, o, lse, B, S, Hq, Hk, sq, sk, sv,
                       so, scale2);
  return true;
}
