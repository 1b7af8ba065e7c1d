// dK/dV of the gfx950 flash attention (see attention.hip for the forward / dQ and the layout
// conventions). Compiled WITHOUT -amdgpu-mfma-vgpr-form (ops/build.py FILE_FLAGS): with one wave
// per SIMD its dK^T/dV^T accumulators sit in AGPRs, which frees the arch VGPRs for whole operand
// bursts (16 ds_read_b128 then 16 MFMAs) instead of read/wait/MFMA interleaving; measured 6 % less
// backward time at the Llama-3-8B shape (scripts/gpu_attn_acc.sh).
#include "attention_common.h"

#include <cstdlib>
#include <string>

namespace {

// ---------------------------------------------------------------------------------------------
// dK, dV (key-major; the kv group's query heads are summed in registers, no atomics). Query
// slices of NH x 32 rows stream through a 2-deep LDS ring (loop unrolled over it). Per 32-row
// half: Q/dO row burst -> S, dP MFMAs (key on the lane, two independent chains), P/dS on the VALU,
// dO^T/Q^T transposed burst -> dV^T, dK^T MFMAs. With NH = 2 the halves are software-pipelined in
// one basic block (half 1's S/dP MFMAs beside half 0's P/dS VALU work, half 0's dV/dK MFMAs beside
// half 1's), and one barrier serves 64 query rows. One wave per SIMD (K, V fragments + both
// accumulators stay in registers; build flag -amdgpu-mfma-vgpr-form keeps the accumulators out of
// copies).
template <int D, bool CAUSAL, int NH>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long sdo, long sdk, long sdv, float scale2, float scale) {
  constexpr int BKV = 128, BQS = 32 * NH, NKS = D / 16, NDB = D / 32, SL = BQS * D * 2, G8 = Img<D>::G8;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * SL];
  __shared__ __attribute__((aligned(16))) float rowc[2][2][BQS];  // [slot][-lse, -delta][row]

  const int nkb = S / BKV, G = Hq / Hk;
  int bhk, kbi;
  xcd_group_map(blockIdx.x, B * Hk, nkb, bhk, kbi);  // causal: key block 0 (sees every query) first
  const int b = bhk / Hk, hk = bhk % Hk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int k0 = kbi * BKV, kw0 = k0 + 32 * w, key = kw0 + l32;
  const int rb0 = Img<D>::row_base(l32, h, 0), rb1 = Img<D>::row_base(l32, h, 1);
  const int tb0 = Img<D>::tr_base(lane, 0), tb1 = Img<D>::tr_base(lane, 1);

  bf16x8_t kf[NKS], vf[NKS];
  {
    const bf16_t* Kr = K + ((long)b * S + key) * sk + (long)hk * D;
    const bf16_t* Vr = V + ((long)b * S + key) * sv + (long)hk * D;
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      kf[kk] = gload8(Kr + 16 * kk + 8 * h);
      vf[kk] = gload8(Vr + 16 * kk + 8 * h);
    }
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      settle(kf[kk]);
      settle(vf[kk]);
    }
  }
  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) {
    dk[i] = zero16();
    dv[i] = zero16();
  }

  const int qs0 = CAUSAL ? k0 : 0;
  const int nsl = (S - qs0) / BQS;  // even (S - qs0 is a multiple of 128)
  const int total = G * nsl;        // even

  Stage<D, BQS> qst, gst;
  qst.init(Q + (long)b * S * sq + (long)hk * G * D, sq, S, tid, G * D);
  gst.init(dO + (long)b * S * sdo + (long)hk * G * D, sdo, S, tid, G * D);
  const float* rsrc = (tid < BQS ? LSE : Delta) + ((long)b * Hq + hk * G) * S + (tid & (BQS - 1));
  float rc = 0.f;
  auto stage_load = [&](int g, int sl) {
    const int qa = qs0 + sl * BQS;
    qst.load(qa, sq, g * D * 2);  // head g of the kv group (the descriptor spans all G heads)
    gst.load(qa, sdo, g * D * 2);
    if (tid < 2 * BQS) rc = rsrc[(long)g * S + qa];
  };
  auto stage_store = [&](int buf) {
    qst.store(smem + buf * 2 * SL);
    gst.store(smem + buf * 2 * SL + SL);
    if (tid < 2 * BQS) rowc[buf][tid / BQS][tid & (BQS - 1)] = -rc;  // -lse, -delta
  };

  stage_load(0, nsl - 1);
  stage_store(0);
  __syncthreads();

  // Query slices are swept from the LAST one down to the key block (heads innermost), so the key
  // blocks of one (batch, kv head) resident on an XCD read the same Q/dO slice at the same time.
  auto slice = [&](auto bufc, int i) {
    constexpr int buf = decltype(bufc)::value;
    const char* Qs = smem + buf * 2 * SL;
    const char* Gs = Qs + SL;
    const int sl = nsl - 1 - i / G;
    const bool more = i + 1 < total;
    if (more) stage_load((i + 1) % G, nsl - 1 - (i + 1) / G);
    const int qa = qs0 + sl * BQS;
    if (!CAUSAL || qa + BQS - 1 >= kw0) {
      // S and dP of half t (rows 32t..32t+31 of the slice): row-operand burst + two MFMA chains.
      // dP's chain starts from -delta (the row constant as the initial accumulator: dS = P * dP'
      // needs no subtraction afterwards)
      auto sdp = [&](int t, f32x16& s, f32x16& dp) {
        bf16x8_t fr[2 * NKS];
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          const int o = ((kk & 1) ? rb1 : rb0) + 4 * G8 * t + 512 * (kk >> 1);
          fr[kk] = lds_b128(Qs + o);
          fr[NKS + kk] = lds_b128(Gs + o);
        }
        s = zero16();
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(&rowc[buf][1][32 * t + 8 * g4 + 4 * h]);
#pragma unroll
          for (int j = 0; j < 4; ++j) dp[4 * g4 + j] = d4[j];
        }
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          s = mfma32(fr[kk], kf[kk], s);
          dp = mfma32(fr[NKS + kk], vf[kk], dp);
        }
      };
      // P = exp2(S*c - lse), dS = P * (dP - delta) on the VALU. The causal mask is compiled only
      // into the diagonal variant (DIAG): a runtime `if` here became an unconditional
      // compare + select per element (64 VALU per slice) on every off-diagonal slice.
      auto pds = [&](int t, f32x16& s, f32x16& dp, auto diagc) {
        constexpr bool DIAG = decltype(diagc)::value;
        const bool diag = DIAG && qa + 32 * t < kw0 + 31;
        const int kq = key - qa - 32 * t - 4 * h;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(&rowc[buf][0][32 * t + 8 * g4 + 4 * h]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g4 + j;
            float p = fast_exp2(fmaf(s[r], scale2, l4[j]));
            if constexpr (DIAG) {
              if (diag) p = kq > 8 * g4 + j ? 0.f : p;
            }
            s[r] = p;
            dp[r] = p * dp[r];
          }
        }
      };
      // dV^T += dO^T P^T, dK^T += Q^T dS^T for half t: transposed burst + MFMAs
      auto acc = [&](int t, const f32x16& s, const f32x16& dp) {
        const bf16x8_t pf0 = acc_to_bf16(s, 0), pf1 = acc_to_bf16(s, 1);
        const bf16x8_t df0 = acc_to_bf16(dp, 0), df1 = acc_to_bf16(dp, 1);
        bf16x8_t fr[4 * NDB];
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const int o0 = tb0 + G8 * (4 * t + 2 * st) + 512 * db, o1 = tb1 + G8 * (4 * t + 2 * st + 1) + 512 * db;
            fr[(2 * st) * NDB + db] = lds_tr8(Gs + o0, Gs + o1);
            fr[(2 * st + 1) * NDB + db] = lds_tr8(Qs + o0, Qs + o1);
          }
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          dv[db] = mfma32(fr[db], pf0, dv[db]);
          dk[db] = mfma32(fr[NDB + db], df0, dk[db]);
        }
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          dv[db] = mfma32(fr[2 * NDB + db], pf1, dv[db]);
          dk[db] = mfma32(fr[3 * NDB + db], df1, dk[db]);
        }
      };
      auto body = [&](auto diagc) {
        f32x16 s[NH], dp[NH];
#pragma unroll
        for (int t = 0; t < NH; ++t) sdp(t, s[t], dp[t]);
#pragma unroll
        for (int t = 0; t < NH; ++t) {
          pds(t, s[t], dp[t], diagc);
          acc(t, s[t], dp[t]);
        }
      };
      if (CAUSAL && qa < kw0 + 31) {
        body(std::integral_constant<bool, CAUSAL>{});
      } else {
        body(std::false_type{});
      }
    }
    if (more) stage_store(buf ^ 1);
    __syncthreads();
  };
  for (int i = 0; i < total; i += 2) {
    slice(IC<0>{}, i);
    slice(IC<1>{}, i + 1);
  }

  bf16_t* dKr = dK + ((long)b * S + key) * sdk + (long)hk * D;
  bf16_t* dVr = dV + ((long)b * S + key) * sdv + (long)hk * D;
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      store4(dKr + 32 * db + 8 * g + 4 * h, dk[db][4 * g] * scale, dk[db][4 * g + 1] * scale,
             dk[db][4 * g + 2] * scale, dk[db][4 * g + 3] * scale);
      store4(dVr + 32 * db + 8 * g + 4 * h, dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Hand-scheduled dK/dV (D = 128, RCA_ATTN_DKDV=hs). Same work split, LDS image and math as the
// kernel above; what changes is who places the instructions. The compiler-scheduled kernel runs
// at 38 % MFMA utilisation at one wave per SIMD (profiles/attention_bwd_r3.md): its P/dS VALU
// work, operand reads and the S/dP -> P/dS -> dV/dK dependencies leave the matrix pipe idle. Here
// every MFMA is an asm statement and each 32-cycle v_mfma_f32_32x32x16_bf16 gets its gap filled
// by hand (sched_barrier fences pin the slots), software-pipelined over the slice's two 32-row
// halves h = 0, 1:
//   P0            DMA of the next Q/dO slice into the other buffer; row fragments R_0; -lse/-delta
//   P1 (16 MFMA)  S_0, dP_0 chains        + R_1 reads (into the registers R_0 frees)
//   P2 (16 MFMA)  S_1, dP_1 chains        + P/dS VALU of half 0 (one row element per slot) + T_0 reads
//   P3 (16 MFMA)  dV, dK += half 0        + P/dS VALU of half 1 + T_1 reads
//   P4 (16 MFMA)  dV, dK += half 1
// then the DMA wait + barrier. Q/dO slices are staged by LDS-DMA and every LDS read is inline asm
// (explicit lgkmcnt waits at phase boundaries), so no staging registers and no compiler-inserted
// DMA drains. MFMA results read by the VALU (S, dP) and VALU results read by MFMAs (P, dS) are
// one phase apart, plus s_nops at the boundaries: the hazard recognizer does not see asm MFMAs.
__device__ __forceinline__ bf16x8_t ldsq(const char* p) {
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(__UINTPTR_TYPE__)p));
  return __builtin_bit_cast(bf16x8_t, v);
}
__device__ __forceinline__ f32x4 ldsf4(const float* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(__UINTPTR_TYPE__)p));
  return v;
}
__device__ __forceinline__ void hs_fence() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ void hs_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// >= 18 wait states between an XDL write and a VALU read of the result (and the reverse)
__device__ __forceinline__ void hs_xdl_gap() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory"); }
#define HS_MFV(acc, a, b) asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define HS_MFA(acc, a, b) asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b))

template <bool CAUSAL>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_hs_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long sdo, long sdk, long sdv, float scale2, float scale) {
  constexpr int D = 128, BKV = 128, BQS = 64, NKS = 8, NDB = 4, SL = BQS * D * 2, G8 = Img<D>::G8;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * SL];
  __shared__ __attribute__((aligned(16))) float rowc[2][2][BQS];  // [slot][-lse, -delta][row]

  const int nkb = S / BKV, G = Hq / Hk;
  int bhk, kbi;
  xcd_group_map(blockIdx.x, B * Hk, nkb, bhk, kbi);
  const int b = bhk / Hk, hk = bhk % Hk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int k0 = kbi * BKV, kw0 = k0 + 32 * w, key = kw0 + l32;
  const int rb0 = Img<D>::row_base(l32, h, 0), rb1 = Img<D>::row_base(l32, h, 1);
  const int tb0 = Img<D>::tr_base(lane, 0), tb1 = Img<D>::tr_base(lane, 1);

  bf16x8_t kf[NKS], vf[NKS];
  {
    const bf16_t* Kr = K + ((long)b * S + key) * sk + (long)hk * D;
    const bf16_t* Vr = V + ((long)b * S + key) * sv + (long)hk * D;
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      kf[kk] = gload8(Kr + 16 * kk + 8 * h);
      vf[kk] = gload8(Vr + 16 * kk + 8 * h);
    }
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      settle(kf[kk]);
      settle(vf[kk]);
    }
  }
  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) {
    dk[i] = zero16();
    dv[i] = zero16();
  }

  const int qs0 = CAUSAL ? k0 : 0;
  const int nsl = (S - qs0) / BQS;
  const int total = G * nsl;  // even
  DmaStage<D, BQS> qst, gst;
  qst.init(Q + (long)b * S * sq + (long)hk * G * D, sq, S, tid, G * D);
  gst.init(dO + (long)b * S * sdo + (long)hk * G * D, sdo, S, tid, G * D);
  const float* rsrc = (tid < BQS ? LSE : Delta) + ((long)b * Hq + hk * G) * S + (tid & (BQS - 1));
  float rc = 0.f;
  auto stage_issue = [&](int g, int sl, int buf) {
    const int qa = qs0 + sl * BQS;
    qst.issue(qa, sq, smem + buf * 2 * SL, g * D * 2);
    gst.issue(qa, sdo, smem + buf * 2 * SL + SL, g * D * 2);
    if (tid < 2 * BQS) rc = rsrc[(long)g * S + qa];
  };
  auto stage_finish = [&](int buf) {
    wait_dma();
    if (tid < 2 * BQS) rowc[buf][tid / BQS][tid & (BQS - 1)] = -rc;  // -lse, -delta
  };
  stage_issue(0, nsl - 1, 0);
  stage_finish(0);
  __syncthreads();

  auto slice = [&](auto bufc, int i) {
    constexpr int buf = decltype(bufc)::value;
    const char* Qs = smem + buf * 2 * SL;
    const char* Gs = Qs + SL;
    const int sl = nsl - 1 - i / G;
    const bool more = i + 1 < total;
    if (more) stage_issue((i + 1) % G, nsl - 1 - (i + 1) / G, buf ^ 1);
    const int qa = qs0 + sl * BQS;
    if (!CAUSAL || qa + BQS - 1 >= kw0) {
      auto body = [&](auto diagc) {
        constexpr bool DIAG = decltype(diagc)::value;
        auto roff = [&](int kk, int t) { return ((kk & 1) ? rb1 : rb0) + 4 * G8 * t + 512 * (kk >> 1); };
        // ---- P0: R_0, the row constants of both halves
        bf16x8_t fq[NKS], fg[NKS];
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          fq[kk] = ldsq(Qs + roff(kk, 0));
          fg[kk] = ldsq(Gs + roff(kk, 0));
        }
        f32x4 nl[2][4], nd[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            nl[t][g4] = ldsf4(&rowc[buf][0][32 * t + 8 * g4 + 4 * h]);
            nd[t][g4] = ldsf4(&rowc[buf][1][32 * t + 8 * g4 + 4 * h]);
          }
        hs_lgkm0();
        hs_fence();
        f32x16 s0 = zero16(), s1 = zero16(), dp0, dp1;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            dp0[4 * g4 + j] = nd[0][g4][j];
            dp1[4 * g4 + j] = nd[1][g4][j];
          }
        hs_fence();
        // ---- P1: S_0 / dP_0 chains + R_1 reads into the freed fragment registers
        bf16x8_t fq1[NKS], fg1[NKS];
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          hs_fence();
          HS_MFV(s0, fq[kk], kf[kk]);
          hs_fence();
          fq1[kk] = ldsq(Qs + roff(kk, 1));
          hs_fence();
          HS_MFV(dp0, fg[kk], vf[kk]);
          hs_fence();
          fg1[kk] = ldsq(Gs + roff(kk, 1));
        }
        hs_fence();
        hs_lgkm0();
        hs_xdl_gap();
        hs_fence();
        // P/dS of half t, element r (one per MFMA slot): p = exp2(S c - lse), dS' = p (dP - delta)
        const int kq0 = key - qa - 4 * h;
        auto pds1 = [&](f32x16& sx, f32x16& dx, int t, int r) {
          const int g4 = r >> 2, j = r & 3;
          float p = fast_exp2(fmaf(sx[r], scale2, nl[t][g4][j]));
          if constexpr (DIAG) p = (kq0 - 32 * t > 8 * g4 + j) ? 0.f : p;
          sx[r] = p;
          dx[r] = p * dx[r];
        };
        // transposed operand f (0..15) of half t: f = (2*st + isq) * NDB + db, st = k-step of the
        // 32-row half, isq 0: dO^T (-> dV), 1: Q^T (-> dK); read just in time, TW operands ahead
        constexpr int TW = 4;
        auto trd = [&](int t, int f) {
          const int st = (f / NDB) >> 1, db = f % NDB, isq = (f / NDB) & 1;
          const int o0 = tb0 + G8 * (4 * t + 2 * st) + 512 * db, o1 = tb1 + G8 * (4 * t + 2 * st + 1) + 512 * db;
          return lds_tr8_asm((isq ? Qs : Gs) + o0, (isq ? Qs : Gs) + o1);
        };
        // MFMA q (0..15) of the dV/dK phase: operand f = (2*st + isdk)*NDB + db with st = q >> 3,
        // db = (q >> 1) & 3, isdk = q & 1 -> f order matches q order below (q -> f(q))
        auto fq_of = [](int q) { return (2 * (q >> 3) + (q & 1)) * NDB + ((q >> 1) & 3); };
        // ---- P2: S_1 / dP_1 chains + P/dS of half 0; the first TW T_0 operands at the end
        bf16x8_t pa0, pb0, da0, db0;
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          hs_fence();
          HS_MFV(s1, fq1[kk], kf[kk]);
          hs_fence();
          pds1(s0, dp0, 0, 2 * kk);
          hs_fence();
          HS_MFV(dp1, fg1[kk], vf[kk]);
          hs_fence();
          pds1(s0, dp0, 0, 2 * kk + 1);
          if (kk == 3) {
            pa0 = acc_to_bf16(s0, 0);
            da0 = acc_to_bf16(dp0, 0);
          }
        }
        hs_fence();
        pb0 = acc_to_bf16(s0, 1);
        db0 = acc_to_bf16(dp0, 1);
        bf16x8_t tw[16];
#pragma unroll
        for (int q = 0; q < TW; ++q) tw[q] = trd(0, fq_of(q));
        hs_xdl_gap();
        hs_fence();
        // ---- P3: dV, dK += half 0 (T_0 read TW ahead) + P/dS of half 1
        bf16x8_t pa1, pb1, da1, db1;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          hs_fence();
          // T_0 operand q landed: the 2 * (later reads in flight) newest LDS ops may stay pending
          {
            const int later = (q + TW < 16 ? TW - 1 : 15 - q);
            if (later >= 3) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
            else if (later == 2) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
            else if (later == 1) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          hs_fence();
          {
            const int st = q >> 3, db = (q >> 1) & 3;
            if (q & 1) HS_MFA(dk[db], tw[q], st ? db0 : da0);
            else HS_MFA(dv[db], tw[q], st ? pb0 : pa0);
          }
          hs_fence();
          if (q + TW < 16) tw[q + TW] = trd(0, fq_of(q + TW));
          pds1(s1, dp1, 1, q);
          if (q == 7) {
            pa1 = acc_to_bf16(s1, 0);
            da1 = acc_to_bf16(dp1, 0);
          }
        }
        hs_fence();
        pb1 = acc_to_bf16(s1, 1);
        db1 = acc_to_bf16(dp1, 1);
#pragma unroll
        for (int q = 0; q < TW; ++q) tw[q] = trd(1, fq_of(q));
        hs_xdl_gap();
        hs_fence();
        // ---- P4: dV, dK += half 1 (T_1 read TW ahead)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          hs_fence();
          {
            const int later = (q + TW < 16 ? TW - 1 : 15 - q);
            if (later >= 3) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
            else if (later == 2) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
            else if (later == 1) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          hs_fence();
          {
            const int st = q >> 3, db = (q >> 1) & 3;
            if (q & 1) HS_MFA(dk[db], tw[q], st ? db1 : da1);
            else HS_MFA(dv[db], tw[q], st ? pb1 : pa1);
          }
          hs_fence();
          if (q + TW < 16) tw[q + TW] = trd(1, fq_of(q + TW));
        }
        hs_fence();
      };
      if (CAUSAL && qa < kw0 + 31) body(std::integral_constant<bool, CAUSAL>{});
      else body(std::false_type{});
    }
    if (more) stage_finish(buf ^ 1);
    __syncthreads();
  };
  for (int i = 0; i < total; i += 2) {
    slice(IC<0>{}, i);
    slice(IC<1>{}, i + 1);
  }

  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
    asm volatile("" : "+a"(dk[db]));
    asm volatile("" : "+a"(dv[db]));
  }
  bf16_t* dKr = dK + ((long)b * S + key) * sdk + (long)hk * D;
  bf16_t* dVr = dV + ((long)b * S + key) * sdv + (long)hk * D;
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      store4(dKr + 32 * db + 8 * g + 4 * h, dk[db][4 * g] * scale, dk[db][4 * g + 1] * scale,
             dk[db][4 * g + 2] * scale, dk[db][4 * g + 3] * scale);
      store4(dVr + 32 * db + 8 * g + 4 * h, dv[db][4 * g], dv[db][4 * g + 1], dv[db][4 * g + 2], dv[db][4 * g + 3]);
    }
  }
}
#undef HS_MFV
#undef HS_MFA

template __global__ void attn_bwd_dkdv_hs_kernel<true>(const bf16_t* __restrict__, const bf16_t* __restrict__,
                                                        const bf16_t* __restrict__, const bf16_t* __restrict__,
                                                        const float* __restrict__, const float* __restrict__,
                                                        bf16_t* __restrict__, bf16_t* __restrict__, int, int, int,
                                                        int, long, long, long, long, long, long, float, float);
template __global__ void attn_bwd_dkdv_hs_kernel<false>(const bf16_t* __restrict__, const bf16_t* __restrict__,
                                                         const bf16_t* __restrict__, const bf16_t* __restrict__,
                                                         const float* __restrict__, const float* __restrict__,
                                                         bf16_t* __restrict__, bf16_t* __restrict__, int, int, int,
                                                         int, long, long, long, long, long, long, float, float);

}  // namespace

void rca_attn_launch_dkdv(int D, bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                          const float* lse, const float* delta, bf16_t* dk, bf16_t* dv, int B, int S, int Hq, int Hk,
                          long sq, long sk, long sv, long sdo, long sdk, long sdv, float scale2, float scale,
                          hipStream_t st) {
  // RCA_ATTN_DKDV_NH=1 selects the unpipelined 32-row-slice variant (A/B measurements);
  // RCA_ATTN_DKDV=hs the hand-scheduled kernel (D = 128)
  static const int nh = [] {
    const char* e = getenv("RCA_ATTN_DKDV_NH");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  static const bool hs = [] {
    const char* e = getenv("RCA_ATTN_DKDV");
    return e && std::string(e) == "hs";
  }();
  const dim3 grid(B * Hk * (S / 128)), block(kThreads);
  if (hs && D == 128) {
    if (causal)
      hipLaunchKernelGGL((attn_bwd_dkdv_hs_kernel<true>), grid, block, 0, st, q, k, v, dout, lse, delta, dk, dv, B, S,
                         Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale);
    else
      hipLaunchKernelGGL((attn_bwd_dkdv_hs_kernel<false>), grid, block, 0, st, q, k, v, dout, lse, delta, dk, dv, B,
                         S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale);
    return;
  }
#define RCA_DKDV(DD, CC, NN)                                                                                           \
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<DD, CC, NN>), grid, block, 0, st, q, k, v, dout, lse, delta, dk, dv, B, S, \
                     Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale)
  if (D == 128) {
    if (causal) {
      if (nh == 1) RCA_DKDV(128, true, 1); else RCA_DKDV(128, true, 2);
    } else {
      if (nh == 1) RCA_DKDV(128, false, 1); else RCA_DKDV(128, false, 2);
    }
  } else {
    if (causal) {
      if (nh == 1) RCA_DKDV(64, true, 1); else RCA_DKDV(64, true, 2);
    } else {
      if (nh == 1) RCA_DKDV(64, false, 1); else RCA_DKDV(64, false, 2);
    }
  }
#undef RCA_DKDV
}
