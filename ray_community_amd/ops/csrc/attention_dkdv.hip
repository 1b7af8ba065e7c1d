// dK/dV of the gfx950 flash attention (see attention.hip for the forward / dQ and the layout
// conventions). Compiled WITHOUT -amdgpu-mfma-vgpr-form (ops/build.py FILE_FLAGS): with one wave
// per SIMD its dK^T/dV^T accumulators sit in AGPRs, which frees the arch VGPRs for whole operand
// bursts (16 ds_read_b128 then 16 MFMAs) instead of read/wait/MFMA interleaving; measured 6 % less
// backward time at the Llama-3-8B shape (scripts/gpu_attn_acc.sh).
#include "attention_common.h"

#include <cstdlib>

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

}  // namespace

void rca_attn_launch_dkdv(int D, bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                          const float* lse, const float* delta, bf16_t* dk, bf16_t* dv, int B, int S, int Hq, int Hk,
                          long sq, long sk, long sv, long sdo, long sdk, long sdv, float scale2, float scale,
                          hipStream_t st) {
  // RCA_ATTN_DKDV_NH=1 selects the unpipelined 32-row-slice variant (A/B measurements)
  static const int nh = [] {
    const char* e = getenv("RCA_ATTN_DKDV_NH");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  const dim3 grid(B * Hk * (S / 128)), block(kThreads);
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
