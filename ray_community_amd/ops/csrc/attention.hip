// Flash attention (causal / full, GQA) forward + backward for gfx950 (MI355X / CDNA4), bf16 I/O,
// fp32 accumulation on v_mfma_f32_32x32x16_bf16.
//
// Layout: q/k/v/o/do/dq/dk/dv are [B, S, H, D] with an arbitrary TOKEN stride (elements) and the
// head stride D, so the kernels read Q/K/V straight out of the fused qkv projection output
// ([B*S, (Hq+2Hk)*D]) and write dQ/dK/dV straight into the fused dqkv gradient: no transposes,
// no contiguous() copies. LSE is [B, Hq, S] fp32 in the log2 domain (scores pre-scaled by
// softmax_scale * log2(e)).
//
// Structure (see cdna_hip_programming.md App. B "Fused attention prefill" / "Attention backward"):
//  * forward   — one workgroup = 4 waves = 128 query rows of one head; Q lives in VGPRs for the
//                whole kernel; K/V tiles of 64 keys are register-staged (global loads issued before
//                the tile's MFMAs, LDS writes after them) into a 2-deep LDS ring with an XOR-swizzled
//                256-B-row image. Swapped product S^T = K.Q^T puts one query row on each lane, so the
//                online-softmax row max/sum are lane-local (+1 cross-half shuffle), and the S^T
//                accumulator is directly the B operand of O^T += V^T.P^T (no LDS round trip for P);
//                V^T fragments come from ds_read_b64_tr_b16 hardware-transposed LDS reads.
//  * dK/dV     — one workgroup = 4 waves = 128 keys of one kv head; each wave keeps its 32 keys' K, V
//                fragments in VGPRs and dK^T/dV^T accumulators in registers while the workgroup
//                sweeps the kv-group's query heads x 32-row query slices (Q/dO slices staged in LDS).
//                S and dP are computed key-on-lane so P and dS are the B operands of dV^T and dK^T.
//                GQA reduction over the query heads happens in registers: no atomics.
//  * dQ        — query-major twin of the forward (recomputes P from LSE, dP from dO.V^T) and
//                accumulates dQ^T = K^T.dS^T in registers: deterministic, no float atomics.
// Reference behaviour: torch SDPA / flash-attention semantics as used by the reference's Train
// examples (python/ray/train/examples, release/train_tests) — the reference itself has no kernel.
#include "attention_common.h"

#include <cstdlib>

// dK/dV lives in attention_dkdv.hip (its own register-form flags)
void rca_attn_launch_dkdv(int D, bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                          const float* lse, const float* delta, bf16_t* dk, bf16_t* dv, int B, int S, int Hq, int Hk,
                          long sq, long sk, long sv, long sdo, long sdk, long sdv, float scale2, float scale,
                          hipStream_t st, bf16_t* dSw, long tiles_bh);
// recompute-free dQ (attention_dq.hip)
long rca_attn_ds_ws_bytes(int B, int S, int Hq, int D, bool causal);
void rca_attn_launch_delta(const bf16_t* o, const bf16_t* dout, float* delta, int B, int S, int Hq, long so, long sdo,
                           hipStream_t st);
void rca_attn_launch_dq_ds(bool causal, const bf16_t* k, const bf16_t* dsw, bf16_t* dq, int B, int S, int Hq, int Hk,
                           long sk, long sdq, float scale, hipStream_t st);
// 64-query-rows-per-wave forward (attention_fwd_wide.hip); false = not selected for this shape
bool rca_attn_launch_fwd_wide(bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse,
                              int B, int S, int Hq, int Hk, long sq, long sk, long sv, long so, float scale2,
                              hipStream_t st);

namespace {

// ---------------------------------------------------------------------------------------------
// Forward. Per 64-key tile each wave runs four clusters: K operand burst (16 x ds_read_b128 into
// registers), S^T MFMAs (two independent 32-key chains), softmax on the VALU, V^T operand burst
// (32 x ds_read_b64_tr_b16), P.V MFMAs. Two workgroups per CU put two waves on every SIMD, so one
// wave's load/VALU clusters run beside the other's MFMA clusters. The loop is unrolled over the
// 2-deep LDS ring so every LDS address is base register + immediate. The online-softmax rescale is
// deferred (only when a row max grows by > 8 in log2 units: P <= 2^8, exact f32 accumulation)
// and wave-uniform.
// DMA: K/V tiles go HBM -> LDS by buffer_load ... lds (DmaStage) instead of the register-staged
// global load + ds_write pair (Stage); RCA_ATTN_DMA=0 selects the latter (A/B).
// NW = 8: one 512-thread workgroup of 8 waves (two per SIMD) covers 256 query rows, so each K/V
// tile staged into LDS serves twice the rows: half the L2 -> LDS DMA bytes per MFMA of the 4-wave
// form (whose two co-resident workgroups each stage their own copy). Waves 0-3 issue the DMA.
template <int D, bool CAUSAL, bool DMA, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_fwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    bf16_t* __restrict__ O, float* __restrict__ LSE, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long so, float scale2) {
  static_assert(NW == 4 || (NW == 8 && DMA), "the 8-wave form stages by LDS-DMA");
  constexpr int BQ = 32 * NW, BK = 64, NKS = D / 16, NDB = D / 32, TILE = BK * D * 2, G8 = Img<D>::G8;
  constexpr float THR = 8.f;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];

  const int nqb = S / BQ, G = Hq / Hk;
  // one (batch, kv head) per group: its G query heads x nqb query blocks share the K/V stream
  int bhk, item;
  xcd_group_map(blockIdx.x, B * Hk, G * nqb, bhk, item);
  const int qr = item / G, b = bhk / Hk, hk = bhk % Hk, hq = hk * G + item % G, bh = b * Hq + hq;
  const int qb = CAUSAL ? nqb - 1 - qr : qr;  // longest causal rows first
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int q0 = qb * BQ, qw0 = q0 + 32 * w, qrow = qw0 + l32;
  const int rb0 = Img<D>::row_base(l32, h, 0), rb1 = Img<D>::row_base(l32, h, 1);
  const int tb0 = Img<D>::tr_base(lane, 0), tb1 = Img<D>::tr_base(lane, 1);

  const bf16_t* Kb = K + (long)b * S * sk + (long)hk * D;
  const bf16_t* Vb = V + (long)b * S * sv + (long)hk * D;
  const bf16_t* Qr = Q + ((long)b * S + qrow) * sq + (long)hq * D;

  bf16x8_t qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf[ks] = gload8(Qr + 16 * ks + 8 * h);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) settle(qf[ks]);

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = zero16();
  float m = -INFINITY, lsum = 0.f;

  const int ntile = CAUSAL ? (q0 + BQ) / BK : S / BK;  // always even (S % 128 == 0)
  std::conditional_t<DMA, DmaStage<D, BK>, Stage<D, BK>> kst, vst;
  kst.init(Kb, sk, S, tid);
  vst.init(Vb, sv, S, tid);
  const bool dma_wave = NW == 4 || __builtin_amdgcn_readfirstlane(w) < 4;  // the staging waves
  if constexpr (DMA) {
    if (dma_wave) {
      kst.issue(0, sk, smem);
      vst.issue(0, sv, smem + TILE);
    }
    wait_dma();
  } else {
    kst.load(0, sk);
    vst.load(0, sv);
    kst.store(smem);
    vst.store(smem + TILE);
  }
  __syncthreads();

  auto tile = [&](auto bufc, int it) {
    constexpr int buf = decltype(bufc)::value;
    const char* Ks = smem + buf * 2 * TILE;
    const char* Vs = Ks + TILE;
    const int kb = it * BK;
    const bool more = it + 1 < ntile;
    if (more) {
      if constexpr (DMA) {  // into the other buffer: every wave left it at the last barrier
        if (dma_wave) {
          kst.issue(kb + BK, sk, smem + (buf ^ 1) * 2 * TILE);
          vst.issue(kb + BK, sv, smem + (buf ^ 1) * 2 * TILE + TILE);
        }
      } else {
        kst.load(kb + BK, sk);
        vst.load(kb + BK, sv);
      }
    }
    if (!CAUSAL || kb <= qw0 + 31) {
      // Two 32-key halves, software-pipelined: half 1's S^T MFMAs issue beside half 0's softmax
      // VALU work, and half 0's P.V MFMAs beside half 1's row max.
      auto qk = [&](int t, auto diagc) {
        constexpr bool DIAG = decltype(diagc)::value;
        bf16x8_t fr[NKS];
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) fr[kk] = lds_b128(Ks + ((kk & 1) ? rb1 : rb0) + 4 * G8 * t + 512 * (kk >> 1));
        f32x16 sx = zero16();
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) sx = mfma32(fr[kk], qf[kk], sx);
        if constexpr (DIAG) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kofs = kb + 32 * t - qw0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            sx[r] = kofs > l32 ? -INFINITY : sx[r];
          }
        }
        return sx;
      };
      auto rescale = [&](float mt_raw) {
        const float mts = mt_raw * scale2;
        if (__builtin_amdgcn_ballot_w64(mts > m + THR) != 0) {
          const float mn = fmaxf(m, mts);
          const float a = mn == -INFINITY ? 1.f : fast_exp2(m - mn);
#pragma unroll
          for (int i = 0; i < NDB; ++i) o[i] *= a;
          lsum *= a;
          m = mn;
        }
      };
      auto softmax = [&](f32x16& sx, bf16x8_t& p0, bf16x8_t& p1) {
        const float nm = -m;
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          sx[r] = fast_exp2(fmaf(sx[r], scale2, nm));
          sx[r + 1] = fast_exp2(fmaf(sx[r + 1], scale2, nm));
          a0 += sx[r];
          a1 += sx[r + 1];
        }
        lsum += a0 + a1;
        p0 = acc_to_bf16(sx, 0);
        p1 = acc_to_bf16(sx, 1);
      };
      auto pv = [&](int t, bf16x8_t p0, bf16x8_t p1) {
        bf16x8_t fr[2 * NDB];
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const int ts = 2 * t + st;
            const char* a0 = Vs + tb0 + G8 * (2 * ts) + 512 * db;
            const char* a1 = Vs + tb1 + G8 * (2 * ts + 1) + 512 * db;
            fr[st * NDB + db] = DMA ? lds_tr8_asm(a0, a1) : lds_tr8(a0, a1);
          }
        if constexpr (DMA) lds_tr_settle(fr);
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[db] = mfma32(fr[db], p0, o[db]);
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[db] = mfma32(fr[NDB + db], p1, o[db]);
      };
      // straight-line bodies (masked / unmasked) so each phase is one basic block the scheduler
      // can interleave: half 1's S MFMAs with half 0's softmax, half 0's PV with half 1's max.
      auto run = [&](auto diagc) {
        f32x16 s0 = qk(0, diagc);
        rescale(xhalf_max(max16(s0, -INFINITY)));
        f32x16 s1 = qk(1, diagc);
        bf16x8_t p00, p01;
        softmax(s0, p00, p01);
        const float mt1 = xhalf_max(max16(s1, -INFINITY));
        pv(0, p00, p01);
        rescale(mt1);
        bf16x8_t p10, p11;
        softmax(s1, p10, p11);
        pv(1, p10, p11);
      };
      if (CAUSAL && kb + BK - 1 > qw0) {
        run(std::integral_constant<bool, CAUSAL>{});
      } else {
        run(std::false_type{});
      }
    }
    if (more) {
      if constexpr (DMA) {
        wait_dma();
      } else {
        kst.store(smem + (buf ^ 1) * 2 * TILE);
        vst.store(smem + (buf ^ 1) * 2 * TILE + TILE);
      }
    }
    __syncthreads();
  };
  for (int it = 0; it < ntile; it += 2) {
    tile(IC<0>{}, it);
    tile(IC<1>{}, it + 1);
  }

  const float lt = xhalf_sum(lsum);
  const float inv = 1.f / lt;
  bf16_t* Or = O + ((long)b * S + qrow) * so + (long)hq * D;
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      store4(Or + 32 * db + 8 * g + 4 * h, o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv,
             o[db][4 * g + 3] * inv);
    }
  }
  if (h == 0) LSE[(long)bh * S + qrow] = m + __log2f(lt);
}

// Explicit instantiations: hipcc (ROCm 7.2) referenced but did not emit the host launch stub of
// one of the two DMA instances per head size when they were only instantiated through launch_fwd
// (an undefined __device_stub__ symbol at load time).
#define RCA_FWD_INST(DD, CC, MM, NN)                                                                          \
  template __global__ void attn_fwd_kernel<DD, CC, MM, NN>(const bf16_t* __restrict__, const bf16_t* __restrict__, \
                                                           const bf16_t* __restrict__, bf16_t* __restrict__,        \
                                                           float* __restrict__, int, int, int, int, long, long, long,  \
                                                           long, float);
RCA_FWD_INST(128, false, true, 4)
RCA_FWD_INST(64, false, true, 4)
RCA_FWD_INST(128, true, true, 4)
RCA_FWD_INST(64, true, true, 4)
RCA_FWD_INST(128, false, true, 8)
RCA_FWD_INST(64, false, true, 8)
RCA_FWD_INST(128, true, true, 8)
RCA_FWD_INST(64, true, true, 8)
#undef RCA_FWD_INST

// ---------------------------------------------------------------------------------------------
// dQ (query-major twin of the forward: recomputes P from LSE and dP = dO.V^T, accumulates
// dQ^T = K^T.dS^T in registers; also writes delta = rowsum(dO * O) for the dK/dV kernel).
// 32-key tiles, 2-deep LDS ring (loop unrolled over it); per
// tile: K-row burst -> S^T MFMAs, V-row burst -> dP^T MFMAs, dS on the VALU, K^T transposed
// burst -> dQ^T MFMAs.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    float* __restrict__ Delta, bf16_t* __restrict__ dQ, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long so, long sdo, long sdq, float scale2, float scale) {
  constexpr int BQ = 128, BK = 32, NKS = D / 16, NDB = D / 32, TILE = BK * D * 2, G8 = Img<D>::G8;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];

  const int nqb = S / BQ, G = Hq / Hk;
  // one (batch, kv head) per group: its G query heads x nqb query blocks share the K/V stream
  int bhk, item;
  xcd_group_map(blockIdx.x, B * Hk, G * nqb, bhk, item);
  const int qr = item / G, b = bhk / Hk, hk = bhk % Hk, hq = hk * G + item % G, bh = b * Hq + hq;
  const int qb = CAUSAL ? nqb - 1 - qr : qr;  // longest causal rows first
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int q0 = qb * BQ, qw0 = q0 + 32 * w, qrow = qw0 + l32;
  const int rb0 = Img<D>::row_base(l32, h, 0), rb1 = Img<D>::row_base(l32, h, 1);
  const int tb0 = Img<D>::tr_base(lane, 0), tb1 = Img<D>::tr_base(lane, 1);

  const bf16_t* Kb = K + (long)b * S * sk + (long)hk * D;
  const bf16_t* Vb = V + (long)b * S * sv + (long)hk * D;
  const bf16_t* Qr = Q + ((long)b * S + qrow) * sq + (long)hq * D;
  const bf16_t* dOr = dO + ((long)b * S + qrow) * sdo + (long)hq * D;

  bf16x8_t qf[NKS], gf[NKS];
#pragma unroll
  for (int kk = 0; kk < NKS; ++kk) {
    qf[kk] = gload8(Qr + 16 * kk + 8 * h);
    gf[kk] = gload8(dOr + 16 * kk + 8 * h);
  }
#pragma unroll
  for (int kk = 0; kk < NKS; ++kk) {
    settle(qf[kk]);
    settle(gf[kk]);
  }
  const float nlse = -LSE[(long)bh * S + qrow];
  // delta = rowsum(dO * O) for this lane's query row, fused here: the lane already holds its half
  // of the dO row (gf), so only the matching O half is loaded; the two halves meet across lanes
  // l / l^32. Written out for the dK/dV kernel, which runs after this one. -delta is the dP
  // chain's initial accumulator (a constant vector), so dS = P * dP' needs no per-tile subtraction.
  f32x16 ndlt;
  {
    const bf16_t* Orow = O + ((long)b * S + qrow) * so + (long)hq * D;
    float acc = 0.f;
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      const bf16x8_t of = gload8(Orow + 16 * kk + 8 * h);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf((float)of[j], (float)gf[kk][j], acc);
    }
    const float d = xhalf_sum(acc);
    if (h == 0) Delta[(long)bh * S + qrow] = d;
#pragma unroll
    for (int i = 0; i < 16; ++i) ndlt[i] = -d;
  }

  f32x16 dq[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dq[i] = zero16();

  const int ntile = CAUSAL ? (q0 + BQ) / BK : S / BK;  // always even
  Stage<D, BK> kst, vst;
  kst.init(Kb, sk, S, tid);
  vst.init(Vb, sv, S, tid);
  kst.load(0, sk);
  vst.load(0, sv);
  kst.store(smem);
  vst.store(smem + TILE);
  __syncthreads();

  auto tile = [&](auto bufc, int it) {
    constexpr int buf = decltype(bufc)::value;
    const char* Ks = smem + buf * 2 * TILE;
    const char* Vs = Ks + TILE;
    const int kb = it * BK;
    const bool more = it + 1 < ntile;
    if (more) {
      kst.load(kb + BK, sk);
      vst.load(kb + BK, sv);
    }
    // one straight-line body per variant (the diagonal tile's mask is compiled only into DIAG):
    // a runtime branch between the S/dP MFMAs and the VALU split the tile into basic blocks the
    // scheduler could not interleave
    auto run = [&](auto diagc) {
      constexpr bool DIAG = decltype(diagc)::value;
      bf16x8_t fr[2 * NKS];
#pragma unroll
      for (int kk = 0; kk < NKS; ++kk) {
        fr[kk] = lds_b128(Ks + ((kk & 1) ? rb1 : rb0) + 512 * (kk >> 1));
        fr[NKS + kk] = lds_b128(Vs + ((kk & 1) ? rb1 : rb0) + 512 * (kk >> 1));
      }
      f32x16 s = zero16(), dp = ndlt;
#pragma unroll
      for (int kk = 0; kk < NKS; ++kk) {
        s = mfma32(fr[kk], qf[kk], s);
        dp = mfma32(fr[NKS + kk], gf[kk], dp);
      }
      if constexpr (DIAG) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kofs = (r & 3) + 8 * (r >> 2) + 4 * h;
          s[r] = kofs > l32 ? -INFINITY : s[r];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = fast_exp2(fmaf(s[r], scale2, nlse)) * dp[r];
      const bf16x8_t d0 = acc_to_bf16(s, 0), d1 = acc_to_bf16(s, 1);
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int db = 0; db < NDB; ++db)
          fr[st * NDB + db] = lds_tr8(Ks + tb0 + G8 * (2 * st) + 512 * db, Ks + tb1 + G8 * (2 * st + 1) + 512 * db);
#pragma unroll
      for (int db = 0; db < NDB; ++db) dq[db] = mfma32(fr[db], d0, dq[db]);
#pragma unroll
      for (int db = 0; db < NDB; ++db) dq[db] = mfma32(fr[NDB + db], d1, dq[db]);
    };
    if (CAUSAL && kb == qw0) {
      run(std::integral_constant<bool, CAUSAL>{});
    } else if (!CAUSAL || kb < qw0) {
      run(std::false_type{});
    }
    if (more) {
      kst.store(smem + (buf ^ 1) * 2 * TILE);
      vst.store(smem + (buf ^ 1) * 2 * TILE + TILE);
    }
    __syncthreads();
  };
  for (int it = 0; it < ntile; it += 2) {
    tile(IC<0>{}, it);
    tile(IC<1>{}, it + 1);
  }

  bf16_t* dQr = dQ + ((long)b * S + qrow) * sdq + (long)hq * D;
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      store4(dQr + 32 * db + 8 * g + 4 * h, dq[db][4 * g] * scale, dq[db][4 * g + 1] * scale,
             dq[db][4 * g + 2] * scale, dq[db][4 * g + 3] * scale);
    }
  }
}

bool attn_dma() {
  static const bool on = [] {
    const char* e = getenv("RCA_ATTN_DMA");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// waves per forward workgroup: 8 (default: one 256-row workgroup per CU, K/V staged once for all
// 8 waves) or 4 (two 128-row workgroups per CU) (RCA_ATTN_FWD_NW; run-time switch
// rca_attn_set_fwd_nw). Interleaved A/B at the 8B shape, 3 rounds: 0.273 / 0.273 / 0.273 ms vs
// 0.279 / 0.278 / 0.279; bitwise-equal outputs (tests/test_attention_gpu.py).
int g_fwd_nw = [] {
  const char* e = getenv("RCA_ATTN_FWD_NW");
  return e && atoi(e) == 4 ? 4 : 8;
}();

template <int D, bool C>
void launch_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                int Hk, long sq, long sk, long sv, long so, float scale2, hipStream_t st) {
  if (D == 128 && rca_attn_launch_fwd_wide(C, q, k, v, o, lse, B, S, Hq, Hk, sq, sk, sv, so, scale2, st)) return;
  if (g_fwd_nw == 8 && S % 256 == 0 && attn_dma()) {
    hipLaunchKernelGGL((attn_fwd_kernel<D, C, true, 8>), dim3(B * Hq * (S / 256)), dim3(512), 0, st, q, k, v, o, lse, B,
                       S, Hq, Hk, sq, sk, sv, so, scale2);
    return;
  }
  const int grid = B * Hq * (S / 128);
  if (attn_dma())
    hipLaunchKernelGGL((attn_fwd_kernel<D, C, true>), dim3(grid), dim3(kThreads), 0, st, q, k, v, o, lse, B, S, Hq, Hk,
                       sq, sk, sv, so, scale2);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<D, C, false>), dim3(grid), dim3(kThreads), 0, st, q, k, v, o, lse, B, S, Hq,
                       Hk, sq, sk, sv, so, scale2);
}

template <int D, bool C>
void launch_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                const float* lse, float* delta, bf16_t* dq, bf16_t* dk, bf16_t* dv, int B, int S, int Hq, int Hk,
                long sq, long sk, long sv, long so, long sdo, long sdq, long sdk, long sdv, float scale2, float scale,
                hipStream_t st, bf16_t* ws) {
  if (ws != nullptr) {
    // recompute-free: delta, then dK/dV (+ the dS tiles), then dQ = dS . K
    const long nb = S / 32, tiles = C ? nb * (nb + 1) / 2 : nb * nb;
    rca_attn_launch_delta(o, dout, delta, B, S, Hq, so, sdo, st);
    rca_attn_launch_dkdv(D, C, q, k, v, dout, lse, delta, dk, dv, B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2,
                         scale, st, ws, tiles);
    rca_attn_launch_dq_ds(C, k, ws, dq, B, S, Hq, Hk, sk, sdq, scale, st);
    return;
  }
  // dQ first: it also produces delta = rowsum(dO * O), which dK/dV reads
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, C>), dim3(B * Hq * (S / 128)), dim3(kThreads), 0, st, q, k, v, o, dout, lse,
                     delta, dq, B, S, Hq, Hk, sq, sk, sv, so, sdo, sdq, scale2, scale);
  rca_attn_launch_dkdv(D, C, q, k, v, dout, lse, delta, dk, dv, B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale,
                       st, nullptr, 0);
}

bool shapes_ok(int B, int S, int Hq, int Hk, int D) {
  return B > 0 && S > 0 && S % 128 == 0 && Hk > 0 && Hq % Hk == 0 && (D == 64 || D == 128) &&
         (long)B * S * Hq < (1L << 31);
}

}  // namespace

RCA_API int rca_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Hq,
                         int Hk, int D, long long sq, long long sk, long long sv, long long so, float scale,
                         int causal, hipStream_t st) {
  if (!shapes_ok(B, S, Hq, Hk, D)) return 1;
  const float scale2 = scale * 1.4426950408889634f;
  auto Q = (const bf16_t*)q;
  auto K = (const bf16_t*)k;
  auto V = (const bf16_t*)v;
  auto O = (bf16_t*)o;
  if (D == 128) {
    if (causal) launch_fwd<128, true>(Q, K, V, O, lse, B, S, Hq, Hk, sq, sk, sv, so, scale2, st);
    else launch_fwd<128, false>(Q, K, V, O, lse, B, S, Hq, Hk, sq, sk, sv, so, scale2, st);
  } else {
    if (causal) launch_fwd<64, true>(Q, K, V, O, lse, B, S, Hq, Hk, sq, sk, sv, so, scale2, st);
    else launch_fwd<64, false>(Q, K, V, O, lse, B, S, Hq, Hk, sq, sk, sv, so, scale2, st);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Backward mode: 1 (default) = recompute-free dQ from the dS tiles the dK/dV kernel writes
// (needs the workspace of rca_attn_bwd_ws_bytes; D = 128), 0 = the dQ kernel that recomputes S, P
// and dP. RCA_ATTN_BWD=0 or rca_attn_set_bwd_mode(0) selects the latter (A/B, equivalence tests).
static int g_bwd_mode = [] {
  const char* e = getenv("RCA_ATTN_BWD");
  return e && atoi(e) == 0 ? 0 : 1;
}();
RCA_API int rca_attn_set_bwd_mode(int mode) {
  const int old = g_bwd_mode;
  g_bwd_mode = mode;
  return old;
}

RCA_API int rca_attn_set_fwd_nw(int nw) {
  const int old = g_fwd_nw;
  g_fwd_nw = nw == 8 ? 8 : 4;
  return old;
}

// workspace bytes rca_attn_bwd2 wants for this shape (0: none, the recompute path runs)
RCA_API long long rca_attn_bwd_ws_bytes(int B, int S, int Hq, int Hk, int D, int causal) {
  if (g_bwd_mode != 1 || !shapes_ok(B, S, Hq, Hk, D)) return 0;
  return rca_attn_ds_ws_bytes(B, S, Hq, D, causal != 0);
}

RCA_API int rca_attn_bwd2(const void* q, const void* k, const void* v, const void* o, const void* dout,
                          const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hk,
                          int D, long long sq, long long sk, long long sv, long long so, long long sdo, long long sdq,
                          long long sdk, long long sdv, float scale, int causal, void* ws, long long ws_bytes,
                          hipStream_t st) {
  if (!shapes_ok(B, S, Hq, Hk, D)) return 1;
  const long need = rca_attn_ds_ws_bytes(B, S, Hq, D, causal != 0);
  bf16_t* w = (ws != nullptr && need > 0 && ws_bytes >= need && D == 128) ? (bf16_t*)ws : nullptr;
  const float scale2 = scale * 1.4426950408889634f;
  auto Q = (const bf16_t*)q;
  auto K = (const bf16_t*)k;
  auto V = (const bf16_t*)v;
  auto O = (const bf16_t*)o;
  auto G = (const bf16_t*)dout;
  auto dQ = (bf16_t*)dq;
  auto dK = (bf16_t*)dk;
  auto dV = (bf16_t*)dv;
#define RCA_BWD(DD, CC)                                                                                            \
  launch_bwd<DD, CC>(Q, K, V, O, G, lse, delta, dQ, dK, dV, B, S, Hq, Hk, sq, sk, sv, so, sdo, sdq, sdk, sdv, scale2, \
                     scale, st, DD == 128 ? w : nullptr)
  if (D == 128) {
    if (causal) RCA_BWD(128, true);
    else RCA_BWD(128, false);
  } else {
    if (causal) RCA_BWD(64, true);
    else RCA_BWD(64, false);
  }
#undef RCA_BWD
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

RCA_API int rca_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int S, int Hq, int Hk,
                         int D, long long sq, long long sk, long long sv, long long so, long long sdo, long long sdq,
                         long long sdk, long long sdv, float scale, int causal, hipStream_t st) {
  if (!shapes_ok(B, S, Hq, Hk, D)) return 1;
  const float scale2 = scale * 1.4426950408889634f;
  auto Q = (const bf16_t*)q;
  auto K = (const bf16_t*)k;
  auto V = (const bf16_t*)v;
  auto O = (const bf16_t*)o;
  auto G = (const bf16_t*)dout;
  auto dQ = (bf16_t*)dq;
  auto dK = (bf16_t*)dk;
  auto dV = (bf16_t*)dv;
#define RCA_BWD(DD, CC)                                                                                            \
  launch_bwd<DD, CC>(Q, K, V, O, G, lse, delta, dQ, dK, dV, B, S, Hq, Hk, sq, sk, sv, so, sdo, sdq, sdk, sdv, scale2, \
                     scale, st, nullptr)
  if (D == 128) {
    if (causal) RCA_BWD(128, true);
    else RCA_BWD(128, false);
  } else {
    if (causal) RCA_BWD(64, true);
    else RCA_BWD(64, false);
  }
#undef RCA_BWD
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
