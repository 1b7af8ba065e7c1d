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
// Hand-scheduled dK/dV (D = 128; the default, RCA_ATTN_DKDV=base for the kernel above). Same work split, LDS image and math as the
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
template <typename F, int... I>
__device__ __forceinline__ void sfor_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// compile-time unrolled loop: f(std::integral_constant<int, i>) for i = 0 .. N-1
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}
// LDS reads as base register + immediate offset (one base VGPR per lane pattern, no per-read
// address registers)
template <int OFF>
__device__ __forceinline__ bf16x8_t ldsq_o(unsigned base) {
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
  return __builtin_bit_cast(bf16x8_t, v);
}
template <int OFF>
__device__ __forceinline__ f32x4 ldsf4_o(unsigned base) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "n"(OFF));
  return v;
}
template <int OFF0, int OFF1>
__device__ __forceinline__ bf16x8_t ldstr_o(unsigned b0, unsigned b1) {
  static_assert(OFF0 < 65536 && OFF1 < 65536, "ds offset field is 16 bits");
  s16x4 a, b;
  asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%5"
               : "=&v"(a), "=&v"(b)
               : "v"(b0), "v"(b1), "n"(OFF0), "n"(OFF1));
  s16x8 r = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, r);
}

__device__ __forceinline__ void hs_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// >= 18 wait states between an XDL write and a VALU read of the result (and the reverse)
__device__ __forceinline__ void hs_xdl_gap() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory"); }
// volatile: kept in the written order relative to the reads and the hazard gaps (a plain asm is
// free to move across them before instruction selection)
#define HS_MFV(acc, a, b) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
// S / dP chains with the K / V fragments (B operand) held in accumulator registers: 64 VGPRs freed
// The leading s_nop: hipcc is free to materialise an asm operand with a copy right in front of the
// statement (v_accvgpr_write of a K/V fragment it keeps in VGPRs under register pressure, a
// v_accvgpr_mov of an accumulator), and its hazard recognizer does not pad copies that feed an asm
// MFMA: without these wait states an MFMA read a stale K fragment (11 wrong dS elements in one
// diagonal tile, scripts/diag/attn_ds_diag.py). The s_nop sits in the MFMA gap with the fillers.
// NOPS: the s_nop operand (3 = 4 wait states; 1 = 2, LLVM's VALU-write -> MFMA-read count)
#define HS_MFK(acc, a, b)                                                                                  \
  do {                                                                                                     \
    if constexpr (NOPS == 1)                                                                               \
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));      \
    else                                                                                                   \
      asm volatile("s_nop 3\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));      \
  } while (0)
#define HS_MFA(acc, a, b)                                                                                  \
  do {                                                                                                     \
    if constexpr (NOPS == 1)                                                                               \
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));      \
    else                                                                                                   \
      asm volatile("s_nop 3\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));      \
  } while (0)
// XDL <-> VALU hazard gap that the registers crossing it pass through: the producer stays above it
// and the consumer below it whatever the compiler reorders
#define HS_GAP "s_nop 7\n\ts_nop 7\n\ts_nop 4"

// DS: the kernel also writes every dS tile (bf16, the dK MFMA's own operand registers) to a workspace
// for the dQ kernel (attention_dq.hip: dQ = dS.K without recomputing S, P and dP). Tile (query block
// qb, key block kb) of 32 x 32 is 2 KB: fragment s (registers 8s..8s+7 of the dS accumulator) of
// lane l at 16-B slot 64 s + (l ^ (4 (l >> 5) + 8 s)), an XOR swizzle under which the dQ kernel's
// transposed reads are bank-conflict-free. Tiles of one (batch, query head) are stored
// qb (qb + 1) / 2 + kb (causal, kb <= qb) or qb nb + kb. The four 16-B stores per query slice are
// inline asm placed in MFMA gaps; the next slice's LDS-DMA is retired with a counted vmcnt(4), so
// the stores stay in flight across the slice barrier.
template <bool CAUSAL, bool DMA = true, bool DS = false, int NOPS = 3>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_hs_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long sdo, long sdk, long sdv, float scale2, float scale, bf16_t* __restrict__ dSw, long tiles_bh) {
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
  const unsigned sbase = (unsigned)(__UINTPTR_TYPE__)smem;
  const unsigned uq0 = sbase + rb0, uq1 = sbase + rb1, ut0 = sbase + tb0, ut1 = sbase + tb1;
  const unsigned ur = (unsigned)(__UINTPTR_TYPE__)&rowc[0][0][0] + 16 * h;
  // DS: per-lane slots of fragments 0 / 1 inside a tile; this wave's key block (wave-uniform)
  const unsigned dsv0 = 16u * (unsigned)(lane ^ (4 * h)), dsv1 = 1024u + 16u * (unsigned)(lane ^ (4 * h + 8));
  const int nb32 = S >> 5, kb32 = __builtin_amdgcn_readfirstlane(kw0 >> 5);
  char* const ds_trash = DS ? (char*)dSw + (long)B * Hq * tiles_bh * 2048 : nullptr;  // masked tiles land here

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
    for (int kk = 0; kk < NKS; ++kk) {  // resident in accumulator registers (the asm operands are "a")
      asm volatile("" : "+a"(kf[kk]));
      asm volatile("" : "+a"(vf[kk]));
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
  std::conditional_t<DMA, DmaStage<D, BQS>, Stage<D, BQS>> qst, gst;
  qst.init(Q + (long)b * S * sq + (long)hk * G * D, sq, S, tid, G * D);
  gst.init(dO + (long)b * S * sdo + (long)hk * G * D, sdo, S, tid, G * D);
  const float* rsrc = (tid < BQS ? LSE : Delta) + ((long)b * Hq + hk * G) * S + (tid & (BQS - 1));
  float rc = 0.f;
  auto stage_issue = [&](int g, int sl, int buf) {
    const int qa = qs0 + sl * BQS;
    if constexpr (DMA) {
      qst.issue(qa, sq, smem + buf * 2 * SL, g * D * 2);
      gst.issue(qa, sdo, smem + buf * 2 * SL + SL, g * D * 2);
    } else {
      qst.load(qa, sq, g * D * 2);
      gst.load(qa, sdo, g * D * 2);
    }
    if constexpr (DS) {  // invisible to hipcc's wait counting (retired by stage_finish's counted wait)
      if (tid < 2 * BQS) {
        const float* pr = rsrc + (long)g * S + qa;
        asm volatile("global_load_dword %0, %1, off" : "=v"(rc) : "v"(pr) : "memory");
      }
    } else {
      if (tid < 2 * BQS) rc = rsrc[(long)g * S + qa];
    }
  };
  // stored: this wave issued its 4 dS stores after the DMA (they may stay in flight)
  auto stage_finish = [&](int buf, bool stored) {
    if constexpr (DS) {
      if (stored) asm volatile("s_waitcnt vmcnt(4)" : "+v"(rc)::"memory");
      else asm volatile("s_waitcnt vmcnt(0)" : "+v"(rc)::"memory");
      if (tid < 2 * BQS) {
        const unsigned ra = (unsigned)(__UINTPTR_TYPE__)&rowc[buf][tid / BQS][tid & (BQS - 1)];
        asm volatile("ds_write_b32 %0, %1" ::"v"(ra), "v"(-rc) : "memory");  // -lse, -delta
      }
      return;
    }
    if constexpr (DMA) {
      wait_dma();
    } else {
      qst.store(smem + buf * 2 * SL);
      gst.store(smem + buf * 2 * SL + SL);
    }
    if (tid < 2 * BQS) rowc[buf][tid / BQS][tid & (BQS - 1)] = -rc;  // -lse, -delta
  };
  // slice barrier: a bare s_barrier in the DS variant (__syncthreads' fence would drain the stores)
  auto slice_barrier = [&]() {
    if constexpr (DS) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      __syncthreads();
    }
  };
  stage_issue(0, nsl - 1, 0);
  stage_finish(0, false);
  slice_barrier();

  auto slice = [&](auto bufc, int i) {
    constexpr int buf = decltype(bufc)::value;
    const char* Qs = smem + buf * 2 * SL;
    const char* Gs = Qs + SL;
    const int sl = nsl - 1 - i / G;
    const bool more = i + 1 < total;
    if (more) stage_issue((i + 1) % G, nsl - 1 - (i + 1) / G, buf ^ 1);
    const int qa = qs0 + sl * BQS;
    const bool run = !CAUSAL || qa + BQS - 1 >= kw0;
    if (run) {
      // DS: tile base of half t (wave-uniform); a causally masked tile goes to the trash tile
      auto ds_tile = [&](int t) -> char* {
        const int qb = (qa >> 5) + t;
        const long idx = CAUSAL ? (long)qb * (qb + 1) / 2 + kb32 : (long)qb * nb32 + kb32;
        char* p = (char*)dSw + ((long)(b * Hq + hk * G + i % G) * tiles_bh + idx) * 2048;
        return (!CAUSAL || qb >= kb32) ? p : ds_trash;
      };
      auto body = [&](auto diagc) {
        constexpr bool DIAG = decltype(diagc)::value;
        constexpr int BO = buf * 2 * SL;  // this slice's buffer; Q image at BO, dO image at BO + SL
        // row operand (kk, half t) of Q (G = 0) or dO (G = 1): base (kk odd ? uq1 : uq0) + immediate
        auto rowread = [&](auto kkc, auto tc, auto gc) {
          constexpr int kk = decltype(kkc)::value, t = decltype(tc)::value, g = decltype(gc)::value;
          constexpr int off = BO + g * SL + 4 * G8 * t + 512 * (kk >> 1);
          return ldsq_o<off>((kk & 1) ? uq1 : uq0);
        };
        // transposed operand f of half t: f = (2 st + isq) NDB + db; isq 0: dO^T, 1: Q^T
        auto trread = [&](auto fc, auto tc) {
          constexpr int f = decltype(fc)::value, t = decltype(tc)::value;
          constexpr int st = (f / NDB) >> 1, db = f % NDB, isq = (f / NDB) & 1;
          constexpr int base = BO + (isq ? 0 : SL) + 512 * db;
          return ldstr_o<base + G8 * (4 * t + 2 * st), base + G8 * (4 * t + 2 * st + 1)>(ut0, ut1);
        };
        auto rowc4 = [&](auto cc, auto tc, auto g4c) {  // -lse (c 0) / -delta (c 1) of rows 32t + 8g4 + 4h ..
          constexpr int c = decltype(cc)::value, t = decltype(tc)::value, g4 = decltype(g4c)::value;
          return ldsf4_o<((buf * 2 + c) * BQS + 32 * t + 8 * g4) * 4>(ur);
        };
        // MFMA q (0..15) of a dV/dK phase reads transposed operand fq_of(q)
        auto fq_of = [](int q) { return (2 * (q >> 3) + (q & 1)) * NDB + ((q >> 1) & 3); };
        const int kq0 = key - qa - 4 * h;
        f32x4 nl[2][4], nd[4];
        // P/dS of half t, element r (one per MFMA slot): p = exp2(S c - lse), dS' = p (dP - delta)
        auto pds1 = [&](f32x16& sx, f32x16& dx, int t, int r) {
          const int g4 = r >> 2, j = r & 3;
          float p = fast_exp2(fmaf(sx[r], scale2, nl[t][g4][j]));
          if constexpr (DIAG) p = (kq0 - 32 * t > 8 * g4 + j) ? 0.f : p;
          sx[r] = p;
          dx[r] = p * dx[r];
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        // ---- P0: R_0 and half 0's row constants (half 1's are read at the end of P1, and its
        // chains initialised at the start of P2: fewer registers live across P1)
        bf16x8_t fq[NKS], fg[NKS];
        sfor<NKS>([&](auto kkc) {
          constexpr int kk = decltype(kkc)::value;
          fq[kk] = rowread(kkc, I0{}, I0{});
          fg[kk] = rowread(kkc, I0{}, I1{});
        });
        sfor<4>([&](auto g4c) {
          constexpr int g4 = decltype(g4c)::value;
          nl[0][g4] = rowc4(I0{}, I0{}, g4c);
          nd[g4] = rowc4(I1{}, I0{}, g4c);
        });
        hs_lgkm0();
        hs_fence();
        f32x16 s0 = zero16(), s1, dp0, dp1;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
          for (int j = 0; j < 4; ++j) dp0[4 * g4 + j] = nd[g4][j];
        hs_fence();
        asm volatile(HS_GAP : "+v"(s0), "+v"(dp0));  // chain inits (VALU) before the first MFMAs read them
        hs_fence();
        // ---- P1: S_0 / dP_0 chains + R_1 reads into the freed fragment registers
        bf16x8_t fq1[NKS], fg1[NKS];
        sfor<NKS>([&](auto kkc) {
          constexpr int kk = decltype(kkc)::value;
          hs_fence();
          HS_MFK(s0, fq[kk], kf[kk]);
          hs_fence();
          fq1[kk] = rowread(kkc, I1{}, I0{});
          hs_fence();
          HS_MFK(dp0, fg[kk], vf[kk]);
          hs_fence();
          fg1[kk] = rowread(kkc, I1{}, I1{});
        });
        hs_fence();
        sfor<4>([&](auto g4c) {
          constexpr int g4 = decltype(g4c)::value;
          nl[1][g4] = rowc4(I0{}, I1{}, g4c);
          nd[g4] = rowc4(I1{}, I1{}, g4c);
        });
        hs_lgkm0();
        hs_fence();
        s1 = zero16();
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
          for (int j = 0; j < 4; ++j) dp1[4 * g4 + j] = nd[g4][j];
        hs_fence();
        // S_0 / dP_0 results before the VALU reads them; S_1 / dP_1 inits before the MFMAs
        asm volatile(HS_GAP : "+v"(s0), "+v"(dp0), "+v"(s1), "+v"(dp1));
        hs_fence();
        // ---- P2: S_1 / dP_1 chains + P/dS of half 0; the first TW T_0 operands at the end
        constexpr int TW = 4;
        bf16x8_t pa0, pb0, da0, db0;
        sfor<NKS>([&](auto kkc) {
          constexpr int kk = decltype(kkc)::value;
          hs_fence();
          HS_MFK(s1, fq1[kk], kf[kk]);
          hs_fence();
          pds1(s0, dp0, 0, 2 * kk);
          hs_fence();
          HS_MFK(dp1, fg1[kk], vf[kk]);
          hs_fence();
          pds1(s0, dp0, 0, 2 * kk + 1);
          if constexpr (kk == 3) {
            pa0 = acc_to_bf16(s0, 0);
            da0 = acc_to_bf16(dp0, 0);
          }
        });
        hs_fence();
        pb0 = acc_to_bf16(s0, 1);
        db0 = acc_to_bf16(dp0, 1);
        bf16x8_t tw[16];
        sfor<TW>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          tw[q] = trread(std::integral_constant<int, (2 * (q >> 3) + (q & 1)) * NDB + ((q >> 1) & 3)>{}, I0{});
        });
        asm volatile(HS_GAP : "+v"(s1), "+v"(dp1), "+v"(pa0), "+v"(pb0), "+v"(da0), "+v"(db0));
        hs_fence();
        // ---- P3: dV, dK += half 0 (T_0 read TW ahead) + P/dS of half 1
        bf16x8_t pa1, pb1, da1, db1;
        auto dvdk_slot = [&](auto qc, auto tc, const bf16x8_t& pa, const bf16x8_t& pb, const bf16x8_t& da,
                             const bf16x8_t& dbb) {
          constexpr int q = decltype(qc)::value;
          constexpr int later = (q + TW < 16 ? TW - 1 : 15 - q);
          hs_fence();
          asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * later) : "memory");  // operand q landed
          hs_fence();
          constexpr int st = q >> 3, db = (q >> 1) & 3;
          if constexpr (q & 1) {
            HS_MFA(dk[db], tw[q], st ? dbb : da);
          } else {
            HS_MFA(dv[db], tw[q], st ? pb : pa);
          }
          hs_fence();
          if constexpr (q + TW < 16)
            tw[q + TW] = trread(
                std::integral_constant<int, (2 * ((q + TW) >> 3) + ((q + TW) & 1)) * NDB + (((q + TW) >> 1) & 3)>{},
                tc);
        };
        char* const dst0 = DS ? ds_tile(0) : nullptr;
        sfor<16>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          (void)dsv0, (void)dsv1, (void)dst0;  // odr-use outside the if constexpr (clang capture of nested generic lambdas)
          dvdk_slot(qc, I0{}, pa0, pb0, da0, db0);
          pds1(s1, dp1, 1, q);
          if constexpr (q == 7) {
            pa1 = acc_to_bf16(s1, 0);
            da1 = acc_to_bf16(dp1, 0);
          }
          if constexpr (DS && q == 2) {
            hs_fence();
            asm volatile("global_store_dwordx4 %0, %1, %2" ::"v"(dsv0), "v"(da0), "s"(dst0) : "memory");
          }
          if constexpr (DS && q == 6) {
            hs_fence();
            asm volatile("global_store_dwordx4 %0, %1, %2" ::"v"(dsv1), "v"(db0), "s"(dst0) : "memory");
          }
        });
        hs_fence();
        pb1 = acc_to_bf16(s1, 1);
        db1 = acc_to_bf16(dp1, 1);
        sfor<TW>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          tw[q] = trread(std::integral_constant<int, (2 * (q >> 3) + (q & 1)) * NDB + ((q >> 1) & 3)>{}, I1{});
        });
        asm volatile(HS_GAP : "+v"(pa1), "+v"(pb1), "+v"(da1), "+v"(db1));
        hs_fence();
        // ---- P4: dV, dK += half 1 (T_1 read TW ahead)
        char* const dst1 = DS ? ds_tile(1) : nullptr;
        sfor<16>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          (void)dsv0, (void)dsv1, (void)dst1;
          dvdk_slot(qc, I1{}, pa1, pb1, da1, db1);
          if constexpr (DS && q == 2) {
            hs_fence();
            asm volatile("global_store_dwordx4 %0, %1, %2" ::"v"(dsv0), "v"(da1), "s"(dst1) : "memory");
          }
          if constexpr (DS && q == 6) {
            hs_fence();
            asm volatile("global_store_dwordx4 %0, %1, %2" ::"v"(dsv1), "v"(db1), "s"(dst1) : "memory");
          }
        });
        hs_fence();
        (void)fq_of;
      };
      if (CAUSAL && qa < kw0 + 31) body(std::integral_constant<bool, CAUSAL>{});
      else body(std::false_type{});
    }
    if (more) stage_finish(buf ^ 1, run);
    slice_barrier();
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
#undef HS_MFK
#undef HS_GAP
#undef HS_MFA

#define RCA_HS_INST(CC, MM, DD, NN)                                                                               \
  template __global__ void attn_bwd_dkdv_hs_kernel<CC, MM, DD, NN>(                                             \
      const bf16_t* __restrict__, const bf16_t* __restrict__, const bf16_t* __restrict__, const bf16_t* __restrict__, \
      const float* __restrict__, const float* __restrict__, bf16_t* __restrict__, bf16_t* __restrict__, int, int, int, \
      int, long, long, long, long, long, long, float, float, bf16_t* __restrict__, long);
RCA_HS_INST(true, true, false, 3)
RCA_HS_INST(false, true, false, 3)
RCA_HS_INST(true, false, false, 3)
RCA_HS_INST(false, false, false, 3)
RCA_HS_INST(true, true, true, 3)
RCA_HS_INST(false, true, true, 3)
RCA_HS_INST(true, true, true, 1)
RCA_HS_INST(false, true, true, 1)
#undef RCA_HS_INST

}  // namespace

// The hand-scheduled dK/dV kernel is the default for D = 128 (RCA_ATTN_DKDV=base selects the
// compiler-scheduled one); rca_attn_set_dkdv_hs switches at run time (same-process A/B and the
// equivalence test), returning the previous setting.
static bool g_dkdv_hs = [] {
  const char* e = getenv("RCA_ATTN_DKDV");
  return !(e && std::string(e) == "base");
}();
static bool g_dkdv_hs_stage = false;
// wait states ahead of each asm MFMA of the dS-storing kernel: the s_nop operand, 1 (2 wait
// states; the default) or 3. 2 is the documented requirement for the hazard these nops cover -- a
// VALU write (or v_accvgpr_write) of a register that the next MFMA reads as its A/B operand:
// cdna_hip_programming.md §3 'A/B operands may be AGPRs' and §5.7 item 2 ("a just-written "v"
// operand or v_accvgpr_write -> MFMA operand (s_nop 1)", from cdna_asm_programming.md Table 38),
// which is also the count LLVM's hazard recognizer inserts for this pair outside asm. Same-process
// A/B: bwd 1.025-1.050 vs 1.058-1.081 ms, 8B step 345.7 vs 349.0 ms median; gradients bitwise
// equal between the two counts on causal and full masks, MHA and GQA group sizes 1-8
// (tests/test_attention_gpu.py::test_ds_kernel_wait_state_variants_agree_bitwise).
static int g_hs_nops = [] {
  const char* e = getenv("RCA_ATTN_HS_NOPS");
  return e && atoi(e) == 3 ? 3 : 1;
}();
RCA_API int rca_attn_set_hs_nops(int n) {
  const int old = g_hs_nops;
  g_hs_nops = n;
  return old;
}
// 0: compiler-scheduled kernel; 1: hand-scheduled (LDS-DMA staging); 2: hand-scheduled with
// register staging
RCA_API int rca_attn_set_dkdv_hs(int on) {
  const int old = g_dkdv_hs ? (g_dkdv_hs_stage ? 2 : 1) : 0;
  g_dkdv_hs = on != 0;
  g_dkdv_hs_stage = on == 2;
  return old;
}

// dSw != nullptr: the hand-scheduled kernel also writes the dS tiles (D = 128 only; the caller checks)
void rca_attn_launch_dkdv(int D, bool causal, const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* dout,
                          const float* lse, const float* delta, bf16_t* dk, bf16_t* dv, int B, int S, int Hq, int Hk,
                          long sq, long sk, long sv, long sdo, long sdk, long sdv, float scale2, float scale,
                          hipStream_t st, bf16_t* dSw, long tiles_bh) {
  // RCA_ATTN_DKDV_NH=1 selects the unpipelined 32-row-slice variant (A/B measurements);
  // the hand-scheduled kernel for D = 128 unless RCA_ATTN_DKDV=base (g_dkdv_hs)
  static const int nh = [] {
    const char* e = getenv("RCA_ATTN_DKDV_NH");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  const bool hs = g_dkdv_hs;
  const dim3 grid(B * Hk * (S / 128)), block(kThreads);
  if (dSw != nullptr) {
#define RCA_DS(CC, NN)                                                                                           \
  hipLaunchKernelGGL((attn_bwd_dkdv_hs_kernel<CC, true, true, NN>), grid, block, 0, st, q, k, v, dout, lse, delta, dk, \
                     dv, B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale, dSw, tiles_bh)
    if (g_hs_nops == 1) {
      if (causal) RCA_DS(true, 1); else RCA_DS(false, 1);
    } else {
      if (causal) RCA_DS(true, 3); else RCA_DS(false, 3);
    }
#undef RCA_DS
    return;
  }
  if (hs && D == 128) {
#define RCA_HS(CC, MM)                                                                                         \
  hipLaunchKernelGGL((attn_bwd_dkdv_hs_kernel<CC, MM, false, 3>), grid, block, 0, st, q, k, v, dout, lse, delta, dk, dv, \
                     B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale, (bf16_t*)nullptr, 0L)
    if (g_dkdv_hs_stage) {  // register staging (bisect / A/B)
      if (causal) RCA_HS(true, false); else RCA_HS(false, false);
    } else {
      if (causal) RCA_HS(true, true); else RCA_HS(false, true);
    }
#undef RCA_HS
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
