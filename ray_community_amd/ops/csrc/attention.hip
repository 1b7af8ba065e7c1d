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
#include "common.h"

#include <cstdlib>
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
    const int row = tid / NCH, ch = tid % NCH;
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

// single v_max3_f32 (plain fmaxf on MFMA results gets canonicalising v_max pairs from hipcc)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ float max16(const f32x16& s, float init) {
  float a = max3f(init, s[0], s[1]), b = max3f(s[2], s[3], s[4]);
  a = max3f(a, s[5], s[6]);
  b = max3f(b, s[7], s[8]);
  a = max3f(a, s[9], s[10]);
  b = max3f(b, s[11], s[12]);
  a = max3f(a, s[13], s[14]);
  return max3f(a, b, s[15]);
}

// ---------------------------------------------------------------------------------------------
// Forward. Per 64-key tile each wave runs four clusters: K operand burst (16 x ds_read_b128 into
// registers), S^T MFMAs (two independent 32-key chains), softmax on the VALU, V^T operand burst
// (32 x ds_read_b64_tr_b16), P.V MFMAs. Two workgroups per CU put two waves on every SIMD, so one
// wave's load/VALU clusters run beside the other's MFMA clusters. The loop is unrolled over the
// 2-deep LDS ring so every LDS address is base register + immediate. The online-softmax rescale is
// deferred (only when a row max grows by > 8 in log2 units: P <= 2^8, exact f32 accumulation)
// and wave-uniform.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void attn_fwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    bf16_t* __restrict__ O, float* __restrict__ LSE, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long so, float scale2) {
  constexpr int BQ = 128, BK = 64, NKS = D / 16, NDB = D / 32, TILE = BK * D * 2, G8 = Img<D>::G8;
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
            fr[st * NDB + db] = lds_tr8(Vs + tb0 + G8 * (2 * ts) + 512 * db, Vs + tb1 + G8 * (2 * ts + 1) + 512 * db);
          }
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
      kst.store(smem + (buf ^ 1) * 2 * TILE);
      vst.store(smem + (buf ^ 1) * 2 * TILE + TILE);
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

// ---------------------------------------------------------------------------------------------
// delta = rowsum(dO * O) (fp32), [B, Hq, S]
template <int D>
__global__ __launch_bounds__(kThreads) void attn_bwd_delta_kernel(const bf16_t* __restrict__ O,
                                                                  const bf16_t* __restrict__ dO,
                                                                  float* __restrict__ delta, int B, int S, int Hq,
                                                                  long so, long sdo) {
  constexpr int LPR = D / 8;  // lanes per (token, head) row
  const long gid = (long)blockIdx.x * kThreads + threadIdx.x;
  const long row = gid / LPR;  // = (b*S + s)*Hq + hq
  const int c = gid % LPR;
  const long total = (long)B * S * Hq;
  float acc = 0.f;
  if (row < total) {
    const long tok = row / Hq;
    const int hq = row % Hq;
    float a[8], g[8];
    unpack8(*reinterpret_cast<const u32x4*>(O + tok * so + (long)hq * D + c * 8), a);
    unpack8(*reinterpret_cast<const u32x4*>(dO + tok * sdo + (long)hq * D + c * 8), g);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * g[i];
  }
#pragma unroll
  for (int off = LPR / 2; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < total && c == 0) {
    const long tok = row / Hq;
    const int hq = row % Hq;
    const long b = tok / S, s = tok % S;
    delta[((b * Hq) + hq) * S + s] = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// dQ (query-major twin of the forward: recomputes P from LSE and dP = dO.V^T, accumulates
// dQ^T = K^T.dS^T in registers). 32-key tiles, 2-deep LDS ring (loop unrolled over it); per
// tile: K-row burst -> S^T MFMAs, V-row burst -> dP^T MFMAs, dS on the VALU, K^T transposed
// burst -> dQ^T MFMAs.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    bf16_t* __restrict__ dQ, int B, int S, int Hq, int Hk, long sq, long sk, long sv, long sdo, long sdq,
    float scale2, float scale) {
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
  const float dlt = Delta[(long)bh * S + qrow];

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
    if (!CAUSAL || kb <= qw0) {
      bf16x8_t fr[2 * NKS];
#pragma unroll
      for (int kk = 0; kk < NKS; ++kk) {
        fr[kk] = lds_b128(Ks + ((kk & 1) ? rb1 : rb0) + 512 * (kk >> 1));
        fr[NKS + kk] = lds_b128(Vs + ((kk & 1) ? rb1 : rb0) + 512 * (kk >> 1));
      }
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int kk = 0; kk < NKS; ++kk) {
        s = mfma32(fr[kk], qf[kk], s);
        dp = mfma32(fr[NKS + kk], gf[kk], dp);
      }
      if (CAUSAL && kb == qw0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kofs = (r & 3) + 8 * (r >> 2) + 4 * h;
          s[r] = kofs > l32 ? -INFINITY : s[r];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = fast_exp2(fmaf(s[r], scale2, nlse)) * (dp[r] - dlt);
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
  __shared__ __attribute__((aligned(16))) float rowc[2][2][BQS];  // [slot][-lse, delta][row]

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
    if (tid < 2 * BQS) rowc[buf][tid / BQS][tid & (BQS - 1)] = tid < BQS ? -rc : rc;
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
      // S and dP of half t (rows 32t..32t+31 of the slice): row-operand burst + two MFMA chains
      auto sdp = [&](int t, f32x16& s, f32x16& dp) {
        bf16x8_t fr[2 * NKS];
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          const int o = ((kk & 1) ? rb1 : rb0) + 4 * G8 * t + 512 * (kk >> 1);
          fr[kk] = lds_b128(Qs + o);
          fr[NKS + kk] = lds_b128(Gs + o);
        }
        s = zero16();
        dp = zero16();
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          s = mfma32(fr[kk], kf[kk], s);
          dp = mfma32(fr[NKS + kk], vf[kk], dp);
        }
      };
      // P = exp2(S*c - lse), dS = P * (dP - delta) on the VALU (causal mask on the diagonal)
      auto pds = [&](int t, f32x16& s, f32x16& dp) {
        const bool diag = CAUSAL && qa + 32 * t < kw0 + 31;
        const int kq = key - qa - 32 * t - 4 * h;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(&rowc[buf][0][32 * t + 8 * g4 + 4 * h]);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(&rowc[buf][1][32 * t + 8 * g4 + 4 * h]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g4 + j;
            float p = fast_exp2(fmaf(s[r], scale2, l4[j]));
            if (diag) p = kq > 8 * g4 + j ? 0.f : p;
            s[r] = p;
            dp[r] = p * (dp[r] - d4[j]);
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
      f32x16 s[NH], dp[NH];
#pragma unroll
      for (int t = 0; t < NH; ++t) sdp(t, s[t], dp[t]);
#pragma unroll
      for (int t = 0; t < NH; ++t) {
        pds(t, s[t], dp[t]);
        acc(t, s[t], dp[t]);
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

template <int D, bool C>
void launch_fwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, float* lse, int B, int S, int Hq,
                int Hk, long sq, long sk, long sv, long so, float scale2, hipStream_t st) {
  const int grid = B * Hq * (S / 128);
  hipLaunchKernelGGL((attn_fwd_kernel<D, C>), dim3(grid), dim3(kThreads), 0, st, q, k, v, o, lse, B, S, Hq, Hk, sq,
                     sk, sv, so, scale2);
}

template <int D, bool C>
void launch_bwd(const bf16_t* q, const bf16_t* k, const bf16_t* v, const bf16_t* o, const bf16_t* dout,
                const float* lse, float* delta, bf16_t* dq, bf16_t* dk, bf16_t* dv, int B, int S, int Hq, int Hk,
                long sq, long sk, long sv, long so, long sdo, long sdq, long sdk, long sdv, float scale2, float scale,
                hipStream_t st) {
  const long rows = (long)B * S * Hq;
  const long threads = rows * (D / 8);
  hipLaunchKernelGGL((attn_bwd_delta_kernel<D>), dim3((threads + kThreads - 1) / kThreads), dim3(kThreads), 0, st, o,
                     dout, delta, B, S, Hq, so, sdo);
  // RCA_ATTN_DKDV_NH=1 selects the unpipelined 32-row-slice variant (A/B measurements)
  static const int nh = [] {
    const char* e = getenv("RCA_ATTN_DKDV_NH");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  if (nh == 1)
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C, 1>), dim3(B * Hk * (S / 128)), dim3(kThreads), 0, st, q, k, v,
                       dout, lse, delta, dk, dv, B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale);
  else
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C, 2>), dim3(B * Hk * (S / 128)), dim3(kThreads), 0, st, q, k, v,
                       dout, lse, delta, dk, dv, B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, C>), dim3(B * Hq * (S / 128)), dim3(kThreads), 0, st, q, k, v, dout, lse,
                     delta, dq, B, S, Hq, Hk, sq, sk, sv, sdo, sdq, scale2, scale);
}

bool shapes_ok(int B, int S, int Hq, int Hk, int D) {
  return B > 0 && S > 0 && S % 128 == 0 && Hk > 0 && Hq % Hk == 0 && (D == 64 || D == 128);
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
                     scale, st)
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
