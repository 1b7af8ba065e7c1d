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

// LDS image of a [rows][D] bf16 tile: 16-byte chunk `ch` of row `row`, XOR-swizzled so that
// (a) 16 lanes reading the same chunk of 16 consecutive rows (ds_read_b128 operand rows) and
// (b) ds_read_b64_tr_b16 reading 4 rows x 32 columns per 32-lane half are both conflict-free.
template <int D>
__device__ __forceinline__ int soff(int row, int ch) {
  if constexpr (D == 128) {
    return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
  } else {
    return row * 128 + ((ch ^ (((row & 1) << 2) | ((row >> 1) & 3))) << 4);
  }
}

template <int D>
__device__ __forceinline__ bf16x8_t lds_row8(const char* base, int row, int ch) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4*>(base + soff<D>(row, ch)));
}

// Transposed 8-element operand: rows r0..r0+3 and r0+8..r0+11 of column `col` of the tile
// (the k order of an MFMA operand taken from an accumulator: j -> 8*(j>>2) + (j&3)).
// Each lane of a 16-lane group passes the address of row (r0 + (i>>2)), columns col0 + 4*(i&3).
template <int D>
__device__ __forceinline__ bf16x8_t lds_tr8(const char* base, int r0, int col0, int lane16) {
  const int q = lane16 >> 2, p = lane16 & 3;
  const int c = col0 + 4 * p;
  const int off0 = soff<D>(r0 + q, c >> 3) + ((c & 4) << 1);
  const int off1 = soff<D>(r0 + 8 + q, c >> 3) + ((c & 4) << 1);
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off0));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off1));
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
// K/V tile staging (64 rows x D) through registers
template <int D, int ROWS>
struct TileStage {
  static constexpr int NCH = D / 8;
  static constexpr int N = ROWS * NCH / kThreads;
  u32x4 r[N];
  __device__ __forceinline__ void load(const bf16_t* base, long stride, int row0, int tid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int id = tid + kThreads * i, row = id / NCH, ch = id % NCH;
      r[i] = *reinterpret_cast<const u32x4*>(base + (long)(row0 + row) * stride + ch * 8);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int id = tid + kThreads * i, row = id / NCH, ch = id % NCH;
      *reinterpret_cast<u32x4*>(lds + soff<D>(row, ch)) = r[i];
    }
  }
};

// ---------------------------------------------------------------------------------------------
// Forward
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void attn_fwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    bf16_t* __restrict__ O, float* __restrict__ LSE, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long so, float scale2) {
  constexpr int BQ = 128, BK = 64, NKS = D / 16, NDB = D / 32, TILE = BK * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE];

  const int nqb = S / BQ, BH = B * Hq;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = CAUSAL ? nqb - 1 - lid / BH : lid / BH;  // longest causal rows first
  const int bh = lid % BH, b = bh / Hq, hq = bh % Hq, hk = hq / (Hq / Hk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int q0 = qb * BQ, qw0 = q0 + 32 * w, qrow = qw0 + l32;

  const bf16_t* Kb = K + (long)b * S * sk + (long)hk * D;
  const bf16_t* Vb = V + (long)b * S * sv + (long)hk * D;
  const bf16_t* Qr = Q + ((long)b * S + qrow) * sq + (long)hq * D;

  bf16x8_t qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf[ks] = gload8(Qr + 16 * ks + 8 * h);

  f32x16 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = zero16();
  float m = -INFINITY, lsum = 0.f;

  const int nkv = CAUSAL ? (q0 + BQ) / BK : S / BK;
  TileStage<D, BK> ks_, vs_;
  ks_.load(Kb, sk, 0, tid);
  vs_.load(Vb, sv, 0, tid);
  ks_.store(smem[0][0], tid);
  vs_.store(smem[0][1], tid);
  __syncthreads();

  for (int it = 0; it < nkv; ++it) {
    const int kb = it * BK;
    if (it + 1 < nkv) {
      ks_.load(Kb, sk, kb + BK, tid);
      vs_.load(Vb, sv, kb + BK, tid);
    }
    const char* Ks = smem[it & 1][0];
    const char* Vs = smem[it & 1][1];
    if (!CAUSAL || kb <= qw0 + 31) {
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = zero16();
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) s[t] = mfma32(lds_row8<D>(Ks, 32 * t + l32, 2 * kk + h), qf[kk], s[t]);
      }
      const bool diag = CAUSAL && (kb + BK - 1 > qw0);
      float mt = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float x = s[t][r] * scale2;
          if (diag) {
            const int key = kb + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
            x = key > qrow ? -INFINITY : x;
          }
          s[t][r] = x;
          mt = fmaxf(mt, x);
        }
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float alpha = fast_exp2(m - mn);
      m = mn;
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(s[t][r] - mn);
          s[t][r] = p;
          ps += p;
        }
      }
      lsum = lsum * alpha + ps;
#pragma unroll
      for (int i = 0; i < NDB; ++i) o[i] *= alpha;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8_t pf = acc_to_bf16(s[t], st);
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const bf16x8_t vf = lds_tr8<D>(Vs, 32 * t + 16 * st + 4 * h, 32 * db + 16 * ((lane >> 4) & 1), lane & 15);
            o[db] = mfma32(vf, pf, o[db]);
          }
        }
      }
    }
    if (it + 1 < nkv) {
      ks_.store(smem[(it + 1) & 1][0], tid);
      vs_.store(smem[(it + 1) & 1][1], tid);
    }
    __syncthreads();
  }

  const float lt = lsum + __shfl_xor(lsum, 32, 64);
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
// dQ (query-major; recomputes P and dP)
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 2) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    bf16_t* __restrict__ dQ, int B, int S, int Hq, int Hk, long sq, long sk, long sv, long sdo, long sdq,
    float scale2, float scale) {
  constexpr int BQ = 128, BK = 64, NKS = D / 16, NDB = D / 32, TILE = BK * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE];

  const int nqb = S / BQ, BH = B * Hq;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = CAUSAL ? nqb - 1 - lid / BH : lid / BH;
  const int bh = lid % BH, b = bh / Hq, hq = bh % Hq, hk = hq / (Hq / Hk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int q0 = qb * BQ, qw0 = q0 + 32 * w, qrow = qw0 + l32;

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
  const float lse = LSE[(long)bh * S + qrow];
  const float dlt = Delta[(long)bh * S + qrow];

  f32x16 dq[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dq[i] = zero16();

  const int nkv = CAUSAL ? (q0 + BQ) / BK : S / BK;
  TileStage<D, BK> ks_, vs_;
  ks_.load(Kb, sk, 0, tid);
  vs_.load(Vb, sv, 0, tid);
  ks_.store(smem[0][0], tid);
  vs_.store(smem[0][1], tid);
  __syncthreads();

  for (int it = 0; it < nkv; ++it) {
    const int kb = it * BK;
    if (it + 1 < nkv) {
      ks_.load(Kb, sk, kb + BK, tid);
      vs_.load(Vb, sv, kb + BK, tid);
    }
    const char* Ks = smem[it & 1][0];
    const char* Vs = smem[it & 1][1];
    if (!CAUSAL || kb <= qw0 + 31) {
      const bool diag = CAUSAL && (kb + BK - 1 > qw0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x16 s = zero16(), dp = zero16();
#pragma unroll
        for (int kk = 0; kk < NKS; ++kk) {
          s = mfma32(lds_row8<D>(Ks, 32 * t + l32, 2 * kk + h), qf[kk], s);
          dp = mfma32(lds_row8<D>(Vs, 32 * t + l32, 2 * kk + h), gf[kk], dp);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fast_exp2(s[r] * scale2 - lse);
          if (diag) {
            const int key = kb + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
            p = key > qrow ? 0.f : p;
          }
          s[r] = p * (dp[r] - dlt);  // dS^T (natural units, before the softmax scale)
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8_t df = acc_to_bf16(s, st);
#pragma unroll
          for (int db = 0; db < NDB; ++db) {
            const bf16x8_t kf = lds_tr8<D>(Ks, 32 * t + 16 * st + 4 * h, 32 * db + 16 * ((lane >> 4) & 1), lane & 15);
            dq[db] = mfma32(kf, df, dq[db]);
          }
        }
      }
    }
    if (it + 1 < nkv) {
      ks_.store(smem[(it + 1) & 1][0], tid);
      vs_.store(smem[(it + 1) & 1][1], tid);
    }
    __syncthreads();
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
// dK, dV (key-major; sums the kv group's query heads in registers)
template <int D, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
    bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int B, int S, int Hq, int Hk, long sq, long sk, long sv,
    long sdo, long sdk, long sdv, float scale2, float scale) {
  constexpr int BKV = 128, BQS = 32, NKS = D / 16, NDB = D / 32, SL = BQS * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2][2][SL];
  __shared__ __attribute__((aligned(16))) float rowc[2][2][BQS];  // [buf][lse, delta][row]

  const int nkb = S / BKV, BHk = B * Hk, G = Hq / Hk;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int kbi = CAUSAL ? lid / BHk : nkb - 1 - lid / BHk;  // causal: key block 0 sees every query
  const int bhk = lid % BHk, b = bhk / Hk, hk = bhk % Hk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int k0 = kbi * BKV, kw0 = k0 + 32 * w, key = kw0 + l32;

  bf16x8_t kf[NKS], vf[NKS];
  {
    const bf16_t* Kr = K + ((long)b * S + key) * sk + (long)hk * D;
    const bf16_t* Vr = V + ((long)b * S + key) * sv + (long)hk * D;
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      kf[kk] = gload8(Kr + 16 * kk + 8 * h);
      vf[kk] = gload8(Vr + 16 * kk + 8 * h);
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
  const int total = G * nsl;

  TileStage<D, BQS> qs_, gs_;
  float rc = 0.f;
  auto stage_load = [&](int idx) {
    const int g = idx / nsl, sl = idx % nsl;
    const int hq = hk * G + g, qa = qs0 + sl * BQS;
    qs_.load(Q + (long)b * S * sq + (long)hq * D, sq, qa, tid);
    gs_.load(dO + (long)b * S * sdo + (long)hq * D, sdo, qa, tid);
    if (tid < 2 * BQS) {
      const float* src = tid < BQS ? LSE : Delta;
      rc = src[((long)b * Hq + hq) * S + qa + (tid & (BQS - 1))];
    }
  };
  auto stage_store = [&](int buf) {
    qs_.store(smem[buf][0], tid);
    gs_.store(smem[buf][1], tid);
    if (tid < 2 * BQS) rowc[buf][tid / BQS][tid & (BQS - 1)] = rc;
  };

  stage_load(0);
  stage_store(0);
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int sl = it % nsl;
    const int qa = qs0 + sl * BQS;
    if (it + 1 < total) stage_load(it + 1);
    const int buf = it & 1;
    const char* Qs = smem[buf][0];
    const char* Gs = smem[buf][1];
    if (!CAUSAL || qa + BQS - 1 >= kw0) {
      const bool diag = CAUSAL && (qa < kw0 + 31);
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int kk = 0; kk < NKS; ++kk) {
        s = mfma32(lds_row8<D>(Qs, l32, 2 * kk + h), kf[kk], s);
        dp = mfma32(lds_row8<D>(Gs, l32, 2 * kk + h), vf[kk], dp);
      }
      // rows of the accumulators are query rows (r&3) + 8(r>>2) + 4h
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(&rowc[buf][0][8 * g4 + 4 * h]);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&rowc[buf][1][8 * g4 + 4 * h]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g4 + i;
          float p = fast_exp2(s[r] * scale2 - l4[i]);
          if (diag) {
            const int q = qa + 8 * g4 + 4 * h + i;
            p = key > q ? 0.f : p;
          }
          s[r] = p;
          dp[r] = p * (dp[r] - d4[i]);
        }
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8_t pf = acc_to_bf16(s, st);
        const bf16x8_t df = acc_to_bf16(dp, st);
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const int col0 = 32 * db + 16 * ((lane >> 4) & 1);
          dv[db] = mfma32(lds_tr8<D>(Gs, 16 * st + 4 * h, col0, lane & 15), pf, dv[db]);
          dk[db] = mfma32(lds_tr8<D>(Qs, 16 * st + 4 * h, col0, lane & 15), df, dk[db]);
        }
      }
    }
    if (it + 1 < total) stage_store(buf ^ 1);
    __syncthreads();
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
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, C>), dim3(B * Hk * (S / 128)), dim3(kThreads), 0, st, q, k, v, dout,
                     lse, delta, dk, dv, B, S, Hq, Hk, sq, sk, sv, sdo, sdk, sdv, scale2, scale);
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
