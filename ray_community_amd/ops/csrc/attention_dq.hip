// Attention backward without recomputation for dQ (D = 128): the hand-scheduled dK/dV kernel
// (attention_dkdv.hip, DS variant) already builds dS = P * (dP - delta) in registers as the bf16
// operand of its dK^T MFMAs; it stores each 32 x 32 tile once (2 KB, fragment order, XOR-swizzled
// slots), and this file's dQ kernel reads them back: dQ = dS . K is a plain GEMM over the key
// dimension, memory-bound on the dS bytes. Against the query-major dQ kernel of attention.hip
// (which recomputes S = Q K^T, P and dP = dO V^T: three MFMA products per tile), the backward does
// four products plus one dS read instead of seven products (cdna_hip_programming.md Appendix B
// 'Attention backward': 5 products per tile is the recompute-free count; the fifth is here).
// Deterministic: every dQ element is summed in one wave's registers, in key order; no atomics.
//
// Also here: delta = rowsum(dO * O), which the dK/dV kernel reads (attention.hip fused it into
// the dQ kernel, which now runs after dK/dV).
#include "attention_common.h"

#include <cstdlib>

namespace {

// delta[b, h, s] = sum_d dO[b, s, h, d] * O[b, s, h, d]: one 16-lane group per 4 consecutive
// (b, s, h) rows (all four rows' loads in flight before any math), 16 B per lane (D = 128). Rows
// run in the tensors' own (token, head) order, so a wave reads 4 KB of consecutive heads of
// consecutive tokens. (In the 8B step the kernel measures ~67 us per layer in either row order,
// against 24 us in isolation: it runs while the side-stream gradient-norm pass streams the
// finished gradient buckets, and both share HBM; profiles/llama8b_r5_perstep_final.md.)
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                         float* __restrict__ Delta, int B, int S, int Hq, long so,
                                                         long sdo) {
  constexpr int R = 4;
  const long row0 = ((long)blockIdx.x * 16 + (threadIdx.x >> 4)) * R;  // (b * S + s) * Hq + h
  const long rows = (long)B * Hq * S;
  if (row0 >= rows) return;
  const int c = threadIdx.x & 15;
  u32x4 ov[R], gv[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const long row = row0 + i < rows ? row0 + i : row0;
    const long tok = row / Hq, h = row % Hq;
    ov[i] = *reinterpret_cast<const u32x4*>(O + tok * so + h * 128 + 8 * c);
    gv[i] = *reinterpret_cast<const u32x4*>(dO + tok * sdo + h * 128 + 8 * c);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    float of[8], gf[8];
    unpack8(ov[i], of);
    unpack8(gv[i], gf);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(of[j], gf[j], acc);
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (c == 0 && row0 + i < rows) {
      const long row = row0 + i, tok = row / Hq, h = row % Hq, b = tok / S, s = tok % S;
      Delta[(b * Hq + h) * S + s] = acc;
    }
  }
}

// dQ from the dS tiles: one workgroup = 4 waves = 128 query rows of one (batch, query head); wave w
// owns query block qb32 = 4 qb + w (32 rows) and accumulates dQ^T = K^T . dS^T (d on the MFMA row,
// query on the lane) over 32-key steps. Each step stages the step's K tile (32 x 128, shared by the
// 4 waves) and each wave's own dS tile (2 KB, fragment order: the LDS-DMA lands it byte for byte)
// into a 4-deep ring kept THREE steps ahead (counted vmcnt, bare s_barrier): the kernel is bound by
// the dS bytes, and the ring keeps ~3 x 8 KB of them in flight per workgroup. K^T fragments are
// ds_read_b64_tr_b16 reads of the K image (as V^T in the forward), dS^T fragments
// ds_read_b64_tr_b16 reads of the fragment-order tiles (conflict-free under the store-side XOR
// swizzle). Causally masked tiles still issue their DMA (of the diagonal tile, never read), so
// every wave's vmcnt counts are the same. Causal: the longest query blocks first.
template <bool CAUSAL, int QW = 1>
__global__ __launch_bounds__(kThreads, 2) void attn_dq_ds_kernel(const bf16_t* __restrict__ K,
                                                                 const bf16_t* __restrict__ dSw,
                                                                 bf16_t* __restrict__ dQ, int B, int S, int Hq,
                                                                 int Hk, long sk, long sdq, long tiles_bh,
                                                                 float scale) {
  // QW query blocks (32 rows each) per wave: the step's K tile is staged once for 4 QW blocks,
  // so QW = 2 halves the K bytes per dS byte through the LDS-DMA path
  constexpr int D = 128, BQ = 128 * QW, BK = 32, NDB = 4, KT = BK * D * 2, DST = 4 * QW * 2048, SLOT = KT + DST,
                NBUF = QW == 1 ? 4 : 3, AHEAD = NBUF - 1,
                OPS = 2 + 2 * QW /* DMA ops per wave per step: 2 K pieces + 2 per dS tile */, G8 = Img<D>::G8;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * SLOT];

  const int nqb = S / BQ, G = Hq / Hk, nb32 = S >> 5;
  int bhk, item;
  xcd_group_map(blockIdx.x, B * Hk, G * nqb, bhk, item);  // the G x nqb blocks of a kv head share K
  const int qr = item / G, b = bhk / Hk, hk = bhk % Hk, hq = hk * G + item % G;
  const int qb = CAUSAL ? nqb - 1 - qr : qr;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qb0 = 4 * QW * qb + QW * w;  // this wave's first 32-row query block (QW consecutive)
  const int nstep = CAUSAL ? 4 * QW * (qb + 1) : nb32;

  DmaStage<D, BK> kst;
  kst.init(K + (long)b * S * sk + (long)hk * D, sk, S, tid);
  const char* dsb = (const char*)dSw + (long)(b * Hq + hq) * tiles_bh * 2048;
  const __amdgpu_buffer_rsrc_t dsr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(dsb), (short)0, (int)(tiles_bh * 2048), 0x00020000);

  auto issue = [&](int st) {
    char* base = smem + (st % NBUF) * SLOT;
    kst.issue(st * BK, sk, base);
#pragma unroll
    for (int j = 0; j < QW; ++j) {
      const int q32 = qb0 + j;
      const long trow = CAUSAL ? (long)q32 * (q32 + 1) / 2 : (long)q32 * nb32;  // tile row of block q32
      const int kb = (!CAUSAL || st <= q32) ? st : q32;  // a masked tile: any valid tile (never read)
      const int so = __builtin_amdgcn_readfirstlane((int)((trow + kb) * 2048));
      char* dl = base + KT + (QW * w + j) * 2048;
#pragma unroll
      for (int pc = 0; pc < 2; ++pc)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dsr, (__attribute__((address_space(3))) void*)(dl + pc * 1024), 16,
                                                 lane * 16 + pc * 1024, so, 0, 0);
    }
  };

  // per-lane read bases: K^T (the forward's V^T reads) and dS^T (two bases: read r of a k-step)
  const int tb0 = Img<D>::tr_base(lane, 0), tb1 = Img<D>::tr_base(lane, 1);
  int dsa[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int sp = (lane >> 4) & 1;
    const int L = 8 * r + 4 * h + ((lane & 15) >> 2) + 32 * (lane & 1);
    dsa[r] = sp * 1024 + 16 * (L ^ (4 * (lane & 1) + 8 * sp)) + 8 * ((lane >> 1) & 1);
  }

  f32x16 dq[QW][NDB];
#pragma unroll
  for (int j = 0; j < QW; ++j)
#pragma unroll
    for (int i = 0; i < NDB; ++i) dq[j][i] = zero16();

  for (int st = 0; st < AHEAD && st < nstep; ++st) issue(st);
  for (int st = 0; st < nstep; ++st) {
    // stage st landed: at most (stages issued after it) x OPS of this wave's DMAs still pending
    const int later = nstep - 1 - st < AHEAD - 1 ? nstep - 1 - st : AHEAD - 1;
    if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPS) : "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of stage st are in; stage st-1 is read
    if (st + AHEAD < nstep) issue(st + AHEAD);  // into the buffer stage st-1 used
    if (!CAUSAL || st <= qb0 + QW - 1) {
      const char* Ks = smem + (st % NBUF) * SLOT;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t fr[NDB + QW];
#pragma unroll
        for (int db = 0; db < NDB; ++db)
          fr[db] = lds_tr8_asm(Ks + tb0 + G8 * (2 * ks) + 512 * db, Ks + tb1 + G8 * (2 * ks + 1) + 512 * db);
#pragma unroll
        for (int j = 0; j < QW; ++j) {
          const char* Ds = Ks + KT + (QW * w + j) * 2048;
          fr[NDB + j] = lds_tr8_asm(Ds + dsa[0] + 256 * ks, Ds + dsa[1] + 256 * ks);
        }
        lds_tr_settle(fr);
#pragma unroll
        for (int j = 0; j < QW; ++j) {
          if (CAUSAL && st > qb0 + j) continue;  // block j's row is complete (wave-uniform)
#pragma unroll
          for (int db = 0; db < NDB; ++db) dq[j][db] = mfma32(fr[db], fr[NDB + j], dq[j][db]);
        }
      }
    }
  }

  // dQ^T accumulators: d = 32 db + (r & 3) + 8 (r >> 2) + 4 h on the registers, the query on the lane
#pragma unroll
  for (int j = 0; j < QW; ++j) {
    const int qrow = (qb0 + j) * 32 + (lane & 31);
    bf16_t* dQr = dQ + ((long)b * S + qrow) * sdq + (long)hq * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(dQr + 32 * db + 8 * g + 4 * h, dq[j][db][4 * g] * scale, dq[j][db][4 * g + 1] * scale,
               dq[j][db][4 * g + 2] * scale, dq[j][db][4 * g + 3] * scale);
    }
  }
}

// explicit instantiations: hipcc does not always emit the host launch stub of a kernel template
// instantiated only through its launcher (an undefined __device_stub__ symbol at load time)
#define RCA_DQ_INST(CC, QQ)                                                                                       \
  template __global__ void attn_dq_ds_kernel<CC, QQ>(const bf16_t* __restrict__, const bf16_t* __restrict__,      \
                                                     bf16_t* __restrict__, int, int, int, int, long, long, long, \
                                                     float);
RCA_DQ_INST(true, 1)
RCA_DQ_INST(false, 1)
RCA_DQ_INST(true, 2)
RCA_DQ_INST(false, 2)
#undef RCA_DQ_INST

}  // namespace

// bytes of the dS workspace for this shape (0: the recompute path, attention.hip); the last 2 KB
// tile is the dK/dV kernel's trash tile for causally masked halves
long rca_attn_ds_ws_bytes(int B, int S, int Hq, int D, bool causal) {
  if (D != 128 || S % 128) return 0;
  const long nb = S / 32, tiles = causal ? nb * (nb + 1) / 2 : nb * nb;
  if (tiles * 2048 >= (1L << 31)) return 0;  // the dQ kernel's per-(batch, head) buffer range is 32-bit
  return ((long)B * Hq * tiles + 1) * 2048;
}

void rca_attn_launch_delta(const bf16_t* o, const bf16_t* dout, float* delta, int B, int S, int Hq, long so, long sdo,
                           hipStream_t st) {
  const long rows = (long)B * Hq * S;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(256), 0, st, o, dout, delta, B, S, Hq,
                     so, sdo);
}

// query blocks per wave of the dQ-from-dS kernel: 2 (default: the K tile staged once per 256 query
// rows) or 1 (RCA_ATTN_DQ_QW; run-time switch rca_attn_set_dq_qw). Interleaved A/B, attention
// backward at the 8B shape: 1.019 / 1.054 / 1.064 ms vs 1.036 / 1.051 / 1.073; with the 8-wave
// forward the 8B step measured 346.25 vs 348.08 ms median (scripts/step_ab.py, 3 rounds); dQ bitwise
// equal to the 1-block form.
static int g_dq_qw = [] {
  const char* e = getenv("RCA_ATTN_DQ_QW");
  return e && atoi(e) == 1 ? 1 : 2;
}();
RCA_API int rca_attn_set_dq_qw(int q) {
  const int old = g_dq_qw;
  g_dq_qw = q == 2 ? 2 : 1;
  return old;
}

void rca_attn_launch_dq_ds(bool causal, const bf16_t* k, const bf16_t* dsw, bf16_t* dq, int B, int S, int Hq, int Hk,
                           long sk, long sdq, float scale, hipStream_t st) {
  const long nb = S / 32, tiles = causal ? nb * (nb + 1) / 2 : nb * nb;
  const int qw = (g_dq_qw == 2 && S % 256 == 0) ? 2 : 1;
  const dim3 grid(B * Hq * (S / (128 * qw))), block(kThreads);
#define RCA_DQ(CC, QQ) \
  hipLaunchKernelGGL((attn_dq_ds_kernel<CC, QQ>), grid, block, 0, st, k, dsw, dq, B, S, Hq, Hk, sk, sdq, tiles, scale)
  if (qw == 2) {
    if (causal) RCA_DQ(true, 2); else RCA_DQ(false, 2);
  } else {
    if (causal) RCA_DQ(true, 1); else RCA_DQ(false, 1);
  }
#undef RCA_DQ
}
