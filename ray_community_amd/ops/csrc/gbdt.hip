// Gradient-histogram construction for the data-parallel GBDT trainers (train/gbdt).
//
// The reference hands boosting to xgboost / lightgbm (python/ray/train/xgboost/xgboost_trainer.py:18,
// python/ray/train/lightgbm/lightgbm_trainer.py): each worker builds per-node gradient histograms over
// its data shard and the workers all-reduce them (rabit / lightgbm sockets). Here the histogram pass
// is this kernel and the all-reduce is RCCL; split finding on the reduced histograms is a few
// vectorised torch ops (train/gbdt/core.py).
//
// Layout (chosen for the GPU, not the CPU): the quantised matrix is FEATURE-major uint8 [F, ld]
// (ld = rows padded to a multiple of 4), so one 32-bit load gives a lane the bins of 4 consecutive
// rows of one feature and a wave reads 256 contiguous bytes; per-row node slots are int32 [ld]
// (-1 = row not in any node being built, also used for the padding) and the gradient statistics are
// float [ld, C] (C = 2: grad, hess; C = 3 adds a row count for min_data_in_leaf).
//
// Each workgroup (16 waves) owns FG features x a row range and accumulates a private histogram of
// cnt nodes x FG features x 256 bins in LDS (folded into per-thread float accumulators after every
// 32768-row chunk), then stores it into a per-workgroup partial
// buffer; a second kernel sums the partials of the row ranges per entry in a fixed order.
//
// Fixed-point LDS accumulation. Measured on gfx950 (scripts/probes/lds_atomic_probe.hip, random bins
// over 256 slots, 16 waves/CU): ds_add_f32 costs ~194 LDS cycles per wave-instruction, ds_add_u32
// 14.5 and ds_add_u64 15.6. So (grad, hess) arrive pre-quantised and packed in ONE 64-bit word per
// row -- signed grad * sg in the high half, hess * sh (>= 0) in the low half -- and each (row,
// feature) is ONE ds_add_u64: the low half never carries (|h_q| <= 2^32 / 32768 per row, rows taken in
// chunks of 32768), the high half adds modulo 2^32 and stays within int32 for the same reason.
// The optional row count (C = 3) is one more ds_add_u32. The flush converts the integer sums back
// with the scales (inv[0] = 1/sg, inv[1] = 1/sh), so the float partials and the reduction are exact
// sums of the quantised values. (First version: two ds_add_f32 per (row, feature) + one global
// float atomic per non-zero entry in the flush: 573 us for 2M x 28 where this form takes a fraction.)
#include "common.h"

namespace {

constexpr int kBins = 256;
constexpr long long kChunk = 32768;  // rows per fixed-point accumulation chunk (see top)
constexpr int kPerThread = 8;        // LDS entries drained per thread: 64 KB / 8 B / 1024 threads

template <bool CNT, int FGT>
__global__ __launch_bounds__(1024) void gbdt_hist_kernel(const unsigned char* __restrict__ bins,
                                                         const int* __restrict__ node,
                                                         const unsigned long long* __restrict__ ghq,
                                                         const float* __restrict__ inv, float* __restrict__ part,
                                                         int F, long long ld, int lo, int cnt, int FG,
                                                         long long rows_per_block) {
  extern __shared__ unsigned long long lq[];
  constexpr int C = CNT ? 3 : 2;
  const int f0 = blockIdx.x * FG;
  const int nf = min(FG, F - f0);
  const int ent = cnt * FG * kBins;  // histogram entries of this workgroup
  unsigned* lc = reinterpret_cast<unsigned*>(lq + ent);
  for (int i = threadIdx.x; i < ent; i += blockDim.x) {
    lq[i] = 0ull;
    if (CNT) lc[i] = 0u;
  }
  __syncthreads();

  // entries this thread drains: i = threadIdx.x + j * 1024, j < kPerThread (ent <= 8192)
  float acc[kPerThread][C];
#pragma unroll
  for (int j = 0; j < kPerThread; ++j)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[j][c] = 0.f;

  const long long r_begin = (long long)blockIdx.y * rows_per_block;  // multiple of 4
  const long long r_end = min(ld, r_begin + rows_per_block);
  const unsigned char* bcol = bins + (long long)f0 * ld;
  const float ig = inv[0], ih = inv[1];
  // rows in chunks of kChunk: the integer sums of one chunk fit their 32-bit halves (see top); after
  // each chunk the LDS integers are folded into per-thread float accumulators and cleared
  for (long long c0 = r_begin; c0 < r_end; c0 += kChunk) {
    const long long c1 = min(r_end, c0 + kChunk);
    for (long long r = c0 + 4 * (long long)threadIdx.x; r < c1; r += 4 * (long long)blockDim.x) {
      // every load of this row quad is issued before the first use (one memory round trip per quad)
      const int4 nd = *reinterpret_cast<const int4*>(node + r);
      const ulonglong2 q01 = reinterpret_cast<const ulonglong2*>(ghq + r)[0];
      const ulonglong2 q23 = reinterpret_cast<const ulonglong2*>(ghq + r)[1];
      unsigned b4[FGT];
#pragma unroll
      for (int f = 0; f < FGT; ++f)
        b4[f] = f < nf ? *reinterpret_cast<const unsigned*>(bcol + (long long)f * ld + r) : 0u;
      const int s[4] = {nd.x - lo, nd.y - lo, nd.z - lo, nd.w - lo};
      const unsigned long long q[4] = {q01.x, q01.y, q23.x, q23.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((unsigned)s[k] >= (unsigned)cnt) continue;
#pragma unroll
        for (int f = 0; f < FGT; ++f) {
          if (f >= nf) break;
          const int e = (s[k] * FG + f) * kBins + ((b4[f] >> (8 * k)) & 0xff);
          atomicAdd(lq + e, q[k]);
          if (CNT) atomicAdd(lc + e, 1u);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
      const int i = threadIdx.x + j * 1024;
      if (i < ent) {
        const unsigned long long v = lq[i];
        acc[j][0] += (float)(int)(unsigned)(v >> 32) * ig;
        acc[j][1] += (float)(unsigned)(v & 0xffffffffull) * ih;
        lq[i] = 0ull;
        if (CNT) {
          acc[j][C - 1] += (float)lc[i];
          lc[i] = 0u;
        }
      }
    }
    __syncthreads();
  }
  float* out = part + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * (long long)ent * C;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    const int i = threadIdx.x + j * 1024;
    if (i < ent)
#pragma unroll
      for (int c = 0; c < C; ++c) out[i * C + c] = acc[j][c];
  }
}

// hist entry (lo + s, f0 + f, b, c) = sum over the gy row ranges of the partials, fixed order.
__global__ __launch_bounds__(256) void gbdt_hist_reduce_kernel(const float* __restrict__ part,
                                                               float* __restrict__ hist, int F, int gx, int gy,
                                                               int lo, int cnt, int FG, int C) {
  const int total = cnt * FG * kBins * C;
  const int bx = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int per_node = FG * kBins * C;
  const int sl = i / per_node;
  const int rem = i - sl * per_node;
  const int f = rem / (kBins * C);
  const int f0 = bx * FG;
  if (f0 + f >= F) return;
  float acc = 0.f;
  const float* p = part + (long long)bx * total + i;
  const long long stride = (long long)gx * total;
  // 8 independent loads in flight per step (the partials are one HBM round trip each); the sum
  // order is fixed: bitwise-reproducible histograms for a given launch geometry
  float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int y = 0;
  for (; y + 8 <= gy; y += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a8[u] += p[(long long)(y + u) * stride];
  }
  for (; y < gy; ++y) a8[0] += p[(long long)y * stride];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc += a8[u];
  const int bc = rem - f * (kBins * C);
  hist[((long long)(lo + sl) * F + f0 + f) * (kBins * C) + bc] = acc;
}

// Exact mode (parity checks; also chosen automatically when the hessians span too many binades
// for the fixed-point scales -- ops.gbdt_histogram): the float (grad, hess) are added in fp64 LDS
// atomics (ds_add_f64), partials and the fixed-order reduction stay fp64 and the result is rounded
// to fp32 once, so it equals an fp64 accumulation on the CPU rounded to fp32 (the CPU exact path)
// up to the last bit of the fp64 sum.
template <bool CNT, int FGT>
__global__ __launch_bounds__(1024) void gbdt_hist_exact_kernel(const unsigned char* __restrict__ bins,
                                                               const int* __restrict__ node,
                                                               const float* __restrict__ gh,
                                                               double* __restrict__ part, int F, long long ld, int lo,
                                                               int cnt, int FG, long long rows_per_block) {
  extern __shared__ double ld64[];
  constexpr int C = CNT ? 3 : 2;
  const int f0 = blockIdx.x * FG;
  const int nf = min(FG, F - f0);
  const int ent = cnt * FG * kBins;
  for (int i = threadIdx.x; i < ent * C; i += blockDim.x) ld64[i] = 0.0;
  __syncthreads();
  const long long r_begin = (long long)blockIdx.y * rows_per_block;
  const long long r_end = min(ld, r_begin + rows_per_block);
  const unsigned char* bcol = bins + (long long)f0 * ld;
  for (long long r = r_begin + 4 * (long long)threadIdx.x; r < r_end; r += 4 * (long long)blockDim.x) {
    const int4 nd = *reinterpret_cast<const int4*>(node + r);
    unsigned b4[FGT];
#pragma unroll
    for (int f = 0; f < FGT; ++f) b4[f] = f < nf ? *reinterpret_cast<const unsigned*>(bcol + (long long)f * ld + r) : 0u;
    const int s[4] = {nd.x - lo, nd.y - lo, nd.z - lo, nd.w - lo};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if ((unsigned)s[k] >= (unsigned)cnt) continue;
      const float* row = gh + (r + k) * C;
      const double g = row[0], h = row[1];
#pragma unroll
      for (int f = 0; f < FGT; ++f) {
        if (f >= nf) break;
        const int e = (s[k] * FG + f) * kBins + ((b4[f] >> (8 * k)) & 0xff);
        atomicAdd(ld64 + e * C, g);
        atomicAdd(ld64 + e * C + 1, h);
        if (CNT) atomicAdd(ld64 + e * C + 2, (double)row[2]);
      }
    }
  }
  __syncthreads();
  double* out = part + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * (long long)ent * C;
  for (int i = threadIdx.x; i < ent * C; i += blockDim.x) out[i] = ld64[i];
}

__global__ __launch_bounds__(256) void gbdt_hist_exact_reduce_kernel(const double* __restrict__ part,
                                                                     float* __restrict__ hist, int F, int gx, int gy,
                                                                     int lo, int cnt, int FG, int C) {
  const int total = cnt * FG * kBins * C;
  const int bx = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int per_node = FG * kBins * C;
  const int sl = i / per_node;
  const int rem = i - sl * per_node;
  const int f = rem / (kBins * C);
  const int f0 = bx * FG;
  if (f0 + f >= F) return;
  double acc = 0.0;
  const double* p = part + (long long)bx * total + i;
  const long long stride = (long long)gx * total;
  for (int y = 0; y < gy; ++y) acc += p[(long long)y * stride];
  const int bc = rem - f * (kBins * C);
  hist[((long long)(lo + sl) * F + f0 + f) * (kBins * C) + bc] = (float)acc;
}

namespace plan {
constexpr int kLdsBytes = 64 * 1024;
// exact mode: one fp64 per (entry, channel)
inline int max_nodes_exact(int C) { return kLdsBytes / (kBins * C * (int)sizeof(double)); }
inline int feat_group_exact(int F, int cnt, int C) {
  return max(1, min(min(F, 4), kLdsBytes / (cnt * kBins * C * (int)sizeof(double))));
}
inline int max_nodes(int C) { return kLdsBytes / (kBins * C * (int)sizeof(float)); }
inline int feat_group(int F, int cnt, int C) {
  return max(1, min(min(F, 4), kLdsBytes / (cnt * kBins * C * (int)sizeof(float))));
}
// ~512 workgroups of 16 waves (2 per CU, as LDS allows), >= 4096 rows each; the partial buffer is
// then <= 512 x 64 KB-worth of floats whatever the row count
inline long long row_blocks(long long ld, int gx) {
  long long gy = (512 + gx - 1) / gx;
  return max(1LL, min(gy, (ld + 4095) / 4096));
}
}  // namespace plan

}  // namespace

// Bytes of the partial-histogram workspace rca_gbdt_hist needs for these sizes.
RCA_API long long rca_gbdt_hist_workspace(int F, long long ld, int L, int C) {
  long long best = 0;
  for (int lo = 0; lo < L; lo += plan::max_nodes(C)) {
    const int cnt = min(plan::max_nodes(C), L - lo);
    const int FG = plan::feat_group(F, cnt, C);
    const int gx = (F + FG - 1) / FG;
    const long long gy = plan::row_blocks(ld, gx);
    best = max(best, gy * gx * (long long)cnt * FG * kBins * C * (long long)sizeof(float));
  }
  return best;
}

// bins [F, ld] u8, node [ld] i32, ghq [ld] u64 (packed fixed-point grad/hess, see top), inv [2] f32
// (1/sg, 1/sh) on the device, hist [L, F, 256, C] f32 (every entry written), work >=
// rca_gbdt_hist_workspace bytes. ld % 4 == 0; C = 3 adds the row count.
RCA_API int rca_gbdt_hist(const unsigned char* bins, const int* node, const unsigned long long* ghq,
                          const float* inv, float* hist, float* work, int F, long long ld, int L, int C,
                          hipStream_t stream) {
  if (F <= 0 || L <= 0 || ld <= 0) return 0;
  if ((ld & 3) != 0 || (C != 2 && C != 3)) return -1;
  for (int lo = 0; lo < L; lo += plan::max_nodes(C)) {
    const int cnt = min(plan::max_nodes(C), L - lo);
    const int FG = plan::feat_group(F, cnt, C);
    const int gx = (F + FG - 1) / FG;
    const long long gy = plan::row_blocks(ld, gx);
    long long rpb = (ld + gy - 1) / gy;
    rpb = (rpb + 3) & ~3LL;
    const int ent = cnt * FG * kBins;
    const size_t lds = (size_t)ent * (sizeof(unsigned long long) + (C == 3 ? sizeof(unsigned) : 0));
    dim3 grid(gx, (unsigned)gy);
#define RCA_GBDT_LAUNCH(CC, FF)                                                                                  \
  hipLaunchKernelGGL((gbdt_hist_kernel<CC, FF>), grid, dim3(1024), lds, stream, bins, node, ghq, inv, work, F, ld, \
                     lo, cnt, FG, rpb)
    if (C == 2) {
      if (FG == 1) RCA_GBDT_LAUNCH(false, 1); else if (FG == 2) RCA_GBDT_LAUNCH(false, 2); else RCA_GBDT_LAUNCH(false, 4);
    } else {
      if (FG == 1) RCA_GBDT_LAUNCH(true, 1); else if (FG == 2) RCA_GBDT_LAUNCH(true, 2); else RCA_GBDT_LAUNCH(true, 4);
    }
#undef RCA_GBDT_LAUNCH
    dim3 rgrid((ent * C + 255) / 256, gx);
    hipLaunchKernelGGL(gbdt_hist_reduce_kernel, rgrid, dim3(256), 0, stream, work, hist, F, gx, (int)gy, lo, cnt,
                       FG, C);
  }
  return (int)hipGetLastError();
}

// Exact-mode workspace bytes and launch (fp64 LDS accumulation, see gbdt_hist_exact_kernel).
RCA_API long long rca_gbdt_hist_exact_workspace(int F, long long ld, int L, int C) {
  long long best = 0;
  for (int lo = 0; lo < L; lo += plan::max_nodes_exact(C)) {
    const int cnt = min(plan::max_nodes_exact(C), L - lo);
    const int FG = plan::feat_group_exact(F, cnt, C);
    const int gx = (F + FG - 1) / FG;
    const long long gy = plan::row_blocks(ld, gx);
    best = max(best, gy * gx * (long long)cnt * FG * kBins * C * (long long)sizeof(double));
  }
  return best;
}

// gh: float [ld, C] (grad, hess[, count]) as is (no quantisation); hist float [L, F, 256, C].
RCA_API int rca_gbdt_hist_exact(const unsigned char* bins, const int* node, const float* gh, float* hist,
                                double* work, int F, long long ld, int L, int C, hipStream_t stream) {
  if (F <= 0 || L <= 0 || ld <= 0) return 0;
  if ((ld & 3) != 0 || (C != 2 && C != 3)) return -1;
  for (int lo = 0; lo < L; lo += plan::max_nodes_exact(C)) {
    const int cnt = min(plan::max_nodes_exact(C), L - lo);
    const int FG = plan::feat_group_exact(F, cnt, C);
    const int gx = (F + FG - 1) / FG;
    const long long gy = plan::row_blocks(ld, gx);
    long long rpb = (ld + gy - 1) / gy;
    rpb = (rpb + 3) & ~3LL;
    const int ent = cnt * FG * kBins;
    const size_t lds = (size_t)ent * C * sizeof(double);
    dim3 grid(gx, (unsigned)gy);
#define RCA_GBDT_EX(CC, FF)                                                                                      \
  hipLaunchKernelGGL((gbdt_hist_exact_kernel<CC, FF>), grid, dim3(1024), lds, stream, bins, node, gh, work, F, ld, \
                     lo, cnt, FG, rpb)
    if (C == 2) {
      if (FG == 1) RCA_GBDT_EX(false, 1); else if (FG == 2) RCA_GBDT_EX(false, 2); else RCA_GBDT_EX(false, 4);
    } else {
      if (FG == 1) RCA_GBDT_EX(true, 1); else if (FG == 2) RCA_GBDT_EX(true, 2); else RCA_GBDT_EX(true, 4);
    }
#undef RCA_GBDT_EX
    dim3 rgrid((ent * C + 255) / 256, gx);
    hipLaunchKernelGGL(gbdt_hist_exact_reduce_kernel, rgrid, dim3(256), 0, stream, work, hist, F, gx, (int)gy, lo,
                       cnt, FG, C);
  }
  return (int)hipGetLastError();
}
