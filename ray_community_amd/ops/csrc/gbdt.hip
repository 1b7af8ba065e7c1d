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
// Each workgroup owns FG features x a row range and accumulates a private histogram of
// cnt nodes x FG features x 256 bins x C channels in LDS with ds_add_f32, then flushes the non-zero
// entries with one global float atomic each. hist is float [L, F, 256, C] (bin 255 = missing) and
// must be zeroed by the caller; slot s of this launch lands in node row lo + s.
#include "common.h"

namespace {

constexpr int kBins = 256;

template <int C>
__global__ __launch_bounds__(256) void gbdt_hist_kernel(const unsigned char* __restrict__ bins,
                                                        const int* __restrict__ node,
                                                        const float* __restrict__ gh, float* __restrict__ hist,
                                                        int F, long long ld, int lo, int cnt, int FG,
                                                        long long rows_per_block) {
  extern __shared__ float lh[];
  const int f0 = blockIdx.x * FG;
  const int nf = min(FG, F - f0);
  const int total = cnt * FG * kBins * C;
  for (int i = threadIdx.x; i < total; i += blockDim.x) lh[i] = 0.f;
  __syncthreads();

  const long long r_begin = (long long)blockIdx.y * rows_per_block;  // multiple of 4
  const long long r_end = min(ld, r_begin + rows_per_block);
  const int* node4 = node;
  for (long long r = r_begin + 4 * (long long)threadIdx.x; r < r_end; r += 4 * (long long)blockDim.x) {
    const int4 nd = *reinterpret_cast<const int4*>(node4 + r);
    int s[4] = {nd.x - lo, nd.y - lo, nd.z - lo, nd.w - lo};
    bool any = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if ((unsigned)s[k] >= (unsigned)cnt) s[k] = -1;
      any |= s[k] >= 0;
    }
    if (!any) continue;
    float g[4][C];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < C; ++c) g[k][c] = gh[(r + k) * C + c];
    for (int f = 0; f < nf; ++f) {
      const unsigned b4 = *reinterpret_cast<const unsigned*>(bins + (long long)(f0 + f) * ld + r);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (s[k] < 0) continue;
        const int b = (b4 >> (8 * k)) & 0xff;
        float* dst = lh + ((s[k] * FG + f) * kBins + b) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) atomicAdd(dst + c, g[k][c]);
      }
    }
  }
  __syncthreads();

  // flush: LDS entry (s, f, b, c) -> hist[((lo + s) * F + f0 + f) * 256 + b][c]
  const int per_node = FG * kBins * C;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const float v = lh[i];
    if (v == 0.f) continue;
    const int sl = i / per_node;
    const int rem = i - sl * per_node;
    const int f = rem / (kBins * C);
    if (f >= nf) continue;
    const int bc = rem - f * (kBins * C);
    atomicAdd(hist + ((long long)(lo + sl) * F + f0 + f) * (kBins * C) + bc, v);
  }
}

}  // namespace

// bins [F, ld] u8, node [ld] i32, gh [ld, C] f32, hist [L, F, 256, C] f32 (zeroed), nodes [0, L).
// ld % 4 == 0, C in {2, 3}. Node chunks and feature groups are sized so a workgroup's private
// histogram fits in 64 KB of LDS.
RCA_API int rca_gbdt_hist(const unsigned char* bins, const int* node, const float* gh, float* hist, int F,
                          long long ld, int L, int C, hipStream_t stream) {
  if (F <= 0 || L <= 0 || ld <= 0) return 0;
  if ((ld & 3) != 0 || (C != 2 && C != 3)) return -1;
  constexpr int kLdsBytes = 64 * 1024;
  const int per_nf = kBins * C * (int)sizeof(float);  // one node x one feature
  const int max_nodes = kLdsBytes / per_nf;           // 32 (C=2) / 21 (C=3) nodes per launch at FG=1
  for (int lo = 0; lo < L; lo += max_nodes) {
    const int cnt = min(max_nodes, L - lo);
    // <= 4 features per workgroup (more workgroups, private histogram cheap to clear and flush)
    const int FG = max(1, min(min(F, 4), kLdsBytes / (cnt * per_nf)));
    const int gx = (F + FG - 1) / FG;
    // rows per workgroup >= 8 x the private histogram's bins, so the clear + flush (one global atomic
    // per non-zero entry) stays a small share of the row work; but keep >= ~1024 workgroups (4 per CU)
    // while each still gets >= 1024 rows
    long long rpb = max(1024LL, 2048LL * cnt);
    long long gy = (ld + rpb - 1) / rpb;
    if ((long long)gx * gy < 1024) {
      gy = max(1LL, min((ld + 1023) / 1024, (1024LL + gx - 1) / gx));
      rpb = (ld + gy - 1) / gy;
    }
    rpb = (rpb + 3) & ~3LL;
    gy = (ld + rpb - 1) / rpb;
    const size_t lds = (size_t)cnt * FG * per_nf;
    dim3 grid(gx, (unsigned)gy);
    if (C == 2)
      hipLaunchKernelGGL(gbdt_hist_kernel<2>, grid, dim3(256), lds, stream, bins, node, gh, hist, F, ld, lo, cnt, FG,
                         rpb);
    else
      hipLaunchKernelGGL(gbdt_hist_kernel<3>, grid, dim3(256), lds, stream, bins, node, gh, hist, F, ld, lo, cnt, FG,
                         rpb);
  }
  return (int)hipGetLastError();
}
