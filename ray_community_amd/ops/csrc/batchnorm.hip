// Fused training-mode BatchNorm (+ residual add) (+ ReLU) for NHWC (channels_last) bf16 activations
// on gfx950 -- the memory-bound glue between ResNet's MIOpen convolutions.
//
// A channels_last [N, C, H, W] tensor is a row-major [R = N*H*W, C] matrix, so every op here is a
// stream of 16-byte vectors (8 channels) with a fixed channel group per thread:
//   fwd: reduce   -> per-block shifted sums   S1 = sum(x - k_c), S2 = sum((x - k_c)^2)   (read x)
//        finalize -> mean, invstd, scale = gamma*invstd, shift = beta - mean*scale, running stats
//        apply    -> out = act(x*scale + shift [+ res])                                   (read x [,res], write out)
//   bwd: reduce   -> per-block sums  Sg = sum(g), Sgx = sum(g*(x - mean)), g = dy*[out > 0] (read dy, out, x)
//        finalize -> dgamma = Sgx*invstd, dbeta = Sg, and dx = A*g + B*x + D coefficients
//        apply    -> dx = A*g + B*x + D  [, dres = g]                                       (read dy, out, x, write dx [,dres])
// The stock path (MIOpen BN fwd = 2 passes + separate ReLU / add / ReLU-backward elementwise kernels)
// moves ~1.6x the bytes and launches 2-3x the kernels.
// The shift k_c = x[0, c] is the same for every block, so partial sums combine by plain addition
// and E[x^2] - E[x]^2 is evaluated on shifted data (no catastrophic cancellation for |mean| >> std).
// Requirements (checked on the host): C % 8 == 0 and (C / 8) divides 256 (C in {8, 16, ..., 2048}).
#include "common.h"

namespace {

constexpr int kThreads = 256;

// MODE 0: forward statistics of x.  MODE 1: backward sums of g and g*(x - mean).
template <int MODE>
__global__ __launch_bounds__(kThreads) void bn_reduce_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ out, const float* __restrict__ mean,
                                                            int relu, long long R, int C, long long rows_per_block,
                                                            float* __restrict__ partial) {
  __shared__ float sm[2 * 2048];
  const int cv = C >> 3;
  const int t = threadIdx.x;
  const int cg = t % cv;           // channel group: channels [8*cg, 8*cg + 8)
  const int r0 = t / cv;           // row offset inside one iteration
  const int rpi = kThreads / cv;   // rows per iteration
  const long long rb = (long long)blockIdx.x * rows_per_block;
  const long long re = rb + rows_per_block < R ? rb + rows_per_block : R;
  float k[8], s1[8], s2[8];
  {
    float tmp[8];
    if (MODE == 0) {
      unpack8(*reinterpret_cast<const u32x4*>(x + cg * 8), tmp);  // row 0: the common shift
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) tmp[j] = mean[cg * 8 + j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k[j] = tmp[j];
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
  }
  for (long long r = rb + r0; r < re; r += rpi) {
    const long long off = r * C + cg * 8;
    float xf[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + off), xf);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = xf[j] - k[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    } else {
      float g[8];
      unpack8(*reinterpret_cast<const u32x4*>(dy + off), g);
      if (relu) {
        float o[8];
        unpack8(*reinterpret_cast<const u32x4*>(out + off), o);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = o[j] > 0.f ? g[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += g[j];
        s2[j] = fmaf(g[j], xf[j] - k[j], s2[j]);
      }
    }
  }
  if (rpi == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      partial[(long long)blockIdx.x * 2 * C + cg * 8 + j] = s1[j];
      partial[(long long)blockIdx.x * 2 * C + C + cg * 8 + j] = s2[j];
    }
    return;
  }
  // rows of one iteration share channels: reduce them through LDS ([rpi][2][C] floats = 16 KB)
  float* mine = sm + r0 * 2 * C;
  if (r0 < rpi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mine[cg * 8 + j] = s1[j];
      mine[C + cg * 8 + j] = s2[j];
    }
  }
  __syncthreads();
  for (int i = t; i < 2 * C; i += kThreads) {
    float acc = 0.f;
    for (int q = 0; q < rpi; ++q) acc += sm[q * 2 * C + i];
    partial[(long long)blockIdx.x * 2 * C + i] = acc;
  }
}

// Column sums of the [nblk][2][C] partials for one 8-channel group per block: each thread folds
// every 256th block row (16 values), then a wave-shuffle + LDS tree reduces over the 256 threads.
// Result: tot[0..7] = S1 (or Sg) and tot[8..15] = S2 (or Sgx) of channels 8*blockIdx.x + j.
__device__ __forceinline__ void reduce_partials(const float* __restrict__ partial, int nblk, int C, float* tot) {
  __shared__ float red[4][16];
  const int cg = blockIdx.x, t = threadIdx.x;
  float a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = 0.f;
  for (int i = t; i < nblk; i += kThreads) {
    const float* p = partial + (long long)i * 2 * C + cg * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] += p[j];
      a[8 + j] += p[C + j];
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = wave_sum(a[j]);
  if ((t & 63) == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) red[t >> 6][j] = a[j];
  }
  __syncthreads();
  if (t < 16) tot[t] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

__global__ __launch_bounds__(kThreads) void bn_fwd_finalize_kernel(const float* __restrict__ partial, int nblk, long long R, int C,
                                                                  const bf16_t* __restrict__ x, const float* __restrict__ gamma,
                                                                  const float* __restrict__ beta, float eps, float momentum,
                                                                  float* __restrict__ running_mean, float* __restrict__ running_var,
                                                                  float* __restrict__ stats /* [4][C]: mean, invstd, scale, shift */) {
  __shared__ float tot[16];
  reduce_partials(partial, nblk, C, tot);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= 8) return;
  const int c = blockIdx.x * 8 + t;
  const float m1 = tot[t] / (float)R;
  float var = tot[8 + t] / (float)R - m1 * m1;  // shifted data: m1 ~ std, no cancellation
  if (var < 0.f) var = 0.f;
  const float mean = bf2f(x[c]) + m1;
  const float invstd = rsqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float bt = beta ? beta[c] : 0.f;
  const float scale = g * invstd;
  stats[c] = mean;
  stats[C + c] = invstd;
  stats[2 * C + c] = scale;
  stats[3 * C + c] = bt - mean * scale;
  if (running_mean) {
    const float unbiased = R > 1 ? var * ((float)R / (float)(R - 1)) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

__global__ __launch_bounds__(kThreads) void bn_bwd_finalize_kernel(const float* __restrict__ partial, int nblk, long long R, int C,
                                                                  const float* __restrict__ stats, const float* __restrict__ gamma,
                                                                  float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                  float* __restrict__ coef /* [3][C]: A, B, D */) {
  __shared__ float tot[16];
  reduce_partials(partial, nblk, C, tot);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= 8) return;
  const int c = blockIdx.x * 8 + t;
  const float sg = tot[t], sgx = tot[8 + t];
  const float mean = stats[c], invstd = stats[C + c];
  const float g = gamma ? gamma[c] : 1.f;
  if (dgamma) dgamma[c] = sgx * invstd;
  if (dbeta) dbeta[c] = sg;
  const float A = g * invstd;
  const float B = -A * invstd * invstd * (sgx / (float)R);
  coef[c] = A;
  coef[C + c] = B;
  coef[2 * C + c] = -A * (sg / (float)R) - B * mean;
}

// out = act(x*scale + shift [+ res]); grid-stride step is a multiple of C/8, so each thread
// keeps one channel group (and its 16 coefficients in registers) for the whole launch.
template <int U>
__global__ __launch_bounds__(kThreads) void bn_fwd_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                               const float* __restrict__ stats, int relu, long long nvec,
                                                               int C, bf16_t* __restrict__ out) {
  const int cv = C >> 3;
  const long long gt = (long long)blockIdx.x * kThreads + threadIdx.x;
  const long long T = (long long)gridDim.x * kThreads;
  const int cg = (int)(gt % cv);
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = stats[2 * C + cg * 8 + j];
    sh[j] = stats[3 * C + cg * 8 + j];
  }
  // U = 4: four 16-B vectors per lane in flight (T is a multiple of C/8, so all four share the
  // channel group); measured slower than U = 1 (g_bn_unroll below)
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  const u32x4* rv = reinterpret_cast<const u32x4*>(res);
  u32x4* ov = reinterpret_cast<u32x4*>(out);
  auto one = [&](const u32x4& xx, const u32x4* rr, long long v) {
    float f[8];
    unpack8(xx, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], sc[j], sh[j]);
    if (rr) {
      float r8[8];
      unpack8(*rr, r8);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += r8[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    }
    ov[v] = pack8(f);
  };
  long long v = gt;
  for (; U == 4 && v + 3 * T < nvec; v += 4 * T) {
    const u32x4 x0 = xv[v], x1 = xv[v + T], x2 = xv[v + 2 * T], x3 = xv[v + 3 * T];
    u32x4 r0, r1, r2, r3;
    if (res) {
      r0 = rv[v];
      r1 = rv[v + T];
      r2 = rv[v + 2 * T];
      r3 = rv[v + 3 * T];
    }
    one(x0, res ? &r0 : nullptr, v);
    one(x1, res ? &r1 : nullptr, v + T);
    one(x2, res ? &r2 : nullptr, v + 2 * T);
    one(x3, res ? &r3 : nullptr, v + 3 * T);
  }
  for (; v < nvec; v += T) {
    const u32x4 x0 = xv[v];
    u32x4 r0;
    if (res) r0 = rv[v];
    one(x0, res ? &r0 : nullptr, v);
  }
}

__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ out,
                                                               const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                                               int relu, long long nvec, int C, bf16_t* __restrict__ dx,
                                                               bf16_t* __restrict__ dres) {
  const int cv = C >> 3;
  const long long gt = (long long)blockIdx.x * kThreads + threadIdx.x;
  const long long T = (long long)gridDim.x * kThreads;
  const int cg = (int)(gt % cv);
  float A[8], B[8], D[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = coef[cg * 8 + j];
    B[j] = coef[C + cg * 8 + j];
    D[j] = coef[2 * C + cg * 8 + j];
  }
  for (long long v = gt; v < nvec; v += T) {
    float g[8], xf[8];
    unpack8(reinterpret_cast<const u32x4*>(dy)[v], g);
    if (relu) {
      float o[8];
      unpack8(reinterpret_cast<const u32x4*>(out)[v], o);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = o[j] > 0.f ? g[j] : 0.f;
      if (dres) reinterpret_cast<u32x4*>(dres)[v] = pack8(g);
    } else if (dres) {
      reinterpret_cast<u32x4*>(dres)[v] = reinterpret_cast<const u32x4*>(dy)[v];
    }
    unpack8(reinterpret_cast<const u32x4*>(x)[v], xf);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = fmaf(A[j], g[j], fmaf(B[j], xf[j], D[j]));
    reinterpret_cast<u32x4*>(dx)[v] = pack8(g);
  }
}

struct Plan {
  int nblk;
  long long rows_per_block;
};

Plan reduce_plan(long long R, int C) {
  const int rpi = kThreads / (C >> 3);
  long long target = (R + (long long)rpi * 32 - 1) / ((long long)rpi * 32);  // >= 32 rows per thread
  if (target > 1024) target = 1024;
  if (target < 1) target = 1;
  long long rpb = (R + target - 1) / target;
  rpb = (rpb + rpi - 1) / rpi * rpi;
  Plan p;
  p.rows_per_block = rpb;
  p.nblk = (int)((R + rpb - 1) / rpb);
  return p;
}

// 1 (default) or 4 vectors in flight per lane in the forward apply pass (RCA_BN_UNROLL=4; run-time
// switch rca_bn_set_unroll for same-process A/Bs). Measured in the folded ResNet-50 inference
// forward (bs 256, 3 interleaved rounds, scripts/diag/replica_alone.py AB_UNROLL=1): 1 vector
// 7.38-7.43 ms, 4 vectors 7.62-7.67 ms, so the single-vector loop stays the default.
int g_bn_unroll = [] {
  const char* e = getenv("RCA_BN_UNROLL");
  return e && atoi(e) == 4 ? 4 : 1;
}();

template <typename... A>
void launch_apply(dim3 grid, dim3 block, int shm, hipStream_t st, A... args) {
  if (g_bn_unroll == 1)
    hipLaunchKernelGGL(bn_fwd_apply_kernel<1>, grid, block, shm, st, args...);
  else
    hipLaunchKernelGGL(bn_fwd_apply_kernel<4>, grid, block, shm, st, args...);
}

int apply_grid(long long nvec) {
  long long g = (nvec + kThreads - 1) / kThreads;
  if (g > 4096) g = 4096;  // 16 blocks per CU; step stays a multiple of 256 >= C/8
  if (g < 1) g = 1;
  return (int)g;
}

bool supported(int C) { return C >= 8 && C <= 2048 && C % 8 == 0 && (kThreads % (C >> 3)) == 0; }

}  // namespace

RCA_API int rca_bn_set_unroll(int u) {
  const int old = g_bn_unroll;
  g_bn_unroll = u == 4 ? 4 : 1;
  return old;
}

// Workspace floats needed by the partial sums of a reduction over [R, C].
RCA_API long long rca_bn_workspace(long long R, int C) {
  if (!supported(C)) return -1;
  Plan p = reduce_plan(R, C);
  return (long long)p.nblk * 2 * C;
}

// Training forward. stats: [4][C] f32 out (mean, invstd, scale, shift). running_* may be null.
RCA_API int rca_bn_fwd(const void* x, const void* res, const float* gamma, const float* beta, float* running_mean,
                       float* running_var, float* stats, float* ws, void* out, long long R, int C, float eps,
                       float momentum, int relu, hipStream_t stream) {
  if (!supported(C) || R < 1) return -1;
  Plan p = reduce_plan(R, C);
  hipLaunchKernelGGL(bn_reduce_kernel<0>, dim3(p.nblk), dim3(kThreads), 0, stream, (const bf16_t*)x, nullptr, nullptr, nullptr,
                     0, R, C, p.rows_per_block, ws);
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(C / 8), dim3(kThreads), 0, stream, ws, p.nblk, R, C, (const bf16_t*)x,
                     gamma, beta, eps, momentum, running_mean, running_var, stats);
  const long long nvec = R * C / 8;
  launch_apply(dim3(apply_grid(nvec)), dim3(kThreads), 0, stream, (const bf16_t*)x, (const bf16_t*)res,
                     stats, relu, nvec, C, (bf16_t*)out);
  return (int)hipGetLastError();
}

// Inference / frozen-statistics forward: stats already holds scale (row 2) and shift (row 3).
RCA_API int rca_bn_apply(const void* x, const void* res, const float* stats, void* out, long long R, int C, int relu,
                         hipStream_t stream) {
  if (!supported(C) || R < 1) return -1;
  const long long nvec = R * C / 8;
  launch_apply(dim3(apply_grid(nvec)), dim3(kThreads), 0, stream, (const bf16_t*)x, (const bf16_t*)res,
                     stats, relu, nvec, C, (bf16_t*)out);
  return (int)hipGetLastError();
}

// Backward. out = the forward output (ReLU mask); dres (optional) receives the residual gradient.
RCA_API int rca_bn_bwd(const void* dy, const void* out, const void* x, const float* stats, const float* gamma, float* dgamma,
                       float* dbeta, float* coef, float* ws, void* dx, void* dres, long long R, int C, int relu,
                       hipStream_t stream) {
  if (!supported(C) || R < 1) return -1;
  Plan p = reduce_plan(R, C);
  hipLaunchKernelGGL(bn_reduce_kernel<1>, dim3(p.nblk), dim3(kThreads), 0, stream, (const bf16_t*)x, (const bf16_t*)dy,
                     (const bf16_t*)out, stats, relu, R, C, p.rows_per_block, ws);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C / 8), dim3(kThreads), 0, stream, ws, p.nblk, R, C, stats, gamma, dgamma,
                     dbeta, coef);
  const long long nvec = R * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(apply_grid(nvec)), dim3(kThreads), 0, stream, (const bf16_t*)dy, (const bf16_t*)out,
                     (const bf16_t*)x, coef, relu, nvec, C, (bf16_t*)dx, (bf16_t*)dres);
  return (int)hipGetLastError();
}
