// RMSNorm forward/backward (optionally fused with the residual add) for gfx950.
//
// Layout: rows x H, bf16, row-major. One wave (64 lanes) owns one row; each lane moves
// 16 B (8 x bf16) per access, so one wave-instruction covers 512 columns. For H a multiple
// of 512 and <= 8192 the row stays in VGPRs between the reduction and the scale pass
// (template VPL = H / 512); otherwise a generic two-pass loop re-reads the row (L1/L2 hit).
//
// Forward (fused): s = x + r (stored if sum_out), y = s * rsqrt(mean(s^2) + eps) * w
// Backward: dx = rstd * (w*dy) - s * rstd^3 / H * sum(s*w*dy) (+ dres), dw = sum_rows dy*s*rstd
// dw is reduced per block in LDS, then across blocks by a column-sum kernel (no atomics,
// bitwise reproducible).
#include "common.h"

template <int VPL>
__global__ __launch_bounds__(256) void rmsnorm_fwd_reg(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                       const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                       bf16_t* __restrict__ sum_out, float* __restrict__ rstd,
                                                       int rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + (size_t)row * H);
  u32x4 pv[VPL];  // the row stays packed in VGPRs: 4 registers per 8 elements
#pragma unroll
  for (int i = 0; i < VPL; ++i) pv[i] = __builtin_nontemporal_load(xr + i * 64 + lane);
  if (res) {
    const u32x4* rr = reinterpret_cast<const u32x4*>(res + (size_t)row * H);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float a[8], t[8];
      unpack8(pv[i], a);
      unpack8(__builtin_nontemporal_load(rr + i * 64 + lane), t);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += t[j];
      pv[i] = pack8(a);  // rounds like an unfused bf16 add
    }
    if (sum_out) {
      u32x4* so = reinterpret_cast<u32x4*>(sum_out + (size_t)row * H);
#pragma unroll
      for (int i = 0; i < VPL; ++i) so[i * 64 + lane] = pv[i];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    float a[8];
    unpack8(pv[i], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)H + eps);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4* yr = reinterpret_cast<u32x4*>(y + (size_t)row * H);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    float a[8], wf[8], o[8];
    unpack8(pv[i], a);
    unpack8(wr[i * 64 + lane], wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(a[j] * r)) * wf[j];
    yr[i * 64 + lane] = pack8(o);
  }
  if (lane == 0) rstd[row] = r;
}

__global__ __launch_bounds__(256) void rmsnorm_fwd_generic(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                           const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                           bf16_t* __restrict__ sum_out, float* __restrict__ rstd,
                                                           int rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = H >> 3;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + (size_t)row * H);
  const u32x4* rr = res ? reinterpret_cast<const u32x4*>(res + (size_t)row * H) : nullptr;
  u32x4* so = (res && sum_out) ? reinterpret_cast<u32x4*>(sum_out + (size_t)row * H) : nullptr;
  float ss = 0.f;
  for (int c = lane; c < nv; c += 64) {
    float v[8];
    unpack8(xr[c], v);
    if (rr) {
      float t[8];
      unpack8(rr[c], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] + t[j]));
      if (so) so[c] = pack8(v);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)H + eps);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4* yr = reinterpret_cast<u32x4*>(y + (size_t)row * H);
  for (int c = lane; c < nv; c += 64) {
    float v[8], wf[8], o[8];
    unpack8(xr[c], v);
    if (rr) {
      float t[8];
      unpack8(rr[c], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] + t[j]));
    }
    unpack8(wr[c], wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(v[j] * r)) * wf[j];
    yr[c] = pack8(o);
  }
  if (lane == 0) rstd[row] = r;
}

// Backward. Each block (4 waves) walks rows with a grid stride; per-lane dw partials for
// the lane's columns live in registers, then the 4 waves are summed through LDS and written
// to dw_part[blockIdx.x][H] (fp32).
template <int VPL>
__global__ __launch_bounds__(256) void rmsnorm_bwd_reg(const bf16_t* __restrict__ s, const bf16_t* __restrict__ dy,
                                                       const bf16_t* __restrict__ w, const float* __restrict__ rstd,
                                                       const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                       float* __restrict__ dw_part, int rows, int H) {
  // Rows stay packed in VGPRs (s, dy: 8 registers per 8 columns); the per-wave dw partial lives
  // in this wave's own LDS slice (lane-private columns: no conflicts, no barrier in the loop), so
  // the kernel holds ~5 waves/SIMD instead of 1 with register accumulators.
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nwave_total = gridDim.x * 4;
  float* accw = lds + (size_t)wid * H;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    f32x4* a4 = reinterpret_cast<f32x4*>(accw + (i * 64 + lane) * 8);
    a4[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    a4[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  const float invH = 1.f / (float)H;
  for (int row = blockIdx.x * 4 + wid; row < rows; row += nwave_total) {
    const u32x4* sr = reinterpret_cast<const u32x4*>(s + (size_t)row * H);
    const u32x4* gr = reinterpret_cast<const u32x4*>(dy + (size_t)row * H);
    u32x4 ps[VPL], pg[VPL];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      ps[i] = __builtin_nontemporal_load(sr + i * 64 + lane);
      pg[i] = __builtin_nontemporal_load(gr + i * 64 + lane);
    }
    const float r = rstd[row];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float sv[8], gv[8], wf[8];
      unpack8(ps[i], sv);
      unpack8(pg[i], gv);
      unpack8(wr[i * 64 + lane], wf);
      f32x4* a4 = reinterpret_cast<f32x4*>(accw + (i * 64 + lane) * 8);
      f32x4 a0 = a4[0], a1 = a4[1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dot += sv[j] * wf[j] * gv[j];
        const float contrib = gv[j] * bf2f(f2bf(sv[j] * r));
        if (j < 4) a0[j] += contrib; else a1[j - 4] += contrib;
      }
      a4[0] = a0;
      a4[1] = a1;
    }
    dot = wave_sum(dot);
    const float c = dot * r * r * r * invH;
    u32x4* xr = reinterpret_cast<u32x4*>(dx + (size_t)row * H);
    const u32x4* drr = dres ? reinterpret_cast<const u32x4*>(dres + (size_t)row * H) : nullptr;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float sv[8], gv[8], wf[8], o[8];
      unpack8(ps[i], sv);
      unpack8(pg[i], gv);
      unpack8(wr[i * 64 + lane], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = r * wf[j] * gv[j] - c * sv[j];
      if (drr) {
        float t[8];
        unpack8(__builtin_nontemporal_load(drr + i * 64 + lane), t);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += t[j];
      }
      xr[i * 64 + lane] = pack8(o);
    }
  }
  __syncthreads();
  float* out = dw_part + (size_t)blockIdx.x * H;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    f32x4 t = *reinterpret_cast<f32x4*>(lds + c);
#pragma unroll
    for (int k = 1; k < 4; ++k) t += *reinterpret_cast<f32x4*>(lds + (size_t)k * H + c);
    *reinterpret_cast<f32x4*>(out + c) = t;
  }
}

// Backward for H = 2048 * CPW (Llama hidden sizes 2048/4096). The per-wave LDS dw slices of
// rmsnorm_bwd_reg cost 4*H*4 B per block (64 KB at H=4096 -> 2 waves/SIMD) and the generic
// two-pass loop keeps only ~3 loads in flight per wave. Here a block walks rows TWO at a time and
// its 4 waves split the columns (wave w owns H/4): each lane keeps its 8*CPW columns' dw partial in
// VGPRs, both rows' s/dy stay packed in VGPRs (4*CPW 16-B loads in flight per lane), and the row
// dot products are combined across the 4 waves through 8 LDS floats (double-buffered by
// iteration parity: one barrier per row pair). No cross-wave dw fold is needed: every column has
// one owner lane, which writes its block partial directly (fixed order: bitwise reproducible).
template <int CPW>
__global__ __launch_bounds__(256) void rmsnorm_bwd_split(const bf16_t* __restrict__ s, const bf16_t* __restrict__ dy,
                                                         const bf16_t* __restrict__ w, const float* __restrict__ rstd,
                                                         const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                         float* __restrict__ dw_part, int rows, int H) {
  __shared__ float dots[2][2][4];  // [parity][row of pair][wave]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cbase = wid * CPW * 64 + lane;  // u32x4 column index of chunk 0 (chunk stride 64)
  float acc[CPW][8];
#pragma unroll
  for (int i = 0; i < CPW; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  float wf[CPW][8];
#pragma unroll
  for (int i = 0; i < CPW; ++i) unpack8(wr[cbase + i * 64], wf[i]);
  const float invH = 1.f / (float)H;
  int parity = 0;
  for (int r0 = blockIdx.x * 2; r0 < rows; r0 += gridDim.x * 2, parity ^= 1) {
    const bool two = r0 + 1 < rows;
    u32x4 ps[2][CPW], pg[2][CPW], pd[2][CPW];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = two ? r0 + k : r0;
      const u32x4* sr = reinterpret_cast<const u32x4*>(s + (size_t)row * H);
      const u32x4* gr = reinterpret_cast<const u32x4*>(dy + (size_t)row * H);
#pragma unroll
      for (int i = 0; i < CPW; ++i) {
        ps[k][i] = __builtin_nontemporal_load(sr + cbase + i * 64);
        pg[k][i] = __builtin_nontemporal_load(gr + cbase + i * 64);
      }
      // the residual gradient is only added after the row-dot barrier: issue its loads now so
      // they are in flight across the reduction instead of starting after it
      if (dres) {
        const u32x4* drr = reinterpret_cast<const u32x4*>(dres + (size_t)row * H);
#pragma unroll
        for (int i = 0; i < CPW; ++i) pd[k][i] = __builtin_nontemporal_load(drr + cbase + i * 64);
      }
    }
    float rr[2], dot[2] = {0.f, 0.f};
    rr[0] = rstd[r0];
    rr[1] = two ? rstd[r0 + 1] : 0.f;  // a missing second row contributes nothing to dw
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int i = 0; i < CPW; ++i) {
        float sv[8], gv[8];
        unpack8(ps[k][i], sv);
        unpack8(pg[k][i], gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dot[k] += sv[j] * wf[i][j] * gv[j];
          acc[i][j] += gv[j] * bf2f(f2bf(sv[j] * rr[k]));
        }
      }
    }
    dot[0] = wave_sum(dot[0]);
    dot[1] = wave_sum(dot[1]);
    if (lane == 0) {
      dots[parity][0][wid] = dot[0];
      dots[parity][1][wid] = dot[1];
    }
    __syncthreads();
    // opaque: stops the compiler keeping pass-1's unpacked fp32 rows (2x the packed VGPRs) alive
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < CPW; ++i) asm volatile("" : "+v"(ps[k][i]), "+v"(pg[k][i]), "+v"(pd[k][i]));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && !two) break;
      const int row = r0 + k;
      const float d = dots[parity][k][0] + dots[parity][k][1] + dots[parity][k][2] + dots[parity][k][3];
      const float r = rr[k];
      const float c = d * r * r * r * invH;
      u32x4* xr = reinterpret_cast<u32x4*>(dx + (size_t)row * H);
#pragma unroll
      for (int i = 0; i < CPW; ++i) {
        float sv[8], gv[8], o[8];
        unpack8(ps[k][i], sv);
        unpack8(pg[k][i], gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r * wf[i][j] * gv[j] - c * sv[j];
        if (dres) {
          float t[8];
          unpack8(pd[k][i], t);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += t[j];
        }
        xr[cbase + i * 64] = pack8(o);
      }
    }
  }
  f32x4* out = reinterpret_cast<f32x4*>(dw_part + (size_t)blockIdx.x * H);
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    out[(cbase + i * 64) * 2] = f32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
    out[(cbase + i * 64) * 2 + 1] = f32x4{acc[i][4], acc[i][5], acc[i][6], acc[i][7]};
  }
}

__global__ __launch_bounds__(256) void rmsnorm_bwd_generic(const bf16_t* __restrict__ s, const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ w, const float* __restrict__ rstd,
                                                           const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                           float* __restrict__ dw_part, int rows, int H) {
  // generic path: one block per grid-stride set of rows, dw partial accumulated in LDS (H <= 40960)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nv = H >> 3;
  for (int c = threadIdx.x; c < 4 * H; c += blockDim.x) lds[c] = 0.f;
  __syncthreads();
  const float invH = 1.f / (float)H;
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  for (int row = blockIdx.x * 4 + wid; row < rows; row += gridDim.x * 4) {
    const u32x4* sr = reinterpret_cast<const u32x4*>(s + (size_t)row * H);
    const u32x4* gr = reinterpret_cast<const u32x4*>(dy + (size_t)row * H);
    const float r = rstd[row];
    float dot = 0.f;
    for (int c = lane; c < nv; c += 64) {
      float sv[8], gv[8], wf[8];
      unpack8(sr[c], sv);
      unpack8(gr[c], gv);
      unpack8(wr[c], wf);
      f32x4* a4 = reinterpret_cast<f32x4*>(lds + (size_t)wid * H + c * 8);
      f32x4 a0 = a4[0], a1 = a4[1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dot += sv[j] * wf[j] * gv[j];
        const float contrib = gv[j] * bf2f(f2bf(sv[j] * r));
        if (j < 4) a0[j] += contrib; else a1[j - 4] += contrib;
      }
      a4[0] = a0;
      a4[1] = a1;
    }
    dot = wave_sum(dot);
    const float cc = dot * r * r * r * invH;
    u32x4* xr = reinterpret_cast<u32x4*>(dx + (size_t)row * H);
    const u32x4* drr = dres ? reinterpret_cast<const u32x4*>(dres + (size_t)row * H) : nullptr;
    for (int c = lane; c < nv; c += 64) {
      float sv[8], gv[8], wf[8], o[8];
      unpack8(sr[c], sv);
      unpack8(gr[c], gv);
      unpack8(wr[c], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = r * wf[j] * gv[j] - cc * sv[j];
      if (drr) {
        float t[8];
        unpack8(drr[c], t);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += t[j];
      }
      xr[c] = pack8(o);
    }
  }
  __syncthreads();
  float* out = dw_part + (size_t)blockIdx.x * H;
  for (int c = threadIdx.x; c < H; c += blockDim.x) out[c] = lds[c] + lds[H + c] + lds[2 * H + c] + lds[3 * H + c];
}

// dw[c] = sum_b part[b][c]; written as bf16 (dw_bf16) and/or accumulated into fp32 (dw_f32 += ...)
// Block = 16 column-quads (64 columns, f32x4 per lane) x 16 row groups; the 16 partial sums per
// column are combined through LDS. Grid = H / 64 blocks, each streaming nb rows of 256 B.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, int nb, int H,
                                                     bf16_t* __restrict__ dw_bf16, float* __restrict__ dw_f32,
                                                     int accumulate) {
  __shared__ f32x4 red[16][16];
  const int cq = threadIdx.x & 15;  // column quad within the block
  const int rg = threadIdx.x >> 4;  // row group
  const int c = (blockIdx.x * 16 + cq) * 4;
  f32x4 t = {0.f, 0.f, 0.f, 0.f};
  if (c < H) {
    for (int b = rg; b < nb; b += 16) t += *reinterpret_cast<const f32x4*>(part + (size_t)b * H + c);
  }
  red[rg][cq] = t;
  __syncthreads();
  if (rg == 0 && c < H) {
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][cq];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = t[j];
      if (dw_f32) dw_f32[c + j] = accumulate ? dw_f32[c + j] + v : v;
      if (dw_bf16) dw_bf16[c + j] = f2bf(accumulate ? bf2f(dw_bf16[c + j]) + v : v);
    }
  }
}

// Wide-grid variant for H % 16 == 0 (the Llama widths): one block per 16 columns (4 quads) x
// 64 row groups, so H = 4096 launches 256 blocks instead of colsum_kernel's 64 (which left 3 of 4
// CUs idle on a latency-bound 16 MB read). Fixed summation order: bitwise reproducible.
__global__ __launch_bounds__(256) void colsum16_kernel(const float* __restrict__ part, int nb, int H,
                                                       bf16_t* __restrict__ dw_bf16, float* __restrict__ dw_f32,
                                                       int accumulate) {
  __shared__ f32x4 red[64][4];
  __shared__ f32x4 red2[4][4];
  const int cq = threadIdx.x & 3;   // column quad within the block's 16 columns
  const int rg = threadIdx.x >> 2;  // row group (64)
  const int c = blockIdx.x * 16 + cq * 4;
  f32x4 t = {0.f, 0.f, 0.f, 0.f};
  for (int b = rg; b < nb; b += 64) t += *reinterpret_cast<const f32x4*>(part + (size_t)b * H + c);
  red[rg][cq] = t;
  __syncthreads();
  if (rg < 4) {  // 4 x 4 threads: quad cq, partial over row groups rg, rg+4, ..
    f32x4 u = red[rg][cq];
#pragma unroll
    for (int k = rg + 4; k < 64; k += 4) u += red[k][cq];
    red2[rg][cq] = u;
  }
  __syncthreads();
  if (rg == 0) {
    f32x4 v = red2[0][cq] + red2[1][cq] + red2[2][cq] + red2[3][cq];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = v[j];
      if (dw_f32) dw_f32[c + j] = accumulate ? dw_f32[c + j] + x : x;
      if (dw_bf16) dw_bf16[c + j] = f2bf(accumulate ? bf2f(dw_bf16[c + j]) + x : x);
    }
  }
}

RCA_API int rca_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* sum_out, float* rstd,
                            int rows, int H, float eps, hipStream_t stream) {
  if (H % 8 != 0) return -1;
  dim3 block(256), grid((rows + 3) / 4);
  auto X = (const bf16_t*)x;
  auto R = (const bf16_t*)res;
  auto W = (const bf16_t*)w;
  auto Y = (bf16_t*)y;
  auto S = (bf16_t*)sum_out;
  switch (H) {
    case 512: hipLaunchKernelGGL(rmsnorm_fwd_reg<1>, grid, block, 0, stream, X, R, W, Y, S, rstd, rows, H, eps); break;
    case 1024: hipLaunchKernelGGL(rmsnorm_fwd_reg<2>, grid, block, 0, stream, X, R, W, Y, S, rstd, rows, H, eps); break;
    case 2048: hipLaunchKernelGGL(rmsnorm_fwd_reg<4>, grid, block, 0, stream, X, R, W, Y, S, rstd, rows, H, eps); break;
    case 4096: hipLaunchKernelGGL(rmsnorm_fwd_reg<8>, grid, block, 0, stream, X, R, W, Y, S, rstd, rows, H, eps); break;
    case 8192: hipLaunchKernelGGL(rmsnorm_fwd_reg<16>, grid, block, 0, stream, X, R, W, Y, S, rstd, rows, H, eps); break;
    default: hipLaunchKernelGGL(rmsnorm_fwd_generic, grid, block, 0, stream, X, R, W, Y, S, rstd, rows, H, eps);
  }
  return (int)hipGetLastError();
}

// H = 2048 / 4096 take the column-split backward kernel (rmsnorm_bwd_split); the others the
// LDS-slice kernels. dw_part must hold rca_rmsnorm_bwd_blocks(rows, H) * H floats (<= 1024 rows).
static inline bool rmsnorm_bwd_split(int H) { return H == 2048 || H == 4096; }

// Number of workgroups (= rows of the fp32 dw partials buffer) rca_rmsnorm_bwd launches for
// (rows, H): the column-split kernel (H = 2048/4096) runs up to 1024 blocks of 2 row pairs each
// (>= 4 waves/SIMD); the LDS-slice kernels keep 2 blocks/CU resident, so at most 512 blocks of
// >= 16 rows.
RCA_API int rca_rmsnorm_bwd_blocks(int rows, int H) {
  const bool split = rmsnorm_bwd_split(H);
  int nb = split ? (rows + 7) / 8 : (rows + 15) / 16;
  const int cap = split ? 1024 : 512;
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  return nb;
}

RCA_API int rca_rmsnorm_bwd(const void* s, const void* dy, const void* w, const float* rstd, const void* dres, void* dx,
                            float* dw_part, void* dw_bf16, float* dw_f32, int accumulate, int rows, int H,
                            hipStream_t stream) {
  if (H % 8 != 0) return -1;
  // dw_part holds rca_rmsnorm_bwd_blocks(rows, H) rows, one per launched block
  const int nb = rca_rmsnorm_bwd_blocks(rows, H);
  const bool split = rmsnorm_bwd_split(H);  // CPW=4 (H=8192) needs 256 VGPRs: generic
  dim3 block(256), grid(nb);
  const size_t lds = split ? 0 : (size_t)4 * H * sizeof(float);
  if (lds > 160 * 1024) return -2;
  auto S = (const bf16_t*)s;
  auto G = (const bf16_t*)dy;
  auto W = (const bf16_t*)w;
  auto DR = (const bf16_t*)dres;
  auto DX = (bf16_t*)dx;
  switch (H) {
    case 512: hipLaunchKernelGGL(rmsnorm_bwd_reg<1>, grid, block, lds, stream, S, G, W, rstd, DR, DX, dw_part, rows, H); break;
    case 1024: hipLaunchKernelGGL(rmsnorm_bwd_reg<2>, grid, block, lds, stream, S, G, W, rstd, DR, DX, dw_part, rows, H); break;
    case 2048: hipLaunchKernelGGL(rmsnorm_bwd_split<1>, grid, block, 0, stream, S, G, W, rstd, DR, DX, dw_part, rows, H); break;
    case 4096: hipLaunchKernelGGL(rmsnorm_bwd_split<2>, grid, block, 0, stream, S, G, W, rstd, DR, DX, dw_part, rows, H); break;
    // wider rows: the register-cached variant drops to 1-2 waves/SIMD; the two-pass generic
    // kernel (second pass served from L2) keeps 7 waves/SIMD
    default: hipLaunchKernelGGL(rmsnorm_bwd_generic, grid, block, lds, stream, S, G, W, rstd, DR, DX, dw_part, rows, H);
  }
  if (H % 16 == 0)
    hipLaunchKernelGGL(colsum16_kernel, dim3(H / 16), dim3(256), 0, stream, dw_part, nb, H, (bf16_t*)dw_bf16, dw_f32,
                       accumulate);
  else
    hipLaunchKernelGGL(colsum_kernel, dim3((H + 63) / 64), dim3(256), 0, stream, dw_part, nb, H, (bf16_t*)dw_bf16,
                       dw_f32, accumulate);
  return (int)hipGetLastError();
}
