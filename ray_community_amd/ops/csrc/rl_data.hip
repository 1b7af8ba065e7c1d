// RLlib and Ray-Data hot ops on gfx950:
//   * GAE (generalised advantage estimation) as a reverse linear-recurrence scan:
//       delta_t = r_t + gamma * (1 - term_t) * nextV_t - V_t
//       A_t     = delta_t + gamma * lambda * (1 - done_t) * A_{t+1}
//     One wave per trajectory row [B, T]; each lane owns a contiguous chunk of T/64 steps,
//     composes its chunk's affine map (A_in -> a + b * A_in), the 64 maps are combined with a
//     reverse wave scan (shuffles), then every lane re-walks its chunk with its carry-in.
//     Work is O(T) per row with a 64-wide critical path of T/64 + log2(64).
//   * advantage standardisation (deterministic two-stage mean / var + in-place normalise)
//   * batched concat: K device buffers -> one buffer in a single launch (SampleBatch.concat)
//   * uint8 HWC image -> normalised bf16/f32 CHW (Data map_batches GPU preprocessing)
#include "common.h"

__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ next_val, const float* __restrict__ last_val,
                                                  const unsigned char* __restrict__ term, const unsigned char* __restrict__ done,
                                                  float* __restrict__ adv, float* __restrict__ tgt, int B, int T, float gamma,
                                                  float lam, float* __restrict__ partial) {
  __shared__ float red[16];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  float s1 = 0.f, s2 = 0.f;
  if (row < B) {
    const long long base = (long long)row * T;
    const int chunk = (T + 63) / 64;
    const int t0 = lane * chunk;
    const int t1 = min(T, t0 + chunk);
    // pass 1: affine map of this chunk, applied right-to-left: A_{t0} = a + b * A_{t1}
    float a = 0.f, b = 1.f;
    for (int t = t1 - 1; t >= t0; --t) {
      const float nv = next_val ? next_val[base + t] : (t + 1 < T ? val[base + t + 1] : (last_val ? last_val[row] : 0.f));
      const float d = rew[base + t] + gamma * (term[base + t] ? 0.f : nv) - val[base + t];
      const float c = gamma * lam * (done[base + t] ? 0.f : 1.f);
      a = d + c * a;
      b = c * b;
    }
    // reverse inclusive scan over lanes: carry into lane L = composition of lanes > L applied to 0
    // compose (a_l, b_l) o (a_r, b_r) = (a_l + b_l * a_r, b_l * b_r), r = lane to the right (later time)
    float ca = a, cb = b;  // inclusive: maps lanes [lane .. 63]
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float ra = __shfl_down(ca, off, 64), rb = __shfl_down(cb, off, 64);
      if (lane + off < 64) {
        ca = ca + cb * ra;
        cb = cb * rb;
      }
    }
    // carry-in for this lane = A at t1 = inclusive value of lane+1 (applied to A_T = 0)
    float carry = __shfl_down(ca, 1, 64);
    if (lane == 63) carry = 0.f;
    // pass 2: re-walk the chunk with the carry
    float A = carry;
    for (int t = t1 - 1; t >= t0; --t) {
      const float nv = next_val ? next_val[base + t] : (t + 1 < T ? val[base + t + 1] : (last_val ? last_val[row] : 0.f));
      const float d = rew[base + t] + gamma * (term[base + t] ? 0.f : nv) - val[base + t];
      const float c = gamma * lam * (done[base + t] ? 0.f : 1.f);
      A = d + c * A;
      adv[base + t] = A;
      if (tgt) tgt[base + t] = A + val[base + t];
      s1 += A;
      s2 += A * A;
    }
  }
  if (partial) {
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) {
      partial[2 * blockIdx.x] = s1;
      partial[2 * blockIdx.x + 1] = s2;
    }
  }
}

// ----------------------------------------------------------------------------- V-trace
// IMPALA off-policy targets (Espeholt et al. 2018; reference: rllib/algorithms/impala/vtrace_torch.py)
// on env-major [B, T] fragments, one wave per trajectory. acc_t = vs_t - V_t obeys the same affine
// right-to-left recurrence as GAE (acc_t = delta_t + k_t * acc_{t+1}), so the wave splits the row
// into 64 chunks, scans the chunk maps across lanes and re-walks each chunk with its carry.
//   rho_t = min(rho_bar, e^{logr_t}), c_t = min(c_bar, e^{logr_t}), disc_t = gamma * (1 - term_t)
//   delta_t = rho_t (r_t + disc_t V'_t - V_t),  k_t = gamma c_t (1 - done_t)
//   pg_t = min(pg_bar, e^{logr_t}) (r_t + disc_t vs'_t - V_t)
// with V'_t = next_val[t] (value of s_{t+1}; exact at truncations) and vs'_t = vs_{t+1} inside an
// episode, V'_t at a cut or at the fragment end.
__global__ __launch_bounds__(256) void vtrace_kernel(const float* __restrict__ logr, const float* __restrict__ rew,
                                                     const float* __restrict__ val, const float* __restrict__ nval,
                                                     const unsigned char* __restrict__ term,
                                                     const unsigned char* __restrict__ done, float* __restrict__ vs,
                                                     float* __restrict__ pg, int B, int T, float gamma, float rho_bar,
                                                     float c_bar, float pg_bar) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= B) return;
  const long long base = (long long)row * T;
  const int chunk = (T + 63) / 64;
  const int t0 = lane * chunk;
  const int t1 = min(T, t0 + chunk);
  float a = 0.f, b = 1.f;
  for (int t = t1 - 1; t >= t0; --t) {
    const float ir = __expf(logr[base + t]);
    const float disc = term[base + t] ? 0.f : gamma;
    const float d = fminf(rho_bar, ir) * (rew[base + t] + disc * nval[base + t] - val[base + t]);
    const float k = done[base + t] ? 0.f : gamma * fminf(c_bar, ir);
    a = d + k * a;
    b = k * b;
  }
  float ca = a, cb = b;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float ra = __shfl_down(ca, off, 64), rb = __shfl_down(cb, off, 64);
    if (lane + off < 64) {
      ca = ca + cb * ra;
      cb = cb * rb;
    }
  }
  float A = __shfl_down(ca, 1, 64);
  if (lane == 63) A = 0.f;
  for (int t = t1 - 1; t >= t0; --t) {
    const float ir = __expf(logr[base + t]);
    const float disc = term[base + t] ? 0.f : gamma;
    const bool cut = done[base + t] || t + 1 >= T;
    const float vs_next = cut ? nval[base + t] : val[base + t + 1] + A;
    const float r = rew[base + t], v = val[base + t];
    const float d = fminf(rho_bar, ir) * (r + disc * nval[base + t] - v);
    const float k = done[base + t] ? 0.f : gamma * fminf(c_bar, ir);
    A = d + k * A;
    vs[base + t] = v + A;
    pg[base + t] = fminf(pg_bar, ir) * (r + disc * vs_next - v);
  }
}

RCA_API int rca_vtrace(const float* logr, const float* rew, const float* val, const float* nval,
                       const unsigned char* term, const unsigned char* done, float* vs, float* pg, int B, int T,
                       float gamma, float rho_bar, float c_bar, float pg_bar, hipStream_t stream) {
  hipLaunchKernelGGL(vtrace_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, logr, rew, val, nval, term, done, vs, pg, B,
                     T, gamma, rho_bar, c_bar, pg_bar);
  return (int)hipGetLastError();
}

// stats[0] = mean, stats[1] = 1 / (std + eps)   (population std, as numpy.std)
__global__ __launch_bounds__(256) void finalize_stats_kernel(const float* __restrict__ partial, int nb, long long n, float eps,
                                                             float* __restrict__ stats) {
  __shared__ float red[16];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    a += partial[2 * i];
    b += partial[2 * i + 1];
  }
  a = block_sum(a, red);
  b = block_sum(b, red);
  if (threadIdx.x == 0) {
    const float mean = a / (float)n;
    const float var = fmaxf(b / (float)n - mean * mean, 0.f);
    stats[0] = mean;
    stats[1] = 1.f / (sqrtf(var) + eps);
  }
}

__global__ __launch_bounds__(256) void moments_partial_kernel(const float* __restrict__ x, long long n, float* __restrict__ partial) {
  __shared__ float red[16];
  float a = 0.f, b = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    a += v;
    b += v * v;
  }
  a = block_sum(a, red);
  b = block_sum(b, red);
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
}

__global__ __launch_bounds__(256) void standardize_kernel(float* __restrict__ x, long long n, const float* __restrict__ stats) {
  const float mean = stats[0], inv = stats[1];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] = (x[i] - mean) * inv;
}

// partial must hold 2 * ceil(B/4) floats when standardize != 0; stats 2 floats.
RCA_API int rca_gae(const float* rew, const float* val, const float* next_val, const float* last_val,
                    const unsigned char* term, const unsigned char* done, float* adv, float* tgt, int B, int T, float gamma,
                    float lam, int standardize, float* partial, float* stats, float eps, hipStream_t stream) {
  const int nb = (B + 3) / 4;
  hipLaunchKernelGGL(gae_kernel, dim3(nb), dim3(256), 0, stream, rew, val, next_val, last_val, term, done, adv, tgt, B, T,
                     gamma, lam, standardize ? partial : (float*)nullptr);
  if (standardize) {
    const long long n = (long long)B * T;
    hipLaunchKernelGGL(finalize_stats_kernel, dim3(1), dim3(256), 0, stream, partial, nb, n, eps, stats);
    long long g = (n + 255) / 256;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(standardize_kernel, dim3((int)g), dim3(256), 0, stream, adv, n, stats);
  }
  return (int)hipGetLastError();
}

// standalone standardisation; partial must hold 2 * 1024 floats
RCA_API int rca_standardize(float* x, long long n, float* partial, float* stats, float eps, hipStream_t stream) {
  long long g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(moments_partial_kernel, dim3((int)g), dim3(256), 0, stream, x, n, partial);
  hipLaunchKernelGGL(finalize_stats_kernel, dim3(1), dim3(256), 0, stream, partial, (int)g, n, eps, stats);
  hipLaunchKernelGGL(standardize_kernel, dim3((int)g), dim3(256), 0, stream, x, n, stats);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------- batched concat
struct CopyDesc {
  const unsigned char* src;
  long long dst_off;
  long long nbytes;
};

// blockIdx.y = segment; each block copies 16 B per lane with a grid stride over the segment.
__global__ __launch_bounds__(256) void batched_copy_kernel(const CopyDesc* __restrict__ descs, unsigned char* __restrict__ dst) {
  const CopyDesc d = descs[blockIdx.y];
  unsigned char* out = dst + d.dst_off;
  const bool aligned = ((((uintptr_t)d.src) | ((uintptr_t)out)) & 15) == 0;
  long long nvec = aligned ? (d.nbytes >> 4) : 0;
  const u32x4* s4 = reinterpret_cast<const u32x4*>(d.src);
  u32x4* o4 = reinterpret_cast<u32x4*>(out);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (long long)gridDim.x * blockDim.x)
    o4[i] = __builtin_nontemporal_load(s4 + i);
  for (long long i = (nvec << 4) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < d.nbytes;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = d.src[i];
}

// descs: device array of K CopyDesc (src pointer, dst byte offset, byte count)
RCA_API int rca_batched_copy(const void* descs, int K, void* dst, long long max_bytes, hipStream_t stream) {
  if (K <= 0) return 0;
  long long gx = (max_bytes / 16 + 255) / 256;
  if (gx > 256) gx = 256;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(batched_copy_kernel, dim3((int)gx, K), dim3(256), 0, stream, (const CopyDesc*)descs,
                     (unsigned char*)dst);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------- image preprocess
// in: uint8 [N, H, W, C] (HWC), out: [N, C, H, W] with out = (in / 255 - mean[c]) * inv_std[c]
// out_dtype 0 = bf16, 1 = f32. One thread per (n, h, w) pixel; C <= 4.
__global__ __launch_bounds__(256) void img_norm_kernel(const unsigned char* __restrict__ in, void* __restrict__ out, long long npix,
                                                       int HW, int C, float m0, float m1, float m2, float m3, float s0, float s1,
                                                       float s2, float s3, int out_dtype) {
  const float mean[4] = {m0, m1, m2, m3};
  const float inv[4] = {s0, s1, s2, s3};
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
    const long long n = p / HW;
    const int hw = (int)(p - n * HW);
    for (int c = 0; c < C; ++c) {
      const float v = ((float)in[p * C + c] * (1.f / 255.f) - mean[c]) * inv[c];
      const long long o = (n * C + c) * (long long)HW + hw;
      if (out_dtype == 0)
        ((bf16_t*)out)[o] = f2bf(v);
      else
        ((float*)out)[o] = v;
    }
  }
}

// channels_last output: out is [N, H, W, C] in memory, i.e. the input's element order, so the op is a
// pure elementwise stream: each thread converts 16 consecutive bytes (one 16-B load) into 16 outputs
// (two 16-B bf16 stores); the channel of element i is i % C.
__global__ __launch_bounds__(256) void img_norm_nhwc_kernel(const unsigned char* __restrict__ in, void* __restrict__ out,
                                                            long long n, int C, float m0, float m1, float m2, float m3,
                                                            float s0, float s1, float s2, float s3, int out_dtype) {
  const float mean[4] = {m0, m1, m2, m3};
  const float inv[4] = {s0, s1, s2, s3};
  const long long nvec = n / 16;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (long long)gridDim.x * blockDim.x) {
    const uint4 raw = reinterpret_cast<const uint4*>(in)[v];
    const unsigned int w[4] = {raw.x, raw.y, raw.z, raw.w};
    int c = (int)((v * 16) % C);
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float b = (float)((w[j >> 2] >> ((j & 3) * 8)) & 0xffu);
      f[j] = (b * (1.f / 255.f) - mean[c]) * inv[c];
      c = (c + 1 == C) ? 0 : c + 1;
    }
    if (out_dtype == 0) {
      uint4 o[2];
      unsigned int* ow = reinterpret_cast<unsigned int*>(o);
#pragma unroll
      for (int j = 0; j < 8; ++j) ow[j] = (unsigned int)f2bf(f[2 * j]) | ((unsigned int)f2bf(f[2 * j + 1]) << 16);
      reinterpret_cast<uint4*>(out)[2 * v] = o[0];
      reinterpret_cast<uint4*>(out)[2 * v + 1] = o[1];
    } else {
      float4* of = reinterpret_cast<float4*>(out) + 4 * v;
#pragma unroll
      for (int j = 0; j < 4; ++j) of[j] = make_float4(f[4 * j], f[4 * j + 1], f[4 * j + 2], f[4 * j + 3]);
    }
  }
  // tail (n % 16 elements), one block
  if (blockIdx.x == 0) {
    for (long long i = nvec * 16 + threadIdx.x; i < n; i += blockDim.x) {
      const int c = (int)(i % C);
      const float val = ((float)in[i] * (1.f / 255.f) - mean[c]) * inv[c];
      if (out_dtype == 0)
        ((bf16_t*)out)[i] = f2bf(val);
      else
        ((float*)out)[i] = val;
    }
  }
}

RCA_API int rca_image_normalize(const void* in, void* out, long long N, int H, int W, int C, const float* mean,
                                const float* stdv, int out_dtype, int channels_last, hipStream_t stream) {
  if (C < 1 || C > 4) return -1;
  float m[4] = {0, 0, 0, 0}, s[4] = {1, 1, 1, 1};
  for (int c = 0; c < C; ++c) {
    m[c] = mean[c];
    s[c] = 1.f / stdv[c];
  }
  const long long npix = N * H * W;
  if (channels_last) {
    const long long n = npix * C;
    long long gv = (n / 16 + 255) / 256;
    if (gv > 8192) gv = 8192;
    if (gv < 1) gv = 1;
    hipLaunchKernelGGL(img_norm_nhwc_kernel, dim3((int)gv), dim3(256), 0, stream, (const unsigned char*)in, out, n, C, m[0], m[1],
                       m[2], m[3], s[0], s[1], s[2], s[3], out_dtype);
    return (int)hipGetLastError();
  }
  long long g = (npix + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(img_norm_kernel, dim3((int)g), dim3(256), 0, stream, (const unsigned char*)in, out, npix, H * W, C, m[0],
                     m[1], m[2], m[3], s[0], s[1], s[2], s[3], out_dtype);
  return (int)hipGetLastError();
}
