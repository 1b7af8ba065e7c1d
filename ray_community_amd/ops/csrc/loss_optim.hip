// Cross-entropy (fwd/bwd, bf16 logits, large vocab) and the flat-buffer AdamW / grad-norm
// kernels for gfx950.
//
// Cross-entropy: one 512-thread block per token row; a single streaming pass computes the
// online (max, sum-exp) per lane over 16-B vectors, merged across the block through LDS.
// The backward writes dlogits (optionally in place over the logits, saving T*V*2 bytes).
//
// AdamW runs over ONE flat fp32 master buffer (the framework keeps all parameters of a
// group contiguous), so a single launch streams ~28 B/param at HBM rate instead of a
// multi-tensor-apply over thousands of small tensors. Global-norm clipping reads the
// squared norm from device memory: no host synchronisation inside the step (graph-safe).
#include "common.h"

// ----------------------------------------------------------------------------- cross-entropy
__global__ __launch_bounds__(512) void ce_fwd_kernel(const bf16_t* __restrict__ logits, const long long* __restrict__ labels,
                                                     float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                     long long ignore_index) {
  __shared__ float sm[16], ss[16];
  const long long row = blockIdx.x;
  const bf16_t* x = logits + row * (long long)V;
  const int nv = (V & 7) ? 0 : (V >> 3);  // rows are 16-B aligned only when V % 8 == 0
  float m = -INFINITY, s = 0.f;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    float f[8];
    unpack8(__builtin_nontemporal_load(xv + c), f);
    float vm = f[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) vm = fmaxf(vm, f[j]);
    const float mn = fmaxf(m, vm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(f[j] - mn);
    s = s * __expf(m - mn) + acc;
    m = mn;
  }
  for (int c = (nv << 3) + threadIdx.x; c < V; c += blockDim.x) {  // tail (V % 8)
    const float f = bf2f(x[c]);
    const float mn = fmaxf(m, f);
    s = s * __expf(m - mn) + __expf(f - mn);
    m = mn;
  }
  // merge (m, s) across the wave then the block
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = -INFINITY;
    const int nw = blockDim.x >> 6;
    for (int i = 0; i < nw; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < nw; ++i) S += (sm[i] == -INFINITY) ? 0.f : ss[i] * __expf(sm[i] - M);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const long long lab = labels[row];
    loss[row] = (lab == ignore_index || lab < 0 || lab >= V) ? 0.f : lse - bf2f(x[lab]);
  }
}

// dlogits[r, j] = g[r] * (softmax_j - [j == label]); g = grad_loss[r] (or grad_scalar if grad_loss is null)
__global__ __launch_bounds__(512) void ce_bwd_kernel(const bf16_t* __restrict__ logits, const long long* __restrict__ labels,
                                                     const float* __restrict__ lse, const float* __restrict__ grad_loss,
                                                     float grad_scalar, bf16_t* __restrict__ dlogits, int V,
                                                     long long ignore_index) {
  const long long row = blockIdx.x;
  const long long lab = labels[row];
  const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
  const float g = ign ? 0.f : (grad_loss ? grad_loss[row] : grad_scalar);
  const float L = lse[row];
  const bf16_t* x = logits + row * (long long)V;
  bf16_t* dx = dlogits + row * (long long)V;
  const int nv = (V & 7) ? 0 : (V >> 3);  // rows are 16-B aligned only when V % 8 == 0
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  u32x4* dv = reinterpret_cast<u32x4*>(dx);
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    float f[8];
    unpack8(xv[c], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(f[j] - L);
      if ((long long)(c * 8 + j) == lab) p -= 1.f;
      f[j] = g * p;
    }
    dv[c] = pack8(f);
  }
  for (int c = (nv << 3) + threadIdx.x; c < V; c += blockDim.x) {
    float p = __expf(bf2f(x[c]) - L);
    if ((long long)c == lab) p -= 1.f;
    dx[c] = f2bf(g * p);
  }
}

RCA_API int rca_ce_fwd(const void* logits, const long long* labels, float* loss, float* lse, long long T, int V,
                       long long ignore_index, hipStream_t stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ce_fwd_kernel, dim3((unsigned)T), dim3(512), 0, stream, (const bf16_t*)logits, labels, loss, lse, V,
                     ignore_index);
  return (int)hipGetLastError();
}

RCA_API int rca_ce_bwd(const void* logits, const long long* labels, const float* lse, const float* grad_loss,
                       float grad_scalar, void* dlogits, long long T, int V, long long ignore_index, hipStream_t stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)T), dim3(512), 0, stream, (const bf16_t*)logits, labels, lse,
                     grad_loss, grad_scalar, (bf16_t*)dlogits, V, ignore_index);
  return (int)hipGetLastError();
}

// One-pass fused cross-entropy forward + backward for the fused linear-CE path: the row stays
// in VGPRs (NPT 16-B vectors per thread, 1024 threads -> up to 131072 bf16 logits), so HBM sees
// exactly one read and one write of the logits: (max, sum-exp) online per lane, one block
// merge, then dlogits = g * (softmax - onehot) written over the logits. g = gscale[0] (a
// device scalar, e.g. 1 / #valid labels: no host sync) or 0 for ignored rows. The label logit
// is read before the block barrier, i.e. before any thread overwrites the row.
template <int NPT>
__global__ __launch_bounds__(1024) void ce_fused_kernel(bf16_t* __restrict__ logits, const long long* __restrict__ labels,
                                                        const float* __restrict__ gscale, float* __restrict__ loss,
                                                        float* __restrict__ lse_out, int V, long long ignore_index) {
  __shared__ float sm[16], ss[16], bc[2];
  const long long row = blockIdx.x;
  bf16_t* x = logits + row * (long long)V;
  const int nv = V >> 3;
  const long long lab = labels[row];
  const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
  float xlab = 0.f;
  if (threadIdx.x == 0 && !ign) xlab = bf2f(x[lab]);
  u32x4* xv = reinterpret_cast<u32x4*>(x);
  u32x4 r[NPT];
  float m = -INFINITY, s = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c < nv) {
      r[i] = __builtin_nontemporal_load(xv + c);
      float f[8];
      unpack8(r[i], f);
      float vm = f[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) vm = fmaxf(vm, f[j]);
      const float mn = fmaxf(m, vm);
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += __expf(f[j] - mn);
      s = s * __expf(m - mn) + acc;
      m = mn;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = -INFINITY;
    for (int i = 0; i < 16; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < 16; ++i) S += (sm[i] == -INFINITY) ? 0.f : ss[i] * __expf(sm[i] - M);
    const float lse = M + __logf(S);
    bc[0] = lse;
    bc[1] = ign ? 0.f : gscale[0];
    lse_out[row] = lse;
    loss[row] = ign ? 0.f : lse - xlab;
  }
  __syncthreads();
  const float L = bc[0], g = bc[1];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c < nv) {
      float f[8];
      unpack8(r[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(f[j] - L);
        if ((long long)(c * 8 + j) == lab) p -= 1.f;
        f[j] = g * p;
      }
      xv[c] = pack8(f);
    }
  }
}

// Contract: V % 8 == 0, V <= 131072, 16-B aligned rows. Returns -1 when the shape is not covered.
RCA_API int rca_ce_fused(void* logits, const long long* labels, const float* gscale, float* loss, float* lse,
                         long long T, int V, long long ignore_index, hipStream_t stream) {
  if (T <= 0) return 0;
  if ((V & 7) || V <= 0 || ((uintptr_t)logits & 15)) return -1;
  const int nv = V >> 3;
  const int npt = (nv + 1023) / 1024;
#define RCA_CE(N)                                                                                          \
  hipLaunchKernelGGL(ce_fused_kernel<N>, dim3((unsigned)T), dim3(1024), 0, stream, (bf16_t*)logits, labels, gscale, \
                     loss, lse, V, ignore_index);                                                          \
  return (int)hipGetLastError()
  if (npt <= 1) { RCA_CE(1); }
  if (npt <= 2) { RCA_CE(2); }
  if (npt <= 4) { RCA_CE(4); }
  if (npt <= 8) { RCA_CE(8); }
  if (npt <= 16) { RCA_CE(16); }
#undef RCA_CE
  return -1;
}

// ----------------------------------------------------------------------------- grad norm
// partial[b] = sum of squares of this block's grid-stride share; dtype 0 = bf16, 1 = f32.
// The LAST block to finish folds the partials into out[0] itself (last-block-done ticket in
// ticket[0], reset by that block), so there is no second single-workgroup launch: on the grad-norm
// side stream such a launch queued behind the backward GEMMs' full-chip waves for ~200 us each
// (68 per 8B step). Hand-off per cdna_hip_programming.md Guideline 16: every block stores its
// partial, drains it (vmcnt(0)), barrier, one lane releases at agent scope and takes a ticket; the
// block that draws nb-1 acquires at agent scope and sums the partials in index order, so the
// result is bit-identical to the two-launch form and run-to-run deterministic.
template <int DT>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const void* __restrict__ g, long long n, float* __restrict__ partial,
                                                            unsigned* __restrict__ ticket, float* __restrict__ out,
                                                            int accumulate) {
  __shared__ float red[16];
  __shared__ int last;
  float acc = 0.f;
  if (DT == 0) {
    const bf16_t* x = (const bf16_t*)g;
    const long long nv = n >> 3;
    const u32x4* xv = reinterpret_cast<const u32x4*>(x);
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    // four independent 16-B loads in flight per lane (one per iteration left the grid latency-bound
    // at ~2.9 TB/s), four accumulators so the FMAs do not serialise on one register
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (; i + 3 * stride < nv; i += 4 * stride) {
      const u32x4 v0 = __builtin_nontemporal_load(xv + i), v1 = __builtin_nontemporal_load(xv + i + stride);
      const u32x4 v2 = __builtin_nontemporal_load(xv + i + 2 * stride);
      const u32x4 v3 = __builtin_nontemporal_load(xv + i + 3 * stride);
      float f0[8], f1[8], f2[8], f3[8];
      unpack8(v0, f0);
      unpack8(v1, f1);
      unpack8(v2, f2);
      unpack8(v3, f3);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a0 = fmaf(f0[j], f0[j], a0);
        a1 = fmaf(f1[j], f1[j], a1);
        a2 = fmaf(f2[j], f2[j], a2);
        a3 = fmaf(f3[j], f3[j], a3);
      }
    }
    for (; i < nv; i += stride) {
      float f[8];
      unpack8(__builtin_nontemporal_load(xv + i), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) a0 = fmaf(f[j], f[j], a0);
    }
    acc = (a0 + a1) + (a2 + a3);
    for (long long i = (nv << 3) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
      const float f = bf2f(x[i]);
      acc += f * f;
    }
  } else {
    const float* x = (const float*)g;
    const long long nv = n >> 2;
    const f32x4* xv = reinterpret_cast<const f32x4*>(x);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x) {
      const f32x4 f = __builtin_nontemporal_load(xv + i);
      acc += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
    }
    for (long long i = (nv << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
      acc += x[i] * x[i];
  }
  acc = block_sum(acc, red);
  const unsigned nb = gridDim.x;
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = acc;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == nb - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  float s = 0.f;
  for (unsigned i = threadIdx.x; i < nb; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    out[0] = accumulate ? out[0] + s : s;
    // re-arm for the next launch on this workspace (stream order: the next launch starts after
    // this block has exited)
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// out[0] (+)= sum(g^2). partial must hold >= RCA_SUMSQ_WS floats (1024 partials + the ticket word
// at index 1024, zero before the first use; the kernel leaves it zero). Deterministic (no float
// atomics: the partials are combined in index order by the last block).
RCA_API int rca_sumsq(const void* g, long long n, int dtype, float* partial, float* out, int accumulate, hipStream_t stream) {
  long long nb = (n / (dtype == 0 ? 8 : 4) + 255) / 256;
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  unsigned* ticket = reinterpret_cast<unsigned*>(partial + 1024);
  if (dtype == 0)
    hipLaunchKernelGGL(sumsq_partial_kernel<0>, dim3((int)nb), dim3(256), 0, stream, g, n, partial, ticket, out, accumulate);
  else
    hipLaunchKernelGGL(sumsq_partial_kernel<1>, dim3((int)nb), dim3(256), 0, stream, g, n, partial, ticket, out, accumulate);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------- AdamW
struct AdamHP {
  float lr, b1, b2, eps, wd, bc1, bc2, grad_mul, max_norm;
};

// global-norm clip of the (grad_mul-scaled) gradient: coef = min(1, max_norm / ||g * grad_mul||)
__device__ __forceinline__ float clip_coef(const float* sumsq, float max_norm, float grad_mul) {
  if (!sumsq || max_norm <= 0.f) return 1.f;
  const float nrm = sqrtf(sumsq[0]) * fabsf(grad_mul);
  return fminf(1.f, max_norm / (nrm + 1e-6f));
}

// Explicit fmas and no compiler contraction: every kernel that inlines this (flat fp32-master,
// split-master, segmented) rounds identically whatever the surrounding code lets the backend fuse
// (with contraction on, the segmented kernel's larger body fused a different subset of the
// mul/add pairs than the flat kernels and the results differed in the last bit).
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamHP& hp) {
#pragma clang fp contract(off)
  m = __builtin_fmaf(hp.b1, m, (1.f - hp.b1) * g);
  v = __builtin_fmaf(hp.b2, v, ((1.f - hp.b2) * g) * g);
  const float mh = m / hp.bc1;
  const float vh = v / hp.bc2;
  const float u = __builtin_fmaf(hp.wd, p, mh / (sqrtf(vh) + hp.eps));
  p = __builtin_fmaf(-hp.lr, u, p);
}

// GDT: 0 = bf16 grads, 1 = f32 grads. p16 (optional) receives the bf16 copy of the master weights.
template <int GDT>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, bf16_t* __restrict__ p16, const void* __restrict__ grad,
                                                    float* __restrict__ m, float* __restrict__ v, long long n, AdamHP hp,
                                                    const float* __restrict__ sumsq) {
  const float gm = hp.grad_mul * clip_coef(sumsq, hp.max_norm, hp.grad_mul);
  const long long nv = n >> 3;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x) {
    float g[8];
    if (GDT == 0) {
      unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(grad) + i), g);
    } else {
      const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(grad) + 2 * i);
      const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(grad) + 2 * i + 1);
      g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w;
    }
    f32x4* pp = reinterpret_cast<f32x4*>(p) + 2 * i;
    f32x4* mp = reinterpret_cast<f32x4*>(m) + 2 * i;
    f32x4* vp = reinterpret_cast<f32x4*>(v) + 2 * i;
    f32x4 P0 = pp[0], P1 = pp[1], M0 = mp[0], M1 = mp[1], V0 = vp[0], V1 = vp[1];
    float P[8] = {P0.x, P0.y, P0.z, P0.w, P1.x, P1.y, P1.z, P1.w};
    float M[8] = {M0.x, M0.y, M0.z, M0.w, M1.x, M1.y, M1.z, M1.w};
    float Vv[8] = {V0.x, V0.y, V0.z, V0.w, V1.x, V1.y, V1.z, V1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) adam_elem(P[j], M[j], Vv[j], g[j] * gm, hp);
    pp[0] = f32x4{P[0], P[1], P[2], P[3]};
    pp[1] = f32x4{P[4], P[5], P[6], P[7]};
    mp[0] = f32x4{M[0], M[1], M[2], M[3]};
    mp[1] = f32x4{M[4], M[5], M[6], M[7]};
    vp[0] = f32x4{Vv[0], Vv[1], Vv[2], Vv[3]};
    vp[1] = f32x4{Vv[4], Vv[5], Vv[6], Vv[7]};
    if (p16) reinterpret_cast<u32x4*>(p16)[i] = pack8(P);
  }
  // tail
  for (long long i = (nv << 3) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float g = (GDT == 0 ? bf2f(((const bf16_t*)grad)[i]) : ((const float*)grad)[i]) * gm;
    float P = p[i], M = m[i], Vv = v[i];
    adam_elem(P, M, Vv, g, hp);
    p[i] = P;
    m[i] = M;
    v[i] = Vv;
    if (p16) p16[i] = f2bf(P);
  }
}

RCA_API int rca_adamw(float* p, void* p16, const void* grad, int grad_dtype, float* m, float* v, long long n, float lr,
                      float b1, float b2, float eps, float wd, float bc1, float bc2, float grad_mul, const float* sumsq,
                      float max_norm, hipStream_t stream) {
  AdamHP hp{lr, b1, b2, eps, wd, bc1, bc2, grad_mul, max_norm};
  long long nb = ((n >> 3) + 255) / 256;
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  if (grad_dtype == 0)
    hipLaunchKernelGGL(adamw_kernel<0>, dim3((int)nb), dim3(256), 0, stream, p, (bf16_t*)p16, grad, m, v, n, hp, sumsq);
  else
    hipLaunchKernelGGL(adamw_kernel<1>, dim3((int)nb), dim3(256), 0, stream, p, (bf16_t*)p16, grad, m, v, n, hp, sumsq);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------- AdamW, split master
// The fp32 master weight is not stored as such: its upper 16 bits are (almost) the bf16 model
// weight the forward reads anyway, so only the low 16 bits are kept beside it. hi = the fp32 bit
// pattern rounded half-up in magnitude to 16 bits ((M + 0x8000) >> 16: the bf16 model weight,
// equal to the RNE conversion except at exact ties, where it is 1 ulp larger in magnitude), lo =
// M & 0xFFFF. Since hi - upper(M) is 1 exactly when lo >= 0x8000, M = ((hi - (lo >> 15)) << 16) | lo
// reconstructs the master bit-exactly. Per parameter the step streams hi + lo (4 B) instead of
// master + bf16 copy (6 B read, 6 B written): 26 instead of 28 B, and 2 B/param less HBM held.
__device__ __forceinline__ float join_master(unsigned hi, unsigned lo) {
  return __uint_as_float(((hi - (lo >> 15)) << 16) | lo);
}
__device__ __forceinline__ void split_master(float p, unsigned& hi, unsigned& lo) {
  const unsigned M = __float_as_uint(p);
  hi = ((M + 0x8000u) >> 16) & 0xffffu;
  lo = M & 0xffffu;
}

// One 8-element group of the split-master update at element index i8 * 8; returns the new hi
// (bf16 model weight) vector. Shared by the flat and the segmented kernels (bitwise the same math).
template <int GDT>
__device__ __forceinline__ u32x4 adamw_split8(bf16_t* __restrict__ hi16, unsigned short* __restrict__ lo16,
                                              const void* __restrict__ grad, float* __restrict__ m,
                                              float* __restrict__ v, long long i, float gm, const AdamHP& hp) {
  float g[8];
  if (GDT == 0) {
    unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(grad) + i), g);
  } else {
    const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(grad) + 2 * i);
    const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(grad) + 2 * i + 1);
    g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w;
  }
  u32x4* hp4 = reinterpret_cast<u32x4*>(hi16) + i;
  u32x4* lp4 = reinterpret_cast<u32x4*>(lo16) + i;
  f32x4* mp = reinterpret_cast<f32x4*>(m) + 2 * i;
  f32x4* vp = reinterpret_cast<f32x4*>(v) + 2 * i;
  // state streams use the default cache policy (measured: non-temporal loads/stores of the
  // read-modify-write state ran the 8B step at 3.7 TB/s vs 5.7 TB/s)
  const u32x4 H = hp4[0], L = lp4[0];
  const f32x4 M0 = mp[0], M1 = mp[1];
  const f32x4 V0 = vp[0], V1 = vp[1];
  float P[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    P[2 * k] = join_master(H[k] & 0xffffu, L[k] & 0xffffu);
    P[2 * k + 1] = join_master(H[k] >> 16, L[k] >> 16);
  }
  float Mv[8] = {M0.x, M0.y, M0.z, M0.w, M1.x, M1.y, M1.z, M1.w};
  float Vv[8] = {V0.x, V0.y, V0.z, V0.w, V1.x, V1.y, V1.z, V1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) adam_elem(P[j], Mv[j], Vv[j], g[j] * gm, hp);
  u32x4 Ho, Lo;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    unsigned h0, l0, h1, l1;
    split_master(P[2 * k], h0, l0);
    split_master(P[2 * k + 1], h1, l1);
    Ho[k] = h0 | (h1 << 16);
    Lo[k] = l0 | (l1 << 16);
  }
  hp4[0] = Ho;
  lp4[0] = Lo;
  mp[0] = f32x4{Mv[0], Mv[1], Mv[2], Mv[3]};
  mp[1] = f32x4{Mv[4], Mv[5], Mv[6], Mv[7]};
  vp[0] = f32x4{Vv[0], Vv[1], Vv[2], Vv[3]};
  vp[1] = f32x4{Vv[4], Vv[5], Vv[6], Vv[7]};
  return Ho;
}

template <int GDT>
__device__ __forceinline__ void adamw_split1(bf16_t* __restrict__ hi16, unsigned short* __restrict__ lo16,
                                             const void* __restrict__ grad, float* __restrict__ m,
                                             float* __restrict__ v, long long i, float gm, const AdamHP& hp) {
  const float g = (GDT == 0 ? bf2f(((const bf16_t*)grad)[i]) : ((const float*)grad)[i]) * gm;
  float P = join_master(hi16[i], lo16[i]), Mv = m[i], Vv = v[i];
  adam_elem(P, Mv, Vv, g, hp);
  unsigned h, l;
  split_master(P, h, l);
  hi16[i] = (bf16_t)h;
  lo16[i] = (unsigned short)l;
  m[i] = Mv;
  v[i] = Vv;
}

template <int GDT>
__global__ __launch_bounds__(256) void adamw_split_kernel(bf16_t* __restrict__ hi16, unsigned short* __restrict__ lo16,
                                                          const void* __restrict__ grad, float* __restrict__ m,
                                                          float* __restrict__ v, long long n, AdamHP hp,
                                                          const float* __restrict__ sumsq) {
  const float gm = hp.grad_mul * clip_coef(sumsq, hp.max_norm, hp.grad_mul);
  const long long nv = n >> 3;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x)
    adamw_split8<GDT>(hi16, lo16, grad, m, v, i, gm, hp);
  for (long long i = (nv << 3) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    adamw_split1<GDT>(hi16, lo16, grad, m, v, i, gm, hp);
}

// Segmented split-master AdamW that also refreshes the transposed bf16 copy W^T [C][R] of every
// matrix segment W [R][C] (the reduction-contiguous operand of the backward dgrad GEMM,
// parallel/fused_linear.py): the new bf16 weights are in registers anyway, so W^T costs one extra
// 2-B write per parameter instead of a separate read + write transpose pass in the backward.
// Segment descriptor (8 x int64, sorted by first tile): {off, n, first tile, W^T pointer (0 =
// plain 1-D range), R, C, decay, 0}. Matrix tiles are 128 x 128 (256-B row pieces on every stream
// and on W^T; a 64 x 64 tiling measured 41 ms vs the flat kernel's 37 ms on the 8B layout): lane
// (ch = t & 15, rp = t >> 4) updates rows 2rp + 32k, 2rp + 1 + 32k (k < 4) x columns 8ch..8ch+7,
// pairs each row pair's new bf16 values into dwords (v_perm) in an LDS image X[j][q] (128 output
// rows x 64 dwords, q XOR-swizzled by 2*(j/8): the 32 lanes of a ds_write_b32 group hit 32 banks)
// and stores W^T with one ds_read_b128 (dword pairs swapped back when j/8 is odd) + one 16-B store
// per 8 outputs. 1-D tiles update 4096 consecutive elements.
template <int GDT>
__global__ __launch_bounds__(256) void adamw_split_seg_kernel(bf16_t* __restrict__ hi16, unsigned short* __restrict__ lo16,
                                                              const void* __restrict__ grad, float* __restrict__ m,
                                                              float* __restrict__ v, const long long* __restrict__ segs,
                                                              int nseg, long long ntiles, AdamHP hp,
                                                              const float* __restrict__ sumsq) {
  __shared__ u32x4 X4[128 * 64 / 4];
  unsigned* X = reinterpret_cast<unsigned*>(X4);
  const float clip = clip_coef(sumsq, hp.max_norm, hp.grad_mul);
  const int t = threadIdx.x;
  // Tiles are walked grid-stride (as the flat kernel's 8-element groups): a block's tiles only
  // move forward, so its segment is found by a forward scan from the previous one (wave-uniform
  // scalar loads), not a search per tile.
  int sgi = 0;
  for (long long b = blockIdx.x; b < ntiles; b += gridDim.x) {
    while (sgi + 1 < nseg && segs[(sgi + 1) * 8 + 2] <= b) ++sgi;
    const long long* sg = segs + sgi * 8;
    const long long off = sg[0], n = sg[1], tile = b - sg[2];
    bf16_t* wt = reinterpret_cast<bf16_t*>(sg[3]);
    AdamHP h = hp;
    if (!sg[6]) h.wd = 0.f;
    const float gm = h.grad_mul * clip;
    if (!wt) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const long long e = tile * 4096 + (k * 256 + t) * 8;
        if (e + 8 <= n) {
          adamw_split8<GDT>(hi16, lo16, grad, m, v, (off + e) >> 3, gm, h);
        } else {
          for (long long j = e; j < n && j < e + 8; ++j) adamw_split1<GDT>(hi16, lo16, grad, m, v, off + j, gm, h);
        }
      }
      continue;
    }
    const int R = (int)sg[4], C = (int)sg[5], tilesC = C >> 7;
    const int r0 = (int)(tile / tilesC) << 7, c0 = (int)(tile % tilesC) << 7;
    const int ch = t & 15, rp = t >> 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long e0 = off + (long long)(r0 + 2 * rp + 32 * k) * C + c0 + ch * 8;
      const u32x4 Ha = adamw_split8<GDT>(hi16, lo16, grad, m, v, e0 >> 3, gm, h);
      const u32x4 Hb = adamw_split8<GDT>(hi16, lo16, grad, m, v, (e0 + C) >> 3, gm, h);
      const int q = (rp + 16 * k) ^ (2 * ch);
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        X[(ch * 8 + 2 * mm) * 64 + q] = __builtin_amdgcn_perm(Hb[mm], Ha[mm], 0x05040100u);
        X[(ch * 8 + 2 * mm + 1) * 64 + q] = __builtin_amdgcn_perm(Hb[mm], Ha[mm], 0x07060302u);
      }
    }
    __syncthreads();
    const int q4 = (t & 15) * 4;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int j = (t >> 4) + 16 * p;
      const int sw = 2 * (j >> 3);
      u32x4 o = X4[(j * 64 + (q4 ^ (sw & ~3))) >> 2];
      if (sw & 2) o = u32x4{o[2], o[3], o[0], o[1]};
      *reinterpret_cast<u32x4*>(wt + (long)(c0 + j) * R + r0 + q4 * 2) = o;
    }
    __syncthreads();  // X is rewritten by this block's next matrix tile
  }
}

static long long g_adamw_split_blocks = 4096;
RCA_API void rca_adamw_split_set_blocks(long long nb) { g_adamw_split_blocks = nb > 0 ? nb : 4096; }

// hi16: the bf16 model weights (in/out), lo16: low halves of the fp32 master bit patterns (in/out).
// Contract: hi16, lo16, grad, m, v 16-B aligned when n >= 8.
RCA_API int rca_adamw_split(void* hi16, void* lo16, const void* grad, int grad_dtype, float* m, float* v, long long n,
                            float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, float grad_mul,
                            const float* sumsq, float max_norm, hipStream_t stream) {
  if (n <= 0) return 0;
  if ((((uintptr_t)hi16 | (uintptr_t)lo16 | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) & 15) && n >= 8) return -1;
  AdamHP hp{lr, b1, b2, eps, wd, bc1, bc2, grad_mul, max_norm};
  long long nb = ((n >> 3) + 255) / 256;
  if (nb > g_adamw_split_blocks) nb = g_adamw_split_blocks;
  if (nb < 1) nb = 1;
  if (grad_dtype == 0)
    hipLaunchKernelGGL(adamw_split_kernel<0>, dim3((int)nb), dim3(256), 0, stream, (bf16_t*)hi16,
                       (unsigned short*)lo16, grad, m, v, n, hp, sumsq);
  else
    hipLaunchKernelGGL(adamw_split_kernel<1>, dim3((int)nb), dim3(256), 0, stream, (bf16_t*)hi16,
                       (unsigned short*)lo16, grad, m, v, n, hp, sumsq);
  return (int)hipGetLastError();
}

// Segmented launch (adamw_split_seg_kernel): segs = device int64 [nseg][8] as documented there,
// nblocks = the last segment's first tile + its tile count (tiles are walked grid-stride by
// min(nblocks, rca_adamw_split_set_blocks) workgroups). Contract: 16-B aligned buffers,
// every segment offset a multiple of 8 elements, matrix R and C multiples of 64.
RCA_API int rca_adamw_split_seg(void* hi16, void* lo16, const void* grad, int grad_dtype, float* m, float* v,
                                const void* segs, int nseg, long long nblocks, float lr, float b1, float b2, float eps,
                                float wd, float bc1, float bc2, float grad_mul, const float* sumsq, float max_norm,
                                hipStream_t stream) {
  if (nseg <= 0 || nblocks <= 0) return 0;
  if (nblocks >= (1LL << 31)) return -2;
  if (((uintptr_t)hi16 | (uintptr_t)lo16 | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  AdamHP hp{lr, b1, b2, eps, wd, bc1, bc2, grad_mul, max_norm};
  // 16384 workgroups: 39.7 ms vs 40.3 at 4096 on the 8B layout (scripts/adamw_seg_bench.py); an
  // explicit rca_adamw_split_set_blocks value applies to both split kernels
  const long long cap = g_adamw_split_blocks == 4096 ? 16384 : g_adamw_split_blocks;
  const unsigned grid = (unsigned)(nblocks < cap ? nblocks : cap);
  if (grad_dtype == 0)
    hipLaunchKernelGGL(adamw_split_seg_kernel<0>, dim3(grid), dim3(256), 0, stream, (bf16_t*)hi16,
                       (unsigned short*)lo16, grad, m, v, (const long long*)segs, nseg, nblocks, hp, sumsq);
  else
    hipLaunchKernelGGL(adamw_split_seg_kernel<1>, dim3(grid), dim3(256), 0, stream, (bf16_t*)hi16,
                       (unsigned short*)lo16, grad, m, v, (const long long*)segs, nseg, nblocks, hp, sumsq);
  return (int)hipGetLastError();
}
