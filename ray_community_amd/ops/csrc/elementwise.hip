// Memory-bound fused elementwise kernels for the Llama training step on gfx950:
//   * SwiGLU fwd/bwd on the fused gate|up projection output
//   * RoPE fwd/bwd (rotate-half convention) applied in place on the fused qkv projection output
// All accesses are 16 B per lane (8 x bf16). Grids are capped at 256 CUs x 8 blocks and
// grid-stride the remainder (cdna_hip_programming.md Guideline 11).
#include "common.h"
#include <stdlib.h>

static inline int grid_for(long long nvec, int block) {
  long long g = (nvec + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// gu: [T, 2F] (gate = gu[:, :F], up = gu[:, F:]), out: [T, F]
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                                         long long T, int F) {
  const int fv = F >> 3;
  const long long n = T * fv;
  // 32-bit index math (host guarantees n < 2^31): 64-bit division is emulated on CDNA
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)n; i += gridDim.x * blockDim.x) {
    const long long t = i / (unsigned)fv;
    const int c = (int)(i - (unsigned)t * fv);
    const u32x4* row = reinterpret_cast<const u32x4*>(gu + t * 2 * (long long)F);
    float g[8], u[8], o[8];
    unpack8(__builtin_nontemporal_load(row + c), g);
    unpack8(__builtin_nontemporal_load(row + fv + c), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(silu_f(g[j]))) * u[j];
    reinterpret_cast<u32x4*>(out + t * (long long)F)[c] = pack8(o);
  }
}

// dgu[:, :F] = dout * up * dsilu(gate); dgu[:, F:] = dout * silu(gate)
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dout,
                                                         bf16_t* __restrict__ dgu, long long T, int F) {
  const int fv = F >> 3;
  const long long n = T * fv;
  // 32-bit index math (host guarantees n < 2^31): 64-bit division is emulated on CDNA
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)n; i += gridDim.x * blockDim.x) {
    const long long t = i / (unsigned)fv;
    const int c = (int)(i - (unsigned)t * fv);
    const u32x4* row = reinterpret_cast<const u32x4*>(gu + t * 2 * (long long)F);
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(row[c], g);
    unpack8(row[fv + c], u);
    unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dout + t * (long long)F) + c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-g[j]));
      const float si = g[j] * sg;
      du[j] = d[j] * bf2f(f2bf(si));
      dg[j] = d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    u32x4* orow = reinterpret_cast<u32x4*>(dgu + t * 2 * (long long)F);
    orow[c] = pack8(dg);
    orow[fv + c] = pack8(du);
  }
}

// ---------------------------------------------------------------------------------------------
// SwiGLU with a transposed copy of its output(s) for the backward weight GEMMs (the wgrad of the
// next linear needs its input reduction-contiguous: [F, T]). One 64 (tokens) x 64 (features)
// tile per workgroup: the row-major result is stored directly, the tile is staged through LDS
// (rows padded to 66 elements: conflict-free column gathers, as transpose_bf16_kernel) and
// stored again transposed -- the transposed copy costs one extra write instead of a separate
// read + write transpose pass.
__device__ __forceinline__ void tile_put8(unsigned* tile32, int row, int col8, const float* v) {
  constexpr int TP = 66;
  unsigned* dst = tile32 + (row * TP + col8) / 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) dst[i] = (unsigned)f2bf(v[2 * i]) | ((unsigned)f2bf(v[2 * i + 1]) << 16);
}

// out_t[c0 + c][r0 .. r0+63] <- tile column c (64 rows), 8 rows per lane-chunk
__device__ __forceinline__ void tile_store_t(const unsigned* tile32, bf16_t* out_t, long ldt, int r0, int c0, int t) {
  constexpr int TP = 66;
  const bf16_t* tile = reinterpret_cast<const bf16_t*>(tile32);
  const int ch = t & 7, rr = t >> 3;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = rr + 32 * p;
    u32x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (unsigned)tile[(ch * 8 + 2 * i) * TP + c] | ((unsigned)tile[(ch * 8 + 2 * i + 1) * TP + c] << 16);
    *reinterpret_cast<u32x4*>(out_t + (long)(c0 + c) * ldt + r0 + ch * 8) = o;
  }
}

__global__ __launch_bounds__(256) void swiglu_fwd_tr_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                                            bf16_t* __restrict__ out_t, int T, int F) {
  __shared__ unsigned tile32[64 * 66 / 2];
  const int tilesF = F >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (bid / tilesF) << 6, c0 = (bid % tilesF) << 6;
  const int t = threadIdx.x, ch = t & 7, rr = t >> 3;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = rr + 32 * p;
    const bf16_t* row = gu + (long)(r0 + r) * 2 * F;
    float g[8], u[8], o[8];
    unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + c0 + ch * 8)), g);
    unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + F + c0 + ch * 8)), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(silu_f(g[j]))) * u[j];
    *reinterpret_cast<u32x4*>(out + (long)(r0 + r) * F + c0 + ch * 8) = pack8(o);
    tile_put8(tile32, r, ch * 8, o);
  }
  __syncthreads();
  tile_store_t(tile32, out_t, T, r0, c0, t);
}

__global__ __launch_bounds__(256) void swiglu_bwd_tr_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dout,
                                                            bf16_t* __restrict__ dgu, bf16_t* __restrict__ dgu_t, int T,
                                                            int F) {
  __shared__ unsigned tg[64 * 66 / 2], tu[64 * 66 / 2];
  const int tilesF = F >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (bid / tilesF) << 6, c0 = (bid % tilesF) << 6;
  const int t = threadIdx.x, ch = t & 7, rr = t >> 3;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = rr + 32 * p;
    const bf16_t* row = gu + (long)(r0 + r) * 2 * F;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(*reinterpret_cast<const u32x4*>(row + c0 + ch * 8), g);
    unpack8(*reinterpret_cast<const u32x4*>(row + F + c0 + ch * 8), u);
    unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(dout + (long)(r0 + r) * F + c0 + ch * 8)), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-g[j]));
      const float si = g[j] * sg;
      du[j] = d[j] * bf2f(f2bf(si));
      dg[j] = d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    bf16_t* orow = dgu + (long)(r0 + r) * 2 * F;
    *reinterpret_cast<u32x4*>(orow + c0 + ch * 8) = pack8(dg);
    *reinterpret_cast<u32x4*>(orow + F + c0 + ch * 8) = pack8(du);
    tile_put8(tg, r, ch * 8, dg);
    tile_put8(tu, r, ch * 8, du);
  }
  __syncthreads();
  tile_store_t(tg, dgu_t, T, r0, c0, t);      // rows [0, F) of dgu^T: the gate half
  tile_store_t(tu, dgu_t, T, r0, F + c0, t);  // rows [F, 2F): the up half
}

// RoPE in place on the first (Hq + Hk) heads of each row of qkv: [T, (Hq + 2*Hk) * D].
// Token t has position pos[t] if pos != nullptr else (t % S). cs: [max_pos, D/2] float2 (cos, sin).
// sign = +1 forward, -1 backward (rotation by -theta is the adjoint).
// One thread handles 8 rotation pairs: x[i..i+7] and x[i+D/2..i+D/2+7].
__global__ __launch_bounds__(256) void rope_kernel(bf16_t* __restrict__ qkv, const float2* __restrict__ cs,
                                                   const int* __restrict__ pos, long long T, int S, int nheads_rot,
                                                   int row_stride, int D, float sign) {
  const int half = D >> 1;
  const int per_head = half >> 3;  // threads per head
  const long long per_row = (long long)nheads_rot * per_head;
  const long long n = T * per_row;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)n; i += gridDim.x * blockDim.x) {
    const long long t = i / (unsigned)per_row;
    const int r = (int)(i - (unsigned)t * (unsigned)per_row);
    const int h = r / per_head;
    const int c = (r - h * per_head) << 3;  // first pair index
    const int p = pos ? pos[t] : (int)((unsigned)t % (unsigned)S);
    bf16_t* base = qkv + t * (long long)row_stride + (long long)h * D;
    u32x4* lo = reinterpret_cast<u32x4*>(base + c);
    u32x4* hi = reinterpret_cast<u32x4*>(base + half + c);
    float a[8], b[8], oa[8], ob[8];
    unpack8(*lo, a);
    unpack8(*hi, b);
    const float4* csr = reinterpret_cast<const float4*>(cs + (long long)p * half + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 q = csr[j];  // (cos_j0, sin_j0, cos_j1, sin_j1)
      const float c0 = q.x, s0 = sign * q.y, c1 = q.z, s1 = sign * q.w;
      oa[2 * j] = a[2 * j] * c0 - b[2 * j] * s0;
      ob[2 * j] = b[2 * j] * c0 + a[2 * j] * s0;
      oa[2 * j + 1] = a[2 * j + 1] * c1 - b[2 * j + 1] * s1;
      ob[2 * j + 1] = b[2 * j + 1] * c1 + a[2 * j + 1] * s1;
    }
    *lo = pack8(oa);
    *hi = pack8(ob);
  }
}

RCA_API int rca_swiglu_fwd(const void* gu, void* out, long long T, int F, hipStream_t stream) {
  if (F % 8) return -1;
  if (T * (F / 8) >= (1LL << 31)) return -2;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(T * (F / 8), 256)), dim3(256), 0, stream, (const bf16_t*)gu,
                     (bf16_t*)out, T, F);
  return (int)hipGetLastError();
}

RCA_API int rca_swiglu_bwd(const void* gu, const void* dout, void* dgu, long long T, int F, hipStream_t stream) {
  if (F % 8) return -1;
  if (T * (F / 8) >= (1LL << 31)) return -2;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(T * (F / 8), 256)), dim3(256), 0, stream, (const bf16_t*)gu,
                     (const bf16_t*)dout, (bf16_t*)dgu, T, F);
  return (int)hipGetLastError();
}

// Contract: T % 64 == 0, F % 64 == 0, 16-B aligned buffers; out_t is [F, T] (fwd) / dgu_t [2F, T] (bwd).
RCA_API int rca_swiglu_fwd_tr(const void* gu, void* out, void* out_t, int T, int F, hipStream_t stream) {
  if ((T & 63) || (F & 63) || T <= 0 || F <= 0) return -1;
  const long long tiles = (long long)(T >> 6) * (F >> 6);
  hipLaunchKernelGGL(swiglu_fwd_tr_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, (const bf16_t*)gu,
                     (bf16_t*)out, (bf16_t*)out_t, T, F);
  return (int)hipGetLastError();
}

RCA_API int rca_swiglu_bwd_tr(const void* gu, const void* dout, void* dgu, void* dgu_t, int T, int F,
                              hipStream_t stream) {
  if ((T & 63) || (F & 63) || T <= 0 || F <= 0) return -1;
  const long long tiles = (long long)(T >> 6) * (F >> 6);
  hipLaunchKernelGGL(swiglu_bwd_tr_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, (const bf16_t*)gu,
                     (const bf16_t*)dout, (bf16_t*)dgu, (bf16_t*)dgu_t, T, F);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Placement probe: where did this workgroup run? out[0] = XCC id (HW_REG_XCC_ID), out[1] = the
// raw HW_REG_HW_ID word (CU / SH / SE fields). Used to map hipExtStreamCreateWithCUMask bits to
// XCDs before partitioning CUs between concurrent streams (parallel/optim.py).
__global__ void probe_hwid_kernel(int* __restrict__ out) {
  if (threadIdx.x == 0) {
    out[0] = (int)__builtin_amdgcn_s_getreg((3 << 11) | 20);   // XCC_ID[3:0]
    out[1] = (int)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
  }
}

RCA_API int rca_probe_hwid(int* out, hipStream_t stream) {
  hipLaunchKernelGGL(probe_hwid_kernel, dim3(1), dim3(64), 0, stream, out);
  return (int)hipGetLastError();
}

RCA_API int rca_rope(void* qkv, const void* cs, const int* pos, long long T, int S, int nheads_rot, int row_stride,
                     int D, int backward, hipStream_t stream) {
  if (D % 16) return -1;
  const long long n = T * nheads_rot * (D / 16);
  if (n >= (1LL << 31)) return -2;
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (bf16_t*)qkv, (const float2*)cs, pos,
                     T, S, nheads_rot, row_stride, D, backward ? -1.f : 1.f);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// bf16 transpose out[C, R] = in[R, C] (row stride ldi, output contiguous), 64 x 64 tiles staged
// through LDS: 16-B global loads along C, 16-B global stores along R (every output row piece is a
// full 128-B line). The LDS tile rows are padded to 66 elements (33 dwords), so the eight lanes
// that gather one output chunk (8 input rows apart) hit eight different banks. Feeds the
// reduction-contiguous operand layouts of the backward GEMMs (parallel/fused_linear.py).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                             int R, int C, long ldi) {
  constexpr int TP = 66;
  __shared__ unsigned tile32[64 * TP / 2];
  bf16_t* tile = reinterpret_cast<bf16_t*>(tile32);
  const int tilesC = C >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (bid / tilesC) << 6, c0 = (bid % tilesC) << 6;
  const int t = threadIdx.x, ch = t & 7, rr = t >> 3;
  u32x4 v[2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
    v[p] = *reinterpret_cast<const u32x4*>(in + (long)(r0 + rr + 32 * p) * ldi + c0 + ch * 8);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    unsigned* dst = tile32 + ((rr + 32 * p) * TP + ch * 8) / 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = v[p][i];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = rr + 32 * p;
    u32x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (unsigned)tile[(ch * 8 + 2 * i) * TP + c] | ((unsigned)tile[(ch * 8 + 2 * i + 1) * TP + c] << 16);
    *reinterpret_cast<u32x4*>(out + (long)(c0 + c) * R + r0 + ch * 8) = o;
  }
}

// RoPE backward fused with the transpose the qkv weight gradient reads: one 128-token x 128-column
// tile (= one head of D = 128) per workgroup, the transpose128 tile scheme below. Each lane holds
// 8 columns of 2 rows; the rotate-half partner (column c +- 64) is the lane 8 apart (same rows):
// one __shfl_xor(.., 8) per register. Heads < nrot are rotated by -theta (the adjoint) and written
// back in place; every head goes to g_t [W][T] transposed. Replaces the in-place rope_kernel pass
// over dq / dk AND the transpose of dqkv: the v heads are only read, the q / k heads read once.
__global__ __launch_bounds__(256) void rope_bwd_tr_kernel(bf16_t* __restrict__ g, const float2* __restrict__ cs,
                                                          const int* __restrict__ pos, bf16_t* __restrict__ g_t,
                                                          int T, int S, int W, int nrot) {
  __shared__ u32x4 W4[128 * 64 / 4];
  unsigned* Wd = reinterpret_cast<unsigned*>(W4);
  const int tilesC = W >> 7;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (bid / tilesC) << 7, c0 = (bid % tilesC) << 7;
  const int t = threadIdx.x, ch = t & 15, rp = t >> 4;
  const bool rot = (c0 >> 7) < nrot;
  const bool hi = ch >= 8;                 // second half of the head: x[c] pairs with x[c - 64]
  const int f0 = (ch & 7) * 8;             // frequency index of this lane's first column
  u32x4 va[4], vb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bf16_t* p = g + (long)(r0 + 2 * rp + 32 * k) * W + c0 + ch * 8;
    va[k] = *reinterpret_cast<const u32x4*>(p);
    vb[k] = *reinterpret_cast<const u32x4*>(p + W);
  }
  if (rot) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        u32x4& v = half ? vb[k] : va[k];
        const int row = r0 + 2 * rp + 32 * k + half;
        const int p_ = pos ? pos[row] : row % S;
        u32x4 w;
#pragma unroll
        for (int m = 0; m < 4; ++m) w[m] = (unsigned)__shfl_xor((int)v[m], 8, 64);
        float a[8], b[8], o[8];
        unpack8(v, a);  // own columns
        unpack8(w, b);  // partner columns (c +- 64)
        const float4* csr = reinterpret_cast<const float4*>(cs + (long)p_ * 64 + f0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 q = csr[j];  // (cos, sin) of frequencies f0 + 2j, f0 + 2j + 1
          // backward = rotation by -theta: lo' = lo c + hi s, hi' = hi c - lo s
          o[2 * j] = hi ? a[2 * j] * q.x - b[2 * j] * q.y : a[2 * j] * q.x + b[2 * j] * q.y;
          o[2 * j + 1] = hi ? a[2 * j + 1] * q.z - b[2 * j + 1] * q.w : a[2 * j + 1] * q.z + b[2 * j + 1] * q.w;
        }
        v = pack8(o);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16_t* p = g + (long)(r0 + 2 * rp + 32 * k) * W + c0 + ch * 8;
      *reinterpret_cast<u32x4*>(p) = va[k];
      *reinterpret_cast<u32x4*>(p + W) = vb[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int q = (rp + 16 * k) ^ (2 * ch);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      Wd[(ch * 8 + 2 * m) * 64 + q] = __builtin_amdgcn_perm(vb[k][m], va[k][m], 0x05040100u);
      Wd[(ch * 8 + 2 * m + 1) * 64 + q] = __builtin_amdgcn_perm(vb[k][m], va[k][m], 0x07060302u);
    }
  }
  __syncthreads();
  const int q4 = (t & 15) * 4;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int j = (t >> 4) + 16 * p;
    const int sw = 2 * (j >> 3);
    u32x4 o = W4[(j * 64 + (q4 ^ (sw & ~3))) >> 2];
    if (sw & 2) o = u32x4{o[2], o[3], o[0], o[1]};
    *reinterpret_cast<u32x4*>(g_t + (long)(c0 + j) * T + r0 + q4 * 2) = o;
  }
}

// 128 x 128 tiles (R, C multiples of 128): 256-B row segments on both the read and the write side
// (the 64 x 64 kernel's 128-B pieces, 8 KB apart, cost DRAM page locality) and no 16-bit LDS
// traffic. Each lane loads two input rows (2q, 2q+1) x 8 columns and pairs them in registers
// (v_perm) into 8 dwords = (out[j][2q], out[j][2q+1]) for its 8 output rows j; the dwords go to an
// LDS image W[j][q] (128 x 64 dwords, XOR-swizzled q' = q ^ 2*(j/8): the 32 lanes of a
// ds_write_b32 group -- 16 column chunks x 2 row pairs -- hit 32 distinct banks), and each output
// 16-B chunk is one ds_read_b128 of 4 consecutive q (the swizzle only swaps dword pairs inside the
// aligned quad when j/8 is odd). Per lane: 8 x 16-B loads in flight, 64 ds_write_b32, 8
// ds_read_b128, 8 x 16-B stores.
__global__ __launch_bounds__(256) void transpose128_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                                int R, int C, long ldi) {
  __shared__ u32x4 W4[128 * 64 / 4];
  unsigned* W = reinterpret_cast<unsigned*>(W4);
  const int tilesC = C >> 7;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (bid / tilesC) << 7, c0 = (bid % tilesC) << 7;
  const int t = threadIdx.x, ch = t & 15, rp = t >> 4;
  u32x4 va[4], vb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bf16_t* p = in + (long)(r0 + 2 * rp + 32 * k) * ldi + c0 + ch * 8;
    va[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    vb[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + ldi));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int q = (rp + 16 * k) ^ (2 * ch);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      // lo halves of both rows -> column 2m, hi halves -> column 2m+1 (v_perm_b32 byte selects)
      W[(ch * 8 + 2 * m) * 64 + q] = __builtin_amdgcn_perm(vb[k][m], va[k][m], 0x05040100u);
      W[(ch * 8 + 2 * m + 1) * 64 + q] = __builtin_amdgcn_perm(vb[k][m], va[k][m], 0x07060302u);
    }
  }
  __syncthreads();
  const int q4 = (t & 15) * 4;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int j = (t >> 4) + 16 * p;
    const int sw = 2 * (j >> 3);
    u32x4 o = W4[(j * 64 + (q4 ^ (sw & ~3))) >> 2];
    if (sw & 2) o = u32x4{o[2], o[3], o[0], o[1]};
    *reinterpret_cast<u32x4*>(out + (long)(c0 + j) * R + r0 + q4 * 2) = o;
  }
}

// g [T][W] contiguous (W = heads x 128), D = 128: the first nrot heads rotated back in place, g_t
// [W][T] = g^T of the result. Contract: T % 128 == 0, W % 128 == 0, 16-B aligned; else -1.
RCA_API int rca_rope_bwd_tr(void* g, const void* cs, const int* pos, void* g_t, int T, int S, int W, int nrot,
                            hipStream_t stream) {
  if (T <= 0 || W <= 0 || (T & 127) || (W & 127) || nrot < 0 || nrot * 128 > W || S <= 0) return -1;
  if (((uintptr_t)g | (uintptr_t)g_t | (uintptr_t)cs) & 15) return -1;
  const long long tiles = (long long)(T >> 7) * (W >> 7);
  if (tiles >= (1LL << 31)) return -2;
  hipLaunchKernelGGL(rope_bwd_tr_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, (bf16_t*)g, (const float2*)cs,
                     pos, (bf16_t*)g_t, T, S, W, nrot);
  return (int)hipGetLastError();
}

RCA_API int rca_transpose_bf16(const void* in, void* out, int R, int C, long long ldi, hipStream_t stream) {
  if (R <= 0 || C <= 0 || (R & 63) || (C & 63) || (ldi & 7) || ldi < C) return -1;
  if (((uintptr_t)in & 15) || ((uintptr_t)out & 15)) return -3;
  // 128 x 128 tiles measured faster only on the ~117 M-element 8B operands (gate_up / down weights,
  // 8192 x 14336 activations: 73 vs 93-95 us); below ~64 M elements the 64 x 64 kernel's 4x more
  // workgroups fill the chip better, and on the 1 G-element dlogits it is ~4 % ahead
  // (scripts/transpose_bench.py). RCA_TRANSPOSE_TILE64=1 forces the 64 x 64 kernel.
  static const bool tile64 = getenv("RCA_TRANSPOSE_TILE64") != nullptr;
  const long long nel = (long long)R * C;
  if (!tile64 && !(R & 127) && !(C & 127) && nel >= (96LL << 20) && nel <= (256LL << 20)) {
    const long long tiles = (long long)(R >> 7) * (C >> 7);
    if (tiles >= (1LL << 31)) return -2;
    hipLaunchKernelGGL(transpose128_bf16_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, (const bf16_t*)in,
                       (bf16_t*)out, R, C, (long)ldi);
    return (int)hipGetLastError();
  }
  const long long tiles = (long long)(R >> 6) * (C >> 6);
  if (tiles >= (1LL << 31)) return -2;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, (const bf16_t*)in,
                     (bf16_t*)out, R, C, (long)ldi);
  return (int)hipGetLastError();
}
