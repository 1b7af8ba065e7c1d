// Fused image augmentation for Data map_batches on gfx950: per-image crop box -> bilinear resize
// (align_corners=False, torch F.interpolate semantics) -> optional horizontal flip -> uint8 /255,
// mean/std normalise -> bf16 or fp32, NCHW or NHWC (channels_last) output. One kernel replaces
// the RandomResizedCrop + RandomHorizontalFlip + ToTensor + Normalize chain: every output pixel
// is produced from 4 source texels in one pass (HBM sees the uint8 source once via L2 and the
// output once).
//
// Mapping: one thread per output pixel (all C channels); a 256-thread block covers 256
// consecutive pixels of one output row segment, so the 4 texel rows it gathers are shared
// through L2. Per-image boxes/flips are tiny device arrays.
#include "common.h"

namespace {

template <int OUT_BF16, int NHWC>
__global__ __launch_bounds__(256) void crop_resize_norm_kernel(const unsigned char* __restrict__ in, void* __restrict__ out,
                                                               const int* __restrict__ boxes,
                                                               const unsigned char* __restrict__ flips, int N, int Hin,
                                                               int Win, int C, int Ho, int Wo, float m0, float m1,
                                                               float m2, float m3, float s0, float s1, float s2, float s3) {
  const float mean[4] = {m0, m1, m2, m3};
  const float inv[4] = {s0, s1, s2, s3};
  const long long total = (long long)N * Ho * Wo;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(p / ((long long)Ho * Wo));
    const int rem = (int)(p - (long long)n * Ho * Wo);
    const int oy = rem / Wo, ox = rem - oy * Wo;
    const int by = boxes[4 * n], bx = boxes[4 * n + 1], bh = boxes[4 * n + 2], bw = boxes[4 * n + 3];
    const int sx_dst = (flips != nullptr && flips[n]) ? (Wo - 1 - ox) : ox;
    // source coordinates inside the box (torch: src = max(0, (dst + 0.5) * in / out - 0.5))
    float sy = fmaxf(0.f, ((float)oy + 0.5f) * ((float)bh / (float)Ho) - 0.5f);
    float sx = fmaxf(0.f, ((float)sx_dst + 0.5f) * ((float)bw / (float)Wo) - 0.5f);
    int y0 = (int)sy, x0 = (int)sx;
    y0 = min(y0, bh - 1);
    x0 = min(x0, bw - 1);
    const int y1 = min(y0 + 1, bh - 1), x1 = min(x0 + 1, bw - 1);
    const float wy = sy - (float)y0, wx = sx - (float)x0;
    const long long img = (long long)n * Hin * Win;
    const unsigned char* r0 = in + (img + (long long)(by + y0) * Win + bx) * C;
    const unsigned char* r1 = in + (img + (long long)(by + y1) * Win + bx) * C;
    for (int c = 0; c < C; ++c) {
      const float a = (float)r0[x0 * C + c], b = (float)r0[x1 * C + c];
      const float d = (float)r1[x0 * C + c], e = (float)r1[x1 * C + c];
      const float top = a + (b - a) * wx, bot = d + (e - d) * wx;
      const float v = ((top + (bot - top) * wy) * (1.f / 255.f) - mean[c]) * inv[c];
      const long long o = NHWC ? (p * C + c) : (((long long)n * C + c) * Ho + oy) * (long long)Wo + ox;
      if (OUT_BF16)
        ((bf16_t*)out)[o] = f2bf(v);
      else
        ((float*)out)[o] = v;
    }
  }
}

}  // namespace

// in: uint8 [N, Hin, Win, C]; boxes: int32 [N, 4] = (y0, x0, h, w) inside the image (validated by
// the caller); flips: uint8 [N] or null. out: [N, C, Ho, Wo] (channels_last=0) or [N, Ho, Wo, C].
RCA_API int rca_crop_resize_normalize(const void* in, void* out, const int* boxes, const unsigned char* flips, int N,
                                      int Hin, int Win, int C, int Ho, int Wo, const float* mean, const float* stdv,
                                      int out_dtype, int channels_last, hipStream_t stream) {
  if (C < 1 || C > 4 || N <= 0 || Ho <= 0 || Wo <= 0) return -1;
  float m[4] = {0, 0, 0, 0}, s[4] = {1, 1, 1, 1};
  for (int c = 0; c < C; ++c) {
    m[c] = mean[c];
    s[c] = 1.f / stdv[c];
  }
  const long long total = (long long)N * Ho * Wo;
  long long g = (total + 255) / 256;
  if (g > 65536) g = 65536;
#define RCA_CR(B, L)                                                                                              \
  hipLaunchKernelGGL((crop_resize_norm_kernel<B, L>), dim3((unsigned)g), dim3(256), 0, stream,                    \
                     (const unsigned char*)in, out, boxes, flips, N, Hin, Win, C, Ho, Wo, m[0], m[1], m[2], m[3], \
                     s[0], s[1], s[2], s[3])
  const int bf = out_dtype == 0;
  if (bf && channels_last) RCA_CR(1, 1);
  else if (bf) RCA_CR(1, 0);
  else if (channels_last) RCA_CR(0, 1);
  else RCA_CR(0, 0);
#undef RCA_CR
  return (int)hipGetLastError();
}
