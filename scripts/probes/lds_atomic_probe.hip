// LDS atomic throughput probe on gfx950: ds_add_f32 vs ds_add_u32 vs ds_add_u64 on random bins
// (the GBDT histogram's access pattern: 64 lanes, 512 distinct float slots).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const unsigned* __restrict__ idx, float* __restrict__ out, int iters,
                                              int span) {
  __shared__ unsigned long long lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  unsigned x = idx[blockIdx.x * blockDim.x + threadIdx.x];
  float* lf = reinterpret_cast<float*>(lds);
  unsigned* lu = reinterpret_cast<unsigned*>(lds);
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    const int b = (x >> 16) % span;
    if (MODE == 0) atomicAdd(lf + 2 * b, 1.0f);
    if (MODE == 1) atomicAdd(lu + 2 * b, 1u);
    if (MODE == 2) atomicAdd(&lds[b], 0x100000001ull);
    if (MODE == 3) { atomicAdd(lf + 2 * b, 1.0f); atomicAdd(lf + 2 * b + 1, 1.0f); }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lf[0] + (float)lu[1];
}

int main() {
  const int blocks = 512, threads = 1024, iters = 4096, span = 256;
  std::vector<unsigned> h(blocks * threads);
  for (auto& v : h) v = rand();
  unsigned* d; float* o;
  hipMalloc(&d, h.size() * 4); hipMalloc(&o, blocks * 4);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64 (packed pair)", "2x ds_add_f32 (g,h)"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(threads), 0, 0, d, o, iters, span);
      if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(threads), 0, 0, d, o, iters, span);
      if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(threads), 0, 0, d, o, iters, span);
      if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(threads), 0, 0, d, o, iters, span);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      const double wave_instr = (double)blocks * threads / 64 * iters * (mode == 3 ? 2 : 1);
      if (rep) printf("%-26s %8.3f ms  %.1f cycles/wave-instr/CU (2.4 GHz, 256 CUs)\n", names[mode], ms,
                      ms * 1e-3 * 2.4e9 * 256 / wave_instr);
    }
  }
  return 0;
}
