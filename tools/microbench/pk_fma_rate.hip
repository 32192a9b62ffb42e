// Throughput of v_pk_fma_f32 vs v_fma_f32 on gfx950 (developer microbenchmark).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int PACKED>
__global__ __launch_bounds__(256) void k(float* out, float a, int iters) {
  if (PACKED) {
    f2 acc[16]; for (int i = 0; i < 16; ++i) acc[i] = (f2){(float)threadIdx.x + i, (float)i};
    f2 w = {a, a};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma(w, acc[i], w);
    float s = 0; for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y; out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    float acc[32]; for (int i = 0; i < 32; ++i) acc[i] = (float)threadIdx.x + i;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 32; ++i) acc[i] = fmaf(a, acc[i], a);
    float s = 0; for (int i = 0; i < 32; ++i) s += acc[i]; out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}
int main() {
  float* d; int blocks = 256 * 16; hipMalloc(&d, blocks * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4096;
  for (int rep = 0; rep < 3; ++rep) {
    for (int packed = 0; packed < 2; ++packed) {
      hipEventRecord(e0);
      if (packed) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, iters);
      else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double flops = 2.0 * 32 * iters * (double)blocks * 256;
      printf("%s: %.3f ms  %.1f TFLOP/s\n", packed ? "v_pk_fma_f32" : "v_fma_f32   ", ms, flops / ms / 1e9);
    }
  }
  hipFree(d);
  return 0;
}
