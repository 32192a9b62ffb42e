// The exact-fp32 input gradient's inner loop in isolation (developer microbenchmark, gfx950):
// per iteration 3 ds_read_b128 of a 6-pair window, 40 wave-uniform weights, 80 v_pk_fma_f32 into
// 8 x 2 accumulator pairs -- as dgrad_tiled's (o, kh) step. Variants drop the LDS reads (window in
// registers) and / or the weight loads (weights in SGPRs for the whole loop), to see which part
// keeps the VALU from its peak.   hipcc -O3 --offload-arch=gfx950 dgrad_loop.hip -o dgrad_loop
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool LDS, bool SLOAD>
__global__ __launch_bounds__(256) void k(const float* __restrict__ wg, float* out, int iters) {
    __shared__ __attribute__((aligned(16))) f2 tile[20 * 40];
    const int tid = threadIdx.x;
    for (int e = tid; e < 20 * 40; e += 256) tile[e] = (f2){(float)e * 1e-3f, 1.f};
    __syncthreads();
    const int ty = tid / 16, tx = (tid % 16) * 2;
    f2 acc[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i][0] = acc[i][1] = (f2){0.f, 0.f};
    f2 v0[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) v0[m] = tile[ty * 40 + tx + m];
    float wc[40];
#pragma unroll
    for (int q = 0; q < 40; ++q) wc[q] = wg[q];
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        const int r = it % 4;
        f2 v[6];
        if (LDS) {
            const f2* row = &tile[(ty + r) * 40 + tx];
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const f4 q = reinterpret_cast<const f4*>(row)[m];
                v[2 * m] = q.xy;
                v[2 * m + 1] = q.zw;
            }
        } else {
#pragma unroll
            for (int m = 0; m < 6; ++m) v[m] = v0[m];
        }
        const float* wr = wg + (it % 8) * 200 + r * 5;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float w = SLOAD ? wr[i * 25 + kw] : wc[i * 5 + kw];
                const f2 w2 = (f2){w, w};
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_elementwise_fma(w2, v[j + 4 - kw], acc[i][j]);
            }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0].x + acc[i][0].y + acc[i][1].x + acc[i][1].y;
    out[blockIdx.x * 256 + tid] = s;
}

int main() {
    float *d, *w;
    const int blocks = 256 * 28, iters = 2048;
    hipMalloc(&d, (size_t)blocks * 256 * 4);
    hipMalloc(&w, 1600 * 4);
    float hw[1600];
    for (int i = 0; i < 1600; ++i) hw[i] = 1e-4f * (i % 37);
    hipMemcpy(w, hw, sizeof(hw), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[4] = {"LDS window + scalar weight loads (dgrad_tiled)", "LDS window, weights in SGPRs    ",
                            "window in VGPRs, scalar weight loads", "window in VGPRs, weights in SGPRs"};
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 4; ++v) {
            hipEventRecord(e0);
            switch (v) {
                case 0: hipLaunchKernelGGL((k<true, true>), dim3(blocks), dim3(256), 0, 0, w, d, iters); break;
                case 1: hipLaunchKernelGGL((k<true, false>), dim3(blocks), dim3(256), 0, 0, w, d, iters); break;
                case 2: hipLaunchKernelGGL((k<false, true>), dim3(blocks), dim3(256), 0, 0, w, d, iters); break;
                default: hipLaunchKernelGGL((k<false, false>), dim3(blocks), dim3(256), 0, 0, w, d, iters); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double flops = 2.0 * 2 * 80 * (double)iters * blocks * 256;  // 80 pk_fma = 160 fma per lane
            printf("%s: %.3f ms  %.1f TFLOP/s\n", names[v], ms, flops / ms / 1e9);
        }
    hipFree(d);
    hipFree(w);
    return 0;
}
