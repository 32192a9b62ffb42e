// Sustained fp32 rates on gfx950 (developer microbenchmark, not product code): the chip's clock
// under a long, all-CU load differs between the vector FMA pipe and the f32 matrix pipe, so each
// loop runs ~0.3 s per launch and is reported as TFLOP/s over the last of 4 launches.
// Variants carry LDS operand traffic like a convolution inner loop (one ds_read per MFMA pair /
// per 16 packed FMAs), so the measurement includes the register-file and LDS power a real kernel
// spends.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float a, int iters) {
    __shared__ f2 lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) lds[i] = (f2){i * 1e-3f, i * 2e-3f};
    __syncthreads();
    const float x = (float)threadIdx.x * 1e-3f;
    float s = 0.f;
    int p = threadIdx.x;
    if constexpr (KIND == 0) {  // v_pk_fma_f32, 16 accumulators, operand pair from LDS per 16 FMAs
        f2 acc[16];
        for (int i = 0; i < 16; ++i) acc[i] = (f2){x + i, x - i};
        for (int it = 0; it < iters; ++it) {
            const f2 v = lds[p & 2047];
            p += 67;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma((f2){a, a}, acc[i], v);
        }
        for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
    } else if constexpr (KIND == 1) {  // 16x16x4 f32 MFMA, 4 accumulators, A from LDS per 2 MFMAs
        f4 acc[4];
        for (int i = 0; i < 4; ++i) acc[i] = (f4){x, x, x, x};
        const float b = a * 0.5f;
        for (int it = 0; it < iters; ++it) {
            const f2 v = lds[p & 2047];
            p += 67;
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, b, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, b, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, a, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(v.y, a, acc[3], 0, 0, 0);
        }
        for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
    } else {  // v_fma_f32 (scalar), 32 accumulators
        float acc[32];
        for (int i = 0; i < 32; ++i) acc[i] = x + i;
        for (int it = 0; it < iters; ++it) {
            const f2 v = lds[p & 2047];
            p += 67;
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = fmaf(a, acc[i], (i & 1) ? v.y : v.x);
        }
        for (int i = 0; i < 32; ++i) s += acc[i];
    }
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
void run(const char* name, float* d, int blocks, int iters, double flops_per_thread_iter) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms = 0.f;
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<KIND>), dim3(blocks), dim3(256), 0, 0, d, 0.999f, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    const double fl = flops_per_thread_iter * iters * (double)blocks * 256;
    printf("%-40s %8.2f ms  %7.1f TFLOP/s\n", name, ms, fl / ms / 1e9);
}

int main() {
    float* d;
    const int blocks = 256 * 8;
    hipMalloc(&d, blocks * 256 * 4);
    run<0>("v_pk_fma_f32 sustained (16 per ds_read)", d, blocks, 160000, 16 * 4.0);
    run<1>("mfma_f32_16x16x4 sustained (4 per ds_read)", d, blocks, 40000, 4 * 32.0);
    run<2>("v_fma_f32 sustained (32 per ds_read)", d, blocks, 80000, 32 * 2.0);
    run<0>("v_pk_fma_f32 sustained (again)", d, blocks, 160000, 16 * 4.0);
    run<1>("mfma_f32_16x16x4 sustained (again)", d, blocks, 40000, 4 * 32.0);
    hipFree(d);
    return 0;
}
