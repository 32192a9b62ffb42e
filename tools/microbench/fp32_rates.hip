// fp32 arithmetic rates on gfx950 (developer microbenchmark, not product code):
// v_fma_f32, v_pk_fma_f32, v_mfma_f32_16x16x4_f32, v_mfma_f32_32x32x2_f32, and one wave
// interleaving f32 MFMAs with independent VALU FMAs (are the matrix and vector pipes additive?),
// and split waves of bf16 MFMAs beside packed-FMA waves.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int KIND, int NV>
__global__ __launch_bounds__(256) void k(float* out, float a, int iters) {
    const float x = (float)threadIdx.x * 1e-3f;
    float s = 0.f;
    if constexpr (KIND == 0) {  // v_fma_f32
        float acc[32];
        for (int i = 0; i < 32; ++i) acc[i] = x + i;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = fmaf(a, acc[i], a);
        for (int i = 0; i < 32; ++i) s += acc[i];
    } else if constexpr (KIND == 1) {  // v_pk_fma_f32
        f2 acc[16];
        for (int i = 0; i < 16; ++i) acc[i] = (f2){x + i, x - i};
        const f2 w = {a, a};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma(w, acc[i], w);
        for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
    } else if constexpr (KIND == 2) {  // 16x16x4 f32 MFMA, 4 independent accumulators (+ NV VALU FMAs each)
        f4 acc[4];
        for (int i = 0; i < 4; ++i) acc[i] = (f4){x, x, x, x};
        float v[NV > 0 ? NV : 1];
        for (int i = 0; i < (NV > 0 ? NV : 1); ++i) v[i] = x + i;
        const float b = a * 0.5f;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
                for (int i = 0; i < NV; ++i) v[i] = fmaf(a, v[i], b);
            }
        }
        for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
        for (int i = 0; i < NV; ++i) s += v[i];
    } else if constexpr (KIND == 3) {  // 32x32x2 f32 MFMA, 2 accumulators
        f16v acc[2];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 16; ++j) acc[i][j] = x;
        const float b = a * 0.5f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
        for (int i = 0; i < 2; ++i) s += acc[i][0] + acc[i][15];
    } else if constexpr (KIND == 4) {  // 4x4x1 16-block f32 MFMA, NV independent accumulators
        f4 acc[NV];
        for (int i = 0; i < NV; ++i) acc[i] = (f4){x, x, x, x};
        const float b = a * 0.5f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int i = 0; i < NV; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
        for (int i = 0; i < NV; ++i) s += acc[i][0] + acc[i][3];
    } else if constexpr (KIND == 5) {  // 16x16x1 4-block f32 MFMA
        f16v acc[2];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 16; ++j) acc[i][j] = x;
        const float b = a * 0.5f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, acc[i], 0, 0, 0);
        for (int i = 0; i < 2; ++i) s += acc[i][0] + acc[i][15];
    } else if constexpr (KIND == 6) {  // 4x4x1 16-block, B operand from LDS (NV MFMAs per ds_read_b32)
        __shared__ float lds[4096];
        for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = i * 1e-3f;
        __syncthreads();
        f4 acc[8];
        for (int i = 0; i < 8; ++i) acc[i] = (f4){x, x, x, x};
        int p = threadIdx.x;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float bv[8 / NV];
#pragma unroll
                for (int q = 0; q < 8 / NV; ++q) bv[q] = lds[(p + 67 * q + 13 * j) & 4095];
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, bv[i / NV], acc[i], 0, 0, 0);
            }
            p = (p + 256) & 4095;
        }
        for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
    } else if constexpr (KIND == 7) {  // wave-specialised: even waves f32 MFMA, odd waves v_pk_fma
        // (NV bit 0: run the MFMA waves, bit 1: run the VALU waves) -- do the two pipes add?
        const int wv = threadIdx.x >> 6;
        if ((wv & 1) == 0 && (NV & 1)) {
            f4 acc[4];
            for (int i = 0; i < 4; ++i) acc[i] = (f4){x, x, x, x};
            const float b = a * 0.5f;
            for (int it = 0; it < iters; ++it)
#pragma unroll
                for (int j = 0; j < 8; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
            for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
        } else if ((wv & 1) == 1 && (NV & 2)) {
            f2 acc[16];
            for (int i = 0; i < 16; ++i) acc[i] = (f2){x + i, x - i};
            const f2 w = {a, a};
            for (int it = 0; it < iters * 8; ++it)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma(w, acc[i], w);
            for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
        }
    } else if constexpr (KIND == 8) {  // wave-specialised: even waves bf16 MFMA 16x16x32, odd v_pk_fma
        const int wv = threadIdx.x >> 6;
        if ((wv & 1) == 0 && (NV & 1)) {
            typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
            bf8 av, bv;
            for (int i = 0; i < 8; ++i) {
                av[i] = (__bf16)(x + i);
                bv[i] = (__bf16)(a * 0.5f - i);
            }
            f4 acc[4];
            for (int i = 0; i < 4; ++i) acc[i] = (f4){x, x, x, x};
            for (int it = 0; it < iters; ++it)
#pragma unroll
                for (int j = 0; j < 8; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i], 0, 0, 0);
            for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
        } else if ((wv & 1) == 1 && (NV & 2)) {
            f2 acc[16];
            for (int i = 0; i < 16; ++i) acc[i] = (f2){x + i, x - i};
            const f2 w = {a, a};
            for (int it = 0; it < iters * 8; ++it)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = __builtin_elementwise_fma(w, acc[i], w);
            for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 4x4x1_16b vs an fmaf chain: same bits? (layout probe: lane l block l/4; A row l%4, B col l%4)
__global__ void exact_check(const float* A, const float* B, float* out_mfma, float* out_fma, int K) {
    const int l = threadIdx.x;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(A[k * 64 + l], B[k * 64 + l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out_mfma[l * 4 + r] = acc[r];
    // reference: block b = l/4, column j = l%4; rows i = r
    const int b = l / 4, j = l % 4;
    for (int r = 0; r < 4; ++r) {
        float v = 0.f;
        for (int k = 0; k < K; ++k) v = fmaf(A[k * 64 + b * 4 + r], B[k * 64 + b * 4 + j], v);
        out_fma[l * 4 + r] = v;
    }
}

template <int KIND, int NV>
void run(const char* name, float* d, int blocks, int iters, double flops_per_thread_iter) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k<KIND, NV>), dim3(blocks), dim3(256), 0, 0, d, 0.999f, 16);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<KIND, NV>), dim3(blocks), dim3(256), 0, 0, d, 0.999f, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = flops_per_thread_iter * iters * (double)blocks * 256;
    printf("%-34s %8.3f ms  %7.1f TFLOP/s\n", name, ms, fl / ms / 1e9);
}

int main() {
    float* d;
    const int blocks = 256 * 8;
    hipMalloc(&d, blocks * 256 * 4);
    const int it = 2048;
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 0>("v_fma_f32", d, blocks, it, 2.0 * 32);
        run<1, 0>("v_pk_fma_f32", d, blocks, it, 2.0 * 32);
        // per thread per iteration: 8 x 4 MFMAs of 16x16x4 (2*1024 flop / 64 lanes = 32 per lane)
        run<2, 0>("mfma_f32_16x16x4", d, blocks, it / 4, 8 * 4 * 32.0);
        run<3, 0>("mfma_f32_32x32x2", d, blocks, it / 4, 8 * 2 * (2.0 * 32 * 32 * 2) / 64);
        run<2, 4>("mfma16x16x4 + 4 fma/4mfma", d, blocks, it / 4, 8 * (4 * 32.0 + 4 * 2));
        run<2, 8>("mfma16x16x4 + 8 fma/4mfma", d, blocks, it / 4, 8 * (4 * 32.0 + 8 * 2));
        run<2, 16>("mfma16x16x4 + 16 fma/4mfma", d, blocks, it / 4, 8 * (4 * 32.0 + 16 * 2));
        run<2, 32>("mfma16x16x4 + 32 fma/4mfma", d, blocks, it / 4, 8 * (4 * 32.0 + 32 * 2));
        run<2, 48>("mfma16x16x4 + 48 fma/4mfma", d, blocks, it / 4, 8 * (4 * 32.0 + 48 * 2));
        run<4, 4>("mfma_f32_4x4x1_16b (4 acc)", d, blocks, it / 4, 8 * 4 * 8.0);
        run<4, 8>("mfma_f32_4x4x1_16b (8 acc)", d, blocks, it / 4, 8 * 8 * 8.0);
        run<5, 0>("mfma_f32_16x16x1_4b", d, blocks, it / 4, 8 * 2 * 32.0);
        run<6, 1>("4x4x1_16b, 1 ds_read_b32 per mfma", d, blocks, it / 4, 8 * 8 * 8.0);
        run<6, 2>("4x4x1_16b, 1 ds_read_b32 per 2", d, blocks, it / 4, 8 * 8 * 8.0);
        run<6, 4>("4x4x1_16b, 1 ds_read_b32 per 4", d, blocks, it / 4, 8 * 8 * 8.0);
        // per thread-iteration averaged over the block: half the threads 32 MFMAs (32 flop/lane
        // each), half 8*16 v_pk_fma (4 flop/lane each)
        run<7, 1>("split waves: MFMA half only", d, blocks, it / 4, 0.5 * 32 * 32.0);
        run<7, 2>("split waves: VALU half only", d, blocks, it / 4, 0.5 * 128 * 4.0);
        run<7, 3>("split waves: both halves", d, blocks, it / 4, 0.5 * 32 * 32.0 + 0.5 * 128 * 4.0);
        // bf16 16x16x32: 2*16*16*32 flop / 64 lanes = 256 per lane per MFMA
        run<8, 1>("split: bf16 MFMA half only", d, blocks, it / 4, 0.5 * 32 * 256.0);
        run<8, 2>("split: VALU half only (bf16 run)", d, blocks, it / 4, 0.5 * 128 * 4.0);
        run<8, 3>("split: bf16 MFMA + VALU halves", d, blocks, it / 4, 0.5 * 32 * 256.0 + 0.5 * 128 * 4.0);
    }
    {
        const int K = 200;
        float *A, *Bm, *o1, *o2;
        hipMallocManaged(&A, K * 64 * 4);
        hipMallocManaged(&Bm, K * 64 * 4);
        hipMallocManaged(&o1, 256 * 4);
        hipMallocManaged(&o2, 256 * 4);
        unsigned st = 12345;
        for (int i = 0; i < K * 64; ++i) {
            st = st * 1664525u + 1013904223u;
            A[i] = (float)(st >> 8) / 16777216.0f;
            st = st * 1664525u + 1013904223u;
            Bm[i] = (float)(st >> 8) / 16777216.0f * 10.f - 3.f;
        }
        hipLaunchKernelGGL(exact_check, dim3(1), dim3(64), 0, 0, A, Bm, o1, o2, K);
        hipDeviceSynchronize();
        int diff = 0, rowmis = 0;
        for (int i = 0; i < 256; ++i) diff += o1[i] != o2[i];
        // layout check: lane l / reg r should be block l/4, col l%4, row r
        printf("4x4x1_16b vs fmaf chain: %d of 256 differ (o1[5]=%.9g o2[5]=%.9g)\n", diff, o1[5], o2[5]);
        (void)rowmis;
    }
    hipFree(d);
    return 0;
}
