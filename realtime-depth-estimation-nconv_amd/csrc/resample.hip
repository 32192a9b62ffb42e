// resample.hip — the guided model's bilinear depth downsampling (models/step2.py:249,277:
// F.interpolate(depth, scale_factor=1/k, mode="bilinear", align_corners=True)) on gfx950.
//
// The reference runs it on the CPU, whose kernel forms the sampling position in fp32: scale =
// fp32(H-1) / (Ho-1), source row = fp32(scale * oh), index = its truncation, lambdas in fp32. At
// KITTI's 352x1216 the last column's position comes out 1214.9999 instead of 1215, so the sample
// mixes the interior pixel 1214 (a depth near 80) with weight 1e-4 into the border pixel (nconv7's
// bias ring): an index arithmetic in another precision (as PyTorch-ROCm's own resampling kernel
// uses) moves that output by ~1e-2. This kernel repeats the CPU's arithmetic, blend included
// (fma(l0h, fma(l0w, a00, l1w * a01), l1h * fma(l0w, a10, l1w * a11))), so its outputs equal the
// reference's (bitwise at the sizes the model uses; tests/test_gpu_guided.py).
//
// One thread per output element, grid-stride; the planes are tiny next to the convolutions around
// them (B x 1 x H/k x W/k), so the kernel is launch-bound and kept simple.
#include "nconv_internal.h"

namespace nconv {

__global__ __launch_bounds__(256) void bilinear_ac(const float* __restrict__ x, int H, int W, float* __restrict__ y,
                                                   int Ho, int Wo, float sh, float sw, long long n) {
    // the position must be rounded before its fraction is taken (the CPU's fp32 steps): no
    // contraction of scale * o into the subtraction (the blend's fmas are explicit)
#pragma clang fp contract(off)
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int ow = (int)(e % Wo);
        const long long t = e / Wo;
        const int oh = (int)(t % Ho);
        const long long pl = t / Ho;
        const float fh = sh * (float)oh, fw = sw * (float)ow;
        const int h0 = (int)fh, w0 = (int)fw;
        const int h1 = h0 + (h0 < H - 1 ? 1 : 0), w1 = w0 + (w0 < W - 1 ? 1 : 0);
        const float lh1 = fh - (float)h0, lw1 = fw - (float)w0;
        const float lh0 = 1.0f - lh1, lw0 = 1.0f - lw1;
        const float* p = x + pl * H * W;
        const float a00 = p[(long long)h0 * W + w0], a01 = p[(long long)h0 * W + w1];
        const float a10 = p[(long long)h1 * W + w0], a11 = p[(long long)h1 * W + w1];
        const float top = fmaf(lw0, a00, lw1 * a01), bot = fmaf(lw0, a10, lw1 * a11);
        y[e] = fmaf(lh0, top, lh1 * bot);
    }
}

int launch_bilinear_ac(const float* x, int B, int C, int H, int W, float* y, int Ho, int Wo, hipStream_t st,
                       const char** why) {
    // align_corners: scale = (in - 1) / (out - 1) in fp32, 0 for a one-pixel output
    const float sh = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
    const float sw = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
    const long long n = (long long)B * C * Ho * Wo;
    if (n == 0) return 0;
    long long blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(bilinear_ac, dim3((unsigned)blocks), dim3(256), 0, st, x, H, W, y, Ho, Wo, sh, sw, n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
