// batchnorm.hip — training-mode BatchNorm2d (+ ReLU) of the RGB-guided model on gfx950.
//
// Replaces nn.BatchNorm2d in training mode (batch statistics, running-stat update) followed by
// nn.ReLU — RGBEncoder (models/step2.py:139-143), Basic2d (:189-191), Basic2dTrans (:207-213) —
// and the autograd of both. HBM-bound passes over NCHW fp32:
//   forward : bn_stats (1 read: per-chunk count / mean / M2, Welford-style), bn_finalize (one
//             block per channel, chunks combined in a fixed tree order with Chan's formula:
//             deterministic, no E[x^2] - E[x]^2 cancellation; running mean / unbiased running var),
//             bn_apply (1 read + 1 write: y = [relu](gamma (x - mean) invstd + beta));
//   backward: bn_bwd_stats (2 reads: per chunk sum g', sum g' (x - mean), sum (x - mean), g' = g
//             masked by the recomputed ReLU), bn_bwd_finalize (fixed order, double), bn_bwd_apply
//             (2 reads + 1 write: gx = gamma invstd (g' - sum g' / N - xhat sum g' xhat / N), formed
//             in double per element).
// Why double in the backward: the saved mean is the batch mean rounded to fp32, so fp32 xhat = (x -
// mean) invstd sums to N (mean_exact - mean) invstd instead of 0, and sum g' / N rounds likewise;
// both leave gx with a systematic nonzero sum, which the preceding convolution's weight gradient
// (sum gx * input, inputs with a large mean such as 0..255 RGB) multiplies by N. At 480x640 that
// moved the RGB encoder convolutions' weight gradients by ~2e-3 of their size against float64 (as
// PyTorch's native GPU BatchNorm does); the reference's CPU kernels accumulate in double. Here
// the backward recovers the exact mean's offset from the fp32 one (sum (x - mean) / N, double) and
// forms each gx in double, so the only error left per element is its final fp32 rounding.
// A chunk is kChunk consecutive elements of one (image, channel) plane, 16 per thread (float4
// loads when the plane size is a multiple of 4).
#include "nconv_internal.h"

namespace nconv {

constexpr int kBT = 256;
constexpr int kChunk = 4096;
constexpr int kPer = kChunk / kBT;  // elements per thread

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();  // red is reused between calls
    if (lane == 0) red[w] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

// Loads the thread's kPer elements of chunk j of plane (b, c): element i = j*kChunk + 4*tid + k
// (+ kBT*4 per float4 group); out-of-plane elements are flagged invalid.
__device__ __forceinline__ void load_chunk(const float* plane, int hw, int j, bool vec, float (&v)[kPer],
                                           bool (&ok)[kPer]) {
    const int base = j * kChunk;
#pragma unroll
    for (int g = 0; g < kPer / 4; ++g) {
        const int i0 = base + (g * kBT + threadIdx.x) * 4;
        if (vec && i0 + 3 < hw) {
            const f4 q = *reinterpret_cast<const f4*>(plane + i0);
            v[4 * g] = q.x;
            v[4 * g + 1] = q.y;
            v[4 * g + 2] = q.z;
            v[4 * g + 3] = q.w;
#pragma unroll
            for (int k = 0; k < 4; ++k) ok[4 * g + k] = true;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ok[4 * g + k] = i0 + k < hw;
                v[4 * g + k] = ok[4 * g + k] ? plane[i0 + k] : 0.f;
            }
        }
    }
}

__device__ __forceinline__ void store_chunk(float* plane, int hw, int j, bool vec, const float (&v)[kPer]) {
    const int base = j * kChunk;
#pragma unroll
    for (int g = 0; g < kPer / 4; ++g) {
        const int i0 = base + (g * kBT + threadIdx.x) * 4;
        if (vec && i0 + 3 < hw) {
            *reinterpret_cast<f4*>(plane + i0) = (f4){v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (i0 + k < hw) plane[i0 + k] = v[4 * g + k];
        }
    }
}

// part[(c * nparts + b * ncp + j) * 3 + {0,1,2}] = (count, mean, M2) of chunk j of plane (b, c)
__global__ __launch_bounds__(kBT) void bn_stats(const float* __restrict__ x, int C, int hw, int ncp, int nparts,
                                                int vec, float* __restrict__ part) {
    __shared__ float red[4];
    const int j = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
    const float* plane = x + ((size_t)b * C + c) * hw;
    float v[kPer];
    bool ok[kPer];
    load_chunk(plane, hw, j, vec != 0, v, ok);
    const int n = min(kChunk, hw - j * kChunk);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kPer; ++k) s += v[k];  // invalid elements are 0
    const float mean = block_sum(s, red) / (float)n;
    float m2 = 0.f;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const float d = ok[k] ? v[k] - mean : 0.f;
        m2 = fmaf(d, d, m2);
    }
    m2 = block_sum(m2, red);
    if (threadIdx.x == 0) {
        float* o = part + ((size_t)c * nparts + (size_t)b * ncp + j) * 3;
        o[0] = (float)n;
        o[1] = mean;
        o[2] = m2;
    }
}

// One block per channel: thread t combines a contiguous run of the chunks (Chan's parallel formula,
// in double), then the 256 runs are combined pairwise in a fixed tree order in LDS -- deterministic,
// and no longer one thread walking 400+ chunks serially.
__device__ __forceinline__ void chan_combine(double& n, double& mean, double& m2, double nb, double mb, double m2b) {
    const double nn = n + nb;
    if (nn == 0.0) return;
    const double d = mb - mean;
    mean += d * nb / nn;
    m2 += m2b + d * d * n * nb / nn;
    n = nn;
}

__global__ __launch_bounds__(kBT) void bn_finalize(const float* __restrict__ part, int C, int nparts, float momentum,
                                                   float eps, float* __restrict__ rmean, float* __restrict__ rvar,
                                                   float* __restrict__ mean_out, float* __restrict__ invstd_out) {
    __shared__ double sn[kBT], sm[kBT], s2[kBT];
    const int c = blockIdx.x, t = threadIdx.x;
    const float* p = part + (size_t)c * nparts * 3;
    const int per = (nparts + kBT - 1) / kBT, k0 = t * per, k1 = min(nparts, k0 + per);
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int k = k0; k < k1; ++k) chan_combine(n, mean, m2, p[3 * k], p[3 * k + 1], p[3 * k + 2]);
    sn[t] = n;
    sm[t] = mean;
    s2[t] = m2;
    __syncthreads();
    for (int h = kBT / 2; h > 0; h >>= 1) {
        if (t < h) {
            double a = sn[t], b = sm[t], q = s2[t];
            chan_combine(a, b, q, sn[t + h], sm[t + h], s2[t + h]);
            sn[t] = a;
            sm[t] = b;
            s2[t] = q;
        }
        __syncthreads();
    }
    if (t == 0) {
        n = sn[0];
        mean = sm[0];
        m2 = s2[0];
        const double var = m2 / n;
        mean_out[c] = (float)mean;
        invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
        if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
        if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * (n > 1.0 ? m2 / (n - 1.0) : var));
    }
}

// fixed-order block sum of per-thread contiguous runs (double), one block per channel
template <int NV>
__device__ __forceinline__ void chan_sums(const float* p, int nparts, double (&out)[NV]) {
    __shared__ double red[NV][kBT];
    const int t = threadIdx.x;
    const int per = (nparts + kBT - 1) / kBT, k0 = t * per, k1 = min(nparts, k0 + per);
    double v[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = 0.0;
    for (int k = k0; k < k1; ++k)
#pragma unroll
        for (int q = 0; q < NV; ++q) v[q] += p[NV * k + q];
#pragma unroll
    for (int q = 0; q < NV; ++q) red[q][t] = v[q];
    __syncthreads();
    for (int h = kBT / 2; h > 0; h >>= 1) {
        if (t < h)
#pragma unroll
            for (int q = 0; q < NV; ++q) red[q][t] += red[q][t + h];
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) out[q] = red[q][0];
}

__device__ __forceinline__ float bn_y(float x, float mu, float is, float g, float bt, bool relu) {
    const float y = fmaf((x - mu) * is, g, bt);
    return relu ? fmaxf(y, 0.f) : y;
}

// one block per (chunk, channel, image): the channel's parameters are wave-uniform loads, the
// chunk's elements go through load_chunk's float4 path (no per-element index division)
__global__ __launch_bounds__(kBT) void bn_apply(const float* __restrict__ x, float* __restrict__ y, int C, int hw,
                                                int vec, const float* __restrict__ mean,
                                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                                const float* __restrict__ beta, int relu) {
    const int j = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
    const size_t off = ((size_t)b * C + c) * hw;
    const float mu = mean[c], is = invstd[c], g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    float v[kPer];
    bool ok[kPer];
    load_chunk(x + off, hw, j, vec != 0, v, ok);
#pragma unroll
    for (int k = 0; k < kPer; ++k) v[k] = bn_y(v[k], mu, is, g, bt, relu);
    store_chunk(y + off, hw, j, vec != 0, v);
}

// part[(c * nparts + b * ncp + j) * 3 + {0,1,2}] = (sum g', sum g' (x - mean), sum (x - mean)) of
// chunk j of plane (b, c); mean = the forward's fp32 batch mean
__global__ __launch_bounds__(kBT) void bn_bwd_stats(const float* __restrict__ gy, const float* __restrict__ x, int C,
                                                    int hw, int ncp, int nparts, int vec,
                                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    int relu, float* __restrict__ part) {
    __shared__ float red[4];
    const int j = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
    const size_t off = ((size_t)b * C + c) * hw;
    float g[kPer], v[kPer];
    bool ok[kPer];
    load_chunk(gy + off, hw, j, vec != 0, g, ok);
    load_chunk(x + off, hw, j, vec != 0, v, ok);
    const float mu = mean[c], is = invstd[c], ga = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    float s = 0.f, sx = 0.f, sd = 0.f;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const float d = v[k] - mu;
        const float gg = (relu && !(fmaf(d * is, ga, bt) > 0.f)) ? 0.f : g[k];  // invalid: g = 0
        s += gg;
        sx = fmaf(gg, d, sx);
        sd += ok[k] ? d : 0.f;
    }
    s = block_sum(s, red);
    sx = block_sum(sx, red);
    sd = block_sum(sd, red);
    if (threadIdx.x == 0) {
        float* o = part + ((size_t)c * nparts + (size_t)b * ncp + j) * 3;
        o[0] = s;
        o[1] = sx;
        o[2] = sd;
    }
}

// sums[c] = {s0, a, k} (double) with gx = gamma invstd (g' - s0 - (x - mean - delta) invstd s1) =
// f (g' - k - a x): delta = sum (x - mean) / N (the exact mean's offset from the fp32 one), s0 =
// sum g' / N, s1 = sum g' xhat / N with xhat about the exact mean, a = invstd s1, k = s0 - (mean +
// delta) a; ggamma = sum g' xhat, gbeta = sum g'
__global__ __launch_bounds__(kBT) void bn_bwd_finalize(const float* __restrict__ part, int C, int nparts, double n,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, double* __restrict__ sums,
                                                       float* __restrict__ ggamma, float* __restrict__ gbeta) {
    const int c = blockIdx.x;
    double v[3];
    chan_sums<3>(part + (size_t)c * nparts * 3, nparts, v);
    if (threadIdx.x == 0) {
        const double is = (double)invstd[c], delta = v[2] / n;
        const double sxh = (v[1] - delta * v[0]) * is;  // sum g' xhat, xhat about the exact mean
        const double s0 = v[0] / n, a = is * (sxh / n);
        sums[3 * c] = s0;
        sums[3 * c + 1] = a;
        sums[3 * c + 2] = s0 - ((double)mean[c] + delta) * a;
        if (gbeta) gbeta[c] = (float)v[0];
        if (ggamma) ggamma[c] = (float)sxh;
    }
}

__global__ __launch_bounds__(kBT) void bn_bwd_apply(const float* __restrict__ gy, const float* __restrict__ x,
                                                    float* __restrict__ gx, int C, int hw, int vec,
                                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    int relu, const double* __restrict__ sums) {
    const int j = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
    const size_t off = ((size_t)b * C + c) * hw;
    const float mu = mean[c], is = invstd[c], ga = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    const double f = (double)ga * (double)is, a = sums[3 * c + 1], k0 = sums[3 * c + 2];
    float g[kPer], v[kPer];
    bool ok[kPer];
    load_chunk(gy + off, hw, j, vec != 0, g, ok);
    load_chunk(x + off, hw, j, vec != 0, v, ok);
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const float gg = (relu && !(fmaf((v[k] - mu) * is, ga, bt) > 0.f)) ? 0.f : g[k];  // the forward's mask
        v[k] = (float)(f * ((double)gg - k0 - a * (double)v[k]));
    }
    store_chunk(gx + off, hw, j, vec != 0, v);
}

// ---- ReLU backward + bias gradient of a convolution (the ConvBlock / bias-only layers):
//      g' = g * (out > 0) (when out is given), gbias = sum of g' over images and pixels ----
__global__ __launch_bounds__(kBT) void relu_bias_stats(const float* __restrict__ g, const float* __restrict__ out,
                                                       float* __restrict__ gm, int C, int hw, int ncp, int nparts,
                                                       int vec, float* __restrict__ part) {
    __shared__ float red[4];
    const int j = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
    const size_t off = ((size_t)b * C + c) * hw;
    float v[kPer], o[kPer];
    bool ok[kPer];
    load_chunk(g + off, hw, j, vec != 0, v, ok);
    if (out) {
        load_chunk(out + off, hw, j, vec != 0, o, ok);
#pragma unroll
        for (int k = 0; k < kPer; ++k) v[k] = o[k] > 0.f ? v[k] : 0.f;
        if (gm) {
            const int base = j * kChunk;
#pragma unroll
            for (int q = 0; q < kPer / 4; ++q) {
                const int i0 = base + (q * kBT + threadIdx.x) * 4;
                if (vec && i0 + 3 < hw) {
                    *reinterpret_cast<f4*>(gm + off + i0) = (f4){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (i0 + k < hw) gm[off + i0 + k] = v[4 * q + k];
                }
            }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kPer; ++k) s += v[k];
    s = block_sum(s, red);
    if (threadIdx.x == 0) part[(size_t)c * nparts + (size_t)b * ncp + j] = s;
}

__global__ __launch_bounds__(kBT) void channel_sum_finalize(const float* __restrict__ part, int C, int nparts,
                                                            float* __restrict__ out) {
    const int c = blockIdx.x;
    double v[1];
    chan_sums<1>(part + (size_t)c * nparts, nparts, v);
    if (threadIdx.x == 0) out[c] = (float)v[0];
}

size_t relu_bias_workspace_bytes(int B, int C, int H, int W) {
    return (size_t)B * ((H * W + kChunk - 1) / kChunk) * C * sizeof(float);
}

int launch_relu_bias_bwd(int B, int C, int H, int W, const float* g, const float* out, float* gm, float* gbias,
                         float* ws, hipStream_t st, const char** why) {
    const int hw = H * W, ncp = (hw + kChunk - 1) / kChunk, nparts = B * ncp;
    const int vec = (hw % 4 == 0) && ((uintptr_t)g % 16 == 0) && (!out || (uintptr_t)out % 16 == 0) &&
                    (!gm || (uintptr_t)gm % 16 == 0);
    hipLaunchKernelGGL(relu_bias_stats, dim3(ncp, C, B), dim3(kBT), 0, st, g, out, gm, C, hw, ncp, nparts, vec, ws);
    if (gbias)
        hipLaunchKernelGGL(channel_sum_finalize, dim3(C), dim3(kBT), 0, st, ws, C, nparts, gbias);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

// ------------------------------------------------------------------------------------------------
static int bn_ncp(const nconv_bn_train& p) { return (p.H * p.W + kChunk - 1) / kChunk; }

// per-chunk partials (3 floats each), then the backward's per-channel sums (3 doubles, 8-B aligned)
static size_t bn_sums_offset(const nconv_bn_train& p) {
    const size_t nparts = (size_t)p.B * bn_ncp(p);
    return (nparts * p.C * 3 * sizeof(float) + 7) & ~(size_t)7;
}

size_t bn_workspace_bytes(const nconv_bn_train& p) { return bn_sums_offset(p) + 3 * (size_t)p.C * sizeof(double); }

int launch_bn_train_fwd(const nconv_bn_train& p, float* ws, hipStream_t st, const char** why) {
    const int hw = p.H * p.W, ncp = bn_ncp(p), nparts = p.B * ncp;
    const int vec = (hw % 4 == 0) && ((uintptr_t)p.x % 16 == 0);
    hipLaunchKernelGGL(bn_stats, dim3(ncp, p.C, p.B), dim3(kBT), 0, st, p.x, p.C, hw, ncp, nparts, vec, ws);
    hipLaunchKernelGGL(bn_finalize, dim3(p.C), dim3(kBT), 0, st, ws, p.C, nparts, p.momentum, p.eps,
                       p.running_mean, p.running_var, p.mean, p.invstd);
    const int vy = vec && ((uintptr_t)p.y % 16 == 0);
    hipLaunchKernelGGL(bn_apply, dim3(ncp, p.C, p.B), dim3(kBT), 0, st, p.x, p.y, p.C, hw, vy, p.mean, p.invstd,
                       p.gamma, p.beta, p.relu);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

int launch_bn_train_bwd(const nconv_bn_train& p, const float* gy, float* gx, float* ggamma, float* gbeta, float* ws,
                        hipStream_t st, const char** why) {
    const int hw = p.H * p.W, ncp = bn_ncp(p), nparts = p.B * ncp;
    const int vec = (hw % 4 == 0) && ((uintptr_t)p.x % 16 == 0) && ((uintptr_t)gy % 16 == 0);
    double* sums = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + bn_sums_offset(p));
    hipLaunchKernelGGL(bn_bwd_stats, dim3(ncp, p.C, p.B), dim3(kBT), 0, st, gy, p.x, p.C, hw, ncp, nparts, vec, p.mean,
                       p.invstd, p.gamma, p.beta, p.relu, ws);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3(p.C), dim3(kBT), 0, st, ws, p.C, nparts, (double)((size_t)p.B * hw),
                       p.mean, p.invstd, sums, ggamma, gbeta);
    if (gx)
        hipLaunchKernelGGL(bn_bwd_apply, dim3(ncp, p.C, p.B), dim3(kBT), 0, st, gy, p.x, gx, p.C, hw,
                           vec && ((uintptr_t)gx % 16 == 0), p.mean, p.invstd, p.gamma, p.beta, p.relu, sums);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
