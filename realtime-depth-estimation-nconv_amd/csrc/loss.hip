// loss.hip — the training loss of the reference (utils.py:95-151 calculate_loss) as three kernels.
//
//   rec  = masked_fill(r, t == 0, 0)                                    utils.py:139
//   e    = rec - t,  diff = t - rec
//   gx   = conv2d(diff, [[1,0,-1],[2,0,-2],[1,0,-1]], padding=1)         utils.py:95-106
//   gy   = conv2d(diff, [[1,2,1],[0,0,0],[-1,-2,-1]], padding=1)         utils.py:109-122
//   L    = 0.8 sqrt(mean e^2) + 0.2 (mean|gx| + mean|gy|)   (gradient loss), else mean e^2
//
// On B planes of (H, W): the training loop calls it on the whole (B, 1, H, W) batch
// (train_step1.py:63; the means run over B*H*W, the Sobel convolutions pad each image on its own),
// the validation loop on element [0] (utils.py:36, B = 1). In PyTorch this is ~45 elementwise /
// reduction launches forward and backward; here, on 16 x 64 pixel tiles whose diff window
// (diff = t - masked r, 2-pixel halo, zero outside the image) is staged once in LDS:
//   loss_partials  per tile: e^2, |gx|, |gy| (the same operation order as train.gradient_x / _y,
//                  so signs match torch exactly), one per-tile partial of each
//   loss_finalize  one block: fixed-order (double) sum of the tile partials -> L and the two
//                  backward coefficients, kept in the workspace for the backward
//   loss_grad      per tile: the signs of gx, gy over the tile + 1-pixel halo into LDS, then
//                  dL/dr = go m [c_e e - c_g sum_q (sign gx(q) Kx(p - q) + sign gy(q) Ky(p - q))]
//                  over the 3x3 neighbours q inside the plane, with torch's sign(0) = 0 for |.|'.
// Deterministic (no atomics). The planes may be row-strided views (the cropped DNET output).
#include "nconv_internal.h"

namespace nconv {

constexpr int kLT = 256;
constexpr int kTH = 16, kTW = 64;                // pixel tile of one workgroup (4 pixels per thread)
constexpr int kDH = kTH + 4, kDW = kTW + 4;      // staged diff window (2-pixel halo)
constexpr int kSH = kTH + 2, kSW = kTW + 2;      // sign window (1-pixel halo)

struct LossPlane {
    const float* r;
    const float* t;
    long long rs, ts;    // row strides (elements)
    long long rbs, tbs;  // image strides (elements)
    int B, H, W;
    // image b's planes
    __device__ __forceinline__ LossPlane image(int b) const {
        LossPlane q = *this;
        q.r += b * rbs;
        q.t += b * tbs;
        return q;
    }
};

__device__ __forceinline__ float loss_diff(const LossPlane& p, int i, int j) {
    // diff = t - masked_fill(r, t == 0, 0); zero outside the plane (conv padding)
    if ((unsigned)i >= (unsigned)p.H || (unsigned)j >= (unsigned)p.W) return 0.f;
    const float t = p.t[i * p.ts + j];
    const float rec = t == 0.f ? 0.f : p.r[i * p.rs + j];
    return t - rec;
}

// gradient_x at (i, j) from a diff window accessor, in train.gradient_x's order
template <typename D>
__device__ __forceinline__ float sobel_x(D d, int i, int j) {
    const float a = d(i - 1, j - 1) - d(i - 1, j + 1);
    const float b = d(i, j - 1) - d(i, j + 1);
    const float c = d(i + 1, j - 1) - d(i + 1, j + 1);
    return (a + 2.f * b) + c;
}
template <typename D>
__device__ __forceinline__ float sobel_y(D d, int i, int j) {
    const float a = d(i - 1, j - 1) - d(i + 1, j - 1);
    const float b = d(i - 1, j) - d(i + 1, j);
    const float c = d(i - 1, j + 1) - d(i + 1, j + 1);
    return (a + 2.f * b) + c;
}

// Tiles of the grid: (tiles per image row band) x (row bands) x B, blockIdx.x linear.
struct LossTile {
    int b, i0, j0;
};
__device__ __forceinline__ LossTile loss_tile(const LossPlane& p) {
    const int ntw = (p.W + kTW - 1) / kTW, nth = (p.H + kTH - 1) / kTH;
    const int t = blockIdx.x;
    LossTile lt;
    lt.b = t / (ntw * nth);
    const int r = t - lt.b * ntw * nth;
    lt.i0 = (r / ntw) * kTH;
    lt.j0 = (r % ntw) * kTW;
    return lt;
}

// The tile's diff window (rows i0-2 .. i0+kTH+1, columns j0-2 .. j0+kTW+1) into LDS: every
// element's t and r loaded first (buffer loads, out-of-plane offsets read 0; r also where t == 0,
// so no load waits on another), then diff = t - masked_fill(r, t == 0, 0).
__device__ __forceinline__ void stage_diff(const LossPlane& p, int i0, int j0, float* dw) {
    constexpr int NS = (kDH * kDW + kLT - 1) / kLT;
    constexpr unsigned OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t rt = plane_rsrc(p.t, (int)(((long long)(p.H - 1) * p.ts + p.W) * 4));
    const __amdgpu_buffer_rsrc_t rr = plane_rsrc(p.r, (int)(((long long)(p.H - 1) * p.rs + p.W) * 4));
    float tv[NS], rv[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const int e = threadIdx.x + kLT * k;
        const int a = e / kDW, c = e - a * kDW, i = i0 - 2 + a, j = j0 - 2 + c;
        const bool in = e < kDH * kDW && (unsigned)i < (unsigned)p.H && (unsigned)j < (unsigned)p.W;
        tv[k] = ld_f32(rt, in ? (unsigned)(i * p.ts + j) * 4u : OOB);
        rv[k] = ld_f32(rr, in ? (unsigned)(i * p.rs + j) * 4u : OOB);
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const int e = threadIdx.x + kLT * k;
        if (e < kDH * kDW) dw[e] = tv[k] - (tv[k] == 0.f ? 0.f : rv[k]);
    }
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

// one workgroup per tile; the partial sums are indexed by tile (a fixed order)
__global__ __launch_bounds__(kLT) void loss_partials(LossPlane pb, int grad_loss, float* __restrict__ part) {
    __shared__ float dw[kDH * kDW];
    __shared__ float red[4];
    const LossTile lt = loss_tile(pb);
    const LossPlane p = pb.image(lt.b);
    stage_diff(p, lt.i0, lt.j0, dw);
    __syncthreads();
    // window accessor in plane coordinates
    auto d = [&](int a, int b) { return dw[(a - lt.i0 + 2) * kDW + (b - lt.j0 + 2)]; };
    float sq = 0.f, ax = 0.f, ay = 0.f;
#pragma unroll
    for (int k = 0; k < kTH * kTW / kLT; ++k) {
        const int e = threadIdx.x + kLT * k, i = lt.i0 + e / kTW, j = lt.j0 + e % kTW;
        if (i < p.H && j < p.W) {
            const float dv = d(i, j);
            sq += dv * dv;  // (rec - t)^2
            if (grad_loss) {
                ax += fabsf(sobel_x(d, i, j));
                ay += fabsf(sobel_y(d, i, j));
            }
        }
    }
    sq = block_sum256(sq, red);
    ax = block_sum256(ax, red);
    ay = block_sum256(ay, red);
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = sq;
        part[3 * blockIdx.x + 1] = ax;
        part[3 * blockIdx.x + 2] = ay;
    }
}

// coef[0] = L, coef[1] = dL/d(e^2 sum) factor c_e (dL/de = c_e e), coef[2] = c_g (0.2 / n)
__global__ __launch_bounds__(kLT) void loss_finalize(const float* __restrict__ part, int nblk, int n, int grad_loss,
                                                      float* __restrict__ loss, float* __restrict__ coef) {
    __shared__ double red[3][kLT];
    double s[3] = {0.0, 0.0, 0.0};
    for (int b = threadIdx.x; b < nblk; b += kLT)
        for (int k = 0; k < 3; ++k) s[k] += part[3 * b + k];
    for (int k = 0; k < 3; ++k) red[k][threadIdx.x] = s[k];
    __syncthreads();
    for (int w = kLT / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float mse = (float)(red[0][0] / n);
        float L, ce, cg;
        if (grad_loss) {
            const float rmse = sqrtf(mse);
            L = rmse * 0.8f + ((float)(red[1][0] / n) + (float)(red[2][0] / n)) * 0.2f;
            ce = 0.8f / (n * rmse);  // d(0.8 sqrt(sum e^2 / n)) / de
            cg = 0.2f / n;
        } else {
            L = mse;
            ce = 2.f / n;
            cg = 0.f;
        }
        loss[0] = L;
        coef[0] = L;
        coef[1] = ce;
        coef[2] = cg;
    }
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(kLT) void loss_grad(LossPlane pb, int grad_loss, const float* __restrict__ coef,
                                                  const float* __restrict__ gout, float* __restrict__ g) {
    __shared__ float dw[kDH * kDW];
    __shared__ float sgx[kSH * kSW], sgy[kSH * kSW];
    const LossTile lt = loss_tile(pb);
    const LossPlane p = pb.image(lt.b);
    const int n = p.H * p.W;
    g += (size_t)lt.b * n;  // contiguous (B, H, W) gradient
    stage_diff(p, lt.i0, lt.j0, dw);
    __syncthreads();
    auto d = [&](int a, int b) { return dw[(a - lt.i0 + 2) * kDW + (b - lt.j0 + 2)]; };
    if (grad_loss) {
        // signs of gx, gy at the tile's pixels and their 1-pixel halo; 0 outside the plane (such
        // neighbours contribute nothing)
        for (int e = threadIdx.x; e < kSH * kSW; e += kLT) {
            const int a = e / kSW, c = e - a * kSW, qi = lt.i0 - 1 + a, qj = lt.j0 - 1 + c;
            const bool in = (unsigned)qi < (unsigned)p.H && (unsigned)qj < (unsigned)p.W;
            sgx[e] = in ? sgnf(sobel_x(d, qi, qj)) : 0.f;
            sgy[e] = in ? sgnf(sobel_y(d, qi, qj)) : 0.f;
        }
        __syncthreads();
    }
    const float go = gout ? gout[0] : 1.f;
    const float ce = coef[1], cg = coef[2];
#pragma unroll
    for (int k = 0; k < kTH * kTW / kLT; ++k) {
        const int e = threadIdx.x + kLT * k, li = e / kTW, lj = e % kTW, i = lt.i0 + li, j = lt.j0 + lj;
        if (i >= p.H || j >= p.W) continue;
        if (p.t[i * p.ts + j] == 0.f) {  // masked_fill: no gradient reaches r here
            g[i * p.W + j] = 0.f;
            continue;
        }
        // dL/drec = c_e e - c_g G,  e = rec - t = -diff(p)
        float acc = ce * (-d(i, j));
        if (grad_loss) {
            float G = 0.f;
#pragma unroll
            for (int qa = -1; qa <= 1; ++qa)
#pragma unroll
                for (int qb = -1; qb <= 1; ++qb) {
                    const int si = (li + 1 + qa) * kSW + (lj + 1 + qb);
                    // Kx(dy, dx) = w(dy) (-dx), Ky(dy, dx) = w(dx) (-dy), (dy, dx) = p - q, w = 1, 2, 1
                    const int dy = -qa, dx = -qb;
                    const float wy = dy == 0 ? 2.f : 1.f, wx = dx == 0 ? 2.f : 1.f;
                    G += sgx[si] * wy * (float)(-dx) + sgy[si] * wx * (float)(-dy);
                }
            // d|gx|/drec = -(d|gx|/ddiff)
            acc -= cg * G;
        }
        g[i * p.W + j] = go * acc;
    }
}

static int loss_tiles(int B, int H, int W) { return B * ((H + kTH - 1) / kTH) * ((W + kTW - 1) / kTW); }

size_t loss_workspace_bytes(int B, int H, int W) { return (3 * (size_t)loss_tiles(B, H, W) + 4) * sizeof(float); }

static int loss_err(const char** why) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

int launch_loss_fwd(const LossArgs& a, int grad_loss, float* loss, float* ws, hipStream_t st, const char** why) {
    const LossPlane p{a.r, a.t, a.rs, a.ts, a.rbs, a.tbs, a.B, a.H, a.W};
    const int nblk = loss_tiles(a.B, a.H, a.W);
    float* coef = ws;
    float* part = ws + 4;
    hipLaunchKernelGGL(loss_partials, dim3(nblk), dim3(kLT), 0, st, p, grad_loss, part);
    hipLaunchKernelGGL(loss_finalize, dim3(1), dim3(kLT), 0, st, part, nblk, a.B * a.H * a.W, grad_loss, loss, coef);
    return loss_err(why);
}

int launch_loss_bwd(const LossArgs& a, int grad_loss, const float* gout, const float* ws, float* g, hipStream_t st,
                    const char** why) {
    const LossPlane p{a.r, a.t, a.rs, a.ts, a.rbs, a.tbs, a.B, a.H, a.W};
    hipLaunchKernelGGL(loss_grad, dim3(loss_tiles(a.B, a.H, a.W)), dim3(kLT), 0, st, p, grad_loss, ws, gout, g);
    return loss_err(why);
}

}  // namespace nconv
