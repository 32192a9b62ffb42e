// nconv_bwd.hip — backward NConv kernels for gfx950 (MI355X).
//
// Autograd of NConv2d.forward (reference models/step1.py:116-149) plus its DNET glue, in closed
// form (D and N/(D+eps) recovered from the saved outputs as cout*s and y-b):
//   gN = gy/(D+eps)          gD = -gy*N/(D+eps)^2 + gcout/s
//   gb = sum gy              gs = -sum gcout*D/s^2
//   gW = corr(x*c, gN) + corr(c, gD) + gs            (weight gradient, "wgrad")
//   G  = W^T (*) {gN, gD}    gx = G_xc*c,  gc = G_c + G_xc*x     (input gradient, "dgrad")
// dgrad is the forward's packed-FP32 structure transposed: a thread owns P input pixels and
// accumulates {G_xc, G_c} += w * {gN, gD} over (o, kh, kw), with {gN, gD} computed from
// (gy, gcout, y, cout) while staging. Its epilogue routes the input gradient through the glue's
// backward: max_pool2d -> the first maximum of the window (recomputed from the producer),
// concat -> channel split, nearest upsample -> a staged plane summed by upsample_bwd_gather.
// wgrad accumulates per-workgroup partial sums in registers over several tiles and a second
// kernel reduces them in a fixed order (bitwise deterministic, no float atomics).
#include "nconv_internal.h"

namespace nconv {

constexpr int kT = 256;

constexpr int pick_chunk(int n, int plane_f2, int budget) {
    int best = 1;
    for (int cc = 1; cc <= n; ++cc)
        if (n % cc == 0 && cc * plane_f2 * 8 <= budget) best = cc;
    return best;
}

// ---- gradient routing from a layer-input pixel to the producer tensors --------------------------
template <int MODE>
__device__ __forceinline__ void route_grad(const LayerDev& d, const BwdArgs& a, int b, int ci, int ih,
                                           int iw, float gxc, float gc_direct, float* tmp_x,
                                           float* tmp_c) {
    const nconv_layer& L = d.L;
    if constexpr (MODE == NCONV_LOAD_PLAIN) {
        const size_t i = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, ih, iw);
        const float x = L.a.x[i], c = L.a.c[i];
        if (a.gxa) a.gxa[i] += gxc * c;
        if (a.gca) a.gca[i] += gc_direct + gxc * x;
    } else if constexpr (MODE == NCONV_LOAD_THRESH) {
        const size_t i = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, ih, iw);
        const float x = L.a.x[i];
        const float c = (x > L.thresh) ? 1.0f : 0.0f;
        if (a.gxa) a.gxa[i] += gxc * c;  // c = (S > thr) carries no gradient
    } else if constexpr (MODE == NCONV_LOAD_POOL2) {
        const size_t i0 = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, 2 * ih, 2 * iw);
        const size_t W2 = (size_t)L.a.W;
        const size_t off[4] = {0, 1, W2, W2 + 1};
        int ax, ac;
        const float x = pool4(L.a.x[i0], L.a.x[i0 + 1], L.a.x[i0 + W2], L.a.x[i0 + W2 + 1], ax);
        const float c = pool4(L.a.c[i0], L.a.c[i0 + 1], L.a.c[i0 + W2], L.a.c[i0 + W2 + 1], ac);
        if (a.gxa) a.gxa[i0 + off[ax]] += gxc * c;
        if (a.gca) a.gca[i0 + off[ac]] += gc_direct + gxc * x;
    } else {
        const bool skip_first = (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST);
        const int first_c = skip_first ? L.a.C : L.b.C;
        const bool from_a = skip_first ? (ci < first_c) : (ci >= first_c);
        float x, c;
        load_xc<MODE>(d, b, ci, ih, iw, x, c);
        const float gx = gxc * c, gc = gc_direct + gxc * x;
        if (from_a) {
            const int ca = skip_first ? ci : ci - first_c;
            const size_t i = plane_idx(b, ca, L.a.C, L.a.H, L.a.W, ih, iw);
            if (a.gxa) a.gxa[i] += gx;
            if (a.gca) a.gca[i] += gc;
        } else {
            const int cb = skip_first ? ci - first_c : ci;
            const size_t i = plane_idx(b, cb, L.b.C, L.H, L.W, ih, iw);
            tmp_x[i] = gx;
            tmp_c[i] = gc;
        }
    }
}

template <int MODE>
__device__ __forceinline__ bool mode_has_tmp() {
    return MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST;
}

// ---- dgrad: tiled, stride 1 ------------------------------------------------------------------------
template <int CIN, int K>
struct DgCfg {
    static constexpr int P = (CIN >= 16) ? 2 : 4;
    static constexpr int TW = 64, TPR = TW / P, TH = kT / TPR;
    static constexpr int OHT = TH + K - 1, OWT = TW + K - 1;
    static constexpr int OWP = (OWT + 1) & ~1;
    static constexpr int PLANE = OHT * OWP;
    static constexpr int NV = P + K - 1;
};

template <int CIN, int COUT, int K, int MODE>
__global__ __launch_bounds__(kT) void dgrad_tiled(LayerDev d, BwdArgs a, float* tmp_x, float* tmp_c) {
    using C = DgCfg<CIN, K>;
    constexpr int OC = pick_chunk(COUT, C::PLANE, 24 * 1024);
    __shared__ __attribute__((aligned(16))) f2 tile[OC * C::PLANE];
    const nconv_layer& L = d.L;
    const float* __restrict__ wgt = L.weight;
    const int tid = threadIdx.x, b = blockIdx.z;
    const int ih0 = blockIdx.y * C::TH, iw0 = blockIdx.x * C::TW;
    const int oh0 = ih0 + L.PH - (K - 1), ow0 = iw0 + L.PW - (K - 1);
    const int ty = tid / C::TPR, tx = (tid % C::TPR) * C::P;

    f2 acc[CIN][C::P];
#pragma unroll
    for (int i = 0; i < CIN; ++i)
#pragma unroll
        for (int j = 0; j < C::P; ++j) acc[i][j] = (f2){0.f, 0.f};

    for (int o0 = 0; o0 < COUT; o0 += OC) {
        if (o0) __syncthreads();
        for (int e = tid; e < OC * C::OHT * C::OWT; e += kT) {
            const int oc = e / (C::OHT * C::OWT);
            const int rem = e - oc * (C::OHT * C::OWT);
            const int r = rem / C::OWT, col = rem - r * C::OWT;
            const int oh = oh0 + r, ow = ow0 + col, o = o0 + oc;
            float gN = 0.f, gD = 0.f;
            if ((unsigned)oh < (unsigned)L.Ho && (unsigned)ow < (unsigned)L.Wo) {
                const size_t i = plane_idx(b, o, COUT, L.Ho, L.Wo, oh, ow);
                const float gco = a.gco ? a.gco[i] : 0.f;
                nconv_grad_nd(a.gy[i], gco, a.y[i], a.co[i], L.eps, L.bias[o], L.wsum[o], gN, gD);
            }
            tile[oc * C::PLANE + r * C::OWP + col] = (f2){gN, gD};
        }
        __syncthreads();
#pragma unroll
        for (int oc = 0; oc < OC; ++oc) {
#pragma unroll
            for (int kh = 0; kh < K; ++kh) {
                const f2* row = &tile[oc * C::PLANE + (ty + K - 1 - kh) * C::OWP + tx];
                f2 v[C::NV];
#pragma unroll
                for (int m = 0; m < C::NV / 2; ++m) {
                    f4 q = reinterpret_cast<const f4*>(row)[m];
                    v[2 * m] = q.xy;
                    v[2 * m + 1] = q.zw;
                }
                if constexpr (C::NV & 1) v[C::NV - 1] = row[C::NV - 1];
                const float* wr = wgt + (size_t)(o0 + oc) * CIN * K * K + kh * K;
#pragma unroll
                for (int kw = 0; kw < K; ++kw)
#pragma unroll
                    for (int i = 0; i < CIN; ++i) {
                        const float w = wr[i * K * K + kw];
                        const f2 w2 = (f2){w, w};
#pragma unroll
                        for (int j = 0; j < C::P; ++j)
                            acc[i][j] = __builtin_elementwise_fma(w2, v[j + K - 1 - kw], acc[i][j]);
                    }
            }
        }
    }

    const int ih = ih0 + ty;
    if (ih >= L.H) return;
#pragma unroll
    for (int i = 0; i < CIN; ++i)
#pragma unroll
        for (int j = 0; j < C::P; ++j) {
            const int iw = iw0 + tx + j;
            if (iw < L.W) route_grad<MODE>(d, a, b, i, ih, iw, acc[i][j].x, acc[i][j].y, tmp_x, tmp_c);
        }
}

// ---- dgrad: generic (any stride / dilation / groups) ------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kT) void dgrad_generic(LayerDev d, BwdArgs a, float* tmp_x, float* tmp_c) {
    const nconv_layer& L = d.L;
    const size_t n = (size_t)L.B * L.Cin * L.H * L.W;
    const int cpg_in = L.Cin / L.groups, cpg_out = L.Cout / L.groups;
    for (size_t idx = (size_t)blockIdx.x * kT + threadIdx.x; idx < n; idx += (size_t)gridDim.x * kT) {
        const int iw = (int)(idx % L.W);
        const int ih = (int)((idx / L.W) % L.H);
        const int ci = (int)((idx / ((size_t)L.W * L.H)) % L.Cin);
        const int b = (int)(idx / ((size_t)L.W * L.H * L.Cin));
        const int g = ci / cpg_in, cl = ci - g * cpg_in;
        float Gxc = 0.f, Gc = 0.f;
        for (int ol = 0; ol < cpg_out; ++ol) {
            const int o = g * cpg_out + ol;
            const float bo = L.bias[o], so = L.wsum[o];
            for (int kh = 0; kh < L.KH; ++kh) {
                const int th = ih + L.PH - kh * L.DH;
                if (th < 0 || th % L.SH) continue;
                const int oh = th / L.SH;
                if (oh >= L.Ho) continue;
                for (int kw = 0; kw < L.KW; ++kw) {
                    const int tw = iw + L.PW - kw * L.DW;
                    if (tw < 0 || tw % L.SW) continue;
                    const int ow = tw / L.SW;
                    if (ow >= L.Wo) continue;
                    const size_t i = plane_idx(b, o, L.Cout, L.Ho, L.Wo, oh, ow);
                    float gN, gD;
                    nconv_grad_nd(a.gy[i], a.gco ? a.gco[i] : 0.f, a.y[i], a.co[i], L.eps, bo, so, gN, gD);
                    const float w = L.weight[(((size_t)o * cpg_in + cl) * L.KH + kh) * L.KW + kw];
                    Gxc = fmaf(w, gN, Gxc);
                    Gc = fmaf(w, gD, Gc);
                }
            }
        }
        route_grad<MODE>(d, a, b, ci, ih, iw, Gxc, Gc, tmp_x, tmp_c);
    }
}

// ---- nearest-upsample backward: low-res pixel gathers the high-res pixels that copied it -----------
__device__ __forceinline__ void up_range(int u, int in, int out, float scale, int& lo, int& hi) {
    if (out == in) { lo = u; hi = u + 1; return; }
    if (out == 2 * in) { lo = 2 * u; hi = 2 * u + 2; return; }
    int h = (int)floorf((float)u / scale) - 2;
    if (h < 0) h = 0;
    while (h < out && nearest_src(h, in, out, scale) < u) ++h;
    lo = h;
    while (h < out && nearest_src(h, in, out, scale) == u) ++h;
    hi = h;
}

__global__ __launch_bounds__(kT) void upsample_bwd_gather(LayerDev d, const float* tmp_x, const float* tmp_c,
                                                          float* gxb, float* gcb) {
    const nconv_layer& L = d.L;
    const int Cb = L.b.C, Hb = L.b.H, Wb = L.b.W;
    const size_t n = (size_t)L.B * Cb * Hb * Wb;
    for (size_t idx = (size_t)blockIdx.x * kT + threadIdx.x; idx < n; idx += (size_t)gridDim.x * kT) {
        const int v = (int)(idx % Wb);
        const int u = (int)((idx / Wb) % Hb);
        const size_t plane = idx / ((size_t)Wb * Hb);  // b*Cb + cb
        int h0, h1, w0, w1;
        up_range(u, Hb, L.H, d.up_scale_h, h0, h1);
        up_range(v, Wb, L.W, d.up_scale_w, w0, w1);
        float sx = 0.f, sc = 0.f;
        for (int h = h0; h < h1; ++h)
            for (int w = w0; w < w1; ++w) {
                const size_t i = (plane * L.H + h) * (size_t)L.W + w;
                sx += tmp_x[i];
                sc += tmp_c[i];
            }
        if (gxb) gxb[idx] += sx;
        if (gcb) gcb[idx] += sc;
    }
}

// ---- wgrad: tiled partial sums, stride 1 ------------------------------------------------------------
template <int CIN, int COUT, int K>
struct WgCfg {
    static constexpr int TH = 4, TW = 64;  // TH*TW == kT: one output pixel per thread while staging
    static constexpr int IHT = TH + K - 1, IWT = TW + K - 1;
    // plane strides = 1 (mod 32) f2 so that the 8 distinct channel planes a wave reads hit 8
    // different bank pairs (bank = dword % 64).
    static constexpr int IPL = ((IHT * IWT + 31) / 32) * 32 + 1;
    static constexpr int GPL = TH * TW + 1;
    static constexpr int NCB = COUT * CIN * K;  // (kh, o, i) combos, kw kept in registers
    static constexpr int NPASS = (NCB + kT - 1) / kT;
    static constexpr int LDS_F2 = CIN * IPL + COUT * GPL;
};

template <int CIN, int COUT, int K, int MODE>
__global__ __launch_bounds__(kT) void wgrad_tiled(LayerDev d, BwdArgs a, float* part, int ntile_w,
                                                  int ntile_h) {
    using C = WgCfg<CIN, COUT, K>;
    extern __shared__ __attribute__((aligned(16))) f2 smem[];
    f2* sin = smem;
    f2* sg = smem + CIN * C::IPL;
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x;
    const int ntiles = ntile_w * ntile_h * L.B;

    f2 acc[C::NPASS][K];
#pragma unroll
    for (int p = 0; p < C::NPASS; ++p)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[p][k] = (f2){0.f, 0.f};
    float gb_acc[COUT], gs_acc[COUT];
#pragma unroll
    for (int o = 0; o < COUT; ++o) gb_acc[o] = gs_acc[o] = 0.f;

    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int tw = t % ntile_w, th = (t / ntile_w) % ntile_h, b = t / (ntile_w * ntile_h);
        const int oh0 = th * C::TH, ow0 = tw * C::TW;
        const int ih0 = oh0 - L.PH, iw0 = ow0 - L.PW;
        __syncthreads();
        {
            const int r = tid / C::TW, col = tid % C::TW;
            const int oh = oh0 + r, ow = ow0 + col;
            const bool in = (oh < L.Ho) && (ow < L.Wo);
#pragma unroll
            for (int o = 0; o < COUT; ++o) {
                float gN = 0.f, gD = 0.f;
                if (in) {
                    const size_t i = plane_idx(b, o, COUT, L.Ho, L.Wo, oh, ow);
                    const float gy = a.gy[i], co = a.co[i];
                    const float gco = a.gco ? a.gco[i] : 0.f;
                    nconv_grad_nd(gy, gco, a.y[i], co, L.eps, L.bias[o], L.wsum[o], gN, gD);
                    gb_acc[o] += gy;
                    gs_acc[o] = fmaf(gco, co, gs_acc[o]);
                }
                sg[o * C::GPL + tid] = (f2){gN, gD};
            }
        }
        for (int e = tid; e < CIN * C::IHT * C::IWT; e += kT) {
            const int ci = e / (C::IHT * C::IWT);
            const int rem = e - ci * (C::IHT * C::IWT);
            const int r = rem / C::IWT, col = rem - r * C::IWT;
            const int ih = ih0 + r, iw = iw0 + col;
            float x = 0.f, c = 0.f;
            if ((unsigned)ih < (unsigned)L.H && (unsigned)iw < (unsigned)L.W) load_xc<MODE>(d, b, ci, ih, iw, x, c);
            sin[ci * C::IPL + r * C::IWT + col] = (f2){x * c, c};
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < C::NPASS; ++p) {
            const int cb = tid + p * kT;
            if (cb < C::NCB) {
                const int i = cb % CIN, o = (cb / CIN) % COUT, kh = cb / (CIN * COUT);
                for (int r = 0; r < C::TH; ++r) {
                    const f2* ir = sin + i * C::IPL + (r + kh) * C::IWT;
                    const f2* gr = sg + o * C::GPL + r * C::TW;
                    f2 win[K];
#pragma unroll
                    for (int k = 0; k < K - 1; ++k) win[k] = ir[k];
#pragma unroll 16
                    for (int col = 0; col < C::TW; ++col) {
                        win[K - 1] = ir[col + K - 1];
                        const f2 g = gr[col];
#pragma unroll
                        for (int k = 0; k < K; ++k) acc[p][k] = __builtin_elementwise_fma(win[k], g, acc[p][k]);
#pragma unroll
                        for (int k = 0; k < K - 1; ++k) win[k] = win[k + 1];
                    }
                }
            }
        }
    }

    // partial[blk] = { gW-partial[COUT*CIN*K*K], sum gy[COUT], sum gco*cout[COUT] }
    float* out = part + (size_t)blockIdx.x * (COUT * CIN * K * K + 2 * COUT);
#pragma unroll
    for (int p = 0; p < C::NPASS; ++p) {
        const int cb = tid + p * kT;
        if (cb < C::NCB) {
            const int i = cb % CIN, o = (cb / CIN) % COUT, kh = cb / (CIN * COUT);
#pragma unroll
            for (int k = 0; k < K; ++k) out[((o * CIN + i) * K + kh) * K + k] = acc[p][k].x + acc[p][k].y;
        }
    }
    // block reduction of gb / gs in a fixed order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
        red[o * kT + tid] = gb_acc[o];
        red[(COUT + o) * kT + tid] = gs_acc[o];
    }
    __syncthreads();
    if (tid < 2 * COUT) {
        float s = 0.f;
        for (int k = 0; k < kT; ++k) s += red[tid * kT + k];
        out[COUT * CIN * K * K + tid] = s;
    }
}

// ---- wgrad: generic partial sums (any stride / dilation / groups) -----------------------------------
// grid = (nchunk, n_weight + 2*Cout): blockIdx.y selects a weight element (or a gb / gs sum),
// blockIdx.x a contiguous chunk of the (b, oh, ow) reduction domain.
template <int MODE>
__global__ __launch_bounds__(kT) void wgrad_generic(LayerDev d, BwdArgs a, float* part, int nchunk) {
    const nconv_layer& L = d.L;
    const int cpg_in = L.Cin / L.groups, cpg_out = L.Cout / L.groups;
    const int fan = cpg_in * L.KH * L.KW;
    const int nw = L.Cout * fan;
    const int widx = blockIdx.y;
    const size_t np = (size_t)L.B * L.Ho * L.Wo;
    const size_t per = (np + nchunk - 1) / nchunk;
    const size_t p0 = (size_t)blockIdx.x * per, p1 = p0 + per < np ? p0 + per : np;
    int o, cl = 0, kh = 0, kw = 0, kind;  // kind 0: weight, 1: gb, 2: gs
    if (widx < nw) {
        kind = 0;
        o = widx / fan;
        int r = widx - o * fan;
        cl = r / (L.KH * L.KW);
        r -= cl * L.KH * L.KW;
        kh = r / L.KW;
        kw = r - kh * L.KW;
    } else if (widx < nw + L.Cout) {
        kind = 1;
        o = widx - nw;
    } else {
        kind = 2;
        o = widx - nw - L.Cout;
    }
    const int ci = (o / cpg_out) * cpg_in + cl;
    const float bo = L.bias[o], so = L.wsum[o];
    float acc = 0.f;
    for (size_t p = p0 + threadIdx.x; p < p1; p += kT) {
        const int ow = (int)(p % L.Wo), oh = (int)((p / L.Wo) % L.Ho), b = (int)(p / ((size_t)L.Wo * L.Ho));
        const size_t i = plane_idx(b, o, L.Cout, L.Ho, L.Wo, oh, ow);
        const float gy = a.gy[i], gco = a.gco ? a.gco[i] : 0.f;
        if (kind == 1) { acc += gy; continue; }
        if (kind == 2) { acc = fmaf(gco, a.co[i], acc); continue; }
        const int ih = oh * L.SH - L.PH + kh * L.DH, iw = ow * L.SW - L.PW + kw * L.DW;
        if ((unsigned)ih >= (unsigned)L.H || (unsigned)iw >= (unsigned)L.W) continue;
        float gN, gD, x, c;
        nconv_grad_nd(gy, gco, a.y[i], a.co[i], L.eps, bo, so, gN, gD);
        load_xc<MODE>(d, b, ci, ih, iw, x, c);
        acc = fmaf(x * c, gN, acc);
        acc = fmaf(c, gD, acc);
    }
    __shared__ float red[kT];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = kT / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[(size_t)blockIdx.x * (nw + 2 * L.Cout) + widx] = red[0];
}

// ---- wgrad: fixed-order reduction of the per-block partials ----------------------------------------
__global__ __launch_bounds__(kT) void wgrad_reduce(const float* part, int nblk, int nw, int cout, int fan,
                                                   const float* wsum, float* gw, float* gb) {
    const int stride = nw + 2 * cout;
    for (int w = blockIdx.x * kT + threadIdx.x; w < nw + cout; w += gridDim.x * kT) {
        if (w < nw) {
            const int o = w / fan;
            float s = 0.f, gsum = 0.f;
            for (int k = 0; k < nblk; ++k) {
                s += part[(size_t)k * stride + w];
                gsum += part[(size_t)k * stride + nw + cout + o];
            }
            const float so = wsum[o];
            const float gs = -gsum / so;  // d/ds of cout = D/s, summed: -sum gco*D/s^2 = -sum(gco*cout)/s
            if (gw) gw[w] = s + gs;
        } else {
            const int o = w - nw;
            float s = 0.f;
            for (int k = 0; k < nblk; ++k) s += part[(size_t)k * stride + nw + o];
            if (gb) gb[o] = s;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------------
static int last_err(const char** why) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

static bool simple_geom(const nconv_layer& L) {
    return L.SH == 1 && L.SW == 1 && L.DH == 1 && L.DW == 1 && L.groups == 1 && L.KH == L.KW;
}

constexpr int kMaxWgBlocks = 1024;

enum Path { kTiled, kGeneric };

static Path pick_path(const nconv_layer& L) {
    if (!simple_geom(L)) return kGeneric;
    const int m = L.load_mode;
    if ((L.Cin == 1 && L.Cout == 8 && L.KH == 5 && m == NCONV_LOAD_THRESH) ||
        (L.Cin == 8 && L.Cout == 8 && L.KH == 5 && (m == NCONV_LOAD_PLAIN || m == NCONV_LOAD_POOL2)) ||
        (L.Cin == 16 && L.Cout == 8 && L.KH == 3 &&
         (m == NCONV_LOAD_UPCAT_SKIP_FIRST || m == NCONV_LOAD_UPCAT_UP_FIRST)) ||
        (L.Cin == 8 && L.Cout == 1 && L.KH == 1 && m == NCONV_LOAD_PLAIN))
        return kTiled;
    return kGeneric;
}

static int generic_chunks(const nconv_layer& L) {
    const size_t np = (size_t)L.B * L.Ho * L.Wo;
    size_t c = (np + 65535) / 65536;
    if (c < 1) c = 1;
    if (c > 64) c = 64;
    return (int)c;
}

static size_t wg_blocks(const nconv_layer& L) {
    const size_t nt = (size_t)((L.Wo + 63) / 64) * ((L.Ho + 3) / 4) * L.B;
    return nt < kMaxWgBlocks ? nt : kMaxWgBlocks;
}

size_t bwd_workspace_bytes(const LayerDev& d) {
    const nconv_layer& L = d.L;
    const int fan = (L.Cin / L.groups) * L.KH * L.KW;
    const size_t stride = (size_t)L.Cout * fan + 2 * L.Cout;
    const size_t nblk = pick_path(L) == kTiled ? wg_blocks(L) : (size_t)generic_chunks(L);
    size_t bytes = nblk * stride * sizeof(float);
    bytes = (bytes + 255) & ~(size_t)255;
    if (L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST)
        bytes += 2 * (size_t)L.B * L.b.C * L.H * L.W * sizeof(float);
    return bytes;
}

template <int CIN, int COUT, int K, int MODE>
static void go_bwd_tiled(const LayerDev& d, const BwdArgs& a, float* part, float* tx, float* tc,
                         hipStream_t st) {
    const nconv_layer& L = d.L;
    using D = DgCfg<CIN, K>;
    if (a.gxa || a.gca || a.gxb || a.gcb) {
        dim3 g((L.W + D::TW - 1) / D::TW, (L.H + D::TH - 1) / D::TH, L.B);
        hipLaunchKernelGGL((dgrad_tiled<CIN, COUT, K, MODE>), g, dim3(kT), 0, st, d, a, tx, tc);
    }
    if (a.gw || a.gb) {
        using W = WgCfg<CIN, COUT, K>;
        const int ntw = (L.Wo + W::TW - 1) / W::TW, nth = (L.Ho + W::TH - 1) / W::TH;
        const int nblk = (int)wg_blocks(L);
        size_t lds = (size_t)W::LDS_F2 * sizeof(f2);
        const size_t red = (size_t)2 * COUT * kT * sizeof(float);
        if (red > lds) lds = red;
        hipLaunchKernelGGL((wgrad_tiled<CIN, COUT, K, MODE>), dim3(nblk), dim3(kT), lds, st, d, a, part, ntw, nth);
        const int nw = COUT * CIN * K * K;
        hipLaunchKernelGGL(wgrad_reduce, dim3((nw + COUT + kT - 1) / kT), dim3(kT), 0, st, part, nblk, nw, COUT,
                           CIN * K * K, L.wsum, a.gw, a.gb);
    }
}

template <int MODE>
static void go_bwd_generic(const LayerDev& d, const BwdArgs& a, float* part, float* tx, float* tc,
                           hipStream_t st) {
    const nconv_layer& L = d.L;
    if (a.gxa || a.gca || a.gxb || a.gcb) {
        const size_t n = (size_t)L.B * L.Cin * L.H * L.W;
        size_t blocks = (n + kT - 1) / kT;
        if (blocks > (1u << 20)) blocks = 1u << 20;
        if (blocks) hipLaunchKernelGGL(dgrad_generic<MODE>, dim3(blocks), dim3(kT), 0, st, d, a, tx, tc);
    }
    if (a.gw || a.gb) {
        const int fan = (L.Cin / L.groups) * L.KH * L.KW;
        const int nw = L.Cout * fan;
        const int nchunk = generic_chunks(L);
        hipLaunchKernelGGL(wgrad_generic<MODE>, dim3(nchunk, nw + 2 * L.Cout), dim3(kT), 0, st, d, a, part, nchunk);
        hipLaunchKernelGGL(wgrad_reduce, dim3((nw + L.Cout + kT - 1) / kT), dim3(kT), 0, st, part, nchunk, nw,
                           L.Cout, fan, L.wsum, a.gw, a.gb);
    }
}

int launch_bwd(const LayerDev& d, const BwdArgs& a, hipStream_t st, const char** why) {
    const nconv_layer& L = d.L;
    if (a.ws_bytes < bwd_workspace_bytes(d)) {
        *why = "workspace too small (see nconv_bwd_workspace_bytes)";
        return -22;
    }
    const int fan = (L.Cin / L.groups) * L.KH * L.KW;
    const size_t stride = (size_t)L.Cout * fan + 2 * L.Cout;
    const Path path = pick_path(L);
    const size_t nblk = path == kTiled ? wg_blocks(L) : (size_t)generic_chunks(L);
    float* part = a.ws;
    float* tx = a.ws + (((nblk * stride * sizeof(float)) + 255) & ~(size_t)255) / sizeof(float);
    float* tc = tx + (size_t)L.B * L.b.C * L.H * L.W;
    const bool up = L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;

    if (path == kTiled) {
        const int m = L.load_mode;
        if (L.Cin == 1 && m == NCONV_LOAD_THRESH) go_bwd_tiled<1, 8, 5, NCONV_LOAD_THRESH>(d, a, part, tx, tc, st);
        else if (L.Cin == 8 && L.Cout == 8 && m == NCONV_LOAD_PLAIN) go_bwd_tiled<8, 8, 5, NCONV_LOAD_PLAIN>(d, a, part, tx, tc, st);
        else if (L.Cin == 8 && L.Cout == 8 && m == NCONV_LOAD_POOL2) go_bwd_tiled<8, 8, 5, NCONV_LOAD_POOL2>(d, a, part, tx, tc, st);
        else if (m == NCONV_LOAD_UPCAT_SKIP_FIRST) go_bwd_tiled<16, 8, 3, NCONV_LOAD_UPCAT_SKIP_FIRST>(d, a, part, tx, tc, st);
        else if (m == NCONV_LOAD_UPCAT_UP_FIRST) go_bwd_tiled<16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST>(d, a, part, tx, tc, st);
        else go_bwd_tiled<8, 1, 1, NCONV_LOAD_PLAIN>(d, a, part, tx, tc, st);
    } else {
        switch (L.load_mode) {
            case NCONV_LOAD_PLAIN: go_bwd_generic<NCONV_LOAD_PLAIN>(d, a, part, tx, tc, st); break;
            case NCONV_LOAD_THRESH: go_bwd_generic<NCONV_LOAD_THRESH>(d, a, part, tx, tc, st); break;
            case NCONV_LOAD_POOL2: go_bwd_generic<NCONV_LOAD_POOL2>(d, a, part, tx, tc, st); break;
            case NCONV_LOAD_UPCAT_SKIP_FIRST: go_bwd_generic<NCONV_LOAD_UPCAT_SKIP_FIRST>(d, a, part, tx, tc, st); break;
            case NCONV_LOAD_UPCAT_UP_FIRST: go_bwd_generic<NCONV_LOAD_UPCAT_UP_FIRST>(d, a, part, tx, tc, st); break;
            default: *why = "unknown load mode"; return -22;
        }
    }
    if (up && (a.gxb || a.gcb)) {
        const size_t n = (size_t)L.B * L.b.C * L.b.H * L.b.W;
        size_t blocks = (n + kT - 1) / kT;
        if (blocks > (1u << 20)) blocks = 1u << 20;
        if (blocks) hipLaunchKernelGGL(upsample_bwd_gather, dim3(blocks), dim3(kT), 0, st, d, tx, tc, a.gxb, a.gcb);
    }
    return last_err(why);
}

}  // namespace nconv
