// nconv_route.h — the input gradient's epilogue: from a layer-input pixel's {G_xc, G_c} to the
// producer tensors through the glue's backward (shared by dgrad_tiled and dgrad_bf).
#pragma once
#include "nconv_common.h"
#include "nconv_internal.h"

namespace nconv {

// ---- gradient routing from a layer-input pixel to the producer tensors --------------------------
// a.accumulate != 0: += into the outputs; == 0: overwrite (every element of every requested output
// is written exactly once, so the caller need not zero-fill; see pool_zero_leftovers).
__device__ __forceinline__ void put(float* p, size_t i, float v, bool acc) {
    if (acc) p[i] += v;
    else p[i] = v;
}

template <int MODE>
__device__ __forceinline__ void route_grad(const LayerDev& d, const BwdArgs& a, int b, int ci, int ih,
                                           int iw, float gxc, float gc_direct, float* tmp_x,
                                           float* tmp_c) {
    const nconv_layer& L = d.L;
    const bool acc = a.accumulate != 0;
    if constexpr (MODE == NCONV_LOAD_PLAIN) {
        const size_t i = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, ih, iw);
        const float x = L.a.x[i], c = L.a.c[i];
        if (a.gxa) put(a.gxa, i, gxc * c, acc);
        if (a.gca) put(a.gca, i, gc_direct + gxc * x, acc);
    } else if constexpr (MODE == NCONV_LOAD_THRESH) {
        const size_t i = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, ih, iw);
        const float x = L.a.x[i];
        const float c = (x > L.thresh) ? 1.0f : 0.0f;
        if (a.gxa) put(a.gxa, i, gxc * c, acc);  // c = (S > thr) carries no gradient
    } else if constexpr (MODE == NCONV_LOAD_POOL2) {
        const size_t i0 = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, 2 * ih, 2 * iw);
        const size_t W2 = (size_t)L.a.W;
        const size_t off[4] = {0, 1, W2, W2 + 1};
        int ax, ac;
        const float x = pool4(L.a.x[i0], L.a.x[i0 + 1], L.a.x[i0 + W2], L.a.x[i0 + W2 + 1], ax);
        const float c = pool4(L.a.c[i0], L.a.c[i0 + 1], L.a.c[i0 + W2], L.a.c[i0 + W2 + 1], ac);
        const float gx = gxc * c, gc = gc_direct + gxc * x;
        if (acc) {
            if (a.gxa) a.gxa[i0 + off[ax]] += gx;
            if (a.gca) a.gca[i0 + off[ac]] += gc;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (a.gxa) a.gxa[i0 + off[k]] = (k == ax) ? gx : 0.f;
                if (a.gca) a.gca[i0 + off[k]] = (k == ac) ? gc : 0.f;
            }
        }
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
            if (a.gxa) put(a.gxa, i, gx, acc);
            if (a.gca) put(a.gca, i, gc, acc);
        } else {
            const int cb = skip_first ? ci - first_c : ci;
            const size_t i = plane_idx(b, cb, L.b.C, L.H, L.W, ih, iw);
            tmp_x[i] = gx;
            tmp_c[i] = gc;
        }
    }
}

// Overwrite mode, POOL2: source rows/cols that no 2x2 window covers (odd source H or W) get 0.
__device__ __forceinline__ void pool_zero_leftovers(const LayerDev& d, const BwdArgs& a, int b, int ci, int ih,
                                                    int iw) {
    const nconv_layer& L = d.L;
    const bool oddh = (L.a.H & 1) && ih == L.H - 1, oddw = (L.a.W & 1) && iw == L.W - 1;
    if (!(oddh || oddw)) return;
    const size_t base = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, 0, 0);
    auto z = [&](int h, int w) {
        if (a.gxa) a.gxa[base + (size_t)h * L.a.W + w] = 0.f;
        if (a.gca) a.gca[base + (size_t)h * L.a.W + w] = 0.f;
    };
    if (oddh) { z(L.a.H - 1, 2 * iw); z(L.a.H - 1, 2 * iw + 1); }
    if (oddw) { z(2 * ih, L.a.W - 1); z(2 * ih + 1, L.a.W - 1); }
    if (oddh && oddw) z(L.a.H - 1, L.a.W - 1);
}

// Four adjacent input pixels (iw .. iw+3, the first nv of them in range) of channel ci, row ih:
// gx = G_xc*c, gc = G_c + G_xc*x routed as route_grad, 16-byte loads and stores where the row
// allows (direct and concatenated full-resolution channels).
template <int MODE>
__device__ __forceinline__ void dg_route4(const LayerDev& d, const BwdArgs& a, int b, int ci, int ih, int iw, int nv,
                                          const float (&gxc)[4], const float (&gcd)[4], float* tmp_x, float* tmp_c) {
    const nconv_layer& L = d.L;
    const bool acc = a.accumulate != 0;
    if constexpr (MODE == NCONV_LOAD_POOL2 || MODE == NCONV_LOAD_THRESH) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < nv) {
                route_grad<MODE>(d, a, b, ci, ih, iw + j, gxc[j], gcd[j], tmp_x, tmp_c);
                if (MODE == NCONV_LOAD_POOL2 && !acc) pool_zero_leftovers(d, a, b, ci, ih, iw + j);
            }
    } else {
        const ChanSrc s = chan_src<MODE>(d, b, ci);
        const bool vec = nv == 4 && (L.W & 3) == 0 && (iw & 3) == 0;
        if (!vec) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < nv) route_grad<MODE>(d, a, b, ci, ih, iw + j, gxc[j], gcd[j], tmp_x, tmp_c);
            return;
        }
        float x[4], c[4];
        if (s.kind == kUp) {
#pragma unroll
            for (int j = 0; j < 4; ++j) load_chan(d, s, ih, iw + j, x[j], c[j]);
        } else {
            const f4 xv = *reinterpret_cast<const f4*>(s.x + (size_t)ih * s.W + iw);
            const f4 cv = *reinterpret_cast<const f4*>(s.c + (size_t)ih * s.W + iw);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                x[j] = xv[j];
                c[j] = cv[j];
            }
        }
        f4 gxv, gcv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            gxv[j] = gxc[j] * c[j];
            gcv[j] = gcd[j] + gxc[j] * x[j];
        }
        float *gxp, *gcp;
        size_t off;
        bool acc_here = acc;
        if (s.kind == kUp) {  // upsampled channel: staged for upsample_bwd_gather
            const int cb = (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST) ? ci - L.a.C : ci;
            off = plane_idx(b, cb, L.b.C, L.H, L.W, ih, iw);
            gxp = tmp_x;
            gcp = tmp_c;
            acc_here = false;
        } else {
            const int ca = (MODE == NCONV_LOAD_UPCAT_UP_FIRST) ? ci - L.b.C : ci;
            off = plane_idx(b, ca, L.a.C, L.a.H, L.a.W, ih, iw);
            gxp = a.gxa;
            gcp = a.gca;
        }
        if (gxp) {
            f4* p = reinterpret_cast<f4*>(gxp + off);
            *p = acc_here ? *p + gxv : gxv;
        }
        if (gcp) {
            f4* p = reinterpret_cast<f4*>(gcp + off);
            *p = acc_here ? *p + gcv : gcv;
        }
    }
}

}  // namespace nconv
