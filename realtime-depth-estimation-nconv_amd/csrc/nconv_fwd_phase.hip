// nconv_fwd_phase.hip — exact-fp32 forward of the upsample-concat 3x3 NConv layers (nconv4, nconv5,
// nconv6 [+ nconv7 tail]) with the nearest-2x-upsampled input channels convolved at their native
// resolution (reference: models/step1.py:78-90, cat((x, F.interpolate(x_low, nearest)), 1) followed
// by NConv2d.forward, :116-149).
//
// Half of such a layer's input channels are up(low): every 2x2 block of the upsampled plane holds
// one low-resolution value. A 3x3 window over up(low) therefore touches only a 2x2 block of low
// pixels, and which taps land on which low pixel depends only on the parity ("phase") of the
// window's first input row / column:
//     first index even:  taps {0,1} -> low pixel m,   tap {2}   -> m + 1
//     first index odd:   tap  {0}   -> low pixel m,   taps {1,2} -> m + 1
// so  sum_{kh,kw} W[kh][kw] * up(v)[ih0+kh][iw0+kw] = sum_{dh,dw} Wp[a][b][dh][dw] * v[m+dh][n+dw]
// with the phase weights Wp (sums of 1, 2 or 4 of the layer's fp32 weights, nconv_phase_weights).
// All arithmetic stays fp32: regrouping w_a*v + w_b*v as (w_a + w_b)*v is a reassociation whose
// error lies inside the usual fp32 dot-product bound (gamma_n * sum |w||v|), unlike a Winograd
// transform, whose error is relative to a whole tile's largest term. The upsampled half then costs
// 4 instead of 9 packed FMAs per pixel and channel (the layer: 208 instead of 288 per pixel pair
// and output channel over 16 inputs) and is staged at a quarter of the pixels.
//
// Tiling as fwd_tiled (256 threads, 16x32 output tile, 2 px per thread, all 8 output channels per
// thread), with one difference: a wave owns four rows of one parity (rows w&1, w&1 + 2, ... of its
// 8-row half), so the phase -- and with it the phase weights -- is wave-uniform and the weights
// ride the scalar cache.
#include "nconv_prologue.h"

namespace nconv {

namespace {

constexpr int kPT = 256, kPTH = 16, kPTW = 32, kPK = 3, kPCO = 8, kPCA = 8, kPCB = 8;
constexpr int kPIH = kPTH + kPK - 1, kPIW = kPTW + kPK - 1;  // native planes: 18 x 34
constexpr int kPIWP = (kPIW + 1) & ~1;
constexpr int kPLH = kPTH / 2 + 2, kPLW = kPTW / 2 + 2;   // low-resolution planes: 10 x 18
constexpr int kPLP = kPLW;
constexpr int kPLStride = kPLH * kPLP + 2;               // + dump slot (threads past the tile)

typedef const float __attribute__((address_space(4))) cfloat;

// One low-resolution plane of source b: thread tid < kPLH * kPLW owns element (tid / kPLW,
// tid % kPLW) of the tile whose origin is (lr0, lc0) in the low plane; outside the plane -> 0
struct LowStager {
    unsigned off;  // byte offset in the plane, or OOB
    int slot;
    __device__ __forceinline__ void init(const nconv_layer& L, int lr0, int lc0, int tid) {
        const int r = tid / kPLW, c = tid - (tid / kPLW) * kPLW;
        const int gr = lr0 + r, gc = lc0 + c;
        const bool in = tid < kPLH * kPLW && (unsigned)gr < (unsigned)L.b.H && (unsigned)gc < (unsigned)L.b.W;
        off = in ? (unsigned)(gr * L.b.W + gc) * 4u : 0x80000000u;
        slot = tid < kPLH * kPLW ? r * kPLP + c : kPLH * kPLP;
    }
    __device__ __forceinline__ void load(const LayerDev& d, int b, int cb, float& x, float& c) const {
        const nconv_layer& L = d.L;
        const size_t base = ((size_t)b * L.b.C + cb) * (size_t)L.b.H * L.b.W;
        const int bytes = L.b.H * L.b.W * 4;
        x = ld_f32(plane_rsrc(L.b.x + base, bytes), off);
        c = ld_f32(plane_rsrc(L.b.c + base, bytes), off);
    }
    __device__ __forceinline__ void store(f2* t, float x, float c) const { t[slot] = (f2){x * c, c}; }
};

// native-resolution planes come from source a (PLAIN load of a's channels)
template <int MODE>
__device__ __forceinline__ ChanSrc native_src(const LayerDev& d, int b, int ca) {
    const nconv_layer& L = d.L;
    ChanSrc s;
    const size_t off = ((size_t)b * L.a.C + ca) * (size_t)L.a.H * L.a.W;
    s.x = L.a.x + off;
    s.c = L.a.c + off;
    s.W = L.a.W;
    s.kind = kDirect;
    s.bytes = L.a.H * L.a.W * 4;
    return s;
}

// PAR = (output-grid origin offset - padding) & 1: the parity of the first input row / column of
// the windows of even output rows / columns (nconv4 / nconv5: padding 1 -> 1; the tail: nconv6
// padding 0 computed from grid offset -1 -> 1).
template <int MODE, bool TAIL, int PAR>
__global__ __launch_bounds__(kPT) void fwd_phase(LayerDev d, float* __restrict__ y, float* __restrict__ yc,
                                                 TailArgs t) {
    using TS = TileStager<kPIH, kPIW, kPIWP, NCONV_LOAD_PLAIN, kPT>;
    constexpr int kStride = TS::PLANE_STRIDE;
    constexpr bool SKIP_FIRST = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST;  // channel order: [a, up(b)]
    __shared__ __attribute__((aligned(16))) f2 tile[2 * kStride];
    __shared__ __attribute__((aligned(16))) f2 low[2 * kPLStride];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int gh = TAIL ? t.out_h : L.Ho, gw = TAIL ? t.out_w : L.Wo;
    const TileCoord tc = xcd_tile((gw + kPTW - 1) / kPTW, (gh + kPTH - 1) / kPTH, L.B);
    const int b = tc.b;
    const int R0 = tc.ty * kPTH, C0 = tc.tx * kPTW;
    const int off = TAIL ? t.off : 0;
    const int oh0 = R0 + off, ow0 = C0 + off;  // tile origin in this layer's output grid
    const int ih0 = oh0 - L.PH, iw0 = ow0 - L.PW;
    // wave w: rows (w >> 1) * 8 + (w & 1) + 2 g, g = lane >> 4: one row parity per wave
    const int g = lane >> 4, jx = lane & 15;
    const int ty = (w >> 1) * 8 + (w & 1) + 2 * g, tx = 2 * jx;
    const int alpha = __builtin_amdgcn_readfirstlane((PAR + (w & 1)) & 1);  // row phase of this wave

    f2 acc[kPCO][2];
#pragma unroll
    for (int o = 0; o < kPCO; ++o) acc[o][0] = acc[o][1] = (f2){0.f, 0.f};

    // ---- native channels: 3x3 over the full-resolution plane (as fwd_tiled) ----
    const int cbase_a = SKIP_FIRST ? 0 : kPCB;  // weight channel index of a's channel 0
    const float* __restrict__ wgt = L.weight;
    const f2* rowbase = &tile[ty * kPIWP + tx];
    auto fma_native = [&](int ca, int bufi) {
        const f2* row = rowbase + bufi * kStride;
        const float* wr = wgt + (size_t)(cbase_a + ca) * kPK * kPK;
#pragma unroll 1
        for (int q = 0; q < kPK; ++q, row += kPIWP, wr += kPK) {
            f2 v[4];
            const f4 q0 = reinterpret_cast<const f4*>(row)[0], q1 = reinterpret_cast<const f4*>(row)[1];
            v[0] = q0.xy; v[1] = q0.zw; v[2] = q1.xy; v[3] = q1.zw;
#pragma unroll
            for (int kw = 0; kw < kPK; ++kw)
#pragma unroll
                for (int o = 0; o < kPCO; ++o) {
                    const float wv = wr[o * (kPCA + kPCB) * kPK * kPK + kw];
                    const f2 w2 = (f2){wv, wv};
                    acc[o][0] = __builtin_elementwise_fma(w2, v[kw], acc[o][0]);
                    acc[o][1] = __builtin_elementwise_fma(w2, v[kw + 1], acc[o][1]);
                }
        }
    };

    // ---- upsampled channels: 2x2 phase taps over the low-resolution plane ----
    // low row of dh = 0 and the pixel pair's low columns: jx .. jx + 1 (pixel 0) and
    // jx + PAR .. jx + PAR + 1 (pixel 1); column phases beta0 = PAR, beta1 = 1 - PAR
    const f2* lowbase = &low[((ty + PAR) >> 1) * kPLP + jx];
    // phase weights: [i][alpha][dh][o][beta][dw] (nconv_phase_weights), 32 floats per (i, alpha, dh)
    const cfloat* wph = (const cfloat*)L.waux;
    auto fma_up = [&](int cb, int bufi) {
        const f2* row = lowbase + bufi * kPLStride;
        const cfloat* wr = wph + ((size_t)cb * 2 + alpha) * 2 * 32;
#pragma unroll 1
        for (int dh = 0; dh < 2; ++dh, row += kPLP, wr += 32) {
            f2 v[3];
            v[0] = row[0];
            v[1] = row[1];
            v[2] = row[2];
#pragma unroll
            for (int o = 0; o < kPCO; ++o)
#pragma unroll
                for (int dw = 0; dw < 2; ++dw) {
                    const float w0 = wr[o * 4 + PAR * 2 + dw];        // pixel 0: beta = PAR
                    const float w1 = wr[o * 4 + (1 - PAR) * 2 + dw];  // pixel 1: beta = 1 - PAR
                    acc[o][0] = __builtin_elementwise_fma((f2){w0, w0}, v[dw], acc[o][0]);
                    acc[o][1] = __builtin_elementwise_fma((f2){w1, w1}, v[PAR + dw], acc[o][1]);
                }
        }
    };

    TS ts;
    ts.init(d, ih0, iw0, tid);
    LowStager ls;
    ls.init(L, (oh0 - L.PH) >> 1, (ow0 - L.PW) >> 1, tid);
    // the first two low planes fly during the whole native phase (one element per thread each)
    float lx0, lc0_, lx1, lc1;
    ls.load(d, b, 0, lx0, lc0_);
    ls.load(d, b, 1, lx1, lc1);
    {
        float xa[TS::NE], ca[TS::NE], xb[TS::NE], cb[TS::NE];
        ts.load(native_src<MODE>(d, b, 0), xa, ca);
        ts.load(native_src<MODE>(d, b, 1), xb, cb);
#pragma unroll 1
        for (int ci = 0; ci < kPCA; ci += 2) {
            ts.store(tile, xa, ca, 0.f);
            __syncthreads();
            ts.load(native_src<MODE>(d, b, ci + 2 < kPCA ? ci + 2 : kPCA - 1), xa, ca);
#ifndef NCONV_PHASE_PROBE_NO_NATIVE  // timing probe only (wrong results): no native-half FMAs
            fma_native(ci, 0);
#endif
            ts.store(tile + kStride, xb, cb, 0.f);
            __syncthreads();
            ts.load(native_src<MODE>(d, b, ci + 3 < kPCA ? ci + 3 : kPCA - 1), xb, cb);
#ifndef NCONV_PHASE_PROBE_NO_NATIVE
            fma_native(ci + 1, 1);
#endif
        }
    }
#pragma unroll 1
    for (int ci = 0; ci < kPCB; ci += 2) {
        ls.store(low, lx0, lc0_);
        __syncthreads();
        ls.load(d, b, ci + 2 < kPCB ? ci + 2 : kPCB - 1, lx0, lc0_);
#ifndef NCONV_PHASE_PROBE_NO_UP  // timing probe only (wrong results): no upsampled-half FMAs
        fma_up(ci, 0);
#endif
        ls.store(low + kPLStride, lx1, lc1);
        __syncthreads();
        ls.load(d, b, ci + 3 < kPCB ? ci + 3 : kPCB - 1, lx1, lc1);
#ifndef NCONV_PHASE_PROBE_NO_UP
        fma_up(ci + 1, 1);
#endif
    }

    // ---- epilogue ----
    const int oh = oh0 + ty;
    if constexpr (!TAIL) {
        // per-plane buffer stores (as fwd_tiled): offsets past the plane are dropped
        constexpr unsigned OOB = 0x80000000u;
        const int ow = ow0 + tx;
        const size_t plane = (size_t)L.Ho * L.Wo;
        const int pbytes = (int)(plane * 4);
        unsigned so[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) so[j] = (oh < L.Ho && ow + j < L.Wo) ? (unsigned)(oh * L.Wo + ow + j) * 4u : OOB;
        const bool vec = (L.Wo % 2) == 0 && ow + 1 < L.Wo && oh < L.Ho;
#pragma unroll
        for (int o = 0; o < kPCO; ++o) {
            float yv[2], cv[2];
            const float s = L.wsum[o], bo = L.bias[o];
#pragma unroll
            for (int j = 0; j < 2; ++j) nconv_epilogue(acc[o][j].x, acc[o][j].y, L.eps, bo, s, yv[j], cv[j]);
            const size_t ofs = ((size_t)b * kPCO + o) * plane;
            const __amdgpu_buffer_rsrc_t ry = plane_rsrc(y + ofs, pbytes), rc = plane_rsrc(yc + ofs, pbytes);
            if (vec) {
                st_f2(ry, so[0], (f2){yv[0], yv[1]});
                st_f2(rc, so[0], (f2){cv[0], cv[1]});
            } else {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    st_f32(ry, so[j], yv[j]);
                    st_f32(rc, so[j], cv[j]);
                }
            }
        }
    } else {
        // nconv6 outputs -> nconv7 (1x1, 8 -> 1) -> cropped final output (as fwd_tiled's tail)
        const int r = R0 + ty;
        if (r >= t.out_h) return;
        const float b7 = t.b7[0], s7 = t.s7[0];
        float ov[2], oc[2];
        // nconv6's outputs -> nconv7's sums (o ascending, as nconv7's own kernel); with t.y6
        // (training) nconv6's outputs are stored too, two pixels per 8-byte store
        constexpr unsigned OOB = 0x80000000u;
        const int owb = ow0 + tx;
        bool inj[2];
        unsigned so[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            inj[j] = (unsigned)oh < (unsigned)L.Ho && (unsigned)(owb + j) < (unsigned)L.Wo;
            so[j] = inj[j] ? (unsigned)(oh * L.Wo + owb + j) * 4u : OOB;
        }
        const bool vec = (L.Wo % 2) == 0 && inj[0] && inj[1];
        const int pbytes = L.Ho * L.Wo * 4;
        float N7[2] = {0.f, 0.f}, D7[2] = {0.f, 0.f};
#pragma unroll
        for (int o = 0; o < kPCO; ++o) {
            float y6[2], c6[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                nconv_epilogue(acc[o][j].x, acc[o][j].y, L.eps, L.bias[o], L.wsum[o], y6[j], c6[j]);
                if (inj[j]) {
                    N7[j] = fmaf(t.w7[o], y6[j] * c6[j], N7[j]);
                    D7[j] = fmaf(t.w7[o], c6[j], D7[j]);
                }
            }
            if (t.y6) {  // training: each pixel of nconv6 lies in exactly one tile
                const size_t ofs = ((size_t)b * kPCO + o) * L.Ho * L.Wo;
                const __amdgpu_buffer_rsrc_t ry = plane_rsrc(t.y6 + ofs, pbytes), rc = plane_rsrc(t.c6 + ofs, pbytes);
                if (vec) {
                    st_f2(ry, so[0], (f2){y6[0], y6[1]});
                    st_f2(rc, so[0], (f2){c6[0], c6[1]});
                } else {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        st_f32(ry, so[j], y6[j]);
                        st_f32(rc, so[j], c6[j]);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            nconv_epilogue(N7[j], D7[j], t.eps7, b7, s7, ov[j], oc[j]);
        }
        const size_t base = ((size_t)b * t.out_h + r) * t.out_w + C0 + tx;
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (C0 + tx + j < t.out_w) {
                y[base + j] = ov[j];
                if (t.out_c) t.out_c[base + j] = oc[j];
            }
    }
}

// Phase weights of n UPCAT layers (PhaseArgs, phase_block: nconv_prologue.h), one block per layer.
__global__ __launch_bounds__(kPrepThreads) void phase_weights(PhaseArgs a) {
    const int l = blockIdx.x;
    phase_block(a.w[l], a.cin[l], a.ci0[l], a.out[l]);
}

}  // namespace

// The layers this path serves: UPCAT, 16 -> 8 channels (8 + 8), 3x3, stride 1, no dilation /
// groups, square padding, exact nearest-2x upsampling of source b, exact-fp32 math, phase weights
// given. (All 8 output channels per thread on 16 x 32 tiles: a caller with few tiles -- DNET's
// eighth-resolution nconv4 -- passes no phase weights and keeps fwd_tiled's channel split.)
bool fwd_phase_supported(const nconv_layer& L, bool tail) {
    (void)tail;
    const bool up = L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;
    if (!up || !L.waux || L.math != NCONV_MATH_FP32) return false;
    if (L.Cin != 16 || L.Cout != 8 || L.a.C != 8 || L.b.C != 8 || L.KH != 3 || L.KW != 3) return false;
    if (L.SH != 1 || L.SW != 1 || L.DH != 1 || L.DW != 1 || L.groups != 1 || L.PH != L.PW) return false;
    return L.H == 2 * L.b.H && L.W == 2 * L.b.W;
}

size_t phase_weight_floats(const nconv_layer& L) {
    const bool up = L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;
    if (!up || L.Cin != 16 || L.Cout != 8 || L.a.C != 8 || L.b.C != 8 || L.KH != 3 || L.KW != 3 || L.groups != 1)
        return 0;
    return (size_t)kPCB * 2 * 2 * 32;
}

template <int MODE, bool TAIL>
static void go_phase(const LayerDev& d, float* y, float* yc, const TailArgs& t, int gh, int gw, int par,
                     hipStream_t st) {
    dim3 grid(((gw + kPTW - 1) / kPTW) * ((gh + kPTH - 1) / kPTH) * d.L.B);  // see xcd_tile
    if (par)
        hipLaunchKernelGGL((fwd_phase<MODE, TAIL, 1>), grid, dim3(kPT), 0, st, d, y, yc, t);
    else
        hipLaunchKernelGGL((fwd_phase<MODE, TAIL, 0>), grid, dim3(kPT), 0, st, d, y, yc, t);
}

bool launch_fwd_phase(const LayerDev& d, float* y, float* yc, const TailArgs& t, bool tail, hipStream_t st) {
    const nconv_layer& L = d.L;
    if (!fwd_phase_supported(L, tail) || (!tail && t.py)) return false;
    const int gh = tail ? t.out_h : L.Ho, gw = tail ? t.out_w : L.Wo;
    const int par = ((tail ? t.off : 0) - L.PH) & 1;
    if (L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST) {
        if (tail) go_phase<NCONV_LOAD_UPCAT_SKIP_FIRST, true>(d, y, yc, t, gh, gw, par, st);
        else go_phase<NCONV_LOAD_UPCAT_SKIP_FIRST, false>(d, y, yc, t, gh, gw, par, st);
    } else {
        if (tail) go_phase<NCONV_LOAD_UPCAT_UP_FIRST, true>(d, y, yc, t, gh, gw, par, st);
        else go_phase<NCONV_LOAD_UPCAT_UP_FIRST, false>(d, y, yc, t, gh, gw, par, st);
    }
    return true;
}

int launch_phase_weights(int n, const float* const* w, const int* cin, const int* up_first, float* const* out,
                         hipStream_t st, const char** why) {
    if (n <= 0) return 0;
    if (n > PhaseArgs::kMax) {
        *why = "too many layers for one nconv_phase_weights launch (max 8)";
        return -22;
    }
    PhaseArgs a{};
    for (int i = 0; i < n; ++i) {
        a.w[i] = w[i];
        a.out[i] = out[i];
        a.ci0[i] = up_first[i];
        a.cin[i] = cin[i];
    }
    hipLaunchKernelGGL(phase_weights, dim3(n), dim3(kPrepThreads), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
