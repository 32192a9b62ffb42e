// nconv_fwd.hip — forward NConv kernels for gfx950 (MI355X).
//
// One launch per NConv2d layer computes, for every output pixel and output channel,
//     N = sum W * (x*c),   D = sum W * c,   y = N/(D+eps) + b,   cout = D/s
// (reference models/step1.py:116-149). N and D share every weight, so each tap is ONE packed
// FP32 FMA  {N,D} += {w,w} * {x*c, c}  (v_pk_fma_f32 with the weight broadcast from an SGPR pair,
// op_sel_hi:[0,1,1]): the weight stream is wave-uniform and rides the scalar cache, the packed
// {x*c, c} operand is staged once per input element in LDS.
//
// Tiling: a 256-thread workgroup owns a TH x 32 output tile of one image; each thread owns 2
// horizontally adjacent pixels (a sliding window of 2+K-1 staged inputs per kernel row feeds
// 2*K*Cout/CS packed FMAs) of Cout/CS output channels, the workgroup's CS channel slices being
// whole waves (TH = 16 / CS rows). Input channels are staged one plane of (TH+K-1) x (32+K-1)
// {x*c, c} pairs at a time into two LDS buffers (register-staged software pipeline), with the
// layer's glue (threshold / 2x2 max-pool / nearest upsample + concat, step1.py:53-90) evaluated
// while staging, so glued tensors never hit HBM. CS = 1 for the full- and half-resolution layers;
// the small layers split the channels so their few pixels still fill the chip (go_tiled).
#include <cstdlib>
#include "nconv_prologue.h"

namespace nconv {

constexpr int kThreads = 256;

template <int CIN, int K, int P_, int NTH, int CS>
struct FwdCfg {
    // P pixels per thread, 16 threads per tile row; the NTH threads form CS groups (one per slice
    // of COUT / CS output channels) of NTH / CS threads each, so NTH / (16 CS) rows per tile
    static constexpr int P = P_, TW = 16 * P, TG = NTH / CS, TH = TG / 16;
    static constexpr int IHT = TH + K - 1, IWT = TW + K - 1;
    static constexpr int IWP = (IWT + 1) & ~1;  // even pitch keeps the f4 reads 16-B aligned
    static constexpr int NV = P + K - 1;         // sliding-window width per kernel row
    static_assert(IWT < 64, "narrow tiles: the buffer-load stager");
};

template <int CIN, int COUT, int K, int MODE, bool TAIL, int P, int NTH, int CS>
__global__ __launch_bounds__(NTH) void fwd_tiled(LayerDev d, float* __restrict__ y, float* __restrict__ yc,
                                                 TailArgs t) {
    using C = FwdCfg<CIN, K, P, NTH, CS>;
    using TS = TileStager<C::IHT, C::IWT, C::IWP, MODE, NTH>;
    constexpr int kStride = TS::PLANE_STRIDE;  // f2 per plane buffer
    constexpr int CO = COUT / CS;              // output channels per thread
    static_assert(COUT % CS == 0 && C::TG % 64 == 0 && (!TAIL || CS == 1), "channel slices are whole waves");
    // CS > 1 (small layers): the input channels staged PG at a time (one load latency and one
    // barrier per group instead of per channel); at most 8 planes of LDS, so up to 8 workgroups
    // stay resident per CU and the small grids run in one round
    constexpr bool ALLP = CS > 1;
    constexpr int PG = CIN < 8 ? CIN : 8;
    static_assert(!ALLP || CIN % PG == 0, "whole plane groups");
    __shared__ __attribute__((aligned(16))) f2 tile[(ALLP ? PG : 2) * kStride];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x;
    const int og = __builtin_amdgcn_readfirstlane(tid / C::TG), lt = tid % C::TG;  // slice, thread in it
    const float* __restrict__ wgt = L.weight + (size_t)og * CO * CIN * K * K;
    const int gh = TAIL ? t.out_h : L.Ho, gw = TAIL ? t.out_w : L.Wo;  // the written grid
    const TileCoord tc = xcd_tile((gw + C::TW - 1) / C::TW, (gh + C::TH - 1) / C::TH, L.B);
    const int b = tc.b;
    const int R0 = tc.ty * C::TH, C0 = tc.tx * C::TW;  // tile origin in the written grid
    const int off = TAIL ? t.off : 0;
    const int oh0 = R0 + off, ow0 = C0 + off;  // tile origin in this layer's output grid
    const int ih0 = oh0 - L.PH, iw0 = ow0 - L.PW;
    const int ty = lt >> 4, tx = (lt & 15) * C::P;

    f2 acc[CO][C::P];
#pragma unroll
    for (int o = 0; o < CO; ++o)
#pragma unroll
        for (int j = 0; j < C::P; ++j) acc[o][j] = (f2){0.f, 0.f};

    // ---- packed-FP32 accumulation of one staged plane: {N, D} += w * {x*c, c} ----
    // One kernel row per iteration, deliberately not unrolled: its K*Cout weights are loaded into
    // SGPRs (s_load) right before use. Unrolling lets the compiler hoist every weight of the plane
    // into SGPRs, which spills them through v_writelane.
    const f2* rowbase = &tile[ty * C::IWP + tx];
    auto row_step = [&](const f2* row, const float* wr) __attribute__((always_inline)) {
            f2 v[C::NV];
            if constexpr (C::P % 2 == 0) {  // even pixel offset: 16-B aligned ds_read_b128
#pragma unroll
                for (int m = 0; m < C::NV / 2; ++m) {
                    f4 qv = reinterpret_cast<const f4*>(row)[m];
                    v[2 * m] = qv.xy;
                    v[2 * m + 1] = qv.zw;
                }
                if constexpr (C::NV & 1) v[C::NV - 1] = row[C::NV - 1];
            } else {
#pragma unroll
                for (int m = 0; m < C::NV; ++m) v[m] = row[m];
            }
#pragma unroll
            for (int kw = 0; kw < K; ++kw)
#pragma unroll
                for (int o = 0; o < CO; ++o) {
                    const float w = wr[o * CIN * K * K + kw];
                    const f2 w2 = (f2){w, w};
#pragma unroll
                    for (int j = 0; j < C::P; ++j) acc[o][j] = __builtin_elementwise_fma(w2, v[j + kw], acc[o][j]);
                }
    };
#ifndef NCONV_TILED_UNROLL_CO
#define NCONV_TILED_UNROLL_CO 2
#endif
    auto fma_plane = [&](int ci, int bufi) {
        const f2* row = rowbase + bufi * kStride;
        const float* wr = wgt + (size_t)ci * K * K;  // weights of (ci, kh) are K contiguous floats
        if constexpr (CO <= NCONV_TILED_UNROLL_CO) {
            // two output channels per thread (the channel-split small layers): the plane's 2 K*K
            // weights fit the SGPRs, so the rows are unrolled and every weight load issued up front
            // (their latency was exposed: < 1 wave per SIMD at the eighth resolution); down3 17 ->
            // 13 us, down2 26.6 -> 24.6, forward +1.1 % (profiles/r5_ab_small_layers_unrolled.log)
#pragma unroll
            for (int q = 0; q < K; ++q) row_step(row + q * C::IWP, wr + q * K);
        } else {
#pragma unroll 1
            for (int q = 0; q < K; ++q, row += C::IWP, wr += K) row_step(row, wr);
        }
    };

    TS ts;
    ts.init(d, ih0, iw0, tid);
    if constexpr (ALLP) {
        // small tiles: a group's loads in flight together, then one store phase and one barrier
        // (the per-plane pipeline below serialises one load latency per plane, which the few FMAs
        // of a small tile's plane cannot cover); the next group's loads fly during this one's FMAs
        float xs[PG][TS::NE], cs_[PG][TS::NE];
#pragma unroll
        for (int i = 0; i < PG; ++i) ts.load(chan_src<MODE>(d, b, i), xs[i], cs_[i]);
#pragma unroll
        for (int g0 = 0; g0 < CIN; g0 += PG) {
            if (g0) __syncthreads();  // every wave is done with the previous group's planes
#pragma unroll
            for (int i = 0; i < PG; ++i) ts.store(tile + i * kStride, xs[i], cs_[i], L.thresh);
            __syncthreads();
            if (g0 + PG < CIN) {
#pragma unroll
                for (int i = 0; i < PG; ++i) ts.load(chan_src<MODE>(d, b, g0 + PG + i), xs[i], cs_[i]);
            }
#pragma unroll 1
            for (int i = 0; i < PG; ++i) fma_plane(g0 + i, i);
        }
    } else {
        // Software pipeline over input channels with two LDS plane buffers and one barrier per
        // channel (a buffer is rewritten two steps after it was read, with a barrier in between).
        // Loads run two planes ahead: plane ci+2's buffer loads are issued right after plane ci is
        // stored, so each has two planes of FMAs to land.
        float xa[TS::NE], ca[TS::NE], xb[TS::NE], cb[TS::NE];
        ts.load(chan_src<MODE>(d, b, 0), xa, ca);
        if (CIN > 1) ts.load(chan_src<MODE>(d, b, 1), xb, cb);
        // The prefetches are unconditional (past the last channel they re-read it, L2-resident):
        // a branch around them would make the wait before each store conservatively drain the
        // other set's loads too.
#pragma unroll 1
        for (int ci = 0; ci < CIN; ci += 2) {
            ts.store(tile, xa, ca, L.thresh);
            __syncthreads();
            ts.load(chan_src<MODE>(d, b, ci + 2 < CIN ? ci + 2 : CIN - 1), xa, ca);
            fma_plane(ci, 0);
            if (ci + 1 < CIN) {
                ts.store(tile + kStride, xb, cb, L.thresh);
                __syncthreads();
                ts.load(chan_src<MODE>(d, b, ci + 3 < CIN ? ci + 3 : CIN - 1), xb, cb);
                fma_plane(ci + 1, 1);
            }
        }
    }

    // ---- epilogue ----
    const int oh = oh0 + ty;
    if constexpr (!TAIL) {
        // Buffer stores through one resource per output plane (base and size in SGPRs, built by
        // scalar ops per channel): the per-lane byte offset is computed once, and pixels outside
        // the output carry an offset past the plane, which the store drops -- no 64-bit address
        // arithmetic and no bounds branches per channel.
        constexpr unsigned OOB = 0x80000000u;
        const int ow = ow0 + tx;
        const size_t plane = (size_t)L.Ho * L.Wo;
        const int pbytes = (int)(plane * 4);
        unsigned so[C::P];
#pragma unroll
        for (int j = 0; j < C::P; ++j)
            so[j] = (oh < L.Ho && ow + j < L.Wo) ? (unsigned)(oh * L.Wo + ow + j) * 4u : OOB;
        const bool vec = (L.Wo % 2) == 0 && (ow + C::P - 1) < L.Wo && oh < L.Ho;  // pairs: 8-byte stores
        // optional fused 2x2 max-pool of the outputs (the next down layer's input, step1.py:62-75):
        // rows oh and oh^1 sit in lanes l and l^16 of one wave (ty = lt >> 4, tile origin even)
        const bool pool = t.py != nullptr;
        const int Hp = L.Ho >> 1, Wp = L.Wo >> 1;
        const size_t pplane = (size_t)Hp * Wp;
        const int ppbytes = (int)(pplane * 4);
        const int pr = oh >> 1, pc0 = ow >> 1;
        const bool pool_row = pool && ((ty & 1) == 0) && pr < Hp;
        constexpr int NPO = C::P > 1 ? C::P / 2 : 1;
        // po: the window's top-left lane (training, P = 1); pcy / pcc (inference, P even): the pooled
        // y leaves from the even rows, the pooled cout from the odd rows (see the epilogue)
        unsigned po[NPO], pcy[NPO], pcc[NPO];
#pragma unroll
        for (int h = 0; h < NPO; ++h) {
            po[h] = (pool_row && pc0 + h < Wp && (C::P > 1 || (lt & 1) == 0)) ? (unsigned)(pr * Wp + pc0 + h) * 4u : OOB;
            const unsigned pp = (pool && pr < Hp && pc0 + h < Wp) ? (unsigned)(pr * Wp + pc0 + h) * 4u : OOB;
            pcy[h] = (ty & 1) == 0 ? pp : OOB;
            pcc[h] = (ty & 1) ? pp : OOB;
        }
#pragma unroll
        for (int oo = 0; oo < CO; ++oo) {
            const int o = og * CO + oo;
            const float s = L.wsum[o], bo = L.bias[o];
            float yv[C::P], cv[C::P];
#pragma unroll
            for (int j = 0; j < C::P; ++j) nconv_epilogue(acc[oo][j].x, acc[oo][j].y, L.eps, bo, s, yv[j], cv[j]);
            if (C::P % 2 == 0 && pool && !t.parg) {  // (uniform) inference pooled copy, every lane joins
                // one v_permlane16_swap of (y, cout) per column leaves rows {y0, c0, y2, c2} and
                // {y1, c1, y3, c3} (rows oh, oh^1 in lanes l, l^16), so their maximum is y's vertical
                // pair maximum in the even rows and cout's in the odd rows; the columns are the lane's
                const size_t pofs = ((size_t)b * COUT + o) * pplane;
                const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(t.py + pofs, ppbytes);
                const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(t.pc + pofs, ppbytes);
                float vm[C::P];
#pragma unroll
                for (int j = 0; j < C::P; ++j) vm[j] = pair_rows_max(yv[j], cv[j]);
#pragma unroll
                for (int h = 0; h < C::P / 2; ++h) {
                    const float pm = __builtin_elementwise_maximum(vm[2 * h], vm[2 * h + 1]);
                    st_f32(rpy, pcy[h], pm);
                    st_f32(rpc, pcc[h], pm);
                }
            } else if (pool) {  // every lane joins the shuffles
                float yb[C::P], cb[C::P];
#pragma unroll
                for (int j = 0; j < C::P; ++j) {
                    yb[j] = shfl_xor16(yv[j]);
                    cb[j] = shfl_xor16(cv[j]);
                }
                const size_t pofs = ((size_t)b * COUT + o) * pplane;
                const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(t.py + pofs, ppbytes);
                const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(t.pc + pofs, ppbytes);
                // with t.parg: each window's first-maximum slots (y in bits 0-1, cout in bits 2-3,
                // slot = 2*row + column), what the training backward routes the pooled gradient by
                unsigned* parg = t.parg ? t.parg + pofs : nullptr;
                if constexpr (C::P == 1) {  // the window's right column sits in lane l^1
                    const float ya = shfl_xor1(yv[0]), ca = shfl_xor1(cv[0]);
                    const float yd = shfl_xor1(yb[0]), cd = shfl_xor1(cb[0]);
                    if (parg) {  // (uniform) training: the first maximum's slot too
                        int ay, ac;
                        st_f32(rpy, po[0], pool4(yv[0], ya, yb[0], yd, ay));
                        st_f32(rpc, po[0], pool4(cv[0], ca, cb[0], cd, ac));
                        if (po[0] != OOB) parg[po[0] >> 2] = (unsigned)(ay | (ac << 2));
                    } else {
                        st_f32(rpy, po[0], pool4v(yv[0], ya, yb[0], yd));
                        st_f32(rpc, po[0], pool4v(cv[0], ca, cb[0], cd));
                    }
                } else if (parg) {
#pragma unroll
                    for (int h = 0; h < C::P / 2; ++h) {
                        int ay, ac;
                        st_f32(rpy, po[h], pool4(yv[2 * h], yv[2 * h + 1], yb[2 * h], yb[2 * h + 1], ay));
                        st_f32(rpc, po[h], pool4(cv[2 * h], cv[2 * h + 1], cb[2 * h], cb[2 * h + 1], ac));
                        if (po[h] != OOB) parg[po[h] >> 2] = (unsigned)(ay | (ac << 2));
                    }
                } else {
#pragma unroll
                    for (int h = 0; h < C::P / 2; ++h) {
                        st_f32(rpy, po[h], pool4v(yv[2 * h], yv[2 * h + 1], yb[2 * h], yb[2 * h + 1]));
                        st_f32(rpc, po[h], pool4v(cv[2 * h], cv[2 * h + 1], cb[2 * h], cb[2 * h + 1]));
                    }
                }
            }
            const size_t ofs = ((size_t)b * COUT + o) * plane;
            const __amdgpu_buffer_rsrc_t ry = plane_rsrc(y + ofs, pbytes), rc = plane_rsrc(yc + ofs, pbytes);
            if (C::P % 2 == 0 && vec) {
#pragma unroll
                for (int q = 0; q < C::P; q += 2) {
                    st_f2(ry, so[q], (f2){yv[q], yv[q + 1]});
                    st_f2(rc, so[q], (f2){cv[q], cv[q + 1]});
                }
            } else {
#pragma unroll
                for (int j = 0; j < C::P; ++j) {
                    st_f32(ry, so[j], yv[j]);
                    st_f32(rc, so[j], cv[j]);
                }
            }
        }
    } else {
        // nconv6 outputs -> nconv7 (1x1, COUT -> 1) -> cropped final output.
        const int r = R0 + ty;
        if (r >= t.out_h) return;
        float s6[COUT], b6[COUT], w7[COUT];
#pragma unroll
        for (int o = 0; o < COUT; ++o) {
            s6[o] = L.wsum[o];
            b6[o] = L.bias[o];
            w7[o] = t.w7[o];
        }
        const float b7 = t.b7[0], s7 = t.s7[0];
        float ov[C::P], oc[C::P];
#pragma unroll
        for (int j = 0; j < C::P; ++j) {
            const int ow = ow0 + tx + j;
            float N7 = 0.f, D7 = 0.f;
            if ((unsigned)oh < (unsigned)L.Ho && (unsigned)ow < (unsigned)L.Wo) {
#pragma unroll
                for (int o = 0; o < COUT; ++o) {
                    float y6, c6;
                    nconv_epilogue(acc[o][j].x, acc[o][j].y, L.eps, b6[o], s6[o], y6, c6);
                    N7 = fmaf(w7[o], y6 * c6, N7);
                    D7 = fmaf(w7[o], c6, D7);
                }
            }
            nconv_epilogue(N7, D7, t.eps7, b7, s7, ov[j], oc[j]);
        }
        const size_t base = ((size_t)b * t.out_h + r) * t.out_w + C0 + tx;
#pragma unroll
        for (int j = 0; j < C::P; ++j)
            if (C0 + tx + j < t.out_w) {
                y[base + j] = ov[j];
                if (t.out_c) t.out_c[base + j] = oc[j];
            }
    }
}

// Any NConv2d configuration (stride, dilation, groups, odd kernels): one thread per output element.
template <int MODE>
__global__ __launch_bounds__(kThreads) void fwd_generic(LayerDev d, float* __restrict__ y,
                                                        float* __restrict__ yc) {
    const nconv_layer& L = d.L;
    const size_t n = (size_t)L.B * L.Cout * L.Ho * L.Wo;
    const int cpg_in = L.Cin / L.groups, cpg_out = L.Cout / L.groups;
    for (size_t idx = (size_t)blockIdx.x * kThreads + threadIdx.x; idx < n;
         idx += (size_t)gridDim.x * kThreads) {
        const int ow = (int)(idx % L.Wo);
        const int oh = (int)((idx / L.Wo) % L.Ho);
        const int o = (int)((idx / ((size_t)L.Wo * L.Ho)) % L.Cout);
        const int b = (int)(idx / ((size_t)L.Wo * L.Ho * L.Cout));
        const int g = o / cpg_out;
        float N = 0.f, D = 0.f;
        for (int cl = 0; cl < cpg_in; ++cl) {
            const int ci = g * cpg_in + cl;
            for (int kh = 0; kh < L.KH; ++kh) {
                const int ih = oh * L.SH - L.PH + kh * L.DH;
                if ((unsigned)ih >= (unsigned)L.H) continue;
                for (int kw = 0; kw < L.KW; ++kw) {
                    const int iw = ow * L.SW - L.PW + kw * L.DW;
                    if ((unsigned)iw >= (unsigned)L.W) continue;
                    float x, c;
                    load_xc<MODE>(d, b, ci, ih, iw, x, c);
                    const float w = L.weight[(((size_t)o * cpg_in + cl) * L.KH + kh) * L.KW + kw];
                    N = fmaf(w, x * c, N);
                    D = fmaf(w, c, D);
                }
            }
        }
        float yv, cv;
        nconv_epilogue(N, D, L.eps, L.bias[o], L.wsum[o], yv, cv);
        y[idx] = yv;
        yc[idx] = cv;
    }
}

// EnforcePos + normalisers (PrepArgs, prep_block: nconv_prologue.h), one block per layer.
__global__ __launch_bounds__(kPrepThreads) void weight_prep(PrepArgs a) {
    const int l = blockIdx.x;
    prep_block(a.w[l], a.s[l], a.cout[l], a.fan_in[l], a.softplus[l]);
}

}  // namespace nconv

// ------------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------------
namespace nconv {

static int last_launch(const char** why) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;  // EIO
    }
    return 0;
}

static bool simple_geometry(const nconv_layer& L) {
    return L.SH == 1 && L.SW == 1 && L.DH == 1 && L.DW == 1 && L.groups == 1 && L.KH == L.KW;
}

template <int CIN, int COUT, int K, int MODE, bool TAIL, int CS>
static void go_tiled_cs(const LayerDev& d, float* y, float* yc, const TailArgs& t, int gh, int gw, hipStream_t st) {
    using C = FwdCfg<CIN, K, 2, 256, CS>;
    dim3 grid(((gw + C::TW - 1) / C::TW) * ((gh + C::TH - 1) / C::TH) * d.L.B);  // see xcd_tile
    hipLaunchKernelGGL((fwd_tiled<CIN, COUT, K, MODE, TAIL, 2, 256, CS>), grid, dim3(256), 0, st, d, y, yc, t);
}

// 2 pixels per thread, 32-column tiles, 256 threads (measured against 1 and 4 pixels: 4 needs
// 105-125 VGPRs, 4 waves/SIMD; 1 doubles the LDS reads per FMA). A thread computes all 8 output
// channels of its pixels while the layer has at least four 16-row tiles per CU (the full and half
// resolution layers); the small quarter / eighth-resolution layers would leave most SIMDs with no
// wave at all, so their waves split the output channels (2 or 4 slices, on 8- or 4-row tiles;
// a slice is whole waves, so its weights stay wave-uniform) and the layer spreads over the whole
// chip. (Thresholds measured: a CS=1 limit of 1024 tiles against 2048 / 4096 / 8192 / never at
// B=8 352x1216, one and two inference streams: profiles/r3_ab_fwd_cs.log.)
#ifndef NCONV_CS1_TILES
#define NCONV_CS1_TILES 1024
#endif
#ifndef NCONV_CS2_TILES
#define NCONV_CS2_TILES 512
#endif
static int tiled_cs(long tiles16, int cout, int mode) {
    (void)mode;
    int cs = tiles16 >= NCONV_CS1_TILES ? 1 : tiles16 >= NCONV_CS2_TILES ? 2 : 4;
    while (cs > 1 && cout % cs) cs >>= 1;
    return cs;
}

template <int CIN, int COUT, int K, int MODE, bool TAIL>
static void go_tiled(const LayerDev& d, float* y, float* yc, const TailArgs& t, int gh, int gw, hipStream_t st) {
    const long tiles16 = (long)((gw + 31) / 32) * ((gh + 15) / 16) * d.L.B;
    const int cs = (TAIL || MODE == NCONV_LOAD_THRESH) ? 1 : tiled_cs(tiles16, COUT, MODE);
    if constexpr (!TAIL && COUT % 8 == 0) {
        if (cs == 4) return go_tiled_cs<CIN, COUT, K, MODE, TAIL, 4>(d, y, yc, t, gh, gw, st);
        if (cs == 2) return go_tiled_cs<CIN, COUT, K, MODE, TAIL, 2>(d, y, yc, t, gh, gw, st);
    }
    go_tiled_cs<CIN, COUT, K, MODE, TAIL, 1>(d, y, yc, t, gh, gw, st);
}

static bool fwd_tiled_shape(const nconv_layer& L) {
    const int m = L.load_mode;
    return simple_geometry(L) &&
           ((L.Cin == 1 && L.Cout == 8 && L.KH == 5 && m == NCONV_LOAD_THRESH) ||
            (L.Cin == 8 && L.Cout == 8 && L.KH == 5 && (m == NCONV_LOAD_PLAIN || m == NCONV_LOAD_POOL2)) ||
            (L.Cin == 16 && L.Cout == 8 && L.KH == 3 &&
             (m == NCONV_LOAD_UPCAT_SKIP_FIRST || m == NCONV_LOAD_UPCAT_UP_FIRST)) ||
            (L.Cin == 8 && L.Cout == 1 && L.KH == 1 && m == NCONV_LOAD_PLAIN));
}

int plan_fwd(const nconv_layer& L) {
    if (fwd_mfma_supported(L, false, false))
        return L.math == NCONV_MATH_BF16X9 ? NCONV_KERNEL_MFMA_BF16X9 : NCONV_KERNEL_MFMA_BF16X3;
    if (fwd_phase_supported(L, false)) return NCONV_KERNEL_TILED_FP32_PHASE;
    return fwd_tiled_shape(L) ? NCONV_KERNEL_TILED_FP32 : NCONV_KERNEL_GENERIC;
}

int launch_fwd(const LayerDev& d, float* y, float* yc, float* py, float* pc, unsigned* parg, hipStream_t st,
               const char** why) {
    const nconv_layer& L = d.L;
    TailArgs t{};
    t.py = py;
    t.pc = pc;
    t.parg = parg;
    if (!parg) {  // the argmax codes are written by the tiled fp32 kernels only
        if (launch_fwd_mfma(d, y, yc, t, false, st)) return last_launch(why);
        if (launch_fwd_phase(d, y, yc, t, false, st)) return last_launch(why);
    } else if (!fwd_tiled_shape(L) || L.math != NCONV_MATH_FP32) {
        *why = "pooling argmax codes need an exact-fp32 tiled layer (8->8 5x5, 1->8 5x5 threshold, 16->8 3x3)";
        return -95;
    }
    if (simple_geometry(L)) {
#define NCONV_TRY(CIN, COUT, K, MODE)                                                       \
    if (L.Cin == CIN && L.Cout == COUT && L.KH == K && L.load_mode == MODE) {               \
        go_tiled<CIN, COUT, K, MODE, false>(d, y, yc, t, L.Ho, L.Wo, st);                   \
        return last_launch(why);                                                             \
    }
        NCONV_TRY(1, 8, 5, NCONV_LOAD_THRESH)
        NCONV_TRY(8, 8, 5, NCONV_LOAD_PLAIN)
        NCONV_TRY(8, 8, 5, NCONV_LOAD_POOL2)
        NCONV_TRY(16, 8, 3, NCONV_LOAD_UPCAT_SKIP_FIRST)
        NCONV_TRY(16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST)
        NCONV_TRY(8, 1, 1, NCONV_LOAD_PLAIN)
#undef NCONV_TRY
    }
    if (py) {
        *why = "fused output pooling is only built for the tiled DNET layer shapes";
        return -95;  // EOPNOTSUPP
    }
    const size_t n = (size_t)L.B * L.Cout * L.Ho * L.Wo;
    size_t blocks = (n + kThreads - 1) / kThreads;
    if (blocks > (1u << 20)) blocks = 1u << 20;
    if (blocks == 0) return 0;
    switch (L.load_mode) {
        case NCONV_LOAD_PLAIN:
            hipLaunchKernelGGL(fwd_generic<NCONV_LOAD_PLAIN>, dim3(blocks), dim3(kThreads), 0, st, d, y, yc);
            break;
        case NCONV_LOAD_THRESH:
            hipLaunchKernelGGL(fwd_generic<NCONV_LOAD_THRESH>, dim3(blocks), dim3(kThreads), 0, st, d, y, yc);
            break;
        case NCONV_LOAD_POOL2:
            hipLaunchKernelGGL(fwd_generic<NCONV_LOAD_POOL2>, dim3(blocks), dim3(kThreads), 0, st, d, y, yc);
            break;
        case NCONV_LOAD_UPCAT_SKIP_FIRST:
            hipLaunchKernelGGL(fwd_generic<NCONV_LOAD_UPCAT_SKIP_FIRST>, dim3(blocks), dim3(kThreads), 0, st, d, y, yc);
            break;
        case NCONV_LOAD_UPCAT_UP_FIRST:
            hipLaunchKernelGGL(fwd_generic<NCONV_LOAD_UPCAT_UP_FIRST>, dim3(blocks), dim3(kThreads), 0, st, d, y, yc);
            break;
        default:
            *why = "unknown load mode";
            return -22;
    }
    return last_launch(why);
}

int launch_fwd_tail(const LayerDev& d, const TailArgs& t, float* out, hipStream_t st, const char** why) {
    const nconv_layer& L = d.L;
    if (!(simple_geometry(L) && L.Cin == 16 && L.Cout == 8 && L.KH == 3 &&
          L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST)) {
        *why = "fused tail is only built for nconv6's geometry (16->8, 3x3, stride 1, upsample-first concat)";
        return -95;  // EOPNOTSUPP
    }
    if (t.out_h <= 0 || t.out_w <= 0) return 0;
    if (t.y6) {  // training outputs: the exact-fp32 phase tail only
        if (L.math != NCONV_MATH_FP32 || !launch_fwd_phase(d, out, nullptr, t, true, st)) {
            *why = "nconv6's outputs from the fused tail need the exact-fp32 phase form (exactly-2x upsampling, waux)";
            return -95;
        }
        return last_launch(why);
    }
    if (launch_fwd_mfma(d, out, nullptr, t, true, st)) return last_launch(why);
    if (launch_fwd_phase(d, out, nullptr, t, true, st)) return last_launch(why);
    go_tiled<16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST, true>(d, out, nullptr, t, t.out_h, t.out_w, st);
    return last_launch(why);
}

int launch_weight_prep(int n, float* const* w, const int* cout, const int* fan_in, const int* sp,
                       float* const* s, hipStream_t st, const char** why) {
    if (n <= 0) return 0;
    if (n > PrepArgs::kMax) {
        *why = "too many layers for one weight_prep launch (max 32)";
        return -22;
    }
    PrepArgs a{};
    for (int i = 0; i < n; ++i) {
        a.w[i] = w[i];
        a.s[i] = s[i];
        a.cout[i] = cout[i];
        a.fan_in[i] = fan_in[i];
        a.softplus[i] = sp ? sp[i] : 0;
    }
    hipLaunchKernelGGL(weight_prep, dim3(n), dim3(kPrepThreads), 0, st, a);
    return last_launch(why);
}

}  // namespace nconv
