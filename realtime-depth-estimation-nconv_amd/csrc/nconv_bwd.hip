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
#include "nconv_route.h"
#include "nconv_prologue.h"

namespace nconv {

constexpr int kT = 256;

constexpr int pick_chunk(int n, int plane_f2, int budget) {
    int best = 1;
    for (int cc = 1; cc <= n; ++cc)
        if (n % cc == 0 && cc * plane_f2 * 8 <= budget) best = cc;
    return best;
}

// Staging of output-side planes {gN, gD} over an OHT x OWT halo tile (origin oh0, ow0) for the
// dgrad: the element map (LDS slot, byte offset in an output plane, or past-the-end for the zero
// padding) is computed once per workgroup; per output channel the four saved planes (gy, gcout,
// y, cout) are read with buffer loads and {gN, gD} are formed at store time. Elements are dealt
// to the 256 threads row-major; slots past the tile go to a dump slot after the plane.
// nconv7 (1x1, padding 2) consumer of this layer's outputs fused into its backward (T7): the
// layer's output gradient at (oh, ow) is nconv7's input gradient there, G_xc = w7[o] gN7, G_c =
// w7[o] gD7 with {gN7, gD7} from nconv7's (gy, y, cout) at (oh + 2, ow + 2); gy = G_xc * cout,
// gcout = G_c + G_xc * y (nconv7's dgrad_tiled<8,1,1> epilogue, same operations).
// (t7_off, t7_nd, t7_gy: nconv_internal.h)

template <int OHT, int OWT, int OWP, bool GP = false, bool T7 = false>
struct GTileStager {
    static constexpr int NT = OHT * OWT;
    static constexpr int NE = (NT + 255) / 256;
    static constexpr int PLANE = OHT * OWP;
    static constexpr int PLANE_STRIDE = PLANE + 2;
    static constexpr int NV = GP ? 7 : 4;  // gy, gcout, y, cout (+ pooled gy, gcout, argmax code)
    static constexpr unsigned OOB = 0x80000000u;
    unsigned lofs[NE];
    unsigned go[NE];
    unsigned gpo[GP ? NE : 1];  // pooled element offsets, window slots (GP)
    unsigned gsub[GP ? NE : 1];
    float t7n[T7 ? NE : 1], t7d[T7 ? NE : 1];  // {gN7, gD7} per element (T7)

    __device__ __forceinline__ void init(const nconv_layer& L, int oh0, int ow0, int tid) {
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + 256 * k;
            const int r = e / OWT, col = e - r * OWT;
            const int oh = oh0 + r, ow = ow0 + col;
            const bool in = e < NT && (unsigned)oh < (unsigned)L.Ho && (unsigned)ow < (unsigned)L.Wo;
            lofs[k] = e < NT ? r * OWP + col : PLANE;
            go[k] = in ? (unsigned)(oh * L.Wo + ow) * 4u : OOB;
            if constexpr (GP) {
                gpo[k] = in ? pool_elem_off(oh, ow, L.Ho >> 1, L.Wo >> 1, OOB) : OOB;
                gsub[k] = (unsigned)(((oh & 1) << 1) | (ow & 1));
            }
        }
    }

    // T7: nconv7's (gy, y, cout) of the elements (loads issued here, {gN7, gD7} formed by t7_form)
    __device__ __forceinline__ void t7_load(const nconv_layer& L, const BwdArgs& a, int b, int oh0, int ow0, int tid,
                                            float (&v)[3][NE]) const {
        const int pl7 = a.t7ph * a.t7pw;
        const size_t base = (size_t)b * pl7;
        const __amdgpu_buffer_rsrc_t rg = plane_rsrc(a.t7gy + base, pl7 * 4);
        const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.t7y + base, pl7 * 4);
        const __amdgpu_buffer_rsrc_t rc = plane_rsrc(a.t7co + base, pl7 * 4);
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + 256 * k;
            const int r = e / OWT, col = e - r * OWT;
            const unsigned off = e < NT ? t7_off(a, oh0 + r, ow0 + col, L.Ho, L.Wo, OOB) : OOB;
            v[0][k] = ld_f32(rg, off);
            v[1][k] = ld_f32(ry, off);
            v[2][k] = ld_f32(rc, off);
        }
    }
    __device__ __forceinline__ void t7_form(const BwdArgs& a, const float (&v)[3][NE]) {
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            if constexpr (T7) t7_nd(a, v[0][k], v[1][k], v[2][k], t7n[k], t7d[k]);
        }
    }

    // raw (gy, gcout, y, cout [, pooled gy, pooled gcout, code]) of output channel o of image b, no wait
    __device__ __forceinline__ void load(const nconv_layer& L, const BwdArgs& a, int b, int o,
                                         float (&v)[NV][NE]) const {
        const int plane = L.Ho * L.Wo;
        const size_t base = ((size_t)b * L.Cout + o) * plane;
        const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + base, plane * 4);
        const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + base, plane * 4);
        const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + base, plane * 4);
        if constexpr (T7) {  // gy / gcout are formed from nconv7's planes at store time
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                v[2][k] = ld_f32(ry, go[k]);
                v[3][k] = ld_f32(rco, go[k]);
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            v[0][k] = ld_f32(rgy, go[k]);
            v[2][k] = ld_f32(ry, go[k]);
            v[3][k] = ld_f32(rco, go[k]);
        }
        // gcout may be absent (= 0): a zero-sized resource then reads 0 -- no branch, since a branch
        // here makes the compiler wait for all of this stage's loads at the join, i.e. right after
        // issuing them instead of behind the next plane's FMAs
        const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + base : a.y, a.gco ? plane * 4 : 0);
#pragma unroll
        for (int k = 0; k < NE; ++k) v[1][k] = ld_f32(rgc, go[k]);
        if constexpr (GP) {
            const int pplane = (L.Ho >> 1) * (L.Wo >> 1);
            const size_t pbase = ((size_t)b * L.Cout + o) * pplane;
            const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(a.gpy + pbase, pplane * 4);
            const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(a.gpc + pbase, pplane * 4);
            const __amdgpu_buffer_rsrc_t rpa = plane_rsrc((const float*)(a.parg + pbase), pplane * 4);
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                v[4][k] = ld_f32(rpy, gpo[k]);
                v[5][k] = ld_f32(rpc, gpo[k]);
                v[6][k] = ld_f32(rpa, gpo[k]);  // the code word, carried as raw bits until store
            }
        }
    }

    __device__ __forceinline__ void store(const nconv_layer& L, int o, const float (&v)[NV][NE], f2* t,
                                          float a_w7 = 0.f) const {
        const float bo = L.bias[o], so = L.wsum[o];
        const float w7 = T7 ? a_w7 : 0.f;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            float gy, gco;
            if constexpr (T7) {
                t7_gy(w7, t7n[k], t7d[k], v[2][k], v[3][k], gy, gco);
            } else {
                gy = v[0][k];
                gco = v[1][k];
            }
            if constexpr (GP) pool_route(gy, gco, v[4][k], v[5][k], __builtin_bit_cast(unsigned, v[6][k]), gsub[k]);
            float gN, gD;  // zero padding: gy = gcout = y = cout = 0 gives gN = gD = 0
            nconv_grad_nd(gy, gco, v[2][k], v[3][k], L.eps, bo, so, gN, gD);
            t[lofs[k]] = (f2){gN, gD};
        }
    }
};

// ---- dgrad: tiled, stride 1 ------------------------------------------------------------------------
template <int CIN, int K>
struct DgCfg {
    static constexpr int P = 2;  // input pixels per thread (f2 epilogue: any even width stays vectorized)
    static constexpr int TPR = 16, TW = TPR * P, TH = kT / TPR;
    static constexpr int OHT = TH + K - 1, OWT = TW + K - 1;
    static constexpr int OWP = (OWT + 1) & ~1;  // even pitch: 16-B aligned window reads
    static constexpr int NV = P + K - 1;
};

template <int P>
struct VecOf;
template <>
struct VecOf<4> { typedef f4 T; };
template <>
struct VecOf<2> { typedef f2 T; };

// ---- fused nconv1 weight gradient (training, exact fp32) ------------------------------------------
// nconv2's input gradient at a pixel p is nconv1's output gradient there (gy1 = G_xc*c1, gcout1 =
// G_c + G_xc*y1), and nconv1 (1 -> 8, 5x5, padding 2, on x0 = S, c0 = (S > 0.01)) has
//     gW1[o][kh][kw] = sum_p gN1[o](p) * S(p + (kh-2, kw-2)) * c0(...) + gD1[o](p) * c0(...)
// whose terms vanish unless c0 = 1 at the tap: a correlation over the ~5 % of pixels that hold a
// depth sample. Per tile: {gN1, gD1} of the 16 x 32 pixels (8 channels) into LDS, the samples of the
// tile's 20 x 36 window listed once (a deterministic block prefix sum), then thread (o, tap) sums
// over the list; plus the dense sums gb1 = sum gy1 and sum gcout1*cout1 (the normaliser's term).
// One partial row per workgroup (wgrad_reduce_sum / wgrad_finish reduce them, deferred or not):
// nconv1's input gradient G[1] is never written to HBM and nconv1 needs no backward kernel.
// (kHeadNw, kHeadStride: nconv_internal.h)

template <int CIN, int TH, int TW>
struct HeadLds {
    static constexpr int RH = TH + 4, RW = TW + 4, RN = RH * RW;  // the tile's 5x5-window region
    static constexpr int NPL = CIN / 2;  // {gN1, gD1} planes held at once (22 KB of LDS, not 38)
    static constexpr int F2 = NPL * TH * TW + RN;                 // {gN1, gD1} planes + sample list
};

template <int CIN, int TH, int TW>
__device__ void head_wgrad_epilogue(const LayerDev& d, const BwdArgs& a, int b, int ih0, int iw0, int ty, int tx,
                                    const f2 (&acc)[CIN][2], f2* smem) {
    static_assert(CIN == 8, "nconv1 has 8 output channels");
    using H = HeadLds<CIN, TH, TW>;
    constexpr int RW = H::RW, RN = H::RN;
    constexpr int NPL = H::NPL;
    f2* gn = smem;                                       // [NPL][TH][TW]
    f2* qlist = smem + NPL * TH * TW;                    // {row << 8 | col, S} of the samples
    f4 vh[CIN - NPL > 0 ? CIN - NPL : 1];                // the second half's {gN1, gD1} (NPL < CIN)
    __shared__ int wtot[4];
    __shared__ float red[4][2 * CIN];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ih = ih0 + ty, iw = iw0 + tx;
    const bool pair = ih < L.H && iw + 1 < L.W && (L.W & 1) == 0;  // both pixels in range, 8-byte aligned
    float sgy[CIN], sgc[CIN];
#pragma unroll
    for (int i = 0; i < CIN; ++i) {
        sgy[i] = sgc[i] = 0.f;
        const size_t idx = plane_idx(b, i, L.a.C, L.a.H, L.a.W, ih < L.H ? ih : 0, iw < L.W ? iw : 0);
        float x[2] = {0.f, 0.f}, c[2] = {0.f, 0.f};
        if (pair) {
            const f2 xv = *reinterpret_cast<const f2*>(L.a.x + idx), cv = *reinterpret_cast<const f2*>(L.a.c + idx);
            x[0] = xv.x; x[1] = xv.y; c[0] = cv.x; c[1] = cv.y;
        } else {
#pragma unroll
            for (int j = 0; j < 2; ++j)
                if (ih < L.H && iw + j < L.W) {
                    x[j] = L.a.x[idx + j];
                    c[j] = L.a.c[idx + j];
                }
        }
        f2 v[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bool ok = ih < L.H && iw + j < L.W;
            const float gy = acc[i][j].x * c[j], gco = acc[i][j].y + acc[i][j].x * x[j];
            float gN = 0.f, gD = 0.f;
            if (ok) {
                if (a.gxa) a.gxa[idx + j] = gy;  // G[1] only when asked for (the input gradient of S)
                if (a.gca) a.gca[idx + j] = gco;
                nconv_grad_nd(gy, gco, x[j], c[j], a.heps, a.hb[i], a.hs[i], gN, gD);
                sgy[i] += gy;
                sgc[i] = fmaf(gco, c[j], sgc[i]);
            }
            v[j] = (f2){gN, gD};
        }
        if (i < NPL) *reinterpret_cast<f4*>(gn + (i * TH + ty) * TW + tx) = (f4){v[0].x, v[0].y, v[1].x, v[1].y};
        else vh[i - NPL] = (f4){v[0].x, v[0].y, v[1].x, v[1].y};
    }
    // the depth samples (c0 = 1) of the window region, listed in (thread, element) order
    const float* Sp = a.hS + (size_t)b * L.H * L.W;
    constexpr int NE = (RN + kT - 1) / kT;
    float sv[NE];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int e = tid * NE + k;  // consecutive elements per thread: the list is row-major
        const int r = e / RW, cc = e - r * RW;
        const int qr = ih0 - 2 + r, qc = iw0 - 2 + cc;
        const bool in = e < RN && (unsigned)qr < (unsigned)L.H && (unsigned)qc < (unsigned)L.W;
        sv[k] = in ? Sp[(size_t)qr * L.W + qc] : 0.f;
        cnt += sv[k] > a.hthresh ? 1 : 0;
    }
    int incl = cnt;  // wave inclusive scan
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const int t = __shfl_up(incl, sh);
        if (lane >= sh) incl += t;
    }
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int off = incl - cnt, total = 0;
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) {
        off += w2 < wv ? wtot[w2] : 0;
        total += wtot[w2];
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        if (sv[k] > a.hthresh) {
            const int e = tid * NE + k;
            qlist[off] = (f2){__builtin_bit_cast(float, ((e / RW) << 8) | (e % RW)), sv[k]};
            ++off;
        }
    }
    // dense sums: wave butterflies, then the four waves in order
#pragma unroll
    for (int i = 0; i < CIN; ++i) {
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            sgy[i] += __shfl_xor(sgy[i], sh);
            sgc[i] += __shfl_xor(sgc[i], sh);
        }
    }
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < CIN; ++i) {
            red[wv][i] = sgy[i];
            red[wv][CIN + i] = sgc[i];
        }
    __syncthreads();
    float* out = a.hpart + (size_t)blockIdx.x * kHeadStride;
    // thread (o, tap) sums its tap over the sample list; with NPL < CIN one half of the channels
    // at a time (the LDS of four planes instead of eight: more workgroups per CU)
    auto tap_sums = [&](int o0) __attribute__((always_inline)) {
        const int t = tid;
        if (t < NPL * 25) {
            const int ol = t / 25, tap = t - ol * 25, kh = tap / 5, kw = tap - kh * 5;
            const f2* g = gn + ol * TH * TW;
            float sn = 0.f, sd = 0.f;
            for (int n = 0; n < total; ++n) {
                const f2 q = qlist[n];
                const int qi = __builtin_bit_cast(int, q.x);
                const int pr = (qi >> 8) - kh, pc = (qi & 255) - kw;  // p = q - (tap - 2), region origin -2
                if ((unsigned)pr < (unsigned)TH && (unsigned)pc < (unsigned)TW) {
                    const f2 v = g[pr * TW + pc];
                    sn = fmaf(v.x, q.y, sn);
                    sd += v.y;
                }
            }
            out[o0 * 25 + t] = sn + sd;
        }
    };
    tap_sums(0);
    if (tid >= kHeadNw && tid < kHeadNw + 2 * CIN) {
        const int k = tid - kHeadNw;
        out[tid] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    }
    if constexpr (NPL < CIN) {
        __syncthreads();  // every tap sum of the first half is done with its planes
#pragma unroll
        for (int i = NPL; i < CIN; ++i) *reinterpret_cast<f4*>(gn + ((i - NPL) * TH + ty) * TW + tx) = vh[i - NPL];
        __syncthreads();
        tap_sums(NPL);
    }
}

// One (output channel o, kernel row kh) step per iteration of the inner loop, not unrolled: its
// Cin*K weights ride SGPRs. The {gN, gD} planes of the output channels are staged one at a time
// into two LDS buffers, the loads two channels ahead (as the forward's input planes).
template <int CIN, int COUT, int K, int MODE, bool GP = false, bool HW = false>
__global__ __launch_bounds__(kT) void dgrad_tiled(LayerDev d, BwdArgs a, float* tmp_x, float* tmp_c) {
    using C = DgCfg<CIN, K>;
    using GS = GTileStager<C::OHT, C::OWT, C::OWP, GP>;
    constexpr int P = C::P;
    // with HW the staging planes' LDS is reused by the head epilogue ({gN1, gD1} planes + sample list)
    constexpr int TILE_F2 = HW && HeadLds<CIN, C::TH, C::TW>::F2 > 2 * GS::PLANE_STRIDE
                                ? HeadLds<CIN, C::TH, C::TW>::F2 : 2 * GS::PLANE_STRIDE;
    __shared__ __attribute__((aligned(16))) f2 tile[TILE_F2];
    const nconv_layer& L = d.L;
    const float* __restrict__ wgt = L.weight;
    const TileCoord tcd = xcd_tile((L.W + C::TW - 1) / C::TW, (L.H + C::TH - 1) / C::TH, L.B);
    const int tid = threadIdx.x, b = tcd.b;
    const int ih0 = tcd.ty * C::TH, iw0 = tcd.tx * C::TW;
    const int oh0 = ih0 + L.PH - (K - 1), ow0 = iw0 + L.PW - (K - 1);
    const int ty = tid / C::TPR, tx = (tid % C::TPR) * P;

    f2 acc[CIN][P];
#pragma unroll
    for (int i = 0; i < CIN; ++i)
#pragma unroll
        for (int j = 0; j < P; ++j) acc[i][j] = (f2){0.f, 0.f};

    auto fma_plane = [&](int o, int bufi) {
        const f2* row = &tile[bufi * GS::PLANE_STRIDE + (ty + K - 1) * C::OWP + tx];
        const float* wr = wgt + (size_t)o * CIN * K * K;
#pragma unroll 1
        for (int kh = 0; kh < K; ++kh, row -= C::OWP, wr += K) {
            f2 v[C::NV];
#pragma unroll
            for (int m = 0; m < C::NV / 2; ++m) {
                f4 qv = reinterpret_cast<const f4*>(row)[m];
                v[2 * m] = qv.xy;
                v[2 * m + 1] = qv.zw;
            }
            if constexpr (C::NV & 1) v[C::NV - 1] = row[C::NV - 1];
#pragma unroll
            for (int kw = 0; kw < K; ++kw)
#pragma unroll
                for (int i = 0; i < CIN; ++i) {
                    const float w = wr[i * K * K + kw];
                    const f2 w2 = (f2){w, w};
#pragma unroll
                    for (int j = 0; j < P; ++j)
                        acc[i][j] = __builtin_elementwise_fma(w2, v[j + K - 1 - kw], acc[i][j]);
                }
        }
    };

    GS gs;
    gs.init(L, oh0, ow0, tid);
    constexpr bool ONE = GP;
    float va[GS::NV][GS::NE], vb[ONE ? 1 : GS::NV][GS::NE];
    gs.load(L, a, b, 0, va);
    if constexpr (ONE) {
        // pooled stager (seven values per element): one plane ahead, one register set -- 85
        // instead of 105 VGPRs, five waves per SIMD instead of four (with the head epilogue's
        // 22 KB of LDS); nconv2's input gradient 353 -> 332 us alone, the graphed step within
        // noise (the weight gradients share the CUs), profiles/r5_ab_dgrad_occupancy.log
#pragma unroll 1
        for (int o = 0; o < COUT; ++o) {
            const int bufi = o & 1;
            gs.store(L, o, va, tile + bufi * GS::PLANE_STRIDE);
            __syncthreads();
            gs.load(L, a, b, o + 1 < COUT ? o + 1 : COUT - 1, va);
            fma_plane(o, bufi);
        }
    } else {
    if (COUT > 1) gs.load(L, a, b, 1, vb);
#pragma unroll 1
    for (int o = 0; o < COUT; o += 2) {
        gs.store(L, o, va, tile);
        __syncthreads();
        gs.load(L, a, b, o + 2 < COUT ? o + 2 : COUT - 1, va);  // unconditional (see fwd_tiled)
        fma_plane(o, 0);
        if (o + 1 < COUT) {
            gs.store(L, o + 1, vb, tile + GS::PLANE_STRIDE);
            __syncthreads();
            gs.load(L, a, b, o + 3 < COUT ? o + 3 : COUT - 1, vb);
            fma_plane(o + 1, 1);
        }
    }
    }

    // ---- epilogue: gx = G_xc*c, gc = G_c + G_xc*x, routed through the glue's backward ----
    if constexpr (HW) {  // nconv2's input gradient feeds nconv1's weight gradient in-tile
        static_assert(MODE == NCONV_LOAD_PLAIN && P == 2, "fused head weight gradient: plain 2-pixel tiles");
        __syncthreads();  // the staging tile is free
        if constexpr (HW) head_wgrad_epilogue<CIN, C::TH, C::TW>(d, a, b, ih0, iw0, ty, tx, acc, tile);
        return;
    }
    const int ih = ih0 + ty;
    if (ih >= L.H) return;
    const int iwb = iw0 + tx;
    const bool full = (L.W % P) == 0 && iwb + P <= L.W;  // P-aligned, fully in range
    const bool accm = a.accumulate != 0;
    typedef typename VecOf<P>::T V;
#pragma unroll
    for (int i = 0; i < CIN; ++i) {
        if constexpr (MODE == NCONV_LOAD_POOL2) {
            if (P == 2 && full && (L.a.W & 3) == 0) {
                // the two pooled pixels' 2x2 windows are 4 columns x 2 rows of the producer: 16-byte
                // loads of x / c for the argmax, 16-byte stores (or read-modify-writes) of gx / gc with
                // 0 at the other three slots (what the reference's max_pool2d backward adds there)
                const size_t W2 = (size_t)L.a.W;
                const size_t i0 = plane_idx(b, i, L.a.C, L.a.H, L.a.W, 2 * ih, 2 * iwb);
                const f4 x0 = *reinterpret_cast<const f4*>(L.a.x + i0);
                const f4 x1 = *reinterpret_cast<const f4*>(L.a.x + i0 + W2);
                const f4 c0 = *reinterpret_cast<const f4*>(L.a.c + i0);
                const f4 c1 = *reinterpret_cast<const f4*>(L.a.c + i0 + W2);
                f4 gx[2], gc[2];
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    int ax, ac;
                    const float xm = pool4(x0[2 * j], x0[2 * j + 1], x1[2 * j], x1[2 * j + 1], ax);
                    const float cm = pool4(c0[2 * j], c0[2 * j + 1], c1[2 * j], c1[2 * j + 1], ac);
                    const float vx = acc[i][j].x * cm, vc = acc[i][j].y + acc[i][j].x * xm;
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        gx[s >> 1][2 * j + (s & 1)] = (s == ax) ? vx : 0.f;
                        gc[s >> 1][2 * j + (s & 1)] = (s == ac) ? vc : 0.f;
                    }
                }
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if (a.gxa) {
                        f4* p = reinterpret_cast<f4*>(a.gxa + i0 + r * W2);
                        *p = accm ? *p + gx[r] : gx[r];
                    }
                    if (a.gca) {
                        f4* p = reinterpret_cast<f4*>(a.gca + i0 + r * W2);
                        *p = accm ? *p + gc[r] : gc[r];
                    }
                }
                if (!accm)
#pragma unroll
                    for (int j = 0; j < P; ++j) pool_zero_leftovers(d, a, b, i, ih, iwb + j);
                continue;
            }
#pragma unroll
            for (int j = 0; j < P; ++j)
                if (iwb + j < L.W) {
                    route_grad<MODE>(d, a, b, i, ih, iwb + j, acc[i][j].x, acc[i][j].y, tmp_x, tmp_c);
                    if (!accm) pool_zero_leftovers(d, a, b, i, ih, iwb + j);
                }
        } else {
            const ChanSrc s = chan_src<MODE>(d, b, i);
            if (!full) {
#pragma unroll
                for (int j = 0; j < P; ++j)
                    if (iwb + j < L.W) route_grad<MODE>(d, a, b, i, ih, iwb + j, acc[i][j].x, acc[i][j].y, tmp_x, tmp_c);
                continue;
            }
            // vector path: P consecutive pixels of one row
            float x[P], c[P];
            if (s.kind == kUp) {
#pragma unroll
                for (int j = 0; j < P; ++j) load_chan(d, s, ih, iwb + j, x[j], c[j]);
            } else {
                const V xv = *reinterpret_cast<const V*>(s.x + ih * s.W + iwb);
#pragma unroll
                for (int j = 0; j < P; ++j) x[j] = xv[j];
                if (s.kind == kThresh) {
#pragma unroll
                    for (int j = 0; j < P; ++j) c[j] = (x[j] > L.thresh) ? 1.0f : 0.0f;
                } else {
                    const V cv = *reinterpret_cast<const V*>(s.c + ih * s.W + iwb);
#pragma unroll
                    for (int j = 0; j < P; ++j) c[j] = cv[j];
                }
            }
            V gxv, gcv;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                gxv[j] = acc[i][j].x * c[j];
                gcv[j] = acc[i][j].y + acc[i][j].x * x[j];
            }
            float *gxp, *gcp;
            size_t off;
            bool acc_here = accm;
            if (s.kind == kUp) {  // upsampled channel: stage for upsample_bwd_gather
                const bool skip_first = (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST);
                const int cb = skip_first ? i - L.a.C : i;
                off = plane_idx(b, cb, L.b.C, L.H, L.W, ih, iwb);
                gxp = tmp_x;
                gcp = tmp_c;
                acc_here = false;
            } else {
                const int ca = (MODE == NCONV_LOAD_UPCAT_UP_FIRST) ? i - L.b.C : i;
                off = plane_idx(b, ca, L.a.C, L.a.H, L.a.W, ih, iwb);
                gxp = a.gxa;
                gcp = (s.kind == kThresh) ? nullptr : a.gca;
            }
            if (gxp) {
                V* p = reinterpret_cast<V*>(gxp + off);
                *p = acc_here ? *p + gxv : gxv;
            }
            if (gcp) {
                V* p = reinterpret_cast<V*>(gcp + off);
                *p = acc_here ? *p + gcv : gcv;
            }
        }
    }
}

// ---- dgrad, phase form for an exactly 2x nearest-upsampled half (16 = 8 + 8 -> 8, 3x3, stride 1) ----
// The upsampled channels' input gradient is only needed summed over each 2x2 block (the
// nearest-upsample backward), and a block's sum is a 4x4 correlation of {gN, gD} with box-summed
// weights. Low pixel (lr, lc) of the tile covers full-resolution rows 2lr + e (e = 0, 1); staged
// output row 2lr + t receives input row 2lr + e through tap kh = e + 2 - t, so t = 0..3 collects the
// taps S(0) = {2}, S(1) = {1, 2}, S(2) = {0, 1}, S(3) = {0} (columns alike):
//     SG[i][lr][lc] = sum_o sum_{t,u} Wb[o][i][t][u] * g[o][2lr + t][2lc + u],  Wb = sum_{S(t) x S(u)} W
// 16 taps per low pixel instead of 4 x 9 per block, and the result goes straight to the producer's
// gradient (gx = SG_xc * c, gc = SG_c + SG_xc * x at the low pixel): no staged full-resolution plane,
// no gather kernel. The 8 skip channels run as in dgrad_tiled. Thread roles: 2 skip pixels x 8
// channels (dgrad_tiled's map) plus one low pixel x 4 upsampled channels, the channel half
// wave-uniform (waves 0-1 / 2-3) so the box weights stay scalar.
__global__ __launch_bounds__(kT) void box_weights(const float* __restrict__ w, int first_up, float* __restrict__ wb) {
    const int e = blockIdx.x * kT + threadIdx.x;  // [o][i][t][u], 8 x 8 x 4 x 4
    if (e < 1024) wb[e] = box_weight(w, first_up, e);
}

template <int MODE, bool T7 = false>
__global__ __launch_bounds__(kT) void dgrad_phase(LayerDev d, BwdArgs a, const float* __restrict__ wbox) {
    using C = DgCfg<16, 3>;
    using GS = GTileStager<C::OHT, C::OWT, C::OWP, false, T7>;
    constexpr int P = C::P, K = 3, CS = 8;
    constexpr int SK0 = (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST) ? 0 : 8;  // first skip channel of W
    static_assert(C::TH % 2 == 0 && C::TW % 2 == 0 && C::OHT >= C::TH + 2 && C::OWT >= C::TW + 2, "low tile");
    __shared__ __attribute__((aligned(16))) f2 tile[2 * GS::PLANE_STRIDE];
    const nconv_layer& L = d.L;
    const float* __restrict__ wgt = L.weight;
    const TileCoord tcd = xcd_tile((L.W + C::TW - 1) / C::TW, (L.H + C::TH - 1) / C::TH, L.B);
    const int tid = threadIdx.x, b = tcd.b;
    const int ih0 = tcd.ty * C::TH, iw0 = tcd.tx * C::TW;
    const int oh0 = ih0 + L.PH - (K - 1), ow0 = iw0 + L.PW - (K - 1);
    const int ty = tid / C::TPR, tx = (tid % C::TPR) * P;
    const int half = __builtin_amdgcn_readfirstlane(tid >> 7);  // upsampled channels 4 half .. +3
    const int lq = tid & 127, lr = lq / (C::TW / 2), lc = lq % (C::TW / 2);
    static_assert((C::TH / 2) * (C::TW / 2) == 128, "one low pixel per thread and channel half");

    f2 acc[CS][P], au[4];
#pragma unroll
    for (int i = 0; i < CS; ++i)
#pragma unroll
        for (int j = 0; j < P; ++j) acc[i][j] = (f2){0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) au[c] = (f2){0.f, 0.f};

    auto fma_plane = [&](int o, int bufi) {
        const f2* pl = &tile[bufi * GS::PLANE_STRIDE];
        const f2* row = pl + (ty + K - 1) * C::OWP + tx;
        const float* wr = wgt + ((size_t)o * 16 + SK0) * K * K;
#pragma unroll 1
        for (int kh = 0; kh < K; ++kh, row -= C::OWP, wr += K) {
            f2 v[C::NV];
#pragma unroll
            for (int m = 0; m < C::NV / 2; ++m) {
                const f4 qv = reinterpret_cast<const f4*>(row)[m];
                v[2 * m] = qv.xy;
                v[2 * m + 1] = qv.zw;
            }
#pragma unroll
            for (int kw = 0; kw < K; ++kw)
#pragma unroll
                for (int i = 0; i < CS; ++i) {
                    const float w = wr[i * K * K + kw];
                    const f2 w2 = (f2){w, w};
#pragma unroll
                    for (int j = 0; j < P; ++j)
                        acc[i][j] = __builtin_elementwise_fma(w2, v[j + K - 1 - kw], acc[i][j]);
                }
        }
        const f2* q = pl + (2 * lr) * C::OWP + 2 * lc;
        const float* wb = wbox + ((size_t)o * 8 + 4 * half) * 16;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f4 q0 = reinterpret_cast<const f4*>(q + t * C::OWP)[0];
            const f4 q1 = reinterpret_cast<const f4*>(q + t * C::OWP)[1];
            const f2 g[4] = {q0.xy, q0.zw, q1.xy, q1.zw};
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float w = wb[c * 16 + t * 4 + u];
                    au[c] = __builtin_elementwise_fma((f2){w, w}, g[u], au[c]);
                }
        }
    };

    GS gs;
    gs.init(L, oh0, ow0, tid);
    // one plane ahead with one register set (as dgrad_tiled's pooled stager): 79 instead of 109
    // VGPRs, six waves per SIMD instead of four; the tail's input gradient 235 -> 200 us alone
    // (profiles/r5_ab_dgrad_phase_one_ahead.log)
    constexpr bool ONE = true;
    float va[4][GS::NE], vb[ONE ? 1 : 4][GS::NE];
    if constexpr (T7) {
        float v7[3][GS::NE];
        gs.t7_load(L, a, b, oh0, ow0, tid, v7);
        gs.load(L, a, b, 0, va);
        if constexpr (!ONE) gs.load(L, a, b, 1, vb);
        gs.t7_form(a, v7);
    } else {
        gs.load(L, a, b, 0, va);
        if constexpr (!ONE) gs.load(L, a, b, 1, vb);
    }
    if constexpr (ONE) {
#pragma unroll 1
        for (int o = 0; o < 8; ++o) {
            const int bufi = o & 1;
            gs.store(L, o, va, tile + bufi * GS::PLANE_STRIDE, T7 ? a.t7w[o] : 0.f);
            __syncthreads();
            gs.load(L, a, b, o + 1 < 8 ? o + 1 : 7, va);
            fma_plane(o, bufi);
        }
    } else {
#pragma unroll 1
    for (int o = 0; o < 8; o += 2) {
        gs.store(L, o, va, tile, T7 ? a.t7w[o] : 0.f);
        __syncthreads();
        gs.load(L, a, b, o + 2 < 8 ? o + 2 : 7, va);
        fma_plane(o, 0);
        gs.store(L, o + 1, vb, tile + GS::PLANE_STRIDE, T7 ? a.t7w[o + 1] : 0.f);
        __syncthreads();
        gs.load(L, a, b, o + 3 < 8 ? o + 3 : 7, vb);
        fma_plane(o + 1, 1);
    }
    }

    const bool accm = a.accumulate != 0;
    // ---- upsampled half: the low pixel's gradient, straight into the producer's planes ----
    {
        const int lh = (ih0 >> 1) + lr, lw = (iw0 >> 1) + lc;
        if (lh < L.b.H && lw < L.b.W) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const size_t off = plane_idx(b, 4 * half + c, L.b.C, L.b.H, L.b.W, lh, lw);
                const float x = L.b.x[off], cf = L.b.c[off];
                if (a.gxb) put(a.gxb, off, au[c].x * cf, accm);
                if (a.gcb) put(a.gcb, off, au[c].y + au[c].x * x, accm);
            }
        }
    }
    // ---- skip half: gx = G_xc*c, gc = G_c + G_xc*x at full resolution ----
    const int ih = ih0 + ty, iwb = iw0 + tx;
    if (ih >= L.H) return;
    const bool full = (L.W % P) == 0 && iwb + P <= L.W;
#pragma unroll
    for (int i = 0; i < CS; ++i) {
        const size_t off = plane_idx(b, i, L.a.C, L.a.H, L.a.W, ih, iwb);
        if (full) {
            const f2 xv = *reinterpret_cast<const f2*>(L.a.x + off);
            const f2 cv = *reinterpret_cast<const f2*>(L.a.c + off);
            const f2 gxv = {acc[i][0].x * cv.x, acc[i][1].x * cv.y};
            const f2 gcv = {acc[i][0].y + acc[i][0].x * xv.x, acc[i][1].y + acc[i][1].x * xv.y};
            if (a.gxa) {
                f2* p = reinterpret_cast<f2*>(a.gxa + off);
                *p = accm ? *p + gxv : gxv;
            }
            if (a.gca) {
                f2* p = reinterpret_cast<f2*>(a.gca + off);
                *p = accm ? *p + gcv : gcv;
            }
        } else {
#pragma unroll
            for (int j = 0; j < P; ++j)
                if (iwb + j < L.W) {
                    const float x = L.a.x[off + j], cf = L.a.c[off + j];
                    if (a.gxa) put(a.gxa, off + j, acc[i][j].x * cf, accm);
                    if (a.gca) put(a.gca, off + j, acc[i][j].y + acc[i][j].x * x, accm);
                }
        }
    }
}

// the phase input gradient applies: exact fp32 backward of a DNET-shaped exactly-2x UpCat layer
static bool dgrad_phase_ok(const nconv_layer& L) {
    const bool up = L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;
    if (!up || L.bwd_math != NCONV_MATH_FP32) return false;
    if (L.Cin != 16 || L.Cout != 8 || L.a.C != 8 || L.b.C != 8 || L.KH != 3 || L.KW != 3) return false;
    if (L.SH != 1 || L.SW != 1 || L.DH != 1 || L.DW != 1 || L.groups != 1) return false;
    return L.a.H == L.H && L.a.W == L.W && L.H == 2 * L.b.H && L.W == 2 * L.b.W;
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
        if (MODE == NCONV_LOAD_POOL2 && !a.accumulate) pool_zero_leftovers(d, a, b, ci, ih, iw);
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
                                                          float* gxb, float* gcb, int accumulate) {
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
        if (accumulate) {
            if (gxb) gxb[idx] += sx;
            if (gcb) gcb[idx] += sc;
        } else {
            if (gxb) gxb[idx] = sx;
            if (gcb) gcb[idx] = sc;
        }
    }
}

// ---- wgrad: tiled partial sums, stride 1 ------------------------------------------------------------
// A thread owns one (o, i) weight pair with all K*K taps in registers and a subset ("sub") of each
// 4 x 64 output tile: rows, or for small Cin*Cout also column segments, so all 256 threads work
// for every layer shape. Per output pixel it reads g = {gN, gD} once and, for each kernel row, one
// new input {x*c, c} into a sliding window: K+1 LDS reads per K*K packed FMAs
// {sum x*c*gN, sum c*gD} += {x*c, c} * {gN, gD}.
constexpr int pow2ceil(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// One kernel row of the weight-gradient correlation over SEGW output columns:
// acc[kw] += in[c + kw] * g[c]  ({x*c, c} * {gN, gD} elementwise). Circular window: input column
// c lives in slot c % K; stepping K columns at a time keeps every slot index a compile-time
// constant, so the window never moves between registers.
template <int K, int SEGW>
__device__ __forceinline__ void wgrad_row(const f2* ir, const f2* gr, f2 (&acc)[K]) {
    f2 win[K];
#pragma unroll
    for (int kw = 0; kw < K - 1; ++kw) win[kw] = ir[kw];
    constexpr int NSTEP = SEGW / K, REM = SEGW % K;
#pragma unroll 2
    for (int st = 0; st < NSTEP; ++st) {
        const int cc = st * K;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const f2 g = gr[cc + j];
            win[(j + K - 1) % K] = ir[cc + j + K - 1];
#pragma unroll
            for (int kw = 0; kw < K; ++kw) acc[kw] = __builtin_elementwise_fma(win[(j + kw) % K], g, acc[kw]);
        }
    }
#pragma unroll
    for (int j = 0; j < REM; ++j) {
        const int cc = NSTEP * K;
        const f2 g = gr[cc + j];
        win[(j + K - 1) % K] = ir[cc + j + K - 1];
#pragma unroll
        for (int kw = 0; kw < K; ++kw) acc[kw] = __builtin_elementwise_fma(win[(j + kw) % K], g, acc[kw]);
    }
}

template <int CIN, int COUT, int K>
struct WgCfg {
    static constexpr int TH = 4, TW = 64;  // TH*TW == kT: one output pixel per thread while staging
    static constexpr int IHT = TH + K - 1, IHTP = (IHT + 3) / 4 * 4, IWT = TW + K - 1;
    // plane strides = 1 (mod 32) f2 so that the distinct channel planes a wave reads hit
    // different bank pairs (bank = dword % 64).
    static constexpr int IPL = ((IHTP * IWT + 31) / 32) * 32 + 1;
    static constexpr int GPL = TH * TW + 1;
    static constexpr int CW = CIN < 8 ? CIN : 8;  // input channels staged per chunk
    static_assert(CIN % CW == 0, "input channel chunking");
    static constexpr int NCH = CIN / CW;
    static constexpr int NCB = COUT * CW;  // (o, i) pairs of one chunk
    static constexpr int NCBP = pow2ceil(NCB);
    static_assert(NCBP <= kT, "wgrad_tiled: Cout*min(Cin,8) must be <= 256");
    static_assert(K <= 7, "wgrad_tiled: kernel rows dispatched through a switch of 7 cases");
    static constexpr int NSUB = kT / NCBP;
    static constexpr int NSEG = NSUB > TH ? NSUB / TH : 1;  // column segments per row
    static constexpr int SEGW = TW / NSEG;
    static constexpr int LDS_F2 = CW * IPL + COUT * GPL;
};

template <int CIN, int COUT, int K, int MODE>
__global__ __launch_bounds__(kT) void wgrad_tiled(LayerDev d, BwdArgs a, float* part, int ntile_w,
                                                  int ntile_h) {
    using C = WgCfg<CIN, COUT, K>;
    extern __shared__ __attribute__((aligned(16))) f2 smem[];
    f2* sin = smem;
    f2* sg = smem + C::CW * C::IPL;
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x;
    const int ntiles = ntile_w * ntile_h * L.B;
    const int cb = tid % C::NCBP, sub = tid / C::NCBP;
    const bool active = cb < C::NCB;
    const int il = active ? cb % C::CW : 0, o = active ? cb / C::CW : 0;
    // rows / column segment of this thread's sub
    const int r_first = (C::NSUB > C::TH) ? sub % C::TH : sub;
    const int r_step = (C::NSUB > C::TH) ? C::TH : C::NSUB;
    const int c_first = (C::NSUB > C::TH) ? (sub / C::TH) * C::SEGW : 0;

    f2 acc[C::NCH][K][K];
#pragma unroll
    for (int ch = 0; ch < C::NCH; ++ch)
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
            for (int kw = 0; kw < K; ++kw) acc[ch][kh][kw] = (f2){0.f, 0.f};
    float gb_acc[COUT], gs_acc[COUT];
#pragma unroll
    for (int oo = 0; oo < COUT; ++oo) gb_acc[oo] = gs_acc[oo] = 0.f;

    // a contiguous run of row-major tiles per block: neighbouring tiles' halos hit the same L2
    const int per_blk = (ntiles + gridDim.x - 1) / gridDim.x;
    const int t_end = min(ntiles, ((int)blockIdx.x + 1) * per_blk);
    for (int t = blockIdx.x * per_blk; t < t_end; ++t) {
        const int tw = t % ntile_w, th = (t / ntile_w) % ntile_h, b = t / (ntile_w * ntile_h);
        const int oh0 = th * C::TH, ow0 = tw * C::TW;
        const int ih0 = oh0 - L.PH, iw0 = ow0 - L.PW;
        __syncthreads();
        {   // g plane: one output pixel per thread per channel; loads clamped and issued up front
            const int r = tid / C::TW, col = tid % C::TW;
            const int oh = oh0 + r, ow = ow0 + col;
            const bool in = (oh < L.Ho) && (ow < L.Wo);
            const int ohc = oh < L.Ho ? oh : L.Ho - 1, owc = ow < L.Wo ? ow : L.Wo - 1;
#pragma unroll
            for (int oo = 0; oo < COUT; ++oo) {
                const size_t gi = plane_idx(b, oo, COUT, L.Ho, L.Wo, ohc, owc);
                const float gy = a.gy[gi], co = a.co[gi], yv = a.y[gi];
                const float gco = a.gco ? a.gco[gi] : 0.f;
                float gN, gD;
                nconv_grad_nd(gy, gco, yv, co, L.eps, L.bias[oo], L.wsum[oo], gN, gD);
                gb_acc[oo] += in ? gy : 0.f;
                gs_acc[oo] = in ? fmaf(gco, co, gs_acc[oo]) : gs_acc[oo];
                sg[oo * C::GPL + tid] = in ? (f2){gN, gD} : (f2){0.f, 0.f};
            }
        }
#pragma unroll
        for (int ch = 0; ch < C::NCH; ++ch) {
            if (ch) __syncthreads();
            for (int ci = 0; ci < C::CW; ++ci)
                stage_plane<C::IHT, C::IWT, C::IWT>(d, chan_src<MODE>(d, b, ch * C::CW + ci), sin + ci * C::IPL, ih0,
                                                    iw0, tid);
            __syncthreads();
            if (active) {
                for (int r = r_first; r < C::TH; r += r_step) {
                    const f2* gr = sg + o * C::GPL + r * C::TW + c_first;
                    // kernel rows one at a time (a runtime loop over a compile-time switch keeps
                    // acc statically indexed without letting the scheduler hoist every row's
                    // LDS reads into registers at once)
#pragma unroll 1
                    for (int kh = 0; kh < K; ++kh) {
                        const f2* ir = sin + il * C::IPL + (r + kh) * C::IWT + c_first;
                        switch (kh) {
#define NCONV_WG_ROW(KH) \
    case KH:             \
        if constexpr (KH < K) wgrad_row<K, C::SEGW>(ir, gr, acc[ch][KH]); \
        break;
                            NCONV_WG_ROW(0)
                            NCONV_WG_ROW(1)
                            NCONV_WG_ROW(2)
                            NCONV_WG_ROW(3)
                            NCONV_WG_ROW(4)
                            NCONV_WG_ROW(5)
                            NCONV_WG_ROW(6)
#undef NCONV_WG_ROW
                        }
                    }
                }
            }
        }
    }

    // ---- combine the subs in a fixed order, then the gb / gs sums; write the partial row ----
    // partial[blk] = { gW-partial[COUT*CIN*K*K], sum gy[COUT], sum gco*cout[COUT] }
    constexpr int NW = COUT * CIN * K * K;
    float* out = part + (size_t)blockIdx.x * (NW + 2 * COUT);
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
    if (active) {
#pragma unroll
        for (int ch = 0; ch < C::NCH; ++ch) {
            const int i = ch * C::CW + il;
#pragma unroll
            for (int kh = 0; kh < K; ++kh)
#pragma unroll
                for (int kw = 0; kw < K; ++kw)
                    red[sub * NW + ((o * CIN + i) * K + kh) * K + kw] = acc[ch][kh][kw].x + acc[ch][kh][kw].y;
        }
    }
    __syncthreads();
    for (int w = tid; w < NW; w += kT) {
        float sum = 0.f;
        for (int sb = 0; sb < C::NSUB; ++sb) sum += red[sb * NW + w];
        out[w] = sum;
    }
    __syncthreads();
#pragma unroll
    for (int oo = 0; oo < COUT; ++oo) {
        red[oo * kT + tid] = gb_acc[oo];
        red[(COUT + oo) * kT + tid] = gs_acc[oo];
    }
    __syncthreads();
    if (tid < 2 * COUT) {
        float sum = 0.f;
        for (int k = 0; k < kT; ++k) sum += red[tid * kT + k];
        out[NW + tid] = sum;
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
// Stage 1: sub[y][e] = sum of part[k][e] over the y-th of kReduceSplit contiguous slices of the
// partial rows, for every entry e of a row (weights, sum gy, sum gco*cout). A 256-thread block owns
// 64 consecutive entries of one slice; its 4 waves sum interleaved rows (coalesced 256-B rows,
// 8 independent loads in flight per lane) and combine the 4 subtotals in LDS in a fixed order.
// Stage 2 (wgrad_finish) adds the kReduceSplit slice sums in order — deterministic, no atomics.
constexpr int kReduceSplit = 16;

// Both stages take a table of up to kMaxRedJobs layers (nconv_wgrad_reduce: every layer of a
// backward pass in two launches instead of two per layer); a block finds its layer by a
// wave-uniform scan of the table's first-block offsets.
struct RedTable {
    RedJob j[kMaxRedJobs];
    int x0[kMaxRedJobs + 1];  // first stage-1 block (64 entries of a row) of each job
    int f0[kMaxRedJobs + 1];  // first stage-2 block of each job
    int n;
};

__device__ __forceinline__ int red_job(const int* first, int n, int blk) {
    int k = 0;
    while (k + 1 < n && blk >= first[k + 1]) ++k;
    return k;
}

// A flat job's chunk sum (nconv_wgrad_reduce_ex): chunk c of kSumChunks contiguous chunks of the
// vector, lane-strided partial sums, then a fixed-order LDS tree.
__device__ __forceinline__ float block_tree_sum(float* red, float s) {
    red[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int h = kT / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    return red[0];
}

__global__ __launch_bounds__(kT) void wgrad_reduce_sum(const RedTable T) {
    __shared__ float red[kT];
    const int k = red_job(T.x0, T.n, blockIdx.x);
    const RedJob& J = T.j[k];
    if (J.flat) {
        const int c = (blockIdx.x - T.x0[k]) * kReduceSplit + blockIdx.y;
        const long long n = J.nblk, per = (n + kSumChunks - 1) / kSumChunks;
        const long long e0 = c * per, e1 = e0 + per < n ? e0 + per : n;
        float s = 0.f;
        for (long long e = e0 + threadIdx.x; e < e1; e += kT) s += J.part[e];
        const float t = block_tree_sum(red, s);
        if (threadIdx.x == 0) J.sub[c] = t;
        return;
    }
    const int stride = J.nw + 2 * J.cout, nblk = J.nblk;
    const float* part = J.part;
    float* sub = const_cast<float*>(J.part) + (size_t)nblk * stride;
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int e = (blockIdx.x - T.x0[k]) * 64 + lane;
    const int per = (nblk + kReduceSplit - 1) / kReduceSplit;
    const int k0 = blockIdx.y * per, k1 = min(nblk, k0 + per);
    float s = 0.f;
    if (e < stride) {
        int r = k0 + grp;
        for (; r + 28 < k1; r += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(r + 4 * u) * stride + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; r < k1; r += 4) s += part[(size_t)r * stride + e];
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (grp == 0 && e < stride)
        sub[(size_t)blockIdx.y * stride + e] = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
}

// Stage 2: tot = sum of the slice sums; gW[w] = tot[w] + gs[o(w)] with gs = -(sum gco*cout)/s
// (d cout / d s, cout = D/s), gb = sum gy.
__device__ __forceinline__ float slice_total(const float* sub, int stride, int e) {
    float t = 0.f;
#pragma unroll
    for (int y = 0; y < kReduceSplit; ++y) t += sub[(size_t)y * stride + e];
    return t;
}

__global__ __launch_bounds__(kT) void wgrad_finish(const RedTable T) {
    __shared__ float red[kT];
    const int k = red_job(T.f0, T.n, blockIdx.x);
    const RedJob& J = T.j[k];
    if (J.flat) {  // the kSumChunks chunk sums: kSumChunks / kT per thread in order, then the tree
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < kSumChunks / kT; ++i) s += J.sub[threadIdx.x * (kSumChunks / kT) + i];
        const float t = block_tree_sum(red, s);
        if (threadIdx.x == 0) J.gb[0] = t;
        return;
    }
    const int nw = J.nw, cout = J.cout, stride = nw + 2 * cout;
    const float* sub = J.part + (size_t)J.nblk * stride;
    const int w = (blockIdx.x - T.f0[k]) * kT + threadIdx.x;
    if (w < nw) {
        const int o = w / J.fan;
        if (J.gw) J.gw[w] = slice_total(sub, stride, w) + (-slice_total(sub, stride, nw + cout + o) / J.wsum[o]);
    } else if (w < nw + cout && J.gb) {
        J.gb[w - nw] = slice_total(sub, stride, w);
    }
}

int launch_wgrad_reduce_multi(int n, const RedJob* jobs, hipStream_t st, const char** why) {
    if (n < 1 || n > kMaxRedJobs) {
        *why = "between 1 and 16 layers per reduction";
        return -22;
    }
    RedTable T;
    T.n = n;
    T.x0[0] = T.f0[0] = 0;
    static_assert(kSumChunks % kReduceSplit == 0 && kSumChunks % kT == 0, "flat chunks");
    for (int k = 0; k < n; ++k) {
        T.j[k] = jobs[k];
        const int stride = jobs[k].nw + 2 * jobs[k].cout;
        T.x0[k + 1] = T.x0[k] + (jobs[k].flat ? kSumChunks / kReduceSplit : (stride + 63) / 64);
        T.f0[k + 1] = T.f0[k] + (jobs[k].flat ? 1 : (jobs[k].nw + jobs[k].cout + kT - 1) / kT);
    }
    for (int k = n + 1; k <= kMaxRedJobs; ++k) T.x0[k] = T.f0[k] = 0;
    hipLaunchKernelGGL(wgrad_reduce_sum, dim3(T.x0[n], kReduceSplit), dim3(kT), 0, st, T);
    hipLaunchKernelGGL(wgrad_finish, dim3(T.f0[n]), dim3(kT), 0, st, T);
    return 0;
}

// part: nblk partial rows followed by kReduceSplit rows of slice sums (see bwd_workspace_bytes);
// with a.defer the rows stay for a later nconv_wgrad_reduce over every layer of the pass
static int launch_wgrad_reduce(const BwdArgs& a, const float* part, int nblk, int nw, int cout, int fan,
                               const float* wsum, hipStream_t st, const char** why) {
    if (a.defer) {
        *a.nparts = nblk;
        return 0;
    }
    const RedJob J{part, wsum, a.gw, a.gb, nblk, nw, cout, fan};
    return launch_wgrad_reduce_multi(1, &J, st, why);
}

// ---- wgrad on the matrix cores (fp32 MFMA 16x16x4, exact f32 products) -----------------------------
// For a 3x3 / 5x5 stride-1 layer the weight gradient is, per output row oh, a GEMM over the
// column index q = ow + kw:
//     gW[o][i][kh][kw] += sum_q  XC[i][oh+kh-PH][q-PW] * gN[o][oh][q-kw]
//                              +  C[i][oh+kh-PH][q-PW] * gD[o][oh][q-kw]
// with rows M = (kh, i) (i fastest) and columns N = (kw, o) (o fastest), K = q: the kernel-row
// shift lives in the A operand (which staged input row) and the kernel-column shift in the B
// operand (which g column), so neither operand is replicated per tap. A workgroup owns a 64-wide
// q strip of one image and walks a segment of output rows: a ring of K+1 staged input rows (one
// new row per output row, no halo re-staging) and a double-buffered {gN, gD} row with a K-1
// column left halo, one barrier per row, the next row's global loads issued before the current
// row's MFMAs. Each wave takes 16 of the 64 columns (4 MFMA k-steps per operand pair) and keeps the
// whole (M x N) tile in accumulators; the four waves' tiles are summed in a fixed order at the end
// into the block's partial row (then wgrad_reduce_sum / wgrad_finish, as for wgrad_tiled).
typedef float f4acc __attribute__((ext_vector_type(4)));

template <int CIN, int COUT, int K>
struct WmCfg {
    static constexpr int TW = 64;
    static constexpr int M = CIN * K, N = COUT * K;
    static constexpr int MT = (M + 15) / 16, NT = (N + 15) / 16;
    // LDS banks of the operand reads (ds_read_b32: bank = dword address mod 32, the two 32-lane
    // halves separate; a half holds k = lane >> 4 in {0, 1} (or {2, 3}) x 16 rows / columns):
    // A: row m = (kh, i) at slot(kh) * SLOT + i * XP + k. XP == 2 (mod 32) puts a kernel row's
    //    channels on 2i + k; for CIN = 8 a 16-row tile holds two kernel rows, in consecutive ring
    //    slots, and SLOT == 16 (mod 32) puts the second on the other 16 banks (the ring's wrap is an
    //    odd number of slots back, == 16 too), so every half reads 32 distinct banks.
    // B: column n = (kw, o) at o * GP + (K-1) - kw + k; lanes with equal o and k - kw read the same
    //    word (broadcast), so a half holds three words per channel, at 4o + {-1, 0, 1} + const with
    //    GP == 4 (mod 32): distinct. (Round 3 had pitches 68 / 72 laid out for 64 banks: 2-way on
    //    A, 4-way on B, ~4.5 K conflict cycles per wave in SQ_LDS_BANK_CONFLICT.)
    static constexpr int XP = TW + 2;
    static constexpr int SLOTS = K + 1;
    static constexpr int SKEW = (2 * CIN) % 32;
    static constexpr int SLOT = CIN * XP + (((SKEW - CIN * XP) % 32) + 32) % 32;
    static constexpr int GW = TW + K - 1;  // g row incl. the left halo
    static constexpr int GP = 68;          // == 4 (mod 32), see above
    static constexpr int ZB = 2;           // padded B columns read the zero row at banks 2, 3 (mod 4): free
    static_assert(GW <= GP, "g row pitch");
    static_assert(XP % 32 == 2 && GP % 32 == 4 && (CIN >= 16 || SLOT % 32 == 16), "bank layout");
    static_assert(COUT % 4 == 0, "g rows are staged four output channels per pass");
    // LDS (floats): xc ring + its zero row | c ring + its zero row | g [buf][part][COUT + 1 rows][GP]
    // (row COUT of each g part is zero). Padded M / N lanes read the zero rows, whose offsets from
    // the xc / gN data equal the c / gD part offsets, so one address per operand serves both parts.
    static constexpr int XR = SLOTS * SLOT;             // the zero row of the xc ring
    static constexpr int C_OFF = XR + GP;               // c ring (its zero row at C_OFF + XR)
    static constexpr int G_OFF = 2 * C_OFF;
    static constexpr int GPART = (COUT + 1) * GP;       // one part of one g buffer
    static constexpr int GBUF = 2 * GPART;
    static constexpr int STAGE = G_OFF + 2 * GBUF;
    static constexpr int RED = 4 * MT * NT * 256;
    static constexpr int LDS = STAGE > RED ? STAGE : RED;
    static constexpr int CPW = (CIN + 3) / 4, OPW = COUT / 4;  // channels staged per wave
};

#ifndef NCONV_WM_WAVES
#define NCONV_WM_WAVES 3
#endif
#ifndef NCONV_WM_STORE_STEP
#define NCONV_WM_STORE_STEP 1  // after which k-step the next row's staging is stored (its loads' latency budget)
#endif
#ifndef NCONV_WM_GP_WAVES
#define NCONV_WM_GP_WAVES 3  // the pooled-gradient (training) instantiation (4: 128 VGPRs, 2 spilled)
#endif
#define NCONV_WM_ATTR __attribute__((amdgpu_waves_per_eu(NCONV_WM_WAVES, 8)))
template <int CIN, int COUT, int K, int MODE, bool GP = false, bool T7 = false>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(GP ? NCONV_WM_GP_WAVES : NCONV_WM_WAVES, 8))) void wgrad_mfma(LayerDev d, BwdArgs a, float* part, int nstrip, int nseg,
                                                 int seg_rows) {
    using C = WmCfg<CIN, COUT, K>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: channel sources stay in SGPRs
    int blk = blockIdx.x;
    const int strip = blk % nstrip;
    blk /= nstrip;
    const int seg = blk % nseg, b = blk / nseg;
    const int ow0 = strip * C::TW;
    const int r0 = seg * seg_rows, r1 = min(L.Ho, r0 + seg_rows);
    constexpr unsigned OOB = 0x80000000u;

    for (int e = tid; e < C::GP; e += kT) {
        lds[C::XR + e] = 0.f;
        lds[C::C_OFF + C::XR + e] = 0.f;
#pragma unroll
        for (int z = 0; z < 4; ++z) lds[C::G_OFF + z * C::GPART + COUT * C::GP + e] = 0.f;
    }

    // per-lane MFMA operand coordinates (A[m = lane&15][k = lane>>4], B[k = lane>>4][n = lane&15])
    const int kq = lane >> 4, ml = lane & 15;
    int a_kh[C::MT], a_ik[C::MT], b_off[C::NT];
#pragma unroll
    for (int t = 0; t < C::MT; ++t) {
        const int m = 16 * t + ml;
        a_kh[t] = m < C::M ? m / CIN : -1;
        a_ik[t] = (m % CIN) * C::XP + kq;
    }
#pragma unroll
    for (int u = 0; u < C::NT; ++u) {
        const int n = 16 * u + ml;
        b_off[u] = n < C::N ? (n % COUT) * C::GP + (K - 1) - n / COUT + kq : COUT * C::GP + C::ZB + kq;
    }

    // ---- staging: one input row (CIN x 64 columns) and one g row (COUT x (64+K-1) columns) ----
    // The g row's 64 + K-1 columns: a main pass (column = lane) for each of the wave's OPW output
    // channels, and one halo pass over all of them -- lane l < OPW (K-1) takes channel w + 4 (l / (K-1))
    // at column 64 + l % (K-1) -- instead of a second pass per channel with K-1 of 64 lanes active.
    // The g tensors are addressed through one resource per image (the channel's plane offset in
    // soffset for the main pass, in the lane's offset for the halo).
    float px[C::CPW], pc[C::CPW];
    constexpr int NG = GP ? 7 : 4;  // gy, gco, y, cout (+ pooled gy, gcout, argmax code)
    constexpr int NH = C::OPW * (K - 1);
    static_assert(NH <= 64, "halo lanes");
    const bool hl = lane < NH;
    const int hkk = hl ? lane / (K - 1) : 0, hcol = 64 + lane % (K - 1), ho = w + 4 * hkk;
    float gq[C::OPW][NG], gh[NG];
    float g7[T7 ? 2 : 1][3];                                     // nconv7's gy, y, cout (T7): main, halo
    float w7n[T7 ? C::OPW : 1], w7d[T7 ? C::OPW : 1];            // nconv7's weight-gradient sums
    float w7nh = 0.f, w7dh = 0.f;
#pragma unroll
    for (int kk = 0; kk < (T7 ? C::OPW : 1); ++kk) w7n[kk] = w7d[kk] = 0.f;
    float gb_acc[C::OPW], gs_acc[C::OPW], gb_h = 0.f, gs_h = 0.f;
#pragma unroll
    for (int kk = 0; kk < C::OPW; ++kk) gb_acc[kk] = gs_acc[kk] = 0.f;

    // UpCat inputs: the wave's channel sources, the up plane's column map and one resource per
    // source image resolved once, not per row (per-row channel resolution cost ~100 SGPR-spill
    // reloads and a general nearest-index path per row); per row only the row map and two offsets.
    constexpr bool UPC = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST;
    const int iw_in = ow0 - L.PW + lane;
    const bool col_in = (unsigned)iw_in < (unsigned)L.W;
    const int sw_up = UPC ? nearest_src(col_in ? iw_in : 0, L.b.W, L.W, d.up_scale_w) : 0;
    bool up_k[C::CPW];
    int so_k[C::CPW];
#pragma unroll
    for (int kk = 0; kk < C::CPW; ++kk) {
        const int i = w + 4 * kk;
        if constexpr (UPC) {
            const bool skip_first = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST;
            const int first_c = skip_first ? L.a.C : L.b.C;
            const bool from_a = skip_first ? (i < first_c) : (i >= first_c);
            up_k[kk] = !from_a;
            so_k[kk] = (from_a ? (skip_first ? i : i - first_c) * L.a.H * L.a.W
                               : (skip_first ? i - first_c : i) * L.b.H * L.b.W) * 4;
        } else {
            up_k[kk] = false;
            so_k[kk] = 0;
        }
    }
    const int abytes = UPC ? L.a.C * L.a.H * L.a.W * 4 : 0, bbytes = UPC ? L.b.C * L.b.H * L.b.W * 4 : 0;
    const float* ax_img = UPC ? L.a.x + (size_t)b * L.a.C * L.a.H * L.a.W : nullptr;
    const float* ac_img = UPC ? L.a.c + (size_t)b * L.a.C * L.a.H * L.a.W : nullptr;
    const float* bx_img = UPC ? L.b.x + (size_t)b * L.b.C * L.b.H * L.b.W : nullptr;
    const float* bc_img = UPC ? L.b.c + (size_t)b * L.b.C * L.b.H * L.b.W : nullptr;
    auto load_in = [&](int ih) {
        if constexpr (UPC) {
            const bool in = (unsigned)ih < (unsigned)L.H && col_in;
            const int sh = nearest_src(in ? ih : 0, L.b.H, L.H, d.up_scale_h);
            const unsigned od = in ? (unsigned)(ih * L.a.W + iw_in) * 4u : OOB;
            const unsigned ou = in ? (unsigned)(sh * L.b.W + sw_up) * 4u : OOB;
#pragma unroll
            for (int kk = 0; kk < C::CPW; ++kk) {
                const int i = w + 4 * kk;
                px[kk] = pc[kk] = 0.f;
                if (i < CIN) {
                    const bool up = up_k[kk];
                    const __amdgpu_buffer_rsrc_t rx = plane_rsrc(up ? bx_img : ax_img, up ? bbytes : abytes);
                    const __amdgpu_buffer_rsrc_t rc = plane_rsrc(up ? bc_img : ac_img, up ? bbytes : abytes);
                    px[kk] = ld_f32s(rx, up ? ou : od, so_k[kk]);
                    pc[kk] = ld_f32s(rc, up ? ou : od, so_k[kk]);
                }
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < C::CPW; ++kk) {
                const int i = w + 4 * kk;
                px[kk] = pc[kk] = 0.f;
                if (i < CIN) load_px<MODE>(d, chan_src<MODE>(d, b, i), ih, iw_in, px[kk], pc[kk]);
            }
        }
    };
    auto store_in = [&](int ih) {
        const int slot = ((ih % C::SLOTS) + C::SLOTS) % C::SLOTS;
#pragma unroll
        for (int kk = 0; kk < C::CPW; ++kk) {
            const int i = w + 4 * kk;
            if (i < CIN) {
                const float cv = (MODE == NCONV_LOAD_THRESH) ? (px[kk] > L.thresh ? 1.0f : 0.0f) : pc[kk];
                lds[slot * C::SLOT + i * C::XP + lane] = px[kk] * cv;
                lds[C::C_OFF + slot * C::SLOT + i * C::XP + lane] = cv;
            }
        }
    };
    const int plane = L.Ho * L.Wo;
    const int Hp = L.Ho >> 1, Wp = L.Wo >> 1, pplane = Hp * Wp;
    auto load_g = [&](int oh) {
        const int ow = ow0 - (K - 1) + lane, owh = ow0 - (K - 1) + hcol;
        const bool row_in = (unsigned)oh < (unsigned)L.Ho;
        const bool in = row_in && (unsigned)ow < (unsigned)L.Wo;
        const bool inh = hl && row_in && (unsigned)owh < (unsigned)L.Wo;
        if constexpr (T7) {
            const int pl7 = a.t7ph * a.t7pw;
            const size_t base7 = (size_t)b * pl7;
            const __amdgpu_buffer_rsrc_t r7g = plane_rsrc(a.t7gy + base7, pl7 * 4);
            const __amdgpu_buffer_rsrc_t r7y = plane_rsrc(a.t7y + base7, pl7 * 4);
            const __amdgpu_buffer_rsrc_t r7c = plane_rsrc(a.t7co + base7, pl7 * 4);
            const unsigned o0 = t7_off(a, oh, ow, L.Ho, L.Wo, OOB), o1 = hl ? t7_off(a, oh, owh, L.Ho, L.Wo, OOB) : OOB;
            g7[0][0] = ld_f32(r7g, o0);
            g7[0][1] = ld_f32(r7y, o0);
            g7[0][2] = ld_f32(r7c, o0);
            g7[1][0] = ld_f32(r7g, o1);
            g7[1][1] = ld_f32(r7y, o1);
            g7[1][2] = ld_f32(r7c, o1);
        }
        const size_t base = (size_t)b * COUT * plane;
        const int bytes = COUT * plane * 4;
        const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + base, bytes);
        const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + base, bytes);
        const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + base, bytes);
        const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + base : a.y, a.gco ? bytes : 0);
        const unsigned off = in ? (unsigned)(oh * L.Wo + ow) * 4u : OOB;
        const unsigned offh = inh ? (unsigned)((ho * L.Ho + oh) * L.Wo + owh) * 4u : OOB;
#pragma unroll
        for (int kk = 0; kk < C::OPW; ++kk) {
            const int so = (w + 4 * kk) * plane * 4;
            gq[kk][1] = ld_f32s(rco, off, so);
            gq[kk][2] = ld_f32s(ry, off, so);
            if constexpr (!T7) {
                gq[kk][0] = ld_f32s(rgy, off, so);
                gq[kk][3] = ld_f32s(rgc, off, so);
            }
        }
        gh[1] = ld_f32(rco, offh);
        gh[2] = ld_f32(ry, offh);
        if constexpr (!T7) {
            gh[0] = ld_f32(rgy, offh);
            gh[3] = ld_f32(rgc, offh);
        }
        if constexpr (GP) {
            const size_t pbase = (size_t)b * COUT * pplane;
            const int pbytes = COUT * pplane * 4;
            const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(a.gpy + pbase, pbytes);
            const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(a.gpc + pbase, pbytes);
            const __amdgpu_buffer_rsrc_t rpa = plane_rsrc((const float*)(a.parg + pbase), pbytes);
            const unsigned po = in ? pool_elem_off(oh, ow, Hp, Wp, OOB) : OOB;
            const unsigned pe = inh ? pool_elem_off(oh, owh, Hp, Wp, OOB) : OOB;
            const unsigned poh = pe != OOB ? pe + (unsigned)(ho * pplane) * 4u : OOB;
#pragma unroll
            for (int kk = 0; kk < C::OPW; ++kk) {
                const int so = (w + 4 * kk) * pplane * 4;
                gq[kk][4] = ld_f32s(rpy, po, so);
                gq[kk][5] = ld_f32s(rpc, po, so);
                gq[kk][6] = ld_f32s(rpa, po, so);
            }
            gh[4] = ld_f32(rpy, poh);
            gh[5] = ld_f32(rpc, poh);
            gh[6] = ld_f32(rpa, poh);
        }
    };
    // the wave's output channels' bias and normaliser, read once (not per row: a load right before
    // its use would put a global-memory round trip into every row)
    float bias_o[C::OPW], wsum_o[C::OPW], w7_o[C::OPW];
#pragma unroll
    for (int kk = 0; kk < C::OPW; ++kk) {
        bias_o[kk] = L.bias[w + 4 * kk];
        wsum_o[kk] = L.wsum[w + 4 * kk];
        w7_o[kk] = T7 ? a.t7w[w + 4 * kk] : 0.f;
    }
    auto store_g = [&](int buf, int oh_cur) {
        float n7[2], d7[2];
        if constexpr (T7)
#pragma unroll
            for (int p = 0; p < 2; ++p) t7_nd(a, g7[p][0], g7[p][1], g7[p][2], n7[p], d7[p]);
        // the 2x2 window slot of the main / halo column (pooled-gradient routing)
        const unsigned sub = (unsigned)((oh_cur & 1) << 1), ow_m = (unsigned)(ow0 - (K - 1) + lane);
        const unsigned ow_h = (unsigned)(ow0 - (K - 1) + hcol);
#pragma unroll
        for (int kk = 0; kk < C::OPW; ++kk) {
            const int o = w + 4 * kk;
            float gy, gco;
            if constexpr (T7) {
                t7_gy(w7_o[kk], n7[0], d7[0], gq[kk][2], gq[kk][1], gy, gco);
                if (lane >= K - 1) {  // nconv7's weight gradient: corr(x*c, gN7) + corr(c, gD7)
                    w7n[kk] = fmaf(gq[kk][2] * gq[kk][1], n7[0], w7n[kk]);
                    w7d[kk] = fmaf(gq[kk][1], d7[0], w7d[kk]);
                }
            } else {
                gy = gq[kk][0];
                gco = gq[kk][3];
            }
            if constexpr (GP)
                pool_route(gy, gco, gq[kk][4], gq[kk][5], __builtin_bit_cast(unsigned, gq[kk][6]), sub | (ow_m & 1u));
            float gN, gD;
            nconv_grad_nd(gy, gco, gq[kk][2], gq[kk][1], L.eps, bias_o[kk], wsum_o[kk], gN, gD);
            float* g = lds + C::G_OFF + buf * C::GBUF + o * C::GP + lane;
            g[0] = gN;
            g[C::GPART] = gD;
            if (lane >= K - 1) {  // this strip's own columns: the bias / wsum gradient sums
                gb_acc[kk] += gy;
                gs_acc[kk] = fmaf(gco, gq[kk][1], gs_acc[kk]);
            }
        }
        {   // halo pass (columns 64 .. 64+K-2, all the strip's own)
            float bo = bias_o[0], so = wsum_o[0], w7 = w7_o[0];
#pragma unroll
            for (int kk = 1; kk < C::OPW; ++kk) {
                bo = hkk == kk ? bias_o[kk] : bo;
                so = hkk == kk ? wsum_o[kk] : so;
                w7 = hkk == kk ? w7_o[kk] : w7;
            }
            float gy, gco;
            if constexpr (T7) {
                t7_gy(w7, n7[1], d7[1], gh[2], gh[1], gy, gco);
                w7nh = fmaf(gh[2] * gh[1], n7[1], w7nh);
                w7dh = fmaf(gh[1], d7[1], w7dh);
            } else {
                gy = gh[0];
                gco = gh[3];
            }
            if constexpr (GP) pool_route(gy, gco, gh[4], gh[5], __builtin_bit_cast(unsigned, gh[6]), sub | (ow_h & 1u));
            float gN, gD;
            nconv_grad_nd(gy, gco, gh[2], gh[1], L.eps, bo, so, gN, gD);
            if (hl) {
                float* g = lds + C::G_OFF + buf * C::GBUF + ho * C::GP + hcol;
                g[0] = gN;
                g[C::GPART] = gD;
            }
            gb_h += gy;
            gs_h = fmaf(gco, gh[1], gs_h);
        }
    };

    f4acc acc[C::MT][C::NT];
#pragma unroll
    for (int t = 0; t < C::MT; ++t)
#pragma unroll
        for (int u = 0; u < C::NT; ++u) acc[t][u] = (f4acc){0.f, 0.f, 0.f, 0.f};

    // The next row is staged DURING this row's MFMAs (its loads before the first half of the k-steps,
    // its stores after it): its input row goes to the ring slot this row does not read (K + 1 slots,
    // K in use), its g row to the other buffer (whose last reader, the previous row, is behind the
    // barrier) -- one barrier per row, and the staging's VALU work interleaved with the MFMAs
    // instead of between barriers.
    if (r0 < r1) {
        for (int kh = 0; kh < K; ++kh) {  // prologue: the segment's first K input rows and g row
            load_in(r0 - L.PH + kh);
            store_in(r0 - L.PH + kh);
        }
        load_g(r0);
        store_g(0, r0);
    }
    __syncthreads();
#pragma unroll 1
    for (int oh = r0; oh < r1; ++oh) {
        const int buf = (oh - r0) & 1;
        const bool more = oh + 1 < r1;
        int ax[C::MT], bn[C::NT];
#pragma unroll
        for (int t = 0; t < C::MT; ++t) {
            const int ih = oh - L.PH + a_kh[t];
            const int slot = ((ih % C::SLOTS) + C::SLOTS) % C::SLOTS;
            ax[t] = a_kh[t] < 0 ? C::XR + kq : slot * C::SLOT + a_ik[t];
        }
#pragma unroll
        for (int u = 0; u < C::NT; ++u) bn[u] = C::G_OFF + buf * C::GBUF + b_off[u];
        if (more) {
            load_in(oh + 1 - L.PH + K - 1);
            load_g(oh + 1);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int q0 = 16 * w + 4 * s;
#pragma unroll
            for (int part = 0; part < 2; ++part) {  // {x*c, gN} then {c, gD}
                float va[C::MT], vb[C::NT];
#pragma unroll
                for (int t = 0; t < C::MT; ++t) va[t] = lds[ax[t] + part * C::C_OFF + q0];
#pragma unroll
                for (int u = 0; u < C::NT; ++u) vb[u] = lds[bn[u] + part * C::GPART + q0];
#pragma unroll
                for (int t = 0; t < C::MT; ++t)
#pragma unroll
                    for (int u = 0; u < C::NT; ++u)
                        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[t], vb[u], acc[t][u], 0, 0, 0);
            }
            if (s == NCONV_WM_STORE_STEP && more) {
                store_in(oh + 1 - L.PH + K - 1);
                store_g(buf ^ 1, oh + 1);
            }
        }
        __syncthreads();
    }

    // ---- the four waves' tiles summed in a fixed order -> this block's partial row ----
    constexpr int NW = COUT * CIN * K * K;
    constexpr int NE = C::MT * C::NT * 256;
    float* out = part + (size_t)blockIdx.x * (NW + 2 * COUT);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < C::MT; ++t)
#pragma unroll
        for (int u = 0; u < C::NT; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) lds[w * NE + (t * C::NT + u) * 256 + r * 64 + lane] = acc[t][u][r];
    __syncthreads();
    for (int e = tid; e < NE; e += kT) {
        const float v = ((lds[e] + lds[NE + e]) + lds[2 * NE + e]) + lds[3 * NE + e];
        const int l = e & 63, r = (e >> 6) & 3, tu = e >> 8;
        const int u = tu % C::NT, t = tu / C::NT;
        const int m = 16 * t + (l >> 4) * 4 + r, n = 16 * u + (l & 15);
        if (m < C::M && n < C::N) {
            const int kh = m / CIN, i = m % CIN, kw = n / COUT, o = n % COUT;
            out[((o * CIN + i) * K + kh) * K + kw] = v;
        }
    }
#pragma unroll
    for (int kk = 0; kk < C::OPW; ++kk) {
        const bool mine = hl && hkk == kk;  // the halo lanes' sums of this channel
        float sb = gb_acc[kk] + (mine ? gb_h : 0.f), ss = gs_acc[kk] + (mine ? gs_h : 0.f);
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            sb += __shfl_xor(sb, sh);
            ss += __shfl_xor(ss, sh);
        }
        if (lane == 0) {
            out[NW + w + 4 * kk] = sb;
            out[NW + COUT + w + 4 * kk] = ss;
        }
    }
    if constexpr (T7) {  // nconv7's partial row: 8 weights, then its (unused) sum gy / sum gcout*cout slots
        float* o7 = a.t7part + (size_t)blockIdx.x * 10;
#pragma unroll
        for (int kk = 0; kk < C::OPW; ++kk) {
            const bool mine = hl && hkk == kk;
            float sn = w7n[kk] + (mine ? w7nh : 0.f), sd = w7d[kk] + (mine ? w7dh : 0.f);
#pragma unroll
            for (int sh = 32; sh > 0; sh >>= 1) {
                sn += __shfl_xor(sn, sh);
                sd += __shfl_xor(sd, sh);
            }
            if (lane == 0) o7[w + 4 * kk] = sn + sd;
        }
        if (tid < 2) o7[8 + tid] = 0.f;
    }
}

// ---- wgrad_mfma over output-row pairs (8 -> 8, 5x5: nconv2 and the down layers) ------------------
// wgrad_mfma's (kh, i) x (kw, o) tile is 40 x 40 for these layers and pads to 48 x 48 (3 x 3 MFMA
// tiles, 69 % of the products useful). Two output rows oh, oh + 1 at once fill the tiles exactly:
// rows M = (r, i), r = 0..K over the K + 1 staged input rows oh - PH + r (48 = 3 tiles), columns
// N = (d, kw, o) over the two g rows oh + d (80 = 5 tiles), so
//     C[(r, i)][(d, kw, o)] += sum_q XC[i][oh - PH + r][q - PW] * gN[o][oh + d][q - kw] (+ C * gD)
// holds the kernel row kh = r - d of output row oh + d: gW[o][i][kh][kw] = C[(kh, i)][(0, kw, o)] +
// C[(kh + 1, i)][(1, kw, o)] (the pairs r = K, d = 0 and r = 0, d = 1 are not taps). 15 MFMAs per
// k-step and operand part for two rows instead of 18, and 8 operand reads instead of 12. The input
// ring holds K + 3 rows (K + 1 in use, two being written for the next pair), the g rows are double
// buffered per pair, the next pair staged under this pair's MFMAs; an odd last row pairs with a
// zero row. Same products, summed in a different
// (fixed) order: within fp32 round-off of wgrad_mfma, deterministic.
template <int CIN, int COUT, int K>
struct Wm2Cfg {
    static constexpr int TW = 64;
    static constexpr int M = (K + 1) * CIN, N = 2 * K * COUT;
    static constexpr int MT = M / 16, NT = N / 16;
    static_assert(M % 16 == 0 && N % 16 == 0, "row-pair tiles fill the MFMA tiles exactly");
    static constexpr int XP = TW + 2;  // == 2 (mod 32): a kernel row's channels on banks 2i + k
    static constexpr int SLOTS = 8;    // K + 3 <= 8: slot = input row & 7
    static_assert(K + 3 <= SLOTS, "input ring");
    // A: a 16-row tile holds two input rows in consecutive slots; SLOT == 16 (mod 32) puts the second
    // on the other 16 banks (and the ring's wrap, 7 slots back, is == 16 too)
    static constexpr int SLOT = CIN * XP + ((((2 * CIN) % 32 - CIN * XP) % 32) + 32) % 32;
    static constexpr int GP = 68;                      // B: channel o at 4o + {kw shifts} (mod 32)
    static constexpr int GROW = COUT * GP + ((((2 - COUT * GP) % 32) + 32) % 32);  // == 2 (mod 32):
    // the tile straddling d = 0 / 1 reads words 4o + {0, 1} and GROW + 4o + {4, 5}: distinct banks
    static constexpr int C_OFF = SLOTS * SLOT;         // c ring after the xc ring
    static constexpr int G_OFF = 2 * C_OFF;
    static constexpr int GPART = 2 * GROW;             // {gN rows d = 0, 1} then {gD rows}
    static constexpr int GBUF = 2 * GPART;
    static constexpr int STAGE = G_OFF + 2 * GBUF;
    static constexpr int TILE = MT * NT * 256;         // one wave's accumulators
    static constexpr int RED = 2 * TILE;               // waves 0 / 1 store, 2 / 3 add
    static constexpr int LDS = STAGE > RED ? STAGE : RED;
    static constexpr int CPW = (CIN + 3) / 4, OPW = COUT / 4;
    static_assert(SLOT % 32 == 16 && XP % 32 == 2 && GP % 32 == 4 && GROW % 32 == 2, "bank layout");
    static_assert(COUT % 4 == 0 && CIN % 4 == 0, "channels staged four per pass");
};

#ifndef NCONV_WM2_WAVES
#define NCONV_WM2_WAVES 3
#endif
#ifndef NCONV_WM2_SCHED
#define NCONV_WM2_SCHED 1
#endif
template <int CIN, int COUT, int K, int MODE, bool GP = false>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(NCONV_WM2_WAVES, 8))) void wgrad_mfma2(
    LayerDev d, BwdArgs a, float* part, int nstrip, int nseg, int seg_rows) {
    using C = Wm2Cfg<CIN, COUT, K>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int strip = blk % nstrip;
    blk /= nstrip;
    const int seg = blk % nseg, b = blk / nseg;
    const int ow0 = strip * C::TW;
    const int r0 = seg * seg_rows, r1 = min(L.Ho, r0 + seg_rows);
    constexpr unsigned OOB = 0x80000000u;

    const int kq = lane >> 4, ml = lane & 15;
    int a_r[C::MT], a_ik[C::MT], b_off[C::NT];
#pragma unroll
    for (int t = 0; t < C::MT; ++t) {
        const int m = 16 * t + ml;
        a_r[t] = m / CIN;
        a_ik[t] = (m % CIN) * C::XP + kq;
    }
#pragma unroll
    for (int u = 0; u < C::NT; ++u) {
        const int n = 16 * u + ml, dd = n / (K * COUT), rem = n % (K * COUT);
        b_off[u] = dd * C::GROW + (rem % COUT) * C::GP + (K - 1) - rem / COUT + kq;
    }

    // ---- staging (as wgrad_mfma, two rows per pair) ----
    constexpr int NG = GP ? 7 : 4;  // gy, gco, y, cout (+ pooled gy, gcout, argmax code)
    constexpr int NH = C::OPW * (K - 1);
    static_assert(NH <= 64, "halo lanes");
    const bool hl = lane < NH;
    const int hkk = hl ? lane / (K - 1) : 0, hcol = 64 + lane % (K - 1), ho = w + 4 * hkk;
    float px[1][C::CPW], pc[1][C::CPW];  // one row's loads in flight at a time (see the loop)
    float gq[1][C::OPW][NG], gh[1][NG];
    float gb_acc[C::OPW], gs_acc[C::OPW], gb_h = 0.f, gs_h = 0.f;
#pragma unroll
    for (int kk = 0; kk < C::OPW; ++kk) gb_acc[kk] = gs_acc[kk] = 0.f;
    const int iw_in = ow0 - L.PW + lane;
    // input row ih (valid: a row of this pair; else zeros, so no value of another segment enters)
    auto load_in = [&](int j, int ih, bool valid) {
#pragma unroll
        for (int kk = 0; kk < C::CPW; ++kk) {
            const int i = w + 4 * kk;
            px[j][kk] = pc[j][kk] = 0.f;
            if (valid) load_px<MODE>(d, chan_src<MODE>(d, b, i), ih, iw_in, px[j][kk], pc[j][kk]);
        }
    };
    auto store_in = [&](int j, int ih) {
        const int slot = ih & (C::SLOTS - 1);
#pragma unroll
        for (int kk = 0; kk < C::CPW; ++kk) {
            const int i = w + 4 * kk;
            const float cv = (MODE == NCONV_LOAD_THRESH) ? (px[j][kk] > L.thresh ? 1.0f : 0.0f) : pc[j][kk];
            lds[slot * C::SLOT + i * C::XP + lane] = px[j][kk] * cv;
            lds[C::C_OFF + slot * C::SLOT + i * C::XP + lane] = cv;
        }
    };
    const int plane = L.Ho * L.Wo;
    const int Hp = L.Ho >> 1, Wp = L.Wo >> 1, pplane = Hp * Wp;
    auto load_g = [&](int j, int oh, bool valid) {
        const int ow = ow0 - (K - 1) + lane, owh = ow0 - (K - 1) + hcol;
        const bool row_in = valid && (unsigned)oh < (unsigned)L.Ho;
        const bool in = row_in && (unsigned)ow < (unsigned)L.Wo;
        const bool inh = hl && row_in && (unsigned)owh < (unsigned)L.Wo;
        const size_t base = (size_t)b * COUT * plane;
        const int bytes = COUT * plane * 4;
        const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + base, bytes);
        const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + base, bytes);
        const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + base, bytes);
        const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + base : a.y, a.gco ? bytes : 0);
        const unsigned off = in ? (unsigned)(oh * L.Wo + ow) * 4u : OOB;
        const unsigned offh = inh ? (unsigned)((ho * L.Ho + oh) * L.Wo + owh) * 4u : OOB;
#pragma unroll
        for (int kk = 0; kk < C::OPW; ++kk) {
            const int so = (w + 4 * kk) * plane * 4;
            gq[j][kk][0] = ld_f32s(rgy, off, so);
            gq[j][kk][1] = ld_f32s(rco, off, so);
            gq[j][kk][2] = ld_f32s(ry, off, so);
            gq[j][kk][3] = ld_f32s(rgc, off, so);
        }
        gh[j][0] = ld_f32(rgy, offh);
        gh[j][1] = ld_f32(rco, offh);
        gh[j][2] = ld_f32(ry, offh);
        gh[j][3] = ld_f32(rgc, offh);
        if constexpr (GP) {
            const size_t pbase = (size_t)b * COUT * pplane;
            const int pbytes = COUT * pplane * 4;
            const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(a.gpy + pbase, pbytes);
            const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(a.gpc + pbase, pbytes);
            const __amdgpu_buffer_rsrc_t rpa = plane_rsrc((const float*)(a.parg + pbase), pbytes);
            const unsigned po = in ? pool_elem_off(oh, ow, Hp, Wp, OOB) : OOB;
            const unsigned pe = inh ? pool_elem_off(oh, owh, Hp, Wp, OOB) : OOB;
            const unsigned poh = pe != OOB ? pe + (unsigned)(ho * pplane) * 4u : OOB;
#pragma unroll
            for (int kk = 0; kk < C::OPW; ++kk) {
                const int so = (w + 4 * kk) * pplane * 4;
                gq[j][kk][4] = ld_f32s(rpy, po, so);
                gq[j][kk][5] = ld_f32s(rpc, po, so);
                gq[j][kk][6] = ld_f32s(rpa, po, so);
            }
            gh[j][4] = ld_f32(rpy, poh);
            gh[j][5] = ld_f32(rpc, poh);
            gh[j][6] = ld_f32(rpa, poh);
        }
    };
    float bias_o[C::OPW], wsum_o[C::OPW];
#pragma unroll
    for (int kk = 0; kk < C::OPW; ++kk) {
        bias_o[kk] = L.bias[w + 4 * kk];
        wsum_o[kk] = L.wsum[w + 4 * kk];
    }
    // g row j of the pair (output row oh_cur) into buffer buf; an invalid row (past the segment)
    // stores zeros and adds nothing to the bias / normaliser sums
    auto store_g = [&](int buf, int j, int dr, int oh_cur, bool valid) {
        const unsigned sub = (unsigned)((oh_cur & 1) << 1), ow_m = (unsigned)(ow0 - (K - 1) + lane);
        const unsigned ow_h = (unsigned)(ow0 - (K - 1) + hcol);
        float* gb_row = lds + C::G_OFF + buf * C::GBUF + dr * C::GROW;
#pragma unroll
        for (int kk = 0; kk < C::OPW; ++kk) {
            const int o = w + 4 * kk;
            float gy = gq[j][kk][0], gco = gq[j][kk][3];
            if constexpr (GP)
                pool_route(gy, gco, gq[j][kk][4], gq[j][kk][5], __builtin_bit_cast(unsigned, gq[j][kk][6]), sub | (ow_m & 1u));
            float gN, gD;
            nconv_grad_nd(gy, gco, gq[j][kk][2], gq[j][kk][1], L.eps, bias_o[kk], wsum_o[kk], gN, gD);
            float* g = gb_row + o * C::GP + lane;
            g[0] = valid ? gN : 0.f;
            g[C::GPART] = valid ? gD : 0.f;
            if (lane >= K - 1) {  // (invalid rows loaded zeros: gy = gco = 0)
                gb_acc[kk] += gy;
                gs_acc[kk] = fmaf(gco, gq[j][kk][1], gs_acc[kk]);
            }
        }
        {   // halo pass (columns 64 .. 64+K-2)
            float bo = bias_o[0], so = wsum_o[0];
#pragma unroll
            for (int kk = 1; kk < C::OPW; ++kk) {
                bo = hkk == kk ? bias_o[kk] : bo;
                so = hkk == kk ? wsum_o[kk] : so;
            }
            float gy = gh[j][0], gco = gh[j][3];
            if constexpr (GP) pool_route(gy, gco, gh[j][4], gh[j][5], __builtin_bit_cast(unsigned, gh[j][6]), sub | (ow_h & 1u));
            float gN, gD;
            nconv_grad_nd(gy, gco, gh[j][2], gh[j][1], L.eps, bo, so, gN, gD);
            if (hl) {
                float* g = gb_row + ho * C::GP + hcol;
                g[0] = valid ? gN : 0.f;
                g[C::GPART] = valid ? gD : 0.f;
            }
            gb_h += gy;
            gs_h = fmaf(gco, gh[j][1], gs_h);
        }
    };

    f4acc acc[C::MT][C::NT];
#pragma unroll
    for (int t = 0; t < C::MT; ++t)
#pragma unroll
        for (int u = 0; u < C::NT; ++u) acc[t][u] = (f4acc){0.f, 0.f, 0.f, 0.f};

    // The next pair's rows are staged DURING this pair's MFMAs, one row (input + g) per half of the
    // k-steps: its input row goes to a ring slot this pair does not read (slots ih + 6, ih + 7 of
    // the 8), its g row to the other buffer (whose last reader, the previous pair, is behind the
    // barrier), so only one row's loads are ever in flight and one barrier per pair suffices.
    if (r0 < r1) {
        for (int r = 0; r <= K; ++r) {  // prologue: the first pair's K + 1 input rows and its g rows
            load_in(0, r0 - L.PH + r, r < K || r0 + 1 < r1);
            store_in(0, r0 - L.PH + r);
        }
        for (int j = 0; j < 2; ++j) {
            load_g(0, r0 + j, j == 0 || r0 + 1 < r1);
            store_g(0, 0, j, r0 + j, j == 0 || r0 + 1 < r1);
        }
    }
    __syncthreads();
#pragma unroll 1
    for (int oh = r0; oh < r1; oh += 2) {
        const int buf = ((oh - r0) >> 1) & 1;
        const int nx = oh + 2;  // the next pair (none past r1: its staging is skipped)
        const bool more = nx < r1;
        int ax[C::MT], bn[C::NT];
#pragma unroll
        for (int t = 0; t < C::MT; ++t) ax[t] = ((oh - L.PH + a_r[t]) & (C::SLOTS - 1)) * C::SLOT + a_ik[t];
#pragma unroll
        for (int u = 0; u < C::NT; ++u) bn[u] = C::G_OFF + buf * C::GBUF + b_off[u];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (more) {  // next pair's row j: input row r = K - 1 + j, g row d = j
                load_in(0, nx - L.PH + K - 1 + j, j == 0 || nx + 1 < r1);
                load_g(0, nx + j, j == 0 || nx + 1 < r1);
            }
#pragma unroll
            for (int s = 2 * j; s < 2 * j + 2; ++s) {
                const int q0 = 16 * w + 4 * s;
#pragma unroll
                for (int pt = 0; pt < 2; ++pt) {  // {x*c, gN} then {c, gD}
                    float va[C::MT], vb[C::NT];
#pragma unroll
                    for (int t = 0; t < C::MT; ++t) va[t] = lds[ax[t] + pt * C::C_OFF + q0];
#pragma unroll
                    for (int u = 0; u < C::NT; ++u) vb[u] = lds[bn[u] + pt * C::GPART + q0];
#pragma unroll
                    for (int t = 0; t < C::MT; ++t)
#pragma unroll
                        for (int u = 0; u < C::NT; ++u)
                            acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[t], vb[u], acc[t][u], 0, 0, 0);
#if NCONV_WM2_SCHED
                    __builtin_amdgcn_sched_barrier(0);  // (operand reads of the next step not hoisted above)
#endif
                }
            }
            if (more) {
                store_in(0, nx - L.PH + K - 1 + j);
                store_g(buf ^ 1, 0, j, nx + j, j == 0 || nx + 1 < r1);
            }
        }
        __syncthreads();
    }

    // ---- the four waves' tiles summed in a fixed order ((w0 + w2) + (w1 + w3)), then each weight
    //      as its two row-pair terms: gW[o][i][kh][kw] = C[(kh, i)][(0, kw, o)] + C[(kh+1, i)][(1, kw, o)]
    constexpr int NW = COUT * CIN * K * K;
    float* out = part + (size_t)blockIdx.x * (NW + 2 * COUT);
    __syncthreads();
    float* red = lds + (w & 1) * C::TILE;
    if (w < 2) {
#pragma unroll
        for (int t = 0; t < C::MT; ++t)
#pragma unroll
            for (int u = 0; u < C::NT; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[(t * C::NT + u) * 256 + r * 64 + lane] = acc[t][u][r];
    }
    __syncthreads();
    if (w >= 2) {
#pragma unroll
        for (int t = 0; t < C::MT; ++t)
#pragma unroll
            for (int u = 0; u < C::NT; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[(t * C::NT + u) * 256 + r * 64 + lane] += acc[t][u][r];
    }
    __syncthreads();
    auto at = [&](int m, int n) {  // the summed C[m][n] (MFMA 16x16 output layout)
        const int t = m >> 4, mm = m & 15, u = n >> 4;
        const int idx = (t * C::NT + u) * 256 + (mm & 3) * 64 + (mm >> 2) * 16 + (n & 15);
        return lds[idx] + lds[C::TILE + idx];
    };
    for (int f = tid; f < NW; f += kT) {  // o fastest: a wave's reads spread over the LDS banks
        const int o = f % COUT, kw = (f / COUT) % K, kh = (f / (COUT * K)) % K, i = f / (COUT * K * K);
        out[((o * CIN + i) * K + kh) * K + kw] =
            at(kh * CIN + i, kw * COUT + o) + at((kh + 1) * CIN + i, K * COUT + kw * COUT + o);
    }
#pragma unroll
    for (int kk = 0; kk < C::OPW; ++kk) {
        const bool mine = hl && hkk == kk;
        float sb = gb_acc[kk] + (mine ? gb_h : 0.f), ss = gs_acc[kk] + (mine ? gs_h : 0.f);
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            sb += __shfl_xor(sb, sh);
            ss += __shfl_xor(ss, sh);
        }
        if (lane == 0) {
            out[NW + w + 4 * kk] = sb;
            out[NW + COUT + w + 4 * kk] = ss;
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

#ifndef NCONV_WG_MAX_BLOCKS
#define NCONV_WG_MAX_BLOCKS 4096  // workspace bound; the launch uses at most one resident round
#endif
constexpr int kMaxWgBlocks = NCONV_WG_MAX_BLOCKS;

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

// wgrad_mfma grid: 64-wide q strips (q = ow + kw spans Wo + K - 1 columns) x row segments x images,
// at most `target` workgroups: NCONV_WM_ROUNDS resident rounds of the instantiation (CUs x blocks
// per CU x rounds; a third, nearly empty round once cost nconv2's weight gradient a third of its
// time). One round (longer row segments: less per-block prologue, fewer partial rows) for the
// weight gradients that share the CUs with the input-gradient chain, two for the tail's (T7), which
// starts the side stream: graphed training step 2.104 -> 2.064 ms same box (one round everywhere
// 2.093, the tail alone at one round 2.137; profiles/r6_ab_wgrad_rounds.log). The workspace is
// sized for the larger round count at the largest possible occupancy (kMfmaRoundsMax).
#ifndef NCONV_WM_ROUNDS
#define NCONV_WM_ROUNDS 1
#endif
#ifndef NCONV_WM_T7_ROUNDS
#define NCONV_WM_T7_ROUNDS 2
#endif
constexpr int kMfmaRounds = NCONV_WM_ROUNDS, kMfmaMaxPerCu = 4;
constexpr int kMfmaRoundsMax = NCONV_WM_T7_ROUNDS > NCONV_WM_ROUNDS ? NCONV_WM_T7_ROUNDS : NCONV_WM_ROUNDS;
struct WmGrid {
    int nstrip, nseg, seg_rows;
    size_t nblk;
};
static int device_cus() { return dev_cus(); }
static WmGrid wm_grid(const nconv_layer& L, int target = 0) {
    if (target <= 0) target = kMfmaRoundsMax * kMfmaMaxPerCu * device_cus();  // workspace bound (every variant)
    WmGrid g;
    g.nstrip = (L.Wo + L.KW - 1 + 63) / 64;
    const int per_img = g.nstrip * L.B;
    int nseg = target / per_img;  // floor: never more blocks than the target (nseg >= 1 below)
    nseg = nseg < 1 ? 1 : (nseg > L.Ho ? L.Ho : nseg);
    g.seg_rows = (L.Ho + nseg - 1) / nseg;
    if (g.seg_rows < 1) g.seg_rows = 1;
    g.nseg = (L.Ho + g.seg_rows - 1) / g.seg_rows;
    if (g.nseg < 1) g.nseg = 1;
    g.nblk = (size_t)g.nstrip * g.nseg * L.B;
    return g;
}
// The 8 -> 8 5x5 weight gradients over output-row pairs (wgrad_mfma2); NCONV_WM_ROW_PAIRS=0: one row
// at a time (wgrad_mfma), for A/B timing
static bool wm_row_pairs() {
    static const bool on = [] {
        const char* e = getenv("NCONV_WM_ROW_PAIRS");
        return !(e && e[0] == '0');
    }();
    return on;
}
// tiled 3x3 / 5x5 layers with several input channels (Cin = 1 has a single-row A tile and stays
// on wgrad_tiled, which reads each g plane once per 4 x 64 tile instead of once per row segment)
static bool wgrad_on_mfma(const nconv_layer& L) { return L.KH > 1 && L.Cin > 1; }

size_t bwd_workspace_bytes(const LayerDev& d) {
    const nconv_layer& L = d.L;
    const int fan = (L.Cin / L.groups) * L.KH * L.KW;
    const size_t stride = (size_t)L.Cout * fan + 2 * L.Cout;
    const Path path = pick_path(L);
    const size_t nblk = path == kTiled ? (wgrad_on_mfma(L) ? wm_grid(L).nblk : wg_blocks(L))
                                       : (size_t)generic_chunks(L);
    size_t bytes = (nblk + kReduceSplit) * stride * sizeof(float);  // partial rows + slice sums
    bytes = (bytes + 255) & ~(size_t)255;
    if (L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST) {
        // staged upsampled-channel planes for upsample_bwd_gather, or dgrad_phase's box weights
        const size_t planes = 2 * (size_t)L.B * L.b.C * L.H * L.W;
        bytes += (planes > 1024 ? planes : 1024) * sizeof(float);
    }
    return bytes;
}

size_t bwd_tail_workspace_bytes(const nconv_layer& L) {
    return (wm_grid(L).nblk + kReduceSplit) * 10 * sizeof(float);
}

size_t bwd_head_workspace_bytes(const nconv_layer& L) {
    using D = DgCfg<8, 5>;
    const size_t nblk = (size_t)((L.W + D::TW - 1) / D::TW) * ((L.H + D::TH - 1) / D::TH) * L.B;
    return (nblk + kReduceSplit) * kHeadStride * sizeof(float);
}

void plan_bwd(const nconv_layer& L, int* dgrad, int* wgrad) {
    if (pick_path(L) == kGeneric) {
        *dgrad = *wgrad = NCONV_KERNEL_GENERIC;
        return;
    }
    const int bf = L.bwd_math == NCONV_MATH_BF16X9 ? NCONV_KERNEL_MFMA_BF16X9 : NCONV_KERNEL_MFMA_BF16X3;
    const bool multi = L.KH > 1 && L.Cin > 1;  // 3x3 / 5x5 layers with several input channels
    const bool fp32 = L.bwd_math == NCONV_MATH_FP32;
    *dgrad = multi && !fp32 ? bf : (dgrad_phase_ok(L) ? NCONV_KERNEL_TILED_FP32_PHASE : NCONV_KERNEL_TILED_FP32);
    *wgrad = multi ? (fp32 ? NCONV_KERNEL_MFMA_FP32 : bf) : NCONV_KERNEL_TILED_FP32;
}

// Returns 0, or -EIO when the bf16 weight-gradient grid would not fit the workspace (it cannot:
// its strips are wider than wgrad_mfma's, for which the workspace is sized; checked anyway, so
// a bf16 request never silently runs another kernel).
template <int CIN, int COUT, int K, int MODE, bool GP = false, bool HW = false, bool T7 = false>
static int go_bwd_tiled(const LayerDev& d, const BwdArgs& a, float* part, float* tx, float* tc,
                        hipStream_t st, const char** why) {
    const nconv_layer& L = d.L;
    using D = DgCfg<CIN, K>;
    if (HW || a.gxa || a.gca || a.gxb || a.gcb) {
        if (K > 1 && CIN > 1 && L.bwd_math != NCONV_MATH_FP32) {  // split-bf16 matrix cores
            if constexpr (K > 1 && CIN > 1)
                go_dgrad_bf<CIN, COUT, K, MODE>(d, a, tx, tc, L.bwd_math == NCONV_MATH_BF16X9 ? 3 : 2, st);
        } else {
            dim3 g(((L.W + D::TW - 1) / D::TW) * ((L.H + D::TH - 1) / D::TH) * L.B);  // see xcd_tile
            constexpr bool up = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST;
            if constexpr (up && CIN == 16 && COUT == 8 && K == 3) {
                if (dgrad_phase_ok(L)) {  // box weights: the caller's, or into the (then unused) staging planes
                    const float* wb = a.box;
                    if (!wb) {
                        hipLaunchKernelGGL(box_weights, dim3(1024 / kT), dim3(kT), 0, st, L.weight,
                                           MODE == NCONV_LOAD_UPCAT_SKIP_FIRST ? 8 : 0, tx);
                        wb = tx;
                    }
                    hipLaunchKernelGGL((dgrad_phase<MODE, T7>), g, dim3(kT), 0, st, d, a, wb);
                } else {
                    hipLaunchKernelGGL((dgrad_tiled<CIN, COUT, K, MODE>), g, dim3(kT), 0, st, d, a, tx, tc);
                }
            } else {
                hipLaunchKernelGGL((dgrad_tiled<CIN, COUT, K, MODE, GP, HW>), g, dim3(kT), 0, st, d, a, tx, tc);
                if constexpr (HW) {  // nconv1's weight-gradient partial rows: one per dgrad workgroup
                    if (a.defer) {
                        *a.hnparts = (int)g.x;
                    } else {
                        const RedJob J{a.hpart, a.hs, a.hgw, a.hgb, (int)g.x, kHeadNw, 8, 25};
                        if (int rc = launch_wgrad_reduce_multi(1, &J, st, why)) return rc;
                    }
                }
            }
        }
    }
    if constexpr (K > 1 && CIN > 1) {
        if ((a.gw || a.gb) && L.bwd_math != NCONV_MATH_FP32) {  // split-bf16 matrix cores
            const int nblk = go_wgrad_bf<CIN, COUT, K, MODE>(d, a, part, (int)wm_grid(L).nblk,
                                                             L.bwd_math == NCONV_MATH_BF16X9 ? 3 : 2, st);
            if (nblk < 0) {
                *why = "bf16 weight-gradient grid exceeds the workspace";
                return -5;
            }
            const int nw = COUT * CIN * K * K;
            return launch_wgrad_reduce(a, part, nblk, nw, COUT, CIN * K * K, L.wsum, st, why);
        } else if (a.gw || a.gb) {
            if constexpr (CIN == 8 && COUT == 8 && K == 5 && !T7) {
                if (wm_row_pairs()) {  // the row-pair form fills its MFMA tiles (wgrad_mfma2)
                    const int per_cu = dev_occupancy((const void*)wgrad_mfma2<CIN, COUT, K, MODE, GP>, kT, 0);
                    const int resident = device_cus() * (per_cu < kMfmaMaxPerCu ? per_cu : kMfmaMaxPerCu);
                    const WmGrid g = wm_grid(L, kMfmaRounds * resident);
                    hipLaunchKernelGGL((wgrad_mfma2<CIN, COUT, K, MODE, GP>), dim3(g.nblk), dim3(kT), 0, st, d, a,
                                       part, g.nstrip, g.nseg, g.seg_rows);
                    const int nw = COUT * CIN * K * K;
                    return launch_wgrad_reduce(a, part, (int)g.nblk, nw, COUT, CIN * K * K, L.wsum, st, why);
                }
            }
            const int per_cu = dev_occupancy((const void*)wgrad_mfma<CIN, COUT, K, MODE, GP, T7>, kT, 0);
            const int resident = device_cus() * (per_cu < kMfmaMaxPerCu ? per_cu : kMfmaMaxPerCu);
            const WmGrid g = wm_grid(L, (T7 ? NCONV_WM_T7_ROUNDS : kMfmaRounds) * resident);
            hipLaunchKernelGGL((wgrad_mfma<CIN, COUT, K, MODE, GP, T7>), dim3(g.nblk), dim3(kT), 0, st, d, a, part,
                               g.nstrip, g.nseg, g.seg_rows);
            if constexpr (T7) {  // nconv7's weight-gradient partial rows: one per wgrad workgroup
                if (a.defer) {
                    *a.t7nparts = (int)g.nblk;
                } else {
                    const RedJob J{a.t7part, a.t7s, a.t7gw, nullptr, (int)g.nblk, 8, 1, 8};
                    if (int rc = launch_wgrad_reduce_multi(1, &J, st, why)) return rc;
                }
            }
            const int nw = COUT * CIN * K * K;
            return launch_wgrad_reduce(a, part, (int)g.nblk, nw, COUT, CIN * K * K, L.wsum, st, why);
        }
    } else if (a.gw || a.gb) {
        using W = WgCfg<CIN, COUT, K>;
        const int ntw = (L.Wo + W::TW - 1) / W::TW, nth = (L.Ho + W::TH - 1) / W::TH;
        const int nblk_ws = (int)wg_blocks(L);
        size_t lds = (size_t)W::LDS_F2 * sizeof(f2);
        size_t red = (size_t)2 * COUT * kT * sizeof(float);
        const size_t red2 = (size_t)W::NSUB * COUT * CIN * K * K * sizeof(float);
        if (red2 > red) red = red2;
        if (red > lds) lds = red;
        // blocks walk runs of tiles: launch at most the resident count (CUs x blocks per CU), so
        // there is no second, partial round (nconv1's 13.4 k tiles: 768 resident at 3 waves/SIMD)
        const int resident = device_cus() * dev_occupancy((const void*)wgrad_tiled<CIN, COUT, K, MODE>, kT, lds);
        const int nblk = nblk_ws < resident ? nblk_ws : resident;
        hipLaunchKernelGGL((wgrad_tiled<CIN, COUT, K, MODE>), dim3(nblk), dim3(kT), lds, st, d, a, part, ntw, nth);
        const int nw = COUT * CIN * K * K;
        return launch_wgrad_reduce(a, part, nblk, nw, COUT, CIN * K * K, L.wsum, st, why);
    }
    return 0;
}

template <int MODE>
static int go_bwd_generic(const LayerDev& d, const BwdArgs& a, float* part, float* tx, float* tc,
                          hipStream_t st, const char** why) {
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
        return launch_wgrad_reduce(a, part, nchunk, nw, L.Cout, fan, L.wsum, st, why);
    }
    return 0;
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
    const size_t nblk = path == kTiled ? (wgrad_on_mfma(L) ? wm_grid(L).nblk : wg_blocks(L))
                                       : (size_t)generic_chunks(L);
    float* part = a.ws;
    float* tx = a.ws + ((((nblk + kReduceSplit) * stride * sizeof(float)) + 255) & ~(size_t)255) / sizeof(float);
    float* tc = tx + (size_t)L.B * L.b.C * L.H * L.W;
    const bool up = L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;

    if (a.gpy || a.gpc || a.parg) {  // pooled-gradient routing: built for the 8->8 5x5 exact-fp32 layers
        if (!(a.gpy && a.gpc && a.parg) || path != kTiled || L.Cin != 8 || L.Cout != 8 || L.KH != 5 ||
            L.load_mode != NCONV_LOAD_PLAIN || L.bwd_math != NCONV_MATH_FP32 || L.Ho < 2 || L.Wo < 2) {
            *why = "pooled-output gradient needs gy_pool, gcout_pool and the argmax codes, on an exact-fp32 "
                   "8->8 5x5 stride-1 layer with plain loads";
            return -95;
        }
        const int rc = a.hpart ? go_bwd_tiled<8, 8, 5, NCONV_LOAD_PLAIN, true, true>(d, a, part, tx, tc, st, why)
                               : go_bwd_tiled<8, 8, 5, NCONV_LOAD_PLAIN, true>(d, a, part, tx, tc, st, why);
        return rc ? rc : last_err(why);
    }
    if (a.t7part) {
        if (!(path == kTiled && dgrad_phase_ok(L) && L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST && L.PH == 0 &&
              L.PW == 0)) {
            *why = "fused tail backward needs nconv6's exact-fp32 geometry (16->8 3x3, padding 0, upsample-first "
                   "exactly-2x concat)";
            return -95;
        }
        const int rc = go_bwd_tiled<16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST, false, false, true>(d, a, part, tx, tc, st, why);
        return rc ? rc : last_err(why);
    }
    if (a.hpart) {
        if (!(path == kTiled && L.Cin == 8 && L.Cout == 8 && L.KH == 5 && L.load_mode == NCONV_LOAD_PLAIN &&
              L.bwd_math == NCONV_MATH_FP32)) {
            *why = "fused head weight gradient needs an exact-fp32 8->8 5x5 stride-1 layer with plain loads";
            return -95;
        }
        const int rc = go_bwd_tiled<8, 8, 5, NCONV_LOAD_PLAIN, false, true>(d, a, part, tx, tc, st, why);
        return rc ? rc : last_err(why);
    }
    if (path == kTiled) {
        const int m = L.load_mode;
        int rc;
        if (L.Cin == 1 && m == NCONV_LOAD_THRESH) rc = go_bwd_tiled<1, 8, 5, NCONV_LOAD_THRESH>(d, a, part, tx, tc, st, why);
        else if (L.Cin == 8 && L.Cout == 8 && m == NCONV_LOAD_PLAIN) rc = go_bwd_tiled<8, 8, 5, NCONV_LOAD_PLAIN>(d, a, part, tx, tc, st, why);
        else if (L.Cin == 8 && L.Cout == 8 && m == NCONV_LOAD_POOL2) rc = go_bwd_tiled<8, 8, 5, NCONV_LOAD_POOL2>(d, a, part, tx, tc, st, why);
        else if (m == NCONV_LOAD_UPCAT_SKIP_FIRST) rc = go_bwd_tiled<16, 8, 3, NCONV_LOAD_UPCAT_SKIP_FIRST>(d, a, part, tx, tc, st, why);
        else if (m == NCONV_LOAD_UPCAT_UP_FIRST) rc = go_bwd_tiled<16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST>(d, a, part, tx, tc, st, why);
        else rc = go_bwd_tiled<8, 1, 1, NCONV_LOAD_PLAIN>(d, a, part, tx, tc, st, why);
        if (rc) return rc;
    } else {
        int rc = 0;
        switch (L.load_mode) {
            case NCONV_LOAD_PLAIN: rc = go_bwd_generic<NCONV_LOAD_PLAIN>(d, a, part, tx, tc, st, why); break;
            case NCONV_LOAD_THRESH: rc = go_bwd_generic<NCONV_LOAD_THRESH>(d, a, part, tx, tc, st, why); break;
            case NCONV_LOAD_POOL2: rc = go_bwd_generic<NCONV_LOAD_POOL2>(d, a, part, tx, tc, st, why); break;
            case NCONV_LOAD_UPCAT_SKIP_FIRST: rc = go_bwd_generic<NCONV_LOAD_UPCAT_SKIP_FIRST>(d, a, part, tx, tc, st, why); break;
            case NCONV_LOAD_UPCAT_UP_FIRST: rc = go_bwd_generic<NCONV_LOAD_UPCAT_UP_FIRST>(d, a, part, tx, tc, st, why); break;
            default: *why = "unknown load mode"; return -22;
        }
        if (rc) return rc;
    }
    if (up && (a.gxb || a.gcb) && !(path == kTiled && dgrad_phase_ok(L))) {  // (dgrad_phase writes them itself)
        const size_t n = (size_t)L.B * L.b.C * L.b.H * L.b.W;
        size_t blocks = (n + kT - 1) / kT;
        if (blocks > (1u << 20)) blocks = 1u << 20;
        if (blocks) hipLaunchKernelGGL(upsample_bwd_gather, dim3(blocks), dim3(kT), 0, st, d, tx, tc, a.gxb, a.gcb,
                                      a.accumulate);
    }
    return last_err(why);
}

}  // namespace nconv
