// nconv_bwd_fused.hip — one-kernel backward of the full-resolution 8 -> 8, 5x5 NConv layers (gfx950).
//
// Autograd of NConv2d.forward (reference models/step1.py:116-149) for DNET's nconv2 (and the
// 8 -> 8 5x5 down layers) in exact fp32, input gradient AND weight gradient in one pass over the
// saved planes. The separate kernels (dgrad_tiled + wgrad_mfma, nconv_bwd.hip) each read gy, gcout,
// y, cout (+ the pooled gradient and its argmax codes) and each form {gN, gD} from them; here a
// workgroup forms {gN, gD} once per element and feeds both:
//   gN = gy/(D+eps), gD = -gy*N/(D+eps)^2 + gcout/s          (nconv_grad_nd, D = cout*s, N/(D+eps) = y-b)
//   G_xc(ih, iw) = sum_{o,kh,kw} W[o][i][kh][kw] gN[o](ih+2-kh, iw+2-kw)    (input gradient, "dgrad")
//   G_c likewise with gD;  gx = G_xc*c,  gc = G_c + G_xc*x
//   gW[o][i][kh][kw] = sum_{oh,ow} gN[o](oh,ow) xc[i](oh+kh-2, ow+kw-2) + gD[o](oh,ow) c[i](..)  ("wgrad")
//
// Layout of the work: a workgroup (4 waves) owns a 64-column strip [c0, c0+64) of one image and
// walks a segment of rows [r0, r1) one row per step, with rings in LDS of the last five staged input
// rows ({x*c, c}, 8 channels x 64 columns) and of the last five {gN, gD} rows (8 channels x 68
// columns: c0-2 .. c0+65). Step s stages input row s+2 and g row s, then
//   * weight gradient of output row s (VALU, packed FP32: lane = (o, i), all 25 taps of that weight
//     in 25 {xc*gN, c*gD} accumulator pairs; wave w takes the 16 columns 16w .. 16w+15 of the strip,
//     q = input column iw pairs with output column ow = iw + 2 - kw, so each (oh, iw, ow) triple is
//     counted by exactly one strip: a g window slides along the row, one new g read per column);
//   * input gradient of input row s-2 (its five g rows s-4 .. s are in the ring): lane = column,
//     wave w the output channels 2w, 2w+1 (weights wave-uniform in SGPRs, as dgrad_tiled), the four
//     waves' partial sums added in a fixed order through LDS in the epilogue, which applies
//     gx = G_xc*c, gc = G_c + G_xc*x and stores the row (or, fused head, forms nconv1's {gN1, gD1}
//     and accumulates nconv1's weight gradient over the depth samples of the five S rows around it:
//     the weight-gradient epilogue of dgrad_tiled<..., HW>, per row).
// No MFMA: the fp32 matrix cores and the packed-FMA VALU do not run side by side on a CU
// (tools/microbench/fp32_rates.hip), and on the VALU the 40 x 40 weight-gradient GEMM carries no
// padding (wgrad_mfma pads it to 48 x 48: 69 % useful). Both gradients' FMAs: 50 packed FMAs per
// pixel, once per element staging, one read of every saved plane.
//
// Partial rows (one per workgroup) as wgrad_mfma's (1600 weights, 8 sum gy, 8 sum gcout*cout), and,
// with the head, as dgrad_tiled<HW>'s (200 weights, 8 + 8 sums), reduced by wgrad_reduce_sum /
// wgrad_finish (deterministic, fixed order).
#include "nconv_internal.h"

namespace nconv {

namespace fb {
constexpr int kT = 256;
constexpr int C = 8;                // Cin = Cout
constexpr int TW = 64;              // strip width
constexpr int GW = TW + 4;          // g columns c0-2 .. c0+65
// LDS pitches (floats) of one channel row: 8 * pitch (mod 64) distinct for the 8 channels, so the
// weight-gradient reads (lanes = (o, i): 8 distinct {x*c, c} or {gN, gD} pairs per instruction)
// fall on distinct banks of ds_read_b64 (bank = dword mod 64); lane = column reads are contiguous
constexpr int XP = 136, GPT = 136;
constexpr int NSX = 5, NSG = 5, NSS = 6;  // ring slots: input rows, g rows, S sample lists
constexpr int XSLOT = C * XP, GSLOT = C * GPT;
constexpr int X_OFF = 0;
constexpr int G_OFF = X_OFF + NSX * XSLOT;
constexpr int R_OFF = G_OFF + NSG * GSLOT;   // the input gradient's per-wave partials [4][8][64] f2
constexpr int H_OFF = R_OFF + 4 * C * 2 * TW;  // nconv1's {gN1, gD1} of the row, [8][64] f2
constexpr int SL = 2 + 2 * GW;               // per S row: count (+ pad), then (column, S) of the samples
constexpr int S_OFF = H_OFF + 2 * C * TW;
constexpr int LDS_MAIN = S_OFF + NSS * SL;
constexpr int FIN = 4 * 50 * 64;             // the waves' weight-gradient accumulators, summed at the end
constexpr int LDS = LDS_MAIN > FIN ? LDS_MAIN : FIN;
constexpr int NW = C * C * 25;               // 1600 weights
constexpr unsigned OOB = 0x80000000u;
static_assert(XP >= 2 * TW && GPT >= 2 * GW, "pitches");
}  // namespace fb

__device__ __forceinline__ int ring(int r, int n) { return ((r % n) + n) % n; }
typedef const float __attribute__((address_space(4))) cfloat;

template <bool GP, bool HW>
__global__ __launch_bounds__(fb::kT) __attribute__((amdgpu_waves_per_eu(2, 2))) void bwd_fused(
    LayerDev d, BwdArgs a, float* part, int nstrip, int nseg, int seg_rows) {
    using namespace fb;
    __shared__ __attribute__((aligned(16))) float lds[LDS];
    const nconv_layer& L = d.L;
    // the weights through the constant address space: scalar loads (the loop's global stores would
    // otherwise keep the compiler from proving them unclobbered, and it issues per-lane vector loads)
    const cfloat* wgt = (const cfloat*)L.weight;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const TileCoord tc = xcd_tile(nstrip, nseg, L.B);
    const int b = tc.b, c0 = tc.tx * TW;
    const int H = L.H, W = L.W;
    const int r0 = tc.ty * seg_rows, r1 = min(H, r0 + seg_rows);
    const int plane = H * W;

    // ---- per-image resources (one per saved tensor: the channel plane rides soffset) ----
    const size_t img = (size_t)b * C * plane;
    const int ibytes = C * plane * 4;
    const __amdgpu_buffer_rsrc_t rax = plane_rsrc(L.a.x + img, ibytes), rac = plane_rsrc(L.a.c + img, ibytes);
    const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + img, ibytes), rco = plane_rsrc(a.co + img, ibytes);
    const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + img, ibytes);
    const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + img : a.y, a.gco ? ibytes : 0);
    const int Hp = H >> 1, Wp = W >> 1, pplane = Hp * Wp;
    const size_t pimg = (size_t)b * C * pplane;
    const int pbytes = C * pplane * 4;
    const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(GP ? a.gpy + pimg : a.y, GP ? pbytes : 0);
    const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(GP ? a.gpc + pimg : a.y, GP ? pbytes : 0);
    const __amdgpu_buffer_rsrc_t rpa = plane_rsrc(GP ? (const float*)(a.parg + pimg) : a.y, GP ? pbytes : 0);

    // ---- input rows: wave w stages channels w, w + 4 (lane = column c0 + lane) ----
    float px[2], pc[2];
    auto load_x = [&](int ih) {
        const bool in = (unsigned)ih < (unsigned)H && c0 + lane < W;
        const unsigned off = in ? (unsigned)(ih * W + c0 + lane) * 4u : OOB;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            px[k] = ld_f32s(rax, off, (w + 4 * k) * plane * 4);
            pc[k] = ld_f32s(rac, off, (w + 4 * k) * plane * 4);
        }
    };
    auto store_x = [&](int ih) {
        float* xs = lds + X_OFF + ring(ih, NSX) * XSLOT + 2 * lane;
#pragma unroll
        for (int k = 0; k < 2; ++k) *reinterpret_cast<f2*>(xs + (w + 4 * k) * XP) = (f2){px[k] * pc[k], pc[k]};
    };

    // ---- g rows: wave w forms {gN, gD} of channels w, w + 4 at the 64 columns c0-2+lane, and one
    //      halo pass (lanes 0..7: channel w + 4 (lane >> 2), column c0 + 62 + (lane & 3)) ----
    constexpr int NG = GP ? 7 : 4;  // gy, cout, y, gcout (+ pooled gy, pooled gcout, argmax code)
    float gq[2][NG], gh[NG];
    const bool hl = lane < 8;
    const int hk = (lane >> 2) & 1, ho = w + 4 * hk;
    const int owm = c0 - 2 + lane, owh = c0 + 62 + (lane & 3);
    auto load_g = [&](int oh) {
        const bool row_in = (unsigned)oh < (unsigned)H;
        const bool in = row_in && (unsigned)owm < (unsigned)W;
        const bool inh = hl && row_in && (unsigned)owh < (unsigned)W;
        const unsigned off = in ? (unsigned)(oh * W + owm) * 4u : OOB;
        const unsigned offh = inh ? (unsigned)((ho * H + oh) * W + owh) * 4u : OOB;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int so = (w + 4 * k) * plane * 4;
            gq[k][0] = ld_f32s(rgy, off, so);
            gq[k][1] = ld_f32s(rco, off, so);
            gq[k][2] = ld_f32s(ry, off, so);
            gq[k][3] = ld_f32s(rgc, off, so);
        }
        gh[0] = ld_f32(rgy, offh);
        gh[1] = ld_f32(rco, offh);
        gh[2] = ld_f32(ry, offh);
        gh[3] = ld_f32(rgc, offh);
        if constexpr (GP) {
            const unsigned po = in ? pool_elem_off(oh, owm, Hp, Wp, OOB) : OOB;
            const unsigned pe = inh ? pool_elem_off(oh, owh, Hp, Wp, OOB) : OOB;
            const unsigned poh = pe != OOB ? pe + (unsigned)(ho * pplane) * 4u : OOB;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int so = (w + 4 * k) * pplane * 4;
                gq[k][4] = ld_f32s(rpy, po, so);
                gq[k][5] = ld_f32s(rpc, po, so);
                gq[k][6] = ld_f32s(rpa, po, so);
            }
            gh[4] = ld_f32(rpy, poh);
            gh[5] = ld_f32(rpc, poh);
            gh[6] = ld_f32(rpa, poh);
        }
    };
    float bias_o[2], wsum_o[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        bias_o[k] = L.bias[w + 4 * k];
        wsum_o[k] = L.wsum[w + 4 * k];
    }
    const float bias_h = hk ? bias_o[1] : bias_o[0], wsum_h = hk ? wsum_o[1] : wsum_o[0];
    float gb_acc[2] = {0.f, 0.f}, gs_acc[2] = {0.f, 0.f}, gb_h = 0.f, gs_h = 0.f;
    // own output columns for the bias / normaliser sums: c0 .. c0+63 (main lanes >= 2, halo columns
    // c0+62, c0+63); rows r0 .. r1-1 (count)
    auto store_g = [&](int oh, bool count) {
        float* gs = lds + G_OFF + ring(oh, NSG) * GSLOT;
        const unsigned sub = (unsigned)((oh & 1) << 1);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float gy = gq[k][0], gco = gq[k][3];
            if constexpr (GP) pool_route(gy, gco, gq[k][4], gq[k][5], __builtin_bit_cast(unsigned, gq[k][6]),
                                         sub | ((unsigned)owm & 1u));
            float gN, gD;
            nconv_grad_nd(gy, gco, gq[k][2], gq[k][1], L.eps, bias_o[k], wsum_o[k], gN, gD);
            *reinterpret_cast<f2*>(gs + (w + 4 * k) * GPT + 2 * lane) = (f2){gN, gD};
            if (count && lane >= 2) {
                gb_acc[k] += gy;
                gs_acc[k] = fmaf(gco, gq[k][1], gs_acc[k]);
            }
        }
        float gy = gh[0], gco = gh[3];
        if constexpr (GP) pool_route(gy, gco, gh[4], gh[5], __builtin_bit_cast(unsigned, gh[6]), sub | ((unsigned)owh & 1u));
        float gN, gD;
        nconv_grad_nd(gy, gco, gh[2], gh[1], L.eps, bias_h, wsum_h, gN, gD);
        if (hl) {
            *reinterpret_cast<f2*>(gs + ho * GPT + 2 * (64 + (lane & 3))) = (f2){gN, gD};
            if (count && (lane & 3) < 2) {
                gb_h += gy;
                gs_h = fmaf(gco, gh[1], gs_h);
            }
        }
    };

    // ---- fused head (nconv1's weight gradient): S rows as sample lists, built by wave 3 ----
    float sv0 = 0.f, sv1 = 0.f;
    const __amdgpu_buffer_rsrc_t rS = plane_rsrc(HW ? a.hS + (size_t)b * plane : a.y, HW ? plane * 4 : 0);
    auto load_s = [&](int r) {
        if constexpr (HW) {
            const bool row_in = (unsigned)r < (unsigned)H;
            const int cm = c0 - 2 + lane, ch = c0 + 62 + lane;
            sv0 = ld_f32(rS, row_in && (unsigned)cm < (unsigned)W ? (unsigned)(r * W + cm) * 4u : OOB);
            sv1 = ld_f32(rS, row_in && lane < 4 && (unsigned)ch < (unsigned)W ? (unsigned)(r * W + ch) * 4u : OOB);
        }
    };
    auto store_s = [&](int r) {
        if constexpr (HW) {
            if (w == 3) {
                float* lst = lds + S_OFF + ring(r, NSS) * SL;
                f2* ent = reinterpret_cast<f2*>(lst + 2);
                const bool p0 = sv0 > a.hthresh;
                const unsigned long long m0 = __ballot(p0);
                const int n0 = __popcll(m0);
                if (p0) ent[__popcll(m0 & ((1ull << lane) - 1ull))] = (f2){__builtin_bit_cast(float, lane), sv0};
                const bool p1 = lane < 4 && sv1 > a.hthresh;
                const unsigned long long m1 = __ballot(p1);
                if (p1) ent[n0 + __popcll(m1 & ((1ull << lane) - 1ull))] = (f2){__builtin_bit_cast(float, 64 + lane), sv1};
                if (lane == 0) lst[0] = __builtin_bit_cast(float, n0 + __popcll(m1));
            }
        }
    };
    // the input gradient's epilogue needs (x, c) of its row: channels 2w, 2w + 1 at column c0 + lane
    float ex[2], ec[2];
    auto load_e = [&](int ih) {
        const bool in = (unsigned)ih < (unsigned)H && c0 + lane < W;
        const unsigned off = in ? (unsigned)(ih * W + c0 + lane) * 4u : OOB;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            ex[k] = ld_f32s(rax, off, (2 * w + k) * plane * 4);
            ec[k] = ld_f32s(rac, off, (2 * w + k) * plane * 4);
        }
    };

    // weight-gradient accumulators: lane = (o = lane >> 3, i = lane & 7), [kh][kw] {xc*gN, c*gD}
    f2 wacc[5][5];
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) wacc[kh][kw] = (f2){0.f, 0.f};
    const int wo = lane >> 3, wi = lane & 7;
    float hn_acc = 0.f, hd_acc = 0.f;          // fused head: thread (o1, tap) < 200
    float sgy[2] = {0.f, 0.f}, sgc[2] = {0.f, 0.f};  // fused head: sum gy1, sum gcout1*c1 of channels 2w, 2w+1

    if (r0 < r1) {
        for (int r = r0 - 2; r < r0 + 2; ++r) {  // prologue: input rows r0-2 .. r0+1, g rows r0-2, r0-1
            load_x(r);
            store_x(r);
        }
        for (int r = r0 - 2; r < r0; ++r) {
            load_g(r);
            store_g(r, false);
            load_s(r);
            store_s(r);
        }
        load_x(r0 + 2);
        load_g(r0);
        load_s(r0);
        load_e(r0 - 2);
    }
    const int last = r1 + 1;  // the last staged row (g rows up to r1 + 1 feed input-gradient rows r1-2, r1-1)
#pragma unroll 1
    for (int s = r0; s < r1 + 2; ++s) {
        const bool wg = s < r1, dg = s >= r0 + 2;
        store_x(s + 2);
        store_g(s, wg);
        store_s(s);
        const float exc[2] = {ex[0], ex[1]}, ecc[2] = {ec[0], ec[1]};
        __syncthreads();
        {   // the next step's loads, in flight under this step's FMAs (rows past the segment clamped)
            load_x(min(s + 3, last));
            load_g(min(s + 1, last));
            load_s(min(s + 1, last));
            load_e(s - 1);
        }
        if (wg) {  // ---- weight gradient of output row s: columns 16w .. 16w+15 of the strip ----
            const float* gr = lds + G_OFF + ring(s, NSG) * GSLOT + wo * GPT;
            const float* xr[5];
#pragma unroll
            for (int kh = 0; kh < 5; ++kh) xr[kh] = lds + X_OFF + ring(s - 2 + kh, NSX) * XSLOT + wi * XP;
            const int j0 = 16 * w;
            f2 gwin[5];  // gwin[k] = {gN, gD} at strip column j + k - 2 (g column index j + k)
#pragma unroll
            for (int k = 0; k < 4; ++k) gwin[k] = *reinterpret_cast<const f2*>(gr + 2 * (j0 + k));
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int j = j0 + t;
                gwin[4] = *reinterpret_cast<const f2*>(gr + 2 * (j + 4));
                f2 xv[5];
#pragma unroll
                for (int kh = 0; kh < 5; ++kh) xv[kh] = *reinterpret_cast<const f2*>(xr[kh] + 2 * j);
#pragma unroll
                for (int kh = 0; kh < 5; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 5; ++kw) wacc[kh][kw] = __builtin_elementwise_fma(xv[kh], gwin[4 - kw], wacc[kh][kw]);
#pragma unroll
                for (int k = 0; k < 4; ++k) gwin[k] = gwin[k + 1];
            }
        }
        if (dg) {  // ---- input gradient of input row s - 2: output channels 2w, 2w + 1 ----
            f2 acc[C];
#pragma unroll
            for (int i = 0; i < C; ++i) acc[i] = (f2){0.f, 0.f};
#pragma unroll 1
            for (int oo = 0; oo < 2; ++oo) {
                const int o = 2 * w + oo;
#pragma unroll 1
                for (int kh = 0; kh < 5; ++kh) {  // g row (s-2) + 2 - kh
                    const float* gr = lds + G_OFF + ring(s - kh, NSG) * GSLOT + o * GPT + 2 * lane;
                    f2 v[5];
#pragma unroll
                    for (int k = 0; k < 5; ++k) v[k] = *reinterpret_cast<const f2*>(gr + 2 * k);
                    const cfloat* wr = wgt + (o * C) * 25 + kh * 5;
#pragma unroll
                    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
                        for (int i = 0; i < C; ++i) {
                            const float wv = wr[i * 25 + kw];
                            acc[i] = __builtin_elementwise_fma((f2){wv, wv}, v[4 - kw], acc[i]);
                        }
                }
            }
            float* rp = lds + R_OFF + w * (C * 2 * TW) + 2 * lane;
#pragma unroll
            for (int i = 0; i < C; ++i) *reinterpret_cast<f2*>(rp + i * 2 * TW) = acc[i];
        }
        __syncthreads();
        if (dg) {  // ---- epilogue of input row ih = s - 2: channels 2w, 2w + 1 at column c0 + lane ----
            const int ih = s - 2, iw = c0 + lane;
            const bool ok = iw < W;
            f2 G[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float* rp = lds + R_OFF + (2 * w + k) * 2 * TW + 2 * lane;
                constexpr int WS = C * 2 * TW;
                G[k] = ((*reinterpret_cast<const f2*>(rp) + *reinterpret_cast<const f2*>(rp + WS)) +
                        *reinterpret_cast<const f2*>(rp + 2 * WS)) + *reinterpret_cast<const f2*>(rp + 3 * WS);
            }
            const unsigned eoff = ok ? (unsigned)(ih * W + iw) * 4u : OOB;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int i = 2 * w + k;
                const float gy = G[k].x * ecc[k], gco = G[k].y + G[k].x * exc[k];
                const int so = i * plane * 4;
                if constexpr (HW) {
                    if (a.gxa) st_f32(plane_rsrc(a.gxa + img, ibytes), eoff + so, gy);
                    if (a.gca) st_f32(plane_rsrc(a.gca + img, ibytes), eoff + so, gco);
                    float gN1 = 0.f, gD1 = 0.f;
                    if (ok) {
                        nconv_grad_nd(gy, gco, exc[k], ecc[k], a.heps, a.hb[i], a.hs[i], gN1, gD1);
                        sgy[k] += gy;
                        sgc[k] = fmaf(gco, ecc[k], sgc[k]);
                    }
                    *reinterpret_cast<f2*>(lds + H_OFF + i * 2 * TW + 2 * lane) = (f2){gN1, gD1};
                } else {
                    // gcout of a thresholded source has no gradient path; PLAIN here (host checks)
                    if (a.gxa) {
                        const __amdgpu_buffer_rsrc_t r = plane_rsrc(a.gxa + img, ibytes);
                        const float prev = a.accumulate ? ld_f32(r, eoff + so) : 0.f;
                        if (ok) st_f32(r, eoff + so, a.accumulate ? prev + gy : gy);
                    }
                    if (a.gca) {
                        const __amdgpu_buffer_rsrc_t r = plane_rsrc(a.gca + img, ibytes);
                        const float prev = a.accumulate ? ld_f32(r, eoff + so) : 0.f;
                        if (ok) st_f32(r, eoff + so, a.accumulate ? prev + gco : gco);
                    }
                }
            }
            if constexpr (HW) {
                __syncthreads();
                if (tid < 200) {  // thread (o1, tap): sum over the samples of S row ih + kh - 2
                    const int o1 = tid / 25, tap = tid - o1 * 25, kh = tap / 5, kw = tap - kh * 5;
                    const float* lst = lds + S_OFF + ring(ih + kh - 2, NSS) * SL;
                    const int n = __builtin_bit_cast(int, lst[0]);
                    const f2* ent = reinterpret_cast<const f2*>(lst + 2);
                    const f2* hn = reinterpret_cast<const f2*>(lds + H_OFF + o1 * 2 * TW);
                    for (int e = 0; e < n; ++e) {
                        const f2 q = ent[e];
                        const int jj = __builtin_bit_cast(int, q.x) - kw;  // strip column of the output pixel
                        if ((unsigned)jj < (unsigned)TW) {
                            const f2 h = hn[jj];
                            hn_acc = fmaf(h.x, q.y, hn_acc);
                            hd_acc += h.y;
                        }
                    }
                }
            }
        }
    }

    // ---- partial rows: the four waves' weight-gradient accumulators summed in a fixed order ----
    __syncthreads();
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
            const int e = (kh * 5 + kw) * 2;
            lds[(w * 50 + e) * 64 + lane] = wacc[kh][kw].x;
            lds[(w * 50 + e + 1) * 64 + lane] = wacc[kh][kw].y;
        }
    __syncthreads();
    float* out = part + (size_t)blockIdx.x * (NW + 2 * C);
    for (int idx = tid; idx < NW; idx += kT) {
        const int o = idx / 200, i = (idx / 25) & 7, tap = idx % 25;
        const int src = o * 8 + i, e = tap * 2;
        const float vx = ((lds[(0 * 50 + e) * 64 + src] + lds[(1 * 50 + e) * 64 + src]) + lds[(2 * 50 + e) * 64 + src]) +
                         lds[(3 * 50 + e) * 64 + src];
        const float vy = ((lds[(0 * 50 + e + 1) * 64 + src] + lds[(1 * 50 + e + 1) * 64 + src]) +
                          lds[(2 * 50 + e + 1) * 64 + src]) + lds[(3 * 50 + e + 1) * 64 + src];
        out[idx] = vx + vy;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const bool mine = hl && hk == k;
        float sb = gb_acc[k] + (mine ? gb_h : 0.f), ss = gs_acc[k] + (mine ? gs_h : 0.f);
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            sb += __shfl_xor(sb, sh);
            ss += __shfl_xor(ss, sh);
        }
        if (lane == 0) {
            out[NW + w + 4 * k] = sb;
            out[NW + C + w + 4 * k] = ss;
        }
    }
    if constexpr (HW) {
        float* oh = a.hpart + (size_t)blockIdx.x * kHeadStride;
        if (tid < 200) oh[tid] = hn_acc + hd_acc;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float sb = sgy[k], ss = sgc[k];
#pragma unroll
            for (int sh = 32; sh > 0; sh >>= 1) {
                sb += __shfl_xor(sb, sh);
                ss += __shfl_xor(ss, sh);
            }
            if (lane == 0) {
                oh[200 + 2 * w + k] = sb;
                oh[208 + 2 * w + k] = ss;
            }
        }
    }
}

// Grid of the fused backward: 64-column strips x row segments x images, about `rounds` resident
// rounds of the kernel (2 workgroups per CU: 67 KB of LDS each), at most max_blocks (the partial-row
// workspace) workgroups.
FusedGrid fused_grid(const nconv_layer& L, int max_blocks) {
    FusedGrid g;
    g.nstrip = (L.W + fb::TW - 1) / fb::TW;
    const int per_img = g.nstrip * L.B;
    static int rounds = [] {
        const char* e = getenv("NCONV_FB_ROUNDS");
        const int r = e ? atoi(e) : 3;
        return r > 0 ? r : 3;
    }();
    const int resident = dev_cus() * 2;
    int target = rounds * resident;
    if (target > max_blocks) target = max_blocks;
    int nseg = target / per_img;  // floor: never more workgroups than the target
    nseg = nseg < 1 ? 1 : (nseg > L.H ? L.H : nseg);
    g.seg_rows = (L.H + nseg - 1) / nseg;
    g.nseg = (L.H + g.seg_rows - 1) / g.seg_rows;
    g.nblk = g.nstrip * g.nseg * L.B;
    return g;
}

bool fused_bwd_ok(const nconv_layer& L) {
    return L.Cin == 8 && L.Cout == 8 && L.KH == 5 && L.KW == 5 && L.PH == 2 && L.PW == 2 && L.SH == 1 &&
           L.SW == 1 && L.DH == 1 && L.DW == 1 && L.groups == 1 && L.load_mode == NCONV_LOAD_PLAIN &&
           L.bwd_math == NCONV_MATH_FP32 && L.Ho == L.H && L.Wo == L.W && L.H >= 1 && L.W >= 1;
}

int launch_bwd_fused(const LayerDev& d, const BwdArgs& a, float* part, int max_blocks, bool gp, bool hw,
                     hipStream_t st) {
    const FusedGrid g = fused_grid(d.L, max_blocks);
    if (g.nblk > max_blocks || g.nblk <= 0) return -1;
    const dim3 grid(g.nblk), blk(fb::kT);
    if (gp && hw) hipLaunchKernelGGL((bwd_fused<true, true>), grid, blk, 0, st, d, a, part, g.nstrip, g.nseg, g.seg_rows);
    else if (gp) hipLaunchKernelGGL((bwd_fused<true, false>), grid, blk, 0, st, d, a, part, g.nstrip, g.nseg, g.seg_rows);
    else if (hw) hipLaunchKernelGGL((bwd_fused<false, true>), grid, blk, 0, st, d, a, part, g.nstrip, g.nseg, g.seg_rows);
    else hipLaunchKernelGGL((bwd_fused<false, false>), grid, blk, 0, st, d, a, part, g.nstrip, g.nseg, g.seg_rows);
    return g.nblk;
}

}  // namespace nconv
