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
constexpr int H_OFF = R_OFF + 4 * C * 2 * TW;  // nconv1's {gN1, gD1} of a row, [2 (row parity)][8][64] f2
constexpr int SL = 2 + 2 * GW;               // per S row: count (+ pad), then (column, S) of the samples
constexpr int S_OFF = H_OFF + 2 * 2 * C * TW;
constexpr int W_OFF = S_OFF + NSS * SL;
constexpr int LDS_MAIN = W_OFF;
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

    // Step s computes from the rings and stages the NEXT step's rows at its end: the loads are
    // issued at the top of step s (in flight under its FMAs) and stored to LDS after its epilogue,
    // inside the same iteration -- no loaded register lives across the loop back-edge (the
    // compiler would copy it there and wait for the load at the copy). The epilogue's (x, c) loads
    // go first: loads return in order, so waiting for them does not wait for the row loads.
    if (r0 < r1) {
        for (int r = r0 - 2; r <= r0 + 2; ++r) {  // prologue: input rows r0-2 .. r0+2, g rows r0-2 .. r0
            load_x(r);
            store_x(r);
        }
        for (int r = r0 - 2; r <= r0; ++r) {
            load_g(r);
            store_g(r, r >= r0);
            load_s(r);
            store_s(r);
        }
        __syncthreads();
    }
    const int last = r1 + 1;  // the last staged row (g rows up to r1 + 1 feed input-gradient rows r1-2, r1-1)
    float hbk[2], hsk[2];      // fused head: nconv1's bias / normaliser of channels 2w, 2w + 1
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        hbk[k] = HW ? a.hb[2 * w + k] : 0.f;
        hsk[k] = HW ? a.hs[2 * w + k] : 1.f;
    }
    // fused head: nconv1's weight-gradient sums of input row ih (its {gN1, gD1} row in the parity
    // buffer the epilogue wrote), thread (o1, tap) over the samples of S row ih + kh - 2; run at the
    // top of the NEXT step (beside the other waves' FMAs, no barrier of its own)
    auto head_list = [&](int ih) {
        if constexpr (HW) {
            if (tid < 200) {
                const int o1 = tid / 25, tap = tid - o1 * 25, kh = tap / 5, kw = tap - kh * 5;
                const float* lst = lds + S_OFF + ring(ih + kh - 2, NSS) * SL;
                const int n = __builtin_bit_cast(int, lst[0]);
                const f2* ent = reinterpret_cast<const f2*>(lst + 2);
                const f2* hn = reinterpret_cast<const f2*>(lds + H_OFF + ((ih & 1) * C + o1) * 2 * TW);
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
    };
#pragma unroll 1
    for (int s = r0; s < r1 + 2; ++s) {
        const bool wg = s < r1, dg = s >= r0 + 2;
        const int nx = min(s + 1, last);  // the next step's g / S row (clamped: the last step re-loads)
        load_e(s - 2);
        load_x(min(s + 3, last));
        load_g(nx);
        load_s(nx);
        const float* exc = ex;
        const float* ecc = ec;
        if (s >= r0 + 3) head_list(s - 3);  // the previous step's input-gradient row
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
                        nconv_grad_nd(gy, gco, exc[k], ecc[k], a.heps, hbk[k], hsk[k], gN1, gD1);
                        sgy[k] += gy;
                        sgc[k] = fmaf(gco, ecc[k], sgc[k]);
                    }
                    *reinterpret_cast<f2*>(lds + H_OFF + ((ih & 1) * C + i) * 2 * TW + 2 * lane) = (f2){gN1, gD1};
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
        }
        if (s + 1 < r1 + 2) {  // stage the next step's rows (their slots' previous rows are done)
            store_x(s + 3);
            store_g(s + 1, s + 1 < r1);
            store_s(s + 1);
        }
        __syncthreads();
    }
    if (r0 < r1) head_list(r1 - 1);  // the last input-gradient row

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



// ================================================================================================
// nconv6 + nconv7 (the training tail) in one backward kernel.
//
// nconv6 is 16 -> 8, 3x3, padding 0 over cat(up2x(x23) [channels 0..7], x2 [8..15]) (step1.py:88-90,
// UP_FIRST), and its output feeds nconv7 (1x1, padding 2), whose backward is folded in as in
// dgrad_phase<T7> / wgrad_mfma<T7>: nconv6's (gy, gcout) are formed from nconv7's (gy, y, cout) while
// {gN, gD} are staged, nconv7's weight gradient is summed beside nconv6's. Row-streaming strips as
// bwd_fused (input rows s of a 64-column strip, segments of an even number of rows):
//   * weight gradient of output row s (lane = (o, i8): the upsampled channel i8 and the skip channel
//     8 + i8, 9 taps each; the input rows s .. s+2 staged at full resolution, the upsampled half
//     expanded from its low plane at staging);
//   * skip-channel input gradient of input row s (g rows s-2 .. s; lane = column, wave = output-
//     channel pair, the four waves' partials summed in a fixed order);
//   * after each odd row s = 2p + 1, the upsampled channels' gradient of low row p straight into the
//     low-resolution producer: the nearest-upsample backward sums a 2x2 block, which is a 4x4
//     correlation of {gN, gD} (g rows 2p-2 .. 2p+1) with box-summed weights (dgrad_phase's form;
//     lane = (low column, channel half), box weights broadcast from LDS).
namespace ft {
constexpr int kT = 256;
constexpr int CO = 8, CI = 16, TW = 64, LW = TW / 2;
constexpr int GW = TW + 2;               // g columns c0-2 .. c0+63
constexpr int XP = 136, GPT = 136;       // channel-row pitches (floats), 8 * pitch distinct mod 64
constexpr int NSX = 3, NSG = 4;
constexpr int XSLOT = CI * XP, GSLOT = CO * GPT;
constexpr int X_OFF = 0;
constexpr int G_OFF = X_OFF + NSX * XSLOT;
constexpr int RS_OFF = G_OFF + NSG * GSLOT;      // skip partials [4][8][64] f2
constexpr int RU_OFF = RS_OFF + 4 * 8 * 2 * TW;  // upsampled partials [4][8][32] f2
constexpr int WB_OFF = RU_OFF + 4 * 8 * 2 * LW;  // box weights [o][t][u][i]
constexpr int LDS_MAIN = WB_OFF + CO * 16 * 8;
constexpr int FIN = 4 * 36 * 64;
constexpr int LDS = LDS_MAIN > FIN ? LDS_MAIN : FIN;
constexpr int NW = CO * CI * 9;          // 1152 weights
constexpr unsigned OOB = 0x80000000u;
static_assert(XP >= 2 * TW && GPT >= 2 * GW, "pitches");
}  // namespace ft

__global__ __launch_bounds__(ft::kT) __attribute__((amdgpu_waves_per_eu(2, 2))) void bwd_fused_tail(
    LayerDev d, BwdArgs a, float* part, int nstrip, int nseg, int seg_rows) {
    using namespace ft;
    __shared__ __attribute__((aligned(16))) float lds[LDS];
    const nconv_layer& L = d.L;
    const cfloat* wgt = (const cfloat*)L.weight;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const TileCoord tc = xcd_tile(nstrip, nseg, L.B);
    const int b = tc.b, c0 = tc.tx * TW;
    const int H = L.H, W = L.W, Ho = L.Ho, Wo = L.Wo, Hl = L.b.H, Wl = L.b.W;
    const int r0 = tc.ty * seg_rows, r1 = min(H, r0 + seg_rows);
    const int plane = H * W, lplane = Hl * Wl, oplane = Ho * Wo;

    // box weights [o][t][u][i] (t, u = 0..3 collect the taps S(0) = {2}, S(1) = {1, 2}, S(2) = {0, 1},
    // S(3) = {0}; dgrad_phase / box_weights), from the upsampled channels' weights (0..7)
    for (int e = tid; e < CO * 16 * 8; e += kT) {
        const int i = e & 7, u = (e >> 3) & 3, t = (e >> 5) & 3, o = e >> 7;
        const cfloat* wk = wgt + ((size_t)o * CI + i) * 9;
        const int h0 = t == 0 ? 2 : (t == 1 ? 1 : 0), nh = (t == 1 || t == 2) ? 2 : 1;
        const int w0 = u == 0 ? 2 : (u == 1 ? 1 : 0), nw = (u == 1 || u == 2) ? 2 : 1;
        float sum = 0.f;
        for (int r = 0; r < nh; ++r)
            for (int c = 0; c < nw; ++c) sum += wk[(h0 + r) * 3 + w0 + c];
        lds[WB_OFF + e] = sum;
    }

    // ---- resources ----
    const __amdgpu_buffer_rsrc_t rax = plane_rsrc(L.a.x + (size_t)b * 8 * plane, 8 * plane * 4);
    const __amdgpu_buffer_rsrc_t rac = plane_rsrc(L.a.c + (size_t)b * 8 * plane, 8 * plane * 4);
    const __amdgpu_buffer_rsrc_t rbx = plane_rsrc(L.b.x + (size_t)b * 8 * lplane, 8 * lplane * 4);
    const __amdgpu_buffer_rsrc_t rbc = plane_rsrc(L.b.c + (size_t)b * 8 * lplane, 8 * lplane * 4);
    const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + (size_t)b * CO * oplane, CO * oplane * 4);
    const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + (size_t)b * CO * oplane, CO * oplane * 4);
    const int pl7 = a.t7ph * a.t7pw;
    const __amdgpu_buffer_rsrc_t r7g = plane_rsrc(a.t7gy + (size_t)b * pl7, pl7 * 4);
    const __amdgpu_buffer_rsrc_t r7y = plane_rsrc(a.t7y + (size_t)b * pl7, pl7 * 4);
    const __amdgpu_buffer_rsrc_t r7c = plane_rsrc(a.t7co + (size_t)b * pl7, pl7 * 4);

    // ---- input rows: wave w stages the upsampled channels w, w + 4 and the skip channels 8 + w, 12 + w ----
    float px[4], pc[4];
    const int iwl = c0 + lane;
    auto load_x = [&](int ih) {
        const bool in = (unsigned)ih < (unsigned)H && iwl < W;
        const unsigned off = in ? (unsigned)(ih * W + iwl) * 4u : OOB;
        const unsigned offl = in ? (unsigned)((ih >> 1) * Wl + (iwl >> 1)) * 4u : OOB;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            px[k] = ld_f32s(rbx, offl, (w + 4 * k) * lplane * 4);
            pc[k] = ld_f32s(rbc, offl, (w + 4 * k) * lplane * 4);
            px[2 + k] = ld_f32s(rax, off, (w + 4 * k) * plane * 4);
            pc[2 + k] = ld_f32s(rac, off, (w + 4 * k) * plane * 4);
        }
    };
    auto store_x = [&](int ih) {
        float* xs = lds + X_OFF + ring(ih, NSX) * XSLOT + 2 * lane;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ch = (k < 2 ? 0 : 8) + w + 4 * (k & 1);
            *reinterpret_cast<f2*>(xs + ch * XP) = (f2){px[k] * pc[k], pc[k]};
        }
    };

    // ---- g rows (nconv6's output row oh, columns c0-2+m, m = 0..65): {gN, gD} of channels w, w+4 from
    //      nconv7's planes; main pass m = lane, halo lanes 0..3: channel w + 4 (lane >> 1), m = 64 + (lane & 1) ----
    float g7[2][3], gv[2][2], gvh[2];
    const bool hl = lane < 4;
    const int hk = (lane >> 1) & 1, ho = w + 4 * hk;
    const int owm = c0 - 2 + lane, owh = c0 + 62 + (lane & 1);
    auto load_g = [&](int oh) {
        const unsigned o7 = t7_off(a, oh, owm, Ho, Wo, OOB), o7h = hl ? t7_off(a, oh, owh, Ho, Wo, OOB) : OOB;
        g7[0][0] = ld_f32(r7g, o7);
        g7[0][1] = ld_f32(r7y, o7);
        g7[0][2] = ld_f32(r7c, o7);
        g7[1][0] = ld_f32(r7g, o7h);
        g7[1][1] = ld_f32(r7y, o7h);
        g7[1][2] = ld_f32(r7c, o7h);
        const bool in = (unsigned)oh < (unsigned)Ho && (unsigned)owm < (unsigned)Wo;
        const bool inh = hl && (unsigned)oh < (unsigned)Ho && (unsigned)owh < (unsigned)Wo;
        const unsigned off = in ? (unsigned)(oh * Wo + owm) * 4u : OOB;
        const unsigned offh = inh ? (unsigned)((ho * Ho + oh) * Wo + owh) * 4u : OOB;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            gv[k][0] = ld_f32s(ry, off, (w + 4 * k) * oplane * 4);
            gv[k][1] = ld_f32s(rco, off, (w + 4 * k) * oplane * 4);
        }
        gvh[0] = ld_f32(ry, offh);
        gvh[1] = ld_f32(rco, offh);
    };
    float bias_o[2], wsum_o[2], w7_o[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        bias_o[k] = L.bias[w + 4 * k];
        wsum_o[k] = L.wsum[w + 4 * k];
        w7_o[k] = a.t7w[w + 4 * k];
    }
    const float bias_h = hk ? bias_o[1] : bias_o[0], wsum_h = hk ? wsum_o[1] : wsum_o[0], w7_h = hk ? w7_o[1] : w7_o[0];
    float gb_acc[2] = {0.f, 0.f}, gs_acc[2] = {0.f, 0.f}, gb_h = 0.f, gs_h = 0.f;
    float w7n[2] = {0.f, 0.f}, w7d[2] = {0.f, 0.f}, w7nh = 0.f, w7dh = 0.f;
    auto store_g = [&](int oh, bool count) {
        float* gs = lds + G_OFF + ring(oh, NSG) * GSLOT;
        float n7, d7, n7h, d7h;
        t7_nd(a, g7[0][0], g7[0][1], g7[0][2], n7, d7);
        t7_nd(a, g7[1][0], g7[1][1], g7[1][2], n7h, d7h);
        const bool own = count && lane >= 2;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float gy, gco, gN, gD;
            t7_gy(w7_o[k], n7, d7, gv[k][0], gv[k][1], gy, gco);
            nconv_grad_nd(gy, gco, gv[k][0], gv[k][1], L.eps, bias_o[k], wsum_o[k], gN, gD);
            *reinterpret_cast<f2*>(gs + (w + 4 * k) * GPT + 2 * lane) = (f2){gN, gD};
            if (own) {
                gb_acc[k] += gy;
                gs_acc[k] = fmaf(gco, gv[k][1], gs_acc[k]);
                w7n[k] = fmaf(gv[k][0] * gv[k][1], n7, w7n[k]);  // nconv7: corr(x*c, gN7) + corr(c, gD7)
                w7d[k] = fmaf(gv[k][1], d7, w7d[k]);
            }
        }
        float gy, gco, gN, gD;
        t7_gy(w7_h, n7h, d7h, gvh[0], gvh[1], gy, gco);
        nconv_grad_nd(gy, gco, gvh[0], gvh[1], L.eps, bias_h, wsum_h, gN, gD);
        if (hl) {
            *reinterpret_cast<f2*>(gs + ho * GPT + 2 * (64 + (lane & 1))) = (f2){gN, gD};
            if (count) {
                gb_h += gy;
                gs_h = fmaf(gco, gvh[1], gs_h);
                w7nh = fmaf(gvh[0] * gvh[1], n7h, w7nh);
                w7dh = fmaf(gvh[1], d7h, w7dh);
            }
        }
    };
    // epilogue inputs: the skip row's (x, c) for channels 2w, 2w+1 at column c0 + lane; the low row's
    // (x, c) of channel i = tid >> 5 at low column c0/2 + (tid & 31)
    float ex[2], ec[2], ux = 0.f, uc = 0.f;
    auto load_e = [&](int ih) {
        const bool in = (unsigned)ih < (unsigned)H && iwl < W;
        const unsigned off = in ? (unsigned)(ih * W + iwl) * 4u : OOB;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            ex[k] = ld_f32s(rax, off, (2 * w + k) * plane * 4);
            ec[k] = ld_f32s(rac, off, (2 * w + k) * plane * 4);
        }
    };
    const int uq = tid & 31, ui = tid >> 5, uql = (c0 >> 1) + uq;
    auto load_u = [&](int p) {
        const bool in = (unsigned)p < (unsigned)Hl && uql < Wl;
        // (the channel differs between the wave's two 32-lane halves: its plane offset rides the
        // per-lane offset, not soffset, which must be wave-uniform)
        const unsigned off = (in ? (unsigned)(p * Wl + uql) * 4u : OOB) + (unsigned)(ui * lplane * 4);
        ux = ld_f32(rbx, off);
        uc = ld_f32(rbc, off);
    };

    f2 wu[3][3], wsk[3][3];  // weight-gradient accumulators: lane (o, i8), upsampled i8 / skip 8 + i8
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) wu[kh][kw] = wsk[kh][kw] = (f2){0.f, 0.f};
    const int wo = lane >> 3, wi = lane & 7;

    // as bwd_fused: the next step's rows are loaded at the top of step s and staged at its end (no
    // loaded register across the back-edge); the epilogues' loads are issued first
    if (r0 < r1) {
        for (int r = r0; r <= r0 + 2; ++r) {  // prologue: input rows r0 .. r0+2; g rows r0-2 .. r0
            load_x(r);
            store_x(r);
        }
        for (int r = r0 - 2; r <= r0; ++r) {
            load_g(r);
            store_g(r, r >= r0);
        }
        __syncthreads();
    }
    const bool accm = a.accumulate != 0;
#pragma unroll 1
    for (int s = r0; s < r1; ++s) {
        const bool up = (s & 1) != 0;  // low row (s - 1) / 2 complete after this row
        load_e(s);
        load_u(s >> 1);
        load_x(min(s + 3, r1 + 1));  // (rows past the segment clamped: staged, unused)
        load_g(min(s + 1, r1));
        const float* exc = ex;
        const float* ecc = ec;
        const float uxc = ux, ucc = uc;
        if (s < Ho) {  // ---- weight gradient of output row s: columns 16w .. 16w+15 ----
            const float* gr = lds + G_OFF + ring(s, NSG) * GSLOT + wo * GPT;
            const float* xu[3];
            const float* xk[3];
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                xu[kh] = lds + X_OFF + ring(s + kh, NSX) * XSLOT + wi * XP;
                xk[kh] = xu[kh] + 8 * XP;
            }
            const int j0 = 16 * w;
            f2 gwin[3];  // gwin[k] = g at local column j + k  (ow = iw - 2 + k, i.e. kw = 2 - k)
#pragma unroll
            for (int k = 0; k < 2; ++k) gwin[k] = *reinterpret_cast<const f2*>(gr + 2 * (j0 + k));
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int j = j0 + t;
                gwin[2] = *reinterpret_cast<const f2*>(gr + 2 * (j + 2));
                f2 vu[3], vk[3];
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    vu[kh] = *reinterpret_cast<const f2*>(xu[kh] + 2 * j);
                    vk[kh] = *reinterpret_cast<const f2*>(xk[kh] + 2 * j);
                }
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        wu[kh][kw] = __builtin_elementwise_fma(vu[kh], gwin[2 - kw], wu[kh][kw]);
                        wsk[kh][kw] = __builtin_elementwise_fma(vk[kh], gwin[2 - kw], wsk[kh][kw]);
                    }
                gwin[0] = gwin[1];
                gwin[1] = gwin[2];
            }
        }
        {   // ---- skip-channel input gradient of input row s: output channels 2w, 2w + 1 ----
            f2 acc[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = (f2){0.f, 0.f};
#pragma unroll 1
            for (int oo = 0; oo < 2; ++oo) {
                const int o = 2 * w + oo;
#pragma unroll 1
                for (int kh = 0; kh < 3; ++kh) {  // g row s - kh, columns iw - kw -> local j + 2 - kw
                    const float* gr = lds + G_OFF + ring(s - kh, NSG) * GSLOT + o * GPT + 2 * lane;
                    f2 v[3];
#pragma unroll
                    for (int k = 0; k < 3; ++k) v[k] = *reinterpret_cast<const f2*>(gr + 2 * k);
                    const cfloat* wr = wgt + ((size_t)o * CI + 8) * 9 + kh * 3;
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const float wv = wr[i * 9 + kw];
                            acc[i] = __builtin_elementwise_fma((f2){wv, wv}, v[2 - kw], acc[i]);
                        }
                }
            }
            float* rp = lds + RS_OFF + w * (8 * 2 * TW) + 2 * lane;
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<f2*>(rp + i * 2 * TW) = acc[i];
        }
        if (up) {  // ---- upsampled channels of low row p = (s - 1) / 2: g rows 2p-2 .. 2p+1 = s-3 .. s ----
            const int q = lane & 31, ih4 = lane >> 5;  // low column, channel half (4 ih4 .. 4 ih4 + 3)
            f2 au[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) au[c] = (f2){0.f, 0.f};
#pragma unroll 1
            for (int oo = 0; oo < 2; ++oo) {
                const int o = 2 * w + oo;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float* gr = lds + G_OFF + ring(s - 3 + t, NSG) * GSLOT + o * GPT + 4 * q;
                    const f4 q0 = *reinterpret_cast<const f4*>(gr), q1 = *reinterpret_cast<const f4*>(gr + 4);
                    const f2 g[4] = {q0.xy, q0.zw, q1.xy, q1.zw};
                    const float* wb = lds + WB_OFF + (o * 16 + t * 4) * 8 + 4 * ih4;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const f4 wv = *reinterpret_cast<const f4*>(wb + u * 8);
#pragma unroll
                        for (int c = 0; c < 4; ++c) au[c] = __builtin_elementwise_fma((f2){wv[c], wv[c]}, g[u], au[c]);
                    }
                }
            }
            float* rp = lds + RU_OFF + w * (8 * 2 * LW) + 2 * q;
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<f2*>(rp + (4 * ih4 + c) * 2 * LW) = au[c];
        }
        __syncthreads();
        {   // ---- skip epilogue: input row s, channels 2w, 2w + 1 -> gxa / gca ----
            const bool ok = iwl < W;
            const unsigned eoff = ok ? (unsigned)(s * W + iwl) * 4u : OOB;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int i = 2 * w + k;
                const float* rp = lds + RS_OFF + i * 2 * TW + 2 * lane;
                constexpr int WS = 8 * 2 * TW;
                const f2 G = ((*reinterpret_cast<const f2*>(rp) + *reinterpret_cast<const f2*>(rp + WS)) +
                              *reinterpret_cast<const f2*>(rp + 2 * WS)) + *reinterpret_cast<const f2*>(rp + 3 * WS);
                const float gx = G.x * ecc[k], gc = G.y + G.x * exc[k];
                const unsigned o = eoff + (unsigned)(i * plane * 4);
                if (a.gxa) {
                    const __amdgpu_buffer_rsrc_t r = plane_rsrc(a.gxa + (size_t)b * 8 * plane, 8 * plane * 4);
                    const float prev = accm ? ld_f32(r, o) : 0.f;
                    if (ok) st_f32(r, o, accm ? prev + gx : gx);
                }
                if (a.gca) {
                    const __amdgpu_buffer_rsrc_t r = plane_rsrc(a.gca + (size_t)b * 8 * plane, 8 * plane * 4);
                    const float prev = accm ? ld_f32(r, o) : 0.f;
                    if (ok) st_f32(r, o, accm ? prev + gc : gc);
                }
            }
        }
        if (up) {  // ---- upsampled epilogue: low row p, channel ui, low column c0/2 + uq -> gxb / gcb ----
            const int p = (s - 1) >> 1;
            const bool ok = p < Hl && uql < Wl;
            const float* rp = lds + RU_OFF + ui * 2 * LW + 2 * uq;
            constexpr int WS = 8 * 2 * LW;
            const f2 G = ((*reinterpret_cast<const f2*>(rp) + *reinterpret_cast<const f2*>(rp + WS)) +
                          *reinterpret_cast<const f2*>(rp + 2 * WS)) + *reinterpret_cast<const f2*>(rp + 3 * WS);
            const float gx = G.x * ucc, gc = G.y + G.x * uxc;
            const unsigned o = ok ? (unsigned)((ui * Hl + p) * Wl + uql) * 4u : OOB;
            if (a.gxb) {
                const __amdgpu_buffer_rsrc_t r = plane_rsrc(a.gxb + (size_t)b * 8 * lplane, 8 * lplane * 4);
                const float prev = accm ? ld_f32(r, o) : 0.f;
                if (ok) st_f32(r, o, accm ? prev + gx : gx);
            }
            if (a.gcb) {
                const __amdgpu_buffer_rsrc_t r = plane_rsrc(a.gcb + (size_t)b * 8 * lplane, 8 * lplane * 4);
                const float prev = accm ? ld_f32(r, o) : 0.f;
                if (ok) st_f32(r, o, accm ? prev + gc : gc);
            }
        }
        if (s + 1 < r1) {  // stage the next step's rows (their slots' previous rows are done)
            store_x(s + 3);
            store_g(s + 1, true);
        }
        __syncthreads();
    }

    // ---- partial rows ----
    __syncthreads();
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int e = (kh * 3 + kw) * 2;
            lds[(w * 36 + e) * 64 + lane] = wu[kh][kw].x;
            lds[(w * 36 + e + 1) * 64 + lane] = wu[kh][kw].y;
            lds[(w * 36 + 18 + e) * 64 + lane] = wsk[kh][kw].x;
            lds[(w * 36 + 18 + e + 1) * 64 + lane] = wsk[kh][kw].y;
        }
    __syncthreads();
    float* out = part + (size_t)blockIdx.x * (NW + 2 * CO);
    for (int idx = tid; idx < NW; idx += kT) {  // gW[o][i][kh][kw], i < 8 upsampled, 8.. skip
        const int o = idx / 144, i = (idx / 9) % 16, tap = idx % 9;
        const int src = o * 8 + (i & 7), e = (i < 8 ? 0 : 18) + tap * 2;
        float v[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
            v[pp] = ((lds[(0 * 36 + e + pp) * 64 + src] + lds[(1 * 36 + e + pp) * 64 + src]) +
                     lds[(2 * 36 + e + pp) * 64 + src]) + lds[(3 * 36 + e + pp) * 64 + src];
        out[idx] = v[0] + v[1];
    }
    float* o7 = a.t7part + (size_t)blockIdx.x * 10;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const bool mine = hl && hk == k;
        float sb = gb_acc[k] + (mine ? gb_h : 0.f), ss = gs_acc[k] + (mine ? gs_h : 0.f);
        float sn = w7n[k] + (mine ? w7nh : 0.f), sd = w7d[k] + (mine ? w7dh : 0.f);
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            sb += __shfl_xor(sb, sh);
            ss += __shfl_xor(ss, sh);
            sn += __shfl_xor(sn, sh);
            sd += __shfl_xor(sd, sh);
        }
        if (lane == 0) {
            out[NW + w + 4 * k] = sb;
            out[NW + CO + w + 4 * k] = ss;
            o7[w + 4 * k] = sn + sd;
        }
    }
    if (tid < 2) o7[8 + tid] = 0.f;
}

bool fused_tail_bwd_ok(const nconv_layer& L) {
    return L.Cin == 16 && L.Cout == 8 && L.a.C == 8 && L.b.C == 8 && L.KH == 3 && L.KW == 3 && L.PH == 0 &&
           L.PW == 0 && L.SH == 1 && L.SW == 1 && L.DH == 1 && L.DW == 1 && L.groups == 1 &&
           L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST && L.bwd_math == NCONV_MATH_FP32 && L.a.H == L.H &&
           L.a.W == L.W && L.H == 2 * L.b.H && L.W == 2 * L.b.W && L.Ho == L.H - 2 && L.Wo == L.W - 2 && L.H >= 2;
}

int launch_bwd_fused_tail(const LayerDev& d, const BwdArgs& a, float* part, int max_blocks, hipStream_t st) {
    const nconv_layer& L = d.L;
    const int nstrip = (L.W + ft::TW - 1) / ft::TW, per_img = nstrip * L.B;
    static int rounds = [] {
        const char* e = getenv("NCONV_FB_ROUNDS");
        const int r = e ? atoi(e) : 3;
        return r > 0 ? r : 3;
    }();
    int target = rounds * dev_cus() * 2;
    if (target > max_blocks) target = max_blocks;
    int nseg = target / per_img;
    nseg = nseg < 1 ? 1 : (nseg > L.H / 2 ? L.H / 2 : nseg);
    int seg_rows = (L.H + nseg - 1) / nseg;
    seg_rows += seg_rows & 1;  // even: a low row's two full-resolution rows in one segment
    nseg = (L.H + seg_rows - 1) / seg_rows;
    const int nblk = nstrip * nseg * L.B;
    if (nblk > max_blocks || nblk <= 0) return -1;
    hipLaunchKernelGGL(bwd_fused_tail, dim3(nblk), dim3(ft::kT), 0, st, d, a, part, nstrip, nseg, seg_rows);
    return nblk;
}

}  // namespace nconv
