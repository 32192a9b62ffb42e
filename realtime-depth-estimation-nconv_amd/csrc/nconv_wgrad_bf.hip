// nconv_wgrad_bf.hip — NConv weight gradient on the bf16 matrix cores with split operands (gfx950).
//
// The same GEMM as wgrad_mfma (nconv_bwd.hip), per output row oh, over the column index
// q = ow - o0 + kw of a strip of output columns [o0, o0 + OW):
//     gW[(kh, i)][(kw, o)] += sum_q  XC[i][oh+kh-PH][o0+q-PW] * gN[o][oh][o0+q-kw]  +  C[...] * gD[...]
// (gN, gD zero outside the strip's own columns, so every output column is counted once) on
// v_mfma_f32_16x16x32_bf16 instead of the fp32 16x16x4 MFMA (1/16 of the bf16 rate). Every operand
// is split into NP bf16 parts, v = v0 + v1 (+ v2), and each product is formed from the split terms
// of the math mode (two parts: the three terms hi*hi, lo*hi, hi*lo, <= ~1.1e-5 relative per
// product, inside the backward's 1e-3 normwise tolerance; three parts: all nine, exact) with fp32
// accumulation.
//
// A strip is 128 q = four k-steps of 32, one per wave; each wave computes every (M, N) tile of its
// k-step, and the four waves' tiles are summed in a fixed order at the end into the block's
// partial row (then wgrad_reduce_sum / wgrad_finish). Staging deals two adjacent columns to a lane
// (so every LDS store is a packed bf16 pair, one ds_write_b32) and channels to waves (wave-uniform
// buffer resources).
//
// LDS (bf16):
//   A  [plane][ring slot][q8][i ^ sw(q8)]   16-byte entries (8 consecutive q): the K+1 most recent
//                                input rows (x*c parts, c parts); one new row per output row; an A
//                                fragment is one ds_read_b128 (conflict-free); the channel swizzle
//                                sw(q8) = (q8 >> 1) & 3 keeps the staging stores at 2-way (free)
//   G  [buf][plane][copy][o][index]   the output row's {gN, gD} parts, formed from (gy, gcout, y,
//                                cout) and split once while staging; copy s holds g[c'] at index
//                                c' + K - 1 + s. B[q][(kw, o)] = g[o][q - kw] is read from it
//                                directly: whatever the kw shift one copy has the fragment's 8
//                                values at a 4-byte-aligned start (two ds_read2_b32, no shifted
//                                copies per kw). Rows are 65 dwords apart (dword 65 past a row's
//                                start is the next row's zero pad), rows 4..7 264 dwords after rows
//                                0..3 and the odd copy 528 after the even one: conflict-free reads.
// Per output row: read the row's fragments, store the next input row and g row (double-buffered),
// issue the loads of the row after, the MFMAs, one barrier.
#include "nconv_internal.h"

namespace nconv {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

constexpr int kWbT = 256;

template <int CIN, int COUT, int K, int NP>
struct WbCfg {
    static constexpr int SQ = 128;  // q columns per strip: four k-steps of 32, one per wave
    static constexpr int Q8 = SQ / 8;
    static constexpr int OW = SQ - (K - 1);  // output columns owned by a strip
    static constexpr int M = K * CIN, N = K * COUT;
    static constexpr int MT = (M + 15) / 16, NT = (N + 15) / 16;
    static constexpr int UNITS = MT * NT;  // (M, N) tiles, all of them in every wave
    static constexpr int SLOTS = K + 1;
    static constexpr int NPL = 2 * NP;  // planes: operand parts, then conf / gD parts
    static constexpr int A_SLOT = Q8 * CIN * 16;  // bytes per (plane, slot): a multiple of 256
    static constexpr int A_PLANE = SLOTS * A_SLOT;
    static constexpr int G_OFF = NPL * A_PLANE;
    static constexpr int GP = 65, G_HALF = 264, G_COPY = 528, G_PLANE = 1056;  // dwords
    static constexpr int G_BUF = NPL * G_PLANE;                                // dwords
    static constexpr int ZERO_OFF = G_OFF + 2 * G_BUF * 4;                     // bytes
    static constexpr int STAGE = ZERO_OFF + 16;
    static constexpr int RED = 4 * UNITS * 256 * 4;  // the waves' tiles at the end (bytes)
    static constexpr int LDS = STAGE > RED ? STAGE : RED;
    static constexpr int CPW = CIN / 4, OPW = COUT / 4;  // input / output channels per wave
    static constexpr int HALO = (K - 1) / 2;             // G dword of column 0 (K - 1 is even)
    static_assert(A_SLOT % 256 == 0, "bank layout");
    static_assert(COUT == 8 && (CIN == 8 || CIN == 16) && (K % 2) == 1 && OW <= 2 * 64, "DNET layer shapes");
    static_assert(3 * GP + G_HALF + GP + 1 <= G_COPY && G_COPY + 3 * GP + G_HALF + GP + 1 <= G_PLANE, "G image");
};

__device__ __forceinline__ constexpr int g_row(int o) { return (o & 3) * 65 + (o >> 2) * 264; }

template <int NP>
__device__ __forceinline__ constexpr bool wb_term(int i, int j) {
    return NP == 2 ? i + j <= 1 : true;
}

// (a, b) -> NP packed bf16 pairs, each the rounding of what the previous pairs left
template <int NP>
__device__ __forceinline__ void split2(float a, float b, unsigned (&out)[NP]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const bf16x2 h = {(__bf16)a, (__bf16)b};
        out[p] = __builtin_bit_cast(unsigned, h);
        if (p + 1 < NP) {
            a -= (float)h[0];
            b -= (float)h[1];
        }
    }
}

template <int CIN, int COUT, int K, int MODE, int NP>
__global__ __launch_bounds__(kWbT) void wgrad_bf(LayerDev d, BwdArgs a, float* part, int nstrip, int nseg,
                                                 int seg_rows) {
    using C = WbCfg<CIN, COUT, K, NP>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int strip = blk % nstrip;
    blk /= nstrip;
    const int seg = blk % nseg, b = blk / nseg;
    const int o0 = strip * C::OW;
    const int r0 = seg * seg_rows, r1 = min(L.Ho, r0 + seg_rows);
    constexpr unsigned OOB = 0x80000000u;

    // the G image's pads and the zero slot read 0
    for (int e = tid; e < 2 * C::G_BUF + 4; e += kWbT) reinterpret_cast<unsigned*>(lds + C::G_OFF)[e] = 0u;

    // ---- per-lane fragment coordinates: A row m = (kh, i), B column n = (kw, o); k-step = wave ----
    const int mi = lane & 15, h = lane >> 4;
    const int q8 = 4 * w + h;
    int a_kh[C::MT], a_pos[C::MT], b_pos[C::NT];
#pragma unroll
    for (int t = 0; t < C::MT; ++t) {
        const int m = 16 * t + mi, i = m % CIN;
        a_kh[t] = m < C::M ? m / CIN : -1;
        a_pos[t] = (q8 * CIN + (i ^ ((q8 >> 1) & 3))) * 16;
    }
#pragma unroll
    for (int u = 0; u < C::NT; ++u) {
        // g[o][q - kw] for q = 8 q8 .. +7: indices c0 .. c0+7 of copy 0, from the copy whose start is even
        const int n = 16 * u + mi, kw = n / COUT, o = n % COUT, c0 = 8 * q8 + (K - 1) - kw, sc = c0 & 1;
        b_pos[u] = n < C::N ? 4 * (sc * C::G_COPY + g_row(o) + ((c0 + sc) >> 1)) : -1;
    }

    // ---- staging: lanes take column pairs, waves channels ----
    float ax[C::CPW][2], ac[C::CPW][2];
    float gq[C::OPW][2][4];
    float gb_acc[C::OPW], gs_acc[C::OPW];  // bias / wsum gradient sums of this wave's channels
#pragma unroll
    for (int k = 0; k < C::OPW; ++k) gb_acc[k] = gs_acc[k] = 0.f;
    auto load_in = [&](int ih) {
#pragma unroll
        for (int k = 0; k < C::CPW; ++k) {
            const ChanSrc sc = chan_src<MODE>(d, b, w * C::CPW + k);
#pragma unroll
            for (int j = 0; j < 2; ++j) load_px<MODE>(d, sc, ih, o0 - L.PW + 2 * lane + j, ax[k][j], ac[k][j]);
        }
    };
    const int a_st = ((lane >> 2) * CIN) * 16 + (lane & 3) * 4, a_sw = (lane >> 3) & 3;
    auto store_in = [&](int slot) {
#pragma unroll
        for (int k = 0; k < C::CPW; ++k) {
            const int i = w * C::CPW + k;
            float cv[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) cv[j] = (MODE == NCONV_LOAD_THRESH) ? (ax[k][j] > L.thresh ? 1.0f : 0.0f) : ac[k][j];
            unsigned px[NP], pc[NP];
            split2<NP>(ax[k][0] * cv[0], ax[k][1] * cv[1], px);
            split2<NP>(cv[0], cv[1], pc);
            unsigned char* base = lds + slot * C::A_SLOT + a_st + (i ^ a_sw) * 16;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                *reinterpret_cast<unsigned*>(base + p * C::A_PLANE) = px[p];
                *reinterpret_cast<unsigned*>(base + (NP + p) * C::A_PLANE) = pc[p];
            }
        }
    };
    const int plane = L.Ho * L.Wo;
    bool g_in[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) g_in[j] = 2 * lane + j < C::OW && o0 + 2 * lane + j < L.Wo;
    const size_t img = (size_t)b * COUT * plane;  // one resource per saved tensor, the channel in soffset
    const int img_bytes = COUT * plane * 4;
    const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + img, img_bytes);
    const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + img, img_bytes);
    const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + img, img_bytes);
    const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + img : a.gy, a.gco ? img_bytes : 0);
    auto load_g = [&](int oh) {
#pragma unroll
        for (int k = 0; k < C::OPW; ++k) {
            const int so = (w * C::OPW + k) * plane * 4;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const unsigned off = g_in[j] ? (unsigned)(oh * L.Wo + o0 + 2 * lane + j) * 4u : OOB;
                gq[k][j][0] = ld_f32s(rgy, off, so);
                gq[k][j][1] = ld_f32s(rco, off, so);
                gq[k][j][2] = ld_f32s(ry, off, so);
                gq[k][j][3] = ld_f32s(rgc, off, so);  // (no gcout: a zero-size resource reads 0)
            }
        }
    };
    const bool g_st = lane + C::HALO < C::GP;  // the lane's G dword lies inside its row
    float bias_o[C::OPW], wsum_o[C::OPW];        // read once, not per row
#pragma unroll
    for (int k = 0; k < C::OPW; ++k) {
        bias_o[k] = L.bias[w * C::OPW + k];
        wsum_o[k] = L.wsum[w * C::OPW + k];
    }
    auto store_g = [&](int buf, bool count) {  // count: a new row (its bias / wsum sums taken)
#pragma unroll
        for (int k = 0; k < C::OPW; ++k) {
            const int o = w * C::OPW + k;
            const float bo = bias_o[k], so = wsum_o[k];
            float gN[2], gD[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                nconv_grad_nd(gq[k][j][0], gq[k][j][3], gq[k][j][2], gq[k][j][1], L.eps, bo, so, gN[j], gD[j]);
                gN[j] = g_in[j] ? gN[j] : 0.f;
                gD[j] = g_in[j] ? gD[j] : 0.f;
                // (0 outside the strip's own columns)
                gb_acc[k] = count ? gb_acc[k] + gq[k][j][0] : gb_acc[k];
                gs_acc[k] = count ? fmaf(gq[k][j][3], gq[k][j][1], gs_acc[k]) : gs_acc[k];
            }
            unsigned pn[NP], pd[NP];
            split2<NP>(gN[0], gN[1], pn);
            split2<NP>(gD[0], gD[1], pd);
            unsigned* base = reinterpret_cast<unsigned*>(lds + C::G_OFF) + buf * C::G_BUF + g_row(o) + C::HALO + lane;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                // the odd copy's dword: (g[2 lane - 1], g[2 lane]), the first from the previous lane
                const unsigned prev_n = __builtin_amdgcn_update_dpp(0u, pn[p], 0x138, 0xf, 0xf, false);  // wave_shr:1
                const unsigned prev_d = __builtin_amdgcn_update_dpp(0u, pd[p], 0x138, 0xf, 0xf, false);
                if (g_st) {
                    base[p * C::G_PLANE] = pn[p];
                    base[(NP + p) * C::G_PLANE] = pd[p];
                    base[p * C::G_PLANE + C::G_COPY] = __builtin_amdgcn_alignbit(pn[p], prev_n, 16);
                    base[(NP + p) * C::G_PLANE + C::G_COPY] = __builtin_amdgcn_alignbit(pd[p], prev_d, 16);
                }
            }
        }
    };

    f4v acc[C::MT][C::NT];
#pragma unroll
    for (int t = 0; t < C::MT; ++t)
#pragma unroll
        for (int u = 0; u < C::NT; ++u) acc[t][u] = (f4v){0.f, 0.f, 0.f, 0.f};

    auto mod_slots = [](int v) { return ((v % C::SLOTS) + C::SLOTS) % C::SLOTS; };
    __syncthreads();  // (the G pads are zero before any row is stored)
    if (r0 < r1) {
        for (int kh = 0; kh < K; ++kh) {  // prologue: the segment's first K input rows, its first g row
            load_in(r0 - L.PH + kh);
            store_in(mod_slots(r0 - L.PH + kh));
        }
        load_g(r0);
        store_g(0, true);
        load_in(r0 + 1 - L.PH + K - 1);
        load_g(r0 + 1 < r1 ? r0 + 1 : r0);
        __syncthreads();
    }
    int s0 = mod_slots(r0 - L.PH);  // ring slot of input row oh - PH
#pragma unroll 1
    for (int oh = r0; oh < r1; ++oh) {
        const int buf = (oh - r0) & 1;
        bf16x8 fa[C::MT][C::NPL], fb[C::NT][C::NPL];
#pragma unroll
        for (int t = 0; t < C::MT; ++t) {
            int sl = s0 + a_kh[t];
            sl = sl >= C::SLOTS ? sl - C::SLOTS : sl;
            const int ao = a_kh[t] < 0 ? C::ZERO_OFF : sl * C::A_SLOT + a_pos[t];
            const int ap = a_kh[t] < 0 ? 0 : C::A_PLANE;
#pragma unroll
            for (int p = 0; p < C::NPL; ++p) fa[t][p] = *reinterpret_cast<const bf16x8*>(lds + ao + p * ap);
        }
#pragma unroll
        for (int u = 0; u < C::NT; ++u) {
            const int bo = b_pos[u] < 0 ? C::ZERO_OFF : C::G_OFF + 4 * buf * C::G_BUF + b_pos[u];
            const int bp = b_pos[u] < 0 ? 0 : 4 * C::G_PLANE;
#pragma unroll
            for (int p = 0; p < C::NPL; ++p) {
                const unsigned* q = reinterpret_cast<const unsigned*>(lds + bo + p * bp);
                fb[u][p] = __builtin_bit_cast(bf16x8, (u4v){q[0], q[1], q[2], q[3]});
            }
        }
        {   // the next row's input row and g row, then its loads. Unconditional (after the last row
            // they fill a ring slot and a g buffer no MFMA of this row reads): a branch here would make
            // the compiler copy the in-flight load registers, i.e. wait for them, before the MFMAs
            store_in(s0 + K >= C::SLOTS ? s0 + K - C::SLOTS : s0 + K);
            store_g(buf ^ 1, oh + 1 < r1);
            const int nx = oh + 2 < r1 ? oh + 2 : r1 - 1;
            load_in(nx - L.PH + K - 1);
            load_g(nx);
        }
        // smallest terms first: (input part i, g part j) of x*c . gN and of c . gD
#pragma unroll
        for (int s = 2 * (NP - 1); s >= 0; --s)
#pragma unroll
            for (int i = NP - 1; i >= 0; --i) {
                const int j = s - i;
                if (j < 0 || j >= NP || !wb_term<NP>(i, j)) continue;
#pragma unroll
                for (int t = 0; t < C::MT; ++t)
#pragma unroll
                    for (int u = 0; u < C::NT; ++u)
                        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][i], fb[u][j], acc[t][u], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < C::MT; ++t)
#pragma unroll
                    for (int u = 0; u < C::NT; ++u)
                        acc[t][u] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][NP + i], fb[u][NP + j], acc[t][u], 0, 0, 0);
            }
        s0 = s0 + 1 == C::SLOTS ? 0 : s0 + 1;
        __syncthreads();
    }

    // ---- the four k-steps' tiles summed in a fixed order -> this block's partial row ----
    constexpr int NW = COUT * CIN * K * K;
    float* out = part + (size_t)blockIdx.x * (NW + 2 * COUT);
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < C::MT; ++t)
#pragma unroll
        for (int u = 0; u < C::NT; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((w * C::UNITS + t * C::NT + u) * 4 + r) * 64 + lane] = acc[t][u][r];
    __syncthreads();
    for (int e = tid; e < C::UNITS * 256; e += kWbT) {
        const int unit = e >> 8, l = e & 63, r = (e >> 6) & 3;
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) v += red[((ww * C::UNITS + unit) * 4 + r) * 64 + l];
        const int t = unit / C::NT, u = unit % C::NT;
        const int m = 16 * t + (l >> 4) * 4 + r, n = 16 * u + (l & 15);
        if (m < C::M && n < C::N) {
            const int kh = m / CIN, i = m % CIN, kw = n / COUT, o = n % COUT;
            out[((o * CIN + i) * K + kh) * K + kw] = v;
        }
    }
    // bias / wsum sums: each wave's channels, lanes combined in a fixed butterfly order
#pragma unroll
    for (int k = 0; k < C::OPW; ++k) {
        float sb = gb_acc[k], ss = gs_acc[k];
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) {
            sb += __shfl_xor(sb, sh);
            ss += __shfl_xor(ss, sh);
        }
        if (lane == 0) {
            out[NW + w * C::OPW + k] = sb;
            out[NW + COUT + w * C::OPW + k] = ss;
        }
    }
}

}  // namespace

// Launch: strips of OW output columns x row segments x images, one resident round of workgroups
// (at most max_blocks, the workspace's partial rows); returns the number of blocks written.
template <int CIN, int COUT, int K, int MODE, int NP>
static int go_wgrad_bf_np(const LayerDev& d, const BwdArgs& a, float* part, int max_blocks, hipStream_t st) {
    using C = WbCfg<CIN, COUT, K, NP>;
    const nconv_layer& L = d.L;
    const int per_cu = dev_occupancy((const void*)wgrad_bf<CIN, COUT, K, MODE, NP>, kWbT, 0);
    const int cus = dev_cus();
    int target = per_cu * cus;
    if (target > max_blocks) target = max_blocks;
    const int nstrip = (L.Wo + C::OW - 1) / C::OW;
    const int per_img = nstrip * L.B;
    int nseg = target / per_img;
    nseg = nseg < 1 ? 1 : (nseg > L.Ho ? L.Ho : nseg);
    int seg_rows = (L.Ho + nseg - 1) / nseg;
    if (seg_rows < 1) seg_rows = 1;
    nseg = (L.Ho + seg_rows - 1) / seg_rows;
    const int nblk = nstrip * nseg * L.B;
    if (nblk > max_blocks) return -1;
    hipLaunchKernelGGL((wgrad_bf<CIN, COUT, K, MODE, NP>), dim3(nblk), dim3(kWbT), 0, st, d, a, part, nstrip, nseg,
                       seg_rows);
    return nblk;
}

template <int CIN, int COUT, int K, int MODE>
int go_wgrad_bf(const LayerDev& d, const BwdArgs& a, float* part, int max_blocks, int np, hipStream_t st) {
    if (np == 3) return go_wgrad_bf_np<CIN, COUT, K, MODE, 3>(d, a, part, max_blocks, st);
    return go_wgrad_bf_np<CIN, COUT, K, MODE, 2>(d, a, part, max_blocks, st);
}

template int go_wgrad_bf<8, 8, 5, NCONV_LOAD_PLAIN>(const LayerDev&, const BwdArgs&, float*, int, int, hipStream_t);
template int go_wgrad_bf<8, 8, 5, NCONV_LOAD_POOL2>(const LayerDev&, const BwdArgs&, float*, int, int, hipStream_t);
template int go_wgrad_bf<16, 8, 3, NCONV_LOAD_UPCAT_SKIP_FIRST>(const LayerDev&, const BwdArgs&, float*, int, int,
                                                                hipStream_t);
template int go_wgrad_bf<16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST>(const LayerDev&, const BwdArgs&, float*, int, int,
                                                              hipStream_t);

}  // namespace nconv
