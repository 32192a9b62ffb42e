// nconv_wgrad_bf.hip — NConv weight gradient on the bf16 matrix cores with split operands (gfx950).
//
// The same GEMM as wgrad_mfma (nconv_bwd.hip), per output row oh and 64-wide strip of the column
// index q = ow + kw:
//     gW[(kh, i)][(kw, o)] += sum_q  XC[i][oh+kh-PH][q-PW] * gN[o][oh][q-kw]  +  C[...] * gD[...]
// on v_mfma_f32_16x16x32_bf16 instead of the fp32 16x16x4 MFMA (1/16 of the bf16 rate). Every
// operand is split into NP bf16 parts, v = v0 + v1 (+ v2), and each product is formed from the
// split terms of the math mode (two parts: the three terms hi*hi, lo*hi, hi*lo, <= ~1.1e-5 relative
// per product, inside the backward's 1e-3 normwise tolerance; three parts: all nine, exact) with
// fp32 accumulation.
//
// LDS (bf16):
//   A  [plane][ring slot][q8][i]      16-byte entries (8 consecutive q): the K+1 most recent input
//                                     rows (x*c parts, c parts); one new row per output row, no halo
//                                     re-staging; an A fragment is one ds_read_b128
//   G  [buf][plane][copy][o][c]       the output row's {gN, gD} parts over the strip + its K-1 left
//                                     halo, formed from (gy, gcout, y, cout) and split once while
//                                     staging, stored twice: copy s holds g[c] at index c + s.
//                                     B[q][(kw, o)] = g[o][q - kw] is read from it directly: whatever
//                                     the kw shift, one of the copies has the fragment's 8 values at
//                                     a 4-byte-aligned start (two ds_read2_b32, no shifted copies per
//                                     kw); row pitch 37 dwords and the copies 8 * 37 + 16 dwords
//                                     apart keep the reads free of bank conflicts
// A-fragment lane groups stay on 256 contiguous bytes per q8 (conflict-free). Channels are dealt
// to waves (wave-uniform buffer resources), columns to lanes. Per output row: store the new input
// row and the next g row (double-buffered), issue the following row's loads, MFMAs, one barrier.
// Wave w takes k-step w & 1 (32 of the 64 q) and every other (M, N) tile; the tiles' partial sums
// are combined in a fixed order at the end into the block's partial row (then wgrad_reduce_sum /
// wgrad_finish).
#include "nconv_internal.h"

namespace nconv {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kWbT = 256;

template <int CIN, int COUT, int K, int NP>
struct WbCfg {
    static constexpr int SW = 64;  // q columns per strip: two k-steps of 32 (one per lane in staging)
    static constexpr int Q8 = SW / 8;
    static constexpr int M = K * CIN, N = K * COUT;
    static constexpr int MT = (M + 15) / 16, NT = (N + 15) / 16;
    static constexpr int UNITS = MT * NT;             // (M, N) tiles
    static constexpr int UPW = (UNITS + 1) / 2;       // tiles per wave (two waves per k-step)
    static constexpr int SLOTS = K + 1;
    static constexpr int NPL = 2 * NP;                // planes: operand parts, then conf / gD parts
    static constexpr int A_SLOT = Q8 * CIN * 16;      // bytes per (plane, slot): a multiple of 256
    static constexpr int A_PLANE = SLOTS * A_SLOT;
    static constexpr int G_OFF = NPL * A_PLANE;
    static constexpr int GW = SW + K - 1;             // g columns incl. the left halo
    static constexpr int GPB = 37 * 4;                       // row pitch (bytes), holds GW + 1 bf16
    static constexpr int G_COPY = (8 * 37 + 16) * 4;         // the odd-shift copy
    static constexpr int G_PLANE = 2 * G_COPY;
    static constexpr int G_BUF = NPL * G_PLANE;
    static constexpr int ZERO_OFF = G_OFF + 2 * G_BUF;
    static constexpr int STAGE = ZERO_OFF + 32;
    static constexpr int RED = 4 * UPW * 256 * 4;     // the waves' tiles at the end (bytes)
    static constexpr int LDS = STAGE > RED ? STAGE : RED;
    static constexpr int CPW = CIN / 4, OPW = COUT / 4;  // input / output channels per wave
    static_assert(A_SLOT % 256 == 0, "bank layout");
    static_assert(COUT == 8 && (CIN == 8 || CIN == 16) && (K % 2) == 1 && GW <= 2 * SW && 2 * (GW + 1) <= GPB,
                  "DNET layer shapes");
};

template <int NP>
__device__ __forceinline__ constexpr bool wb_term(int i, int j) {
    return NP == 2 ? i + j <= 1 : true;
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
    const int q0 = strip * C::SW;
    const int r0 = seg * seg_rows, r1 = min(L.Ho, r0 + seg_rows);
    constexpr unsigned OOB = 0x80000000u;

    if (tid < 2) *reinterpret_cast<f4*>(lds + C::ZERO_OFF + 16 * tid) = (f4){0.f, 0.f, 0.f, 0.f};

    // ---- per-lane fragment coordinates: A row m = (kh, i), B column n = (kw, o); k-step ks ----
    const int mi = lane & 15, h = lane >> 4, ks = w & 1, us = w >> 1;
    const int q8 = 4 * ks + h;
    int a_kh[C::UPW], a_off[C::UPW], b_off[C::UPW];
#pragma unroll
    for (int k = 0; k < C::UPW; ++k) {
        const int e = 2 * k + us;  // this wave's tiles: every other one
        const int t = e < C::UNITS ? e / C::NT : 0, u = e < C::UNITS ? e % C::NT : 0;
        const int m = 16 * t + mi, n = 16 * u + mi;
        a_kh[k] = (e < C::UNITS && m < C::M) ? m / CIN : -1;
        a_off[k] = (q8 * CIN + m % CIN) * 16;
        // B fragment: g[o][q - kw] for q = q0 + 8 q8 .. +7 = G columns c0 .. c0+7, c0 = 8 q8 + K-1-kw,
        // from the copy whose index c0 + s is even
        const int kw = n / COUT, o = n % COUT, c0 = 8 * q8 + (K - 1) - kw, sc = c0 & 1;
        b_off[k] = (e < C::UNITS && n < C::N) ? sc * C::G_COPY + o * C::GPB + 2 * (c0 + sc) : -1;
    }

    // ---- staging: lane = column, waves = channels (wave-uniform sources) ----
    float ax[C::CPW], ac[C::CPW];
    float gq[C::OPW][2][4];
    float gb_acc[C::OPW], gs_acc[C::OPW];  // bias / wsum gradient sums of this wave's channels
#pragma unroll
    for (int k = 0; k < C::OPW; ++k) gb_acc[k] = gs_acc[k] = 0.f;
    auto load_in = [&](int ih) {
#pragma unroll
        for (int k = 0; k < C::CPW; ++k) {
            const ChanSrc sc = chan_src<MODE>(d, b, w * C::CPW + k);
            load_px<MODE>(d, sc, ih, q0 - L.PW + lane, ax[k], ac[k]);
        }
    };
    auto store_in = [&](int ih) {
        const int slot = ((ih % C::SLOTS) + C::SLOTS) % C::SLOTS;
#pragma unroll
        for (int k = 0; k < C::CPW; ++k) {
            const int i = w * C::CPW + k;
            const float cv = (MODE == NCONV_LOAD_THRESH) ? (ax[k] > L.thresh ? 1.0f : 0.0f) : ac[k];
            float xc = ax[k] * cv, cc = cv;
            unsigned char* base = lds + slot * C::A_SLOT + ((lane >> 3) * CIN + i) * 16 + (lane & 7) * 2;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const __bf16 hx = (__bf16)xc, hc = (__bf16)cc;
                *reinterpret_cast<__bf16*>(base + p * C::A_PLANE) = hx;
                *reinterpret_cast<__bf16*>(base + (NP + p) * C::A_PLANE) = hc;
                xc -= (float)hx;
                cc -= (float)hc;
            }
        }
    };
    const int plane = L.Ho * L.Wo;
    auto load_g = [&](int oh) {
#pragma unroll
        for (int k = 0; k < C::OPW; ++k) {
            const int o = w * C::OPW + k;
            const size_t base = ((size_t)b * COUT + o) * plane;
            const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + base, plane * 4);
            const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + base, plane * 4);
            const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + base, plane * 4);
            const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + base : a.gy, a.gco ? plane * 4 : 0);
#pragma unroll
            for (int z = 0; z < 2; ++z) {
                const int c = z * 64 + lane, ow = q0 - (K - 1) + c;
                const bool in = c < C::GW && (unsigned)oh < (unsigned)L.Ho && (unsigned)ow < (unsigned)L.Wo;
                const unsigned off = in ? (unsigned)(oh * L.Wo + ow) * 4u : OOB;
                gq[k][z][0] = ld_f32(rgy, off);
                gq[k][z][1] = ld_f32(rco, off);
                gq[k][z][2] = ld_f32(ry, off);
                gq[k][z][3] = ld_f32(rgc, off);  // (no gcout: a zero-size resource reads 0)
            }
        }
    };
    auto store_g = [&](int buf) {
#pragma unroll
        for (int k = 0; k < C::OPW; ++k) {
            const int o = w * C::OPW + k;
            const float bo = L.bias[o], so = L.wsum[o];
#pragma unroll
            for (int z = 0; z < 2; ++z) {
                const int c = z * 64 + lane;
                if (c >= C::GW) continue;
                float gN, gD;
                nconv_grad_nd(gq[k][z][0], gq[k][z][3], gq[k][z][2], gq[k][z][1], L.eps, bo, so, gN, gD);
                unsigned char* base = lds + C::G_OFF + buf * C::G_BUF + o * C::GPB + 2 * c;
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const __bf16 hn = (__bf16)gN, hd = (__bf16)gD;
#pragma unroll
                    for (int sc = 0; sc < 2; ++sc) {  // both copies (the odd one one index later)
                        *reinterpret_cast<__bf16*>(base + p * C::G_PLANE + sc * (C::G_COPY + 2)) = hn;
                        *reinterpret_cast<__bf16*>(base + (NP + p) * C::G_PLANE + sc * (C::G_COPY + 2)) = hd;
                    }
                    gN -= (float)hn;
                    gD -= (float)hd;
                }
                if (c >= K - 1) {  // this strip's own output columns: the bias / wsum gradient sums
                    gb_acc[k] += gq[k][z][0];
                    gs_acc[k] = fmaf(gq[k][z][3], gq[k][z][1], gs_acc[k]);
                }
            }
        }
    };
    // 16 bytes from a 4-byte-aligned LDS address (two ds_read2_b32)
    auto rd16 = [&](int byte) -> bf16x8 {
        typedef unsigned u4_ __attribute__((ext_vector_type(4)));
        const unsigned* p = reinterpret_cast<const unsigned*>(lds + byte);
        return __builtin_bit_cast(bf16x8, (u4_){p[0], p[1], p[2], p[3]});
    };

    f4v acc[C::UPW];
#pragma unroll
    for (int k = 0; k < C::UPW; ++k) acc[k] = (f4v){0.f, 0.f, 0.f, 0.f};

    if (r0 < r1) {
        for (int kh = 0; kh < K; ++kh) {  // prologue: the segment's first K input rows, its first g row
            load_in(r0 - L.PH + kh);
            store_in(r0 - L.PH + kh);
        }
        load_g(r0);
        store_g(r0 & 1);
        load_in(r0 + 1 - L.PH + K - 1);
        load_g(r0 + 1 < r1 ? r0 + 1 : r0);
        __syncthreads();
    }
#pragma unroll 1
    for (int oh = r0; oh < r1; ++oh) {
        const int buf = oh & 1;
        if (oh + 1 < r1) {  // (block-uniform) the next row's input row and g row, then its loads
            store_in(oh + 1 - L.PH + K - 1);
            store_g(buf ^ 1);
            const int nx = oh + 2 < r1 ? oh + 2 : oh + 1;
            load_in(nx - L.PH + K - 1);
            load_g(nx);
        }
#pragma unroll
        for (int k = 0; k < C::UPW; ++k) {
            if (2 * k + us >= C::UNITS) continue;  // (wave-uniform)
            bf16x8 fa[C::NPL], fb[C::NPL];
            const int ih = oh - L.PH + a_kh[k];
            const int slot = ((ih % C::SLOTS) + C::SLOTS) % C::SLOTS;
            const int ao = a_kh[k] < 0 ? C::ZERO_OFF : slot * C::A_SLOT + a_off[k];
            const int ap = a_kh[k] < 0 ? 0 : C::A_PLANE;
            const int bo = b_off[k] < 0 ? C::ZERO_OFF : C::G_OFF + buf * C::G_BUF + b_off[k];
            const int bp = b_off[k] < 0 ? 0 : C::G_PLANE;
#pragma unroll
            for (int p = 0; p < C::NPL; ++p) {
                fa[p] = *reinterpret_cast<const bf16x8*>(lds + ao + p * ap);
                fb[p] = rd16(bo + p * bp);
            }
            // smallest terms first: (input part i, g part j) of x*c . gN and of c . gD
#pragma unroll
            for (int s = 2 * (NP - 1); s >= 0; --s)
#pragma unroll
                for (int i = NP - 1; i >= 0; --i) {
                    const int j = s - i;
                    if (j < 0 || j >= NP || !wb_term<NP>(i, j)) continue;
                    acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[k], 0, 0, 0);
                    acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[NP + i], fb[NP + j], acc[k], 0, 0, 0);
                }
        }
        __syncthreads();
    }

    // ---- the two k-steps' tiles summed in a fixed order -> this block's partial row ----
    constexpr int NW = COUT * CIN * K * K;
    float* out = part + (size_t)blockIdx.x * (NW + 2 * COUT);
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < C::UPW; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((w * C::UPW + k) * 4 + r) * 64 + lane] = acc[k][r];
    __syncthreads();
    for (int e = tid; e < C::UNITS * 256; e += kWbT) {
        const int unit = e >> 8, l = e & 63, r = (e >> 6) & 3;
        const int k = unit >> 1, usx = unit & 1;  // unit = 2 k + us
        // the unit's two waves: w = 2 us + ks, k-step 0 then 1
        const float v = red[(((2 * usx) * C::UPW + k) * 4 + r) * 64 + l] +
                        red[(((2 * usx + 1) * C::UPW + k) * 4 + r) * 64 + l];
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

// Launch: strips of 64 q (q = ow + kw spans Wo + K - 1 columns) x row segments x images, at most
// two resident rounds of workgroups; returns the number of blocks (partial rows) written.
template <int CIN, int COUT, int K, int MODE, int NP>
static int go_wgrad_bf_np(const LayerDev& d, const BwdArgs& a, float* part, int max_blocks, hipStream_t st) {
    const nconv_layer& L = d.L;
    static int per_cu = 0;
    if (per_cu == 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wgrad_bf<CIN, COUT, K, MODE, NP>, kWbT, 0) != hipSuccess ||
            n <= 0)
            n = 1;
        per_cu = n;
    }
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int target = 2 * per_cu * cus;
    if (target > max_blocks) target = max_blocks;
    const int nstrip = (L.Wo + K - 1 + 63) / 64;
    const int per_img = nstrip * L.B;
    int nseg = target / per_img;
    nseg = nseg < 1 ? 1 : (nseg > L.Ho ? L.Ho : nseg);
    int seg_rows = (L.Ho + nseg - 1) / nseg;
    if (seg_rows < 1) seg_rows = 1;
    nseg = (L.Ho + seg_rows - 1) / seg_rows;
    const int nblk = nstrip * nseg * L.B;
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
