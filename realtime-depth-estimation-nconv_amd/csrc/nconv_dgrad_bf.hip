// nconv_dgrad_bf.hip — NConv input gradient on the bf16 matrix cores with split operands (gfx950).
//
// The transposed convolution of the backward (nconv_bwd.hip's header)
//     G_xc[i][ih][iw] = sum_{o,kh,kw} W[o][i][kh][kw] * gN[o][ih+PH-kh][iw+PW-kw]      (G_c: gD)
// as a GEMM per group of R = 16 / Cin input rows on v_mfma_f32_16x16x32_bf16:
//     A[m][(kh', kw, o)] = g[o][top - kh'][iw0 + m + PW - kw]      m: 16 adjacent input columns
//     B[(kh', kw, o)][(rr, i)] = W[o][i][kh' - (R-1) + rr][kw]      (0 outside the kernel)
// where top = ih0 + PH + R - 1 is the newest output row the group reads: the input-row offset rr
// lives in B, so one A fragment feeds all R rows and all Cin channels (N = R * Cin = 16). The k
// index runs over (kw, kh', o) with o innermost: a k-group of 8 is one (kh', kw) pair, i.e. one
// output pixel's 8 channels — a 16-byte LDS entry, so every A fragment is one ds_read_b128 and the
// kw shift costs nothing. Operands are split into NP bf16 parts (bf16x3: hi*hi + lo*hi + hi*lo,
// <= ~1.1e-5 relative per product; bf16x9: all nine, exact) with fp32 accumulation; the weights'
// B fragments stay in registers for the workgroup's lifetime.
//
// Block = 256 threads, a strip of SW = 124 input columns (8 M-tiles of 16 = 128 computed, the last
// K - 1 discarded: the 128 staged g columns cover exactly SW + K - 1), a segment of rows, 4 waves
// x 2 M-tiles. LDS: a ring of KH2 + R g rows (KH2 = K + R - 1 read per group, R staged for the
// next), [plane][slot][column][o] bf16, planes = gN parts then gD parts; the slot pitch is a
// multiple of 256 B so the two k-groups of a ds_read_b128 lane group (same kw, adjacent kh') are
// conflict-free. Staging: thread = (row, column) of the R new g rows (R = 1: column, channel
// half), its 8 (4) channels' (gy, gcout, y, cout) -> {gN, gD} -> split -> one 16-byte (8-byte)
// store per plane. Per group: fragments + MFMAs, store the next rows, issue the loads after
// that, epilogue (gx = G_xc*c, gc = G_c + G_xc*x routed through the glue's backward, 4 adjacent
// pixels per lane), one barrier.
#include "nconv_internal.h"
#include "nconv_route.h"

namespace nconv {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kDbT = 256;
constexpr unsigned kOOBd = 0x80000000u;

template <int CIN, int COUT, int K, int NP>
struct DbCfg {
    static constexpr int R = 16 / CIN;             // input rows per GEMM (N = R * CIN = 16)
    static constexpr int SQ = 128;                 // staged g columns = computed input columns
    static constexpr int SW = 124;                 // stored input columns per strip (<= SQ - K + 1, 4-aligned)
    static constexpr int KH2 = K + R - 1;          // g rows one group reads
    static constexpr int KHE = (KH2 + 1) & ~1;     // per kw, rounded up to pairs (a duplicate fills)
    static constexpr int NG = ((K * KHE + 3) / 4) * 4;  // k-groups incl. duplicates
    static constexpr int NKS = NG / 4;             // k-steps of 32
    static constexpr int SL = KH2 + R;             // ring slots
    static constexpr int SP = 2304;                // slot pitch (bytes): 144 entries >= SQ + K - 1, = 9 * 256
    static constexpr int PLANE = SL * SP;
    static constexpr int NPL = 2 * NP;
    static constexpr int LDS = NPL * PLANE;
    static constexpr int CPT = R == 2 ? 8 : 4;     // g channels per staging thread
    static_assert(COUT == 8 && (CIN == 8 || CIN == 16) && SW + K - 1 <= SQ && SQ + K - 1 <= SP / 16, "DNET shapes");
};

template <int NP>
__device__ __forceinline__ constexpr bool db_term(int i, int j) {
    return NP == 2 ? i + j <= 1 : true;
}

// k-group p -> (kh', kw); duplicates repeat the previous group's pair (their B rows are zero)
template <int K, int KH2, int KHE>
__device__ __forceinline__ void group_of(int p, int& khp, int& kw, bool& real) {
    const int lim = K * KHE;  // (KHE even: a pair of groups always shares kw)
    const int q = p < lim ? p : lim - 1;
    kw = q / KHE;
    khp = q % KHE;
    real = p < lim && khp < KH2;
    if (khp >= KH2) khp = KH2 - 1;
}

template <int CIN, int COUT, int K, int MODE, int NP>
__global__ __launch_bounds__(kDbT) void dgrad_bf(LayerDev d, BwdArgs a, float* tmp_x, float* tmp_c, int nstrip,
                                                 int nseg, int seg_rows) {
    using C = DbCfg<CIN, COUT, K, NP>;
    constexpr int R = C::R;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS];
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int strip = blk % nstrip;
    blk /= nstrip;
    const int seg = blk % nseg, b = blk / nseg;
    const int iw0 = strip * C::SW;
    const int r0 = seg * seg_rows, r1 = min(L.H, r0 + seg_rows);
    const int ow0 = iw0 + L.PW - (K - 1);  // output column of staged g column 0

    // ---- B fragments (weights), registers for the block's lifetime ----
    const int mi = lane & 15, h = lane >> 4;
    bf16x8 bw[C::NKS][NP];
    {
        const int rr = mi / CIN, i = mi % CIN;
#pragma unroll
        for (int ks = 0; ks < C::NKS; ++ks) {
            int khp, kw;
            bool real;
            group_of<K, C::KH2, C::KHE>(4 * ks + h, khp, kw, real);
            const int kh = khp - (R - 1) + rr;
            float v[8];
#pragma unroll
            for (int o = 0; o < 8; ++o)
                v[o] = (real && kh >= 0 && kh < K) ? L.weight[((o * CIN + i) * K + kh) * K + kw] : 0.f;
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                float r = v[o];
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const __bf16 hb = (__bf16)r;
                    bw[ks][p][o] = hb;
                    if (p + 1 < NP) r -= (float)hb;
                }
            }
        }
    }
    // A fragment coordinates per k-step: the k-group's kh' and byte offset of (column m, kw)
    int a_khp[C::NKS], a_col[C::NKS];
#pragma unroll
    for (int ks = 0; ks < C::NKS; ++ks) {
        int khp, kw;
        bool real;
        group_of<K, C::KH2, C::KHE>(4 * ks + h, khp, kw, real);
        a_khp[ks] = khp;
        a_col[ks] = (mi + (K - 1) - kw) * 16;
    }

    // ---- staging: thread = (row rr, column) [R = 2] or (column, channel half) [R = 1] ----
    const int s_col = tid & 127;
    const int s_rr = R == 2 ? w >> 1 : 0;
    const int s_o0 = R == 2 ? 0 : (w >> 1) * 4;  // (wave-uniform: one buffer resource per channel)
    const int plane_o = L.Ho * L.Wo;
    float gq[C::CPT][4];
    bool g_ok = false;
    // one resource per saved tensor over the image's COUT planes, the channel in soffset
    const size_t img = (size_t)b * COUT * plane_o;
    const int img_bytes = COUT * plane_o * 4;
    const __amdgpu_buffer_rsrc_t rgy = plane_rsrc(a.gy + img, img_bytes);
    const __amdgpu_buffer_rsrc_t rco = plane_rsrc(a.co + img, img_bytes);
    const __amdgpu_buffer_rsrc_t ry = plane_rsrc(a.y + img, img_bytes);
    const __amdgpu_buffer_rsrc_t rgc = plane_rsrc(a.gco ? a.gco + img : a.gy, a.gco ? img_bytes : 0);
    auto load_g = [&](int top) {  // rows top - R + 1 .. top of the ring: this thread's one
        const int oh = top - (R - 1) + s_rr, ow = ow0 + s_col;
        g_ok = (unsigned)oh < (unsigned)L.Ho && (unsigned)ow < (unsigned)L.Wo;
        const unsigned off = g_ok ? (unsigned)(oh * L.Wo + ow) * 4u : kOOBd;
#pragma unroll
        for (int k = 0; k < C::CPT; ++k) {
            const int so = (s_o0 + k) * plane_o * 4;
            gq[k][0] = ld_f32s(rgy, off, so);
            gq[k][1] = ld_f32s(rco, off, so);
            gq[k][2] = ld_f32s(ry, off, so);
            gq[k][3] = ld_f32s(rgc, off, so);
        }
    };
    auto slot_of = [](int oh) { return ((oh % C::SL) + C::SL) % C::SL; };
    auto store_g = [&](int top) {
        const int oh = top - (R - 1) + s_rr;
        unsigned char* base = lds + slot_of(oh) * C::SP + s_col * 16 + s_o0 * 2;
        float gN[C::CPT], gD[C::CPT];
#pragma unroll
        for (int k = 0; k < C::CPT; ++k) {
            const int o = s_o0 + k;
            nconv_grad_nd(gq[k][0], gq[k][3], gq[k][2], gq[k][1], L.eps, L.bias[o], L.wsum[o], gN[k], gD[k]);
            gN[k] = g_ok ? gN[k] : 0.f;
            gD[k] = g_ok ? gD[k] : 0.f;
        }
        if constexpr (C::CPT == 8) {
            bf16x8 pn[NP], pd[NP];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float rn = gN[k], rd = gD[k];
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const __bf16 hn = (__bf16)rn, hd = (__bf16)rd;
                    pn[p][k] = hn;
                    pd[p][k] = hd;
                    if (p + 1 < NP) {
                        rn -= (float)hn;
                        rd -= (float)hd;
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                *reinterpret_cast<bf16x8*>(base + p * C::PLANE) = pn[p];
                *reinterpret_cast<bf16x8*>(base + (NP + p) * C::PLANE) = pd[p];
            }
        } else {
            bf16x4 pn[NP], pd[NP];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float rn = gN[k], rd = gD[k];
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const __bf16 hn = (__bf16)rn, hd = (__bf16)rd;
                    pn[p][k] = hn;
                    pd[p][k] = hd;
                    if (p + 1 < NP) {
                        rn -= (float)hn;
                        rd -= (float)hd;
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                *reinterpret_cast<bf16x4*>(base + p * C::PLANE) = pn[p];
                *reinterpret_cast<bf16x4*>(base + (NP + p) * C::PLANE) = pd[p];
            }
        }
    };

    if (r0 >= r1) return;  // (block-uniform)
    // prologue: the first group's KH2 g rows, R at a time, then the next group's loads
    const int top0 = r0 + L.PH + R - 1;
    for (int t = top0 - C::KH2 + R; t <= top0; t += R) {
        load_g(t);
        store_g(t);
    }
    load_g(top0 + R);
    __syncthreads();

#pragma unroll 1
    for (int ih0 = r0; ih0 < r1; ih0 += R) {
        const int top = ih0 + L.PH + R - 1;
        const int st = slot_of(top);
        f4v accN[2], accD[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) accN[t] = accD[t] = (f4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < C::NKS; ++ks) {
            int sl = st - a_khp[ks];
            sl = sl < 0 ? sl + C::SL : sl;
            bf16x8 fa[2][C::NPL];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int off = sl * C::SP + (2 * w + t) * 256 + a_col[ks];
#pragma unroll
                for (int p = 0; p < C::NPL; ++p) fa[t][p] = *reinterpret_cast<const bf16x8*>(lds + off + p * C::PLANE);
            }
#pragma unroll
            for (int s = 2 * (NP - 1); s >= 0; --s)
#pragma unroll
                for (int i = NP - 1; i >= 0; --i) {
                    const int j = s - i;
                    if (j < 0 || j >= NP || !db_term<NP>(i, j)) continue;
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        accN[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][i], bw[ks][j], accN[t], 0, 0, 0);
                        accD[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][NP + i], bw[ks][j], accD[t], 0, 0, 0);
                    }
                }
        }
        if (ih0 + R < r1) {  // (block-uniform) the next group's rows, then the loads after them
            store_g(top + R);
            load_g(top + 2 * R);
        }
        // epilogue: lane = (rr, i) column of the tile, 4 adjacent input columns
        {
            const int rr = mi / CIN, i = mi % CIN;
            const int ih = ih0 + rr;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int m0 = (2 * w + t) * 16 + 4 * h;
                const int iw = iw0 + m0;
                int nv = min(C::SW - m0, L.W - iw);
                nv = nv > 4 ? 4 : nv;
                if (ih < r1 && nv > 0) {
                    const float gx[4] = {accN[t][0], accN[t][1], accN[t][2], accN[t][3]};
                    const float gc[4] = {accD[t][0], accD[t][1], accD[t][2], accD[t][3]};
                    dg_route4<MODE>(d, a, b, i, ih, iw, nv, gx, gc, tmp_x, tmp_c);
                }
            }
        }
        __syncthreads();
    }
}

}  // namespace

template <int CIN, int COUT, int K, int MODE, int NP>
static void go_dgrad_bf_np(const LayerDev& d, const BwdArgs& a, float* tmp_x, float* tmp_c, hipStream_t st) {
    using C = DbCfg<CIN, COUT, K, NP>;
    const nconv_layer& L = d.L;
    const int per_cu = dev_occupancy((const void*)dgrad_bf<CIN, COUT, K, MODE, NP>, kDbT, 0);
    const int cus = dev_cus();
    const int target = per_cu * cus;
    const int nstrip = (L.W + C::SW - 1) / C::SW;
    const int per_img = nstrip * L.B;
    int nseg = target / per_img;
    nseg = nseg < 1 ? 1 : (nseg > L.H ? L.H : nseg);
    int seg_rows = (L.H + nseg - 1) / nseg;
    seg_rows = (seg_rows + C::R - 1) / C::R * C::R;  // whole row groups
    nseg = (L.H + seg_rows - 1) / seg_rows;
    hipLaunchKernelGGL((dgrad_bf<CIN, COUT, K, MODE, NP>), dim3(nstrip * nseg * L.B), dim3(kDbT), 0, st, d, a, tmp_x,
                       tmp_c, nstrip, nseg, seg_rows);
}

template <int CIN, int COUT, int K, int MODE>
void go_dgrad_bf(const LayerDev& d, const BwdArgs& a, float* tmp_x, float* tmp_c, int np, hipStream_t st) {
    if (np == 3) go_dgrad_bf_np<CIN, COUT, K, MODE, 3>(d, a, tmp_x, tmp_c, st);
    else go_dgrad_bf_np<CIN, COUT, K, MODE, 2>(d, a, tmp_x, tmp_c, st);
}

template void go_dgrad_bf<8, 8, 5, NCONV_LOAD_PLAIN>(const LayerDev&, const BwdArgs&, float*, float*, int, hipStream_t);
template void go_dgrad_bf<8, 8, 5, NCONV_LOAD_POOL2>(const LayerDev&, const BwdArgs&, float*, float*, int, hipStream_t);
template void go_dgrad_bf<16, 8, 3, NCONV_LOAD_UPCAT_SKIP_FIRST>(const LayerDev&, const BwdArgs&, float*, float*, int,
                                                                hipStream_t);
template void go_dgrad_bf<16, 8, 3, NCONV_LOAD_UPCAT_UP_FIRST>(const LayerDev&, const BwdArgs&, float*, float*, int,
                                                              hipStream_t);

}  // namespace nconv
