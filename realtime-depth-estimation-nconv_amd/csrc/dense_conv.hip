// dense_conv.hip — dense convolutions of the RGB-guided model on the gfx950 matrix cores.
//
// The RGB encoder (models/step2.py:134-154) and the fusion decoder (step2.py:156-297) are plain
// K x C x R x S contractions, so they run as implicit GEMMs on v_mfma_f32_32x32x2_f32 (fp32 in,
// fp32 accumulate: exact f32 products, the precision of the reference's fp32 convolutions):
//   A = weights  [Cout][k]        (M = output channels, 32 per tile)
//   B = im2col   [k][pixel]       (N = 32 output columns of one output row)
//   k = (tap, input channel)      (K, input channels staged 8 at a time)
// A workgroup (4 waves) owns an output tile of TH rows x 32 columns x all Cout of one image; each
// wave owns TH/4 rows. Per 8-channel chunk the input patch (with halo) and the chunk's packed
// weights are staged in LDS (loads for the next chunk issued before this chunk's MFMAs); an MFMA
// k-step pairs two input channels (lane half kk = lane >> 5 takes channel 2p + kk), so every
// operand read is one ds_read_b32 at a compile-time offset from a per-lane base. The epilogue
// applies bias (eval BatchNorm folded in by nconv_dense_pack), ReLU and the RGBEncoder 1x1
// shortcut (computed from the centre tap of the same patch) and writes a channel range of the
// output tensor, so torch.cat of the decoder never materialises: convolutions write their half
// of the concatenated tensor and the next one reads two sources.
//
// Kinds: 3x3 pad 1 stride 1|2; 1x1 stride 1|2; ConvTranspose 4x4 stride 2 pad 1 as four
// output-parity classes, each a 2x2 gather over the input's 3x3 neighbourhood.
#include "nconv_internal.h"

namespace nconv {

constexpr int kDT = 256;
constexpr int kCK = 8;  // input channels per staged chunk

constexpr int round_mod64(int n, int target) {  // smallest m >= n with m % 64 == target
    return n + (((target - n) % 64) + 64) % 64;
}

template <int COUT, int KIND, int S>
struct DcCfg {
    static constexpr bool TR = KIND == NCONV_DENSE_TRANSPOSED_4X4;
    static constexpr int TAPS = KIND == NCONV_DENSE_3X3 ? 9 : (KIND == NCONV_DENSE_1X1 ? 1 : 4);
    static constexpr int SP = TR ? 1 : S;                 // patch stride
    static constexpr int KS = KIND == NCONV_DENSE_1X1 ? 1 : 3;
    static constexpr int TH = SP == 1 ? 8 : 4, RW = TH / 4, TW = 32;
    static constexpr int PR = (TH - 1) * SP + KS, PC = (TW - 1) * SP + KS;
    static constexpr int ROW = PC;
    // B reads: 32 lanes on the columns of one patch row, lane half kk on the channel plane:
    // kk * PLANE must shift to the other 32 banks (stride 1) or the odd banks (stride 2)
    static constexpr int PLANE = SP == 1 ? round_mod64(PR * ROW, 32) : ((PR * ROW) | 1);
    static constexpr int MT = COUT / 32;
    static constexpr int COP = COUT == 32 ? 32 : 96;      // A reads: kk * COP == 32 (mod 64)
    static constexpr int W_OFF = kCK * PLANE;
    static constexpr int WS_OFF = W_OFF + TAPS * kCK * COP;  // shortcut weights [ci][COP]
    static constexpr int LDS = WS_OFF + kCK * COP;
    static constexpr int NP = (kCK * PR * PC + kDT - 1) / kDT;        // patch elements per thread
    static constexpr int NW4 = (TAPS * kCK * COUT / 4 + kDT - 1) / kDT;  // weight float4s per thread
    static constexpr int NS4 = (kCK * COUT / 4 + kDT - 1) / kDT;
    static constexpr int CENTER = KIND == NCONV_DENSE_3X3 ? 4 : 0;   // tap of the 1x1 shortcut
};

typedef float f16v __attribute__((ext_vector_type(16)));

template <int COUT, int KIND, int S, bool SC>
__global__ __launch_bounds__(kDT) void dense_conv_mfma(nconv_dense_conv p, int ntx, int nty) {
    using C = DcCfg<COUT, KIND, S>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int tx = blk % ntx;
    blk /= ntx;
    const int ty = blk % nty;
    blk /= nty;
    const int cls = C::TR ? blk % 4 : 0;  // output parity class (transposed)
    const int b = C::TR ? blk / 4 : blk;
    const int pa = cls >> 1, pb = cls & 1;
    const int oy0 = ty * C::TH, ox0 = tx * C::TW;  // tile origin (output grid, or class grid)
    const int pad = C::TR ? 1 : (C::KS / 2);
    const int iy0 = oy0 * C::SP - pad, ix0 = ox0 * C::SP - pad;  // patch origin in the input
    const int Cin = p.C0 + p.C1;
    const int nchunk = (Cin + kCK - 1) / kCK;
    const int HW = p.H * p.W;

    // ---- staging: patch (8 channels x PR x PC, zero outside the image / past Cin) + weights ----
    float pv[C::NP];
    f4 wv[C::NW4], sv[C::NS4];
    auto load_chunk = [&](int ch) {
#pragma unroll
        for (int k = 0; k < C::NP; ++k) {
            const int e = tid + kDT * k;
            const int ci = e / (C::PR * C::PC), rem = e - ci * (C::PR * C::PC);
            const int r = rem / C::PC, c = rem - r * C::PC;
            const int gc = ch * kCK + ci, iy = iy0 + r, ix = ix0 + c;
            const bool in = e < kCK * C::PR * C::PC && gc < Cin && (unsigned)iy < (unsigned)p.H &&
                            (unsigned)ix < (unsigned)p.W;
            const float* src = gc < p.C0 ? p.x0 + ((size_t)b * p.C0 + gc) * HW
                                         : p.x1 + ((size_t)b * p.C1 + (gc - p.C0)) * HW;
            pv[k] = in ? src[iy * p.W + ix] : 0.f;
        }
        const f4* wg = reinterpret_cast<const f4*>(p.wpack + ((size_t)cls * nchunk + ch) * C::TAPS * kCK * COUT);
#pragma unroll
        for (int k = 0; k < C::NW4; ++k) {
            const int e = tid + kDT * k;
            if (e < C::TAPS * kCK * COUT / 4) wv[k] = wg[e];
        }
        if constexpr (SC) {
            const f4* sg = reinterpret_cast<const f4*>(p.wshort + (size_t)ch * kCK * COUT);
#pragma unroll
            for (int k = 0; k < C::NS4; ++k) {
                const int e = tid + kDT * k;
                if (e < kCK * COUT / 4) sv[k] = sg[e];
            }
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int k = 0; k < C::NP; ++k) {
            const int e = tid + kDT * k;
            if (e < kCK * C::PR * C::PC) {
                const int ci = e / (C::PR * C::PC), rem = e - ci * (C::PR * C::PC);
                const int r = rem / C::PC, c = rem - r * C::PC;
                lds[ci * C::PLANE + r * C::ROW + c] = pv[k];
            }
        }
#pragma unroll
        for (int k = 0; k < C::NW4; ++k) {
            const int e = tid + kDT * k;
            if (e < C::TAPS * kCK * COUT / 4) {
                const int row = e / (COUT / 4), c4 = e - row * (COUT / 4);
                *reinterpret_cast<f4*>(&lds[C::W_OFF + row * C::COP + 4 * c4]) = wv[k];
            }
        }
        if constexpr (SC) {
#pragma unroll
            for (int k = 0; k < C::NS4; ++k) {
                const int e = tid + kDT * k;
                if (e < kCK * COUT / 4) {
                    const int row = e / (COUT / 4), c4 = e - row * (COUT / 4);
                    *reinterpret_cast<f4*>(&lds[C::WS_OFF + row * C::COP + 4 * c4]) = sv[k];
                }
            }
        }
    };

    // ---- per-lane operand bases ----
    const int kk = lane >> 5, li = lane & 31;
    const int abase = C::W_OFF + kk * C::COP + li;               // + (tap*8 + 2p)*COP + mt*32
    const int sbase = C::WS_OFF + kk * C::COP + li;
    const int bbase = kk * C::PLANE + (w * C::RW * C::SP + (C::TR ? pa : 0)) * C::ROW + li * C::SP + (C::TR ? pb : 0);

    f16v acc[C::MT][C::RW], acs[SC ? C::MT : 1][SC ? C::RW : 1];
#pragma unroll
    for (int m = 0; m < C::MT; ++m)
#pragma unroll
        for (int r = 0; r < C::RW; ++r) {
            acc[m][r] = (f16v){};
            if constexpr (SC) acs[m][r] = (f16v){};
        }

    load_chunk(0);
#pragma unroll 1
    for (int ch = 0; ch < nchunk; ++ch) {
        if (ch) __syncthreads();  // the previous chunk's MFMAs are done with the LDS
        store_chunk();
        __syncthreads();
        load_chunk(ch + 1 < nchunk ? ch + 1 : ch);  // next chunk in flight during the MFMAs
        // taps one per iteration (not unrolled: unrolling all 9 x 4 k-steps lets the scheduler
        // hoist every operand read of the chunk into registers); the 4 channel pairs unrolled
#pragma unroll 1
        for (int t = 0; t < C::TAPS; ++t) {
            // patch offset of this tap: 3x3 / 1x1 (kh, kw); transposed: the parity class picks
            // rows (1 - tr) + pa and columns (1 - tc) + pb (pa, pb folded into bbase)
            const int dr = C::TR ? 1 - t / 2 : (C::KS == 3 ? t / 3 : 0);
            const int dc = C::TR ? 1 - t % 2 : (C::KS == 3 ? t % 3 : 0);
            const float* ap = lds + abase + t * kCK * C::COP;
            const float* bp = lds + bbase + dr * C::ROW + dc;
#pragma unroll
            for (int pp = 0; pp < kCK / 2; ++pp) {
                float av[C::MT], bv[C::RW];
#pragma unroll
                for (int m = 0; m < C::MT; ++m) av[m] = ap[2 * pp * C::COP + 32 * m];
#pragma unroll
                for (int r = 0; r < C::RW; ++r) bv[r] = bp[2 * pp * C::PLANE + r * C::SP * C::ROW];
#pragma unroll
                for (int m = 0; m < C::MT; ++m)
#pragma unroll
                    for (int r = 0; r < C::RW; ++r)
                        acc[m][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m], bv[r], acc[m][r], 0, 0, 0);
                if constexpr (SC) {
                    if (t == C::CENTER) {
#pragma unroll
                        for (int m = 0; m < C::MT; ++m) {
                            const float sa = lds[sbase + 2 * pp * C::COP + 32 * m];
#pragma unroll
                            for (int r = 0; r < C::RW; ++r)
                                acs[m][r] = __builtin_amdgcn_mfma_f32_32x32x2f32(sa, bv[r], acs[m][r], 0, 0, 0);
                        }
                    }
                }
            }
        }
    }

    // ---- epilogue: bias, ReLU, shortcut; C[row = co][col = pixel]: col = lane & 31,
    //      row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5) for register q ----
    const int Hc = C::TR ? p.Ho / 2 : p.Ho, Wc = C::TR ? p.Wo / 2 : p.Wo;  // (class) grid
    const int ox = ox0 + li;
#pragma unroll
    for (int r = 0; r < C::RW; ++r) {
        const int oy = oy0 + w * C::RW + r;
        if (oy >= Hc || ox >= Wc) continue;
        const int oyo = C::TR ? 2 * oy + pa : oy, oxo = C::TR ? 2 * ox + pb : ox;
#pragma unroll
        for (int m = 0; m < C::MT; ++m)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int co = 32 * m + (q & 3) + 8 * (q >> 2) + 4 * kk;
                if (co >= p.Cout) continue;
                float v = acc[m][r][q] + (p.bias ? p.bias[co] : 0.f);
                if (p.relu) v = fmaxf(v, 0.f);
                if constexpr (SC) v += acs[m][r][q];
                p.out[(((size_t)b * p.out_C + p.out_c0 + co) * p.Ho + oyo) * p.Wo + oxo] = v;
            }
    }
}

// ---- weight packing: (Cout, Cin, kh, kw) [conv] / (Cin, Cout, 4, 4) [transposed] ->
//      [class][chunk][tap][ci 8][Cout], times an optional per-Cout scale (eval BatchNorm) --------
__global__ __launch_bounds__(kDT) void dense_pack(int kind, int Cin, int Cout, const float* w, const float* scale,
                                                  float* wp) {
    const int taps = kind == NCONV_DENSE_3X3 ? 9 : (kind == NCONV_DENSE_1X1 ? 1 : 4);
    const int ncls = kind == NCONV_DENSE_TRANSPOSED_4X4 ? 4 : 1;
    const int nchunk = (Cin + kCK - 1) / kCK;
    const size_t n = (size_t)ncls * nchunk * taps * kCK * Cout;
    for (size_t e = (size_t)blockIdx.x * kDT + threadIdx.x; e < n; e += (size_t)gridDim.x * kDT) {
        const int co = (int)(e % Cout);
        size_t r = e / Cout;
        const int cil = (int)(r % kCK);
        r /= kCK;
        const int t = (int)(r % taps);
        r /= taps;
        const int ch = (int)(r % nchunk);
        const int cls = (int)(r / nchunk);
        const int ci = ch * kCK + cil;
        float v = 0.f;
        if (ci < Cin) {
            if (kind == NCONV_DENSE_3X3) {
                v = w[((size_t)co * Cin + ci) * 9 + t];
            } else if (kind == NCONV_DENSE_1X1) {
                v = w[(size_t)co * Cin + ci];
            } else {  // ConvTranspose2d weight (Cin, Cout, 4, 4): class (pa, pb), tap (tr, tc)
                const int pa = cls >> 1, pb = cls & 1, tr = t >> 1, tc = t & 1;
                const int kh = 1 - pa + 2 * tr, kw = 1 - pb + 2 * tc;
                v = w[(((size_t)ci * Cout + co) * 4 + kh) * 4 + kw];
            }
            if (scale) v *= scale[co];
        }
        wp[e] = v;
    }
}

// ---- 3x3 convolution to ONE output channel + residual (the depth heads, step2.py:259,278):
//      out = conv3x3(x, pad 1) + res. Thread = 4 adjacent pixels of a 16 x 64 tile; input
//      channels staged one plane at a time; weights are wave-uniform (SGPR). ---------------------
__global__ __launch_bounds__(kDT) void conv3x3_c1(const float* __restrict__ x, int Cin, int H, int W,
                                                 const float* __restrict__ wt, const float* __restrict__ res,
                                                 float* __restrict__ out, int ntx, int nty) {
    constexpr int TW = 64, TH = 16, PW = TW + 2, PH = TH + 2;
    __shared__ float pl[2][PH * PW];
    int blk = blockIdx.x;
    const int tx = blk % ntx;
    blk /= ntx;
    const int ty = blk % nty, b = blk / nty;
    const int tid = threadIdx.x;
    const int r = tid >> 4, c0 = (tid & 15) * 4;
    const int y0 = ty * TH, x0 = tx * TW;
    const size_t HW = (size_t)H * W;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    float st[(PH * PW + kDT - 1) / kDT];
    auto load = [&](int ci) {
#pragma unroll
        for (int k = 0; k < (PH * PW + kDT - 1) / kDT; ++k) {
            const int e = tid + kDT * k;
            const int pr = e / PW, pc = e - pr * PW;
            const int iy = y0 - 1 + pr, ix = x0 - 1 + pc;
            const bool in = e < PH * PW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
            st[k] = in ? x[((size_t)b * Cin + ci) * HW + (size_t)iy * W + ix] : 0.f;
        }
    };
    load(0);
#pragma unroll 1
    for (int ci = 0; ci < Cin; ++ci) {
        float* t = pl[ci & 1];
#pragma unroll
        for (int k = 0; k < (PH * PW + kDT - 1) / kDT; ++k) {
            const int e = tid + kDT * k;
            if (e < PH * PW) t[e] = st[k];
        }
        __syncthreads();
        load(ci + 1 < Cin ? ci + 1 : ci);
        const float* wr = wt + ci * 9;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            float v[6];
#pragma unroll
            for (int m = 0; m < 6; ++m) v[m] = t[(r + kh) * PW + c0 + m];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = fmaf(wr[kh * 3 + kw], v[j + kw], acc[j]);
        }
    }
    const int y = y0 + r;
    if (y >= H) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int xx = x0 + c0 + j;
        if (xx < W) {
            const size_t i = (size_t)b * HW + (size_t)y * W + xx;
            out[i] = acc[j] + (res ? res[i] : 0.f);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------------
size_t dense_packed_floats(int kind, int Cin, int Cout) {
    const int taps = kind == NCONV_DENSE_3X3 ? 9 : (kind == NCONV_DENSE_1X1 ? 1 : 4);
    const int ncls = kind == NCONV_DENSE_TRANSPOSED_4X4 ? 4 : 1;
    return (size_t)ncls * ((Cin + kCK - 1) / kCK) * taps * kCK * Cout;
}

int launch_dense_pack(int kind, int Cin, int Cout, const float* w, const float* scale, float* wp, hipStream_t st,
                      const char** why) {
    const size_t n = dense_packed_floats(kind, Cin, Cout);
    size_t blocks = (n + kDT - 1) / kDT;
    if (blocks > 4096) blocks = 4096;
    if (blocks) hipLaunchKernelGGL(dense_pack, dim3(blocks), dim3(kDT), 0, st, kind, Cin, Cout, w, scale, wp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

template <int COUT, int KIND, int S, bool SC>
static void go_dense(const nconv_dense_conv& p, hipStream_t st) {
    using C = DcCfg<COUT, KIND, S>;
    const int Hc = C::TR ? p.Ho / 2 : p.Ho, Wc = C::TR ? p.Wo / 2 : p.Wo;
    const int ntx = (Wc + C::TW - 1) / C::TW, nty = (Hc + C::TH - 1) / C::TH;
    const int blocks = ntx * nty * p.B * (C::TR ? 4 : 1);
    hipLaunchKernelGGL((dense_conv_mfma<COUT, KIND, S, SC>), dim3(blocks), dim3(kDT), 0, st, p, ntx, nty);
}

int launch_dense_conv(const nconv_dense_conv& p, hipStream_t st, const char** why) {
    const bool sc = p.wshort != nullptr;
    const int co = p.Cout <= 32 ? 32 : 64;
#define NCONV_DC(COUT_, KIND_, S_, SC_)                                                   \
    if (co == COUT_ && p.kind == KIND_ && p.stride == S_ && sc == SC_) {                  \
        go_dense<COUT_, KIND_, S_, SC_>(p, st);                                             \
        hipError_t e = hipGetLastError();                                                   \
        if (e != hipSuccess) {                                                              \
            *why = hipGetErrorString(e);                                                    \
            return -5;                                                                      \
        }                                                                                   \
        return 0;                                                                           \
    }
    NCONV_DC(32, NCONV_DENSE_3X3, 1, false)
    NCONV_DC(64, NCONV_DENSE_3X3, 1, false)
    NCONV_DC(32, NCONV_DENSE_3X3, 1, true)
    NCONV_DC(64, NCONV_DENSE_3X3, 1, true)
    NCONV_DC(32, NCONV_DENSE_3X3, 2, true)
    NCONV_DC(64, NCONV_DENSE_3X3, 2, true)
    NCONV_DC(32, NCONV_DENSE_3X3, 2, false)
    NCONV_DC(64, NCONV_DENSE_3X3, 2, false)
    NCONV_DC(32, NCONV_DENSE_1X1, 1, false)
    NCONV_DC(64, NCONV_DENSE_1X1, 1, false)
    NCONV_DC(32, NCONV_DENSE_1X1, 2, false)
    NCONV_DC(64, NCONV_DENSE_1X1, 2, false)
    NCONV_DC(32, NCONV_DENSE_TRANSPOSED_4X4, 2, false)
    NCONV_DC(64, NCONV_DENSE_TRANSPOSED_4X4, 2, false)
#undef NCONV_DC
    *why = "no dense-conv kernel for this (Cout, kind, stride, shortcut) combination";
    return -95;
}

int launch_conv3x3_c1(const float* x, int B, int Cin, int H, int W, const float* w, const float* res, float* out,
                      hipStream_t st, const char** why) {
    const int ntx = (W + 63) / 64, nty = (H + 15) / 16;
    hipLaunchKernelGGL(conv3x3_c1, dim3(ntx * nty * B), dim3(kDT), 0, st, x, Cin, H, W, w, res, out, ntx, nty);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
