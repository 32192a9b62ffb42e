// dense_conv.hip — dense convolutions of the RGB-guided model on the gfx950 matrix cores.
//
// The RGB encoder (models/step2.py:134-154) and the fusion decoder (step2.py:156-297) are plain
// K x C x R x S contractions, so they run as implicit GEMMs on v_mfma_f32_32x32x2_f32 (fp32 in,
// fp32 accumulate: exact f32 products, the precision of the reference's fp32 convolutions):
//   A = weights  [Cout][k]        (M = output channels, 32 or 64 per tile)
//   B = im2col   [k][pixel]       (N = 32 output columns of one output row)
//   k = (tap, input channel)      (K, input channels staged 8 at a time)
// A workgroup (4 waves) owns an output tile of TH rows x 32 columns x one output-channel tile of
// one image; each wave owns TH/4 rows. Per 8-channel chunk the input patch (with halo) and the
// chunk's packed weights are staged in LDS (loads for the next chunk issued before this chunk's
// MFMAs); an MFMA k-step pairs two input channels (lane half kk = lane >> 5 takes channel 2p + kk),
// so every operand read is one ds_read_b32 at a compile-time offset from a per-lane base. The
// epilogue applies bias (eval BatchNorm folded in by nconv_dense_pack), ReLU and the RGBEncoder
// 1x1 shortcut (computed from the centre tap of the same patch) and writes a channel range of the
// output tensor, so torch.cat of the decoder never materialises: convolutions write their half
// of the concatenated tensor and the next one reads two sources.
//
// Kinds: 3x3 pad 1 stride 1|2; 1x1 stride 1|2; ConvTranspose 4x4 stride 2 pad 1 as four
// output-parity classes, each a 2x2 gather over the input's 3x3 neighbourhood (output 2H or,
// cropped, 2H-1); Conv 4x4 stride 2 pad 1. Output channels are tiled by 32 or 64
// (dense_cout_tile), one tile per workgroup, so any Cout runs.
//
// Training (dense.py's autograd functions): the input gradient of every kind is this same kernel
// on re-arranged weights — 3x3 / 1x1 stride 1: transposed (+ flipped) kernel; stride 2: the
// transposed 4x4 convolution with the 3x3 / 1x1 kernel embedded; ConvTranspose 4x4: the 4x4 s2
// convolution with the same weights — and the weight gradient is dense_wgrad_mfma below.
#include "nconv_internal.h"

namespace nconv {

#ifndef NCONV_DENSE_TH32
#define NCONV_DENSE_TH32 1  // row multiplier of the 32-output-channel tiles (2: 8-12 % slower)
#endif
constexpr int kDT = 256;
constexpr int kCK = 8;  // input channels per staged chunk

__host__ __device__ constexpr int dense_taps(int kind) {
    return kind == NCONV_DENSE_3X3 ? 9 : kind == NCONV_DENSE_1X1 ? 1 : kind == NCONV_DENSE_TRANSPOSED_4X4 ? 4 : 16;
}

int dense_cout_tile(int Cout) {
    if (Cout <= 32) return 32;
    const int p32 = (Cout + 31) / 32 * 32, p64 = (Cout + 63) / 64 * 64;
    return p32 < p64 ? 32 : 64;  // less padding; ties: 64 (the patch is staged once, not twice)
}

template <int COUT, int KIND, int S>
struct DcCfg {
    static constexpr bool TR = KIND == NCONV_DENSE_TRANSPOSED_4X4;
    static constexpr int TAPS = dense_taps(KIND);
    static constexpr int SP = TR ? 1 : S;                 // patch stride
    static constexpr int KS = KIND == NCONV_DENSE_1X1 ? 1 : (KIND == NCONV_DENSE_CONV4X4_S2 ? 4 : 3);
    static constexpr int PAD = KIND == NCONV_DENSE_1X1 ? 0 : 1;
    // rows per wave: 4 (2 strided) with 32 output channels, 2 (1) with 64: 4 MFMAs per 4-5 LDS reads
    static constexpr int TH = (SP == 1 ? 8 : 4) * (COUT == 32 ? NCONV_DENSE_TH32 : 1), RW = TH / 4, TW = 32;
    static constexpr int PR = (TH - 1) * SP + KS, PC = (TW - 1) * SP + KS;
    static constexpr int ROW = PC;
    // B reads (ds_read_b32): 32 lanes on the columns of one patch row form one bank group, lane
    // half kk (the other group) the next channel plane, so the planes need no padding and the
    // patch image is the linear element order: element e of the chunk lands at lds[e].
    static constexpr int PLANE = PR * ROW;
    static constexpr int MT = COUT / 32;
    static constexpr int COP = COUT == 32 ? 32 : 96;      // A reads: kk * COP == 32 (mod 64)
    static constexpr int W_OFF = (kCK * PLANE + 3) & ~3;  // 16-byte aligned weight rows
    static constexpr int WS_OFF = W_OFF + TAPS * kCK * COP;  // shortcut weights [ci][COP]
    static constexpr int LDS = WS_OFF + kCK * COP;
    static constexpr int NP = (kCK * PR * PC + kDT - 1) / kDT;        // patch elements per thread
    static constexpr int NW4 = (TAPS * kCK * COUT / 4 + kDT - 1) / kDT;  // weight float4s per thread
    static constexpr int NS4 = (kCK * COUT / 4 + kDT - 1) / kDT;
    static constexpr int CENTER = KIND == NCONV_DENSE_3X3 ? 4 : 0;   // tap of the 1x1 shortcut
};

typedef float f16v __attribute__((ext_vector_type(16)));

template <int COUT, int KIND, int S, bool SC, bool STR = false>
__global__ __launch_bounds__(kDT) void dense_conv_mfma(nconv_dense_conv p, int ntx, int nty, int ncot) {
    using C = DcCfg<COUT, KIND, S>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int tx = blk % ntx;
    blk /= ntx;
    const int ty = blk % nty;
    blk /= nty;
    const int cot = blk % ncot;  // output-channel tile
    blk /= ncot;
    const int cls = C::TR ? blk % 4 : 0;  // output parity class (transposed)
    const int b = C::TR ? blk / 4 : blk;
    const int pa = cls >> 1, pb = cls & 1;
    const int oy0 = ty * C::TH, ox0 = tx * C::TW;  // tile origin (output grid, or class grid)
    const int iy0 = oy0 * C::SP - C::PAD, ix0 = ox0 * C::SP - C::PAD;  // patch origin in the input
    const int Cin = p.C0 + p.C1;
    const int nchunk = (Cin + kCK - 1) / kCK;
    const int HW = p.H * p.W;

    // ---- staging: patch (8 channels x PR x PC, zero outside the image / past Cin) + weights ----
    // Each thread's patch elements keep one byte offset each within a channel plane of the source
    // (out-of-image elements: past the buffer's end, read as 0), computed once; a chunk's loads are
    // buffer loads of that offset from a per-chunk resource (the chunk's first channel) -- no
    // address arithmetic per chunk. Channels past Cin read past the resource's end (0) as well.
    constexpr unsigned OOB = 0x80000000u;
    unsigned poff[C::NP];
#pragma unroll
    for (int k = 0; k < C::NP; ++k) {
        const int e = tid + kDT * k;
        const int ci = e / (C::PR * C::PC), rem = e - ci * (C::PR * C::PC);
        const int r = rem / C::PC, c = rem - r * C::PC;
        const int iy = iy0 + r, ix = ix0 + c;
        const bool in = e < kCK * C::PR * C::PC && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        poff[k] = in ? (unsigned)(ci * HW + iy * p.W + ix) * 4u : OOB;
    }
    const int bytes0 = p.C0 * HW * 4, bytes1 = p.C1 * HW * 4;
    float pv[C::NP], pv1[STR ? C::NP : 1];
    unsigned pshift = 0;
    f4 wv[C::NW4], sv[C::NS4];
    // Branch-free (a branch here made the compiler wait for the chunk's loads at the join, right
    // after issuing them, instead of behind the chunk's MFMAs): with STR == false (the host found
    // no chunk straddling the two sources) one load per element from a per-chunk resource chosen
    // by uniform selects; with STR, two loads per element, the wrong source's out of range.
    auto load_chunk = [&](int ch) {
        const int g0 = ch * kCK;  // first channel of the chunk
        if constexpr (!STR) {
            const bool a = g0 < p.C0;
            const float* base = a ? p.x0 + ((size_t)b * p.C0 + g0) * HW
                                  : p.x1 + ((size_t)b * p.C1 + (g0 - p.C0)) * HW;
            const int nbytes = a ? bytes0 - g0 * HW * 4 : bytes1 - (g0 - p.C0) * HW * 4;
            const __amdgpu_buffer_rsrc_t rs = plane_rsrc(base, nbytes);
#pragma unroll
            for (int k = 0; k < C::NP; ++k) pv[k] = ld_f32(rs, poff[k]);
        } else {  // a chunk may straddle the two sources: both loads, the wrong one out of range
            // x0's part: channels g0 .. C0-1 (none once g0 >= C0); x1's channel 0 sits at chunk
            // offset `shift` (negative once g0 > C0: the resource then starts at x1's channel g0 - C0)
            const bool a0 = g0 < p.C0;
            const __amdgpu_buffer_rsrc_t r0 = plane_rsrc(p.x0 + ((size_t)b * p.C0 + (a0 ? g0 : 0)) * HW,
                                                         a0 ? bytes0 - g0 * HW * 4 : 0);
            const int c1 = a0 ? 0 : g0 - p.C0;
            const __amdgpu_buffer_rsrc_t r1 = plane_rsrc(p.x1 + ((size_t)b * p.C1 + c1) * HW, bytes1 - c1 * HW * 4);
            const unsigned shift = a0 ? (unsigned)(p.C0 - g0) * HW * 4u : 0u;
            pshift = shift;  // the two values are selected at store time, not here (no wait)
#pragma unroll
            for (int k = 0; k < C::NP; ++k) {
                const bool in1 = poff[k] != OOB && poff[k] >= shift;
                pv[k] = ld_f32(r0, poff[k]);
                pv1[k] = ld_f32(r1, in1 ? poff[k] - shift : OOB);
            }
        }
        const f4* wg = reinterpret_cast<const f4*>(
            p.wpack + (((size_t)cls * ncot + cot) * nchunk + ch) * C::TAPS * kCK * COUT);
#pragma unroll
        for (int k = 0; k < C::NW4; ++k) {
            const int e = tid + kDT * k;
            if (e < C::TAPS * kCK * COUT / 4) wv[k] = wg[e];
        }
        if constexpr (SC) {
            const f4* sg = reinterpret_cast<const f4*>(p.wshort + ((size_t)cot * nchunk + ch) * kCK * COUT);
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
            float v = pv[k];
            if constexpr (STR) v = (poff[k] != OOB && poff[k] >= pshift) ? pv1[k] : v;
            if (e < kCK * C::PR * C::PC) lds[e] = v;
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
            // patch offset of this tap: (kh, kw); transposed: the parity class picks rows
            // (1 - tr) + pa and columns (1 - tc) + pb (pa, pb folded into bbase)
            const int dr = C::TR ? 1 - t / 2 : t / C::KS;
            const int dc = C::TR ? 1 - t % 2 : t % C::KS;
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
    //      row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5) for register q. Stores through one
    //      resource over the image's output channel range: the lane's byte offset (its pixel and
    //      lane-half channel) once, each register's channel offset a uniform soffset; pixels and
    //      channels outside the output are dropped by the range check ----
    const int Hc = C::TR ? p.H : p.Ho, Wc = C::TR ? p.W : p.Wo;  // (class) grid
    const int ox = ox0 + li;
    const int HWo = p.Ho * p.Wo;
    const int co0 = cot * COUT;  // first output channel of this tile
    const int nco = p.Cout - co0 < COUT ? p.Cout - co0 : COUT;
    const __amdgpu_buffer_rsrc_t ro =
        plane_rsrc(p.out + ((size_t)b * p.out_C + p.out_c0 + co0) * HWo, nco * HWo * 4);
#pragma unroll
    for (int r = 0; r < C::RW; ++r) {
        const int oy = oy0 + w * C::RW + r;
        const int oyo = C::TR ? 2 * oy + pa : oy, oxo = C::TR ? 2 * ox + pb : ox;
        const bool in = oy < Hc && ox < Wc && oyo < p.Ho && oxo < p.Wo;  // (cropped transposed output)
        const unsigned lo = in ? (unsigned)(4 * kk * HWo + oyo * p.Wo + oxo) * 4u : OOB;
#pragma unroll
        for (int m = 0; m < C::MT; ++m)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int cr = 32 * m + (q & 3) + 8 * (q >> 2);  // channel in the tile, lane half 0
                const int co = co0 + cr + 4 * kk;
                float v = acc[m][r][q] + ((p.bias && co < p.Cout) ? p.bias[co] : 0.f);
                if (p.relu) v = fmaxf(v, 0.f);
                if constexpr (SC) v += acs[m][r][q];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), ro, (int)lo, cr * HWo * 4, 0);
            }
    }
}

// ------------------------------------------------------------------------------------------------
// 3x3 stride-1 convolution with exact products on the bf16 matrix cores (NCONV_DENSE_MATH_BF16X9;
// NCONV_DENSE_MATH_BF16X6: the six largest partial products).
// Every fp32 operand v is split into three bf16 parts v = v0 + v1 + v2 (v0 = bf16(v),
// v1 = bf16(v - v0), v2 = v - v0 - v1: at most 8 significant bits, exact), so each of the nine
// partial products vi*wj is exact in fp32 and their sum is v*w exactly; the only rounding is the
// fp32 accumulation, as in the fp32-MFMA kernel above (which is an fmaf chain, bitwise; this one
// sums in another order, so results agree to fp32 accumulation error, not bitwise). Nine
// v_mfma_f32_32x32x16_bf16 (32 cycles each) per 32x32x16 block against eight
// v_mfma_f32_32x32x2_f32 (64 cycles each): 288 against 512 cycles.
// GEMM as above (A = weights, B = patch, C[co][pixel]), with k = (tap pair, 8 input channels): a
// k-step takes taps 2s (lane half 0) and 2s + 1 (lane half 1) of one 8-channel chunk; the tenth
// tap is zero (A rows zero, B fragment zeroed). LDS images, every fragment one ds_read_b128 of 32
// consecutive 16-byte entries:
//   patch   [part 3][position PR x PC][8 channels]         (bf16x8 per position and part)
//   weights [k-step 5][part 3][lane half 2][co COUT][8 ci]  (bf16x8 per row)
// ------------------------------------------------------------------------------------------------
typedef __bf16 dbf16x8 __attribute__((ext_vector_type(8)));

template <int COUT, int KIND = NCONV_DENSE_3X3, int S = 1, bool SC = false>
struct Db9Cfg {  // (16 rows for the 32-channel tiles, 2 waves/SIMD: not faster)
    static constexpr bool TR = KIND == NCONV_DENSE_TRANSPOSED_4X4;  // four output-parity classes
    static constexpr int TAPS = dense_taps(KIND), NKS = (TAPS + 1) / 2;  // k-steps: tap pairs
    static constexpr int KS = KIND == NCONV_DENSE_CONV4X4_S2 ? 4 : 3;    // patch extent per pixel
    static constexpr int SP = TR ? 1 : S;                            // patch stride
    static constexpr int TH = SP == 1 ? 8 : 4, RW = TH / 4, TW = 32, MT = COUT / 32;
    static constexpr int PR = (TH - 1) * SP + KS, PC = (TW - 1) * SP + KS, ROW = PC, NPOS = PR * PC;
    static constexpr int PLANEB = NPOS * 16;                         // bytes of one part's image
    static constexpr int DUMP = 3 * PLANEB;                          // slot of positions past the tile
    static constexpr int WOFF = DUMP + 3 * 16;                       // weight image (bytes)
    static constexpr int WROWS = NKS * 3 * 2 * COUT;                 // 16-byte rows per chunk
    static constexpr int NWL = (WROWS + kDT - 1) / kDT;              // rows per thread (the last
    static constexpr int SOFF = WOFF + NWL * kDT * 16;               //  round's excess: zeros, past the image)
    static constexpr int SROWS = SC ? 3 * 2 * COUT : 0;              // shortcut image rows per chunk
    static constexpr int NSL = (SROWS + kDT - 1) / kDT;
    static constexpr int LDSB = SOFF + NSL * kDT * 16;
    static constexpr int NPP = (NPOS + kDT - 1) / kDT;               // positions per thread
    // tap t's patch offset (row, column) from the pixel's patch origin (transposed: the parity
    // class's (pa, pb) added at run time)
    static constexpr int tr_(int t) { return TR ? 1 - t / 2 : t / KS; }
    static constexpr int tc_(int t) { return TR ? 1 - t % 2 : t % KS; }
    static constexpr int off(int t) { return tr_(t) * ROW + tc_(t); }
    // lane half 1's offset from lane half 0's in k-step s (the padded tenth tap of a 3x3: 0)
    static constexpr int delta(int s) { return 2 * s + 1 < TAPS ? off(2 * s + 1) - off(2 * s) : 0; }
};
typedef unsigned du4 __attribute__((ext_vector_type(4)));

// v (8 lanes) -> three bf16x8 parts summing to v exactly
__device__ __forceinline__ void dsplit3(const float (&v)[8], dbf16x8 (&o)[3]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 h0 = (__bf16)v[j];
        const float r1 = v[j] - (float)h0;
        const __bf16 h1 = (__bf16)r1;
        o[0][j] = h0;
        o[1][j] = h1;
        o[2][j] = (__bf16)(r1 - (float)h1);
    }
}

#ifndef NCONV_DB9_KUNROLL
#define NCONV_DB9_KUNROLL 5  // k-steps per unrolled body (1: 4 % slower)
#endif
#ifndef NCONV_DB9_S2
#define NCONV_DB9_S2 1  // stride-2 3x3 on the split-bf16 kernel
#endif
#ifndef NCONV_DB9_SC
#define NCONV_DB9_SC 1  // the fused 1x1 shortcut on the split-bf16 kernel
#endif
#ifndef NCONV_DB9_TR
#define NCONV_DB9_TR 1  // the transposed 4x4 and the 4x4 stride 2 on the split-bf16 kernel
#endif
#ifndef NCONV_WB9
#define NCONV_WB9 1  // the 3x3 weight gradient on the split-bf16 kernel
#endif
#ifndef NCONV_WB9_S2
#define NCONV_WB9_S2 1  // ... its stride-2 form too
#endif
#ifndef NCONV_DB9_WAVES64
#define NCONV_DB9_WAVES64 2
#endif
#ifndef NCONV_DB9_WAVES32
#define NCONV_DB9_WAVES32 3
#endif
template <int COUT, int NTERM, int KIND, int S, bool SC>
__global__ __launch_bounds__(kDT) __attribute__((amdgpu_waves_per_eu(COUT == 64 ? NCONV_DB9_WAVES64 : NCONV_DB9_WAVES32)))
void dense_conv_bf9(nconv_dense_conv p, int ntx, int nty, int ncot) {
    using C = Db9Cfg<COUT, KIND, S, SC>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDSB];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int tx = blk % ntx;
    blk /= ntx;
    const int ty = blk % nty;
    blk /= nty;
    const int cot = blk % ncot;
    blk /= ncot;
    const int cls = C::TR ? blk % 4 : 0;  // output parity class (transposed)
    const int b = C::TR ? blk / 4 : blk;
    const int pa = cls >> 1, pb = cls & 1;
    const int oy0 = ty * C::TH, ox0 = tx * C::TW;  // tile origin (output grid, or class grid)
    const int iy0 = oy0 * C::SP - 1, ix0 = ox0 * C::SP - 1;
    const int Cin = p.C0 + p.C1;
    const int nchunk = (Cin + kCK - 1) / kCK;
    const int HW = p.H * p.W;

    constexpr unsigned OOB = 0x80000000u;
    unsigned poff[C::NPP];
#pragma unroll
    for (int k = 0; k < C::NPP; ++k) {
        const int e = tid + kDT * k;
        const int r = e / C::PC, c = e - r * C::PC;
        const int iy = iy0 + r, ix = ix0 + c;
        const bool in = e < C::NPOS && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
        poff[k] = in ? (unsigned)(iy * p.W + ix) * 4u : OOB;
    }
    // each source's planes of image b behind one resource; a chunk's channel c comes from x0 or
    // x1 by a uniform select (a chunk may straddle the two), channels past Cin read past x1's end
    const __amdgpu_buffer_rsrc_t rs0 = plane_rsrc(p.x0 + (size_t)b * p.C0 * HW, p.C0 * HW * 4);
    const __amdgpu_buffer_rsrc_t rs1 =
        plane_rsrc(p.C1 > 0 ? p.x1 + (size_t)b * p.C1 * HW : p.x0, p.C1 > 0 ? p.C1 * HW * 4 : 0);
    // the pre-split weight image of (class, cot, chunk) behind the fp32 one (nconv_dense_pack)
    const size_t fp32_floats = (size_t)(C::TR ? 4 : 1) * ncot * nchunk * C::TAPS * kCK * COUT;
    const unsigned char* wimg = reinterpret_cast<const unsigned char*>(p.wpack + fp32_floats) +
                                ((size_t)cls * ncot + cot) * nchunk * C::WROWS * 16;
    // the shortcut's pre-split image (a 1x1 nconv_dense_pack: [cot][chunk][part][half][co], half 1 zero)
    const unsigned char* simg = SC ? reinterpret_cast<const unsigned char*>(p.wshort + (size_t)ncot * nchunk * kCK * COUT) +
                                         (size_t)cot * nchunk * C::SROWS * 16
                                   : nullptr;
    float pv[C::NPP][8];
    du4 wv[C::NWL], sv[SC ? C::NSL : 1];
    auto load_chunk = [&](int ch) {
        const int g0 = ch * kCK;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int g = g0 + c;
            const bool a = g < p.C0;
            const __amdgpu_buffer_rsrc_t rs = a ? rs0 : rs1;
            const int so = (a ? g : g - p.C0) * HW * 4;
#pragma unroll
            for (int k = 0; k < C::NPP; ++k) pv[k][c] = ld_f32s(rs, poff[k], so);
        }
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(wimg + (size_t)ch * C::WROWS * 16), (short)0, C::WROWS * 16, 0x00020000);
#pragma unroll
        for (int k = 0; k < C::NWL; ++k) wv[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, (tid + kDT * k) * 16, 0, 0);
        if constexpr (SC) {
            const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(simg + (size_t)ch * C::SROWS * 16), (short)0, C::SROWS * 16, 0x00020000);
#pragma unroll
            for (int k = 0; k < C::NSL; ++k) sv[k] = __builtin_amdgcn_raw_buffer_load_b128(rsc, (tid + kDT * k) * 16, 0, 0);
        }
    };
    auto store_chunk = [&](unsigned char* L) {
#pragma unroll
        for (int k = 0; k < C::NPP; ++k) {
            const int e = tid + kDT * k;
            dbf16x8 sp[3];
            dsplit3(pv[k], sp);
            const bool in = e < C::NPOS;  // past the tile: the dump slots (no branch)
            const int a = in ? e * 16 : C::DUMP, da = in ? C::PLANEB : 16;
#pragma unroll
            for (int i = 0; i < 3; ++i) *reinterpret_cast<dbf16x8*>(L + a + i * da) = sp[i];
        }
#pragma unroll
        for (int k = 0; k < C::NWL; ++k) *reinterpret_cast<du4*>(L + C::WOFF + (tid + kDT * k) * 16) = wv[k];
        if constexpr (SC) {
#pragma unroll
            for (int k = 0; k < C::NSL; ++k) *reinterpret_cast<du4*>(L + C::SOFF + (tid + kDT * k) * 16) = sv[k];
        }
    };

    const int kk = lane >> 5, li = lane & 31;
    const int abase = C::WOFF + (kk * COUT + li) * 16;
    const int sbase = C::SOFF + (kk * COUT + li) * 16;
    const int bbase = ((w * C::RW * C::SP + (C::TR ? pa : 0)) * C::ROW + li * C::SP + (C::TR ? pb : 0)) * 16;

    f16v acc[C::MT][C::RW], acs[SC ? C::MT : 1][SC ? C::RW : 1];
#pragma unroll
    for (int m = 0; m < C::MT; ++m)
#pragma unroll
        for (int r = 0; r < C::RW; ++r) {
            acc[m][r] = (f16v){};
            if constexpr (SC) acs[m][r] = (f16v){};
        }

    auto mma_chunk = [&](const unsigned char* L) {
#pragma unroll NCONV_DB9_KUNROLL
        for (int s = 0; s < C::NKS; ++s) {
            // lane half 0: tap 2s, lane half 1: tap 2s + 1 (C::delta(s) positions further)
            const int bb = bbase + (kk ? C::delta(s) * 16 : 0) + C::off(2 * s) * 16;
            dbf16x8 av[3][C::MT], bv[3][C::RW];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int m = 0; m < C::MT; ++m)
                    av[i][m] = *reinterpret_cast<const dbf16x8*>(L + abase + (s * 3 + i) * 2 * COUT * 16 + 32 * m * 16);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int r = 0; r < C::RW; ++r) {
                    bv[i][r] = *reinterpret_cast<const dbf16x8*>(L + bb + i * C::PLANEB + r * C::SP * C::ROW * 16);
                    if (2 * s + 1 == C::TAPS && kk) bv[i][r] = (dbf16x8){};  // the padded tap
                }
            // smallest terms first; NTERM 6 (bf16x6) drops the three below ~2^-23 |v w|
            constexpr int ti[9] = {2, 2, 1, 2, 1, 0, 1, 0, 0}, tj[9] = {2, 1, 2, 0, 1, 2, 0, 1, 0};
#pragma unroll
            for (int q = 9 - NTERM; q < 9; ++q)
#pragma unroll
                for (int m = 0; m < C::MT; ++m)
#pragma unroll
                    for (int r = 0; r < C::RW; ++r)
                        acc[m][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[ti[q]][m], bv[tj[q]][r], acc[m][r], 0, 0, 0);
            if constexpr (SC) {
                if (s == 2) {  // the 1x1 shortcut: the centre tap (lane half 0 of k-step 2; half 1's rows zero)
                    dbf16x8 as[3][C::MT];
#pragma unroll
                    for (int i = 0; i < 3; ++i)
#pragma unroll
                        for (int m = 0; m < C::MT; ++m)
                            as[i][m] = *reinterpret_cast<const dbf16x8*>(L + sbase + i * 2 * COUT * 16 + 32 * m * 16);
#pragma unroll
                    for (int q = 9 - NTERM; q < 9; ++q)
#pragma unroll
                        for (int m = 0; m < C::MT; ++m)
#pragma unroll
                            for (int r = 0; r < C::RW; ++r)
                                acs[m][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as[ti[q]][m], bv[tj[q]][r], acs[m][r], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // (two LDS images, the next chunk stored under this one's MFMAs with one barrier per chunk,
    // measured 7-13 % slower for the 32-channel tiles: two workgroups per CU instead of three)
    load_chunk(0);
#pragma unroll 1
    for (int ch = 0; ch < nchunk; ++ch) {
        store_chunk(lds);
        __syncthreads();
        load_chunk(ch + 1 < nchunk ? ch + 1 : ch);  // next chunk in flight during the MFMAs
        mma_chunk(lds);
        __syncthreads();  // this chunk's MFMAs are done with the LDS
    }
    const int Hc = C::TR ? p.H : p.Ho, Wc = C::TR ? p.W : p.Wo;  // (class) grid
    const int ox = ox0 + li;
    const int HWo = p.Ho * p.Wo;
    const int co0 = cot * COUT;
    const int nco = p.Cout - co0 < COUT ? p.Cout - co0 : COUT;
    const __amdgpu_buffer_rsrc_t ro = plane_rsrc(p.out + ((size_t)b * p.out_C + p.out_c0 + co0) * HWo, nco * HWo * 4);
#pragma unroll
    for (int r = 0; r < C::RW; ++r) {
        const int oy = oy0 + w * C::RW + r;
        const int oyo = C::TR ? 2 * oy + pa : oy, oxo = C::TR ? 2 * ox + pb : ox;
        const bool in = oy < Hc && ox < Wc && oyo < p.Ho && oxo < p.Wo;  // (cropped transposed output)
        const unsigned lo = in ? (unsigned)(4 * kk * HWo + oyo * p.Wo + oxo) * 4u : OOB;
#pragma unroll
        for (int m = 0; m < C::MT; ++m)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int cr = 32 * m + (q & 3) + 8 * (q >> 2);
                const int co = co0 + cr + 4 * kk;
                float v = acc[m][r][q] + ((p.bias && co < p.Cout) ? p.bias[co] : 0.f);
                if (p.relu) v = fmaxf(v, 0.f);
                if constexpr (SC) v += acs[m][r][q];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), ro, (int)lo, cr * HWo * 4, 0);
            }
    }
}

// ---- weight packing: (Cout, Cin, kh, kw) [conv] / (Cin, Cout, 4, 4) [transposed] ->
//      [class][cout tile][chunk][tap][ci 8][T], times an optional per-Cout scale (eval
//      BatchNorm); channels past Cin / Cout are zero ----------------------------------------------
// 3x3: one wave per (output-channel tile, input chunk, 8 output channels): their 8 x 8 x 9
// weights (72 contiguous floats per output channel) read coalesced into LDS, then both images'
// entries of those channels written from there (32-byte / 128-byte runs)
template <int T>
__global__ __launch_bounds__(64) void dense_pack3x3(int Cin, int Cout, const float* w, const float* scale,
                                                    float* wp) {
    constexpr int G = 8;  // output channels per wave
    __shared__ float wt[G * 73];
    const int nchunk = (Cin + kCK - 1) / kCK, ncot = (Cout + T - 1) / T;
    int blk = blockIdx.x;
    const int sub = blk % (T / G);
    blk /= T / G;
    const int ch = blk % nchunk, cot = blk / nchunk;
    const int tid = threadIdx.x, c0 = sub * G;
    float v[G * 72 / 64], sc[G * 72 / 64];  // all loads in flight together
#pragma unroll
    for (int k = 0; k < G * 72 / 64; ++k) {
        const int e = tid + 64 * k, col = e / 72, rem = e - col * 72;
        const int o = cot * T + c0 + col, ci = ch * kCK + rem / 9;
        const bool in = o < Cout && ci < Cin;
        v[k] = in ? w[((size_t)o * Cin + ch * kCK) * 9 + rem] : 0.f;
        sc[k] = in && scale ? scale[o] : 1.f;
    }
#pragma unroll
    for (int k = 0; k < G * 72 / 64; ++k) {
        const int e = tid + 64 * k, col = e / 72, rem = e - col * 72;
        wt[col * 73 + rem] = v[k] * sc[k];
    }
    __syncthreads();
    float* f = wp + ((size_t)cot * nchunk + ch) * 9 * kCK * T;  // [tap][ci][T]
    for (int e = tid; e < 72 * G; e += 64) {
        const int col = e % G, r = e / G, cil = r % kCK, t = r / kCK;
        f[r * T + c0 + col] = wt[col * 73 + cil * 9 + t];
    }
    unsigned char* img = reinterpret_cast<unsigned char*>(wp + (size_t)ncot * nchunk * 9 * kCK * T) +
                         ((size_t)cot * nchunk + ch) * 30 * T * 16;
    for (int e = tid; e < 30 * G; e += 64) {
        const int col = e % G, r = e / G, kk = r % 2, part = (r / 2) % 3, s = r / 6, tap = 2 * s + kk;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = tap < 9 ? wt[col * 73 + c * 9 + tap] : 0.f;
        dbf16x8 sp[3];
        dsplit3(v, sp);
        *reinterpret_cast<dbf16x8*>(img + ((size_t)r * T + c0 + col) * 16) = part == 0 ? sp[0] : part == 1 ? sp[1] : sp[2];
    }
}

// the other kinds: one thread per element of the fp32 image
__global__ __launch_bounds__(kDT) void dense_pack(int kind, int Cin, int Cout, int T, const float* w,
                                                  const float* scale, float* wp) {
    const int taps = dense_taps(kind);
    const int ncls = kind == NCONV_DENSE_TRANSPOSED_4X4 ? 4 : 1;
    const int nchunk = (Cin + kCK - 1) / kCK;
    const int ncot = (Cout + T - 1) / T;
    const size_t n = (size_t)ncls * ncot * nchunk * taps * kCK * T;
    for (size_t e = (size_t)blockIdx.x * kDT + threadIdx.x; e < n; e += (size_t)gridDim.x * kDT) {
        const int col = (int)(e % T);
        size_t r = e / T;
        const int cil = (int)(r % kCK);
        r /= kCK;
        const int t = (int)(r % taps);
        r /= taps;
        const int ch = (int)(r % nchunk);
        r /= nchunk;
        const int cot = (int)(r % ncot);
        const int cls = (int)(r / ncot);
        const int ci = ch * kCK + cil, co = cot * T + col;
        float v = 0.f;
        if (ci < Cin && co < Cout) {
            if (kind == NCONV_DENSE_3X3) {
                v = w[((size_t)co * Cin + ci) * 9 + t];
            } else if (kind == NCONV_DENSE_1X1) {
                v = w[(size_t)co * Cin + ci];
            } else if (kind == NCONV_DENSE_CONV4X4_S2) {
                v = w[((size_t)co * Cin + ci) * 16 + t];
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
//      channels staged NCONV_C1_CB planes per barrier (the next group's loads in flight during
//      this group's FMAs; the sums in the same channel order as one plane at a time, bitwise);
//      weights are wave-uniform (SGPR). ---------------------------------------------------------
#ifndef NCONV_C1_CB
#define NCONV_C1_CB 4
#endif
__global__ __launch_bounds__(kDT) void conv3x3_c1(const float* __restrict__ x, int Cin, int H, int W,
                                                 const float* __restrict__ wt, const float* __restrict__ res,
                                                 float* __restrict__ out, int ntx, int nty) {
    constexpr int TW = 64, TH = 16, PW = TW + 2, PH = TH + 2, CB = NCONV_C1_CB;
    constexpr int NE = (PH * PW + kDT - 1) / kDT;
    __shared__ float pl[2][CB][PH * PW];
    int blk = blockIdx.x;
    const int tx = blk % ntx;
    blk /= ntx;
    const int ty = blk % nty, b = blk / nty;
    const int tid = threadIdx.x;
    const int r = tid >> 4, c0 = (tid & 15) * 4;
    const int y0 = ty * TH, x0 = tx * TW;
    const size_t HW = (size_t)H * W;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    float st[CB][NE];
    unsigned off[NE];  // each staged element's offset in its plane (0x80000000: outside, reads 0)
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int e = tid + kDT * k;
        const int pr = e / PW, pc = e - pr * PW;
        const int iy = y0 - 1 + pr, ix = x0 - 1 + pc;
        const bool in = e < PH * PW && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        off[k] = in ? (unsigned)(iy * W + ix) * 4u : 0x80000000u;
    }
    const __amdgpu_buffer_rsrc_t rx = plane_rsrc(x + (size_t)b * Cin * HW, (int)(Cin * HW * 4));
    auto load = [&](int c) {  // channels c .. c + CB - 1 (past Cin: out of range, 0)
#pragma unroll
        for (int q = 0; q < CB; ++q)
#pragma unroll
            for (int k = 0; k < NE; ++k) st[q][k] = ld_f32s(rx, off[k], (c + q) * (int)HW * 4);
    };
    load(0);
#pragma unroll 1
    for (int cg = 0; cg < Cin; cg += CB) {
        float(*t)[PH * PW] = pl[(cg / CB) & 1];
#pragma unroll
        for (int q = 0; q < CB; ++q)
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const int e = tid + kDT * k;
                if (e < PH * PW) t[q][e] = st[q][k];
            }
        __syncthreads();
        load(cg + CB < Cin ? cg + CB : cg);
#pragma unroll
        for (int q = 0; q < CB; ++q) {
            if (cg + q >= Cin) break;
            const float* wr = wt + (cg + q) * 9;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                float v[6];
#pragma unroll
                for (int m = 0; m < 6; ++m) v[m] = t[q][(r + kh) * PW + c0 + m];
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[j] = fmaf(wr[kh * 3 + kw], v[j + kw], acc[j]);
            }
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
// Weight gradients (training):  gW[m][n] = sum over images and pixels p of
//     D[m][p] * P[n / TAPS][patch(p, n % TAPS)]
//   Conv2d 3x3 pad 1 / 1x1, stride S:  pixels = output grid, D = dL/dy (m = co),
//       P = the input x (n = ci*TAPS + kh*KS + kw) at (oy*S + kh - PAD, ox*S + kw - PAD);
//   ConvTranspose2d 4x4 s2 p1:         pixels = input grid, D = the input x (m = ci),
//       P = dL/dy (n = co*16 + kh*4 + kw) at (2 iy - 1 + kh, 2 ix - 1 + kw)
// so gW's own layout (Conv2d (Cout, Cin, k, k) / ConvTranspose2d (Cin, Cout, 4, 4)) is [m][n].
// Implicit GEMM on v_mfma_f32_32x32x2_f32 with K = pixels (2 per MFMA). The (M, N) plane is cut
// into groups of one 32-row m-tile x NT 32-column n-tiles (NT x 32 columns = whole input
// channels: 32 x 9 taps, 16 x 16 taps, 64 x 1); a workgroup owns GM x GN groups (D rows and
// patch channels staged once for all of them) and walks a contiguous range of TH x 32 pixel
// tiles. Wave w takes group w % (GM GN) on the pixels of its row share (1/4, 1/2 or all of the
// tile), so every wave does the same MFMA work and every loaded byte feeds up to 4 waves. Per
// tile, D and the patch planes are staged in LDS with buffer loads (the next tile's loads in
// flight during the MFMAs); pixel q = q0 + 2j + kk of k-step j sits at a compile-time offset
// from a per-wave base. Each wave writes its partial [32][NT*32] to slice ks * RG + row-group;
// dense_wgrad_reduce adds the slices in a fixed order (deterministic, no float atomics).
// ------------------------------------------------------------------------------------------------
// pixel tile rows of the weight gradient: 4 x 32, 2 x 32 where the strided patch is tall (3x3 s2,
// transposed). (8 x 32 for the stride-1 3x3 with one m-tile per workgroup measured 1-2 % slower:
// profiles/r5_ab_dense_wgrad_tall_tiles.log)
__host__ __device__ constexpr int wgd_th(int kind, int s, int) {
    return (kind == NCONV_DENSE_TRANSPOSED_4X4 || (kind == NCONV_DENSE_3X3 && s == 2)) ? 2 : 4;
}
__host__ __device__ constexpr int wgd_ntb(int kind) {
    return kind == NCONV_DENSE_3X3 ? 9 : (kind == NCONV_DENSE_1X1 ? 2 : 8);
}
// column tiles per group for a GEMM of N columns: wgd_ntb, or 1 when N fits one tile
// (the 1- and 3-channel inputs of depth_conv / rgb_encoder0, a 1x1 of <= 32 channels)
constexpr int wgd_nt(int kind, int N) { return N <= 32 ? 1 : wgd_ntb(kind); }

template <int KIND, int S, int NT, int GM, int GN>
struct WgdCfg {
    static constexpr bool TR = KIND == NCONV_DENSE_TRANSPOSED_4X4;
    static constexpr int TAPS = KIND == NCONV_DENSE_3X3 ? 9 : (KIND == NCONV_DENSE_1X1 ? 1 : 16);
    static constexpr int KS = KIND == NCONV_DENSE_3X3 ? 3 : (KIND == NCONV_DENSE_1X1 ? 1 : 4);
    static constexpr int NCOLS = 32 * NT;  // columns per group
    // patch channels per group: whole channels (wgd_ntb), or every channel a one-tile group may touch
    static constexpr int CPG = NCOLS % TAPS == 0 ? NCOLS / TAPS : (NCOLS - 1) / TAPS + 2;
    static constexpr int CPB = GN * CPG;   // patch channels staged per workgroup
    static constexpr int GB = GM * GN, RG = 4 / GB;  // groups per workgroup, row-groups (waves per group)
    // pixel tile: wgd_th x 32
    static constexpr int TH = wgd_th(KIND, S, GM), TW = 32, NPX = TH * TW;
    static constexpr int PPW = NPX / RG;   // pixels per wave per tile (a multiple of 16)
    // patch geometry: LDS step between neighbouring pixels (1x1 stages only the sampled
    // positions), global step between neighbouring LDS columns, patch origin = pixel * OS - PAD
    static constexpr int LS = KIND == NCONV_DENSE_1X1 ? 1 : (TR ? 2 : S);
    static constexpr int GS = KIND == NCONV_DENSE_1X1 ? S : 1;
    static constexpr int OS = TR ? 2 : S;
    static constexpr int PAD = KIND == NCONV_DENSE_1X1 ? 0 : 1;
    static constexpr int PR = (TH - 1) * LS + KS, PC = (TW - 1) * LS + KS;
    static constexpr int PPLANE = PR * PC;
    static constexpr int DP = NPX + 2;     // D row pitch: rows m, m+1 two banks apart
    static constexpr int D_OFF = (CPB * PPLANE + 3) & ~3;
    static constexpr int BUF = (D_OFF + GM * 32 * DP + 3) & ~3;  // one tile's staging (patch, then D)
    static constexpr int LDS = BUF > 4 * 16 * 64 ? BUF : 4 * 16 * 64;  // (+ the wave-partial sums)
    static constexpr int NDE = GM * 32 * NPX / kDT;  // D elements per thread
    static constexpr int NPG = (CPG * PPLANE + kDT - 1) / kDT;  // patch elements per thread and group
    static_assert(PPW % 16 == 0 && (GM * 32 * NPX) % kDT == 0, "wave / thread shares");
};

struct WgdArgs {
    const float* d0;
    const float* d1;
    int dC0, dC1;  // direct operand: M = dC0 + dC1 channels on the pixel grid
    int Hp, Wp;    // pixel grid
    const float* p0;
    const float* p1;
    int pC0, pC1;  // patch operand channels
    int Hs, Ws;    // patch source planes
    int M, N;      // N = (pC0 + pC1) * TAPS
    int ntx, nty, nbm, nbn, nks;  // tiles; workgroup groups along M and N; K slices
    long long ntiles;
};

template <int KIND, int S, int NT, int GM, int GN>
__global__ __launch_bounds__(kDT) void dense_wgrad_mfma(WgdArgs a, float* __restrict__ part) {
    using C = WgdCfg<KIND, S, NT, GM, GN>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int bn = blk % a.nbn;
    blk /= a.nbn;
    const int bm = blk % a.nbm, ks = blk / a.nbm;
    const int m0 = bm * GM * 32, n0 = bn * GN * C::NCOLS;  // the workgroup's first row / column
    const int Cp = a.pC0 + a.pC1;
    const int c_lo = n0 / C::TAPS;
    const long long t0 = a.ntiles * ks / a.nks, t1 = a.ntiles * (ks + 1) / a.nks;
    const size_t HWp = (size_t)a.Hp * a.Wp, HWs = (size_t)a.Hs * a.Ws;
    static_assert(GN == 1 || C::NCOLS % C::TAPS == 0, "groups of whole channels");

    // this wave's group (m-tile gmi, n-group gni) and pixel share [q0, q0 + PPW) of each tile
    const int gi = w % C::GB, rg = w / C::GB;
    const int gmi = gi % GM, gni = gi / GM;
    const int q0 = rg * C::PPW;
    const int kk = lane >> 5, li = lane & 31;
    const int abase = C::D_OFF + (gmi * 32 + li) * C::DP + kk;  // + q
    int bbase[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        const int nl = gni * C::NCOLS + 32 * u + li;  // column within the workgroup
        const int ci = nl / C::TAPS, tap = nl % C::TAPS;
        const int kh = tap / C::KS, kw = tap % C::KS;
        bbase[u] = ci * C::PPLANE + kh * C::PC + kw + kk * C::LS;  // + r*LS*PC + c*LS
    }

    f16v acc[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = (f16v){};

    // Staging loads are buffer loads: the image's planes sit behind one SGPR resource per
    // source, elements outside the image / channel range carry an offset past it and read 0
    // (no per-element masks or 64-bit addresses live across the load latency). The patch is
    // staged group by group, so the source of a group's channels is wave-uniform whenever the
    // concatenation boundary is a multiple of 32 channels (16 for the transposed kernel) — every
    // concatenation of the guided model; otherwise that group reads each element from both
    // sources (one out of range) and adds them.
    constexpr unsigned OOB = 0x80000000u;
    // LDS-DMA staging (buffer_load ... lds): every staged element goes from HBM straight into its
    // LDS slot -- no staging registers, so the weight-gradient accumulators (NT x 16 per lane) and
    // the rest fit two waves per SIMD, and one workgroup's loads hide behind the other's MFMAs.
    // A wave's 64 elements of one load are consecutive in the LDS image (the DMA writes wave base
    // + lane x 4): the patch planes are unpadded and a D row (NPX >= 64 pixels) never splits a wave.
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    auto glds = [&](__amdgpu_buffer_rsrc_t r, float* dst, unsigned off) __attribute__((always_inline)) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 4, off, 0, 0, 0);
    };
    const int wb = 64 * w;  // the wave's first element of each load
    // Per-block constants of the staging (the element -> LDS slot map is the same for every tile):
    // each patch element's byte offset from its tile's patch origin (channel plane included;
    // 0x80000000 for the channels past the input, which then reads 0 whatever the tile), and each
    // D element's pixel offset. An interior tile then costs one add per element; tiles touching
    // the image border take the general path with per-element bounds.
    constexpr unsigned OOB_REL = 0x80000000u;
    unsigned prel[GN][C::NPG];
    bool gwhole[GN];  // the group's channels come from one source
#pragma unroll
    for (int g = 0; g < GN; ++g) {
        const int gc0 = c_lo + g * C::CPG;
        const bool hi = a.p1 != nullptr && gc0 >= a.pC0;
        gwhole[g] = !(a.p1 != nullptr && gc0 < a.pC0 && gc0 + C::CPG > a.pC0);
        const int cb = hi ? a.pC0 : 0;
#pragma unroll
        for (int k = 0; k < C::NPG; ++k) {
            const int e = tid + kDT * k;
            const int ci = e / C::PPLANE, rem = e % C::PPLANE;
            const int r = rem / C::PC, c = rem % C::PC;
            prel[g][k] = (gc0 + ci < Cp && e < C::CPG * C::PPLANE)
                             ? ((unsigned)(gc0 + ci - cb) * (unsigned)HWs + (unsigned)(r * C::GS * a.Ws + c * C::GS)) * 4u
                             : OOB_REL;
        }
    }
    const int dq = tid % C::NPX;
    const unsigned drel = (unsigned)((dq / C::TW) * a.Wp + dq % C::TW) * 4u;
    // the block's tiles walk (tx, ty, b) in order from t0
    int tx_c = (int)(t0 % a.ntx), ty_c = (int)((t0 / a.ntx) % a.nty), b_c = (int)(t0 / ((long long)a.ntx * a.nty));
    auto stage = [&](int tx, int ty, int b, float* lds) __attribute__((always_inline)) {
        int tq = tid;
        asm volatile("" : "+v"(tq));
        const int py0 = ty * C::TH, px0 = tx * C::TW;
        const int iy0 = py0 * C::OS - C::PAD, ix0 = px0 * C::OS - C::PAD;
        const bool dfull = py0 + C::TH <= a.Hp && px0 + C::TW <= a.Wp;
        const bool pfull = iy0 >= 0 && ix0 >= 0 && iy0 + (C::PR - 1) * C::GS < a.Hs && ix0 + (C::PC - 1) * C::GS < a.Ws;
        {
            unsigned ob;
            if (dfull) {
                ob = (unsigned)(py0 * a.Wp + px0) * 4u + drel;
            } else {
                const int py = py0 + dq / C::TW, px = px0 + dq % C::TW;
                ob = (py < a.Hp && px < a.Wp) ? (unsigned)(py * a.Wp + px) * 4u : OOB;
            }
            const __amdgpu_buffer_rsrc_t rd0 = plane_rsrc(a.d0 + (size_t)b * a.dC0 * HWp, (int)(a.dC0 * HWp * 4));
            const __amdgpu_buffer_rsrc_t rd1 =
                plane_rsrc(a.d1 ? a.d1 + (size_t)b * a.dC1 * HWp : a.d0, (int)((a.d1 ? a.dC1 : 0) * HWp * 4));
            const int mw = __builtin_amdgcn_readfirstlane(m0 + tid / C::NPX);  // NPX >= 64: per wave
#pragma unroll
            for (int k = 0; k < C::NDE; ++k) {
                const int m = mw + (kDT / C::NPX) * k;
                const bool s1 = m >= a.dC0;
                const int mm = s1 ? m - a.dC0 : m;
                const unsigned off = (m < a.M && ob != OOB) ? (unsigned)(mm * HWp) * 4u + ob : OOB;
                const int e0 = wb + kDT * k;
                glds(s1 ? rd1 : rd0, lds + C::D_OFF + (e0 / C::NPX) * C::DP + e0 % C::NPX, off);
            }
        }
        const __amdgpu_buffer_rsrc_t rp0 = plane_rsrc(a.p0 + (size_t)b * a.pC0 * HWs, (int)(a.pC0 * HWs * 4));
        const __amdgpu_buffer_rsrc_t rp1 =
            plane_rsrc(a.p1 ? a.p1 + (size_t)b * a.pC1 * HWs : a.p0, (int)((a.p1 ? a.pC1 : 0) * HWs * 4));
        const unsigned pbase = (unsigned)(iy0 * a.Ws + ix0) * 4u;  // used by interior tiles only
#pragma unroll
        for (int g = 0; g < GN; ++g) {
            const int gc0 = c_lo + g * C::CPG;
            const bool hi = a.p1 != nullptr && gc0 >= a.pC0;
            const int cb = hi ? a.pC0 : 0;
            const __amdgpu_buffer_rsrc_t rp = hi ? rp1 : rp0;
            if (pfull && gwhole[g]) {
#pragma unroll
                for (int k = 0; k < C::NPG; ++k)
                    if ((k + 1) * kDT <= C::CPG * C::PPLANE || tq + kDT * k < C::CPG * C::PPLANE)
                        glds(rp, lds + g * C::CPG * C::PPLANE + wb + kDT * k, pbase + prel[g][k]);
                continue;
            }
#pragma unroll
            for (int k = 0; k < C::NPG; ++k) {
                const int e = tq + kDT * k;
                if ((k + 1) * kDT <= C::CPG * C::PPLANE || e < C::CPG * C::PPLANE) {
                    const int ci = e / C::PPLANE, rem = e % C::PPLANE;
                    const int r = rem / C::PC, c = rem % C::PC;
                    const int gc = gc0 + ci, iy = iy0 + r * C::GS, ix = ix0 + c * C::GS;
                    const bool ok = gc < Cp && (unsigned)iy < (unsigned)a.Hs && (unsigned)ix < (unsigned)a.Ws;
                    const unsigned pix = (unsigned)(iy * a.Ws + ix);
                    float* dst = lds + g * C::CPG * C::PPLANE + wb + kDT * k;
                    if (gwhole[g]) {
                        glds(rp, dst, ok ? ((unsigned)(gc - cb) * (unsigned)HWs + pix) * 4u : OOB);
                    } else if (gc < a.pC0) {  // the group's channels come from both sources: each lane one
                        glds(rp0, dst, ok ? ((unsigned)gc * (unsigned)HWs + pix) * 4u : OOB);
                    } else {
                        glds(rp1, dst, ok ? ((unsigned)(gc - a.pC0) * (unsigned)HWs + pix) * 4u : OOB);
                    }
                }
            }
        }
    };

    auto next_tile = [&]() __attribute__((always_inline)) {
        if (++tx_c == a.ntx) {
            tx_c = 0;
            if (++ty_c == a.nty) {
                ty_c = 0;
                ++b_c;
            }
        }
    };
    // one buffer: the loads of one workgroup hide behind the MFMAs of the CU's other workgroup (a
    // double-buffered single workgroup per CU measured slower, 704.6 against 614.0 us for the
    // 32-channel 3x3: profiles/r5_ab_dense_wgrad_db.log; removed in round 6)
#pragma unroll 1
    for (long long t = t0; t < t1; ++t) {
        const float* lb = lds;
        __syncthreads();  // the previous tile's MFMAs are done with the LDS
        stage(tx_c, ty_c, b_c, lds);
        next_tile();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the wave's pixels in segments of 16 (8 k-steps) inside one tile row
#pragma unroll 1
        for (int sg = 0; sg < C::PPW / 16; ++sg) {
            const int q = q0 + 16 * sg, r = q / C::TW, c = q % C::TW;
            const int aoff = abase + q, boff = r * C::LS * C::PC + c * C::LS;
#pragma unroll 2
            for (int j = 0; j < 8; ++j) {
                const float av = lb[aoff + 2 * j];
#pragma unroll
                for (int u = 0; u < NT; ++u) {
                    const float bv = lb[bbase[u] + boff + 2 * j * C::LS];
                    acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[u], 0, 0, 0);
                }
            }
        }
    }

    // ---- the block's partial [GM*32][GN*NT*32] -> slice ks: C[row = m][col = n]. The RG waves of
    //      a group hold the same tile over different pixels: summed here in LDS (fixed order, one
    //      n-tile at a time), so the block writes one slice, not RG (RG x less partial traffic
    //      for dense_wgrad_reduce) ----
    float* out = part + (size_t)ks * a.M * a.N;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        __syncthreads();  // the LDS is free (after the MFMAs / the previous tile)
#pragma unroll
        for (int q = 0; q < 16; ++q) lds[(w * 16 + q) * 64 + lane] = acc[u][q];
        __syncthreads();
        for (int e = tid; e < C::GB * 1024; e += kDT) {
            const int g2 = e >> 10, q = (e >> 6) & 15, l = e & 63;
            float v = lds[(g2 * 16 + q) * 64 + l];
#pragma unroll
            for (int r2 = 1; r2 < C::RG; ++r2) v += lds[((g2 + C::GB * r2) * 16 + q) * 64 + l];
            const int n = n0 + (g2 / GM) * C::NCOLS + 32 * u + (l & 31);
            const int m = m0 + (g2 % GM) * 32 + (q & 3) + 8 * (q >> 2) + 4 * (l >> 5);
            if (n < a.N && m < a.M) out[(size_t)m * a.N + n] = v;
        }
    }
}

// gw[e] = sum over the nsl slices of part[slice][e]: 64 elements x 4 slice phases per block,
// each phase summing every 4th slice in order, the phases combined in a fixed order.
__global__ __launch_bounds__(kDT) void dense_wgrad_reduce(const float* __restrict__ part, int nsl, int mn,
                                                          float* __restrict__ gw) {
    __shared__ float red[4][64];
    const int col = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + col;
    float s = 0.f;
    if (e < mn) {
#pragma unroll 8
        for (int k = ph; k < nsl; k += 4) s += part[(size_t)k * mn + e];
    }
    red[ph][col] = s;
    __syncthreads();
    if (ph == 0 && e < mn) gw[e] = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
}

// dense_wgrad_reduce over fp64 partials (dense_wgrad_tr_rows), summed in fp64, rounded once.
__global__ __launch_bounds__(kDT) void dense_wgrad_reduce_d(const double* __restrict__ part, int nsl, int mn,
                                                            float* __restrict__ gw) {
    __shared__ double red[4][64];
    const int col = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + col;
    double s = 0.0;
    if (e < mn) {
#pragma unroll 8
        for (int k = ph; k < nsl; k += 4) s += part[(size_t)k * mn + e];
    }
    red[ph][col] = s;
    __syncthreads();
    if (ph == 0 && e < mn) gw[e] = (float)(((red[0][col] + red[1][col]) + red[2][col]) + red[3][col]);
}

// ---- the transposed convolution's weight-gradient rows of the few channels concatenated beside
//      whole 32-channel groups (UpCat's depth channel and 32 / 64 features, step2.py:173) ----
// On the matrix cores those rows would take a whole 32-row m-tile each (M = 33 / 65 padded to 64 /
// 96: half or a third of the tile work wasted); here they are a GEMV on the vector ALU that
// streams dL/dy once:
//   out[j][co*16 + kh*4 + kw] = sum over (b, oy, ox) with oy + 1 - kh, ox + 1 - kw even of
//       gy[b][co][oy][ox] * x1[b][j][(oy + 1 - kh) / 2][(ox + 1 - kw) / 2]
// Each dL/dy element meets two kernel rows (kh of its row parity) and two columns. Workgroup =
// one channel co of one image over a 16-row x 256-column block of dL/dy: thread = column, its 16
// rows read coalesced, the x1 window (10 rows x 130 columns per channel) staged in LDS; the 16
// tap sums of the workgroup reduced over its threads in a fixed order into its partial slot
// part[slice][co * 16 + tap], slice = (image, row block, column block); dense_wgrad_reduce adds
// the slices in a fixed order (deterministic).
constexpr int kTrRows = 16, kTrCols = 256;
constexpr int kTrXH = kTrRows / 2 + 2, kTrXW = kTrCols / 2 + 2;  // x1 window
constexpr int kTrMaxC1 = 2, kTrMaxG = 6;                          // channels; Cout <= 16 * kTrMaxG
__global__ __launch_bounds__(256) void dense_wgrad_tr_rows(const float* __restrict__ x1, int C1, int H, int W,
                                                           const float* __restrict__ gy, int Cout, int Ho, int Wo,
                                                           int nry, int nrx, double* __restrict__ part) {
    __shared__ float sx[kTrMaxC1 * kTrXH * kTrXW];
    __shared__ double red[4][kTrMaxC1 * 16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int blk = blockIdx.x;
    const int co = blk % Cout;
    blk /= Cout;
    const int rx = blk % nrx;
    blk /= nrx;
    const int ry = blk % nry, b = blk / nry;
    const int oy0 = ry * kTrRows, ox0 = rx * kTrCols;
    const int iy0 = oy0 / 2 - 1, ix0 = ox0 / 2 - 1;
    for (int e = tid; e < C1 * kTrXH * kTrXW; e += 256) {
        const int j = e / (kTrXH * kTrXW), r = (e / kTrXW) % kTrXH, c = e % kTrXW;
        const int iy = iy0 + r, ix = ix0 + c;
        sx[e] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? x1[(((size_t)b * C1 + j) * H + iy) * W + ix]
                                                                         : 0.f;
    }
    const int ox = ox0 + tid;
    float gv[kTrRows];
    const float* gp = gy + (((size_t)b * Cout + co) * Ho + oy0) * Wo + ox;
#pragma unroll
    for (int r = 0; r < kTrRows; ++r) gv[r] = (ox < Wo && oy0 + r < Ho) ? gp[(size_t)r * Wo] : 0.f;
    __syncthreads();
    // this column's two kernel columns (kw of the parity of ox + 1) and their x1 columns
    const int kwa = (ox + 1) & 1;                  // kw in {kwa, kwa + 2}
    const int xca = (ox + 1 - kwa) / 2 - ix0;      // x1 column of kw = kwa; kw = kwa + 2: xca - 1
    // acc[j][kh][i]: kernel column kw = kwa + 2 i (the thread's column parity; kh is the row's,
    // known per unrolled row since the block's first row is even). Exact products summed in fp64,
    // the partials kept in fp64 down to the final reduction: dL/dy of the BatchNorm after this
    // convolution has zero mean per channel while the depth channel has a large mean (0..80 m), so
    // the sum is a small difference of large terms -- in fp32 its rounding reached 1.4e-3 of the
    // largest gradient (golden f9, fuse1.upcat.upf.conv.weight; the reference's own: 5e-6)
    double acc[kTrMaxC1][4][2];
#pragma unroll
    for (int j = 0; j < kTrMaxC1; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[j][t][0] = acc[j][t][1] = 0.0;
#pragma unroll
    for (int r = 0; r < kTrRows; ++r) {
        const int kha = (r + 1) & 1;                    // oy0 even: kh in {kha, kha + 2}
        const int xra = (oy0 + r + 1 - kha) / 2 - iy0;  // x1 row of kh = kha; kh = kha + 2: xra - 1
#pragma unroll
        for (int j = 0; j < kTrMaxC1; ++j) {
            if (j >= C1) continue;
            const float* xs = sx + j * kTrXH * kTrXW;
            const float x00 = xs[xra * kTrXW + xca], x01 = xs[xra * kTrXW + xca - 1];
            const float x10 = xs[(xra - 1) * kTrXW + xca], x11 = xs[(xra - 1) * kTrXW + xca - 1];
            const double g = (double)gv[r];
            acc[j][kha][0] = __builtin_fma(g, (double)x00, acc[j][kha][0]);
            acc[j][kha][1] = __builtin_fma(g, (double)x01, acc[j][kha][1]);
            acc[j][kha + 2][0] = __builtin_fma(g, (double)x10, acc[j][kha + 2][0]);
            acc[j][kha + 2][1] = __builtin_fma(g, (double)x11, acc[j][kha + 2][1]);
        }
    }
    // the workgroup's 16 (x C1) tap sums: wave butterflies, then the four waves in order
#pragma unroll
    for (int j = 0; j < kTrMaxC1; ++j) {
        if (j >= C1) continue;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int kh = t >> 2, kw = t & 3;
            double v = (kw & 1) == kwa ? acc[j][kh][kw >> 1] : 0.0;
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m);
            if (lane == 0) red[wv][j * 16 + t] = v;
        }
    }
    __syncthreads();
    if (tid < C1 * 16) {
        const int j = tid >> 4, t = tid & 15;
        const size_t slice = ((size_t)b * nry + ry) * nrx + rx;
        part[(slice * C1 + j) * (size_t)(Cout * 16) + co * 16 + t] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient of the 3x3 stride-1 convolution on the bf16 matrix cores (split-bf16 maths):
//   gW[co][ci][tap] = sum over pixels p of D[co][p] * X[ci][p + tap]
// as nine GEMMs C_tap[co][ci] (M = 32 output channels, N = 32 input channels, K = pixels) on
// v_mfma_f32_32x32x16_bf16, both operands split into three bf16 parts (nine or six terms, as the
// forward). A = D[co][16 pixels]: 8 consecutive pixels per lane half, one ds_read_b128 of a
// [part][co][pixel] image. B = X[16 pixels + tap][ci]: the patch image is channel-innermost
// ([part][position][32 channels]), so a lane's 8 pixels of one channel are a column of it, read
// with two ds_read_b64_tr_b16 (4 rows x 16 channels per 16-lane group, delivered column-major):
// the tap shift moves whole 64-byte rows, so every address stays aligned (pixel-contiguous
// images would put 7 of 9 taps' fragments off the 16-byte alignment ds_read_b128 needs).
// Tiles, split-K slices and the partial layout are dense_wgrad_mfma<3x3, 1, 9, 1, 1>'s: a workgroup
// owns 32 output channels x 32 input channels x 9 taps and walks a contiguous range of 4 x 32
// pixel tiles; wave w takes tile row w; the four waves' tiles are summed in LDS in a fixed order
// and the block writes one slice (dense_wgrad_reduce adds the slices in a fixed order).
// ------------------------------------------------------------------------------------------------
typedef short dv4s __attribute__((ext_vector_type(4)));
typedef short dv8s __attribute__((ext_vector_type(8)));
template <int S>
struct Wb9 {  // tiles as dense_wgrad_mfma's: 4 x 32 pixels (stride 2: 2 x 32, its patch is twice as wide)
    static constexpr int TH = S == 1 ? 4 : 2, TW = 32, NPX = TH * TW;
    static constexpr int PR = (TH - 1) * S + 3, PC = (TW - 1) * S + 3, NPOS = PR * PC;
    static constexpr int PPW = NPX / 4, NKW = PPW / 16;  // pixels and 16-pixel k-steps per wave
    static constexpr int NDI = 32 * NPX / 8 / kDT;      // D items (channel, 8 pixels) per thread
    static constexpr int PPART = NPOS * 64;          // bytes of one part's patch image (32 channels)
    static constexpr int PDUMP = 3 * PPART;          // slots of positions past the patch
    static constexpr int DB = NPX * 2 + 16;          // bytes per D row (16-byte pad: conflict-free A reads)
    static constexpr int DOFF = PDUMP + 64;
    static constexpr int DPART = 32 * DB;
    static constexpr int LDSB = DOFF + 3 * DPART;    // (the epilogue reuses the first 16 KB)
    static constexpr int NPW = (NPOS + 63) / 64;     // positions per lane (wave = one 8-channel group)
};

template <int NTERM, int S>
__global__ __launch_bounds__(kDT, 2) void dense_wgrad_bf9(WgdArgs a, float* __restrict__ part) {
    using C = Wb9<S>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDSB];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int blk = blockIdx.x;
    const int bn = blk % a.nbn;
    blk /= a.nbn;
    const int bm = blk % a.nbm, ks = blk / a.nbm;
    const int m0 = bm * 32, c_lo = bn * 32;  // first output channel, first input channel
    const int Cp = a.pC0 + a.pC1;
    const long long t0 = a.ntiles * ks / a.nks, t1 = a.ntiles * (ks + 1) / a.nks;
    const int HWp = a.Hp * a.Wp, HWs = a.Hs * a.Ws;
    constexpr unsigned OOB = 0x80000000u;

    // staging registers: wave w stages input channels c_lo + 8w .. + 7 at NPW positions per lane,
    // and 2 (output channel, 8-pixel segment) items of D per thread
    float xv[C::NPW][8], dv[C::NDI][8];
    int tx_c = (int)(t0 % a.ntx), ty_c = (int)((t0 / a.ntx) % a.nty), b_c = (int)(t0 / ((long long)a.ntx * a.nty));
    auto load_tile = [&](int tx, int ty, int b) {
        const int py0 = ty * C::TH, px0 = tx * C::TW, iy0 = py0 * S - 1, ix0 = px0 * S - 1;
        const __amdgpu_buffer_rsrc_t rp0 = plane_rsrc(a.p0 + (size_t)b * a.pC0 * HWs, a.pC0 * HWs * 4);
        const __amdgpu_buffer_rsrc_t rp1 =
            plane_rsrc(a.pC1 > 0 ? a.p1 + (size_t)b * a.pC1 * HWs : a.p0, a.pC1 > 0 ? a.pC1 * HWs * 4 : 0);
        unsigned po[C::NPW];
#pragma unroll
        for (int k = 0; k < C::NPW; ++k) {
            const int pos = lane + 64 * k, r = pos / C::PC, c = pos - r * C::PC;
            const int iy = iy0 + r, ix = ix0 + c;
            po[k] = pos < C::NPOS && (unsigned)iy < (unsigned)a.Hs && (unsigned)ix < (unsigned)a.Ws
                        ? (unsigned)(iy * a.Ws + ix) * 4u : OOB;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ci = c_lo + 8 * w + j;  // wave-uniform
            const bool s0 = ci < a.pC0;
            const __amdgpu_buffer_rsrc_t rs = s0 ? rp0 : rp1;
            const int so = (s0 ? ci : ci - a.pC0) * HWs * 4;  // past Cp: out of range, reads 0
#pragma unroll
            for (int k = 0; k < C::NPW; ++k) xv[k][j] = ld_f32s(rs, po[k], so);
        }
        const __amdgpu_buffer_rsrc_t rd = plane_rsrc(a.d0 + (size_t)b * a.dC0 * HWp, a.dC0 * HWp * 4);
#pragma unroll
        for (int k = 0; k < C::NDI; ++k) {
            const int it = tid + kDT * k, col = it / (C::NPX / 8), seg = it % (C::NPX / 8);
            const int py = py0 + (seg >> 2), px = px0 + (seg & 3) * 8, co = m0 + col;
            const bool ok = co < a.M && py < a.Hp;
            const unsigned base = (unsigned)(co * HWp + py * a.Wp + px) * 4u;
#pragma unroll
            for (int j = 0; j < 8; ++j) dv[k][j] = ld_f32(rd, ok && px + j < a.Wp ? base + 4u * j : OOB);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int k = 0; k < C::NPW; ++k) {
            const int pos = lane + 64 * k;
            dbf16x8 sp[3];
            dsplit3(xv[k], sp);
            const bool in = pos < C::NPOS;
            const int at = in ? pos * 64 + w * 16 : C::PDUMP + w * 16, da = in ? C::PPART : 0;
#pragma unroll
            for (int i = 0; i < 3; ++i) *reinterpret_cast<dbf16x8*>(lds + at + i * da) = sp[i];
        }
#pragma unroll
        for (int k = 0; k < C::NDI; ++k) {
            const int it = tid + kDT * k, col = it / (C::NPX / 8), seg = it % (C::NPX / 8);
            dbf16x8 sp[3];
            dsplit3(dv[k], sp);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                *reinterpret_cast<dbf16x8*>(lds + C::DOFF + i * C::DPART + col * C::DB + seg * 16) = sp[i];
        }
    };
    auto next_tile = [&]() {
        if (++tx_c == a.ntx) {
            tx_c = 0;
            if (++ty_c == a.nty) {
                ty_c = 0;
                ++b_c;
            }
        }
    };

    const int kk = lane >> 5, li = lane & 31;
    const int g = lane >> 4, il = lane & 15, q = il >> 2, pq = il & 3;
    // the wave's pixels: tile row prow, columns pcol0 .. + PPW - 1
    const int prow = w * C::PPW / C::TW, pcol0 = w * C::PPW % C::TW;
    // A: D row li, pixels (the k-step's 16) + 8 kk
    const int abase = C::DOFF + li * C::DB + (w * C::PPW + 8 * kk) * 2;
    // B (transposed reads): block row q = pixel 8 kk + 4 h + q of the k-step (patch column S x its
    // column), channels 16 (g & 1) + 4 pq .. + 3
    const int bbase = (prow * S * C::PC + (pcol0 + 8 * kk + q) * S) * 64 + (16 * (g & 1) + 4 * pq) * 2;

    f16v acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = (f16v){};
    typedef __attribute__((address_space(3))) dv4s* lds4_t;
    auto trd = [&](int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t)(lds + off)); };

    if (t0 < t1) load_tile(tx_c, ty_c, b_c);
#pragma unroll 1
    for (long long t = t0; t < t1; ++t) {
        store_tile();
        next_tile();
        __syncthreads();
        if (t + 1 < t1) load_tile(tx_c, ty_c, b_c);  // the next tile's loads in flight during the MFMAs
#pragma unroll
        for (int s2 = 0; s2 < C::NKW; ++s2) {  // the wave's 16-pixel k-steps
            dbf16x8 av[3];
#pragma unroll
            for (int i = 0; i < 3; ++i)
                av[i] = *reinterpret_cast<const dbf16x8*>(lds + abase + i * C::DPART + s2 * 32);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int kh = tap / 3, kw = tap % 3;
                const int bo = bbase + (kh * C::PC + s2 * 16 * S + kw) * 64;
                dbf16x8 bv[3];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const dv4s lo = trd(bo + i * C::PPART), hi = trd(bo + i * C::PPART + 4 * S * 64);
                    const dv8s v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    bv[i] = __builtin_bit_cast(dbf16x8, v);
                }
                constexpr int ti[9] = {2, 2, 1, 2, 1, 0, 1, 0, 0}, tj[9] = {2, 1, 2, 0, 1, 2, 0, 1, 0};
#pragma unroll
                for (int qq = 9 - NTERM; qq < 9; ++qq)
                    acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[ti[qq]], bv[tj[qq]], acc[tap], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();  // this tile's MFMAs are done with the LDS
    }

    // ---- the four waves' C_tap summed in LDS (fixed order), one slice per block: C[row = co][col = ci],
    //      col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) for register r ----
    float* lf = reinterpret_cast<float*>(lds);
    float* out = part + (size_t)ks * a.M * a.N;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) lf[(w * 16 + r) * 64 + lane] = acc[tap][r];
        __syncthreads();
        for (int e = tid; e < 1024; e += kDT) {
            const int r = (e >> 6) & 15, l = e & 63;
            const float v = ((lf[r * 64 + l] + lf[(16 + r) * 64 + l]) + lf[(32 + r) * 64 + l]) + lf[(48 + r) * 64 + l];
            const int co = m0 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), ci = c_lo + (l & 31);
            if (co < a.M && ci < Cp) out[(size_t)co * a.N + ci * 9 + tap] = v;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------------
static size_t dense_fp32_floats(int kind, int Cin, int Cout) {
    const int ncls = kind == NCONV_DENSE_TRANSPOSED_4X4 ? 4 : 1;
    const int T = dense_cout_tile(Cout);
    return (size_t)ncls * ((Cout + T - 1) / T) * ((Cin + kCK - 1) / kCK) * dense_taps(kind) * kCK * T;
}
// the fp32 image, then dense_conv_bf9's pre-split one: rows of 8 bf16 (16 bytes) in
// [class][cot][chunk][k-step][part][half][co] order, NKS k-steps of two taps (a padded odd tap and
// the 1x1's second half zero): 6 NKS T rows = 24 NKS T floats per (class, cot, chunk)
static size_t dense_bf9_floats(int kind, int Cin, int Cout) {
    const int ncls = kind == NCONV_DENSE_TRANSPOSED_4X4 ? 4 : 1;
    const int T = dense_cout_tile(Cout), nks = (dense_taps(kind) + 1) / 2;
    return (size_t)ncls * ((Cout + T - 1) / T) * ((Cin + kCK - 1) / kCK) * 24 * nks * T;
}

// the pre-split image of the other kinds (1x1, transposed 4x4, 4x4 stride 2), one row per thread
// (3x3: dense_pack3x3); values as dense_pack's, then split
__global__ __launch_bounds__(kDT) void dense_pack_bf9(int kind, int Cin, int Cout, int T, const float* w,
                                                      const float* scale, unsigned char* img, size_t rows) {
    const int taps = dense_taps(kind), nks = (taps + 1) / 2;
    const int nchunk = (Cin + kCK - 1) / kCK, ncot = (Cout + T - 1) / T;
    for (size_t e = (size_t)blockIdx.x * kDT + threadIdx.x; e < rows; e += (size_t)gridDim.x * kDT) {
        const int col = (int)(e % T);
        size_t r = e / T;
        const int kk = (int)(r % 2);
        r /= 2;
        const int part = (int)(r % 3);
        r /= 3;
        const int s = (int)(r % nks);
        r /= nks;
        const int ch = (int)(r % nchunk);
        r /= nchunk;
        const int cot = (int)(r % ncot), cls = (int)(r / ncot);
        const int t = 2 * s + kk, co = cot * T + col;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int ci = ch * kCK + c;
            float x = 0.f;
            if (t < taps && ci < Cin && co < Cout) {
                if (kind == NCONV_DENSE_1X1) {
                    x = w[(size_t)co * Cin + ci];
                } else if (kind == NCONV_DENSE_CONV4X4_S2) {
                    x = w[((size_t)co * Cin + ci) * 16 + t];
                } else {  // ConvTranspose2d weight (Cin, Cout, 4, 4): class (pa, pb), tap (tr, tc)
                    const int pa = cls >> 1, pb = cls & 1, tr = t >> 1, tc = t & 1;
                    x = w[(((size_t)ci * Cout + co) * 4 + (1 - pa + 2 * tr)) * 4 + (1 - pb + 2 * tc)];
                }
                if (scale) x *= scale[co];
            }
            v[c] = x;
        }
        dbf16x8 sp[3];
        dsplit3(v, sp);
        *reinterpret_cast<dbf16x8*>(img + e * 16) = part == 0 ? sp[0] : part == 1 ? sp[1] : sp[2];
    }
}
size_t dense_packed_floats(int kind, int Cin, int Cout) {
    return dense_fp32_floats(kind, Cin, Cout) + dense_bf9_floats(kind, Cin, Cout);
}

int launch_dense_pack(int kind, int Cin, int Cout, const float* w, const float* scale, float* wp, hipStream_t st,
                      const char** why) {
    if (kind == NCONV_DENSE_3X3) {
        const int T = dense_cout_tile(Cout);
        const int nb = ((Cout + T - 1) / T) * ((Cin + kCK - 1) / kCK) * (T / 8);
        if (T == 32)
            hipLaunchKernelGGL(dense_pack3x3<32>, dim3(nb), dim3(64), 0, st, Cin, Cout, w, scale, wp);
        else
            hipLaunchKernelGGL(dense_pack3x3<64>, dim3(nb), dim3(64), 0, st, Cin, Cout, w, scale, wp);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            *why = hipGetErrorString(e);
            return -5;
        }
        return 0;
    }
    const size_t n = dense_fp32_floats(kind, Cin, Cout);
    size_t blocks = (n + kDT - 1) / kDT;
    if (blocks > 4096) blocks = 4096;
    if (blocks)
        hipLaunchKernelGGL(dense_pack, dim3(blocks), dim3(kDT), 0, st, kind, Cin, Cout, dense_cout_tile(Cout), w,
                           scale, wp);
    if (const size_t rows = dense_bf9_floats(kind, Cin, Cout) / 4) {
        size_t b9 = (rows + kDT - 1) / kDT;
        if (b9 > 4096) b9 = 4096;
        hipLaunchKernelGGL(dense_pack_bf9, dim3(b9), dim3(kDT), 0, st, kind, Cin, Cout, dense_cout_tile(Cout), w,
                           scale, reinterpret_cast<unsigned char*>(wp + n), rows);
    }
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
    const int Hc = C::TR ? p.H : p.Ho, Wc = C::TR ? p.W : p.Wo;
    const int ntx = (Wc + C::TW - 1) / C::TW, nty = (Hc + C::TH - 1) / C::TH;
    const int ncot = (p.Cout + COUT - 1) / COUT;
    const int blocks = ntx * nty * ncot * p.B * (C::TR ? 4 : 1);
    if (p.C1 > 0 && p.C0 % kCK != 0)  // a chunk holds channels of both sources
        hipLaunchKernelGGL((dense_conv_mfma<COUT, KIND, S, SC, true>), dim3(blocks), dim3(kDT), 0, st, p, ntx, nty,
                           ncot);
    else
        hipLaunchKernelGGL((dense_conv_mfma<COUT, KIND, S, SC, false>), dim3(blocks), dim3(kDT), 0, st, p, ntx,
                           nty, ncot);
}

// p.math BF16X9 / BF16X6: every kind but the 1x1 (3x3 stride 1 or 2 with or without the fused
// shortcut, the transposed 4x4 and the 4x4 stride 2) on dense_conv_bf9; the 1x1 (half of each
// k-step would be padding) keeps the fp32 MFMA kernel
template <int COUT, int NTERM, int KIND, int S, bool SC>
static void go_dense_bf9(const nconv_dense_conv& p, hipStream_t st) {
    using C = Db9Cfg<COUT, KIND, S, SC>;
    const int Hc = C::TR ? p.H : p.Ho, Wc = C::TR ? p.W : p.Wo;
    const int ntx = (Wc + C::TW - 1) / C::TW, nty = (Hc + C::TH - 1) / C::TH;
    const int ncot = (p.Cout + COUT - 1) / COUT;
    hipLaunchKernelGGL((dense_conv_bf9<COUT, NTERM, KIND, S, SC>), dim3(ntx * nty * ncot * p.B * (C::TR ? 4 : 1)),
                       dim3(kDT), 0, st, p, ntx, nty, ncot);
}
template <int COUT, int NTERM>
static void go_dense_bf9_k(const nconv_dense_conv& p, bool sc, hipStream_t st) {
    if (p.kind == NCONV_DENSE_TRANSPOSED_4X4)
        go_dense_bf9<COUT, NTERM, NCONV_DENSE_TRANSPOSED_4X4, 2, false>(p, st);
    else if (p.kind == NCONV_DENSE_CONV4X4_S2)
        go_dense_bf9<COUT, NTERM, NCONV_DENSE_CONV4X4_S2, 2, false>(p, st);
    else if (p.stride == 1)
        sc ? go_dense_bf9<COUT, NTERM, NCONV_DENSE_3X3, 1, true>(p, st) : go_dense_bf9<COUT, NTERM, NCONV_DENSE_3X3, 1, false>(p, st);
    else
        sc ? go_dense_bf9<COUT, NTERM, NCONV_DENSE_3X3, 2, true>(p, st) : go_dense_bf9<COUT, NTERM, NCONV_DENSE_3X3, 2, false>(p, st);
}

int launch_dense_conv(const nconv_dense_conv& p, hipStream_t st, const char** why) {
    const bool sc = p.wshort != nullptr;
    const int co = dense_cout_tile(p.Cout);
    const bool bf9_kind = p.kind == NCONV_DENSE_3X3 ? (p.stride == 1 || NCONV_DB9_S2) && (!sc || NCONV_DB9_SC)
                                                   : p.kind != NCONV_DENSE_1X1 && NCONV_DB9_TR;
    if (p.math != NCONV_DENSE_MATH_FP32 && bf9_kind) {
        const int nt = p.math == NCONV_DENSE_MATH_BF16X9 ? 9 : 6;
        if (co == 32)
            nt == 9 ? go_dense_bf9_k<32, 9>(p, sc, st) : go_dense_bf9_k<32, 6>(p, sc, st);
        else
            nt == 9 ? go_dense_bf9_k<64, 9>(p, sc, st) : go_dense_bf9_k<64, 6>(p, sc, st);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            *why = hipGetErrorString(e);
            return -5;
        }
        return 0;
    }
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
    NCONV_DC(32, NCONV_DENSE_CONV4X4_S2, 2, false)
    NCONV_DC(64, NCONV_DENSE_CONV4X4_S2, 2, false)
#undef NCONV_DC
    *why = "no dense-conv kernel for this (kind, stride, shortcut) combination";
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

// ---- weight gradient ----
struct WgdPlan {
    WgdArgs a;
    int nt, gm, gn, rg;
    bool bf9;  // dense_wgrad_bf9
};
// the split-bf16 weight gradient: 3x3 (stride 1 or 2) with 32-channel x 9-tap n-groups (Cin >= 4)
static bool wgrad_bf9(const nconv_dense_wgrad& g, int nt) {
    return g.math != NCONV_DENSE_MATH_FP32 && g.kind == NCONV_DENSE_3X3 && nt == 9 && (g.stride == 1 || NCONV_WB9_S2) &&
           NCONV_WB9;
}

static WgdPlan wgrad_plan(const nconv_dense_wgrad& g) {
    WgdPlan pl{};
    WgdArgs& a = pl.a;
    const int cin = g.C0 + g.C1;
    const bool tr = g.kind == NCONV_DENSE_TRANSPOSED_4X4;
    if (!tr) {  // Conv2d: D = dL/dy, patch = x
        a.d0 = g.gy;
        a.d1 = nullptr;
        a.dC0 = g.Cout;
        a.dC1 = 0;
        a.Hp = g.Ho;
        a.Wp = g.Wo;
        a.p0 = g.x0;
        a.p1 = g.x1;
        a.pC0 = g.C0;
        a.pC1 = g.C1;
        a.Hs = g.H;
        a.Ws = g.W;
        a.M = g.Cout;
        a.N = cin * dense_taps(g.kind);
    } else {  // ConvTranspose2d: D = x, patch = dL/dy
        a.d0 = g.x0;
        a.d1 = g.x1;
        a.dC0 = g.C0;
        a.dC1 = g.C1;
        a.Hp = g.H;
        a.Wp = g.W;
        a.p0 = g.gy;
        a.p1 = nullptr;
        a.pC0 = g.Cout;
        a.pC1 = 0;
        a.Hs = g.Ho;
        a.Ws = g.Wo;
        a.M = cin;
        a.N = g.Cout * 16;
    }
    pl.nt = wgd_nt(g.kind, a.N);
    const int nmg = (a.M + 31) / 32, nng = (a.N + 32 * pl.nt - 1) / (32 * pl.nt);
    // groups per workgroup: pairs along M and N where they divide evenly; the strided 3x3
    // stages tall patches, so it pairs along M only; dense_wgrad_bf9 takes one m-tile
    pl.bf9 = wgrad_bf9(g, pl.nt);
    pl.gm = (pl.nt > 1 && nmg % 2 == 0 && !pl.bf9) ? 2 : 1;
    // (LDS-DMA staging: one n-group per workgroup, so two workgroups fit a CU's LDS)
    pl.gn = 1;
    pl.rg = 4 / (pl.gm * pl.gn);
    const int th = wgd_th(g.kind, g.stride, pl.gm);
    a.ntx = (a.Wp + 31) / 32;
    a.nty = (a.Hp + th - 1) / th;
    a.ntiles = (long long)g.B * a.ntx * a.nty;
    a.nbm = nmg / pl.gm;
    a.nbn = nng / pl.gn;
    long long nks = 512 / (a.nbm * a.nbn);  // two workgroups per CU
    if (nks < 1) nks = 1;
    if (nks > a.ntiles) nks = a.ntiles;
    a.nks = (int)nks;
    return pl;
}

// The transposed kind with one source of a few channels beside one of whole 32-channel groups:
// the matrix cores take the large source's rows, dense_wgrad_tr_rows the small one's
// (NCONV_WGD_TR_ROWS=0: all on the matrix cores). Returns 0 (no split), 1 (x1 small), 2 (x0 small).
static int tr_rows_split(const nconv_dense_wgrad& g) {
    const char* e = getenv("NCONV_WGD_TR_ROWS");
    if ((e && e[0] == '0') || g.kind != NCONV_DENSE_TRANSPOSED_4X4 || !g.x1 || g.C0 <= 0 || g.C1 <= 0 ||
        g.Cout % 16 != 0 || g.Cout > 16 * kTrMaxG)
        return 0;
    if (g.C1 <= kTrMaxC1 && g.C0 % 32 == 0) return 1;
    if (g.C0 <= kTrMaxC1 && g.C1 % 32 == 0) return 2;
    return 0;
}
// the large source alone, its gradient rows where they sit in gw
static nconv_dense_wgrad tr_rows_main(const nconv_dense_wgrad& g) {
    nconv_dense_wgrad m = g;
    if (tr_rows_split(g) == 2) {
        m.x0 = g.x1;
        m.C0 = g.C1;
        m.gw = g.gw + (size_t)g.C0 * g.Cout * 16;
    }
    m.x1 = nullptr;
    m.C1 = 0;
    return m;
}
struct TrRowsGrid {
    int nry, nrx, nslice;
};
static TrRowsGrid tr_rows_grid(const nconv_dense_wgrad& g) {
    TrRowsGrid r;
    r.nry = (g.Ho + kTrRows - 1) / kTrRows;
    r.nrx = (g.Wo + kTrCols - 1) / kTrCols;
    r.nslice = g.B * r.nry * r.nrx;
    return r;
}

static size_t main_wgrad_bytes(const nconv_dense_wgrad& g) {
    const WgdPlan pl = wgrad_plan(g);
    return (size_t)pl.a.nks * pl.a.M * pl.a.N * sizeof(float);
}

size_t dense_wgrad_workspace_bytes(const nconv_dense_wgrad& g) {
    if (!tr_rows_split(g)) return main_wgrad_bytes(g);
    const size_t a = (main_wgrad_bytes(tr_rows_main(g)) + 255) & ~(size_t)255;
    const int cs = tr_rows_split(g) == 1 ? g.C1 : g.C0;
    return a + (size_t)tr_rows_grid(g).nslice * cs * g.Cout * 16 * sizeof(double);
}

template <int KIND, int S, int NT>
static bool go_wgrad(const WgdPlan& pl, float* ws, hipStream_t st) {
    const dim3 grid(pl.a.nbm * pl.a.nbn * pl.a.nks), blk(kDT);
    if (pl.gn != 1) return false;  // (one n-group per workgroup: LDS-DMA staging)
    if (pl.gm == 1)
        hipLaunchKernelGGL((dense_wgrad_mfma<KIND, S, NT, 1, 1>), grid, blk, 0, st, pl.a, ws);
    else if constexpr (NT > 1)
        hipLaunchKernelGGL((dense_wgrad_mfma<KIND, S, NT, 2, 1>), grid, blk, 0, st, pl.a, ws);
    else
        return false;
    return true;
}

static int launch_dense_wgrad_main(const nconv_dense_wgrad& g, float* ws, hipStream_t st, const char** why);

int launch_dense_wgrad(const nconv_dense_wgrad& g, float* ws, size_t ws_bytes, hipStream_t st, const char** why) {
    if (ws_bytes < dense_wgrad_workspace_bytes(g)) {
        *why = "workspace too small (see nconv_dense_wgrad_workspace_bytes)";
        return -22;
    }
    const int sp = tr_rows_split(g);
    if (!sp) return launch_dense_wgrad_main(g, ws, st, why);
    const nconv_dense_wgrad m = tr_rows_main(g);  // the large source's rows
    if (int rc = launch_dense_wgrad_main(m, ws, st, why)) return rc;
    const TrRowsGrid r = tr_rows_grid(g);
    double* part = reinterpret_cast<double*>(ws + ((main_wgrad_bytes(m) + 255) & ~(size_t)255) / sizeof(float));
    const float* xs = sp == 1 ? g.x1 : g.x0;
    const int cs = sp == 1 ? g.C1 : g.C0;
    hipLaunchKernelGGL(dense_wgrad_tr_rows, dim3(r.nslice * g.Cout), dim3(256), 0, st, xs, cs, g.H, g.W, g.gy, g.Cout,
                       g.Ho, g.Wo, r.nry, r.nrx, part);
    const int mn = cs * g.Cout * 16;
    hipLaunchKernelGGL(dense_wgrad_reduce_d, dim3((mn + 63) / 64), dim3(kDT), 0, st, part, r.nslice, mn,
                       sp == 1 ? g.gw + (size_t)g.C0 * g.Cout * 16 : g.gw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

static int launch_dense_wgrad_main(const nconv_dense_wgrad& g, float* ws, hipStream_t st, const char** why) {
    const WgdPlan pl = wgrad_plan(g);
    bool ok = false;
    if (pl.bf9) {
        const dim3 grid(pl.a.nbm * pl.a.nbn * pl.a.nks), blk(kDT);
        const bool x9 = g.math == NCONV_DENSE_MATH_BF16X9;
        if (g.stride == 1 && x9)
            hipLaunchKernelGGL((dense_wgrad_bf9<9, 1>), grid, blk, 0, st, pl.a, ws);
        else if (g.stride == 1)
            hipLaunchKernelGGL((dense_wgrad_bf9<6, 1>), grid, blk, 0, st, pl.a, ws);
        else if (x9)
            hipLaunchKernelGGL((dense_wgrad_bf9<9, 2>), grid, blk, 0, st, pl.a, ws);
        else
            hipLaunchKernelGGL((dense_wgrad_bf9<6, 2>), grid, blk, 0, st, pl.a, ws);
        ok = true;
    }
#define NCONV_WG(KIND_, S_)                                                                     \
    if (g.kind == KIND_ && g.stride == S_)                                                     \
        ok = pl.nt == 1 ? go_wgrad<KIND_, S_, 1>(pl, ws, st) : go_wgrad<KIND_, S_, wgd_ntb(KIND_)>(pl, ws, st);
    if (!ok) NCONV_WG(NCONV_DENSE_3X3, 1)
    if (!ok) NCONV_WG(NCONV_DENSE_3X3, 2)
    NCONV_WG(NCONV_DENSE_1X1, 1)
    NCONV_WG(NCONV_DENSE_1X1, 2)
    NCONV_WG(NCONV_DENSE_TRANSPOSED_4X4, 2)
#undef NCONV_WG
    if (!ok) {
        *why = "no weight-gradient kernel for this (kind, stride, grouping)";
        return -95;
    }
    const int mn = pl.a.M * pl.a.N;
    hipLaunchKernelGGL(dense_wgrad_reduce, dim3((mn + 63) / 64), dim3(kDT), 0, st, ws, pl.a.nks, mn, g.gw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
