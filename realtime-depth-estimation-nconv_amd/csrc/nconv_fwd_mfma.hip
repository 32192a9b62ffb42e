// nconv_fwd_mfma.hip — NConv forward on the bf16 matrix cores, split-bf16 ("bf16x3") arithmetic.
//
// The 8-output-channel NConv layers of DNET (step1.py:39-46: 8->8 5x5, 16->8 3x3) are
// FP32-compute bound on the vector ALU (arithmetic intensity 32-50 flop/B against a ridge of
// 19.7). gfx950 has no reduced-precision f32 MFMA (no xf32), but its bf16 MFMA runs at 16x the
// FP32 rate, so each fp32 operand v is split into v = hi + lo (hi = bf16(v), lo = bf16(v - hi))
// and every product is formed as  a_hi*b_hi + a_lo*b_hi + a_hi*b_lo  with fp32 accumulation.
// The dropped a_lo*b_lo and the split residuals are <= 2^-18 |a*b| each, so a product carries a
// relative error <= ~1.1e-5 and — every term of N and D being a product of a positive weight and
// a non-negative confidence (times the data for N) — so do the sums: inside the 1e-4 forward
// tolerance with two orders of magnitude to spare in practice (errors are
// unbiased; tests/test_gpu_layers.py measures them). NCONV_MATH_FP32 keeps the exact VALU path.
//
// GEMM shape (v_mfma_f32_16x16x32_bf16): a 16x16 output tile is 16 adjacent output columns (the
// A rows, u) x (8 output channels o, 2 output rows s) (the B columns). The row shift s lives in
// the weights: with k = (kh' in [0, K], kw, 8 input channels), B[k][(o, s)] = W[o][ci][kh'-s][kw]
// (0 outside the kernel), A[u][k] = input[ci][row0 + kh'][col0 + u + kw], so one A fragment feeds
// both output rows and all 8 output channels and no B column is wasted (8 channels alone would
// fill half of a 16-wide tile). N and D share B and accumulate in separate tiles.
//
// Data flow per 256-thread workgroup (TH x 32 output pixels, all 8 channels): the layer's input
// glue (2x2 max-pool / nearest-upsample + concat, step1.py:62-90) is evaluated while staging the
// (TH+K-1) x (32+K-1) halo tile; each position's 8-channel vectors {x*c, c} are split and stored
// as four bf16x8 planes (x*c hi/lo, c hi/lo), so every A fragment is one conflict-free
// ds_read_b128 (16 lanes read 256 contiguous bytes). The weights' B fragments are built once per
// workgroup into registers. Epilogue per lane: 4 adjacent pixels of one (channel, row):
// y = N/(D+eps)+b, cout = D/s, 16-B stores, optionally the fused 2x2 max-pooled copies (rows s=0/1
// of a pixel pair sit in lanes l, l^8) or nconv7 (1x1 over the 8 channels = lanes l^1, l^2, l^4)
// with the crop, as the VALU kernels of nconv_fwd.hip do.
//
// Exact products (NCONV_MATH_BF16X9): with three parts per operand, v = v0 + v1 + v2 (v0 = bf16(v),
// v1 = bf16(v - v0), v2 = v - v0 - v1, which has at most 8 significant bits and is exact in bf16),
// the decomposition is exact, every partial product vi*wj of two 8-bit significands is exact in
// fp32, and all nine enter the fp32 accumulator: sum_ij vi*wj = v*w exactly, so the only rounding
// is the fp32 accumulation, as in any fp32 convolution. The kernels are the same with NP = 3 parts
// (three planes per operand, three B fragments per k-step) and nine MFMAs per {N, D} k-step,
// smallest terms first.
#include <cstdlib>
#include "nconv_internal.h"

namespace nconv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int kMfThreads = 256;

enum MfEpi { kEpiPlain = 0, kEpiPool = 1, kEpiTail = 2 };

template <int CIN, int K, int TH, int NP = 2>
struct MfCfg {
    static constexpr int G = CIN / 8;  // 8-channel groups (one bf16x8 per position and part)
    static constexpr int TW = 32;      // two 16-column MFMA tiles
    static constexpr int IH = TH + K - 1, IW = TW + K - 1;
    static constexpr int NPOS = IH * IW;
    static constexpr int NE = (NPOS + kMfThreads - 1) / kMfThreads;  // positions per thread
    static constexpr int PSTRIDE = NPOS * 16;                        // bytes of one plane
    static constexpr int NPL = 2 * NP;                               // planes: x*c parts, c parts
    static constexpr int LDS_IN = NPL * G * PSTRIDE;                 // [g][plane][pos] bf16x8
    static constexpr int NKP = (K + 1) * K * G;                      // k positions (kh', kw, g)
    static constexpr int NT = (NKP + 3) / 4;                         // k-steps (4 positions each)
    static constexpr int NRP = TH / 2;                               // row pairs, NRP / 4 per wave
    static_assert(CIN % 8 == 0 && NRP % 4 == 0, "tile shape");
};

// Split products: which (data part i, weight part j) terms a math mode forms. Two parts (bf16x3):
// i + j <= 1 (the lo*lo term dropped). Three parts (bf16x9): all nine (exact products).
template <int NP>
__device__ __forceinline__ constexpr bool use_term(int i, int j) {
    return NP == 2 ? i + j <= 1 : true;
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// v = sum of NP bf16 parts, each the bf16 rounding of what the previous parts left (VT: a bf16
// vector of N lanes)
template <int NP, typename VT, int N>
__device__ __forceinline__ void split_parts(const float (&v)[N], VT (&out)[NP]) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        float r = v[j];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const __bf16 h = (__bf16)r;
            out[p][j] = h;
            if (p + 1 < NP) r -= (float)h;
        }
    }
}

constexpr unsigned kOOB = 0x80000000u;
constexpr int kOutPitch = 36;  // floats per row of a wave's output-transpose region
constexpr int kTrBytes = 4 * 16 * kOutPitch * 4;  // four waves' regions (y, then cout, through one)


// One position's 8 channels of {x*c, c} into the planes of a tile (base = plane 0 of the
// position's channel group): x*c parts in planes 0 .. NP-1, c parts in NP .. 2NP-1.
template <typename C>
__device__ __forceinline__ void store_planes(unsigned char* base, const float (&p)[8], const float (&q)[8]) {
    constexpr int NP = C::NPL / 2;
    bf16x8 sp[NP], sq[NP];
    split_parts<NP>(p, sp);
    split_parts<NP>(q, sq);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        *reinterpret_cast<bf16x8*>(base + i * C::PSTRIDE) = sp[i];
        *reinterpret_cast<bf16x8*>(base + (NP + i) * C::PSTRIDE) = sq[i];
    }
}

// Staging of one tile's halo: per thread NE positions x CIN channels of {x, c}, loaded into
// registers (load: glue evaluated, no wait) and later split into the 2 NP bf16x8 planes (store).
template <int CIN, int K, int MODE, int TH, int NP>
struct MfStage {
    using C = MfCfg<CIN, K, TH, NP>;
    static constexpr bool UP = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST;
    static constexpr unsigned OOB = 0x80000000u;
    float xv[C::NE][CIN], cv[C::NE][CIN];

    __device__ __forceinline__ void load(const LayerDev& d, int b, int ih0, int iw0, int tid) {
        const nconv_layer& L = d.L;
        unsigned ga[C::NE], gb[UP ? C::NE : 1];
#pragma unroll
        for (int k = 0; k < C::NE; ++k) {
            const int e = tid + kMfThreads * k;
            const int r = e / C::IW, col = e - r * C::IW;
            const int ih = ih0 + r, iw = iw0 + col;
            const bool in = e < C::NPOS && (unsigned)ih < (unsigned)L.H && (unsigned)iw < (unsigned)L.W;
            if constexpr (MODE == NCONV_LOAD_POOL2)
                ga[k] = in ? (unsigned)((2 * ih) * L.a.W + 2 * iw) * 4u : OOB;
            else
                ga[k] = in ? (unsigned)(ih * L.a.W + iw) * 4u : OOB;
            if constexpr (UP) {
                const int sh = nearest_src(ih, L.b.H, L.H, d.up_scale_h);
                const int sw = nearest_src(iw, L.b.W, L.W, d.up_scale_w);
                gb[k] = in ? (unsigned)(sh * L.b.W + sw) * 4u : OOB;
            }
        }
        // One buffer resource per source tensor of this image (all its channels; the host checks
        // the size fits), the channel's plane offset in the scalar offset: 4 resources instead of
        // 2 per input channel, which kept the 16-channel kernels spilling scalar registers.
        int pa = L.a.H * L.a.W * 4;
        int pb = UP ? L.b.H * L.b.W * 4 : 0;
        // (opaque per call: keeps the per-channel offsets out of the tile loop's invariant SGPRs)
        asm volatile("" : "+s"(pa), "+s"(pb));
        const __amdgpu_buffer_rsrc_t rax = plane_rsrc(L.a.x + (size_t)b * L.a.C * (pa / 4), L.a.C * pa);
        const __amdgpu_buffer_rsrc_t rac = plane_rsrc(L.a.c + (size_t)b * L.a.C * (pa / 4), L.a.C * pa);
        const __amdgpu_buffer_rsrc_t rbx = UP ? plane_rsrc(L.b.x + (size_t)b * L.b.C * (pb / 4), L.b.C * pb) : rax;
        const __amdgpu_buffer_rsrc_t rbc = UP ? plane_rsrc(L.b.c + (size_t)b * L.b.C * (pb / 4), L.b.C * pb) : rac;
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
            if constexpr (MODE == NCONV_LOAD_POOL2) {
                const unsigned row = (unsigned)L.a.W * 4u;
                const int so = ci * pa;
#pragma unroll
                for (int k = 0; k < C::NE; ++k) {
                    const unsigned o2 = ga[k] == OOB ? OOB : ga[k] + row;
                    const f2 x0 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rax, ga[k], so, 0));
                    const f2 x1 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rax, o2, so, 0));
                    const f2 c0 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rac, ga[k], so, 0));
                    const f2 c1 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rac, o2, so, 0));
                    xv[k][ci] = pool4v(x0.x, x0.y, x1.x, x1.y);
                    cv[k][ci] = pool4v(c0.x, c0.y, c1.x, c1.y);
                }
            } else {
                // channel ci of the concatenation: source a or (nearest-upsampled) b, wave-uniform
                bool from_a = true;
                int cs = ci;
                if constexpr (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST) {
                    from_a = ci < L.a.C;
                    cs = from_a ? ci : ci - L.a.C;
                } else if constexpr (MODE == NCONV_LOAD_UPCAT_UP_FIRST) {
                    from_a = ci >= L.b.C;
                    cs = from_a ? ci - L.b.C : ci;
                }
#pragma unroll
                for (int k = 0; k < C::NE; ++k) {
                    if (!UP || from_a) {
                        xv[k][ci] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rax, ga[k], cs * pa, 0));
                        cv[k][ci] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rac, ga[k], cs * pa, 0));
                    } else {
                        xv[k][ci] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbx, gb[UP ? k : 0], cs * pb, 0));
                        cv[k][ci] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbc, gb[UP ? k : 0], cs * pb, 0));
                    }
                }
            }
        }
    }

    static constexpr int BYTES = 0;  // no LDS of its own
    static constexpr bool SELF_SYNC = false;
    __device__ __forceinline__ void issue(const LayerDev& d, const TailArgs&, int b, int ih0, int iw0, unsigned char*,
                                          int tid) {
        load(d, b, ih0, iw0, tid);
    }
    __device__ __forceinline__ void to_planes(const LayerDev&, const TailArgs&, int, int, unsigned char* lds,
                                              unsigned char*, int tid) const {
        store(lds, tid);
    }

    __device__ __forceinline__ void store(unsigned char* lds, int tid) const {
#pragma unroll
        for (int k = 0; k < C::NE; ++k) {
            const int e = tid + kMfThreads * k;
            if (C::NE * kMfThreads != C::NPOS && e >= C::NPOS) continue;
#pragma unroll
            for (int g = 0; g < C::G; ++g) {
                float p[8], q[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    q[j] = cv[k][8 * g + j];
                    p[j] = xv[k][8 * g + j] * q[j];
                }
                store_planes<C>(lds + g * C::NPL * C::PSTRIDE + e * 16, p, q);
            }
        }
    }
};

__device__ __forceinline__ int floor_div4(int v) { return v >> 2; }  // arithmetic shift: floor

// Staging through LDS-DMA (buffer_load_dwordx4 ... lds): no registers hold the halo in flight and
// one wave-instruction moves 1 KiB, four times the bytes of a dword load. The fp32 source rows are
// copied as aligned 16-byte vectors (row width a multiple of 4 floats, so a vector is wholly in or
// out of the image; out-of-image vectors carry an offset past the resource and land as zeros, the
// convolution's padding): source a at the layer's resolution (IH rows x 10 vectors per channel),
// and for the upsample-concat modes source b at its own half resolution (IH/2+1 rows x 6 vectors),
// the exact 2x nearest upsampling being applied when the planes are formed. Sections (a.x, a.c,
// b.x, b.c) are padded to whole 1-KiB pieces; LDS is lane-linear within a piece.
template <int CIN, int K, int MODE, int TH, int NP>
struct DmaStage {
    using C = MfCfg<CIN, K, TH, NP>;
    static constexpr bool UP = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST;
    static constexpr int CA = UP ? CIN / 2 : CIN, CB = UP ? CIN / 2 : 0;
    static constexpr int NVA = 10, SRA = C::IH;            // source a: vectors per row, rows
    static constexpr int NVB = 6, SRB = C::IH / 2 + 1;     // source b (half resolution)
    static constexpr int PA = (CA * SRA * NVA + 63) / 64;  // 1-KiB pieces per tensor of source a
    static constexpr int PB = UP ? (CB * SRB * NVB + 63) / 64 : 0;
    static constexpr int NPC = 2 * PA + 2 * PB;  // pieces
    static constexpr int BYTES = NPC * 1024;
    static_assert(4 * NVA >= C::IW + 3 && 4 * NVB >= (C::IW + 1) / 2 + 4, "staged columns cover the halo");

    static constexpr bool SELF_SYNC = true;
    __device__ __forceinline__ void issue(const LayerDev& d, const TailArgs&, int b, int ih0, int iw0,
                                          unsigned char* stage, int tid) const {
        const nconv_layer& L = d.L;
        const int wave = tid >> 6, lane = tid & 63;
#pragma unroll 1
        for (int j = wave; j < NPC; j += 4) {  // wave-uniform piece index
            const int sec = j < 2 * PA ? j / PA : 2 + (j - 2 * PA) / PB;
            const int jj = sec < 2 ? j - sec * PA : j - 2 * PA - (sec - 2) * PB;
            const bool a = sec < 2;
            const nconv_src& sr = a ? L.a : L.b;
            const int Cs = a ? CA : CB, SR = a ? SRA : SRB, NV = a ? NVA : NVB;
            const int r0 = a ? ih0 : (ih0 >> 1), c0 = 4 * floor_div4(a ? iw0 : (iw0 >> 1));
            const float* base = ((sec & 1) ? sr.c : sr.x) + (size_t)b * Cs * sr.H * sr.W;
            const __amdgpu_buffer_rsrc_t rs = plane_rsrc(base, Cs * sr.H * sr.W * 4);
            const int f = jj * 64 + lane;
            const int ch = f / (SR * NV), rem = f - ch * (SR * NV), row = rem / NV, vec = rem - row * NV;
            const int gr = r0 + row, gc = c0 + 4 * vec;
            const bool ok = ch < Cs && (unsigned)gr < (unsigned)sr.H && (unsigned)gc < (unsigned)sr.W;
            const unsigned go = ok ? (unsigned)((ch * sr.H + gr) * sr.W + gc) * 4u : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, (int)go, 0, 0, 0);
        }
    }

    // Wait for this wave's pieces, then (all pieces landed) form the bf16 planes.
    __device__ __forceinline__ void to_planes(const LayerDev& d, const TailArgs&, int ih0, int iw0, unsigned char* lds,
                                              unsigned char* stage, int tid) const {
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
        __syncthreads();
        const float* S = reinterpret_cast<const float*>(stage);
        const int sha = iw0 - 4 * floor_div4(iw0);                   // column shift in source a rows
        const int rb0 = ih0 >> 1, cb0 = 4 * floor_div4(iw0 >> 1);  // source b origin
#pragma unroll
        for (int k = 0; k < C::NE; ++k) {
            const int e = tid + kMfThreads * k;
            if (C::NE * kMfThreads != C::NPOS && e >= C::NPOS) continue;
            const int r = e / C::IW, col = e - r * C::IW;
            const int ia = r * (NVA * 4) + col + sha;
            const int ib = (((ih0 + r) >> 1) - rb0) * (NVB * 4) + ((iw0 + col) >> 1) - cb0;
#pragma unroll
            for (int g = 0; g < C::G; ++g) {
                float p[8], q[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int ci = 8 * g + j;
                    bool from_a = true;
                    int cs = ci;
                    if constexpr (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST) {
                        from_a = ci < CA;
                        cs = from_a ? ci : ci - CA;
                    } else if constexpr (MODE == NCONV_LOAD_UPCAT_UP_FIRST) {
                        from_a = ci >= CB;
                        cs = from_a ? ci - CB : ci;
                    }
                    float xv, cv;
                    if (from_a) {
                        xv = S[cs * SRA * NVA * 4 + ia];
                        cv = S[PA * 256 + cs * SRA * NVA * 4 + ia];
                    } else {
                        xv = S[2 * PA * 256 + cs * SRB * NVB * 4 + ib];
                        cv = S[(2 * PA + PB) * 256 + cs * SRB * NVB * 4 + ib];
                    }
                    q[j] = cv;
                    p[j] = xv * cv;
                }
                store_planes<C>(lds + g * C::NPL * C::PSTRIDE + e * 16, p, q);
            }
        }
    }
};

// Fused head (nconv_fwd_head): nconv2's input (x1, c1) = nconv1(S, S > thresh) is computed here,
// per tile, from the (TH+8) x 40 sparse-depth halo, so it never exists in HBM. nconv1 runs on the
// vector ALU in exact fp32 (packed {N, D} FMAs, the same tap order as fwd_tiled's nconv1, so the
// values equal the unfused layer's), then feeds the split-bf16 planes like a loaded input.
constexpr int kModeHead = 100;

// One position's 4 channels (a bf16x4 half of the position's 16-byte slot) into the planes.
template <typename C>
__device__ __forceinline__ void store_half_planes(unsigned char* base, const float (&p)[4], const float (&q)[4]) {
    constexpr int NP = C::NPL / 2;
    bf16x4 sp[NP], sq[NP];
    split_parts<NP>(p, sp);
    split_parts<NP>(q, sq);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        *reinterpret_cast<bf16x4*>(base + i * C::PSTRIDE) = sp[i];
        *reinterpret_cast<bf16x4*>(base + (NP + i) * C::PSTRIDE) = sq[i];
    }
}

template <int TH, int NP>
struct HeadStage {
    using C = MfCfg<8, 5, TH, NP>;
    static constexpr int SH = C::IH + 4, SW = C::IW + 4;  // nconv1's own 5x5 halo around the tile
    static constexpr int NS = SH * SW, NES = (NS + kMfThreads - 1) / kMfThreads;
    static constexpr int WOFF = NS * 8;                   // {S * c0, c0} pairs, then
    static constexpr int BYTES = WOFF + 2 * 25 * 16;      // nconv1's weights [half][kw][kh][o4]
    static constexpr bool SELF_SYNC = true;
    float sv[NES];

    // nconv1's weights into LDS once per workgroup (visible after to_planes' first barrier), in
    // the order the column loop reads them: one broadcast float4 (4 output channels) per tap.
    __device__ __forceinline__ void init(const TailArgs& t, unsigned char* stage, int tid) const {
        if (tid < 200) {
            const int half = tid / 100, rem = tid - 100 * half;
            const int kw = rem / 20, kh = (rem / 4) % 5, o = rem % 4;
            reinterpret_cast<float*>(stage + WOFF)[tid] = t.w1[(half * 4 + o) * 25 + kh * 5 + kw];
        }
    }

    __device__ __forceinline__ void issue(const LayerDev& d, const TailArgs& t, int b, int ih0, int iw0,
                                          unsigned char*, int tid) {
        const int H = d.L.H, W = d.L.W;
        const __amdgpu_buffer_rsrc_t rs = plane_rsrc(t.s_in + (size_t)b * H * W, H * W * 4);
#pragma unroll
        for (int k = 0; k < NES; ++k) {
            const int e = tid + kMfThreads * k;
            const int r = e / SW, col = e - r * SW;
            const int ih = ih0 - 2 + r, iw = iw0 - 2 + col;
            const bool in = e < NS && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            sv[k] = ld_f32(rs, in ? (unsigned)(ih * W + iw) * 4u : kOOB);
        }
    }

    __device__ __forceinline__ void to_planes(const LayerDev& d, const TailArgs& t, int ih0, int iw0,
                                              unsigned char* lds, unsigned char* stage, int tid) const {
        f2* T = reinterpret_cast<f2*>(stage);
#pragma unroll
        for (int k = 0; k < NES; ++k) {
            const int e = tid + kMfThreads * k;
            const float c0 = sv[k] > t.thresh1 ? 1.0f : 0.0f;  // step1.py:53
            if (NES * kMfThreads == NS || e < NS) T[e] = (f2){sv[k] * c0, c0};
        }
        __syncthreads();  // (also: every wave is done with the previous tile's planes)
        // nconv1: wave w computes output channels 4 (w & 1) .. +3 for column quads — one staged
        // column and 4 consecutive rows per lane, half of the (IH / 4) x 36 quads per wave pair.
        // The weights come from LDS (broadcast reads; per-lane global weight loads were
        // vector-memory reads the loop waited on each iteration together with the previous tile's
        // outstanding stores, and scalar loads also stalled it); consecutive lanes read consecutive
        // {x*c, c} pairs, so the window reads are free of LDS bank conflicts.
        static_assert(C::IW == 36 && C::IH % 4 == 0, "36 staged columns, whole row quads");
        const int H = d.L.H, W = d.L.W;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, half = wave & 1;
        constexpr int NQ = (C::IH / 4) * C::IW, PERW = (NQ + 1) / 2;
        static_assert(PERW <= 64, "one quad per lane");
        const int tq = (wave >> 1) * PERW + lane;
        if (lane < PERW && tq < NQ) {
            const int rq = tq / C::IW, c = tq - rq * C::IW, r0 = 4 * rq;
            const f4* wl = reinterpret_cast<const f4*>(stage + WOFF) + half * 25;
            f2 acc[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int o = 0; o < 4; ++o) acc[j][o] = (f2){0.f, 0.f};

#pragma unroll 1
            for (int kw = 0; kw < 5; ++kw) {
                const f2* col = T + r0 * SW + c + kw;
                f2 v[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) v[m] = col[m * SW];
#pragma unroll
                for (int kh = 0; kh < 5; ++kh) {
                    const f4 w4 = wl[kw * 5 + kh];
#pragma unroll
                    for (int o = 0; o < 4; ++o) {
                        const float w = w4[o];
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[j][o] = __builtin_elementwise_fma((f2){w, w}, v[j + kh], acc[j][o]);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = r0 + j;
                const bool in = (unsigned)(ih0 + r) < (unsigned)H && (unsigned)(iw0 + c) < (unsigned)W;
                float p[4], q[4];
#pragma unroll
                for (int o = 0; o < 4; ++o) {
                    float xv, cv;
                    nconv_epilogue(acc[j][o].x, acc[j][o].y, t.eps1, t.b1[half * 4 + o], t.s1[half * 4 + o], xv, cv);
                    q[o] = in ? cv : 0.f;  // nconv2's zero padding outside the image
                    p[o] = in ? xv * cv : 0.f;
                }
                store_half_planes<C>(lds + (r * C::IW + c) * 16 + half * 8, p, q);
            }
        }
    }
};

// The fused head with nconv1 on the matrix cores as well (the default; -DNCONV_HEAD_NC1_VALU keeps
// the exact-fp32 vector-ALU nconv1 above). GEMM per v_mfma_f32_16x16x32_bf16, per block of 16
// columns x 4 rows of nconv1's (IH x IW) output region: D[(o, s')][u] = sum_k A[(o, s')][k] B[k][u]
// with k = (kw: the lane group, kh': 8 consecutive rows of the window), so the lane holding output
// column u reads 8 consecutive rows of one staged column: the thresholded depth is staged
// column-major (NP bf16 parts of S*c0, then c0 — c0 in {0, 1} is exact, so D takes NP split
// products, one per weight part, and N the split terms of the math mode), one 16-byte row window
// per (part, k-step) read as dwords (row offsets are even, not multiples of 8). A (the weights'
// NP parts, W1[o][kh' - s'][kw] for the window of output rows 4g + 2m + s') is independent of the
// row pair m and lives in LDS. The lane's outputs are 4 channels of one position: the bf16x4
// halves of nconv2's planes, written directly.
template <int TH, int NP>
struct HeadStageMf {
    using C = MfCfg<8, 5, TH, NP>;
    static constexpr int SH = C::IH + 4, SW = C::IW + 4;  // nconv1's input halo
    static constexpr int NS = SH * SW, NES = (NS + kMfThreads - 1) / kMfThreads;
    static constexpr int NCB = (C::IW + 15) / 16, NG = C::IH / 4;  // column blocks, row groups
    static constexpr int CW = 16 * NCB + 4;  // staged columns read (past SW: zeros)
    static constexpr int RS = SH + 4;        // rows per staged column (+ zero rows), 2 B each
    static constexpr int COLB = RS * 2;      // bytes per staged column: 40 (conflict-free b32 reads)
    static constexpr int PART = CW * COLB;   // bytes per part
    static constexpr int AOFF = (NP + 1) * PART;          // weights' A fragments [step][part][lane] bf16x8
    static constexpr int BOFF = AOFF + 2 * NP * 64 * 16;  // nconv1's bias[8], 1 / s[8]
    static constexpr int BYTES = BOFF + 16 * 4;
    static constexpr bool SELF_SYNC = true;
    static_assert(C::IH % 4 == 0 && RS % 2 == 0 && (PART % 16) == 0, "layout");
    float sv[NES];

    __device__ __forceinline__ void init(const TailArgs& t, unsigned char* stage, int tid) const {
        // zero the staged parts once: the padding rows / columns are read (against zero weights)
        // and must hold finite values; the staging below rewrites only the SH x SW interior
        for (int i = tid; i < AOFF / 16; i += kMfThreads) reinterpret_cast<f4*>(stage)[i] = (f4){0.f, 0.f, 0.f, 0.f};
        // A fragment of lane l for k-step st (kw = 4 st + kg) and weight part
        const int l = tid & 63;
        for (int f = tid >> 6; f < 2 * NP; f += 4) {
            const int st = f / NP, part = f - st * NP;
            const int i = l & 15, o = i & 7, sp = i >> 3, kg = l >> 4, kw = 4 * st + kg;
            float w[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int kh = e - sp;
                w[e] = (kw < 5 && kh >= 0 && kh < 5) ? t.w1[(o * 5 + kh) * 5 + kw] : 0.f;
            }
            bf16x8 wp[NP];
            split_parts<NP>(w, wp);
            *reinterpret_cast<bf16x8*>(stage + AOFF + (f * 64 + l) * 16) = wp[part];
        }
        if (tid < 16)
            reinterpret_cast<float*>(stage + BOFF)[tid] = tid < 8 ? t.b1[tid] : __builtin_amdgcn_rcpf(t.s1[tid - 8]);
    }

    __device__ __forceinline__ void issue(const LayerDev& d, const TailArgs& t, int b, int ih0, int iw0,
                                          unsigned char*, int tid) {
        const int H = d.L.H, W = d.L.W;
        const __amdgpu_buffer_rsrc_t rs = plane_rsrc(t.s_in + (size_t)b * H * W, H * W * 4);
#pragma unroll
        for (int k = 0; k < NES; ++k) {
            const int e = tid + kMfThreads * k;
            const int r = e / SW, col = e - r * SW;
            const int ih = ih0 - 2 + r, iw = iw0 - 2 + col;
            const bool in = e < NS && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            sv[k] = ld_f32(rs, in ? (unsigned)(ih * W + iw) * 4u : kOOB);
        }
    }

    // 8 consecutive bf16 of a staged column from a 4-byte-aligned address (two ds_read2_b32)
    static __device__ __forceinline__ bf16x8 rd_window(const unsigned char* q) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const unsigned* w = reinterpret_cast<const unsigned*>(q);
        return __builtin_bit_cast(bf16x8, (u32x4){w[0], w[1], w[2], w[3]});
    }

    __device__ __forceinline__ void to_planes(const LayerDev& d, const TailArgs& t, int ih0, int iw0,
                                              unsigned char* lds, unsigned char* stage, int tid) const {
        // (every wave has finished the previous tile's nconv1 reads: the barrier before the MFMA
        // phase separates them from these writes)
#pragma unroll
        for (int k = 0; k < NES; ++k) {
            const int e = tid + kMfThreads * k;
            if (NES * kMfThreads != NS && e >= NS) continue;
            const int r = e / SW, col = e - r * SW;
            const float c0 = sv[k] > t.thresh1 ? 1.0f : 0.0f;  // step1.py:53
            float p = sv[k] * c0;
            unsigned char* q = stage + col * COLB + r * 2;
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const __bf16 h = (__bf16)p;
                *reinterpret_cast<__bf16*>(q + i * PART) = h;
                if (i + 1 < NP) p -= (float)h;
            }
            *reinterpret_cast<__bf16*>(q + NP * PART) = (__bf16)c0;
        }
        __syncthreads();
        const int H = d.L.H, W = d.L.W;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        const int u = lane & 15, kg = lane >> 4, half = kg & 1, sp = lane >> 5;
        bf16x8 a[2][NP];
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int j = 0; j < NP; ++j)
                a[st][j] = *reinterpret_cast<const bf16x8*>(stage + AOFF + ((st * NP + j) * 64 + lane) * 16);
        // (from LDS: a global load here would wait for the previous tile's stores as well)
        const f4 bias = reinterpret_cast<const f4*>(stage + BOFF)[half];
        const f4 rs1 = reinterpret_cast<const f4*>(stage + BOFF)[2 + half];
        typedef float f4_ __attribute__((ext_vector_type(4)));
#pragma unroll 1
        for (int blk = wave; blk < NG * NCB; blk += 4) {
            const int g = blk / NCB, cb = blk - g * NCB;
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const int r0 = 4 * g + 2 * m;  // first window row (staged coordinates)
                f4_ n = {0.f, 0.f, 0.f, 0.f}, dd = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int st = 0; st < 2; ++st) {
                    const int kw = st == 0 ? kg : 4;  // k-step 1: only group 0 (kw 4) has weights
                    const unsigned char* q = stage + (16 * cb + u + kw) * COLB + r0 * 2;
                    bf16x8 pw[NP];
#pragma unroll
                    for (int i = 0; i < NP; ++i) pw[i] = rd_window(q + i * PART);
                    const bf16x8 cz = rd_window(q + NP * PART);
                    // smallest terms first: N over the (data part i, weight part j) terms of the
                    // mode, D over the weight parts (c0 is exact)
#pragma unroll
                    for (int s = 2 * (NP - 1); s >= 0; --s) {
#pragma unroll
                        for (int i = NP - 1; i >= 0; --i) {
                            const int j = s - i;
                            if (j < 0 || j >= NP || !use_term<NP>(i, j)) continue;
                            n = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[st][j], pw[i], n, 0, 0, 0);
                        }
                        if (s < NP) dd = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[st][s], cz, dd, 0, 0, 0);
                    }
                }
                // lane: channels 4 half .. +3 of nconv1 output (row r0 + sp, column 16 cb + u)
                const int row = r0 + sp, col = 16 * cb + u;
                const bool in = (unsigned)(ih0 + row) < (unsigned)H && (unsigned)(iw0 + col) < (unsigned)W;
                float pv[4], qv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float xv = n[r] * __builtin_amdgcn_rcpf(dd[r] + t.eps1) + bias[r];
                    const float cv = dd[r] * rs1[r];
                    qv[r] = in ? cv : 0.f;  // nconv2's zero padding outside the image
                    pv[r] = in ? xv * cv : 0.f;
                }
                if (col < C::IW) store_half_planes<C>(lds + (row * C::IW + col) * 16 + half * 8, pv, qv);
            }
        }
    }
};

// Persistent: gridDim.x (a multiple of 8) workgroups walk the tiles; the next tile's halo loads
// are in flight while the current one's MFMAs and epilogue run.
#ifndef NCONV_MF_TH5
#define NCONV_MF_TH5 8  // output rows per tile of the 5x5 layers
#endif
#ifndef NCONV_MF_TH_TAIL
// output rows per tile of the fused nconv6+7 tail: 16 (two row pairs per wave; its LDS, without
// the epilogue transposes, still fits two workgroups per CU): 151 vs 162 us at B=8 352x1216.
// (nconv4/5 keep 8: at 16 their LDS admits one workgroup per CU, 50 vs 44 us.)
#define NCONV_MF_TH_TAIL 16
#endif
#ifndef NCONV_MF_TH_HEAD
#define NCONV_MF_TH_HEAD 8  // output rows per tile of the fused nconv1+nconv2 head
#endif
#ifndef NCONV_MFMA_WAVES
#define NCONV_MFMA_WAVES 3  // waves per SIMD: 168 VGPRs (3 workgroups per CU) without spilling
#endif
// POOL2 staging holds four values per element before pooling: 2 waves per SIMD (no spills)
#ifndef NCONV_MFMA_HEAD_WAVES
#define NCONV_MFMA_HEAD_WAVES 3  // fused head
#endif
#ifndef NCONV_MFMA_UP_WAVES
#define NCONV_MFMA_UP_WAVES 2  // the 16-channel upsample-concat layers (nconv4/5/6): no spills
#endif
// three-part (exact-product) kernels: three B fragments per k-step and 1.5x the staged planes
#ifndef NCONV_MFMA_X9_WAVES
#define NCONV_MFMA_X9_WAVES 2
#endif
template <int MODE, bool DMA, int NP>
constexpr int mf_waves() {
    return NP == 3 ? NCONV_MFMA_X9_WAVES
           : MODE == kModeHead ? NCONV_MFMA_HEAD_WAVES
           : DMA || MODE == NCONV_LOAD_POOL2 ? 2
           : (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST) ? NCONV_MFMA_UP_WAVES
                                                                                         : NCONV_MFMA_WAVES;
}
template <int CIN, int K, int MODE, int TH, bool DMA, int NP>
using StageOf = typename std::conditional<
    MODE == kModeHead,
#ifdef NCONV_HEAD_NC1_VALU
    HeadStage<TH, NP>,
#else
    HeadStageMf<TH, NP>,
#endif
    typename std::conditional<DMA, DmaStage<CIN, K, MODE, TH, NP>, MfStage<CIN, K, MODE, TH, NP>>::type>::type;
template <int CIN, int K, int MODE, int EPI, int TH, int NP>
constexpr int mf_lds_bytes(bool dma) {
    return MfCfg<CIN, K, TH, NP>::LDS_IN + (EPI == kEpiTail ? 0 : kTrBytes) +
           (MODE == kModeHead ? StageOf<CIN, K, MODE, TH, false, NP>::BYTES
                              : dma ? DmaStage<CIN, K, MODE, TH, NP>::BYTES : 0);
}
template <int CIN, int K, int MODE, int EPI, int TH, bool VEC, bool DMA, int NP>
__global__ __launch_bounds__(kMfThreads) __attribute__((amdgpu_waves_per_eu(mf_waves<MODE, DMA, NP>(), mf_waves<MODE, DMA, NP>()))) void fwd_mfma(LayerDev d, float* __restrict__ y, float* __restrict__ yc,
                                                       TailArgs t) {
    using C = MfCfg<CIN, K, TH, NP>;
    using Stage = StageOf<CIN, K, MODE, TH, DMA, NP>;
    // input planes, (non-tail) four waves' output-transpose regions (y and cout), DMA staging
    __shared__ __attribute__((aligned(16))) unsigned char lds[mf_lds_bytes<CIN, K, MODE, EPI, TH, NP>(DMA)];
    unsigned char* const stage = lds + C::LDS_IN + (EPI == kEpiTail ? 0 : kTrBytes);
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool tail = EPI == kEpiTail;
    const int gh = tail ? t.out_h : L.Ho, gw = tail ? t.out_w : L.Wo;  // the written grid
    const int ntx = (gw + C::TW - 1) / C::TW, nty = (gh + TH - 1) / TH;
    const int ntiles = ntx * nty * L.B;
    const int off = tail ? t.off : 0;

    Stage st;
    if constexpr (MODE == kModeHead) {
        st.init(t, stage, threadIdx.x);
        __syncthreads();  // (init's LDS writes before any thread's first staging writes)
    }
    int v = blockIdx.x;
    // The block's tiles: virtual ids v, v + gridDim.x, ... map (xcd_tile) to linear tiles t, t + G8,
    // ... (G8 = gridDim.x / 8), so after one mapping the walk advances (tx, ty, b) by a fixed
    // stride — no per-tile integer divisions by the runtime grid extents.
    TileCoord tc = xcd_tile(ntx, nty, L.B, v < ntiles ? v : ntiles - 1);
    const int g8 = (int)gridDim.x / 8, step_ty = g8 / ntx, step_tx = g8 - step_ty * ntx;
    auto advance = [&](TileCoord c) {
        c.tx += step_tx;
        c.ty += step_ty;
        if (c.tx >= ntx) {
            c.tx -= ntx;
            c.ty += 1;
        }
        while (c.ty >= nty) {
            c.ty -= nty;
            c.b += 1;
        }
        return c;
    };
    // loads are unconditional (a block without tiles loads the last one and never uses it)
    st.issue(d, t, tc.b, tc.ty * TH + off - L.PH, tc.tx * C::TW + off - L.PW, stage, tid);

    // ---- B fragments (weights' NP parts, once per workgroup) and per-lane A offsets ----
    const int u = lane & 15, h = lane >> 4;
    const int o = lane & 7, s = (lane >> 3) & 1;  // this lane's B / C column (o, s)
    bf16x8 bw[C::NT][NP];
    int aoff[C::NT];
#pragma unroll
    for (int q = 0; q < C::NT; ++q) {
        const int pos = 4 * q + h;
        float w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = 0.f;
        int a = (1 * C::IW) * 16;  // padding positions read (kh'=1, kw=0): inside both rows' windows
        if (pos < C::NKP) {
            const int g = pos % C::G, qq = pos / C::G, kw = qq % K, khp = qq / K, kh = khp - s;
            a = g * C::NPL * C::PSTRIDE + (khp * C::IW + kw) * 16;
            if (kh >= 0 && kh < K) {
                const float* wp = L.weight + ((size_t)(o * CIN + g * 8) * K + kh) * K + kw;
#pragma unroll
                for (int j = 0; j < 8; ++j) w[j] = wp[j * K * K];
            }
        }
        split_parts<NP>(w, bw[q]);
        aoff[q] = a + u * 16;
    }
    const float eps = L.eps, bo = L.bias[o];
    const float rcp_s = __builtin_amdgcn_rcpf(L.wsum[o]);

    // One tile: form its planes from the registers of `cur` (loaded one tile earlier), then
    // reload `cur` with tile `tn`, whose loads fly during this tile's MFMAs and epilogue. (A
    // second register stage, two tiles of cover, measured slower: 221 vs 166 us for the tail.)
    auto body = [&](Stage& cur, const TileCoord tc, const TileCoord tn) {
        const int b = tc.b;
        const int R0 = tc.ty * TH, C0 = tc.tx * C::TW;  // tile origin in the written grid
        const int oh0 = R0 + off, ow0 = C0 + off;         // ... in this layer's output grid
        cur.to_planes(d, t, oh0 - L.PH, ow0 - L.PW, lds, stage, tid);
        __syncthreads();
        cur.issue(d, t, tn.b, tn.ty * TH + off - L.PH, tn.tx * C::TW + off - L.PW, stage, tid);

        // ---- MFMAs: wave w takes the row pairs rp = w, w+4, ..., both 16-column halves ct ----
        typedef float f4_ __attribute__((ext_vector_type(4)));
#pragma unroll 1
        for (int rpi = 0; rpi < C::NRP / 4; ++rpi) {
            const int rp = wave + 4 * rpi;
            // the 16 x 16 {N, D} tiles of column half ct (16 ct .. +15) of row pair rp
            // one k-step of one column half: the split terms of N (x*c parts) and D (c parts)
            // against the weights' parts, smallest terms first
            auto terms = [&](const bf16x8 (&an)[NP], const bf16x8 (&ad)[NP], const bf16x8 (&b)[NP], f4_& n,
                             f4_& dd) {
#pragma unroll
                for (int sum = 2 * (NP - 1); sum >= 0; --sum)
#pragma unroll
                    for (int i = NP - 1; i >= 0; --i) {
                        const int j = sum - i;
                        if (j < 0 || j >= NP || !use_term<NP>(i, j)) continue;
                        n = __builtin_amdgcn_mfma_f32_16x16x32_bf16(an[i], b[j], n, 0, 0, 0);
                        dd = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad[i], b[j], dd, 0, 0, 0);
                    }
            };
            auto ld_parts = [&](const unsigned char* p, bf16x8 (&an)[NP], bf16x8 (&ad)[NP]) {
#pragma unroll
                for (int i = 0; i < NP; ++i) {
                    an[i] = *reinterpret_cast<const bf16x8*>(p + i * C::PSTRIDE);
                    ad[i] = *reinterpret_cast<const bf16x8*>(p + (NP + i) * C::PSTRIDE);
                }
            };
            // the 16 x 16 {N, D} tiles of column half ct (16 ct .. +15) of row pair rp
            auto mma = [&](int ct, f4_& n, f4_& dd) {
                const unsigned char* tb = lds + (2 * rp * C::IW + 16 * ct) * 16;
                n = (f4_){0.f, 0.f, 0.f, 0.f};
                dd = (f4_){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int q = 0; q < C::NT; ++q) {
                    bf16x8 an[NP], ad[NP];
                    ld_parts(tb + aoff[q], an, ad);
                    terms(an, ad, bw[q], n, dd);
                }
            };

            // both column halves, k-step outer: each k-step's A-fragment reads are in flight
            // together and feed two accumulator pairs, which hides the LDS latency that one half's
            // dependent MFMAs per k-step leave exposed
            auto mma2 = [&](f4_ (&n)[2], f4_ (&dd)[2]) {
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    n[ct] = (f4_){0.f, 0.f, 0.f, 0.f};
                    dd[ct] = (f4_){0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int q = 0; q < C::NT; ++q) {
                    bf16x8 an[2][NP], ad[2][NP];
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct) ld_parts(lds + (2 * rp * C::IW + 16 * ct) * 16 + aoff[q], an[ct], ad[ct]);
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct) terms(an[ct], ad[ct], bw[q], n[ct], dd[ct]);
                }
            };

            // ---- epilogue: this lane holds (o, row oh, columns 16 ct + 4 h .. +3) per half ct ----
            // Every global store is an unconditional buffer store; lanes with nothing to write carry
            // an offset past the resource (dropped by the hardware). The number of stores per tile is
            // thus static, so the wait for the next tile's loads (issued before these stores) does not
            // also wait for the stores to complete.
            if constexpr (EPI != kEpiTail) {
                float yv[2][4], cv[2][4];
                {
                    f4_ accN[2], accD[2];
                    mma2(accN, accD);
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            yv[ct][r] = accN[ct][r] * __builtin_amdgcn_rcpf(accD[ct][r] + eps) + bo;
                            cv[ct][r] = accD[ct][r] * rcp_s;
                        }
                }
                // Transpose the row pair through this wave's LDS region ([o + 8 s][32 columns], pitch
                // 36 floats: conflict-free f4 writes), so that each global store instruction writes
                // eight whole 128-byte rows (lane: channel l>>3, columns 4 (l&7) .. +3) instead of
                // sixteen 64-byte pieces.
                // (y, then cout, through the same region: DS operations of one wave execute in
                // order, so the cout writes cannot overtake the y reads)
                float* wt = reinterpret_cast<float*>(lds + C::LDS_IN) + wave * (16 * kOutPitch);
                const int o8 = lane >> 3, qc = 4 * (lane & 7);
                f4 ry[2], rcv[2];
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
                    *reinterpret_cast<f4*>(wt + (o + 8 * s) * kOutPitch + 16 * ct + 4 * h) =
                        (f4){yv[ct][0], yv[ct][1], yv[ct][2], yv[ct][3]};
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int i = 0; i < 2; ++i) ry[i] = *reinterpret_cast<const f4*>(wt + (o8 + 8 * i) * kOutPitch + qc);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
                    *reinterpret_cast<f4*>(wt + (o + 8 * s) * kOutPitch + 16 * ct + 4 * h) =
                        (f4){cv[ct][0], cv[ct][1], cv[ct][2], cv[ct][3]};
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int i = 0; i < 2; ++i) rcv[i] = *reinterpret_cast<const f4*>(wt + (o8 + 8 * i) * kOutPitch + qc);
                __builtin_amdgcn_wave_barrier();
                const int row0 = oh0 + 2 * rp, col = ow0 + qc;
                const unsigned obytes = (unsigned)(8 * L.Ho * L.Wo) * 4u;
                const __amdgpu_buffer_rsrc_t rsy = plane_rsrc(y + (size_t)b * 8 * L.Ho * L.Wo, obytes);
                const __amdgpu_buffer_rsrc_t rsc = plane_rsrc(yc + (size_t)b * 8 * L.Ho * L.Wo, obytes);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const unsigned rowoff = (unsigned)((o8 * L.Ho + row0 + i) * L.Wo) * 4u;
                    const bool rok = row0 + i < L.Ho;
                    if constexpr (VEC) {  // Wo % 4 == 0: the 4 columns are all in or all out
                        const unsigned so = rok && col < L.Wo ? rowoff + (unsigned)col * 4u : kOOB;
                        st_f4(rsy, so, ry[i]);
                        st_f4(rsc, so, rcv[i]);
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const unsigned so = rok && col + r < L.Wo ? rowoff + (unsigned)(col + r) * 4u : kOOB;
                            st_f32(rsy, so, ry[i][r]);
                            st_f32(rsc, so, rcv[i][r]);
                        }
                    }
                }
                if constexpr (EPI == kEpiPool) {  // 2x2 max-pool of the row pair, both rows in this lane
                    const int Hp = L.Ho >> 1, Wp = L.Wo >> 1, pr = row0 >> 1, pc0 = col >> 1;
                    const unsigned pbytes = (unsigned)(8 * Hp * Wp) * 4u;
                    const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(t.py + (size_t)b * 8 * Hp * Wp, pbytes);
                    const __amdgpu_buffer_rsrc_t rpc = plane_rsrc(t.pc + (size_t)b * 8 * Hp * Wp, pbytes);
                    float pyv[2], pcv[2];
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        pyv[hh] = pool4v(ry[0][2 * hh], ry[0][2 * hh + 1], ry[1][2 * hh], ry[1][2 * hh + 1]);
                        pcv[hh] = pool4v(rcv[0][2 * hh], rcv[0][2 * hh + 1], rcv[1][2 * hh], rcv[1][2 * hh + 1]);
                    }
                    const unsigned prow = (unsigned)((o8 * Hp + pr) * Wp) * 4u;
                    if constexpr (VEC) {  // Wp even, pc0 even: one 8-byte store of both pooled columns
                        const unsigned po = pr < Hp && pc0 < Wp ? prow + (unsigned)pc0 * 4u : kOOB;
                        st_f2(rpy, po, (f2){pyv[0], pyv[1]});
                        st_f2(rpc, po, (f2){pcv[0], pcv[1]});
                    } else {
#pragma unroll
                        for (int hh = 0; hh < 2; ++hh) {
                            const unsigned po = pr < Hp && pc0 + hh < Wp ? prow + (unsigned)(pc0 + hh) * 4u : kOOB;
                            st_f32(rpy, po, pyv[hh]);
                            st_f32(rpc, po, pcv[hh]);
                        }
                    }
                }
            } else {
                // nconv7 (1x1, 8 -> 1) over the 8 channels in lanes l^1, l^2, l^4, then the crop
                const int oh = oh0 + 2 * rp + s;
                const float w7 = t.w7[o];
                const float b7 = t.b7[0], s7 = t.s7[0];
                const unsigned obytes = (unsigned)(t.out_h * t.out_w) * 4u;
                const __amdgpu_buffer_rsrc_t ro = plane_rsrc(y + (size_t)b * t.out_h * t.out_w, obytes);
                const __amdgpu_buffer_rsrc_t rc = plane_rsrc(t.out_c ? t.out_c + (size_t)b * t.out_h * t.out_w : y,
                                                             t.out_c ? obytes : 0);
                const int orow = R0 + 2 * rp + s;
                const bool wr = o == 0 && orow < t.out_h;
                const unsigned rowoff = (unsigned)(orow * t.out_w) * 4u;
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    f4_ accN, accD;
                    mma(ct, accN, accD);
                    const int ow = ow0 + 16 * ct + 4 * h, ocol = C0 + 16 * ct + 4 * h;
                    float n7[4], d7[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float yv = accN[r] * __builtin_amdgcn_rcpf(accD[r] + eps) + bo;
                        const float cv = accD[r] * rcp_s;
                        const bool ok = (unsigned)oh < (unsigned)L.Ho && (unsigned)(ow + r) < (unsigned)L.Wo;
                        n7[r] = ok ? w7 * (yv * cv) : 0.f;
                        d7[r] = ok ? w7 * cv : 0.f;
                    }
#pragma unroll
                    for (int m = 1; m < 8; m <<= 1)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            n7[r] += __shfl_xor(n7[r], m);
                            d7[r] += __shfl_xor(d7[r], m);
                        }
                    float ov[4], oc[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) nconv_epilogue(n7[r], d7[r], t.eps7, b7, s7, ov[r], oc[r]);
                    if constexpr (VEC) {  // out_w % 4 == 0
                        const unsigned so = wr && ocol < t.out_w ? rowoff + (unsigned)ocol * 4u : kOOB;
                        st_f4(ro, so, (f4){ov[0], ov[1], ov[2], ov[3]});
                        st_f4(rc, so, (f4){oc[0], oc[1], oc[2], oc[3]});
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const unsigned so = wr && ocol + r < t.out_w ? rowoff + (unsigned)(ocol + r) * 4u : kOOB;
                            st_f32(ro, so, ov[r]);
                            st_f32(rc, so, oc[r]);
                        }
                    }
                }
            }
        }
        // every wave is done reading the planes before the next tile's are formed (DmaStage's own
        // barrier, after its wait, does this there; a __syncthreads here would drain the DMA)
        if constexpr (!Stage::SELF_SYNC) __syncthreads();
    };

    const int G = (int)gridDim.x;
#pragma unroll 1
    for (; v < ntiles; v += G) {
        const TileCoord tn = v + G < ntiles ? advance(tc) : tc;  // (the last tile re-loads itself)
        body(st, tc, tn);
        tc = tn;
    }
}

// Persistent grid: resident workgroups per CU (by waves per SIMD and LDS) x CUs, a multiple of 8
// (one XCD per blockIdx % 8).
int mfma_grid_blocks(int waves, int lds_bytes) {
    const int cus = dev_cus();
    int per_cu = waves < (160 * 1024) / lds_bytes ? waves : (160 * 1024) / lds_bytes;
    return (cus * (per_cu > 0 ? per_cu : 1) + 7) / 8 * 8;
}

template <int CIN, int K, int MODE, int EPI, int TH, bool DMA, int NP>
void go_mfma(const LayerDev& d, float* y, float* yc, const TailArgs& t, int gh, int gw, hipStream_t st) {
    using C = MfCfg<CIN, K, TH, NP>;
    const int ntiles = ((gw + C::TW - 1) / C::TW) * ((gh + TH - 1) / TH) * d.L.B;
    int grid = mfma_grid_blocks(mf_waves<MODE, DMA, NP>(), mf_lds_bytes<CIN, K, MODE, EPI, TH, NP>(DMA));
    if (ntiles < grid) grid = (ntiles + 7) / 8 * 8;
    if (gw % 4 == 0)
        hipLaunchKernelGGL((fwd_mfma<CIN, K, MODE, EPI, TH, true, DMA, NP>), grid, dim3(kMfThreads), 0, st, d, y, yc, t);
    else
        hipLaunchKernelGGL((fwd_mfma<CIN, K, MODE, EPI, TH, false, DMA, NP>), grid, dim3(kMfThreads), 0, st, d, y, yc, t);
}

// LDS-DMA staging: rows of every source a multiple of 4 floats (16-B vectors never straddle a row
// end), exact 2x upsampling of source b with 8 + 8 channels, per-image sources below 2 GiB.
// Measured slower than register staging at two workgroups per CU (nconv2 198 vs 179 us, the tail
// 272 vs 169 us at B=8 352x1216): compiled in only with -DNCONV_MFMA_DMA=1 (build-time experiment).
#ifndef NCONV_MFMA_DMA
#define NCONV_MFMA_DMA 0
#endif
bool dma_ok(const nconv_layer& L, int cin) {
    if (L.load_mode != NCONV_LOAD_PLAIN && L.load_mode != NCONV_LOAD_UPCAT_SKIP_FIRST &&
        L.load_mode != NCONV_LOAD_UPCAT_UP_FIRST)
        return false;
    const bool up = L.load_mode != NCONV_LOAD_PLAIN;
    auto fine = [](const nconv_src& s) {
        return s.W % 4 == 0 && ((uintptr_t)s.x % 16) == 0 && ((uintptr_t)s.c % 16) == 0 &&
               (long long)s.C * s.H * s.W * 4 < (1LL << 31);
    };
    if (!fine(L.a)) return false;
    if (!up) return L.a.C == cin && L.a.H == L.H && L.a.W == L.W;
    return fine(L.b) && L.a.C == cin / 2 && L.b.C == cin / 2 && L.a.H == L.H && L.a.W == L.W && L.H == 2 * L.b.H &&
           L.W == 2 * L.b.W;
}

template <int CIN, int K, int MODE, int EPI, int TH, int NP>
void go_mfma_np(const LayerDev& d, float* y, float* yc, const TailArgs& t, int gh, int gw, hipStream_t st) {
    if constexpr (MODE == NCONV_LOAD_POOL2 || NP != 2 || !NCONV_MFMA_DMA)
        go_mfma<CIN, K, MODE, EPI, TH, false, NP>(d, y, yc, t, gh, gw, st);
    else if (dma_ok(d.L, CIN))
        go_mfma<CIN, K, MODE, EPI, TH, true, NP>(d, y, yc, t, gh, gw, st);
    else
        go_mfma<CIN, K, MODE, EPI, TH, false, NP>(d, y, yc, t, gh, gw, st);
}

// NP = 2 split parts (bf16x3) or 3 (bf16x9, exact products) by the layer's math
template <int CIN, int K, int MODE, int EPI, int TH>
void go_mfma_any(const LayerDev& d, float* y, float* yc, const TailArgs& t, int gh, int gw, hipStream_t st) {
    if (d.L.math == NCONV_MATH_BF16X9)
        go_mfma_np<CIN, K, MODE, EPI, TH, 3>(d, y, yc, t, gh, gw, st);
    else
        go_mfma_np<CIN, K, MODE, EPI, TH, 2>(d, y, yc, t, gh, gw, st);
}

}  // namespace

int launch_fwd_head(const LayerDev& d2, const TailArgs& t, float* y, float* yc, hipStream_t st, const char** why) {
    // (16-row tiles recompute less of nconv1's halo but fit two workgroups per CU instead of three:
    // 228 vs 215 us at B=8 352x1216)
    if (d2.L.math == NCONV_MATH_BF16X9)
        go_mfma<8, 5, kModeHead, kEpiPool, NCONV_MF_TH_HEAD, false, 3>(d2, y, yc, t, d2.L.Ho, d2.L.Wo, st);
    else
        go_mfma<8, 5, kModeHead, kEpiPool, NCONV_MF_TH_HEAD, false, 2>(d2, y, yc, t, d2.L.Ho, d2.L.Wo, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

// True when the layer has a matrix-core kernel: matrix-core math, 8 output channels, 8 input
// channels with a 5x5 kernel or 16 with a 3x3, stride 1, no dilation / groups (the dispatch of
// launch_fwd_mfma below; nconv_plan reports it).
bool fwd_mfma_supported(const nconv_layer& L, bool tail, bool pool) {
    if ((L.math != NCONV_MATH_BF16X3 && L.math != NCONV_MATH_BF16X9) || L.Cout != 8 || L.KH != L.KW || L.SH != 1 ||
        L.SW != 1 || L.DH != 1 || L.DW != 1 || L.groups != 1)
        return false;
    // MfStage addresses one image's channels of a source through one buffer resource
    auto image_fits = [](const nconv_src& s) { return (long long)s.C * s.H * s.W * 4 < (1LL << 31); };
    const bool up = L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;
    if (!image_fits(L.a) || (up && !image_fits(L.b))) return false;
    if (L.Cin == 8 && L.KH == 5 && L.load_mode == NCONV_LOAD_PLAIN) return !tail;
    if (L.Cin == 8 && L.KH == 5 && L.load_mode == NCONV_LOAD_POOL2) return !tail && !pool;
    if (L.Cin == 16 && L.KH == 3 && !pool)
        return (L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST && !tail) || L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST;
    return false;
}

// Returns true (and launches) when fwd_mfma_supported.
bool launch_fwd_mfma(const LayerDev& d, float* y, float* yc, const TailArgs& t, bool tail, hipStream_t st) {
    const nconv_layer& L = d.L;
    const bool pool = !tail && t.py != nullptr;
    if (!fwd_mfma_supported(L, tail, pool)) return false;
    const int gh = tail ? t.out_h : L.Ho, gw = tail ? t.out_w : L.Wo;
    if (L.Cin == 8 && L.KH == 5 && L.load_mode == NCONV_LOAD_PLAIN && !tail) {
        if (pool)
            go_mfma_any<8, 5, NCONV_LOAD_PLAIN, kEpiPool, NCONV_MF_TH5>(d, y, yc, t, gh, gw, st);
        else
            go_mfma_any<8, 5, NCONV_LOAD_PLAIN, kEpiPlain, NCONV_MF_TH5>(d, y, yc, t, gh, gw, st);
        return true;
    }
    if (L.Cin == 8 && L.KH == 5 && L.load_mode == NCONV_LOAD_POOL2 && !tail && !pool) {
        go_mfma_any<8, 5, NCONV_LOAD_POOL2, kEpiPlain, 8>(d, y, yc, t, gh, gw, st);
        return true;
    }
    if (L.Cin == 16 && L.KH == 3 && !pool) {
        if (L.load_mode == NCONV_LOAD_UPCAT_SKIP_FIRST && !tail) {
            go_mfma_any<16, 3, NCONV_LOAD_UPCAT_SKIP_FIRST, kEpiPlain, 8>(d, y, yc, t, gh, gw, st);
            return true;
        }
        if (L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST) {
            if (tail && L.math == NCONV_MATH_BF16X9)  // (16-row tiles of three-part planes: one workgroup per CU)
                go_mfma_np<16, 3, NCONV_LOAD_UPCAT_UP_FIRST, kEpiTail, 8, 3>(d, y, nullptr, t, gh, gw, st);
            else if (tail)
                go_mfma_np<16, 3, NCONV_LOAD_UPCAT_UP_FIRST, kEpiTail, NCONV_MF_TH_TAIL, 2>(d, y, nullptr, t, gh, gw, st);
            else
                go_mfma_any<16, 3, NCONV_LOAD_UPCAT_UP_FIRST, kEpiPlain, 8>(d, y, yc, t, gh, gw, st);
            return true;
        }
    }
    return false;  // (unreachable: fwd_mfma_supported)
}

}  // namespace nconv
