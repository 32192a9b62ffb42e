// nconv_fwd_head.hip — exact-fp32 fused head: nconv1 on the thresholded sparse depth evaluated
// inside nconv2's tile (its 8-channel output never reaches HBM), nconv2 with the pooled copy for
// down1 (reference: models/step1.py:53-58 and NConv2d.forward :116-149; glue of :62).
//
// Three reductions of the work the unfused exact pair does, all in fp32:
//  1. nconv1 skips zero taps. Its input is {S*c0, c0} with c0 = (S > thresh): on depth of ~5 %
//     density most of a 5x5 window is exactly zero, and adding an exact +-0 product leaves an fp32
//     sum unchanged, so visiting only the nonzero taps in the dense tap order (kh, kw) gives the
//     dense sums bit for bit. Per halo pixel a 25-bit window mask built from per-row bitmasks of
//     the staged depth tile drives the loop (lanes iterate to their wave's largest popcount).
//  2. nconv2's data sums N2 pack two pixels per v_pk_fma_f32 ({N(p), N(p+16)} += w * {xc, xc'}),
//     half the instructions of the {N, D} packing; the halo planes hold column pairs (c, c+16) so
//     each operand is one aligned LDS pair.
//  3. nconv2's confidence mass D2 = sum_i W2[o,i] * (W1[i] * c0) / s1[i] (nconv1's cout = D1 / s1,
//     step1.py:141-147) is one 9x9 convolution of the binary mask c0 with the composed weights
//     W21[o] = sum_i W2[o,i] (x) W1[i] / s1[i] (nconv_head_weights: fp64, rounded once): 81 taps
//     instead of 8 x 25, and it runs on the bf16 matrix cores without leaving fp32: c0 is 0 or 1
//     (exact in bf16) and each fp32 W21 is the exact sum of three bf16 parts (hi, mid, lo: 8
//     significand bits each), so every product is exact and v_mfma_f32_16x16x32_bf16 accumulates
//     the three part sums in fp32, added in the epilogue. All terms are non-negative (softplus
//     weights), so the regrouping keeps the error inside the fp32 bound of the sum, and D2 is
//     exactly 0 where the reference's is (no sample in the 9x9 window). The matrix cores take the
//     work off the vector ALU, which the rest of the kernel keeps busy. Only where nconv2's zero
//     padding truncates its window (tiles within 2 px of the image edge) is the composition not a
//     plain convolution; those tiles sum W2 * c1 from nconv1's c1 as the unfused path does.
// Interior-tile outputs therefore differ from the unfused exact pair only through D2's rounding;
// N2, nconv1 and the edge tiles match it bit for bit.
#include "nconv_prologue.h"

namespace nconv {

namespace {

constexpr int kHT = 256, kHTH = 16, kHTW = 32;
constexpr int kSH = kHTH + 8, kSW = kHTW + 8;     // depth tile: 24 x 40 (two 5x5 halos)
constexpr int kHH = kHTH + 4, kHW = kHTW + 4;     // nconv1 outputs nconv2 reads: 20 x 36
constexpr int kHP = kHW - 16;                     // halo pair slots per row: (c, c + 16), c < 20
constexpr int kHPlane = kHH * kHP;                // f2 per halo pair plane
constexpr int kHPS = kHPlane + 1;                 // plane stride: each plane ends in its own dump slot
// nconv_head_weights' output: the D2 operand fragments (kFrag dwords), then W2 as [ci][kh][kw][o].
// Fragment (b, ks, lane) of v_mfma_f32_16x16x32_bf16's A: row = lane & 15 = 4 * (o - 4b) + part
// (part 3 = 0), k = 8 * (lane >> 4) + j over 12 tap chunks 4 ks + (lane >> 4) of 8:
// chunk q < 9 = taps (q, 0..7), chunk 9 = (0..7, 8), chunk 10 = (8, 8) in j = 0, chunk 11 = none.
constexpr int kFrag = 2 * 3 * 64 * 4;
// D2 operand tables in the plane region (bytes): the B fragment of 8 mask bits from a 256-entry
// table of bf16 {0, 1} octets, the bit octets of each row window (mask rows x columns c..c+7) and
// of each column window (mask column c + 8, rows r..r+7) at the same pitch
constexpr int kLut = 0, kW8R = 4096, kW8C = kW8R + kSH * kSW, kTabEnd = kW8C + kHTH * kSW;
constexpr int kDP = 8 * 64 + 16;                  // D2 transpose: channel pitch (floats)
constexpr int kDOff = (kTabEnd + 15) & ~15;       // D2 transpose region, behind the tables (bytes)

typedef const float __attribute__((address_space(4))) cfloat;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// TR (training): nconv1's outputs of the tile's own 16 x 32 pixels also go to HBM (the backward
// reads them) and the pooled copies come with their argmax words (nconv_fwd_pooled's codes).
template <bool TR>
__global__ __launch_bounds__(kHT) __attribute__((amdgpu_waves_per_eu(5, 8))) void fwd_head_exact(LayerDev d2, TailArgs t, float* __restrict__ y,
                                                      float* __restrict__ yc) {
    const nconv_layer& L = d2.L;  // nconv2 (8 -> 8, 5x5, padding 2); nconv1 through t
    // LDS (30.5 KB: five workgroups per CU): the depth tile's S * c0 (c0 = (S * c0 > thresh): S
    // itself where S > thresh, NaN * 0 = NaN and +-0 otherwise), nconv1's weights, the nonzero
    // masks, and one region holding first the mask pairs of the interior D2, then nconv1's
    // x * c (or, in edge tiles, c) as 8 planes of column pairs
    __shared__ __attribute__((aligned(16))) float sx[kSH * kSW];
    __shared__ __attribute__((aligned(16))) f2 hp[8 * kHPS];  // 8 pair planes, each + a dump slot
    __shared__ __attribute__((aligned(16))) float w1t[25 * 8];       // nconv1 weights [tap][o]
    __shared__ unsigned long long rowmask[kSH];  // nonzero taps of nconv1 (x * c0 or c0 nonzero)
    __shared__ unsigned long long c0row[kSH];    // c0 per mask row (bits = columns)
    __shared__ unsigned c0col[kSW];              // c0 per mask column (bits = rows)
    __shared__ int tile_nan;                     // a NaN among the staged S * c0 (S NaN or -inf)
    static_assert(kDOff + 8 * kDP * 4 <= (int)sizeof(hp), "D2 tables and transpose fit the plane region");
    const int tid = threadIdx.x;
    const int H = L.Ho, W = L.Wo;
    const TileCoord tc = xcd_tile((W + kHTW - 1) / kHTW, (H + kHTH - 1) / kHTH, L.B);
    const int b = tc.b, R0 = tc.ty * kHTH, C0 = tc.tx * kHTW;
    const bool interior = R0 >= 2 && R0 + kHTH + 2 <= H && C0 >= 2 && C0 + kHTW + 2 <= W;

    // ---- stage the depth tile (origin R0 - 4, C0 - 4), its nonzero masks and nconv1's weights ----
    if (tid < kSH) rowmask[tid] = c0row[tid] = 0ull;
    if (tid < kSW) c0col[tid] = 0u;
    if (tid == 0) tile_nan = 0;
    if (tid < 200) w1t[tid] = t.w1[(tid & 7) * 25 + (tid >> 3)];
    __syncthreads();
    {
        const __amdgpu_buffer_rsrc_t rs = plane_rsrc(t.s_in + (size_t)b * H * W, H * W * 4);
        constexpr int NE = (kSH * kSW + kHT - 1) / kHT;
        float sv[NE];
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + kHT * k, r = e / kSW, c = e - (e / kSW) * kSW;
            const int gr = R0 - 4 + r, gc = C0 - 4 + c;
            const bool in = e < kSH * kSW && (unsigned)gr < (unsigned)H && (unsigned)gc < (unsigned)W;
            sv[k] = ld_f32(rs, in ? (unsigned)(gr * W + gc) * 4u : 0x80000000u);
        }
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + kHT * k, r = e / kSW, c = e - (e / kSW) * kSW;
            if (e < kSH * kSW) {
                const float c0 = sv[k] > t.thresh1 ? 1.0f : 0.0f;  // step1.py:53
                const float xc = sv[k] * c0;
                sx[e] = xc;
                if (!(xc == 0.f && c0 == 0.f)) atomicOr(&rowmask[r], 1ull << c);  // NaN counts as nonzero
                if (xc != xc) tile_nan = 1;
                if (c0 != 0.f) {
                    atomicOr(&c0row[r], 1ull << c);
                    atomicOr(&c0col[c], 1u << r);
                }
            }
        }
    }
    __syncthreads();

    // ---- nconv2: thread = pixels (ty, j) and (ty, j + 16) of the 16 x 32 tile ----
    const int ty = tid >> 4, j = tid & 15;
    f2 accN[8], accD[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) accN[o] = accD[o] = (f2){0.f, 0.f};

    // ---- nconv1 on the 20 x 36 halo (origin R0 - 2, C0 - 2), nonzero taps only; writes x * c
    //      (want_c false) or c (want_c true, edge tiles' second pass) into the pair planes ----
    constexpr int NH = (kHH * kHW + kHT - 1) / kHT;  // 3 halo pixels per thread (the last partly)
    // exact_c0: c0 formed per visited tap (the tile holds a NaN S * c0); otherwise every visited
    // tap has c0 = 1 (S * c0 is nonzero only where c0 = 1, or NaN)
    auto nconv1_pass = [&](bool want_c, auto exact_c0) __attribute__((always_inline)) {
#pragma unroll 1
        for (int k = 0; k < NH; ++k) {
            const int e = tid + kHT * k;
            const int r = e / kHW, c = e - (e / kHW) * kHW;
            const int gr = R0 - 2 + r, gc = C0 - 2 + c;
            const bool valid = e < kHH * kHW;
            const bool in = valid && (unsigned)gr < (unsigned)H && (unsigned)gc < (unsigned)W;
            unsigned m = 0;
#ifndef NCONV_HEAD_PROBE_NO_N1  // timing probe only (wrong results): no nconv1 taps
#pragma unroll
            for (int kh = 0; kh < 5; ++kh) m |= (unsigned)((rowmask[(valid ? r : 0) + kh] >> c) & 31ull) << (5 * kh);
#endif
            m = in ? m : 0u;
            // tap tp = 5 kh + kw of the window at halo pixel (r, c) is staged at sxb[35 kh + tp]
            const float* const sxb = sx + r * kSW + c;
            // the first tap peeled: acc = fma(w, v, +0), the FMA into +0 the dense order starts
            // with (bitwise, the sign of zero included: a window without taps takes v = {0, 0}, and
            // a plain product w * 0 would give -0 for a negative eval-mode weight); no zero-filled
            // accumulators carried into the loop (the compiler kept two copies of that fill, one
            // per path into it)
            f2 acc[8];
            {
                const bool any = m != 0u;
                const int tp = any ? __builtin_ctz(m) : 0;
                m &= m - 1u;
                const int kh = (tp * 13) >> 6;
                const float xr = sxb[kh * (kSW - 5) + tp];
                const float xc = any ? xr : 0.f;
                const float cv = decltype(exact_c0)::value ? (xc > t.thresh1 ? 1.0f : 0.0f) : 1.0f;
                const f2 v = (f2){xc, any ? cv : 0.f};
                const f4 wa = reinterpret_cast<const f4*>(w1t)[tp * 2], wb = reinterpret_cast<const f4*>(w1t)[tp * 2 + 1];
                const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
                for (int o = 0; o < 8; ++o) acc[o] = __builtin_elementwise_fma((f2){wv[o], wv[o]}, v, (f2){0.f, 0.f});
            }
            while (m) {
                const int tp = __builtin_ctz(m);
                m &= m - 1;
                const int kh = (tp * 13) >> 6;  // tp / 5 for tp < 25
                const float xc = sxb[kh * (kSW - 5) + tp];
                const f2 v = (f2){xc, decltype(exact_c0)::value ? (xc > t.thresh1 ? 1.0f : 0.0f) : 1.0f};
                const f4 wa = reinterpret_cast<const f4*>(w1t)[tp * 2], wb = reinterpret_cast<const f4*>(w1t)[tp * 2 + 1];
                const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
                for (int o = 0; o < 8; ++o) acc[o] = __builtin_elementwise_fma((f2){wv[o], wv[o]}, v, acc[o]);
            }
            // float offsets of this pixel in a pair plane (.x of pair c, .y of pair c - 16), or the
            // plane's own dump slot: every lane stores, no branches, and the channel's plane is a
            // constant offset (the LDS store's immediate)
            const int h0 = (valid && c < kHP) ? (r * kHP + c) * 2 : kHPlane * 2;
            const int h1 = (valid && c >= 16) ? (r * kHP + c - 16) * 2 + 1 : kHPlane * 2 + 1;
            float* const p0 = reinterpret_cast<float*>(hp) + h0;
            float* const p1 = reinterpret_cast<float*>(hp) + h1;
            // TR: the tile's own pixels (halo rows / columns 2 .. 17 / 2 .. 33) to nconv1's outputs
            const unsigned own = (TR && !want_c && in && (unsigned)(r - 2) < (unsigned)kHTH &&
                                  (unsigned)(c - 2) < (unsigned)kHTW) ? (unsigned)(gr * W + gc) * 4u : 0x80000000u;
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                // outside the image no tap was visited (m = 0): N = D = 0, so cout = 0 and
                // y * cout = b1 * 0 = +-0 -- nconv2's zero padding without a select
                float y1, cc1;
                nconv_epilogue(acc[o].x, acc[o].y, t.eps1, t.b1[o], t.s1[o], y1, cc1);
                if constexpr (TR) {
                    const size_t po1 = ((size_t)b * 8 + o) * H * W;
                    st_f32(plane_rsrc(t.y1 + po1, H * W * 4), own, y1);
                    st_f32(plane_rsrc(t.c1 + po1, H * W * 4), own, cc1);
                }
                const float v = want_c ? cc1 : y1 * cc1;  // nconv2's staged x * c, or c
                p0[o * kHPS * 2] = v;
                p1[o * kHPS * 2] = v;
            }
        }
    };
    auto nconv1_planes = [&](bool want_c) __attribute__((always_inline)) {
        if (tile_nan) nconv1_pass(want_c, std::true_type{});
        else nconv1_pass(want_c, std::false_type{});
    };
    nconv1_planes(false);
    __syncthreads();

    // nconv2's weights transposed to [ci][kh][kw][o] (nconv_head_weights, after W21): one kernel
    // row's 40 weights are contiguous -- three scalar loads instead of sixteen
    const cfloat* w2t = (const cfloat*)L.waux + kFrag;
    // N2 (or, for edge tiles, D2 from c1) over the 8 halo pair planes: {N(p), N(p+16)} += w * pair
    auto sum_planes = [&](f2 (&acc)[8]) __attribute__((always_inline)) {
#pragma unroll 1
        for (int ci = 0; ci < 8; ++ci) {
            const f2* row = hp + ci * kHPS + ty * kHP + j;
            const cfloat* wr = w2t + ci * 200;
#pragma unroll 1
            for (int kh = 0; kh < 5; ++kh, row += kHP, wr += 40) {
                f2 v[5];
#pragma unroll
                for (int kw = 0; kw < 5; ++kw) v[kw] = row[kw];
#pragma unroll
                for (int kw = 0; kw < 5; ++kw)
#pragma unroll
                    for (int o = 0; o < 8; ++o) {
                        const float wv = wr[kw * 8 + o];
                        acc[o] = __builtin_elementwise_fma((f2){wv, wv}, v[kw], acc[o]);
                    }
            }
        }
    };
#ifndef NCONV_HEAD_PROBE_NO_N2  // timing probe only (wrong results): no nconv2 data sums
    sum_planes(accN);
#endif
    __syncthreads();  // every wave is done reading the x * c planes
    if (!interior) {
        // edge tile: nconv2's zero padding truncates the window -- D2 = W2 * c1 as the unfused
        // path, with c1 from a second nonzero-tap pass of nconv1 into the planes
        nconv1_planes(true);
        __syncthreads();
        sum_planes(accD);
    } else {
        // interior D2 on the matrix cores, after N2 (no D2 registers live through nconv1 and N2):
        // the operand tables in the freed plane region, each GEMM block's results straight to the
        // transpose region behind them, then to the thread's pixels (ty, j), (ty, j + 16). Wave w's
        // pixels (4w + (nb >> 1), 16 (nb & 1) + n) are the 16 columns of GEMM block nb; lane (g, n)
        // holds D2 of channels g (bb = 0) and 4 + g (bb = 1)
        unsigned char* const tb = reinterpret_cast<unsigned char*>(hp);
        float* const dt = reinterpret_cast<float*>(tb + kDOff);
        {   // table entry tid: bf16 1.0 where bit j of tid is set
            unsigned dq[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                dq[i] = ((tid >> (2 * i)) & 1u) * 0x3F80u + ((tid >> (2 * i + 1)) & 1u) * 0x3F800000u;
            reinterpret_cast<uint4*>(tb + kLut)[tid] = make_uint4(dq[0], dq[1], dq[2], dq[3]);
        }
        for (int e = tid; e < kSH * kSW; e += kHT) {
            const int r = e / kSW, c = e - r * kSW;
            tb[kW8R + e] = (unsigned char)(c0row[r] >> c);
            if (r < kHTH) tb[kW8C + e] = c < kHTW ? (unsigned char)(c0col[c + 8] >> r) : 0;
        }
        __syncthreads();
        {
            const int lane = tid & 63, g = lane >> 4, n = lane & 15, w = tid >> 6;
            const uint4* fr = reinterpret_cast<const uint4*>(L.waux) + lane;
            bf16x8 A[2][3];
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                for (int ks = 0; ks < 3; ++ks) A[bb][ks] = __builtin_bit_cast(bf16x8, fr[(bb * 3 + ks) * 64]);
            // byte offsets of this lane's chunk octets for K step ks (pixel (4w, n) + per-block immediates)
            const int pb = w * 4 * kSW + n;
            const int o0 = kW8R + g * kSW + pb, o1 = kW8R + (4 + g) * kSW + pb;
            const int o2 = g == 0 ? kW8R + 8 * kSW + pb : (g == 1 ? kW8C + pb : kW8R + 8 * kSW + 8 + pb);
#pragma unroll
            for (int nb = 0; nb < 8; ++nb) {
                const int po = (nb >> 1) * kSW + 16 * (nb & 1);
                const bf16x8 B0 = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(tb + kLut)[tb[o0 + po]]);
                const bf16x8 B1 = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(tb + kLut)[tb[o1 + po]]);
                const bf16x8 B2 = __builtin_bit_cast(bf16x8, reinterpret_cast<const uint4*>(tb + kLut)[tb[o2 + po]]);
#pragma unroll
                for (int bb = 0; bb < 2; ++bb) {
                    f4 acc = (f4){0.f, 0.f, 0.f, 0.f};
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[bb][0], B0, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[bb][1], B1, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[bb][2], B2, acc, 0, 0, 0);
                    dt[(4 * bb + g) * kDP + (4 * w + (nb >> 1)) * kHTW + 16 * (nb & 1) + n] =
                        (acc.x + acc.y) + acc.z;  // hi + mid, then + lo
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int o = 0; o < 8; ++o) accD[o] = (f2){dt[o * kDP + ty * kHTW + j], dt[o * kDP + ty * kHTW + j + 16]};
    }

    // ---- epilogue: y, cout and their 2x2 max-pooled copies (the input of down1) ----
    constexpr unsigned OOB = 0x80000000u;
    const int oh = R0 + ty;
    const size_t plane = (size_t)H * W;
    const int pbytes = (int)(plane * 4);
    const int Hp = H >> 1, Wp = W >> 1;
    const size_t pplane = (size_t)Hp * Wp;
    const int ppbytes = (int)(pplane * 4);
    // training: the pooled pair and argmax leave from the window's top-left lane; inference: the
    // pooled y from the even rows' even lanes, the pooled cout from the odd rows' (see below)
    unsigned so[2], po[2], pcy[2], pcc[2];
    const bool pool_col = ((j & 1) == 0) && (oh >> 1) < Hp;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ow = C0 + j + 16 * h;
        so[h] = (oh < H && ow < W) ? (unsigned)(oh * W + ow) * 4u : OOB;
        const unsigned pp = (pool_col && (ow >> 1) < Wp) ? (unsigned)((oh >> 1) * Wp + (ow >> 1)) * 4u : OOB;
        po[h] = (ty & 1) == 0 ? pp : OOB;
        pcy[h] = po[h];
        pcc[h] = (ty & 1) ? pp : OOB;
    }
#pragma unroll
    for (int o = 0; o < 8; ++o) {
        float yv[2], cv[2];
        const float s = L.wsum[o], bo = L.bias[o];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float N = h ? accN[o].y : accN[o].x, D = h ? accD[o].y : accD[o].x;
            nconv_epilogue(N, D, L.eps, bo, s, yv[h], cv[h]);
        }
        const size_t ofs = ((size_t)b * 8 + o) * plane;
        const __amdgpu_buffer_rsrc_t ry = plane_rsrc(y + ofs, pbytes), rc = plane_rsrc(yc + ofs, pbytes);
        const size_t pofs = ((size_t)b * 8 + o) * pplane;
        const __amdgpu_buffer_rsrc_t rpy = plane_rsrc(t.py + pofs, ppbytes), rpc = plane_rsrc(t.pc + pofs, ppbytes);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            st_f32(ry, so[h], yv[h]);
            st_f32(rc, so[h], cv[h]);
#ifdef NCONV_HEAD_PROBE_NO_POOL  // timing probe only (wrong results): no pooled copies
            continue;
#endif
            if constexpr (TR) {  // the first maximum's slot too (the backward's routing)
                // window (r, c) (r, c+1) (r+1, c) (r+1, c+1): lanes l, l^1, l^16, l^17 (torch order)
                const float yb = shfl_xor16(yv[h]), cb = shfl_xor16(cv[h]);
                const float ya = shfl_xor1(yv[h]), yd = shfl_xor1(yb), ca = shfl_xor1(cv[h]), cd = shfl_xor1(cb);
                int ay, ac;
                st_f32(rpy, po[h], pool4(yv[h], ya, yb, yd, ay));
                st_f32(rpc, po[h], pool4(cv[h], ca, cb, cd, ac));
                st_f32(plane_rsrc((const float*)(t.parg + pofs), ppbytes), po[h],
                       __builtin_bit_cast(float, (unsigned)(ay | (ac << 2))));
            } else {
                // the value alone: one v_permlane16_swap of (y, cout) leaves rows {y0, c0, y2, c2}
                // and {y1, c1, y3, c3} (16-lane rows = tile rows), so their maximum is y's vertical
                // pair maximum in the even rows and cout's in the odd rows; then the column pair
                const float vm = pair_rows_max(yv[h], cv[h]);
                const float pm = __builtin_elementwise_maximum(vm, shfl_xor1(vm));
                st_f32(rpy, pcy[h], pm);
                st_f32(rpc, pcc[h], pm);
            }
        }
    }
}

// W21[o][qh][qw] = sum_i (1 / s1[i]) sum_{kh + kh' = qh, kw + kw' = qw} W2[o][i][kh][kw] W1[i][kh'][kw']
// in fp64, rounded once to fp32 (s1 = nconv1's weight sums, as the forward's cout = D1 / s1 uses
// them), then split exactly into bf16 hi + mid + lo (truncations: each remainder is exact in fp32
// and the last has at most 8 significant bits) and written into the D2 fragments (kFrag). One
// 64-lane block per (qh, qw): lane (o, i) forms channel i's term, the 8 terms of an output are
// summed over lanes in a fixed butterfly order; block 81 writes W2 transposed to [i][kh][kw][o],
// block 82 zeroes the fragment slots no tap fills.
__device__ __forceinline__ int frag_slot(int o, int part, int chunk, int j) {
    const int row = 4 * (o & 3) + part, ks = chunk >> 2, g = chunk & 3;
    return (((o >> 2) * 3 + ks) * 64 + g * 16 + row) * 8 + j;  // bf16 index
}

// One unit of nconv_head_weights per wave: units 0..80 the composed tap (qh, qw) = (u / 9, u % 9),
// 81 the transposed W2, 82 the zero padding of the fragment table. s1i = s1[lane & 7].
constexpr int kHeadUnits = 83;
__device__ __forceinline__ void head_weights_unit(const float* __restrict__ w1, float s1i,
                                                  const float* __restrict__ w2, float* __restrict__ out,
                                                  int blk, int lane) {
    unsigned short* const fb = reinterpret_cast<unsigned short*>(out);
    if (blk == 81) {
        for (int e = lane; e < 1600; e += 64) {  // W2t[ci][kh][kw][o] = W2[o][ci][kh][kw]
            const int o = e & 7, kk = (e >> 3) % 25, ci = e / 200;
            out[kFrag + e] = w2[(o * 8 + ci) * 25 + kk];
        }
        return;
    }
    if (blk == 82) {
        for (int e = lane; e < kFrag * 2; e += 64) {
            const int j = e & 7, l = (e >> 3) & 63, ks = (e >> 9) % 3;
            const int part = l & 3, chunk = 4 * ks + (l >> 4);
            if (part == 3 || chunk == 11 || (chunk == 10 && j != 0)) fb[e] = 0;
        }
        return;
    }
    const int qh = blk / 9, qw = blk % 9, o = lane >> 3, i = lane & 7;
    // all 25 (kh, kw) unrolled, the valid ones accumulated in (kh, kw) order by explicit fp64 FMAs:
    // every load of the unit is issued up front (a loop with data-dependent bounds waited on each)
    double si = 0.0;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh) {
        const int kh1 = qh - kh;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
            const int kw1 = qw - kw;
            const bool v = kh1 >= 0 && kh1 <= 4 && kw1 >= 0 && kw1 <= 4;
            const double a = (double)w2[((o * 8 + i) * 5 + kh) * 5 + kw];
            const double b = (double)w1[v ? (i * 5 + kh1) * 5 + kw1 : 0];
            si = v ? __builtin_fma(a, b, si) : si;
        }
    }
    si /= (double)s1i;
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) si += __shfl_xor(si, m);
    if (i == 0) {
        const float w = (float)si;
        const float hi = __uint_as_float(__float_as_uint(w) & 0xFFFF0000u);
        const float r = w - hi;
        const float mid = __uint_as_float(__float_as_uint(r) & 0xFFFF0000u);
        const float lo = r - mid;
        const int chunk = qw < 8 ? qh : (qh < 8 ? 9 : 10);
        const int j = qw < 8 ? qw : (qh < 8 ? qh : 0);
        fb[frag_slot(o, 0, chunk, j)] = (unsigned short)(__float_as_uint(hi) >> 16);
        fb[frag_slot(o, 1, chunk, j)] = (unsigned short)(__float_as_uint(mid) >> 16);
        fb[frag_slot(o, 2, chunk, j)] = (unsigned short)(__float_as_uint(lo) >> 16);
    }
}

__global__ __launch_bounds__(64) void head_weights(const float* __restrict__ w1, const float* __restrict__ s1,
                                                   const float* __restrict__ w2, float* __restrict__ out) {
    head_weights_unit(w1, s1[threadIdx.x & 7], w2, out, blockIdx.x, threadIdx.x);
}

// The inference weight prologue in one launch (nconv_weight_prologue): blocks [0, nprep) the
// normalisers of the layers (prep_block, no softplus: eval mode), then the head's units four per
// block (a wave each; nconv1's s1 recomputed by the wave with row_sum_wave, the arithmetic of
// prep_block, so bitwise the normaliser nconv_weight_prep writes), then one block per phase-weight
// layer. Every block reads the weights only, so no order between the roles is needed.
__global__ __launch_bounds__(kPrepThreads) void weight_prologue(PrepArgs prep, int nprep, const float* __restrict__ w1,
                                                                 const float* __restrict__ w2, float* __restrict__ w21,
                                                                 PhaseArgs ph, int nphase) {
    const int nhead = w21 ? (kHeadUnits + 3) / 4 : 0;
    int blk = blockIdx.x;
    if (blk < nprep) {
        prep_block(prep.w[blk], prep.s[blk], prep.cout[blk], prep.fan_in[blk], 0);
        return;
    }
    blk -= nprep;
    if (blk < nhead) {
        const int lane = threadIdx.x & 63, unit = 4 * blk + (threadIdx.x >> 6);
        if (unit >= kHeadUnits) return;
        // s1 as row_sum_wave sums each row (lane-strided terms from +0, then the butterfly), the
        // eight rows' loads issued together (one row after another waited on each)
        float v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = lane < 25 ? w1[r * 25 + lane] : 0.f;
        float s1i = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            float sr = 0.f;
            if (lane < 25) sr += v[r];
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) sr += __shfl_xor(sr, m);
            if ((lane & 7) == r) s1i = sr;
        }
        head_weights_unit(w1, s1i, w2, w21, unit, lane);
        return;
    }
    blk -= nhead;
    if (blk < nphase) phase_block(ph.w[blk], ph.cin[blk], ph.ci0[blk], ph.out[blk]);
}

// The training weight prologue in one launch (nconv_train_prologue): EnforcePos in place and every
// weight-only input of the training pass formed from the transformed weights. Blocks [0, nprep):
// the layers no other role reads (prep_block: softplus in place, then the normalisers). Then
// kTrainHeadBlocks head blocks, eight head units each (a wave per unit): each stages nconv1's and
// nconv2's weights into LDS through enforce_pos and works from there; the writes of the
// transformed weights (and the normalisers) wait for every head block's staging reads, so the
// block that finishes last (a counter in *sync, left at 0 for the next call) writes them. Then
// one block per phase layer, the layer's only reader: staged the same way, written back, its
// normalisers, phase weights and box weights. Every output is bitwise what weight_prep +
// head_weights + phase_weights + box_weights write (the same device functions on the same values).
// 512 threads per workgroup: eight head units per head workgroup; the prep and phase roles use
// the first 256 (the others leave before any barrier).
constexpr int kTrainProThreads = 512, kTrainHeadBlocks = (kHeadUnits + 7) / 8;
__global__ __launch_bounds__(kTrainProThreads) void train_prologue(PrepArgs prep, int nprep, float* w1, float* w2,
                                                               float* s1, float* s2, int sp1, int sp2,
                                                               float* w21, unsigned* sync, TrainPhaseArgs ph,
                                                               int nphase) {
    __shared__ float lw[1800 + 8];  // head: W1 (200), W2 (1600), s1 (8); phase: W (1152)
    __shared__ int last;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int blk = blockIdx.x;
    if (blk < nprep) {
        if (tid < kPrepThreads) prep_block(prep.w[blk], prep.s[blk], prep.cout[blk], prep.fan_in[blk], prep.softplus[blk]);
        return;
    }
    blk -= nprep;
    if (w21) {
        if (blk < kTrainHeadBlocks) {
            for (int e = tid; e < 1800; e += kTrainProThreads) {
                const bool one = e < 200;
                const float v = one ? w1[e] : w2[e - 200];
                lw[e] = (one ? sp1 : sp2) ? enforce_pos(v) : v;
            }
            __syncthreads();
            {  // s1: prep_block's wave sums (a wave per row)
                const float v = row_sum_wave(lw + wave * 25, 25, lane);
                if (lane == 0) lw[1800 + wave] = v;
            }
            __syncthreads();
            const int u = 8 * blk + wave;
            if (u < kHeadUnits) head_weights_unit(lw, lw[1800 + (lane & 7)], lw + 200, w21, u, lane);
            // every head block's reads of w1 / w2 are done before it counts itself
            __syncthreads();
            if (tid == 0) {
                __threadfence();
                last = atomicAdd(sync, 1u) == (unsigned)(kTrainHeadBlocks - 1);
            }
            __syncthreads();
            if (!last) return;
            __threadfence();
            for (int e = tid; e < 1800; e += kTrainProThreads) {
                if (e < 200) {
                    if (sp1) w1[e] = lw[e];
                } else if (sp2) {
                    w2[e - 200] = lw[e];
                }
            }
            if (tid < 8) s1[tid] = lw[1800 + tid];
            {  // s2 (rows of 200)
                const float v = row_sum_wave(lw + 200 + wave * 200, 200, lane);
                if (lane == 0) s2[wave] = v;
            }
            if (tid == 0) atomicExch(sync, 0u);
            return;
        }
        blk -= kTrainHeadBlocks;
    }
    if (blk < nphase && tid < kPrepThreads) {
        float* W = ph.w[blk];
        const int sp = ph.sp[blk];
        for (int e = tid; e < 1152; e += kPrepThreads) lw[e] = sp ? enforce_pos(W[e]) : W[e];
        __syncthreads();
        if (sp)
            for (int e = tid; e < 1152; e += kPrepThreads) W[e] = lw[e];
        for (int o = wave; o < 8; o += kPrepThreads / 64) {
            const float v = row_sum_wave(lw + o * 144, 144, lane);
            if (lane == 0) ph.s[blk][o] = v;
        }
        phase_block(lw, 16, ph.ci0[blk], ph.out[blk]);
        if (float* bx = ph.box[blk])
            for (int e = tid; e < 1024; e += kPrepThreads) bx[e] = box_weight(lw, ph.ci0[blk], e);
    }
}

}  // namespace

int launch_fwd_head_exact(const LayerDev& d2, const TailArgs& t, float* y, float* yc, hipStream_t st,
                          const char** why) {
    const nconv_layer& L = d2.L;
    dim3 grid(((L.Wo + kHTW - 1) / kHTW) * ((L.Ho + kHTH - 1) / kHTH) * L.B);  // see xcd_tile
    if (t.y1) hipLaunchKernelGGL(fwd_head_exact<true>, grid, dim3(kHT), 0, st, d2, t, y, yc);
    else hipLaunchKernelGGL(fwd_head_exact<false>, grid, dim3(kHT), 0, st, d2, t, y, yc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

int launch_weight_prologue(int n, float* const* w, const int* cout, const int* fan_in, float* const* s,
                           const float* w1, const float* w2, float* w21, int nphase, const float* const* pw,
                           const int* pcin, const int* pup_first, float* const* pout, hipStream_t st,
                           const char** why) {
    if (n < 0 || n > PrepArgs::kMax || nphase < 0 || nphase > PhaseArgs::kMax) {
        *why = "too many layers for one nconv_weight_prologue launch (max 32 normalisers, 8 phase layers)";
        return -22;
    }
    PrepArgs a{};
    for (int i = 0; i < n; ++i) {
        a.w[i] = w[i];
        a.s[i] = s[i];
        a.cout[i] = cout[i];
        a.fan_in[i] = fan_in[i];
    }
    PhaseArgs p{};
    for (int i = 0; i < nphase; ++i) {
        p.w[i] = pw[i];
        p.out[i] = pout[i];
        p.ci0[i] = pup_first[i];
        p.cin[i] = pcin[i];
    }
    const int blocks = n + (w21 ? (kHeadUnits + 3) / 4 : 0) + nphase;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(weight_prologue, dim3(blocks), dim3(kPrepThreads), 0, st, a, n, w1, w2, w21, p, nphase);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

int launch_head_weights(const float* w1, const float* s1, const float* w2, float* out, hipStream_t st,
                        const char** why) {
    hipLaunchKernelGGL(head_weights, dim3(kHeadUnits), dim3(64), 0, st, w1, s1, w2, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

int launch_train_prologue(int n, float* const* w, const int* cout, const int* fan_in, const int* sp,
                          float* const* s, int head1, int head2, float* w21, unsigned* sync, int nphase,
                          const int* players, const int* pup_first, float* const* pout, float* const* pbox,
                          hipStream_t st, const char** why) {
    if (n < 0 || n > PrepArgs::kMax || nphase < 0 || nphase > TrainPhaseArgs::kMax) {
        *why = "too many layers for one nconv_train_prologue launch (max 32 layers, 8 phase layers)";
        return -22;
    }
    PrepArgs a{};
    TrainPhaseArgs p{};
    int nprep = 0;
    for (int i = 0; i < n; ++i) {
        bool own = w21 && (i == head1 || i == head2);
        for (int k = 0; k < nphase; ++k) own = own || players[k] == i;
        if (own) continue;
        a.w[nprep] = w[i];
        a.s[nprep] = s[i];
        a.cout[nprep] = cout[i];
        a.fan_in[nprep] = fan_in[i];
        a.softplus[nprep] = sp ? sp[i] : 0;
        ++nprep;
    }
    for (int k = 0; k < nphase; ++k) {
        const int i = players[k];
        p.w[k] = w[i];
        p.s[k] = s[i];
        p.out[k] = pout[k];
        p.box[k] = pbox ? pbox[k] : nullptr;
        p.sp[k] = sp ? sp[i] : 0;
        p.ci0[k] = pup_first[k];
    }
    float *w1 = nullptr, *w2 = nullptr, *s1 = nullptr, *s2 = nullptr;
    int sp1 = 0, sp2 = 0;
    if (w21) {
        w1 = w[head1], w2 = w[head2], s1 = s[head1], s2 = s[head2];
        sp1 = sp ? sp[head1] : 0, sp2 = sp ? sp[head2] : 0;
    }
    const int blocks = nprep + (w21 ? kTrainHeadBlocks : 0) + nphase;
    if (blocks == 0) return 0;
    static_assert(kTrainProThreads / 64 == 8, "a wave per nconv1 / nconv2 row");
    hipLaunchKernelGGL(train_prologue, dim3(blocks), dim3(kTrainProThreads), 0, st, a, nprep, w1, w2, s1, s2, sp1, sp2,
                       w21, sync, p, nphase);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
