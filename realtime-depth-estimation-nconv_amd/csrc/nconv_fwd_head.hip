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
//     instead of 8 x 25. All terms are non-negative (softplus weights, c0 in {0, 1}), so the
//     regrouping keeps the error inside the fp32 bound of the sum, and D2 is exactly 0 where the
//     reference's is (no sample in the 9x9 window). Only where nconv2's zero padding truncates its
//     window (tiles within 2 px of the image edge) is the composition not a plain convolution;
//     those tiles sum W2 * c1 from nconv1's c1 as the unfused path does.
// Interior-tile outputs therefore differ from the unfused exact pair only through D2's rounding;
// N2, nconv1 and the edge tiles match it bit for bit.
#include "nconv_internal.h"

namespace nconv {

namespace {

constexpr int kHT = 256, kHTH = 16, kHTW = 32;
constexpr int kSH = kHTH + 8, kSW = kHTW + 8;     // depth tile: 24 x 40 (two 5x5 halos)
constexpr int kHH = kHTH + 4, kHW = kHTW + 4;     // nconv1 outputs nconv2 reads: 20 x 36
constexpr int kHP = kHW - 16;                     // halo pair slots per row: (c, c + 16), c < 20
constexpr int kCP = kSW - 16;                     // mask pair slots per row: c < 24
constexpr int kHPlane = kHH * kHP;                // f2 per halo pair plane
constexpr int kHPS = kHPlane + 1;                 // plane stride: each plane ends in its own dump slot
constexpr int kW21 = 9 * 8 * 9;                   // composed weights, then W2 as [ci][kh][kw][o]

typedef const float __attribute__((address_space(4))) cfloat;

// TR (training): nconv1's outputs of the tile's own 16 x 32 pixels also go to HBM (the backward
// reads them) and the pooled copies come with their argmax words (nconv_fwd_pooled's codes).
template <bool TR>
__global__ __launch_bounds__(kHT) void fwd_head_exact(LayerDev d2, TailArgs t, float* __restrict__ y,
                                                      float* __restrict__ yc) {
    const nconv_layer& L = d2.L;  // nconv2 (8 -> 8, 5x5, padding 2); nconv1 through t
    // LDS (30.5 KB: five workgroups per CU): the depth tile's S * c0 (c0 = (S * c0 > thresh): S
    // itself where S > thresh, NaN * 0 = NaN and +-0 otherwise), nconv1's weights, the nonzero
    // masks, and one region holding first the mask pairs of the interior D2, then nconv1's
    // x * c (or, in edge tiles, c) as 8 planes of column pairs
    __shared__ __attribute__((aligned(16))) float sx[kSH * kSW];
    __shared__ __attribute__((aligned(16))) f2 hp[8 * kHPS];  // 8 pair planes, each + a dump slot
    __shared__ __attribute__((aligned(16))) float w1t[25 * 8];       // nconv1 weights [tap][o]
    __shared__ unsigned long long rowmask[kSH];
    f2* const c0p = hp;  // {c0(c), c0(c + 16)}, kSH x kCP, until the interior D2 is done
    static_assert(kSH * kCP <= 8 * kHPS, "mask pairs fit the plane region");
    const int tid = threadIdx.x;
    const int H = L.Ho, W = L.Wo;
    const TileCoord tc = xcd_tile((W + kHTW - 1) / kHTW, (H + kHTH - 1) / kHTH, L.B);
    const int b = tc.b, R0 = tc.ty * kHTH, C0 = tc.tx * kHTW;
    const bool interior = R0 >= 2 && R0 + kHTH + 2 <= H && C0 >= 2 && C0 + kHTW + 2 <= W;

    // ---- stage the depth tile (origin R0 - 4, C0 - 4), its nonzero masks and nconv1's weights ----
    if (tid < kSH) rowmask[tid] = 0ull;
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
                if (c < kCP) reinterpret_cast<float*>(c0p)[(r * kCP + c) * 2] = c0;
                if (c >= 16) reinterpret_cast<float*>(c0p)[(r * kCP + c - 16) * 2 + 1] = c0;
                if (!(xc == 0.f && c0 == 0.f)) atomicOr(&rowmask[r], 1ull << c);  // NaN counts as nonzero
            }
        }
    }
    __syncthreads();

    // ---- nconv2: thread = pixels (ty, j) and (ty, j + 16) of the 16 x 32 tile ----
    const int ty = tid >> 4, j = tid & 15;
    f2 accN[8], accD[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) accN[o] = accD[o] = (f2){0.f, 0.f};

#ifdef NCONV_HEAD_PROBE_NO_D2  // timing probe only (wrong results): no interior confidence sums
    if (false) {
#else
    if (interior) {
#endif
        // D2 = W21 * c0 over the 9 x 9 window (mask tile origin R0 - 4 = output row - 4); rows in
        // two steps of <= 5 taps: 40 weights in SGPRs at a time, as nconv2's rows
        const cfloat* w21 = (const cfloat*)L.waux;  // [qh][o][qw]
#pragma unroll 1
        for (int qh = 0; qh < 9; ++qh) {
            const f2* row = c0p + (ty + qh) * kCP + j;
            const cfloat* wr = w21 + qh * 72;
            f2 v[9];
#pragma unroll
            for (int qw = 0; qw < 9; ++qw) v[qw] = row[qw];
#pragma unroll
            for (int qw = 0; qw < 5; ++qw)
#pragma unroll
                for (int o = 0; o < 8; ++o) {
                    const float wv = wr[o * 9 + qw];
                    accD[o] = __builtin_elementwise_fma((f2){wv, wv}, v[qw], accD[o]);
                }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int qw = 5; qw < 9; ++qw)
#pragma unroll
                for (int o = 0; o < 8; ++o) {
                    const float wv = wr[o * 9 + qw];
                    accD[o] = __builtin_elementwise_fma((f2){wv, wv}, v[qw], accD[o]);
                }
        }
    }
    __syncthreads();  // the mask pairs are dead: the region becomes nconv1's planes

    // ---- nconv1 on the 20 x 36 halo (origin R0 - 2, C0 - 2), nonzero taps only; writes x * c
    //      (want_c false) or c (want_c true, edge tiles' second pass) into the pair planes ----
    constexpr int NH = (kHH * kHW + kHT - 1) / kHT;  // 3 halo pixels per thread (the last partly)
    auto nconv1_planes = [&](bool want_c) {
#pragma unroll 1
        for (int k = 0; k < NH; ++k) {
            const int e = tid + kHT * k;
            const int r = e / kHW, c = e - (e / kHW) * kHW;
            const int gr = R0 - 2 + r, gc = C0 - 2 + c;
            const bool valid = e < kHH * kHW;
            const bool in = valid && (unsigned)gr < (unsigned)H && (unsigned)gc < (unsigned)W;
            f2 acc[8];
#pragma unroll
            for (int o = 0; o < 8; ++o) acc[o] = (f2){0.f, 0.f};
            unsigned m = 0;
#ifdef NCONV_HEAD_PROBE_NO_N1  // timing probe only (wrong results): no nconv1 taps
            if (false) {
#else
            if (in) {
#endif
#pragma unroll
                for (int kh = 0; kh < 5; ++kh) m |= (unsigned)((rowmask[r + kh] >> c) & 31ull) << (5 * kh);
            }
            while (m) {
                const int tp = __builtin_ctz(m);
                m &= m - 1;
                const int kh = (tp * 13) >> 6, kw = tp - 5 * kh;  // tp / 5 for tp < 25
                const float xc = sx[(r + kh) * kSW + c + kw];
                const f2 v = (f2){xc, xc > t.thresh1 ? 1.0f : 0.0f};  // {S * c0, c0}
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
    nconv1_planes(false);
    __syncthreads();

    // nconv2's weights transposed to [ci][kh][kw][o] (nconv_head_weights, after W21): one kernel
    // row's 40 weights are contiguous -- three scalar loads instead of sixteen
    const cfloat* w2t = (const cfloat*)L.waux + kW21;
    // N2 (or, for edge tiles, D2 from c1) over the 8 halo pair planes: {N(p), N(p+16)} += w * pair
    auto sum_planes = [&](f2 (&acc)[8]) {
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
    if (!interior) {
        // edge tile: nconv2's zero padding truncates the window -- D2 = W2 * c1 as the unfused
        // path, with c1 from a second nonzero-tap pass of nconv1 into the planes
        __syncthreads();  // every wave is done reading the x * c planes
        nconv1_planes(true);
        __syncthreads();
        sum_planes(accD);
    }

    // ---- epilogue: y, cout and their 2x2 max-pooled copies (the input of down1) ----
    constexpr unsigned OOB = 0x80000000u;
    const int oh = R0 + ty;
    const size_t plane = (size_t)H * W;
    const int pbytes = (int)(plane * 4);
    const int Hp = H >> 1, Wp = W >> 1;
    const size_t pplane = (size_t)Hp * Wp;
    const int ppbytes = (int)(pplane * 4);
    unsigned so[2], po[2];
    const bool pool_lane = ((ty & 1) == 0) && ((j & 1) == 0) && (oh >> 1) < Hp;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ow = C0 + j + 16 * h;
        so[h] = (oh < H && ow < W) ? (unsigned)(oh * W + ow) * 4u : OOB;
        po[h] = (pool_lane && (ow >> 1) < Wp) ? (unsigned)((oh >> 1) * Wp + (ow >> 1)) * 4u : OOB;
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
            // window (r, c) (r, c+1) (r+1, c) (r+1, c+1): lanes l, l^1, l^16, l^17 (torch order)
            const float yb = shfl_xor16(yv[h]), cb = shfl_xor16(cv[h]);
            const float ya = shfl_xor1(yv[h]), yd = shfl_xor1(yb), ca = shfl_xor1(cv[h]), cd = shfl_xor1(cb);
            if constexpr (TR) {  // the first maximum's slot too (the backward's routing)
                int ay, ac;
                st_f32(rpy, po[h], pool4(yv[h], ya, yb, yd, ay));
                st_f32(rpc, po[h], pool4(cv[h], ca, cb, cd, ac));
                st_f32(plane_rsrc((const float*)(t.parg + pofs), ppbytes), po[h],
                       __builtin_bit_cast(float, (unsigned)(ay | (ac << 2))));
            } else {
                st_f32(rpy, po[h], pool4v(yv[h], ya, yb, yd));
                st_f32(rpc, po[h], pool4v(cv[h], ca, cb, cd));
            }
        }
    }
}

// W21[qh][o][qw] = sum_i (1 / s1[i]) sum_{kh + kh' = qh, kw + kw' = qw} W2[o][i][kh][kw] W1[i][kh'][kw']
// in fp64, rounded once (s1 = nconv1's weight sums, as the forward's cout = D1 / s1 uses them).
// One 64-lane block per (qh, qw): lane (o, i) forms channel i's term, the 8 terms of an output
// are summed over lanes in a fixed butterfly order; block 81 writes W2 transposed to [i][kh][kw][o].
__global__ __launch_bounds__(64) void head_weights(const float* __restrict__ w1, const float* __restrict__ s1,
                                                   const float* __restrict__ w2, float* __restrict__ out) {
    const int blk = blockIdx.x, lane = threadIdx.x;
    if (blk == 81) {
        for (int e = lane; e < 1600; e += 64) {  // W2t[ci][kh][kw][o] = W2[o][ci][kh][kw]
            const int o = e & 7, kk = (e >> 3) % 25, ci = e / 200;
            out[kW21 + e] = w2[(o * 8 + ci) * 25 + kk];
        }
        return;
    }
    const int qh = blk / 9, qw = blk % 9, o = lane >> 3, i = lane & 7;
    double si = 0.0;
    for (int kh = 0; kh < 5; ++kh) {
        const int kh1 = qh - kh;
        if (kh1 < 0 || kh1 > 4) continue;
        for (int kw = 0; kw < 5; ++kw) {
            const int kw1 = qw - kw;
            if (kw1 < 0 || kw1 > 4) continue;
            si += (double)w2[((o * 8 + i) * 5 + kh) * 5 + kw] * (double)w1[(i * 5 + kh1) * 5 + kw1];
        }
    }
    si /= (double)s1[i];
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) si += __shfl_xor(si, m);
    if (i == 0) out[(qh * 8 + o) * 9 + qw] = (float)si;
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

int launch_head_weights(const float* w1, const float* s1, const float* w2, float* out, hipStream_t st,
                        const char** why) {
    hipLaunchKernelGGL(head_weights, dim3(82), dim3(64), 0, st, w1, s1, w2, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
