// nconv_fwd_tail.hip — exact-fp32 fused tail (nconv6 + nconv7 + crop, models/step1.py:88-94) with
// nconv6's skip-half confidence mass composed back to nconv1's thresholded input and evaluated on
// the bf16 matrix cores (nconv_tail.h), the exact head's idea one level further.
//
// Work per output pixel and channel of nconv6 (16 -> 8, 3x3, padding 0, cat(up(x23), x2)):
//  * skip half (nconv2's outputs, 8 channels x 9 taps): only the data sums N on the vector ALU, two
//    pixels per v_pk_fma_f32 ({N(p), N(p+1)} += w * {xc(c + kw), xc(c + 1 + kw)}: one FMA per tap
//    instead of the {N, D} pair's two); the confidence mass D6s = W621 (x) c0 (11 x 11, nconv_tail.h)
//    on the matrix cores -- 64 v_mfma_f32_16x16x32_bf16 per wave instead of 576 packed FMAs per
//    thread. Only where nconv2's zero padding truncates the window the composition is not a plain
//    convolution: tiles within 5 px of the image edge sum D6s = W6 (x) c2 on the vector ALU in a
//    second pass over nconv2's confidence planes (as the head's edge tiles do);
//  * upsampled half (nconv5's outputs at half resolution): the phase form of nconv_fwd_phase.hip (4
//    instead of 9 taps per pixel) with N and D as pixel pairs, {w(beta0), w(beta1)} * {v(p), v(p+1)};
//  * nconv7 (1x1) in the epilogue, the cropped output written directly.
// With the head's product planes (a_product: nconv_fwd_head_xc wrote nconv2's y * cout where y was,
// the exact product the staging used to form) an interior tile reads one plane per skip channel
// instead of two. Every fp32 product is an fp32 product; D6s differs from summing W6 * c2 only by the
// rounding of the composed weights and of the sum order.
#include "nconv_tail.h"

namespace nconv {

namespace {

constexpr int kT = 256, kTH = 16, kTW = 32;
constexpr int kWH = kTH + 10, kWW = kTW + 10;  // c0 window of a tile: 26 x 42 (origin: tile - 4)
constexpr int kTP = 42;                        // octet table pitch (bytes), = the window width
// composition-phase LDS (bytes): the 256-entry LUT of bf16 {0,1} octets, the row / column / corner
// octet tables, then per wave a D6s transposition region (4 channels x 128 pixels, channel pitch 144)
constexpr int kLut = 0, kW8R = 4096, kW8C = kW8R + kWH * kTP, kW8K = kW8C + kTH * kTP;
constexpr int kTabEnd = kW8K + kTH * kTP;
constexpr int kDP = 144, kDWave = 4 * kDP;           // floats
constexpr int kDOff = (kTabEnd + 15) & ~15;          // bytes
constexpr int kCompBytes = kDOff + 4 * kDWave * 4;
// plane-phase LDS: native float planes (18 x 34 used, pitch 36) x 2 buffers, then low pair planes
// (10 rows x 17 used pair slots {v[c], v[c+1]}, pitch 18) for x*c and c x 2 buffers
constexpr int kNH = kTH + 2, kNW = kTW + 2, kNP = 36;
constexpr int kNPlane = kNH * kNP, kNStride = kNPlane + 4;  // floats (+ a dump slot, 16-B aligned)
constexpr int kLH = kTH / 2 + 2, kLW = kTW / 2 + 2, kLP = 18;
constexpr int kLPlane = kLH * kLP, kLStride = kLPlane + 2;  // f2 slots (+ dump)
constexpr int kLOff = 2 * kNStride * 4;                      // bytes
constexpr int kPlaneBytes = kLOff + 4 * kLStride * 8;
constexpr int kLdsBytes = kCompBytes > kPlaneBytes ? kCompBytes : kPlaneBytes;
constexpr int kNE = (kNH * kNW + kT - 1) / kT;  // native elements per thread (3)
constexpr int kSE = (kWH * kWW + kT - 1) / kT;  // c0 window elements per thread (5)
static_assert(kLH * kLW <= kT, "one low element per thread");

typedef const float __attribute__((address_space(4))) cfloat;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// PAR: (output-grid origin offset - padding) & 1 (fwd_phase's). PROD: source a holds nconv2's y *
// cout (the head's product planes) instead of y.
template <int PAR, bool PROD>
__global__ __launch_bounds__(kT) void fwd_tail_comp(LayerDev d, float* __restrict__ out, TailArgs t,
                                                    const float* __restrict__ s_in, float thresh,
                                                    const float* __restrict__ frag) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kLdsBytes];
    __shared__ unsigned long long c0row[kWH];  // c0 per window row (bits = columns)
    __shared__ unsigned c0col[kWW];            // c0 per window column (bits = rows)
    const nconv_layer& L = d.L;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const TileCoord tc = xcd_tile((t.out_w + kTW - 1) / kTW, (t.out_h + kTH - 1) / kTH, L.B);
    const int b = tc.b;
    const int R0 = tc.ty * kTH, C0 = tc.tx * kTW;
    const int oh0 = R0 + t.off, ow0 = C0 + t.off;  // tile origin in nconv6's grid (= nconv2's rows)
    // wave w: rows rb + 2 g (g = lane >> 4) of one parity, columns 2 jx, 2 jx + 1
    const int g = lane >> 4, jx = lane & 15;
    const int rb = (w >> 1) * 8 + (w & 1);
    const int ty = rb + 2 * g, tx = 2 * jx;
    const int alpha = __builtin_amdgcn_readfirstlane((PAR + (w & 1)) & 1);  // row phase of this wave
    // the composition holds for every nconv6 pixel of the tile (nconv2's windows untruncated)
    const bool comp = oh0 >= 2 && oh0 + kTH - 1 <= L.H - 5 && ow0 >= 2 && ow0 + kTW - 1 <= L.W - 5;
    float* const fl = reinterpret_cast<float*>(lds);

    f2 accN[8], accD[8];  // {N, D} of pixels (ty, tx) and (ty, tx + 1)
#pragma unroll
    for (int o = 0; o < 8; ++o) accN[o] = accD[o] = (f2){0.f, 0.f};

    // ---- native (skip) staging: 18 x 34 elements of the a planes, pitch kNP, 3 per thread ----
    unsigned ga[kNE];
    int lofs[kNE];
#pragma unroll
    for (int k = 0; k < kNE; ++k) {
        const int e = tid + kT * k, r = e / kNW, c = e - (e / kNW) * kNW;
        const int ih = oh0 + r, iw = ow0 + c;
        const bool in = e < kNH * kNW && (unsigned)ih < (unsigned)L.H && (unsigned)iw < (unsigned)L.W;
        ga[k] = in ? (unsigned)(ih * L.a.W + iw) * 4u : 0x80000000u;
        lofs[k] = e < kNH * kNW ? r * kNP + c : kNPlane;
    }
    const int pbytes_a = L.a.H * L.a.W * 4;
    const float* const xa = L.a.x + (size_t)b * L.a.C * L.a.H * L.a.W;
    const float* const ca = L.a.c + (size_t)b * L.a.C * L.a.H * L.a.W;
    // one skip channel's staged value: x*c (PROD: as stored; else formed here) or c
    auto nload = [&](int ci, bool cpass, float (&v)[kNE], float (&u)[kNE]) __attribute__((always_inline)) {
        const size_t po = (size_t)ci * L.a.H * L.a.W;
        const __amdgpu_buffer_rsrc_t rx = plane_rsrc((cpass ? ca : xa) + po, pbytes_a);
        const __amdgpu_buffer_rsrc_t rc = plane_rsrc(ca + po, pbytes_a);
#pragma unroll
        for (int k = 0; k < kNE; ++k) {
            v[k] = ld_f32(rx, ga[k]);
            if (!PROD && !cpass) u[k] = ld_f32(rc, ga[k]);
        }
    };
    auto nstore = [&](float* pl, bool cpass, const float (&v)[kNE], const float (&u)[kNE]) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < kNE; ++k) pl[lofs[k]] = (PROD || cpass) ? v[k] : v[k] * u[k];
    };
    // the first two skip planes fly during the composition phase
    float va[kNE], ua[kNE], vb[kNE], ub[kNE];
    nload(0, false, va, ua);
    nload(1, false, vb, ub);

    // ---- D6s on the matrix cores (interior tiles) ----
    if (comp) {
        if (tid < kWH) c0row[tid] = 0ull;
        if (tid < kWW) c0col[tid] = 0u;
        float sv[kSE];
        const __amdgpu_buffer_rsrc_t rs = plane_rsrc(s_in + (size_t)b * L.H * L.W, L.H * L.W * 4);
#pragma unroll
        for (int k = 0; k < kSE; ++k) {  // (outside the image S reads 0: nconv1's zero padding, c0 = 0)
            const int e = tid + kT * k, r = e / kWW, c = e - (e / kWW) * kWW;
            const int gr = oh0 - 4 + r, gc = ow0 - 4 + c;
            const bool in = e < kWH * kWW && (unsigned)gr < (unsigned)L.H && (unsigned)gc < (unsigned)L.W;
            sv[k] = ld_f32(rs, in ? (unsigned)(gr * L.W + gc) * 4u : 0x80000000u);
        }
        __syncthreads();  // masks zeroed
#pragma unroll
        for (int k = 0; k < kSE; ++k) {
            const int e = tid + kT * k, r = e / kWW, c = e - (e / kWW) * kWW;
            if (e < kWH * kWW && sv[k] > thresh) {  // c0 = (S > thresh), step1.py:53 (NaN: 0)
                atomicOr(&c0row[r], 1ull << c);
                atomicOr(&c0col[c], 1u << r);
            }
        }
        __syncthreads();
        {   // tables: LUT entry tid = bf16 1.0 where bit j of tid is set; the octets of each window row
            // (columns c..c+7), column (rows r..r+7) and 3 x 3 corner (rows r+8..r+10, columns c+8..c+10)
            unsigned dq[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                dq[i] = ((tid >> (2 * i)) & 1u) * 0x3F80u + ((tid >> (2 * i + 1)) & 1u) * 0x3F800000u;
            reinterpret_cast<uint4*>(lds + kLut)[tid] = make_uint4(dq[0], dq[1], dq[2], dq[3]);
            for (int e = tid; e < kWH * kTP; e += kT) {
                const int r = e / kTP, c = e - r * kTP;
                lds[kW8R + e] = (unsigned char)(c0row[r] >> c);
                if (r < kTH) {
                    lds[kW8C + e] = (unsigned char)(c0col[c] >> r);
                    const int c8 = c + 8 < kWW ? c + 8 : kWW - 1;
                    lds[kW8K + e] = (unsigned char)(((c0row[r + 8] >> c8) & 7ull) | (((c0row[r + 9] >> c8) & 7ull) << 3) |
                                                    (((c0row[r + 10] >> c8) & 3ull) << 6));
                }
            }
        }
        __syncthreads();
        // GEMM blocks nb = 0..7 of wave w: its own pixels, row rb + 2 (nb >> 1), columns 16 (nb & 1) + n
        const int n = lane & 15;
        const uint4* fr = reinterpret_cast<const uint4*>(frag) + lane;
        // byte offset of this lane's chunk octet per K step (chunk q = 4 ks + g), pixel (rb, n)
        const int pb = rb * kTP + n;
        const int o0 = kW8R + g * kTP + pb, o1 = kW8R + (4 + g) * kTP + pb;
        const int o2 = (g < 3 ? kW8R + (8 + g) * kTP : kW8C + 8) + pb;
        const int o3 = (g < 2 ? kW8C + 9 + g : (g == 2 ? kW8K : kW8R + 10 * kTP + 10)) + pb;
        const uint4* lut = reinterpret_cast<const uint4*>(lds + kLut);
        float* const dt = fl + kDOff / 4 + w * kDWave;
        // one channel half (bb) at a time: its A fragments and results only (the B fragments are
        // re-read from LDS for the second half rather than kept: fewer live registers)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            bf16x8 A[4];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) A[ks] = __builtin_bit_cast(bf16x8, fr[(bb * 4 + ks) * 64]);
#pragma unroll
            for (int nb = 0; nb < 8; ++nb) {
                const int po = 2 * (nb >> 1) * kTP + 16 * (nb & 1);
                f4 acc = (f4){0.f, 0.f, 0.f, 0.f};
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], __builtin_bit_cast(bf16x8, lut[lds[o0 + po]]), acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], __builtin_bit_cast(bf16x8, lut[lds[o1 + po]]), acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], __builtin_bit_cast(bf16x8, lut[lds[o2 + po]]), acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[3], __builtin_bit_cast(bf16x8, lut[lds[o3 + po]]), acc, 0, 0, 0);
                // GEMM layout (lane (g, n): channel 4 bb + g of block nb's pixel n) -> the wave's own
                // LDS region; the wave's pixels are its threads' pixels, so no workgroup barrier
                dt[g * kDP + (nb >> 1) * 32 + 16 * (nb & 1) + n] = (acc.x + acc.y) + acc.z;  // hi + mid, + lo
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int c = 0; c < 4; ++c) accD[4 * bb + c] = *reinterpret_cast<const f2*>(dt + c * kDP + g * 32 + tx);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();  // the composition region is free: the planes take it

    // ---- skip half: packed pixel pairs over the staged planes ----
    const cfloat* wgt = (const cfloat*)L.weight;  // (constant address space: scalar loads)
    auto fma_native = [&](f2 (&acc)[8], int ci, const float* pl) __attribute__((always_inline)) {
        const float* row = pl + ty * kNP + tx;
        const cfloat* wr = wgt + (size_t)(8 + ci) * 9;  // cat(up(low), skip): skip channels 8..15
#pragma unroll 1
        for (int kh = 0; kh < 3; ++kh, row += kNP, wr += 3) {
            const f2 v01 = *reinterpret_cast<const f2*>(row);
            const f2 v23 = *reinterpret_cast<const f2*>(row + 2);
            const f2 v[3] = {v01, (f2){v01.y, v23.x}, v23};
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                for (int o = 0; o < 8; ++o) {
                    const float wv = wr[o * 144 + kw];
                    acc[o] = __builtin_elementwise_fma((f2){wv, wv}, v[kw], acc[o]);
                }
        }
    };
    float* const pn0 = fl;
    float* const pn1 = fl + kNStride;
    auto native_pass = [&](f2 (&acc)[8], bool cpass) __attribute__((always_inline)) {
        // two plane buffers, one barrier per channel, loads two planes ahead (as fwd_phase); the
        // prefetches past the last channel re-read it (L2-resident), no branch around them
#pragma unroll 1
        for (int ci = 0; ci < 8; ci += 2) {
            nstore(pn0, cpass, va, ua);
            __syncthreads();
            nload(ci + 2 < 8 ? ci + 2 : 7, cpass, va, ua);
            fma_native(acc, ci, pn0);
            nstore(pn1, cpass, vb, ub);
            __syncthreads();
            nload(ci + 3 < 8 ? ci + 3 : 7, cpass, vb, ub);
            fma_native(acc, ci + 1, pn1);
        }
    };
    native_pass(accN, false);
    if (!comp) {  // edge tile: D6s = W6 * c2 from nconv2's confidence planes
        nload(0, true, va, ua);
        nload(1, true, vb, ub);
        native_pass(accD, true);
    }

    // ---- upsampled half: phase taps over the low-resolution planes, N and D as pixel pairs ----
    // low element (lr, lc) of the tile (origin ((oh0 - PH) >> 1, (ow0 - PW) >> 1) in nconv5's grid)
    const int lr = tid / kLW, lcc = tid - (tid / kLW) * kLW;
    unsigned lofs_low;
    {
        const int gr = ((oh0 - L.PH) >> 1) + lr, gc = ((ow0 - L.PW) >> 1) + lcc;
        const bool in = tid < kLH * kLW && (unsigned)gr < (unsigned)L.b.H && (unsigned)gc < (unsigned)L.b.W;
        lofs_low = in ? (unsigned)(gr * L.b.W + gc) * 4u : 0x80000000u;
    }
    const int pbytes_b = L.b.H * L.b.W * 4;
    auto lload = [&](int cb, float& x, float& c) __attribute__((always_inline)) {
        const size_t base = ((size_t)b * L.b.C + cb) * (size_t)L.b.H * L.b.W;
        x = ld_f32(plane_rsrc(L.b.x + base, pbytes_b), lofs_low);
        c = ld_f32(plane_rsrc(L.b.c + base, pbytes_b), lofs_low);
    };
    float* const lowf = fl + kLOff / 4;  // 4 pair planes: (x*c, c) x 2 buffers
    // element (lr, lc) is the .x of pair slot lc and the .y of slot lc - 1 (threads past the tile and
    // slot -1 write the plane's dump slot)
    const int sx = tid < kLH * kLW ? 2 * (lr * kLP + lcc) : 2 * kLPlane;
    const int sy = (tid < kLH * kLW && lcc > 0) ? 2 * (lr * kLP + lcc - 1) + 1 : 2 * kLPlane + 1;
    auto lstore = [&](int bufi, float x, float c) __attribute__((always_inline)) {
        float* px = lowf + bufi * 2 * kLStride * 2;
        float* pc = px + kLStride * 2;
        const float xc = x * c;
        px[sx] = xc;
        px[sy] = xc;
        pc[sx] = c;
        pc[sy] = c;
    };
    // nconv6's phase weights re-laid [i][alpha][dh][o][dw][beta] (nconv_tail.h, after the fragments):
    // a pixel pair's two weights {w(beta = PAR), w(beta = 1 - PAR)} are one SGPR pair
    const cfloat* wph = (const cfloat*)frag + kTailFrag;
    auto fma_up = [&](int cb, int bufi) __attribute__((always_inline)) {
        const f2* rx = reinterpret_cast<const f2*>(lowf + bufi * 2 * kLStride * 2) + ((ty + PAR) >> 1) * kLP + jx;
        const f2* rc = rx + kLStride;
        const cfloat* wr = wph + ((size_t)cb * 2 + alpha) * 2 * 32;
#pragma unroll 1
        for (int dh = 0; dh < 2; ++dh, rx += kLP, rc += kLP, wr += 32) {
            const f2 x0 = rx[0], x1 = rx[1], c0 = rc[0], c1 = rc[1];
#pragma unroll
            for (int o = 0; o < 8; ++o)
#pragma unroll
                for (int dw = 0; dw < 2; ++dw) {
                    // pixel 0 (column phase PAR) reads low column jx + dw, pixel 1 (phase 1 - PAR)
                    // jx + PAR + dw: the pair slot jx + dw (PAR = 1) or its first value twice
                    const float w0 = wr[o * 4 + dw * 2 + PAR], w1 = wr[o * 4 + dw * 2 + 1 - PAR];
                    const f2 xs = dw ? x1 : x0, cs = dw ? c1 : c0;
                    const f2 vx = PAR ? xs : (f2){xs.x, xs.x}, vc = PAR ? cs : (f2){cs.x, cs.x};
                    accN[o] = __builtin_elementwise_fma((f2){w0, w1}, vx, accN[o]);
                    accD[o] = __builtin_elementwise_fma((f2){w0, w1}, vc, accD[o]);
                }
        }
    };
    {
        float lx0, lc0, lx1, lc1;
        lload(0, lx0, lc0);
        lload(1, lx1, lc1);
#pragma unroll 1
        for (int cb = 0; cb < 8; cb += 2) {
            lstore(0, lx0, lc0);
            __syncthreads();
            lload(cb + 2 < 8 ? cb + 2 : 7, lx0, lc0);
            fma_up(cb, 0);
            lstore(1, lx1, lc1);
            __syncthreads();
            lload(cb + 3 < 8 ? cb + 3 : 7, lx1, lc1);
            fma_up(cb + 1, 1);
        }
    }

    // ---- epilogue: nconv6's outputs -> nconv7 (1x1, 8 -> 1) -> the cropped output (fwd_phase's) ----
    const int oh = oh0 + ty;
    const int r = R0 + ty;
    if (r >= t.out_h) return;
    const float b7 = t.b7[0], s7 = t.s7[0];
    constexpr unsigned OOB = 0x80000000u;
    const int owb = ow0 + tx;
    bool inj[2];
    unsigned so[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        inj[j] = (unsigned)oh < (unsigned)L.Ho && (unsigned)(owb + j) < (unsigned)L.Wo;
        so[j] = inj[j] ? (unsigned)(oh * L.Wo + owb + j) * 4u : OOB;
    }
    const bool vec = (L.Wo % 2) == 0 && inj[0] && inj[1];
    const int pbytes6 = L.Ho * L.Wo * 4;
    float N7[2] = {0.f, 0.f}, D7[2] = {0.f, 0.f};
#pragma unroll
    for (int o = 0; o < 8; ++o) {
        float y6[2], c6[2];
        nconv_epilogue(accN[o].x, accD[o].x, L.eps, L.bias[o], L.wsum[o], y6[0], c6[0]);
        nconv_epilogue(accN[o].y, accD[o].y, L.eps, L.bias[o], L.wsum[o], y6[1], c6[1]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (inj[j]) {
                N7[j] = fmaf(t.w7[o], y6[j] * c6[j], N7[j]);
                D7[j] = fmaf(t.w7[o], c6[j], D7[j]);
            }
        if (t.y6) {  // training: each pixel of nconv6 lies in exactly one tile
            const size_t ofs = ((size_t)b * 8 + o) * L.Ho * L.Wo;
            const __amdgpu_buffer_rsrc_t ry = plane_rsrc(t.y6 + ofs, pbytes6), rc = plane_rsrc(t.c6 + ofs, pbytes6);
            if (vec) {
                st_f2(ry, so[0], (f2){y6[0], y6[1]});
                st_f2(rc, so[0], (f2){c6[0], c6[1]});
            } else {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    st_f32(ry, so[j], y6[j]);
                    st_f32(rc, so[j], c6[j]);
                }
            }
        }
    }
    float ov[2], oc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) nconv_epilogue(N7[j], D7[j], t.eps7, b7, s7, ov[j], oc[j]);
    const size_t base = ((size_t)b * t.out_h + r) * t.out_w + C0 + tx;
#pragma unroll
    for (int j = 0; j < 2; ++j)
        if (C0 + tx + j < t.out_w) {
            out[base + j] = ov[j];
            if (t.out_c) t.out_c[base + j] = oc[j];
        }
}

// nconv_tail_weights as its own launch: four units per 256-thread block (nconv_tail.h), the
// normalisers read from the layers' wsum (what the forward divides by)
__global__ __launch_bounds__(kPrepThreads) void tail_weights(const float* __restrict__ w1, const float* __restrict__ s1,
                                                             const float* __restrict__ w2, const float* __restrict__ s2,
                                                             const float* __restrict__ w6, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, unit = 4 * blockIdx.x + (threadIdx.x >> 6);
    if (unit >= kTailUnits) return;
    tail_weights_unit(w1, w2, w6, s1[lane & 7], s2[lane >> 3], out, unit, lane);
}

}  // namespace

// The geometry the composed tail serves: nconv6 of DNET (16 -> 8 = 8 upsampled + 8 skip channels,
// upsampled first, 3x3, padding 0, stride 1, exactly-2x upsampling, exact fp32, phase weights given).
bool fwd_tail_comp_supported(const nconv_layer& L) {
    return L.load_mode == NCONV_LOAD_UPCAT_UP_FIRST && L.waux && L.math == NCONV_MATH_FP32 && L.Cin == 16 &&
           L.Cout == 8 && L.a.C == 8 && L.b.C == 8 && L.KH == 3 && L.KW == 3 && L.SH == 1 && L.SW == 1 &&
           L.DH == 1 && L.DW == 1 && L.groups == 1 && L.PH == 0 && L.PW == 0 && L.H == 2 * L.b.H &&
           L.W == 2 * L.b.W && L.a.H == L.H && L.a.W == L.W;
}

int launch_fwd_tail_comp(const LayerDev& d, const TailArgs& t, float* out, const float* s_in, float thresh,
                         const float* frag, bool a_product, hipStream_t st, const char** why) {
    const nconv_layer& L = d.L;
    const dim3 grid(((t.out_w + kTW - 1) / kTW) * ((t.out_h + kTH - 1) / kTH) * L.B);  // see xcd_tile
    const int par = (t.off - L.PH) & 1;
#define NCONV_GO(P, PR) hipLaunchKernelGGL((fwd_tail_comp<P, PR>), grid, dim3(kT), 0, st, d, out, t, s_in, thresh, frag)
    if (par) {
        if (a_product) NCONV_GO(1, true);
        else NCONV_GO(1, false);
    } else {
        if (a_product) NCONV_GO(0, true);
        else NCONV_GO(0, false);
    }
#undef NCONV_GO
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

int launch_tail_weights(const float* w1, const float* s1, const float* w2, const float* s2, const float* w6,
                        float* out, hipStream_t st, const char** why) {
    hipLaunchKernelGGL(tail_weights, dim3((kTailUnits + 3) / 4), dim3(kPrepThreads), 0, st, w1, s1, w2, s2, w6, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return -5;
    }
    return 0;
}

}  // namespace nconv
