// nconv_tail.h — the composed confidence weights of the fused tail's skip half, shared by the
// inference weight prologue (nconv_fwd_head.hip) and nconv_tail_weights (nconv_fwd_tail.hip).
//
// nconv6 (models/step1.py:88-90; 16 -> 8, 3x3, padding 0, cat(up(x23), x2)) reads nconv2's outputs
// as its skip half. Its confidence mass over that half is
//     D6s[o](p) = sum_i sum_{a,b} W6[o][8 + i][a][b] * c2[i](p + (a, b)),   c2 = D2 / s2,
// and wherever nconv2's window is not truncated by its zero padding, D2 = W21 (x) c0 (the exact
// head's composition, nconv_fwd_head.hip: c0 = (S > thresh) the thresholded sparse input). So
//     D6s[o](p) = sum_{U,V < 11} W621[o][U][V] * c0(p + (U - 4, V - 4)),
//     W621[o][U][V] = sum_i (1 / s2[i]) sum_{a,b} W6[o][8 + i][a][b] * W21[i][U - a][V - b],
//     W21[i][u][v]  = sum_j (1 / s1[j]) sum_{kh + kh' = u, kw + kw' = v} W2[i][j][kh][kw] W1[j][kh'][kw'],
// an 11 x 11 convolution of the binary mask: the fused tail evaluates it on the bf16 matrix cores
// with exact products (c0 is 0 or 1; each fp32 W621 is the exact sum of three bf16 parts), as the
// head does for D2, instead of 72 fp32 FMAs per pixel and channel on the vector ALU. The composition
// is formed in fp64 and rounded once to fp32; all terms are non-negative (softplus weights), so the
// regrouping keeps D6s inside the fp32 bound of the sum, and D6s is exactly 0 where the reference's
// is (no sample in the window).
//
// Operand layout: v_mfma_f32_16x16x32_bf16's A fragments [bb][ks][lane] x 8 bf16 (bb = output
// channels 4bb .. 4bb + 3, ks = K step of 4 tap chunks): lane l holds row l & 15 = 4 (o & 3) + part
// (part 3 = 0) and chunk q = 4 ks + (l >> 4), 8 taps j of the chunk:
//   q  0..10  taps (U = q, V = j)                (a row octet of the mask)
//   q 11..13  taps (U = j, V = 8 + q - 11)       (a column octet)
//   q 14      taps (8 + j / 3, 8 + j % 3), j < 8 (the 3 x 3 corner without (10, 10))
//   q 15      tap (10, 10) in j = 0              (a row octet whose other taps weigh 0)
#pragma once
#include "nconv_prologue.h"

namespace nconv {

constexpr int kTailFrag = 2 * 4 * 64 * 4;  // dwords of A fragments
constexpr int kTailPhase = 1024;           // then nconv6's phase weights, re-laid (below)
constexpr int kTailFloats = kTailFrag + kTailPhase;  // = NCONV_TAIL_WEIGHTS_FLOATS
constexpr int kTailUnits = 123;  // 121 composed taps, the fragment padding, the phase weights

__device__ __forceinline__ int tail_frag_slot(int o, int part, int q, int j) {  // bf16 index
    return (((o >> 2) * 4 + (q >> 2)) * 64 + (q & 3) * 16 + 4 * (o & 3) + part) * 8 + j;
}

// Whether fragment element (q, j) carries a tap (the others are zero padding)
__device__ __forceinline__ bool tail_slot_used(int q, int j) { return q < 15 || j == 0; }

// One unit of the tail weights per wave: units 0..120 the composed tap (U, V) = (u / 11, u % 11),
// unit 121 the zero padding of the fragment table, unit 122 nconv6's phase weights (phase_block's
// sums in its order, so bitwise nconv_phase_weights' values) re-laid as [i][alpha][dh][o][dw][beta]
// after the fragments: the fused tail's pixel pair (tail columns c, c + 1: opposite column phases)
// then takes its two weights as one SGPR pair. w1 (8, 1, 5, 5), w2 (8, 8, 5, 5), w6 (8, 16, 3,
// 3); s1j = s1[lane & 7] (nconv1's normaliser of channel j), s2i = s2[lane >> 3] (nconv2's of channel
// i), both as the forward uses them. Lane (i, j) = (lane >> 3, lane & 7): first W21[i][.][.] of the
// 3 x 3 taps (U - a, V - b) over nconv1's channel j, summed over j by a fixed xor butterfly; then
// (i, o = j): nconv6's 9 taps of channel 8 + i, summed over i by a second butterfly. fp64 throughout,
// rounded once, split into hi + mid + lo bf16 truncations (each remainder exact in fp32).
__device__ __forceinline__ void tail_weights_unit(const float* __restrict__ w1, const float* __restrict__ w2,
                                                  const float* __restrict__ w6, float s1j, float s2i,
                                                  float* __restrict__ out, int unit, int lane) {
    unsigned short* const fb = reinterpret_cast<unsigned short*>(out);
    if (unit == 122) {
        for (int e = lane; e < kTailPhase; e += 64) {
            const int bt = e & 1, dw = (e >> 1) & 1, rest = e >> 2;  // rest = ((i * 2 + a) * 2 + dh) * 8 + o
            const int o = rest & 7, dh = (rest >> 3) & 1, al = (rest >> 4) & 1, i = rest >> 5;
            const int kh_lo = al == 0 ? (dh == 0 ? 0 : 2) : (dh == 0 ? 0 : 1);
            const int kh_hi = al == 0 ? (dh == 0 ? 1 : 2) : (dh == 0 ? 0 : 2);
            const int kw_lo = bt == 0 ? (dw == 0 ? 0 : 2) : (dw == 0 ? 0 : 1);
            const int kw_hi = bt == 0 ? (dw == 0 ? 1 : 2) : (dw == 0 ? 0 : 2);
            const float* wo = w6 + ((size_t)o * 16 + i) * 9;  // (nconv6's upsampled channels are 0..7)
            float s = 0.f;
            for (int kh = kh_lo; kh <= kh_hi; ++kh)
                for (int kw = kw_lo; kw <= kw_hi; ++kw) s += wo[kh * 3 + kw];
            out[kTailFrag + e] = s;
        }
        return;
    }
    if (unit == 121) {
        for (int e = lane; e < kTailFrag * 2; e += 64) {
            const int j = e & 7, l = (e >> 3) & 63, ks = (e >> 9) & 3;
            const int part = l & 3, q = 4 * ks + (l >> 4);
            if (part == 3 || !tail_slot_used(q, j)) fb[e] = 0;
        }
        return;
    }
    const int U = unit / 11, V = unit % 11, i = lane >> 3, j = lane & 7;
    float a2[25], a1[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) {
        a2[k] = w2[(i * 8 + j) * 25 + k];
        a1[k] = w1[j * 25 + k];
    }
    double t[9];
#pragma unroll
    for (int ab = 0; ab < 9; ++ab) {
        const int u = U - ab / 3, v = V - ab % 3;
        double s = 0.0;
#pragma unroll
        for (int kh = 0; kh < 5; ++kh) {
#pragma unroll
            for (int kw = 0; kw < 5; ++kw) {
                const int kh1 = u - kh, kw1 = v - kw;
                const bool ok = kh1 >= 0 && kh1 <= 4 && kw1 >= 0 && kw1 <= 4;
                const double p = (double)a2[kh * 5 + kw] * (double)a1[ok ? kh1 * 5 + kw1 : 0];
                s = ok ? s + p : s;
            }
        }
        t[ab] = s / (double)s1j;
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1)
#pragma unroll
        for (int ab = 0; ab < 9; ++ab) t[ab] += __shfl_xor(t[ab], m);
    // lane (i, o = j): nconv6's skip channel 8 + i of output o
    const int o = j;
    double s = 0.0;
#pragma unroll
    for (int ab = 0; ab < 9; ++ab) s = __builtin_fma((double)w6[(o * 16 + 8 + i) * 9 + ab], t[ab], s);
    s /= (double)s2i;
#pragma unroll
    for (int m = 8; m < 64; m <<= 1) s += __shfl_xor(s, m);
    if (i == 0) {
        const float w = (float)s;
        const float hi = __uint_as_float(__float_as_uint(w) & 0xFFFF0000u);
        const float r = w - hi;
        const float mid = __uint_as_float(__float_as_uint(r) & 0xFFFF0000u);
        const float lo = r - mid;
        int q, jj;
        if (V <= 7) {
            q = U, jj = V;
        } else if (U <= 7) {
            q = 11 + (V - 8), jj = U;
        } else {
            const int k = (U - 8) * 3 + (V - 8);
            q = k < 8 ? 14 : 15, jj = k < 8 ? k : 0;
        }
        fb[tail_frag_slot(o, 0, q, jj)] = (unsigned short)(__float_as_uint(hi) >> 16);
        fb[tail_frag_slot(o, 1, q, jj)] = (unsigned short)(__float_as_uint(mid) >> 16);
        fb[tail_frag_slot(o, 2, q, jj)] = (unsigned short)(__float_as_uint(lo) >> 16);
    }
}

}  // namespace nconv

static_assert(nconv::kTailFloats == NCONV_TAIL_WEIGHTS_FLOATS, "tail weight buffer size (include/nconv.h)");
