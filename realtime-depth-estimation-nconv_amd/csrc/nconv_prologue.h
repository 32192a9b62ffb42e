// nconv_prologue.h — bodies of the weight-only prologue kernels, shared by their own launches
// (nconv_weight_prep, nconv_phase_weights) and by the one-launch inference prologue
// (nconv_weight_prologue, nconv_fwd_head.hip), so that every output is bitwise the same whichever
// launch computes it.
#pragma once
#include "nconv_internal.h"

namespace nconv {

constexpr int kPrepThreads = 256;  // threads of a prep / phase block

// EnforcePos (softplus, beta=10, threshold=20; step1.py:190-207) in place + s[o] = sum W[o].
struct PrepArgs {
    static constexpr int kMax = 32;
    float* w[kMax];
    float* s[kMax];
    int cout[kMax];
    int fan_in[kMax];
    int softplus[kMax];
};

// The normaliser of one weight row (step1.py:141-144) by one wave: lane-strided partial sums, then
// a fixed-order xor butterfly (every lane ends with the same value).
__device__ __forceinline__ float row_sum_wave(const float* wr, int fan, int lane) {
    float s = 0.f;
    if (fan <= 256) {  // (every DNET layer) the lane's loads issued together, added in the same order
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = wr[lane + 64 * k < fan ? lane + 64 * k : 0];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (lane + 64 * k < fan) s += v[k];
    } else {
        for (int i = lane; i < fan; i += 64) s += wr[i];
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m);
    return s;
}

// EnforcePos's softplus of one weight, shared by every launch that applies it (weight_prep, the
// training prologue's staging); GPU tests hold the two bitwise equal on both sides of the threshold.
__device__ __forceinline__ float enforce_pos(float v) {
    const float bv = v * 10.0f;
    return (bv > 20.0f) ? v : log1pf(expf(bv)) / 10.0f;
}

// One layer per 256-thread block: optional in-place softplus, then one wave per row for s[o]
// (lanes stride the row, coalesced), instead of one thread walking ~200 dependent loads.
__device__ __forceinline__ void prep_block(float* w, float* s, int cout, int fan, int softplus) {
    const int n = cout * fan;
    if (softplus) {
        for (int i = threadIdx.x; i < n; i += kPrepThreads) w[i] = enforce_pos(w[i]);
        __syncthreads();
        __threadfence_block();
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int o = wave; o < cout; o += kPrepThreads / 64) {
        const float v = row_sum_wave(w + (size_t)o * fan, fan, lane);
        if (lane == 0) s[o] = v;
    }
}

// Phase weights of the upsampled channels of n UPCAT layers (nconv_fwd_phase.hip), one block per
// layer: out[((i * 2 + a) * 2 + dh) * 32 + o * 4 + bt * 2 + dw] = sum over kh in S(a, dh), kw in
// S(bt, dw) of W[o][ci][kh][kw] (kh ascending, then kw), ci = the layer's input channel of up
// channel i; S(0,0) = {0,1}, S(0,1) = {2}, S(1,0) = {0}, S(1,1) = {1,2}.
struct PhaseArgs {
    static constexpr int kMax = 8;
    const float* w[kMax];
    float* out[kMax];
    int ci0[kMax];  // input channel of up channel 0
    int cin[kMax];
};

// Box weights of an exactly-2x UPCAT layer's upsampled half for the phase-form input gradient
// (dgrad_phase, nconv_bwd.hip): entry e = [o][i][t][u] (8 x 8 x 4 x 4) = the sum of W[o][first_up +
// i][kh][kw] over kh in S(t), kw in S(u), S(0) = {2}, S(1) = {1, 2}, S(2) = {0, 1}, S(3) = {0}
// (row-major order). Shared by the box_weights launch and the training prologue (bitwise equal).
__device__ __forceinline__ float box_weight(const float* w, int first_up, int e) {
    const int u = e & 3, t = (e >> 2) & 3, i = (e >> 4) & 7, o = e >> 7;
    const float* wk = w + ((size_t)o * 16 + first_up + i) * 9;
    const int h0 = t == 0 ? 2 : (t == 1 ? 1 : 0), nh = (t == 1 || t == 2) ? 2 : 1;
    const int w0 = u == 0 ? 2 : (u == 1 ? 1 : 0), nw = (u == 1 || u == 2) ? 2 : 1;
    float sum = 0.f;
    for (int r = 0; r < nh; ++r)
        for (int c = 0; c < nw; ++c) sum += wk[(h0 + r) * 3 + w0 + c];
    return sum;
}

// Training prologue (nconv_train_prologue): per phase layer (16 -> 8 3x3) its weight (EnforcePos
// applied in place when sp), normalisers, phase weights and optional box weights.
struct TrainPhaseArgs {
    static constexpr int kMax = 8;
    float* w[kMax];
    float* s[kMax];
    float* out[kMax];
    float* box[kMax];
    int sp[kMax];
    int ci0[kMax];
};

__device__ __forceinline__ void phase_block(const float* W, int cin, int ci0, float* out) {
    constexpr int kUp = 8;  // upsampled input channels (and output channels) of the phase form
    for (int e = threadIdx.x; e < kUp * 2 * 2 * 32; e += kPrepThreads) {
        const int i = e >> 7, al = (e >> 6) & 1, dh = (e >> 5) & 1, o = (e >> 2) & 7, bt = (e >> 1) & 1, dw = e & 1;
        const int kh_lo = al == 0 ? (dh == 0 ? 0 : 2) : (dh == 0 ? 0 : 1);
        const int kh_hi = al == 0 ? (dh == 0 ? 1 : 2) : (dh == 0 ? 0 : 2);
        const int kw_lo = bt == 0 ? (dw == 0 ? 0 : 2) : (dw == 0 ? 0 : 1);
        const int kw_hi = bt == 0 ? (dw == 0 ? 1 : 2) : (dw == 0 ? 0 : 2);
        const float* wo = W + ((size_t)o * cin + ci0 + i) * 9;
        float s = 0.f;
        for (int kh = kh_lo; kh <= kh_hi; ++kh)
            for (int kw = kw_lo; kw <= kw_hi; ++kw) s += wo[kh * 3 + kw];
        out[e] = s;
    }
}

}  // namespace nconv
