// nconv_common.h — device-side helpers shared by the forward and backward NConv kernels (gfx950).
//
// Reference semantics restated here (all in models/step1.py of the reference):
//   * threshold confidence c0 = float(S > 0.01)                       step1.py:53
//   * independent 2x2/s2 max-pooling of data and confidence            step1.py:62-75
//     (torch max_pool2d: a later element wins iff it is > the running max or is NaN,
//      so ties keep the FIRST maximum in row-major window order)
//   * nearest upsampling to a given size (torch: src = dst>>1 when out == 2*in,
//     else min(floor(dst * (float)in/out), in-1))                       step1.py:78-89
//   * channel concat, skip first (nconv4/5) or upsampled first (nconv6) step1.py:80,85,90
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "../../include/nconv.h"

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// Layer descriptor as the kernels see it: the C-ABI struct plus host-derived constants.
struct LayerDev {
    nconv_layer L;
    float up_scale_h;  // (float)b.H / H   (UPCAT modes)
    float up_scale_w;  // (float)b.W / W
};

__device__ __forceinline__ int nearest_src(int dst, int in, int out, float scale) {
    if (out == in) return dst;
    if (out == 2 * in) return dst >> 1;
    int s = (int)floorf((float)dst * scale);
    return s < in - 1 ? s : in - 1;
}

// torch max_pool2d window scan: (v > m) || isnan(v) replaces; returns the window slot 0..3.
__device__ __forceinline__ float pool4(float v0, float v1, float v2, float v3, int& arg) {
    float m = v0;
    arg = 0;
    if (v1 > m || v1 != v1) { m = v1; arg = 1; }
    if (v2 > m || v2 != v2) { m = v2; arg = 2; }
    if (v3 > m || v3 != v3) { m = v3; arg = 3; }
    return m;
}

// The pooled value alone (no argmax): the window's maximum, NaN if any element is NaN -- the value
// max_pool2d returns, as two v_maximum3_f32 (IEEE 754-2019 maximum, NaN-propagating; gfx950)
// instead of pool4's compare / select chain. Ties need no order for the value; the one difference
// is the sign of a zero maximum (+0 where a window holds both -0 and +0 in that order), which no
// consumer distinguishes (w * (+-0) terms leave a sum unchanged).
__device__ __forceinline__ float pool4v(float v0, float v1, float v2, float v3) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(v0, v1),
                                         __builtin_elementwise_maximum(v2, v3));
}

// Cross-lane reads without the LDS crossbar (ds_bpermute): xor 1 by a DPP quad permutation,
// xor 16 by v_permlane16_swap (gfx950; swapping a copy of v with itself gives rows {1,0,3,2} in
// one of the two results depending on the row's parity), xor 17 as both.
__device__ __forceinline__ float shfl_xor1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float shfl_xor16(float v) {
    const int iv = __builtin_bit_cast(int, v);
    const auto r = __builtin_amdgcn_permlane16_swap(iv, iv, false, false);
    return __builtin_bit_cast(float, ((threadIdx.x >> 4) & 1) ? r[0] : r[1]);
}
__device__ __forceinline__ float shfl_xor17(float v) { return shfl_xor1(shfl_xor16(v)); }

// Vertical 2x2-pool pairs of two values at once: v_permlane16_swap(a, b) swaps a's odd 16-lane rows
// with b's even rows, leaving {a0, b0, a2, b2} and {a1, b1, a3, b3}; their maximum is a's row-pair
// maximum in the even rows and b's in the odd rows (IEEE maximum: NaN wins, order-free). The
// results are copied out of the builtin's vector before the bit casts: hipcc (ROCm 7.2) lowers
// __builtin_bit_cast of an element of that vector to element 0 whatever the index.
__device__ __forceinline__ float pair_rows_max(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, a), __builtin_bit_cast(int, b), false, false);
    const int r0 = r[0], r1 = r[1];
    return __builtin_elementwise_maximum(__builtin_bit_cast(float, r0), __builtin_bit_cast(float, r1));
}

__device__ __forceinline__ size_t plane_idx(int b, int c, int C, int H, int W, int h, int w) {
    return (((size_t)b * C + c) * H + h) * (size_t)W + w;
}

// Layer input (x, c) at logical position (b, ci, ih, iw), which must be in range. The glue op of
// the layer's load mode is evaluated here, so no glued intermediate tensor ever exists in HBM.
template <int MODE>
__device__ __forceinline__ void load_xc(const LayerDev& d, int b, int ci, int ih, int iw, float& x,
                                        float& c) {
    const nconv_layer& L = d.L;
    if constexpr (MODE == NCONV_LOAD_PLAIN) {
        size_t i = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, ih, iw);
        x = L.a.x[i];
        c = L.a.c[i];
    } else if constexpr (MODE == NCONV_LOAD_THRESH) {
        x = L.a.x[plane_idx(b, ci, L.a.C, L.a.H, L.a.W, ih, iw)];
        c = (x > L.thresh) ? 1.0f : 0.0f;
    } else if constexpr (MODE == NCONV_LOAD_POOL2) {
        size_t i = plane_idx(b, ci, L.a.C, L.a.H, L.a.W, 2 * ih, 2 * iw);
        size_t W2 = (size_t)L.a.W;
        if ((L.a.W & 1) == 0) {  // 8-byte aligned window rows: one dwordx2 per row
            f2 x0 = *(const f2*)(L.a.x + i), x1 = *(const f2*)(L.a.x + i + W2);
            f2 c0 = *(const f2*)(L.a.c + i), c1 = *(const f2*)(L.a.c + i + W2);
            x = pool4v(x0.x, x0.y, x1.x, x1.y);
            c = pool4v(c0.x, c0.y, c1.x, c1.y);
        } else {
            x = pool4v(L.a.x[i], L.a.x[i + 1], L.a.x[i + W2], L.a.x[i + W2 + 1]);
            c = pool4v(L.a.c[i], L.a.c[i + 1], L.a.c[i + W2], L.a.c[i + W2 + 1]);
        }
    } else {
        const bool skip_first = (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST);
        const int first_c = skip_first ? L.a.C : L.b.C;
        const bool from_a = skip_first ? (ci < first_c) : (ci >= first_c);
        if (from_a) {
            int ca = skip_first ? ci : ci - first_c;
            size_t i = plane_idx(b, ca, L.a.C, L.a.H, L.a.W, ih, iw);
            x = L.a.x[i];
            c = L.a.c[i];
        } else {
            int cb = skip_first ? ci - first_c : ci;
            int sh = nearest_src(ih, L.b.H, L.H, d.up_scale_h);
            int sw = nearest_src(iw, L.b.W, L.W, d.up_scale_w);
            size_t i = plane_idx(b, cb, L.b.C, L.b.H, L.b.W, sh, sw);
            x = L.b.x[i];
            c = L.b.c[i];
        }
    }
}

// XCD-aware tile order (MI355X: 8 XCDs, each with its own L2; workgroups are dealt round-robin,
// so blocks b and b+8 share an XCD). Launch a 1-D grid of ntx*nty*nb blocks; this bijection gives
// each XCD group a contiguous run of row-major tiles, so the halo rows and columns neighbouring
// tiles share are fetched into one L2 instead of two or three (speed only, never correctness).
struct TileCoord {
    int tx, ty, b;
};
__device__ __forceinline__ TileCoord xcd_tile(int ntx, int nty, int nb, int bid) {
    const int total = ntx * nty * nb;
    const int q = total / 8, r = total % 8, xcd = bid % 8, loc = bid / 8;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    TileCoord c;
    c.tx = t % ntx;
    c.ty = (t / ntx) % nty;
    c.b = t / (ntx * nty);
    return c;
}
__device__ __forceinline__ TileCoord xcd_tile(int ntx, int nty, int nb) { return xcd_tile(ntx, nty, nb, blockIdx.x); }
// Persistent grids: a workgroup walks the virtual ids blockIdx.x + i * gridDim.x; with gridDim.x a
// multiple of 8 these stay on the workgroup's own XCD, so xcd_tile's mapping still holds.

// Epilogue of NConv2d.forward (step1.py:123-147):  y = N / (D + eps) + b,   cout = D / s.
// The quotients use v_rcp_f32 (1 ulp) and a multiply instead of the ~10-instruction IEEE division
// sequence: the results differ from IEEE division by at most 2 ulp, far inside the 1e-4 relative
// tolerance (the fp32 sums N and D already differ from the reference's summation order by more).
// -DNCONV_IEEE_DIV restores correctly rounded division.
__device__ __forceinline__ void nconv_epilogue(float N, float D, float eps, float bias, float s,
                                               float& y, float& co) {
#ifdef NCONV_IEEE_DIV
    y = N / (D + eps) + bias;
    co = D / s;
#else
    y = N * __builtin_amdgcn_rcpf(D + eps) + bias;
    co = D * __builtin_amdgcn_rcpf(s);
#endif
}

// Closed-form gradient of the epilogue w.r.t. N and D, from the saved outputs.
// Reciprocal-based like nconv_epilogue (<= 2 ulp from IEEE division; -DNCONV_IEEE_DIV restores it).
__device__ __forceinline__ void nconv_grad_nd(float gy, float gco, float y, float co, float eps,
                                              float bias, float s, float& gN, float& gD) {
    const float D = co * s;
    const float den = D + eps;
    const float r = y - bias;  // = N / (D + eps)
#ifdef NCONV_IEEE_DIV
    gN = gy / den;
    gD = -(gy * r) / den + gco / s;
#else
    const float rd = __builtin_amdgcn_rcpf(den);
    gN = gy * rd;
    gD = fmaf(-(gy * r), rd, gco * __builtin_amdgcn_rcpf(s));
#endif
}

// ------------------------------------------------------------------------------------------------
// Tile staging. A layer-input channel's source is resolved once per (image, channel) — a
// wave-uniform decision — so the per-element work is one bounds test, 32-bit plane offsets,
// the glue's loads and one ds_write_b64.
// ------------------------------------------------------------------------------------------------
enum ChanKind { kDirect = 0, kThresh = 1, kPool = 2, kUp = 3 };

struct ChanSrc {
    const float* x;
    const float* c;
    int W;      // row pitch of the source plane
    int kind;   // ChanKind
    int bytes;  // size of the source plane in bytes
};

template <int MODE>
__device__ __forceinline__ ChanSrc chan_src(const LayerDev& d, int b, int ci) {
    const nconv_layer& L = d.L;
    ChanSrc s;
    if constexpr (MODE == NCONV_LOAD_PLAIN || MODE == NCONV_LOAD_THRESH || MODE == NCONV_LOAD_POOL2) {
        const size_t off = ((size_t)b * L.a.C + ci) * (size_t)L.a.H * L.a.W;
        s.x = L.a.x + off;
        s.c = (MODE == NCONV_LOAD_THRESH) ? nullptr : L.a.c + off;
        s.W = L.a.W;
        s.kind = (MODE == NCONV_LOAD_PLAIN) ? kDirect : (MODE == NCONV_LOAD_THRESH) ? kThresh : kPool;
        s.bytes = L.a.H * L.a.W * 4;
    } else {
        const bool skip_first = (MODE == NCONV_LOAD_UPCAT_SKIP_FIRST);
        const int first_c = skip_first ? L.a.C : L.b.C;
        const bool from_a = skip_first ? (ci < first_c) : (ci >= first_c);
        if (from_a) {
            const int ca = skip_first ? ci : ci - first_c;
            const size_t off = ((size_t)b * L.a.C + ca) * (size_t)L.a.H * L.a.W;
            s.x = L.a.x + off;
            s.c = L.a.c + off;
            s.W = L.a.W;
            s.kind = kDirect;
            s.bytes = L.a.H * L.a.W * 4;
        } else {
            const int cb = skip_first ? ci - first_c : ci;
            const size_t off = ((size_t)b * L.b.C + cb) * (size_t)L.b.H * L.b.W;
            s.x = L.b.x + off;
            s.c = L.b.c + off;
            s.W = L.b.W;
            s.kind = kUp;
            s.bytes = L.b.H * L.b.W * 4;
        }
    }
    return s;
}

// (x, c) of the layer input at (ih, iw), in range, from a resolved channel source.
__device__ __forceinline__ void load_chan(const LayerDev& d, const ChanSrc& s, int ih, int iw, float& x,
                                          float& c) {
    if (s.kind == kDirect) {
        const int i = ih * s.W + iw;
        x = s.x[i];
        c = s.c[i];
    } else if (s.kind == kThresh) {
        x = s.x[ih * s.W + iw];
        c = (x > d.L.thresh) ? 1.0f : 0.0f;
    } else if (s.kind == kPool) {
        const int i = (2 * ih) * s.W + 2 * iw;
        if ((s.W & 1) == 0) {
            const f2 x0 = *(const f2*)(s.x + i), x1 = *(const f2*)(s.x + i + s.W);
            const f2 c0 = *(const f2*)(s.c + i), c1 = *(const f2*)(s.c + i + s.W);
            x = pool4v(x0.x, x0.y, x1.x, x1.y);
            c = pool4v(c0.x, c0.y, c1.x, c1.y);
        } else {
            x = pool4v(s.x[i], s.x[i + 1], s.x[i + s.W], s.x[i + s.W + 1]);
            c = pool4v(s.c[i], s.c[i + 1], s.c[i + s.W], s.c[i + s.W + 1]);
        }
    } else {
        const int sh = nearest_src(ih, d.L.b.H, d.L.H, d.up_scale_h);
        const int sw = nearest_src(iw, d.L.b.W, d.L.W, d.up_scale_w);
        const int i = sh * s.W + sw;
        x = s.x[i];
        c = s.c[i];
    }
}

// One channel plane of {x*c, c} over an IHT x IWT halo tile (origin ih0, iw0) (the weight
// gradient's staging, wgrad_tiled), in a load phase (global -> registers) and a store phase
// (registers -> LDS, row pitch IWP). 256 threads, IWT >= 64: lanes map to columns, waves to rows; every address is clamped into the source plane so all of a thread's loads are issued
// before the first is consumed, and out-of-range elements are zeroed at store time. The plane
// must hold round_up(IHT, 4) rows: the last row group is written unconditionally.
template <int IHT, int IWT, int IWP>
struct PlaneRegs {
    static_assert(IWT >= 64, "lanes map to columns");
    static constexpr int NR = (IHT + 3) / 4;  // rows per thread (waves stride 4 rows)
    static constexpr int NCH = IWT / 64;      // full 64-column chunks
    static constexpr int EX = IWT % 64;       // remaining halo columns, one pass over EX x IHT
    static_assert(EX * IHT <= 256, "one pass for the remaining halo columns");
    float x[NCH][NR], c[NCH][NR];
    float ex, ec;

    __device__ __forceinline__ void load(const LayerDev& d, const ChanSrc& s, int ih0, int iw0, int tid) {
        const int H = d.L.H, W = d.L.W;
        const int lane = tid & 63, r0 = tid >> 6;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int iw = iw0 + ch * 64 + lane;
            const int iwc = iw < 0 ? 0 : (iw >= W ? W - 1 : iw);
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const int ih = ih0 + r0 + 4 * k;
                const int ihc = ih < 0 ? 0 : (ih >= H ? H - 1 : ih);
                load_chan(d, s, ihc, iwc, x[ch][k], c[ch][k]);
            }
        }
        if constexpr (EX != 0) {
            const int r = tid / EX, iw = iw0 + NCH * 64 + tid % EX;
            int ih = ih0 + (r < IHT ? r : IHT - 1);
            ih = ih < 0 ? 0 : (ih >= H ? H - 1 : ih);
            const int iwc = iw < 0 ? 0 : (iw >= W ? W - 1 : iw);
            load_chan(d, s, ih, iwc, ex, ec);
        }
    }

    __device__ __forceinline__ void store(const LayerDev& d, f2* t, int ih0, int iw0, int tid) const {
        const int H = d.L.H, W = d.L.W;
        const int lane = tid & 63, r0 = tid >> 6;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int col = ch * 64 + lane;
            const bool wok = (unsigned)(iw0 + col) < (unsigned)W;
#pragma unroll
            for (int k = 0; k < NR; ++k) {  // rows >= IHT land in the plane's padding rows
                const int r = r0 + 4 * k;
                const bool ok = wok && (unsigned)(ih0 + r) < (unsigned)H;
                const float xv = ok ? x[ch][k] : 0.f, cv = ok ? c[ch][k] : 0.f;
                t[r * IWP + col] = (f2){xv * cv, cv};
            }
        }
        if constexpr (EX != 0) {
            const int r = tid / EX, cx = NCH * 64 + tid % EX;
            const bool ok = (unsigned)(ih0 + r) < (unsigned)H && (unsigned)(iw0 + cx) < (unsigned)W;
            const float xv = ok ? ex : 0.f, cv = ok ? ec : 0.f;
            if (tid < EX * IHT) t[r * IWP + cx] = (f2){xv * cv, cv};
        }
    }
};

// Load and store back to back (no pipelining): one staged plane.
template <int IHT, int IWT, int IWP>
__device__ __forceinline__ void stage_plane(const LayerDev& d, const ChanSrc& s, f2* t, int ih0, int iw0,
                                            int tid) {
    PlaneRegs<IHT, IWT, IWP> r;
    r.load(d, s, ih0, iw0, tid);
    r.store(d, t, ih0, iw0, tid);
}

// ------------------------------------------------------------------------------------------------
// Tile staging through buffer loads, for tiles narrower than a wave (IWT < 64). Every input
// channel plane of a layer shares one geometry, so each thread's element map — its LDS slots, and
// its byte offsets into a full-resolution (source a) and a nearest-upsampled (source b) plane — is
// computed once per workgroup. Per plane a load is then one buffer_load with the plane's base in
// an SGPR resource and the precomputed offset, no address arithmetic; out-of-image elements carry
// an offset past the resource's size, for which the hardware returns 0 (the zero padding).
// Elements are dealt to the NTH threads in row-major order, so consecutive lanes read consecutive
// columns; slots past the tile go to a dump slot after the plane (PLANE_STRIDE).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const float* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ float ld_f32(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
// with a wave-uniform byte offset in soffset (a plane of a multi-plane resource); the range check
// covers voffset + soffset, so an out-of-range voffset (>= 2^31) still reads 0
__device__ __forceinline__ float ld_f32s(__amdgpu_buffer_rsrc_t r, unsigned off, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0));
}

// Pooled-gradient routing (training backward of a layer whose outputs feed a 2x2 max-pool that
// nconv_fwd_pooled materialised with its argmax codes): the output element at window slot `sub`
// (2*row + column) receives the pooled element's gradient when it is that window's first maximum
// (y's slot in code bits 0-1, cout's in bits 2-3), +0 otherwise -- max_pool2d's backward added to
// the other consumer's gradient. Byte offset of the pooled element, or OOB past the pooled plane
// (odd last rows / columns, which no window covers: the load then returns 0).
__device__ __forceinline__ unsigned pool_elem_off(int oh, int ow, int Hp, int Wp, unsigned oob) {
    return ((oh >> 1) < Hp && (ow >> 1) < Wp) ? (unsigned)((oh >> 1) * Wp + (ow >> 1)) * 4u : oob;
}
__device__ __forceinline__ void pool_route(float& gy, float& gco, float gpy, float gpc, unsigned code, unsigned sub) {
    gy += ((code & 3u) == sub) ? gpy : 0.f;
    gco += (((code >> 2) & 3u) == sub) ? gpc : 0.f;
}

__device__ __forceinline__ void st_f32(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, 0);
}
__device__ __forceinline__ void st_f2(__amdgpu_buffer_rsrc_t r, unsigned off, f2 v) {
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, (int)off, 0, 0);
}
__device__ __forceinline__ void st_f4(__amdgpu_buffer_rsrc_t r, unsigned off, f4 v) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, (int)off, 0, 0);
}

template <int IHT, int IWT, int IWP, int MODE, int NTH = 256>
struct TileStager {
    static constexpr int NT = IHT * IWT;
    static constexpr int NE = (NT + NTH - 1) / NTH;  // elements per thread
    static constexpr int PLANE = IHT * IWP;      // f2 slots of the plane ...
    static constexpr int PLANE_STRIDE = PLANE + 2;  // ... + the dump slot, 16-B aligned
    static constexpr bool UP = MODE == NCONV_LOAD_UPCAT_SKIP_FIRST || MODE == NCONV_LOAD_UPCAT_UP_FIRST;
    static constexpr unsigned OOB = 0x80000000u;
    unsigned lofs[NE];       // f2 slot in the plane
    unsigned ga[NE];         // byte offset in a source-a plane (POOL2: of the window's top-left)
    unsigned gb[UP ? NE : 1];  // byte offset in a source-b plane (nearest upsampling)

    __device__ __forceinline__ void init(const LayerDev& d, int ih0, int iw0, int tid) {
        const nconv_layer& L = d.L;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const int e = tid + NTH * k;
            const int r = e / IWT, col = e - r * IWT;
            const int ih = ih0 + r, iw = iw0 + col;
            const bool in = e < NT && (unsigned)ih < (unsigned)L.H && (unsigned)iw < (unsigned)L.W;
            lofs[k] = e < NT ? r * IWP + col : PLANE;
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
    }

    // Issue the loads of one channel plane (no wait). THRESH leaves c to store().
    __device__ __forceinline__ void load(const ChanSrc& s, float (&x)[NE], float (&c)[NE]) const {
        const __amdgpu_buffer_rsrc_t rx = plane_rsrc(s.x, s.bytes);
        if constexpr (MODE == NCONV_LOAD_THRESH) {
#pragma unroll
            for (int k = 0; k < NE; ++k) x[k] = ld_f32(rx, ga[k]);
        } else if constexpr (MODE == NCONV_LOAD_POOL2) {
            const __amdgpu_buffer_rsrc_t rc = plane_rsrc(s.c, s.bytes);
            const unsigned row = (unsigned)s.W * 4u;
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const unsigned o2 = ga[k] == OOB ? OOB : ga[k] + row;
                const f2 x0 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, ga[k], 0, 0));
                const f2 x1 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, o2, 0, 0));
                const f2 c0 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rc, ga[k], 0, 0));
                const f2 c1 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rc, o2, 0, 0));
                x[k] = pool4v(x0.x, x0.y, x1.x, x1.y);
                c[k] = pool4v(c0.x, c0.y, c1.x, c1.y);
            }
        } else {
            const __amdgpu_buffer_rsrc_t rc = plane_rsrc(s.c, s.bytes);
            const bool up = UP && s.kind == kUp;  // wave-uniform
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const unsigned o = UP ? (up ? gb[UP ? k : 0] : ga[k]) : ga[k];
                x[k] = ld_f32(rx, o);
                c[k] = ld_f32(rc, o);
            }
        }
    }

    __device__ __forceinline__ void store(f2* t, const float (&x)[NE], const float (&c)[NE], float thresh) const {
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const float cv = (MODE == NCONV_LOAD_THRESH) ? (x[k] > thresh ? 1.0f : 0.0f) : c[k];
            t[lofs[k]] = (f2){x[k] * cv, cv};
        }
    }
};

// (x, c) of layer-input pixel (ih, iw) of a resolved channel, zero outside the image (buffer
// loads: out-of-range offsets read 0). THRESH leaves c to the caller.
template <int MODE>
__device__ __forceinline__ void load_px(const LayerDev& d, const ChanSrc& s, int ih, int iw, float& x, float& c) {
    const nconv_layer& L = d.L;
    const bool in = (unsigned)ih < (unsigned)L.H && (unsigned)iw < (unsigned)L.W;
    constexpr unsigned OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t rx = plane_rsrc(s.x, s.bytes);
    if constexpr (MODE == NCONV_LOAD_THRESH) {
        x = ld_f32(rx, in ? (unsigned)(ih * s.W + iw) * 4u : OOB);
        c = 0.f;
    } else if constexpr (MODE == NCONV_LOAD_POOL2) {
        const __amdgpu_buffer_rsrc_t rc = plane_rsrc(s.c, s.bytes);
        const unsigned o1 = in ? (unsigned)((2 * ih) * s.W + 2 * iw) * 4u : OOB;
        const unsigned o2 = in ? o1 + (unsigned)s.W * 4u : OOB;
        const f2 x0 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, o1, 0, 0));
        const f2 x1 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rx, o2, 0, 0));
        const f2 c0 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rc, o1, 0, 0));
        const f2 c1 = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rc, o2, 0, 0));
        x = pool4v(x0.x, x0.y, x1.x, x1.y);
        c = pool4v(c0.x, c0.y, c1.x, c1.y);
    } else {
        const __amdgpu_buffer_rsrc_t rc = plane_rsrc(s.c, s.bytes);
        unsigned off;
        if (s.kind == kUp) {
            const int sh = nearest_src(in ? ih : 0, L.b.H, L.H, d.up_scale_h);
            const int sw = nearest_src(in ? iw : 0, L.b.W, L.W, d.up_scale_w);
            off = in ? (unsigned)(sh * s.W + sw) * 4u : OOB;
        } else {
            off = in ? (unsigned)(ih * s.W + iw) * 4u : OOB;
        }
        x = ld_f32(rx, off);
        c = ld_f32(rc, off);
    }
}

