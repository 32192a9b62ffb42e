// nconv_internal.h — launcher interface between the C-ABI layer (nconv_capi.hip) and the kernel
// translation units. Not part of the public ABI.
#pragma once
#include "nconv_common.h"

namespace nconv {

struct TailArgs {
    const float* w7;
    const float* b7;
    const float* s7;
    float eps7;
    int off;
    int out_h, out_w;
    float* out_c;
    float* py;  // optional 2x2 max-pooled copies of y / cout (non-tail launches), (B,Cout,Ho/2,Wo/2)
    float* pc;
    unsigned* parg;  // optional (with py): per pooled element the two first-maximum slots
    // fused head (nconv_fwd_head): nconv1 evaluated while staging nconv2's input
    const float* s_in;  // sparse depth (B, 1, H, W)
    const float* w1;    // nconv1 weight (8, 1, 5, 5), bias, s[o]
    const float* b1;
    const float* s1;
    float eps1, thresh1;
    float* y1;  // optional (training): nconv1's outputs (B, 8, H, W) written by the fused head
    float* c1;
    float* y6;  // optional (training): nconv6's outputs written by the fused tail (phase kernel)
    float* c6;
};

struct BwdArgs {
    const float* y;
    const float* co;
    const float* gy;
    const float* gco;  // may be null (= 0)
    float* gxa;
    float* gca;
    float* gxb;
    float* gcb;
    float* gw;
    float* gb;
    float* ws;  // workspace
    size_t ws_bytes;
    int accumulate;  // 1: += into gxa/gca/gxb/gcb; 0: overwrite every element
    int defer;       // 1: leave the weight gradient as partial rows (reduced by launch_wgrad_reduce_multi)
    int* nparts;     // out (defer): the number of partial rows written
    // optional: gradient of the 2x2 max-pooled outputs (B, Cout, Ho/2, Wo/2) and the pooling argmax
    // codes (nconv_fwd_pooled), routed into gy / gcout while {gN, gD} are formed (pool_route)
    const float* gpy;
    const float* gpc;
    const unsigned* parg;
    // optional fused weight gradient of the producer nconv1 (1 -> 8, 5x5, threshold load, padding 2)
    // in the input gradient's epilogue: its sparse input S, bias, normaliser, eps, threshold, and
    // the per-workgroup partial rows (200 weights, 8 sum gy, 8 sum gcout*cout) it writes
    const float* hS;
    const float* hb;
    const float* hs;
    float heps, hthresh;
    float* hpart;
    float* hgw;       // nconv1's gW / gb (undeferred: reduced right after the kernel)
    float* hgb;
    int* hnparts;     // out (defer): the number of nconv1 partial rows written
    // optional fused backward of the consumer nconv7 (8 -> 1, 1x1, padding 2) of this layer's
    // outputs: gy / gco of this layer are formed from nconv7's (gy, y, cout) planes (B, 1, Ho + 4,
    // Wo + 4) and its weights; nconv7's weight gradient goes to t7part (10-float partial rows)
    const float* t7w;
    const float* t7b;
    const float* t7s;
    float t7eps;
    const float* t7gy;
    const float* t7y;
    const float* t7co;
    float* t7part;
    float* t7gw;
    int* t7nparts;
    int t7ph, t7pw, t7pc0;  // nconv7's planes: (t7ph, t7pw) holding its grid from row / column t7pc0
    const float* box;  // optional precomputed box weights of an exactly-2x UPCAT layer (dgrad_phase)
};
// nconv7 (1x1, padding 2) consumer fused into its producer's backward (T7): byte offset of nconv6
// pixel (oh, ow) in nconv7's planes -- its (Ho + 4) x (Wo + 4) grid, or the window of it that DNET's
// crop keeps (t7ph x t7pw from row / column t7pc0) -- or oob outside nconv6's grid or the window (a
// zero gradient there); nconv7's {gN7, gD7} from its (gy, y, cout) (its cout gradient is 0);
// nconv6's (gy, gcout) from them and w7[o] as nconv7's own 1x1 input gradient forms them
// (dgrad_tiled<8,1,1>'s epilogue, same operations)
__device__ __forceinline__ unsigned t7_off(const BwdArgs& a, int oh, int ow, int Ho, int Wo, unsigned oob) {
    const int r = oh + 2 - a.t7pc0, c = ow + 2 - a.t7pc0;
    return ((unsigned)oh < (unsigned)Ho && (unsigned)ow < (unsigned)Wo && (unsigned)r < (unsigned)a.t7ph &&
            (unsigned)c < (unsigned)a.t7pw)
               ? (unsigned)(r * a.t7pw + c) * 4u
               : oob;
}
__device__ __forceinline__ void t7_nd(const BwdArgs& a, float gy9, float y9, float co9, float& gN7, float& gD7) {
    nconv_grad_nd(gy9, 0.f, y9, co9, a.t7eps, a.t7b[0], a.t7s[0], gN7, gD7);
}
__device__ __forceinline__ void t7_gy(float w7, float gN7, float gD7, float y, float co, float& gy, float& gco) {
    const float gxc = fmaf(w7, gN7, 0.f), gc = fmaf(w7, gD7, 0.f);  // the 1x1 dgrad's accumulators
    gy = gxc * co;
    gco = fmaf(gxc, y, gc);
}
size_t bwd_tail_workspace_bytes(const nconv_layer& L6);
size_t bwd_head_workspace_bytes(const nconv_layer& L2);

// One layer's deferred weight-gradient reduction (nconv_wgrad_reduce): its workspace's partial rows.
struct RedJob {
    const float* part;  // nblk partial rows of nw + 2 cout floats, then the kReduceSplit slice rows
    const float* wsum;
    float* gw;
    float* gb;
    int nblk, nw, cout, fan;
    // flat (nconv_wgrad_reduce_ex sums): gb[0] = the sum of part[0 .. nblk) (nw = 0, cout = 1) in a
    // fixed order -- kSumChunks chunk sums into sub, then their tree
    int flat;
    float* sub;
};
constexpr int kMaxRedJobs = 16;
constexpr int kSumChunks = 1024;
int launch_wgrad_reduce_multi(int n, const RedJob* jobs, hipStream_t st, const char** why);

// Forward. Return 0, or a negative errno with *why set.
int launch_fwd(const LayerDev& d, float* y, float* yc, float* py, float* pc, unsigned* parg, hipStream_t st,
               const char** why);
bool fwd_mfma_supported(const nconv_layer& L, bool tail, bool pool);
bool launch_fwd_mfma(const LayerDev& d, float* y, float* yc, const TailArgs& t, bool tail, hipStream_t st);
// exact-fp32 UPCAT layers with the upsampled half at native resolution (nconv_fwd_phase.hip)
bool fwd_phase_supported(const nconv_layer& L, bool tail);
bool launch_fwd_phase(const LayerDev& d, float* y, float* yc, const TailArgs& t, bool tail, hipStream_t st);
size_t phase_weight_floats(const nconv_layer& L);
int launch_phase_weights(int n, const float* const* w, const int* cin, const int* up_first, float* const* out,
                         hipStream_t st, const char** why);
// enum nconv_kernel of the forward / input-gradient / weight-gradient launches (nconv_plan)
int plan_fwd(const nconv_layer& L);
void plan_bwd(const nconv_layer& L, int* dgrad, int* wgrad);
int launch_fwd_head(const LayerDev& d2, const TailArgs& t, float* y, float* yc, hipStream_t st, const char** why);
// exact-fp32 fused head (nconv_fwd_head.hip); d2.L.waux = the composed confidence weights
int launch_fwd_head_exact(const LayerDev& d2, const TailArgs& t, float* y, float* yc, hipStream_t st,
                          const char** why);
int launch_weight_prologue(int n, float* const* w, const int* cout, const int* fan_in, float* const* s,
                           const float* w1, const float* w2, float* w21, int nphase, const float* const* pw,
                           const int* pcin, const int* pup_first, float* const* pout, hipStream_t st,
                           const char** why);
int launch_train_prologue(int n, float* const* w, const int* cout, const int* fan_in, const int* sp,
                          float* const* s, int head1, int head2, float* w21, unsigned* sync, int nphase,
                          const int* players, const int* pup_first, float* const* pout, float* const* pbox,
                          hipStream_t st, const char** why);
int launch_head_weights(const float* w1, const float* s1, const float* w2, float* out, hipStream_t st,
                        const char** why);
int launch_fwd_tail(const LayerDev& d, const TailArgs& t, float* out, hipStream_t st, const char** why);
int launch_weight_prep(int n, float* const* w, const int* cout, const int* fan_in, const int* sp,
                       float* const* s, hipStream_t st, const char** why);

// Grid sizing (nconv_occ.hip): CUs of the current device, resident workgroups per CU of a kernel
// on it (>= 1); cached per device ordinal, thread-safe.
int dev_cus();
int dev_occupancy(const void* kernel, int threads, size_t dyn_lds);

// Backward.
size_t bwd_workspace_bytes(const LayerDev& d);
// weight gradient on the bf16 matrix cores (nconv_wgrad_bf.hip): np = 2 (bf16x3) or 3 (bf16x9) split
// parts; at most max_blocks partial rows into part; returns the number written
template <int CIN, int COUT, int K, int MODE>
int go_wgrad_bf(const LayerDev& d, const BwdArgs& a, float* part, int max_blocks, int np, hipStream_t st);
// input gradient on the bf16 matrix cores (nconv_dgrad_bf.hip), np as go_wgrad_bf
template <int CIN, int COUT, int K, int MODE>
void go_dgrad_bf(const LayerDev& d, const BwdArgs& a, float* tmp_x, float* tmp_c, int np, hipStream_t st);
int launch_bwd(const LayerDev& d, const BwdArgs& a, hipStream_t st, const char** why);
// nconv1's weight-gradient partial rows of the fused head (200 weights, 8 sum gy, 8 sum gcout*cout)
constexpr int kHeadNw = 8 * 25, kHeadStride = kHeadNw + 16;
// Dense convolutions (RGB-guided model).
int dense_cout_tile(int Cout);
size_t dense_packed_floats(int kind, int Cin, int Cout);
int launch_dense_pack(int kind, int Cin, int Cout, const float* w, const float* scale, float* wp, hipStream_t st,
                      const char** why);
int launch_dense_conv(const nconv_dense_conv& p, hipStream_t st, const char** why);
int launch_bilinear_ac(const float* x, int B, int C, int H, int W, float* y, int Ho, int Wo, hipStream_t st,
                       const char** why);
int launch_conv3x3_c1(const float* x, int B, int Cin, int H, int W, const float* w, const float* res, float* out,
                      hipStream_t st, const char** why);
size_t dense_wgrad_workspace_bytes(const nconv_dense_wgrad& g);
int launch_dense_wgrad(const nconv_dense_wgrad& g, float* ws, size_t ws_bytes, hipStream_t st, const char** why);

// Training-mode BatchNorm (+ ReLU).
size_t bn_workspace_bytes(const nconv_bn_train& p);
int launch_bn_train_fwd(const nconv_bn_train& p, float* ws, hipStream_t st, const char** why);
size_t relu_bias_workspace_bytes(int B, int C, int H, int W);
int launch_relu_bias_bwd(int B, int C, int H, int W, const float* g, const float* out, float* gm, float* gbias,
                         float* ws, hipStream_t st, const char** why);
int launch_bn_train_bwd(const nconv_bn_train& p, const float* gy, float* gx, float* ggamma, float* gbeta, float* ws,
                        hipStream_t st, const char** why);

// Training loss (utils.py calculate_loss) on B planes.
struct LossArgs {
    const float* r;
    const float* t;
    long long rbs, rs;  // image / row strides of r (elements)
    long long tbs, ts;  // ... of t
    int B, H, W;
};
size_t loss_workspace_bytes(int B, int H, int W);
int launch_loss_fwd(const LossArgs& a, int grad_loss, float* loss, float* ws, hipStream_t st, const char** why);
int launch_loss_bwd(const LossArgs& a, int grad_loss, const float* gout, const float* ws, float* g, hipStream_t st,
                    const char** why);

}  // namespace nconv
