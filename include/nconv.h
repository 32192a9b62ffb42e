/*
 * nconv.h — C ABI of libnconv.so, the MI355X (gfx950) normalized-convolution library.
 *
 * The reference (lllllcf/Realtime-Depth-Estimation-Nconv) has no native code: its boundary is the
 * PyTorch nn.Module API of models/step1.py. Each entry point below replaces a specific group of
 * PyTorch ops the reference issues on its hot path; the replaced file:line is cited per function.
 * The Python host layer (realtime-depth-estimation-nconv_amd/) binds these with ctypes; see
 * INTEGRATION.md for the binding a maintainer of the reference would add.
 *
 * Conventions (all entry points):
 *   - every buffer is a caller-owned device pointer to contiguous fp32 NCHW memory; the library
 *     never allocates, frees or synchronises;
 *   - work is enqueued on `stream` (a hipStream_t passed as void*; NULL = the null stream);
 *   - return 0 on success or a negative errno-style code; nconv_last_error() then describes it
 *     (thread-local string, valid until the next call on the same thread);
 *   - stateless and re-entrant; safe to capture into a hipGraph (no host sync inside).
 */
#ifndef NCONV_H
#define NCONV_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NCONV_ABI_VERSION 22

/* How a layer's input (data x, confidence c) is produced from its source tensors. These are the
 * DNET glue ops fused into the layer's load stage (models/step1.py:53,61-90). */
enum nconv_load_mode {
    NCONV_LOAD_PLAIN = 0,            /* x = a.x, c = a.c                                   (step1.py:57,92)    */
    NCONV_LOAD_THRESH = 1,           /* x = a.x, c = float(a.x > thresh)                    (step1.py:53-56)    */
    NCONV_LOAD_POOL2 = 2,            /* x = maxpool2x2(a.x), c = maxpool2x2(a.c), independent (step1.py:62-75) */
    NCONV_LOAD_UPCAT_SKIP_FIRST = 3, /* x = cat(a.x, up(b.x)), c likewise                   (step1.py:78-85)    */
    NCONV_LOAD_UPCAT_UP_FIRST = 4    /* x = cat(up(b.x), a.x), c likewise                   (step1.py:88-90)    */
};

/* Arithmetic of the NConv sums (nconv_layer.math: forward N = W*(x*c), D = W*c; nconv_layer.bwd_math:
 * the backward's products). The zero value is the reference's arithmetic (F.conv2d in fp32,
 * models/step1.py:119-122), so a zero-initialised descriptor computes exact fp32. */
enum nconv_math {
    NCONV_MATH_FP32 = 0,   /* default: exact fp32 products (forward: packed FP32 FMA on the vector ALU;
                              backward: fp32 matrix cores for the weight gradient, packed FP32 for the
                              input gradient) */
    NCONV_MATH_BF16X3 = 1, /* bf16 matrix cores on split operands, v = hi + lo, products
                              hi*hi + lo*hi + hi*lo in fp32 (<= ~1.1e-5 relative per product), for
                              the 8-output-channel 5x5 (8 in) / 3x3 (16 in) layers; others FP32 */
    NCONV_MATH_BF16X9 = 2  /* exact products on the bf16 matrix cores: v = v0 + v1 + v2 and
                              w = w0 + w1 + w2 (three bf16 parts, an exact decomposition), all nine
                              partial products (each exact in fp32) accumulated in fp32, for the same
                              layers as BF16X3; others FP32 */
};

/* Kernel family a launch runs (nconv_plan). */
enum nconv_kernel {
    NCONV_KERNEL_GENERIC = 0,     /* direct one-thread-per-element kernels (any NConv2d geometry)       */
    NCONV_KERNEL_TILED_FP32 = 1,  /* LDS-tiled, exact fp32 products on the vector ALU (packed FP32)     */
    NCONV_KERNEL_MFMA_FP32 = 2,   /* fp32 matrix cores, exact fp32 products                            */
    NCONV_KERNEL_MFMA_BF16X3 = 3, /* bf16 matrix cores, two-part split operands (NCONV_MATH_BF16X3)    */
    NCONV_KERNEL_MFMA_BF16X9 = 4, /* bf16 matrix cores, three-part split, exact products (BF16X9)      */
    NCONV_KERNEL_TILED_FP32_PHASE = 5 /* as TILED_FP32, the nearest-2x-upsampled half of the input
                                     channels at native resolution: forward with phase weights
                                     (nconv_layer.waux, nconv_phase_weights); input gradient as
                                     4x4 box-summed weights per low pixel (exact-2x UpCat layers
                                     with bwd_math FP32, no waux needed)                         */
};

/* One source tensor pair (data, confidence), physical shape (B, C, H, W). */
typedef struct nconv_src {
    const float* x;
    const float* c; /* may be NULL for NCONV_LOAD_THRESH */
    int C, H, W;
} nconv_src;

/* One NConv2d application (models/step1.py:97-149) plus its fused input glue. */
typedef struct nconv_layer {
    int B;
    int Cin, H, W;     /* logical layer input, after the glue (e.g. H = a.H/2 for POOL2)      */
    int Cout, Ho, Wo;  /* output: Ho = (H + 2PH - DH(KH-1) - 1)/SH + 1                         */
    int KH, KW, SH, SW, PH, PW, DH, DW, groups;
    float eps;         /* NConv2d.eps = 1e-7 (step1.py:103)                                     */
    int load_mode;     /* enum nconv_load_mode                                                  */
    float thresh;      /* NCONV_LOAD_THRESH threshold, 0.01 in DNET (step1.py:53)               */
    nconv_src a;       /* plain / thresholded / pooled / skip source                             */
    nconv_src b;       /* low-resolution source of the UPCAT modes (unused otherwise)            */
    const float* weight; /* (Cout, Cin/groups, KH, KW), positive in practice                   */
    const float* bias;   /* (Cout)                                                              */
    const float* wsum;   /* (Cout): s[o] = sum of weight[o] (step1.py:141-144), see nconv_weight_prep */
    int math;            /* enum nconv_math of the forward sums (0 = NCONV_MATH_FP32; unknown: -EINVAL) */
    int bwd_math;        /* enum nconv_math of the backward's products (nconv_bwd, weight and input
                            gradient of the 3x3 / 5x5 layers with Cin > 1): 0 = NCONV_MATH_FP32
                            (exact products), BF16X3 / BF16X9 = split-bf16 matrix cores; unknown:
                            -EINVAL */
    const float* waux;   /* optional precomputed auxiliary weights (NULL = unused):
                            - UPCAT layer: its phase weights (nconv_phase_weights). With exact-fp32
                              math, 16 -> 8 channels (8 + 8), 3x3, stride 1 and an exact nearest 2x
                              upsampling (H = 2 b.H, W = 2 b.W) the forward then convolves source b
                              at its own resolution: 4 fp32 taps of summed weights instead of 9 per
                              pixel (the regrouping (w1 + w2) * v of w1 * v + w2 * v); ignored
                              otherwise;
                            - nconv2 of nconv_fwd_head with exact-fp32 math: the composed
                              confidence weights (nconv_head_weights), required there */
} nconv_layer;

/* ABI version, for the Python loader's sanity check. */
int nconv_abi_version(void);

/* Description of the last error on this thread ("" if none). */
const char* nconv_last_error(void);

/* EnforcePos + confidence-normaliser prologue for n layers in ONE launch.
 * Replaces EnforcePos.__call__ (models/step1.py:190-193, softplus beta=10 threshold=20 at :206-207,
 * applied in place when apply_softplus[i] != 0, i.e. module.training) and the per-layer
 * s = weight.view(Cout,-1).sum(-1) of NConv2d.forward (models/step1.py:141-144).
 * weights[i] has counts[i] = Cout_i * fan_in_i floats; wsums[i] receives Cout_i floats. */
int nconv_weight_prep(int n, float* const* weights, const int* couts, const int* fan_ins,
                      const int* apply_softplus, float* const* wsums, void* stream);

/* Phase weights (nconv_layer.waux) of n UPCAT layers with 8 output channels, 3x3 kernels and 8
 * nearest-2x-upsampled input channels, one launch; call after nconv_weight_prep (they are sums of
 * the current weights: 1, 2 or 4 fp32 weights each, in a fixed order). weights[i] is the layer's
 * (8, cins[i], 3, 3) weight, its upsampled channels are [up_first[i], up_first[i] + 8) (8 for
 * cat(skip, up(low)), 0 for cat(up(low), skip)); wphases[i] receives 1024 floats
 * (= nconv_phase_weights_floats of the layer). The nearest-2x upsampling maps a 3x3 window onto a
 * 2x2 block of source-b pixels; which taps share a pixel depends only on the parity of the window's
 * first row / column (models/step1.py:78-90 glue + :119-122). */
size_t nconv_phase_weights_floats(const nconv_layer* L); /* 0 if L has no phase form */
int nconv_phase_weights(int n, const float* const* weights, const int* cins, const int* up_first,
                        float* const* wphases, void* stream);

/* The inference (eval-mode) weight prologue in ONE launch: the normalisers wsums[i] of n layers
 * (nconv_weight_prep with apply_softplus all 0: EnforcePos is inactive outside training), the exact
 * fused head's auxiliary weights (nconv_head_weights of nconv1 head_w1 (8, 1, 5, 5) and nconv2
 * head_w2 (8, 8, 5, 5) into w21; nconv1's s1 recomputed in-kernel with nconv_weight_prep's
 * arithmetic; skipped when w21 is NULL) and the phase weights of nphase UpCat layers
 * (nconv_phase_weights' arguments). Every output is bitwise what the three separate calls write;
 * the roles read the weights only, so they need no order (replaces three launches per forward). */
int nconv_weight_prologue(int n, float* const* weights, const int* couts, const int* fan_ins,
                          float* const* wsums, const float* head_w1, const float* head_w2, float* w21,
                          int nphase, const float* const* phase_weights, const int* phase_cins,
                          const int* phase_up_first, float* const* wphases, void* stream);

/* The training pass's weight prologue in one launch (replaces models/step1.py:190-207's EnforcePos
 * pre-hooks of DNET's nine layers, whose forward then needs the normalisers and the auxiliaries
 * below: five launches -- nconv_weight_prep, nconv_head_weights, nconv_phase_weights and the three
 * backward box-weight builds -- become one). Layer i (weights[i], couts[i] x fan_ins[i]) gets
 * EnforcePos's softplus in place when softplus[i] (softplus may be NULL: none) and its normalisers
 * in wsums[i]. With w21 != NULL, layers head1 / head2 are nconv1 (8 x 1 x 5 x 5) and nconv2 (8 x 8 x
 * 5 x 5) and w21 receives the exact head's weights (nconv_head_weights, NCONV_HEAD_WEIGHTS_FLOATS);
 * `sync` is then a device counter that is 0 before the call and is left 0 by it (the head's
 * workgroups write nconv1 / nconv2 back once all of them have staged them: one counter per stream
 * that runs this concurrently).
 * Phase layer k is layer phase_layers[k] (8 x 16 x 3 x 3, upsampled channels from phase_up_first[k]
 * = 0 or 8): wphases[k] receives its phase weights (nconv_phase_weights) and, when wboxes and
 * wboxes[k] are non-NULL, wboxes[k] its 1,024 box weights for the phase-form input gradient
 * (nconv_bwd_io.box_weights). Each output is bitwise what the separate calls write after
 * nconv_weight_prep. Every role applies the softplus while staging; a layer is written back by its
 * only reader, or by the last head workgroup. Returns 0 or -EINVAL. */
int nconv_train_prologue(int n, float* const* weights, const int* couts, const int* fan_ins, const int* softplus,
                         float* const* wsums, int head1, int head2, float* w21, unsigned int* sync, int nphase,
                         const int* phase_layers, const int* phase_up_first, float* const* wphases,
                         float* const* wboxes, void* stream);

/* Forward of one NConv2d with fused input glue.
 * Replaces models/step1.py:119-147 (2x F.conv2d, mul, div, bias add, confidence normalisation)
 * plus the glue op that feeds it (step1.py:53 / 62-75 / 78-90).
 * y, cout: (B, Cout, Ho, Wo). */
int nconv_fwd(const nconv_layer* L, float* y, float* cout, void* stream);

/* nconv_fwd plus, in the same launch, the 2x2/s2 max-pool of both outputs (torch semantics:
 * first maximum wins, NaN propagates) into y_pool, cout_pool (B, Cout, Ho/2, Wo/2): the input of
 * the next down layer (models/step1.py:62-75), which then loads it with NCONV_LOAD_PLAIN instead
 * of re-reading and pooling the full-resolution tensors. Built for the tiled DNET layer shapes
 * (returns -EOPNOTSUPP otherwise). argmax (may be NULL; exact-fp32 tiled layers only): one 32-bit
 * word per pooled element (not a byte: the backward's staging then loads it like its float
 * operands, with no conversion ahead of its use), the window slot (2*row + column) of y's first
 * maximum in bits 0-1 and of cout's in bits 2-3 -- what nconv_bwd_ex routes the pooled tensors' gradient by (the indices of
 * max_pool2d_with_indices, step1.py:62-75 under autograd). */
int nconv_fwd_pooled(const nconv_layer* L, float* y, float* cout, float* y_pool, float* cout_pool,
                     unsigned int* argmax, void* stream);

/* Fused head: nconv1 on the thresholded sparse depth (models/step1.py:53-57;
 * L1: Cin 1, Cout 8, 5x5, padding 2, NCONV_LOAD_THRESH) is evaluated while staging nconv2's input
 * tile (step1.py:58; L2: 8 -> 8, 5x5, padding 2, stride 1; its sources are not read), so nconv1's
 * 8-channel output never reaches HBM. Writes nconv2's y, cout (B, 8, H, W) and their 2x2 max-pooled
 * copies (B, 8, H/2, W/2) like nconv_fwd_pooled. L2->math selects the arithmetic:
 *  - NCONV_MATH_FP32: exact fp32 (nconv_fwd_head.hip). nconv1 visits only the nonzero taps of each
 *    window (bitwise its dense sums); nconv2's confidence mass D2 is the 9x9 convolution of the
 *    binary mask c0 with the composed weights sum_i W2[o,i] (x) W1[i] / s1[i] that L2->waux must
 *    hold (nconv_head_weights), on the bf16 matrix cores with exact products (c0 is 0 or 1, each
 *    weight the exact sum of three bf16 parts) and fp32 accumulation, except in tiles whose window
 *    nconv2's zero padding truncates;
 *  - NCONV_MATH_BF16X3 / BF16X9: the matrix-core head (nconv1 uses the same split).
 * Training (exact fp32 only; all three or NULL): y1, cout1 (B, 8, H, W) receive nconv1's outputs
 * (bitwise nconv_fwd's: the nonzero-tap sums are the dense sums) for the backward, argmax the
 * pooling codes as nconv_fwd_pooled's. */
int nconv_fwd_head(const nconv_layer* L1, const nconv_layer* L2, float* y, float* cout, float* y_pool,
                   float* cout_pool, unsigned int* argmax, float* y1, float* cout1, void* stream);

/* Auxiliary weights of the exact fused head (L2->waux of nconv_fwd_head): w21 receives
 * NCONV_HEAD_WEIGHTS_FLOATS floats. First the composed confidence weights W21[o][qh][qw] = sum_i
 * (1 / s1[i]) sum W2[o][i][kh][kw] W1[i][kh'][kw'] over kh + kh' = qh, kw + kw' = qw (fp64, rounded
 * once to fp32; s1 = L1->wsum), each split exactly into three bf16 parts and laid out as the A
 * operands of the head's matrix-core D2 (1536 dwords, nconv_fwd_head.hip kFrag), then nconv2's
 * weights transposed to [i][kh][kw][o] (1600 floats). nconv1's cout = D1 / s1
 * (models/step1.py:141-147), so nconv2's D2 = sum_i W2[o,i] * c1[i] = W21[o] * c0 wherever nconv2's
 * window is not truncated by its zero padding. Call after nconv_weight_prep. */
#define NCONV_HEAD_WEIGHTS_FLOATS 3136
int nconv_head_weights(const nconv_layer* L1, const nconv_layer* L2, float* w21, void* stream);

/* Fused tail: the last 3x3 NConv (nconv6, step1.py:88-90) with its 1x1 successor (nconv7,
 * step1.py:92) evaluated in the epilogue, written straight into the (cropped) output
 * (step1.py:94). L6 describes nconv6 (stride 1, no dilation, groups 1). Output pixel (r, c) of
 * `out` (B, 1, out_h, out_w) is nconv7's output at (r + crop0, c + crop0) of its (Ho6+2*p7) x
 * (Wo6+2*p7) grid, i.e. nconv6 pixel (r + crop0 - p7, c + crop0 - p7); positions in nconv7's zero
 * border get b7. crop0 = 1 is DNET's crop; crop0 = 0 with the full grid is nconv7's whole output.
 * out_c (nullable) receives the matching output confidence. Training (exact fp32, exactly-2x
 * phase form only; both or NULL): y6, cout6 (B, Cout6, Ho6, Wo6) receive nconv6's outputs, which
 * the backward reads; the output window must then cover every nconv6 pixel (crop0 <= p7,
 * crop0 + out_h - p7 >= Ho6, crop0 + out_w - p7 >= Wo6), else -EINVAL. */
int nconv_fwd_tail(const nconv_layer* L6, const float* w7, const float* b7, const float* wsum7,
                   int cin7, int p7, float eps7, float* out, float* out_c, int out_h, int out_w, int crop0,
                   float* y6, float* cout6, void* stream);

/* Which kernels nconv_fwd (without fused pooling) and nconv_bwd run for L (enum nconv_kernel):
 * the arithmetic a descriptor selects, made observable to hosts and tests. Host-only (no device
 * work); any output pointer may be NULL. Returns 0 or -EINVAL for an invalid descriptor. */
int nconv_plan(const nconv_layer* L, int* fwd_kernel, int* dgrad_kernel, int* wgrad_kernel);

/* Workspace needed by nconv_bwd (bytes). */
size_t nconv_bwd_workspace_bytes(const nconv_layer* L);

/* Backward of nconv_fwd (autograd of models/step1.py:116-149 plus the glue's backward:
 * max_pool2d routes to the first maximum of each window, nearest-upsample sums, cat splits).
 * Inputs: y, cout (the forward outputs), gy, gcout (their gradients; gcout may be NULL = 0).
 * Outputs (any may be NULL if not needed):
 *   gxa, gca : gradients of source a's (x, c)      — same shape as a
 *   gxb, gcb : gradients of source b's (x, c)      — same shape as b (UPCAT modes)
 *              with (flags & NCONV_BWD_ACCUMULATE) these four are added into; otherwise every
 *              element is overwritten (no zero-fill needed)
 *   gw       : (Cout, Cin/groups, KH, KW) weight gradient, OVERWRITTEN
 *   gbias    : (Cout) bias gradient, OVERWRITTEN
 * The closed form: gN = gy/(D+eps), gD = -gy*N/(D+eps)^2 + gcout/s,
 *   gb = sum gy, gs = -sum gcout*D/s^2, gW = corr(x*c, gN) + corr(c, gD) + gs,
 *   g(xc) = W^T * gN, gx = g(xc)*c, gc = W^T * gD + g(xc)*x.
 * D and N/(D+eps) are recovered from the saved outputs as cout*s and y-b. */
#define NCONV_BWD_ACCUMULATE 1u
/* (flags & NCONV_BWD_DEFER_REDUCE): the weight gradient is left in the workspace as per-workgroup
 * partial rows and nconv_bwd returns their number (>= 0; 0 when gw and gbias are both NULL) instead
 * of 0; gw / gbias are written by a later nconv_wgrad_reduce over that workspace (which must stay
 * untouched until then). A training backward defers every layer and reduces them all in two
 * launches instead of two per layer. Same sums, same fixed order: the result is bitwise that of
 * the undeferred call. */
#define NCONV_BWD_DEFER_REDUCE 2u
/* Accepted and ignored since ABI 21: the input and the weight gradient always run as two kernels
 * (the one-kernel form of ABI 19-20 measured slower and was removed). */
#define NCONV_BWD_SEPARATE 4u

int nconv_bwd(const nconv_layer* L, const float* y, const float* cout, const float* gy,
              const float* gcout, float* gxa, float* gca, float* gxb, float* gcb, float* gw,
              float* gbias, void* workspace, size_t workspace_bytes, unsigned flags, void* stream);

/* nconv_bwd with its tensors in one struct, plus the gradient arriving through a 2x2 max-pool of
 * this layer's outputs (training: the next down layer read the y_pool / cout_pool that
 * nconv_fwd_pooled materialised, so its input gradient is pooled-sized): gy_pool, gcout_pool
 * (B, Cout, Ho/2, Wo/2) are added to gy / gcout at each window's first maximum, as pool_argmax
 * (that nconv_fwd_pooled call's codes) records -- the max_pool2d backward of step1.py:62-75 summed
 * with the other consumer's gradient, without a full-resolution read-modify-write. All three or
 * none; with them, built for the exact-fp32 8->8 5x5 stride-1 layers with NCONV_LOAD_PLAIN
 * (-EOPNOTSUPP otherwise). Returns as nconv_bwd. */
typedef struct nconv_bwd_io {
    const float* y;
    const float* cout;
    const float* gy;
    const float* gcout;             /* may be NULL (= 0) */
    float* gxa;
    float* gca;
    float* gxb;
    float* gcb;
    float* gw;
    float* gbias;
    const float* gy_pool;           /* optional pooled-output gradient (see above) */
    const float* gcout_pool;
    const unsigned int* pool_argmax;
    /* optional: the weight gradient of the layer that produced L's input, fused into L's input
     * gradient (DNET training: nconv2's backward computes nconv1's gW / gb in-tile, so nconv1's
     * input gradient never reaches HBM and nconv1 needs no nconv_bwd). head = nconv1's descriptor
     * (1 -> 8, 5x5, padding 2, stride 1, NCONV_LOAD_THRESH on the sparse depth; its output is L's
     * source a); L must be an exact-fp32 8 -> 8 5x5 layer with NCONV_LOAD_PLAIN. head_workspace:
     * nconv_bwd_head_workspace_bytes(L) bytes. Without NCONV_BWD_DEFER_REDUCE head_gw / head_gbias
     * are written in this call; with it head_nparts receives the partial-row count for
     * nconv_wgrad_reduce (layer head, workspace head_workspace). gxa / gca (nconv1's output
     * gradient) are then optional. */
    const nconv_layer* head;
    void* head_workspace;
    size_t head_workspace_bytes;
    float* head_gw;
    float* head_gbias;
    int head_nparts;                /* out */
    /* optional: the backward of the 1x1 layer that consumes L's outputs, fused into L's (DNET
     * training: nconv7, 8 -> 1, 1x1, padding 2, after nconv6). tail = nconv7's descriptor; tail_y,
     * tail_cout, tail_gy its outputs and their gradient, (B, 1, Ho + 4, Wo + 4); its cout gradient
     * is taken as 0 (DNET discards nconv7's confidence). L's gy / gcout are then formed in-kernel
     * from them (gy, gcout above are ignored and may be NULL), so nconv7's input gradient never
     * reaches HBM; nconv7's weight gradient goes to tail_gw (tail_workspace of
     * nconv_bwd_tail_workspace_bytes(L) bytes; with NCONV_BWD_DEFER_REDUCE tail_nparts partial rows
     * for nconv_wgrad_reduce, layer tail). nconv7's bias gradient (the sum of tail_gy) is left to
     * the caller (it is computed by the call that requests L's gw / gbias: a call with only the
     * input gradients computes none of nconv7's; tail_gw without gw / gbias is -EINVAL). L must
     * be nconv6's exact-fp32 geometry (16 -> 8 3x3, padding 0, upsample-first exactly-2x concat). */
    const nconv_layer* tail;
    const float* tail_y;
    const float* tail_cout;
    const float* tail_gy;
    void* tail_workspace;
    size_t tail_workspace_bytes;
    float* tail_gw;
    int tail_nparts;                /* out */
    /* ABI 20. optional: the box weights of an exactly-2x UPCAT layer's phase-form input gradient
     * (nconv_train_prologue wboxes), else built by a launch of this call. */
    const float* box_weights;
    /* ABI 20. The tail planes' extent: all zero = nconv7's whole (Ho + 4) x (Wo + 4) grid;
     * otherwise (B, 1, tail_h, tail_w) holding the grid from row / column tail_crop0 (DNET's crop,
     * step1.py:94: the training output written cropped by nconv_fwd_tail); gradient outside the
     * window is 0. */
    int tail_crop0;
    int tail_h;
    int tail_w;
} nconv_bwd_io;

int nconv_bwd_ex(const nconv_layer* L, nconv_bwd_io* io, void* workspace, size_t workspace_bytes,
                 unsigned flags, void* stream);
size_t nconv_bwd_head_workspace_bytes(const nconv_layer* L);
size_t nconv_bwd_tail_workspace_bytes(const nconv_layer* L);

/* Weight / bias gradients of n (1..16) layers whose nconv_bwd ran with NCONV_BWD_DEFER_REDUCE:
 * layers[k] the descriptor of that call (its weight normaliser wsum is read), workspaces[k] and
 * nparts[k] its workspace and return value, gw[k] / gbias[k] the outputs (either may be NULL;
 * layers with nparts[k] == 0 are skipped). Two launches on `stream`. Returns 0 or -EINVAL. */
int nconv_wgrad_reduce(int n, const nconv_layer* layers, void* const* workspaces, const int* nparts,
                       float* const* gw, float* const* gbias, void* stream);

/* nconv_wgrad_reduce plus nsum plain sums in the same two launches (n + nsum in 1..16): sum_out[k]
 * = the sum of sum_x[k][0 .. sum_n[k]) in a fixed order (bitwise deterministic; DNET training:
 * nconv7's bias gradient, the sum of its output gradient, without two launches of its own).
 * sum_workspace: nconv_sum_workspace_bytes(nsum) bytes. n may be 0. Returns 0 or -EINVAL. */
int nconv_wgrad_reduce_ex(int n, const nconv_layer* layers, void* const* workspaces, const int* nparts,
                          float* const* gw, float* const* gbias, int nsum, const float* const* sum_x,
                          const long long* sum_n, float* const* sum_out, void* sum_workspace,
                          size_t sum_workspace_bytes, void* stream);
size_t nconv_sum_workspace_bytes(int nsum);

/* ------------------------------------------------------------------------------------------
 * Dense convolutions of the RGB-guided model on the matrix cores (fp32 MFMA, exact f32 products).
 * Replace the nn.Conv2d / nn.ConvTranspose2d (+ eval BatchNorm + ReLU + residual add + torch.cat)
 * sequences of models/step2.py: RGBEncoder (:134-154), ConvBlock (:290-297), Basic2d (:178-195),
 * Basic2dTrans (:197-214), UpCat / NewFusionBlock cat (:173-175, :229-231), Conv3x3 heads (:156-158,
 * :259, :278). Inference (eval) semantics: BatchNorm uses its running statistics, folded into
 * the packed weights (scale) and the bias.
 * ------------------------------------------------------------------------------------------ */
enum nconv_dense_kind {
    NCONV_DENSE_3X3 = 0,            /* Conv2d 3x3, padding 1, stride 1 or 2                      */
    NCONV_DENSE_1X1 = 1,            /* Conv2d 1x1, padding 0, stride 1 or 2                      */
    NCONV_DENSE_TRANSPOSED_4X4 = 2, /* ConvTranspose2d 4x4, stride 2, padding 1 (Ho = 2H, or the
                                       cropped 2H - 1)                                           */
    NCONV_DENSE_CONV4X4_S2 = 3      /* Conv2d 4x4, stride 2, padding 1, Ho = (H - 1) / 2 + 1: the
                                       input gradient of the transposed convolution              */
};

typedef struct nconv_dense_conv {
    int B;
    const float* x0; int C0;   /* input = cat(x0, x1) along channels: x0 (B, C0, H, W)          */
    const float* x1; int C1;   /* x1 (B, C1, H, W), or NULL / 0                                   */
    int H, W;
    int Cout, Ho, Wo;          /* any Cout >= 1 (tiled by 32 or 64 output channels)               */
    int kind, stride;
    const float* wpack;        /* nconv_dense_pack output                                         */
    const float* bias;         /* (Cout) or NULL                                                   */
    int relu;                  /* 1: max(., 0) after the bias                                      */
    const float* wshort;       /* optional packed 1x1 shortcut (same stride) added after the ReLU  */
    float* out;                /* output channels [out_c0, out_c0 + Cout) of (B, out_C, Ho, Wo)    */
    int out_C, out_c0;
    int math;                  /* enum nconv_dense_math (ABI 22; 0 = fp32 MFMA)                     */
} nconv_dense_conv;

/* Arithmetic of every kind but the 1x1 (3x3 stride 1 or 2 with or without the 1x1 shortcut, the
 * transposed 4x4, the 4x4 stride 2: the RGB encoder, the fusion decoder and their input
 * gradients); the 1x1 always runs NCONV_DENSE_MATH_FP32.
 * Both split forms sum in fp32 on the matrix cores in another order than the fp32-MFMA kernel (an
 * fmaf chain), so results agree with it to fp32 accumulation error, not bitwise. */
enum nconv_dense_math {
    NCONV_DENSE_MATH_FP32 = 0,  /* v_mfma_f32_32x32x2_f32: exact f32 products                      */
    NCONV_DENSE_MATH_BF16X9 = 2,/* exact products on the bf16 matrix cores: both operands split into
                                   three bf16 parts (an exact decomposition), all nine partial
                                   products (each exact in fp32) accumulated in fp32              */
    NCONV_DENSE_MATH_BF16X6 = 3 /* the six largest of those nine terms: each product within
                                   ~2^-23 relative (the dropped v1*w2 + v2*w1 + v2*w2)             */
};

/* Floats of a packed weight buffer for (kind, Cin, Cout) (the fp32 image, then the pre-split bf16
 * image of the split-bf16 maths, ABI 22). */
size_t nconv_dense_packed_floats(int kind, int Cin, int Cout);

/* Pack w — Conv2d (Cout, Cin, k, k) or ConvTranspose2d (Cin, Cout, 4, 4) — into the kernel's
 * layout, multiplying output channel o by scale[o] if scale != NULL (eval BatchNorm folding).
 * The layout depends on (kind, Cin, Cout) only: a pack is valid for every call with those. */
int nconv_dense_pack(int kind, int Cin, int Cout, const float* w, const float* scale, float* wpack,
                     void* stream);

/* out[:, out_c0:out_c0+Cout] = [relu](conv(cat(x0, x1)) + bias) [+ conv1x1_shortcut(cat(x0, x1))] */
int nconv_dense_conv_fwd(const nconv_dense_conv* c, void* stream);

/* 3x3 (padding 1, stride 1) convolution to one output channel plus a residual:
 * out = conv3x3(x; w (1, Cin, 3, 3)) + res, all (B, ., H, W); res may be NULL
 * (the depth heads `depth + Conv3x3(fout)`, models/step2.py:259,278). */
int nconv_conv3x3_c1(const float* x, int B, int Cin, int H, int W, const float* w, const float* res,
                     float* out, void* stream);

/* Bilinear resampling with align_corners=True of (B, C, H, W) planes to (B, C, Ho, Wo): the guided
 * model's depth downsampling F.interpolate(depth, scale_factor=1/k, mode="bilinear",
 * align_corners=True) (models/step2.py:249,277), with the sampling arithmetic of the reference's
 * CPU kernel: scale = fp32(H-1) / (Ho-1), source coordinate fp32(scale * o), truncated index,
 * fp32 lambdas, blend fma(l0h, fma(l0w, a00, l1w*a01), l1h*fma(l0w, a10, l1w*a11)). x and y must
 * not overlap. */
int nconv_bilinear_ac(const float* x, int B, int C, int H, int W, float* y, int Ho, int Wo, void* stream);

/* ------------------------------------------------------------------------------------------
 * Training of the guided model: the weight gradient of a dense convolution.
 * Replaces the autograd of nn.Conv2d / nn.ConvTranspose2d (convolution_backward, weight part) for
 * the layers of models/step2.py listed above. The input gradient of a convolution is another
 * convolution of dL/dy and runs on nconv_dense_conv_fwd with re-arranged weights (3x3 / 1x1
 * stride 1: transposed, flipped; stride 2: NCONV_DENSE_TRANSPOSED_4X4 with the 3x3 / 1x1 kernel
 * embedded, output cropped to H x W; transposed 4x4: NCONV_DENSE_CONV4X4_S2, same weights).
 * The bias gradient is the sum of dL/dy over images and pixels.
 * ------------------------------------------------------------------------------------------ */
typedef struct nconv_dense_wgrad {
    int B;
    int kind, stride;          /* the forward convolution: NCONV_DENSE_3X3 / _1X1 (stride 1|2),
                                  NCONV_DENSE_TRANSPOSED_4X4 (stride 2)                           */
    const float* x0; int C0;   /* forward input = cat(x0, x1) along channels, (B, C0 + C1, H, W)  */
    const float* x1; int C1;   /* NULL / 0 for one source                                         */
    int H, W;
    const float* gy;           /* dL/dy, (B, Cout, Ho, Wo)                                        */
    int Cout, Ho, Wo;
    float* gw;                 /* OVERWRITTEN: Conv2d (Cout, Cin, k, k) / ConvTranspose2d
                                  (Cin, Cout, 4, 4). Limits: Cout <= 96 (conv), Cin <= 96
                                  (transposed), Cin <= 64 (1x1)                                   */
    int math;                  /* enum nconv_dense_math (ABI 22): the split-bf16 maths run the 3x3
                                  gradient (stride 1 or 2, >= 4 input channels) on the bf16 matrix
                                  cores; every other shape the fp32 MFMA kernel                   */
} nconv_dense_wgrad;

/* Workspace of nconv_dense_conv_wgrad in bytes (0 if the descriptor is invalid). */
size_t nconv_dense_wgrad_workspace_bytes(const nconv_dense_wgrad* g);

/* gw = dL/dW: deterministic (fixed-order reduction of per-workgroup partial sums). */
int nconv_dense_conv_wgrad(const nconv_dense_wgrad* g, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Training-mode BatchNorm2d + optional ReLU: batch statistics, running statistics updated in
 * place (momentum, unbiased running variance) — the nn.BatchNorm2d(train) -> nn.ReLU pairs of
 * models/step2.py:139-143 (RGBEncoder), :189-191 (Basic2d), :207-213 (Basic2dTrans) — and its
 * backward (the ReLU mask recomputed from x). Deterministic (fixed-order reductions).
 * ------------------------------------------------------------------------------------------ */
typedef struct nconv_bn_train {
    int B, C, H, W;
    const float* x;            /* (B, C, H, W) input                                              */
    const float* gamma;        /* (C) or NULL (= 1)                                               */
    const float* beta;         /* (C) or NULL (= 0)                                               */
    float* running_mean;       /* (C) updated by the forward, or NULL                             */
    float* running_var;        /* (C) updated by the forward (unbiased variance), or NULL         */
    float momentum, eps;
    int relu;                  /* 1: y = max(BN(x), 0)                                            */
    float* y;                  /* (B, C, H, W) forward output                                     */
    float* mean;               /* (C) batch mean: written by the forward, read by the backward    */
    float* invstd;             /* (C) 1/sqrt(biased batch variance + eps): likewise               */
} nconv_bn_train;

/* Workspace of nconv_bn_train_fwd / _bwd in bytes (0 if the descriptor is invalid). */
size_t nconv_bn_workspace_bytes(const nconv_bn_train* p);

int nconv_bn_train_fwd(const nconv_bn_train* p, void* workspace, size_t workspace_bytes, void* stream);

/* gx = dL/dx (NULL: skip), ggamma / gbeta = dL/dgamma, dL/dbeta (OVERWRITTEN; NULL: skip),
 * from gy = dL/dy and the forward's x, mean, invstd. */
int nconv_bn_train_bwd(const nconv_bn_train* p, const float* gy, float* gx, float* ggamma, float* gbeta,
                       void* workspace, size_t workspace_bytes, void* stream);

/* Backward of the ReLU after a biased convolution and its bias gradient (ConvBlock, step2.py:
 * 290-297, bias + ReLU fused in nconv_dense_conv_fwd): g_masked = g * (out > 0) (out = the
 * forward's ReLU output; out == NULL: no ReLU, g_masked unused), gbias[c] = sum over images and
 * pixels of the masked gradient (NULL: skip). All (B, C, H, W) except gbias (C). */
size_t nconv_relu_bias_bwd_workspace_bytes(int B, int C, int H, int W);
int nconv_relu_bias_bwd(int B, int C, int H, int W, const float* g, const float* out, float* g_masked,
                        float* gbias, void* workspace, size_t workspace_bytes, void* stream);

/* Training loss of the reference (utils.py:95-151 calculate_loss) on B (H, W) planes: the training
 * loop calls it on the whole (B, 1, H, W) batch (train_step1.py:63), the validation loop on element
 * [0] (utils.py:36; B = 1). rec = r masked to 0 where t == 0; use_gradient_loss != 0:
 * L = 0.8 sqrt(mean (rec - t)^2) + 0.2 (mean |Sobel_x(t - rec)| + mean |Sobel_y(t - rec)|), else
 * L = mean (rec - t)^2; means over B*H*W, each image's Sobel response zero-padded on its own
 * (F.conv2d, padding 1). r and t are fp32 with image / row strides in elements (r may be a cropped
 * view). nconv_depth_loss_fwd writes L to loss[0] (device) and keeps the backward's coefficients in
 * the workspace, which nconv_depth_loss_bwd reads: g (contiguous B x H x W, OVERWRITTEN) =
 * gloss[0] * dL/dr (gloss NULL: 1). Deterministic (fixed-order reductions). */
size_t nconv_depth_loss_workspace_bytes(int B, int H, int W);
int nconv_depth_loss_fwd(const float* r, long long r_image_stride, long long r_row_stride, const float* t,
                         long long t_image_stride, long long t_row_stride, int B, int H, int W, int use_gradient_loss,
                         float* loss, void* workspace, size_t workspace_bytes, void* stream);
int nconv_depth_loss_bwd(const float* r, long long r_image_stride, long long r_row_stride, const float* t,
                         long long t_image_stride, long long t_row_stride, int B, int H, int W, int use_gradient_loss,
                         const float* gloss, const void* workspace, size_t workspace_bytes, float* g, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NCONV_H */
