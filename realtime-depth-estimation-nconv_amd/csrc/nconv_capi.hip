// nconv_capi.hip — the extern "C" boundary of libnconv.so (declared in include/nconv.h).
// Validates every descriptor on the host before anything is enqueued, so a malformed call
// returns -EINVAL instead of launching a kernel with out-of-range indexing.
#include <stdio.h>
#include <string>
#include "nconv_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fn, const char* why) {
    g_err = std::string(fn) + ": " + (why ? why : "error");
    return code;
}

const char* validate(const nconv_layer* L, bool need_c) {
    if (!L) return "null layer descriptor";
    if (L->B <= 0 || L->Cin <= 0 || L->Cout <= 0 || L->H <= 0 || L->W <= 0) return "non-positive B/Cin/Cout/H/W";
    if (L->KH <= 0 || L->KW <= 0 || L->SH <= 0 || L->SW <= 0 || L->DH <= 0 || L->DW <= 0) return "non-positive kernel/stride/dilation";
    if (L->PH < 0 || L->PW < 0) return "negative padding";
    if (L->groups <= 0 || L->Cin % L->groups || L->Cout % L->groups) return "groups must divide Cin and Cout";
    const int ho = (L->H + 2 * L->PH - L->DH * (L->KH - 1) - 1) / L->SH + 1;
    const int wo = (L->W + 2 * L->PW - L->DW * (L->KW - 1) - 1) / L->SW + 1;
    if (ho <= 0 || wo <= 0) return "empty output";
    if (ho != L->Ho || wo != L->Wo) return "Ho/Wo inconsistent with H/W/kernel/stride/padding/dilation";
    if (!L->weight || !L->bias || !L->wsum) return "null weight/bias/wsum";
    if (!L->a.x) return "null source a.x";
    if (L->bwd_math != NCONV_MATH_FP32 && L->bwd_math != NCONV_MATH_BF16X3 && L->bwd_math != NCONV_MATH_BF16X9)
        return "unknown bwd_math (enum nconv_math)";
    if (L->math != NCONV_MATH_FP32 && L->math != NCONV_MATH_BF16X3 && L->math != NCONV_MATH_BF16X9)
        return "unknown math (enum nconv_math)";
    switch (L->load_mode) {
        case NCONV_LOAD_PLAIN:
            if (!L->a.c && need_c) return "null source a.c";
            if (L->a.C != L->Cin || L->a.H != L->H || L->a.W != L->W) return "PLAIN: source a must be (Cin, H, W)";
            break;
        case NCONV_LOAD_THRESH:
            if (L->a.C != L->Cin || L->a.H != L->H || L->a.W != L->W) return "THRESH: source a must be (Cin, H, W)";
            break;
        case NCONV_LOAD_POOL2:
            if (!L->a.c && need_c) return "null source a.c";
            if (L->a.C != L->Cin || L->a.H / 2 != L->H || L->a.W / 2 != L->W) return "POOL2: source a must be (Cin, 2H(+1), 2W(+1))";
            break;
        case NCONV_LOAD_UPCAT_SKIP_FIRST:
        case NCONV_LOAD_UPCAT_UP_FIRST:
            if (!L->a.c || !L->b.x || !L->b.c) return "UPCAT: null source pointer";
            if (L->a.C <= 0 || L->b.C <= 0 || L->a.C + L->b.C != L->Cin) return "UPCAT: a.C + b.C must equal Cin";
            if (L->a.H != L->H || L->a.W != L->W) return "UPCAT: source a must be (Ca, H, W)";
            if (L->b.H <= 0 || L->b.W <= 0) return "UPCAT: empty source b";
            break;
        default:
            return "unknown load mode";
    }
    return nullptr;
}

const char* validate_wgrad(const nconv_dense_wgrad* g) {
    if (!g) return "null descriptor";
    if (g->B <= 0 || g->C0 <= 0 || g->C1 < 0 || g->H <= 0 || g->W <= 0 || g->Cout <= 0)
        return "non-positive B/C0/H/W/Cout";
    if (!g->x0 || (g->C1 > 0 && !g->x1) || !g->gy || !g->gw) return "null pointer";
    if (g->math != NCONV_DENSE_MATH_FP32 && g->math != NCONV_DENSE_MATH_BF16X9 && g->math != NCONV_DENSE_MATH_BF16X6)
        return "unknown math";
    const int cin = g->C0 + g->C1;
    switch (g->kind) {
        case NCONV_DENSE_3X3:
        case NCONV_DENSE_1X1:
            if (g->stride != 1 && g->stride != 2) return "stride must be 1 or 2";
            if (g->Ho != (g->H - 1) / g->stride + 1 || g->Wo != (g->W - 1) / g->stride + 1)
                return "Ho/Wo inconsistent with kind/stride/H/W";
            if (g->Cout > 96) return "weight gradient supports at most 96 output channels";
            if (g->kind == NCONV_DENSE_1X1 && cin > 64) return "1x1 weight gradient supports at most 64 input channels";
            break;
        case NCONV_DENSE_TRANSPOSED_4X4:
            if (g->stride != 2) return "transposed 4x4 has stride 2";
            if ((g->Ho != 2 * g->H && g->Ho != 2 * g->H - 1) || (g->Wo != 2 * g->W && g->Wo != 2 * g->W - 1))
                return "Ho/Wo inconsistent with kind/stride/H/W";
            if (cin > 96) return "transposed weight gradient supports at most 96 input channels";
            break;
        default:
            return "unknown kind (weight gradients: 3x3, 1x1, transposed 4x4)";
    }
    return nullptr;
}

const char* validate_bn(const nconv_bn_train* p) {
    if (!p) return "null descriptor";
    if (p->B <= 0 || p->C <= 0 || p->H <= 0 || p->W <= 0) return "non-positive B/C/H/W";
    if ((long long)p->H * p->W > (1LL << 30)) return "plane too large";
    if (!p->x || !p->mean || !p->invstd) return "null x / mean / invstd";
    if (!(p->eps > 0.f) || p->momentum < 0.f || p->momentum > 1.f) return "eps must be > 0 and momentum in [0, 1]";
    return nullptr;
}

LayerDev make_dev(const nconv_layer* L) {
    LayerDev d;
    d.L = *L;
    d.up_scale_h = (L->b.H > 0) ? (float)L->b.H / (float)L->H : 0.f;
    d.up_scale_w = (L->b.W > 0) ? (float)L->b.W / (float)L->W : 0.f;
    return d;
}

}  // namespace

extern "C" {

int nconv_abi_version(void) { return NCONV_ABI_VERSION; }

const char* nconv_last_error(void) { return g_err.c_str(); }

int nconv_weight_prep(int n, float* const* weights, const int* couts, const int* fan_ins,
                      const int* apply_softplus, float* const* wsums, void* stream) {
    if (n < 0 || (n > 0 && (!weights || !couts || !fan_ins || !wsums)))
        return fail(-22, "nconv_weight_prep", "null argument");
    for (int i = 0; i < n; ++i)
        if (!weights[i] || !wsums[i] || couts[i] <= 0 || fan_ins[i] <= 0)
            return fail(-22, "nconv_weight_prep", "bad layer entry");
    const char* why = nullptr;
    int rc = nconv::launch_weight_prep(n, weights, couts, fan_ins, apply_softplus, wsums,
                                       (hipStream_t)stream, &why);
    return rc ? fail(rc, "nconv_weight_prep", why) : 0;
}

int nconv_fwd(const nconv_layer* L, float* y, float* cout, void* stream) {
    if (const char* why = validate(L, true)) return fail(-22, "nconv_fwd", why);
    if (!y || !cout) return fail(-22, "nconv_fwd", "null output");
    const char* why = nullptr;
    int rc = nconv::launch_fwd(make_dev(L), y, cout, nullptr, nullptr, nullptr, (hipStream_t)stream, &why);
    return rc ? fail(rc, "nconv_fwd", why) : 0;
}

int nconv_fwd_pooled(const nconv_layer* L, float* y, float* cout, float* y_pool, float* cout_pool,
                     unsigned int* argmax, void* stream) {
    if (const char* why = validate(L, true)) return fail(-22, "nconv_fwd_pooled", why);
    if (!y || !cout || !y_pool || !cout_pool) return fail(-22, "nconv_fwd_pooled", "null output");
    if (L->Ho < 2 || L->Wo < 2) return fail(-22, "nconv_fwd_pooled", "output too small to pool");
    const char* why = nullptr;
    int rc = nconv::launch_fwd(make_dev(L), y, cout, y_pool, cout_pool, argmax, (hipStream_t)stream, &why);
    return rc ? fail(rc, "nconv_fwd_pooled", why) : 0;
}

int nconv_fwd_head(const nconv_layer* L1, const nconv_layer* L2, float* y, float* cout, float* y_pool,
                   float* cout_pool, unsigned int* argmax, float* y1, float* cout1, void* stream) {
    const char* fn = "nconv_fwd_head";
    if (const char* why = validate(L1, false)) return fail(-22, fn, why);
    if (!L2) return fail(-22, fn, "null nconv2 descriptor");
    if (!y || !cout || !y_pool || !cout_pool) return fail(-22, fn, "null output");
    if (L1->load_mode != NCONV_LOAD_THRESH || L1->Cin != 1 || L1->Cout != 8 || L1->KH != 5 || L1->KW != 5 ||
        L1->PH != 2 || L1->PW != 2 || L1->SH != 1 || L1->SW != 1 || L1->DH != 1 || L1->DW != 1 || L1->groups != 1)
        return fail(-95, fn, "nconv1 must be 1 -> 8, 5x5, padding 2, stride 1, thresholded input");
    if (L2->B != L1->B || L2->Cin != 8 || L2->Cout != 8 || L2->KH != 5 || L2->KW != 5 || L2->PH != 2 ||
        L2->PW != 2 || L2->SH != 1 || L2->SW != 1 || L2->DH != 1 || L2->DW != 1 || L2->groups != 1)
        return fail(-95, fn, "nconv2 must be 8 -> 8, 5x5, padding 2, stride 1");
    if (L2->H != L1->Ho || L2->W != L1->Wo || L2->Ho != L2->H || L2->Wo != L2->W)
        return fail(-22, fn, "nconv2 geometry inconsistent with nconv1's output");
    if (L2->Ho < 2 || L2->Wo < 2) return fail(-22, fn, "output too small to pool");
    if (!L2->weight || !L2->bias || !L2->wsum) return fail(-22, fn, "null nconv2 weight/bias/wsum");
    const bool exact = L2->math == NCONV_MATH_FP32;
    if (exact && !L2->waux) return fail(-22, fn, "exact-fp32 head needs nconv2's waux = nconv_head_weights output");
    if ((argmax || y1 || cout1) && !(exact && argmax && y1 && cout1))
        return fail(-95, fn, "the training outputs (argmax, y1, cout1: all three) need the exact-fp32 head");
    nconv_layer l2 = *L2;
    l2.load_mode = NCONV_LOAD_PLAIN;
    l2.a = L1->a;  // (the kernel reads the sparse depth through TailArgs)
    nconv::TailArgs t{};
    t.py = y_pool;
    t.pc = cout_pool;
    t.s_in = L1->a.x;
    t.w1 = L1->weight;
    t.b1 = L1->bias;
    t.s1 = L1->wsum;
    t.eps1 = L1->eps;
    t.thresh1 = L1->thresh;
    t.parg = argmax;
    t.y1 = y1;
    t.c1 = cout1;
    const char* why = nullptr;
    int rc = exact ? nconv::launch_fwd_head_exact(make_dev(&l2), t, y, cout, (hipStream_t)stream, &why)
                   : nconv::launch_fwd_head(make_dev(&l2), t, y, cout, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_head_weights(const nconv_layer* L1, const nconv_layer* L2, float* w21, void* stream) {
    const char* fn = "nconv_head_weights";
    if (!L1 || !L2 || !w21) return fail(-22, fn, "null argument");
    if (!L1->weight || !L1->wsum || !L2->weight) return fail(-22, fn, "null weight / wsum");
    if (L1->Cin != 1 || L1->Cout != 8 || L1->KH != 5 || L1->KW != 5 || L2->Cin != 8 || L2->Cout != 8 ||
        L2->KH != 5 || L2->KW != 5 || L1->groups != 1 || L2->groups != 1)
        return fail(-95, fn, "nconv1 must be 1 -> 8 and nconv2 8 -> 8, both 5x5");
    const char* why = nullptr;
    int rc = nconv::launch_head_weights(L1->weight, L1->wsum, L2->weight, w21, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_fwd_tail(const nconv_layer* L6, const float* w7, const float* b7, const float* wsum7,
                   int cin7, int p7, float eps7, float* out, float* out_c, int out_h, int out_w, int crop0,
                   float* y6, float* cout6, void* stream) {
    if (const char* why = validate(L6, true)) return fail(-22, "nconv_fwd_tail", why);
    if (!w7 || !b7 || !wsum7 || !out) return fail(-22, "nconv_fwd_tail", "null tail pointer");
    if (cin7 != L6->Cout) return fail(-22, "nconv_fwd_tail", "nconv7 Cin must equal nconv6 Cout");
    if (p7 < 0 || out_h < 0 || out_w < 0 || crop0 < 0) return fail(-22, "nconv_fwd_tail", "bad tail geometry");
    if (crop0 + out_h > L6->Ho + 2 * p7 || crop0 + out_w > L6->Wo + 2 * p7)
        return fail(-22, "nconv_fwd_tail", "output crop exceeds nconv7's grid");
    if ((y6 == nullptr) != (cout6 == nullptr)) return fail(-22, "nconv_fwd_tail", "y6 and cout6: both or neither");
    // nconv6's outputs are written only where the output window reaches them: with y6 the window
    // must cover every nconv6 pixel (rows / columns crop0 - p7 .. crop0 - p7 + out - 1 of nconv6)
    if (y6 && (crop0 > p7 || crop0 + out_h - p7 < L6->Ho || crop0 + out_w - p7 < L6->Wo))
        return fail(-22, "nconv_fwd_tail", "y6 / cout6 need an output window covering every nconv6 pixel");
    nconv::TailArgs t{w7, b7, wsum7, eps7, crop0 - p7, out_h, out_w, out_c};
    t.y6 = y6;
    t.c6 = cout6;
    const char* why = nullptr;
    int rc = nconv::launch_fwd_tail(make_dev(L6), t, out, (hipStream_t)stream, &why);
    return rc ? fail(rc, "nconv_fwd_tail", why) : 0;
}

int nconv_plan(const nconv_layer* L, int* fwd_kernel, int* dgrad_kernel, int* wgrad_kernel) {
    if (const char* why = validate(L, false)) return fail(-22, "nconv_plan", why);
    int dg, wg;
    nconv::plan_bwd(*L, &dg, &wg);
    if (fwd_kernel) *fwd_kernel = nconv::plan_fwd(*L);
    if (dgrad_kernel) *dgrad_kernel = dg;
    if (wgrad_kernel) *wgrad_kernel = wg;
    return 0;
}

size_t nconv_phase_weights_floats(const nconv_layer* L) {
    if (validate(L, false)) return 0;
    return nconv::phase_weight_floats(*L);
}

int nconv_phase_weights(int n, const float* const* weights, const int* cins, const int* up_first,
                        float* const* wphases, void* stream) {
    const char* fn = "nconv_phase_weights";
    if (n < 0 || (n > 0 && (!weights || !cins || !up_first || !wphases))) return fail(-22, fn, "null argument");
    for (int i = 0; i < n; ++i) {
        if (!weights[i] || !wphases[i]) return fail(-22, fn, "null weight / output");
        if (up_first[i] < 0 || up_first[i] + 8 > cins[i]) return fail(-22, fn, "upsampled channels outside [0, Cin)");
    }
    const char* why = nullptr;
    int rc = nconv::launch_phase_weights(n, weights, cins, up_first, wphases, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_train_prologue(int n, float* const* weights, const int* couts, const int* fan_ins, const int* softplus,
                         float* const* wsums, int head1, int head2, float* w21, unsigned int* sync, int nphase,
                         const int* phase_layers, const int* phase_up_first, float* const* wphases,
                         float* const* wboxes, void* stream) {
    const char* fn = "nconv_train_prologue";
    if (n < 0 || nphase < 0) return fail(-22, fn, "negative count");
    if (n > 0 && (!weights || !couts || !fan_ins || !wsums)) return fail(-22, fn, "null argument");
    for (int i = 0; i < n; ++i)
        if (!weights[i] || !wsums[i] || couts[i] <= 0 || fan_ins[i] <= 0) return fail(-22, fn, "bad layer entry");
    if (w21) {
        if (head1 < 0 || head1 >= n || head2 < 0 || head2 >= n || head1 == head2)
            return fail(-22, fn, "head layers must be two distinct layer indices");
        if (couts[head1] != 8 || fan_ins[head1] != 25 || couts[head2] != 8 || fan_ins[head2] != 200)
            return fail(-22, fn, "head layers must be nconv1 (8 x 1 x 5 x 5) and nconv2 (8 x 8 x 5 x 5)");
        if (!sync) return fail(-22, fn, "head weights need the sync counter");
    }
    if (nphase > 0 && (!phase_layers || !phase_up_first || !wphases)) return fail(-22, fn, "null phase argument");
    for (int k = 0; k < nphase; ++k) {
        const int i = phase_layers[k];
        if (i < 0 || i >= n || !wphases[k]) return fail(-22, fn, "bad phase entry");
        if (couts[i] != 8 || fan_ins[i] != 144) return fail(-22, fn, "phase layers must be 8 x 16 x 3 x 3");
        if (phase_up_first[k] != 0 && phase_up_first[k] != 8) return fail(-22, fn, "up_first must be 0 or 8");
        if (w21 && (i == head1 || i == head2)) return fail(-22, fn, "a layer is both a head and a phase layer");
        for (int j = 0; j < k; ++j)
            if (phase_layers[j] == i) return fail(-22, fn, "a phase layer is listed twice");
    }
    const char* why = nullptr;
    int rc = nconv::launch_train_prologue(n, weights, couts, fan_ins, softplus, wsums, head1, head2, w21, sync,
                                          nphase, phase_layers, phase_up_first, wphases, wboxes, (hipStream_t)stream,
                                          &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_weight_prologue(int n, float* const* weights, const int* couts, const int* fan_ins,
                          float* const* wsums, const float* head_w1, const float* head_w2, float* w21,
                          int nphase, const float* const* phase_weights, const int* phase_cins,
                          const int* phase_up_first, float* const* wphases, void* stream) {
    const char* fn = "nconv_weight_prologue";
    if (n < 0 || nphase < 0) return fail(-22, fn, "negative count");
    if (n > 0 && (!weights || !couts || !fan_ins || !wsums)) return fail(-22, fn, "null argument");
    for (int i = 0; i < n; ++i)
        if (!weights[i] || !wsums[i] || couts[i] <= 0 || fan_ins[i] <= 0) return fail(-22, fn, "bad layer entry");
    if (w21 && (!head_w1 || !head_w2)) return fail(-22, fn, "head weights need head_w1 and head_w2");
    if (nphase > 0 && (!phase_weights || !phase_cins || !phase_up_first || !wphases))
        return fail(-22, fn, "null phase argument");
    for (int i = 0; i < nphase; ++i) {
        if (!phase_weights[i] || !wphases[i]) return fail(-22, fn, "null phase weight / output");
        if (phase_up_first[i] < 0 || phase_up_first[i] + 8 > phase_cins[i])
            return fail(-22, fn, "upsampled channels outside [0, Cin)");
    }
    const char* why = nullptr;
    int rc = nconv::launch_weight_prologue(n, weights, couts, fan_ins, wsums, head_w1, head_w2, w21, nphase,
                                           phase_weights, phase_cins, phase_up_first, wphases,
                                           (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

size_t nconv_bwd_workspace_bytes(const nconv_layer* L) {
    if (validate(L, true)) return 0;
    return nconv::bwd_workspace_bytes(make_dev(L));
}

size_t nconv_bwd_head_workspace_bytes(const nconv_layer* L) {
    if (!L || validate(L, false)) return 0;
    return nconv::bwd_head_workspace_bytes(*L);
}

size_t nconv_bwd_tail_workspace_bytes(const nconv_layer* L) {
    if (!L || validate(L, false)) return 0;
    return nconv::bwd_tail_workspace_bytes(*L);
}

int nconv_bwd_ex(const nconv_layer* L, nconv_bwd_io* io, void* workspace, size_t workspace_bytes,
                 unsigned flags, void* stream) {
    if (const char* why = validate(L, true)) return fail(-22, "nconv_bwd", why);
    if (!io) return fail(-22, "nconv_bwd", "null io");
    if (!io->y || !io->cout || (!io->gy && !io->tail)) return fail(-22, "nconv_bwd", "null y/cout/gy");
    const LayerDev d = make_dev(L);
    const size_t need = nconv::bwd_workspace_bytes(d);
    if (need && (!workspace || workspace_bytes < need)) return fail(-22, "nconv_bwd", "workspace too small");
    const int fan = (L->Cin / L->groups) * L->KH * L->KW;
    if ((long)L->Cout * fan + 2L * L->Cout > 65535)
        return fail(-22, "nconv_bwd", "weight-gradient path supports at most 65535 weights per layer");
    int nparts = 0;
    const int defer = (flags & NCONV_BWD_DEFER_REDUCE) ? 1 : 0;
    nconv::BwdArgs a{io->y, io->cout, io->gy, io->gcout, io->gxa, io->gca, io->gxb, io->gcb, io->gw, io->gbias,
                     (float*)workspace, workspace_bytes, (flags & NCONV_BWD_ACCUMULATE) ? 1 : 0, defer, &nparts,
                     io->gy_pool, io->gcout_pool, io->pool_argmax};
    a.box = io->box_weights;
    io->head_nparts = 0;
    if (const nconv_layer* H = io->head) {
        if (const char* why = validate(H, true)) return fail(-22, "nconv_bwd", why);
        if (H->Cin != 1 || H->Cout != 8 || H->KH != 5 || H->KW != 5 || H->PH != 2 || H->PW != 2 || H->SH != 1 ||
            H->SW != 1 || H->DH != 1 || H->DW != 1 || H->groups != 1 || H->load_mode != NCONV_LOAD_THRESH)
            return fail(-22, "nconv_bwd", "head must be a 1->8 5x5 padding-2 threshold layer (nconv1)");
        if (H->B != L->B || H->Ho != L->H || H->Wo != L->W || L->Cin != 8)
            return fail(-22, "nconv_bwd", "head output does not match the layer's input");
        if ((flags & NCONV_BWD_ACCUMULATE) && (io->gxa || io->gca))
            return fail(-22, "nconv_bwd", "fused head: the head's output gradient is written, not accumulated");
        if (!io->head_workspace || io->head_workspace_bytes < nconv::bwd_head_workspace_bytes(*L))
            return fail(-22, "nconv_bwd", "head workspace too small (nconv_bwd_head_workspace_bytes)");
        if (!defer && !io->head_gw && !io->head_gbias) return fail(-22, "nconv_bwd", "head outputs are NULL");
        a.hS = H->a.x;
        a.hb = H->bias;
        a.hs = H->wsum;
        a.heps = H->eps;
        a.hthresh = H->thresh;
        a.hpart = (float*)io->head_workspace;
        a.hgw = io->head_gw;
        a.hgb = io->head_gbias;
        a.hnparts = &io->head_nparts;
    }
    io->tail_nparts = 0;
    if (const nconv_layer* T = io->tail) {
        if (const char* why = validate(T, true)) return fail(-22, "nconv_bwd", why);
        if (T->Cin != L->Cout || T->Cout != 1 || T->KH != 1 || T->KW != 1 || T->PH != 2 || T->PW != 2 ||
            T->SH != 1 || T->SW != 1 || T->DH != 1 || T->DW != 1 || T->groups != 1 ||
            T->load_mode != NCONV_LOAD_PLAIN || T->B != L->B || T->H != L->Ho || T->W != L->Wo)
            return fail(-22, "nconv_bwd", "tail must be a 1x1 padding-2 layer on this layer's outputs (nconv7)");
        if (!io->tail_y || !io->tail_cout || !io->tail_gy) return fail(-22, "nconv_bwd", "null tail planes");
        // nconv7's planes: its whole (Ho + 4) x (Wo + 4) grid (tail_h = 0), or a window of it
        if (io->tail_h == 0 && io->tail_w == 0 && io->tail_crop0 == 0) {
            a.t7ph = L->Ho + 4, a.t7pw = L->Wo + 4, a.t7pc0 = 0;
        } else {
            if (io->tail_h <= 0 || io->tail_w <= 0 || io->tail_crop0 < 0 || io->tail_crop0 + io->tail_h > L->Ho + 4 ||
                io->tail_crop0 + io->tail_w > L->Wo + 4)
                return fail(-22, "nconv_bwd", "tail window outside nconv7's grid");
            a.t7ph = io->tail_h, a.t7pw = io->tail_w, a.t7pc0 = io->tail_crop0;
        }
        if (!io->tail_workspace || io->tail_workspace_bytes < nconv::bwd_tail_workspace_bytes(*L))
            return fail(-22, "nconv_bwd", "tail workspace too small (nconv_bwd_tail_workspace_bytes)");
        if (!defer && !io->tail_gw && (io->gw || io->gbias)) return fail(-22, "nconv_bwd", "tail output is NULL");
        // nconv7's weight gradient is accumulated inside this layer's weight-gradient pass, which
        // runs only when gw or gbias is requested
        if (io->tail_gw && !io->gw && !io->gbias)
            return fail(-22, "nconv_bwd", "tail_gw needs this layer's weight-gradient pass (gw or gbias)");
        a.t7w = T->weight;
        a.t7b = T->bias;
        a.t7s = T->wsum;
        a.t7eps = T->eps;
        a.t7gy = io->tail_gy;
        a.t7y = io->tail_y;
        a.t7co = io->tail_cout;
        a.t7part = (float*)io->tail_workspace;
        a.t7gw = io->tail_gw;
        a.t7nparts = &io->tail_nparts;
    }
    const char* why = nullptr;
    int rc = nconv::launch_bwd(d, a, (hipStream_t)stream, &why);
    if (rc) return fail(rc, "nconv_bwd", why);
    return defer ? nparts : 0;
}

int nconv_bwd(const nconv_layer* L, const float* y, const float* cout, const float* gy,
              const float* gcout, float* gxa, float* gca, float* gxb, float* gcb, float* gw,
              float* gbias, void* workspace, size_t workspace_bytes, unsigned flags, void* stream) {
    nconv_bwd_io io{};
    io.y = y, io.cout = cout, io.gy = gy, io.gcout = gcout;
    io.gxa = gxa, io.gca = gca, io.gxb = gxb, io.gcb = gcb, io.gw = gw, io.gbias = gbias;
    return nconv_bwd_ex(L, &io, workspace, workspace_bytes, flags, stream);
}

int nconv_wgrad_reduce(int n, const nconv_layer* layers, void* const* workspaces, const int* nparts,
                       float* const* gw, float* const* gbias, void* stream) {
    return nconv_wgrad_reduce_ex(n, layers, workspaces, nparts, gw, gbias, 0, nullptr, nullptr, nullptr, nullptr, 0,
                                 stream);
}

size_t nconv_sum_workspace_bytes(int nsum) { return nsum > 0 ? (size_t)nsum * nconv::kSumChunks * sizeof(float) : 0; }

int nconv_wgrad_reduce_ex(int n, const nconv_layer* layers, void* const* workspaces, const int* nparts,
                          float* const* gw, float* const* gbias, int nsum, const float* const* sum_x,
                          const long long* sum_n, float* const* sum_out, void* sum_workspace,
                          size_t sum_workspace_bytes, void* stream) {
    const char* fn = "nconv_wgrad_reduce";
    if (n < 0 || nsum < 0 || n + nsum < 1 || n + nsum > nconv::kMaxRedJobs)
        return fail(-22, fn, "1..16 layers and sums together");
    if (n > 0 && (!layers || !workspaces || !nparts || !gw || !gbias)) return fail(-22, fn, "null array");
    if (nsum > 0 && (!sum_x || !sum_n || !sum_out)) return fail(-22, fn, "null sum array");
    if (nsum > 0 && (!sum_workspace || sum_workspace_bytes < nconv_sum_workspace_bytes(nsum)))
        return fail(-22, fn, "sum workspace too small (nconv_sum_workspace_bytes)");
    nconv::RedJob jobs[nconv::kMaxRedJobs];
    int m = 0;
    for (int k = 0; k < n; ++k) {
        if (nparts[k] < 0) return fail(-22, fn, "negative partial-row count");
        if (nparts[k] == 0 || (!gw[k] && !gbias[k])) continue;
        const nconv_layer* L = &layers[k];
        if (!workspaces[k] || !L->wsum) return fail(-22, fn, "null workspace / wsum");
        if (L->Cout <= 0 || L->Cin <= 0 || L->groups <= 0 || L->KH <= 0 || L->KW <= 0)
            return fail(-22, fn, "invalid layer geometry");
        const int fan = (L->Cin / L->groups) * L->KH * L->KW;
        jobs[m++] = nconv::RedJob{(const float*)workspaces[k], L->wsum, gw[k], gbias[k], nparts[k],
                                  L->Cout * fan, L->Cout, fan};
    }
    for (int k = 0; k < nsum; ++k) {
        if (!sum_out[k] || sum_n[k] < 0 || sum_n[k] > 0x7fffffffLL || (sum_n[k] > 0 && !sum_x[k]))
            return fail(-22, fn, "bad sum entry");
        float* sub = (float*)sum_workspace + (size_t)k * nconv::kSumChunks;
        jobs[m++] = nconv::RedJob{sum_x[k], nullptr, nullptr, sum_out[k], (int)sum_n[k], 0, 1, 0, 1, sub};
    }
    if (m == 0) return 0;
    const char* why = nullptr;
    const int rc = nconv::launch_wgrad_reduce_multi(m, jobs, (hipStream_t)stream, &why);
    if (rc) return fail(rc, fn, why);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(-5, fn, hipGetErrorString(e));
}

size_t nconv_dense_packed_floats(int kind, int Cin, int Cout) {
    if (kind < NCONV_DENSE_3X3 || kind > NCONV_DENSE_CONV4X4_S2 || Cin <= 0 || Cout <= 0) return 0;
    return nconv::dense_packed_floats(kind, Cin, Cout);
}

int nconv_dense_pack(int kind, int Cin, int Cout, const float* w, const float* scale, float* wpack, void* stream) {
    if (kind < NCONV_DENSE_3X3 || kind > NCONV_DENSE_CONV4X4_S2) return fail(-22, "nconv_dense_pack", "unknown kind");
    if (Cin <= 0 || Cout <= 0) return fail(-22, "nconv_dense_pack", "non-positive Cin/Cout");
    if (!w || !wpack) return fail(-22, "nconv_dense_pack", "null weight pointer");
    const char* why = nullptr;
    int rc = nconv::launch_dense_pack(kind, Cin, Cout, w, scale, wpack, (hipStream_t)stream, &why);
    return rc ? fail(rc, "nconv_dense_pack", why) : 0;
}

int nconv_dense_conv_fwd(const nconv_dense_conv* c, void* stream) {
    const char* fn = "nconv_dense_conv_fwd";
    if (!c) return fail(-22, fn, "null descriptor");
    if (c->B <= 0 || c->H <= 0 || c->W <= 0 || c->C0 <= 0 || c->C1 < 0) return fail(-22, fn, "non-positive B/H/W/C0");
    if (!c->x0 || (c->C1 > 0 && !c->x1)) return fail(-22, fn, "null input pointer");
    if (c->Cout <= 0) return fail(-22, fn, "non-positive Cout");
    if (!c->wpack || !c->out) return fail(-22, fn, "null weight / output pointer");
    if (c->out_c0 < 0 || c->out_c0 + c->Cout > c->out_C) return fail(-22, fn, "output channel range exceeds out_C");
    if (c->math != NCONV_DENSE_MATH_FP32 && c->math != NCONV_DENSE_MATH_BF16X9 && c->math != NCONV_DENSE_MATH_BF16X6)
        return fail(-22, fn, "unknown math");
    int ho, wo;
    switch (c->kind) {
        case NCONV_DENSE_3X3:
            if (c->stride != 1 && c->stride != 2) return fail(-22, fn, "3x3 stride must be 1 or 2");
            ho = (c->H - 1) / c->stride + 1;
            wo = (c->W - 1) / c->stride + 1;
            break;
        case NCONV_DENSE_1X1:
            if (c->stride != 1 && c->stride != 2) return fail(-22, fn, "1x1 stride must be 1 or 2");
            ho = (c->H - 1) / c->stride + 1;
            wo = (c->W - 1) / c->stride + 1;
            if (c->wshort) return fail(-22, fn, "shortcut only with a 3x3 main convolution");
            break;
        case NCONV_DENSE_TRANSPOSED_4X4:
            if (c->stride != 2) return fail(-22, fn, "transposed 4x4 has stride 2");
            if (c->wshort) return fail(-22, fn, "no shortcut for the transposed convolution");
            // 2H x 2W, or cropped by one row / column (the input gradient of a stride-2 conv of
            // an odd-sized input)
            ho = (c->Ho == 2 * c->H - 1) ? c->Ho : 2 * c->H;
            wo = (c->Wo == 2 * c->W - 1) ? c->Wo : 2 * c->W;
            break;
        case NCONV_DENSE_CONV4X4_S2:
            if (c->stride != 2) return fail(-22, fn, "conv 4x4 has stride 2");
            if (c->wshort) return fail(-22, fn, "shortcut only with a 3x3 main convolution");
            ho = (c->H - 1) / 2 + 1;
            wo = (c->W - 1) / 2 + 1;
            break;
        default:
            return fail(-22, fn, "unknown kind");
    }
    if (ho != c->Ho || wo != c->Wo) return fail(-22, fn, "Ho/Wo inconsistent with kind/stride/H/W");
    const char* why = nullptr;
    int rc = nconv::launch_dense_conv(*c, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

size_t nconv_dense_wgrad_workspace_bytes(const nconv_dense_wgrad* g) {
    if (validate_wgrad(g)) return 0;
    return nconv::dense_wgrad_workspace_bytes(*g);
}

int nconv_dense_conv_wgrad(const nconv_dense_wgrad* g, void* workspace, size_t workspace_bytes, void* stream) {
    const char* fn = "nconv_dense_conv_wgrad";
    if (const char* why = validate_wgrad(g)) return fail(-22, fn, why);
    const size_t need = nconv::dense_wgrad_workspace_bytes(*g);
    if (need && (!workspace || workspace_bytes < need)) return fail(-22, fn, "workspace too small");
    const char* why = nullptr;
    int rc = nconv::launch_dense_wgrad(*g, (float*)workspace, workspace_bytes, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

size_t nconv_bn_workspace_bytes(const nconv_bn_train* p) {
    if (validate_bn(p)) return 0;
    return nconv::bn_workspace_bytes(*p);
}

int nconv_bn_train_fwd(const nconv_bn_train* p, void* workspace, size_t workspace_bytes, void* stream) {
    const char* fn = "nconv_bn_train_fwd";
    if (const char* why = validate_bn(p)) return fail(-22, fn, why);
    if (!p->y) return fail(-22, fn, "null y");
    if (!workspace || workspace_bytes < nconv::bn_workspace_bytes(*p)) return fail(-22, fn, "workspace too small");
    const char* why = nullptr;
    int rc = nconv::launch_bn_train_fwd(*p, (float*)workspace, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_bn_train_bwd(const nconv_bn_train* p, const float* gy, float* gx, float* ggamma, float* gbeta,
                       void* workspace, size_t workspace_bytes, void* stream) {
    const char* fn = "nconv_bn_train_bwd";
    if (const char* why = validate_bn(p)) return fail(-22, fn, why);
    if (!gy) return fail(-22, fn, "null gy");
    if (!workspace || workspace_bytes < nconv::bn_workspace_bytes(*p)) return fail(-22, fn, "workspace too small");
    const char* why = nullptr;
    int rc = nconv::launch_bn_train_bwd(*p, gy, gx, ggamma, gbeta, (float*)workspace, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

size_t nconv_relu_bias_bwd_workspace_bytes(int B, int C, int H, int W) {
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
    return nconv::relu_bias_workspace_bytes(B, C, H, W);
}

int nconv_relu_bias_bwd(int B, int C, int H, int W, const float* g, const float* out, float* g_masked,
                        float* gbias, void* workspace, size_t workspace_bytes, void* stream) {
    const char* fn = "nconv_relu_bias_bwd";
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return fail(-22, fn, "non-positive B/C/H/W");
    if ((long long)H * W > (1LL << 30)) return fail(-22, fn, "plane too large");
    if (!g) return fail(-22, fn, "null g");
    if (!workspace || workspace_bytes < nconv::relu_bias_workspace_bytes(B, C, H, W))
        return fail(-22, fn, "workspace too small");
    const char* why = nullptr;
    int rc = nconv::launch_relu_bias_bwd(B, C, H, W, g, out, g_masked, gbias, (float*)workspace, (hipStream_t)stream,
                                         &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_conv3x3_c1(const float* x, int B, int Cin, int H, int W, const float* w, const float* res, float* out,
                     void* stream) {
    const char* fn = "nconv_conv3x3_c1";
    if (!x || !w || !out) return fail(-22, fn, "null pointer");
    if (B <= 0 || Cin <= 0 || H <= 0 || W <= 0) return fail(-22, fn, "non-positive B/Cin/H/W");
    const char* why = nullptr;
    int rc = nconv::launch_conv3x3_c1(x, B, Cin, H, W, w, res, out, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_bilinear_ac(const float* x, int B, int C, int H, int W, float* y, int Ho, int Wo, void* stream) {
    const char* fn = "nconv_bilinear_ac";
    if (!x || !y) return fail(-22, fn, "null pointer");
    if (B < 0 || C < 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return fail(-22, fn, "bad geometry");
    if ((long long)H * W >= (1LL << 31) || (long long)B * C * Ho * Wo >= (1LL << 40)) return fail(-22, fn, "too large");
    const char* why = nullptr;
    int rc = nconv::launch_bilinear_ac(x, B, C, H, W, y, Ho, Wo, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

size_t nconv_depth_loss_workspace_bytes(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0 || (long long)B * H * W > (1LL << 30)) return 0;
    return nconv::loss_workspace_bytes(B, H, W);
}

static const char* validate_loss(const nconv::LossArgs& a, size_t ws_bytes, const void* ws) {
    if (!a.r || !a.t) return "null plane";
    if (a.B <= 0 || a.H <= 0 || a.W <= 0) return "non-positive B/H/W";
    if ((long long)a.B * a.H * a.W > (1LL << 30)) return "batch too large";
    if (a.rs < a.W || a.ts < a.W) return "row stride smaller than W";
    if (a.B > 1 && (a.rbs < a.H * a.rs || a.tbs < a.H * a.ts)) return "image stride smaller than H * row stride";
    if (!ws || ws_bytes < nconv::loss_workspace_bytes(a.B, a.H, a.W)) return "workspace too small";
    return nullptr;
}

int nconv_depth_loss_fwd(const float* r, long long r_image_stride, long long r_row_stride, const float* t,
                         long long t_image_stride, long long t_row_stride, int B, int H, int W, int use_gradient_loss,
                         float* loss, void* workspace, size_t workspace_bytes, void* stream) {
    const char* fn = "nconv_depth_loss_fwd";
    const nconv::LossArgs a{r, t, r_image_stride, r_row_stride, t_image_stride, t_row_stride, B, H, W};
    if (const char* why = validate_loss(a, workspace_bytes, workspace)) return fail(-22, fn, why);
    if (!loss) return fail(-22, fn, "null loss");
    const char* why = nullptr;
    int rc = nconv::launch_loss_fwd(a, use_gradient_loss != 0, loss, (float*)workspace, (hipStream_t)stream, &why);
    return rc ? fail(rc, fn, why) : 0;
}

int nconv_depth_loss_bwd(const float* r, long long r_image_stride, long long r_row_stride, const float* t,
                         long long t_image_stride, long long t_row_stride, int B, int H, int W, int use_gradient_loss,
                         const float* gloss, const void* workspace, size_t workspace_bytes, float* g, void* stream) {
    const char* fn = "nconv_depth_loss_bwd";
    const nconv::LossArgs a{r, t, r_image_stride, r_row_stride, t_image_stride, t_row_stride, B, H, W};
    if (const char* why = validate_loss(a, workspace_bytes, workspace)) return fail(-22, fn, why);
    if (!g) return fail(-22, fn, "null g");
    const char* why = nullptr;
    int rc = nconv::launch_loss_bwd(a, use_gradient_loss != 0, gloss, (const float*)workspace, g, (hipStream_t)stream,
                                    &why);
    return rc ? fail(rc, fn, why) : 0;
}

}  // extern "C"
