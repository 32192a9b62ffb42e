/* A non-Python host of libnconv.so, compiled against include/nconv.h by tests/test_capi_host_cpu.py.
 * Prints the layout of every ABI struct (sizeof / offsetof per field) so the test can compare it
 * with the ctypes binding, then makes host-validated calls that must fail with -EINVAL before any
 * device work (no GPU needed). Plain C99: the header is what a C / cgo / JNI host would include. */
#include <stddef.h>
#include <stdio.h>
#include "nconv.h"

#define F(T, f) printf("\"%s.%s\": [%zu, %zu],\n", #T, #f, offsetof(T, f), sizeof(((T*)0)->f))
#define S(T) printf("\"%s\": [0, %zu],\n", #T, sizeof(T))

int main(void) {
    printf("{\n");
    S(nconv_src);
    F(nconv_src, x); F(nconv_src, c); F(nconv_src, C); F(nconv_src, H); F(nconv_src, W);
    S(nconv_layer);
    F(nconv_layer, B); F(nconv_layer, Cin); F(nconv_layer, H); F(nconv_layer, W); F(nconv_layer, Cout);
    F(nconv_layer, Ho); F(nconv_layer, Wo); F(nconv_layer, KH); F(nconv_layer, KW); F(nconv_layer, SH);
    F(nconv_layer, SW); F(nconv_layer, PH); F(nconv_layer, PW); F(nconv_layer, DH); F(nconv_layer, DW);
    F(nconv_layer, groups); F(nconv_layer, eps); F(nconv_layer, load_mode); F(nconv_layer, thresh);
    F(nconv_layer, a); F(nconv_layer, b); F(nconv_layer, weight); F(nconv_layer, bias); F(nconv_layer, wsum);
    F(nconv_layer, math);
    F(nconv_layer, bwd_math);
    F(nconv_layer, waux);
    S(nconv_dense_conv);
    F(nconv_dense_conv, B); F(nconv_dense_conv, x0); F(nconv_dense_conv, C0); F(nconv_dense_conv, x1);
    F(nconv_dense_conv, C1); F(nconv_dense_conv, H); F(nconv_dense_conv, W); F(nconv_dense_conv, Cout);
    F(nconv_dense_conv, Ho); F(nconv_dense_conv, Wo); F(nconv_dense_conv, kind); F(nconv_dense_conv, stride);
    F(nconv_dense_conv, wpack); F(nconv_dense_conv, bias); F(nconv_dense_conv, relu); F(nconv_dense_conv, wshort);
    F(nconv_dense_conv, out); F(nconv_dense_conv, out_C); F(nconv_dense_conv, out_c0);
    F(nconv_dense_conv, math);
    S(nconv_dense_wgrad);
    F(nconv_dense_wgrad, B); F(nconv_dense_wgrad, kind); F(nconv_dense_wgrad, stride); F(nconv_dense_wgrad, x0);
    F(nconv_dense_wgrad, C0); F(nconv_dense_wgrad, x1); F(nconv_dense_wgrad, C1); F(nconv_dense_wgrad, H);
    F(nconv_dense_wgrad, W); F(nconv_dense_wgrad, gy); F(nconv_dense_wgrad, Cout); F(nconv_dense_wgrad, Ho);
    F(nconv_dense_wgrad, Wo); F(nconv_dense_wgrad, gw);
    F(nconv_dense_wgrad, math);
    S(nconv_bwd_io);
    F(nconv_bwd_io, y); F(nconv_bwd_io, cout); F(nconv_bwd_io, gy); F(nconv_bwd_io, gcout); F(nconv_bwd_io, gxa);
    F(nconv_bwd_io, gca); F(nconv_bwd_io, gxb); F(nconv_bwd_io, gcb); F(nconv_bwd_io, gw); F(nconv_bwd_io, gbias);
    F(nconv_bwd_io, gy_pool); F(nconv_bwd_io, gcout_pool); F(nconv_bwd_io, pool_argmax); F(nconv_bwd_io, head);
    F(nconv_bwd_io, head_workspace); F(nconv_bwd_io, head_workspace_bytes); F(nconv_bwd_io, head_gw);
    F(nconv_bwd_io, head_gbias); F(nconv_bwd_io, head_nparts); F(nconv_bwd_io, tail); F(nconv_bwd_io, tail_y);
    F(nconv_bwd_io, tail_cout); F(nconv_bwd_io, tail_gy); F(nconv_bwd_io, tail_workspace);
    F(nconv_bwd_io, tail_workspace_bytes); F(nconv_bwd_io, tail_gw); F(nconv_bwd_io, tail_nparts);
    F(nconv_bwd_io, box_weights); F(nconv_bwd_io, tail_crop0); F(nconv_bwd_io, tail_h); F(nconv_bwd_io, tail_w);
    S(nconv_bn_train);
    F(nconv_bn_train, B); F(nconv_bn_train, C); F(nconv_bn_train, H); F(nconv_bn_train, W); F(nconv_bn_train, x);
    F(nconv_bn_train, gamma); F(nconv_bn_train, beta); F(nconv_bn_train, running_mean);
    F(nconv_bn_train, running_var); F(nconv_bn_train, momentum); F(nconv_bn_train, eps); F(nconv_bn_train, relu);
    F(nconv_bn_train, y); F(nconv_bn_train, mean); F(nconv_bn_train, invstd);

    /* host-validated calls: a DNET nconv2 descriptor with one defect each */
    nconv_layer L = {0};
    L.B = 1; L.Cin = 8; L.H = 16; L.W = 16; L.Cout = 8; L.Ho = 16; L.Wo = 16;
    L.KH = L.KW = 5; L.SH = L.SW = L.DH = L.DW = L.groups = 1; L.PH = L.PW = 2; L.eps = 1e-7f;
    L.load_mode = NCONV_LOAD_PLAIN; L.thresh = 0.01f; L.math = NCONV_MATH_FP32; L.bwd_math = NCONV_MATH_FP32;
    const float* fake = (const float*)0x1000; /* never dereferenced: validation fails first */
    L.a.x = fake; L.a.c = fake; L.a.C = 8; L.a.H = 16; L.a.W = 16;
    L.weight = L.bias = L.wsum = fake;
    float* out = (float*)0x2000;
    nconv_layer bad = L;
    bad.Ho = 15;
    int rc = nconv_fwd(&bad, out, out, NULL);
    printf("\"rc_bad_ho\": [%d, \"%s\"],\n", rc, nconv_last_error());
    bad = L;
    bad.math = 7;
    rc = nconv_fwd(&bad, out, out, NULL);
    printf("\"rc_bad_math\": [%d, \"%s\"],\n", rc, nconv_last_error());
    bad = L;
    bad.load_mode = 42;
    rc = nconv_fwd(&bad, out, out, NULL);
    printf("\"rc_bad_mode\": [%d, \"%s\"],\n", rc, nconv_last_error());
    printf("\"bwd_ws_ok\": [%zu, 0],\n", nconv_bwd_workspace_bytes(&L));
    /* a descriptor whose math fields are left at zero computes exact fp32 (the reference's) */
    nconv_layer z = L;
    z.math = 0; z.bwd_math = 0;
    int kf = -1, kd = -1, kw = -1;
    rc = nconv_plan(&z, &kf, &kd, &kw);
    printf("\"plan_zero\": [%d, %d, %d, %d, %d],\n", rc, z.math == NCONV_MATH_FP32, kf, kd, kw);
    printf("\"abi\": [%d, %d]\n}\n", nconv_abi_version(), NCONV_ABI_VERSION);
    return 0;
}
