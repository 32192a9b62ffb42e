"""Accuracy class of the forward arithmetics (include/nconv.h enum nconv_math) on the matrix-core
layer shapes, against the fp64 oracle (tests/nconv_cases.oracle_layer):

  * NCONV_MATH_FP32 (vector ALU, fmaf products) is the reference class: one rounding per product
    accumulation, like the reference's fp32 F.conv2d (models/step1.py:119-122).
  * NCONV_MATH_BF16X9 splits both operands into three bf16 parts (an exact decomposition) and
    forms all nine partial products, each exact in fp32, so it must land in the SAME class:
    max relative error <= 6x the fp32 path's on the same inputs (measured: 0.7-1.0x with positive
    weights, 1-4x with signed ones), where the two-part bf16x3 sits up to two orders of magnitude
    higher with signed weights (measured 3e-5 .. 1.4e-2: cancellation exposes its ~1e-5 product
    error).
Signed weights (Kaiming-style, no EnforcePos) are included: exact products do not rely on the
absence of cancellation.
"""
import pytest
import torch

from nconv_cases import LAYER_CASES, oracle_layer, rand_pair

pytestmark = pytest.mark.gpu

MFMA_CASES = [c for c in LAYER_CASES
              if c[0] in ("nconv2_plain", "nconv2_w4", "down_pool_odd", "down_pool_even",
                          "nconv4_upcat_exact", "nconv5_upcat_inexact", "nconv6_upfirst_p0",
                          "nconv6_upfirst_w4")]


def _inputs(case, seed, signed):
    name, mode, cin, cout, k, pad, stride, dil, groups, a_shape, b_shape = case
    g = torch.Generator().manual_seed(seed)
    xa, ca = rand_pair(g, 2, *a_shape, dtype=torch.float64)
    xb = cb = None
    if b_shape is not None:
        xb, cb = rand_pair(g, 2, *b_shape, dtype=torch.float64)
    if signed:
        w = (torch.rand(cout, cin, k, k, generator=g, dtype=torch.float64) - 0.5) * 0.6
        w[:, :, k // 2, k // 2] += 1.0  # keep D = W*c away from zero (y = N / (D + eps))
    else:
        w = torch.rand(cout, cin, k, k, generator=g, dtype=torch.float64) + 0.05
    # round the inputs to fp32 first, so the fp64 oracle sees exactly what the kernels see
    f = lambda t: None if t is None else t.float().double()
    return f(xa), f(ca), f(xb), f(cb), f(w), f(torch.rand(cout, generator=g, dtype=torch.float64) * 0.1)


def _run(nconv_amd, gpu, case, math, tensors):
    name, mode, cin, cout, k, pad, stride, dil, groups, *_ = case
    spec = nconv_amd.LayerSpec(cin, cout, (k, k), (stride, stride), (pad, pad), (dil, dil), groups, 1e-7, mode, 0.01)
    dev = [None if t is None else t.to(gpu, torch.float32).contiguous() for t in tensors]
    s = torch.empty(cout, device=gpu)
    nconv_amd.weight_prep([dev[4]], [False], [s])
    old = nconv_amd.nconv.FORWARD_MATH
    nconv_amd.nconv.FORWARD_MATH = math
    try:
        y, c = nconv_amd.nconv_layer(spec, dev[0], dev[1], dev[2], dev[3], dev[4], dev[5], s)
    finally:
        nconv_amd.nconv.FORWARD_MATH = old
    torch.cuda.synchronize()
    return y.double().cpu(), c.double().cpu()


@pytest.mark.parametrize("signed", [False, True], ids=["positive_w", "signed_w"])
@pytest.mark.parametrize("case", MFMA_CASES, ids=[c[0] for c in MFMA_CASES])
def test_bf16x9_is_fp32_class(nconv_amd, gpu, case, signed):
    lib = nconv_amd._lib
    name, mode, cin, cout, k, pad, stride, dil, groups, *_ = case
    t = _inputs(case, 777, signed)
    ry, rc = oracle_layer(mode, *t, (stride, stride), (pad, pad), (dil, dil), groups)
    errs = {}
    for label, math in (("fp32", lib.MATH_FP32), ("bf16x9", lib.MATH_BF16X9), ("bf16x3", lib.MATH_BF16X3)):
        y, c = _run(nconv_amd, gpu, case, math, t)
        # relative to the magnitude of the sums (cout = D / s carries D's relative error; y's
        # absolute error relative to |y| + 1 covers the divide's conditioning for signed weights)
        ey = ((y - ry).abs() / (ry.abs() + 1.0)).max().item()
        ec = ((c - rc).abs() / (rc.abs() + 1e-3)).max().item()
        errs[label] = max(ey, ec)
    print(f"{name} {'signed' if signed else 'positive'}: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    # same class as the fp32 path (independent rounding sequences: within a small factor of it)
    assert errs["bf16x9"] <= 6 * errs["fp32"] + 2e-7, errs
    if signed:  # where two-part products lose digits to cancellation, exact products do not
        assert errs["bf16x9"] * 3 <= errs["bf16x3"], errs
