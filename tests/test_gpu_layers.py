"""GPU parity of single fused NConv layers (all load modes, tiled and generic paths) against the
oracle (tests/nconv_cases.oracle_layer = reference glue + models/step1.py:116-149) in float64.

Tolerances (written here, from BASELINE.json's north star and SURVEY.md 8(c)):
  forward  : elementwise |gpu - ref| <= 1e-4 * |ref| + 1e-5          (fp32 kernel vs fp64 oracle)
  backward : max|gpu - ref| / max|ref| <= 1e-3 per gradient tensor     
"""
import pytest
import torch

from nconv_cases import LAYER_CASES, THRESH, oracle_layer, rand_pair, rand_weight

pytestmark = pytest.mark.gpu


def _build(case, seed):
    name, mode, cin, cout, k, pad, stride, dil, groups, a_shape, b_shape = case
    g = torch.Generator().manual_seed(seed)
    xa, ca = rand_pair(g, 2, *a_shape, dtype=torch.float64)
    if mode == THRESH:
        xa = xa * (torch.rand(xa.shape, generator=g, dtype=torch.float64) < 0.3)
        ca = None
    if name.endswith("_ties"):  # small integer values and a 3-level confidence: many exact ties
        xa = torch.randint(0, 3, xa.shape, generator=g).double()
        ca = torch.randint(0, 3, ca.shape, generator=g).double() * 0.5
    xb = cb = None
    if b_shape is not None:
        xb, cb = rand_pair(g, 2, *b_shape, dtype=torch.float64)
    w = rand_weight(g, cout, cin // groups, k, k, torch.float64)
    b = torch.rand(cout, generator=g, dtype=torch.float64) * 0.1
    return xa, ca, xb, cb, w, b


def _spec(nconv_amd, case):
    name, mode, cin, cout, k, pad, stride, dil, groups, a_shape, b_shape = case
    return nconv_amd.LayerSpec(cin, cout, (k, k), (stride, stride), (pad, pad), (dil, dil), groups, 1e-7, mode, 0.01)


def _gpu(t, dev, grad=False):
    if t is None:
        return None
    return t.to(dev, torch.float32).contiguous().requires_grad_(grad)


def _wsum(nconv_amd, w):
    s = torch.empty(w.shape[0], device=w.device, dtype=torch.float32)
    nconv_amd.weight_prep([w.detach()], [False], [s])
    return s


@pytest.fixture(params=["bf16x3", "bf16x9", "fp32"])
def fwd_math(request, nconv_amd, monkeypatch):
    """Every forward arithmetic (include/nconv.h enum nconv_math)."""
    monkeypatch.setattr(nconv_amd.nconv, "FORWARD_MATH", nconv_amd.nconv._MATH_NAMES[request.param])
    return request.param


@pytest.mark.parametrize("case", LAYER_CASES, ids=[c[0] for c in LAYER_CASES])
def test_layer_forward(nconv_amd, gpu, case, fwd_math):
    xa, ca, xb, cb, w, b = _build(case, 1234)
    name, mode, *_ = case
    _, _, cin, cout, k, pad, stride, dil, groups, *_ = case
    ry, rc = oracle_layer(mode, xa, ca, xb, cb, w, b, (stride, stride), (pad, pad), (dil, dil), groups)
    gw = _gpu(w, gpu)
    y, c = nconv_amd.nconv_layer(_spec(nconv_amd, case), _gpu(xa, gpu), _gpu(ca, gpu), _gpu(xb, gpu),
                                 _gpu(cb, gpu), gw, _gpu(b, gpu), _wsum(nconv_amd, gw))
    torch.cuda.synchronize()
    assert y.shape == ry.shape and c.shape == rc.shape
    for got, ref in ((y, ry), (c, rc)):
        got = got.double().cpu()
        err = (got - ref).abs()
        bound = 1e-4 * ref.abs() + 1e-5
        assert torch.isfinite(got).all()
        assert (err <= bound).all(), f"{name}: max err {err.max():.3e}, worst ratio {(err / bound).max():.3f}"
        print(f"{name} [{fwd_math}]: max rel err {(err / (ref.abs() + 1e-30)).max():.2e}")


@pytest.fixture(params=["bf16x3", "bf16x9", "fp32"])
def bwd_math(request, nconv_amd, monkeypatch):
    """Every backward arithmetic (include/nconv.h nconv_layer.bwd_math: weight and input gradient)."""
    monkeypatch.setattr(nconv_amd.nconv, "BACKWARD_MATH", nconv_amd.nconv._MATH_NAMES[request.param])
    return request.param


@pytest.mark.parametrize("case", LAYER_CASES, ids=[c[0] for c in LAYER_CASES])
def test_layer_backward(nconv_amd, gpu, case, bwd_math):
    xa, ca, xb, cb, w, b = _build(case, 4321)
    name, mode, cin, cout, k, pad, stride, dil, groups, *_ = case
    leaves = [t.clone().requires_grad_(True) if t is not None else None for t in (xa, ca, xb, cb, w, b)]
    ry, rc = oracle_layer(mode, *leaves, (stride, stride), (pad, pad), (dil, dil), groups)
    g = torch.Generator().manual_seed(99)
    gy = torch.randn(ry.shape, generator=g, dtype=torch.float64)
    gc = torch.randn(rc.shape, generator=g, dtype=torch.float64)
    (ry * gy + rc * gc).sum().backward()

    gl = [_gpu(t, gpu, grad=True) for t in (xa, ca, xb, cb, w, b)]
    wsum = _wsum(nconv_amd, gl[4])
    # the kernels that ran (nconv_plan): a bf16 request on a multi-channel 3x3 / 5x5 layer must run
    # the bf16 matrix-core kernels, never a silent fallback to another arithmetic
    _, dg_k, wg_k = nconv_amd.nconv.kernel_plan(_spec(nconv_amd, case), *gl[:4], gl[4], gl[5], wsum)
    if wg_k != "generic" and cin > 1 and k > 1:
        a_shape, b_shape = case[9], case[10]
        exact_up = b_shape is not None and a_shape[1:] == (2 * b_shape[1], 2 * b_shape[2])
        dg_fp32 = "tiled_fp32_phase" if exact_up else "tiled_fp32"  # dgrad_phase: exact-2x UpCat
        want = (dg_fp32, "mfma_fp32") if bwd_math == "fp32" else ("mfma_" + bwd_math,) * 2
        assert (dg_k, wg_k) == want, (name, bwd_math, dg_k, wg_k)
    y, c = nconv_amd.nconv_layer(_spec(nconv_amd, case), *gl[:4], gl[4], gl[5], wsum)
    (y * gy.to(gpu, torch.float32) + c * gc.to(gpu, torch.float32)).sum().backward()
    torch.cuda.synchronize()
    labels = ("g_xa", "g_ca", "g_xb", "g_cb", "g_w", "g_b")
    for lab, ref_leaf, got_leaf in zip(labels, leaves, gl):
        if ref_leaf is None or ref_leaf.grad is None:
            continue
        ref = ref_leaf.grad
        got = got_leaf.grad.double().cpu()
        rel = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
        assert rel <= 1e-3, f"{name} {lab} [{bwd_math}]: normwise rel err {rel:.3e}"
        if lab == "g_w":
            print(f"{name} g_w [{bwd_math}]: normwise rel err {rel:.2e}")


@pytest.mark.parametrize("case", [c for c in LAYER_CASES if c[0] in ("nconv2_plain", "down_pool_odd",
                                                                      "nconv5_upcat_inexact", "nconv5_upcat_w4",
                                                                      "nconv6_upfirst_w4", "generic_stride2")],
                         ids=lambda c: c[0])
def test_bwd_accumulate_flag(nconv_amd, gpu, case, bwd_math):
    """NCONV_BWD_ACCUMULATE adds into pre-filled input-gradient buffers; without it every element
    is overwritten (garbage-filled buffers must come out identical to zero-filled ones)."""
    import ctypes
    lib = nconv_amd._lib
    xa, ca, xb, cb, w, b = _build(case, 77)
    spec = _spec(nconv_amd, case)
    t = [_gpu(v, gpu) for v in (xa, ca, xb, cb, w, b)]
    wsum = _wsum(nconv_amd, t[4])
    y, co = nconv_amd.nconv.layer_forward_raw(spec, *t[:4], t[4], t[5], wsum)
    gy, gc = torch.randn_like(y), torch.randn_like(co)
    L = spec.descriptor(*t[:4], t[4], t[5], wsum)
    ws_bytes = lib.lib().nconv_bwd_workspace_bytes(ctypes.byref(L))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=gpu)

    def run(fill, flags):
        outs = [torch.full_like(v, fill) if v is not None else None for v in t[:4]]
        gw, gb = torch.empty_like(t[4]), torch.empty_like(t[5])
        rc = lib.lib().nconv_bwd(ctypes.byref(L), lib.ptr(y), lib.ptr(co), lib.ptr(gy), lib.ptr(gc),
                                 *[lib.ptr(o) for o in outs], lib.ptr(gw), lib.ptr(gb), lib.ptr(ws), ws_bytes,
                                 flags, lib.stream_handle(gpu))
        lib.check(rc, "nconv_bwd")
        torch.cuda.synchronize()
        return outs, gw, gb

    o0, gw0, gb0 = run(0.0, 0)
    o1, gw1, gb1 = run(float("nan"), 0)
    o2, gw2, gb2 = run(1.5, lib.BWD_ACCUMULATE)
    for a0, a1, a2 in zip(o0, o1, o2):
        if a0 is None:
            continue
        assert torch.equal(a0, a1), "overwrite mode left unwritten elements"
        torch.testing.assert_close(a2, a0 + 1.5, rtol=1e-6, atol=1e-6)
    assert torch.equal(gw0, gw1) and torch.equal(gw0, gw2) and torch.equal(gb0, gb2)

    # NCONV_BWD_DEFER_REDUCE + nconv_wgrad_reduce (here batched with a second, independent
    # workspace of the same layer): bitwise the undeferred weight / bias gradients
    ws2 = torch.empty(ws_bytes, dtype=torch.uint8, device=gpu)
    outs = [torch.empty_like(v) if v is not None else None for v in t[:4]]
    gws = [torch.full_like(t[4], float("nan")) for _ in range(2)]
    gbs = [torch.full_like(t[5], float("nan")) for _ in range(2)]
    nparts = []
    for wsk in (ws, ws2):
        rc = lib.lib().nconv_bwd(ctypes.byref(L), lib.ptr(y), lib.ptr(co), lib.ptr(gy), lib.ptr(gc),
                                 *[lib.ptr(o) for o in outs], lib.ptr(gws[0]), lib.ptr(gbs[0]), lib.ptr(wsk),
                                 ws_bytes, lib.BWD_DEFER_REDUCE, lib.stream_handle(gpu))
        assert rc > 0, f"deferred nconv_bwd returned {rc}"
        nparts.append(rc)
    layers = (lib.NconvLayer * 2)(L, L)
    VP = ctypes.c_void_p * 2
    rc = lib.lib().nconv_wgrad_reduce(2, layers, VP(ws.data_ptr(), ws2.data_ptr()), (ctypes.c_int * 2)(*nparts),
                                      VP(*[g.data_ptr() for g in gws]), VP(*[g.data_ptr() for g in gbs]),
                                      lib.stream_handle(gpu))
    lib.check(rc, "nconv_wgrad_reduce")
    torch.cuda.synchronize()
    for k in range(2):
        assert torch.equal(gws[k], gw0) and torch.equal(gbs[k], gb0), "deferred reduction differs"


@pytest.mark.parametrize("H,W", [(30, 44), (262, 70)])  # 262 rows: the two-row 5x5 weight gradient
def test_nconv2d_module_train_step(nconv_amd, gpu, H, W):
    """Standalone NConv2d (the reference's layer API): EnforcePos pre-hook + forward + backward."""
    from oracle import nconv_ref as R
    torch.manual_seed(3)
    layer = nconv_amd.NConv2d(8, 8, (5, 5), "softplus", "p", padding=(2, 2)).to(gpu)
    w0 = layer.weight.detach().double().cpu().clone()
    g = torch.Generator().manual_seed(5)
    x, c = rand_pair(g, 2, 8, H, W, dtype=torch.float64)
    layer.train()
    xg, cg = _gpu(x, gpu, True), _gpu(c, gpu, True)
    y, co = layer(xg, cg)
    wr = R.softplus_pos(w0).requires_grad_(True)
    br = layer.bias.detach().double().cpu().clone().requires_grad_(True)
    xr, cr = x.clone().requires_grad_(True), c.clone().requires_grad_(True)
    ry, rc = R.nconv2d(xr, cr, wr, br, (1, 1), (2, 2))
    torch.testing.assert_close(layer.weight.detach().double().cpu(), wr.detach(), rtol=2e-6, atol=2e-7)
    torch.testing.assert_close(y.double().cpu(), ry, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(co.double().cpu(), rc, rtol=1e-4, atol=1e-6)
    gy = torch.randn(ry.shape, generator=g, dtype=torch.float64)
    (ry * gy + rc).sum().backward()
    (y * gy.to(gpu, torch.float32) + co).sum().backward()
    for got, ref in ((xg.grad, xr.grad), (cg.grad, cr.grad), (layer.weight.grad, wr.grad), (layer.bias.grad, br.grad)):
        rel = ((got.double().cpu() - ref).abs().max() / ref.abs().max()).item()
        assert rel <= 1e-3, rel


def test_fwd_head_negative_weights_sign_of_zero(nconv_amd, gpu):
    """Eval mode (no EnforcePos) allows negative nconv1 weights. A window without depth samples then
    sums only zero products; the dense order (an FMA chain from +0, like the reference's
    convolution) gives +0, so the fused head's nconv1 (nonzero taps only, first tap peeled) must
    give +0 too, not w * 0 = -0: nconv1's outputs bitwise, sign of zero included, against the
    separate nconv1 launch, and nconv2's edge-tile outputs likewise."""
    B, H, W = 2, 48, 96
    g = torch.Generator().manual_seed(4242)
    S = (torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.02)
    w1 = _gpu(-rand_weight(g, 8, 1, 5, 5), gpu)
    w2 = _gpu(rand_weight(g, 8, 8, 5, 5), gpu)
    b1 = _gpu(torch.zeros(8), gpu)
    b2 = _gpu(torch.rand(8, generator=g) * 0.1, gpu)
    s1, s2 = _wsum(nconv_amd, w1), _wsum(nconv_amd, w2)
    sp1 = nconv_amd.LayerSpec(1, 8, (5, 5), (1, 1), (2, 2), mode=THRESH)
    sp2 = nconv_amd.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
    Sg = S.to(gpu)
    N = nconv_amd.nconv
    x1, c1 = N.layer_forward_raw(sp1, Sg, None, None, None, w1, b1, s1)
    y0, c0 = N.layer_forward_raw(sp2, x1, c1, None, None, w2, b2, s2)
    w21 = N.head_weights(sp1, sp2, Sg, w1, b1, s1, w2, b2, s2)
    y2, c2, _, _, _, x1h, c1h = N.layer_forward_head(sp1, sp2, Sg, w1, b1, s1, w2, b2, s2, w21, train=True)
    torch.cuda.synchronize()
    bits = lambda t: t.contiguous().view(torch.int32)
    assert (x1 == 0).any() and (c1 == 0).any()  # sample-free windows exist
    assert torch.equal(bits(x1h), bits(x1)) and torch.equal(bits(c1h), bits(c1))
    # (cout = D / s1 with D = +0 and s1 < 0 is -0 in those windows; the old peeled product gave
    # D = -0 and so cout = +0)
    assert torch.signbit(c1[c1 == 0]).all()
    assert torch.equal(bits(y2[:, :, :16]), bits(y0[:, :, :16])) and torch.equal(bits(c2[:, :, :16]), bits(c0[:, :, :16]))


@pytest.mark.parametrize("shape", [(2, 8, 48, 128), (2, 8, 37, 71), (1, 8, 20, 66)])
def test_fwd_pooled_outputs(nconv_amd, gpu, shape):
    """nconv_fwd_pooled: identical y/cout to nconv_fwd, and pooled copies bit-equal to torch's
    max_pool2d of them (first maximum, floor mode; integer data makes ties frequent)."""
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randint(0, 3, shape, generator=g).float()
    c = torch.randint(0, 3, shape, generator=g).float() * 0.5
    spec = nconv_amd.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
    w = _gpu(rand_weight(g, 8, 8, 5, 5), gpu)
    b = _gpu(torch.rand(8, generator=g) * 0.1, gpu)
    ws = _wsum(nconv_amd, w)
    xg, cg = x.to(gpu), c.to(gpu)
    y0, c0 = nconv_amd.nconv.layer_forward_raw(spec, xg, cg, None, None, w, b, ws)
    y1, c1, py, pc = nconv_amd.nconv.layer_forward_pooled(spec, xg, cg, None, None, w, b, ws)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(c0, c1)
    assert torch.equal(py, torch.nn.functional.max_pool2d(y1, 2, 2))
    assert torch.equal(pc, torch.nn.functional.max_pool2d(c1, 2, 2))


@pytest.mark.parametrize("shape", [(2, 48, 128), (1, 37, 70), (3, 64, 96), (1, 352, 1216), (1, 20, 30)])
def test_fwd_head_exact_matches_unfused(nconv_amd, gpu, shape):
    """The exact-fp32 fused head (nconv1 on nonzero taps inside nconv2's tile, nconv2's N from
    two-pixel packed FMAs, its D from the composed 9x9 weights on c0 away from the image edge)
    against nconv1 and nconv2 as two exact launches: the edge tiles (here the top 16 rows) and every
    NaN position agree bit for bit, the rest within D2's regrouping rounding (fp32, non-negative
    terms); the pooled copies are torch's max_pool2d of the fused outputs exactly. The depth
    carries NaN (not > thresh: c0 = 0, S * c0 = NaN) and negative values like the f4 fixture."""
    B, H, W = shape
    g = torch.Generator().manual_seed(H * W + 1)
    S = (torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.05)
    S[torch.rand(B, 1, H, W, generator=g) < 0.002] = float("nan")
    S[torch.rand(B, 1, H, W, generator=g) < 0.002] = -3.0
    w1 = _gpu(rand_weight(g, 8, 1, 5, 5), gpu)
    w2 = _gpu(rand_weight(g, 8, 8, 5, 5), gpu)
    b1 = _gpu(torch.rand(8, generator=g) * 0.1, gpu)
    b2 = _gpu(torch.rand(8, generator=g) * 0.1, gpu)
    s1, s2 = _wsum(nconv_amd, w1), _wsum(nconv_amd, w2)
    sp1 = nconv_amd.LayerSpec(1, 8, (5, 5), (1, 1), (2, 2), mode=THRESH)
    sp2 = nconv_amd.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
    Sg = S.to(gpu)
    N = nconv_amd.nconv
    x1, c1 = N.layer_forward_raw(sp1, Sg, None, None, None, w1, b1, s1)
    y0, c0, py0, pc0 = N.layer_forward_pooled(sp2, x1, c1, None, None, w2, b2, s2)
    w21 = N.head_weights(sp1, sp2, Sg, w1, b1, s1, w2, b2, s2)
    y1, c1f, py1, pc1 = N.layer_forward_head(sp1, sp2, Sg, w1, b1, s1, w2, b2, s2, w21)
    torch.cuda.synchronize()
    for got, ref in ((y1, y0), (c1f, c0)):
        assert torch.equal(torch.isnan(got), torch.isnan(ref))
        assert torch.equal(got[:, :, :16].nan_to_num(7.0), ref[:, :, :16].nan_to_num(7.0))  # edge tiles
        torch.testing.assert_close(got.nan_to_num(7.0), ref.nan_to_num(7.0), rtol=1e-5, atol=1e-6)
    assert torch.equal(py1.nan_to_num(7.0), torch.nn.functional.max_pool2d(y1, 2, 2).nan_to_num(7.0))
    assert torch.equal(pc1, torch.nn.functional.max_pool2d(c1f, 2, 2))

    # training variant: the same nconv2 outputs, nconv1's outputs bitwise the separate nconv1's, and
    # the argmax words are the first-maximum slots of the head's own outputs (torch's indices)
    y2, c2, py2, pc2, arg, x1h, c1h = N.layer_forward_head(sp1, sp2, Sg, w1, b1, s1, w2, b2, s2, w21, train=True)
    torch.cuda.synchronize()
    for a, r in ((y2, y1), (c2, c1f), (py2, py1), (pc2, pc1), (x1h, x1), (c1h, c1)):
        assert torch.equal(a.nan_to_num(7.0), r.nan_to_num(7.0)) and torch.equal(torch.isnan(a), torch.isnan(r))
    Hp, Wp = H // 2, W // 2
    for plane, bits in ((y2, 0), (c2, 2)):
        _, idx = torch.nn.functional.max_pool2d(plane, 2, 2, return_indices=True)
        slot = ((idx // W) % 2) * 2 + (idx % W) % 2
        assert torch.equal((arg >> bits) & 3, slot.to(torch.int32)), bits


@pytest.mark.parametrize("shape", [(2, 48, 128), (1, 37, 70), (1, 352, 1216)])
def test_fwd_head_matches_unfused(nconv_amd, gpu, shape, monkeypatch):
    """nconv_fwd_head (nconv1 evaluated inside nconv2's staging, on the matrix cores in the same
    split-bf16 arithmetic as nconv2) against nconv1 (exact fp32) and nconv2 as two launches: the
    two differ by nconv1's split-product rounding (<= ~1.1e-5 relative per product), so nconv2's
    outputs and pooled copies agree within the forward tolerance, 1e-4 relative; the pooled copies
    must be torch's max_pool2d of the fused outputs exactly."""
    monkeypatch.setattr(nconv_amd.nconv, "FORWARD_MATH", nconv_amd._lib.MATH_BF16X3)
    B, H, W = shape
    g = torch.Generator().manual_seed(H * W)
    S = (torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.05)
    w1 = _gpu(rand_weight(g, 8, 1, 5, 5), gpu)
    w2 = _gpu(rand_weight(g, 8, 8, 5, 5), gpu)
    b1 = _gpu(torch.rand(8, generator=g) * 0.1, gpu)
    b2 = _gpu(torch.rand(8, generator=g) * 0.1, gpu)
    s1, s2 = _wsum(nconv_amd, w1), _wsum(nconv_amd, w2)
    sp1 = nconv_amd.LayerSpec(1, 8, (5, 5), (1, 1), (2, 2), mode=THRESH)
    sp2 = nconv_amd.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
    Sg = S.to(gpu)
    N = nconv_amd.nconv
    x1, c1 = N.layer_forward_raw(sp1, Sg, None, None, None, w1, b1, s1)
    y0, c0, py0, pc0 = N.layer_forward_pooled(sp2, x1, c1, None, None, w2, b2, s2)
    y1, c1f, py1, pc1 = N.layer_forward_head(sp1, sp2, Sg, w1, b1, s1, w2, b2, s2)
    torch.cuda.synchronize()
    for got, ref in ((y1, y0), (c1f, c0), (py1, py0), (pc1, pc0)):
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)
    assert torch.equal(py1, torch.nn.functional.max_pool2d(y1, 2, 2))
    assert torch.equal(pc1, torch.nn.functional.max_pool2d(c1f, 2, 2))


# Exact-2x UPCAT layers on the phase path (nconv_layer.wphase, nconv_fwd_phase.hip): both channel
# orders, paddings 0 / 1 / 2 (both phase parities), ragged widths, tiles cut by the image edge.
# (name, mode, pad, a-shape, b-shape)
PHASE_CASES = [
    ("skip_p1", 3, 1, (8, 24, 70), (8, 12, 35)),
    ("skip_p1_w4", 3, 1, (8, 26, 72), (8, 13, 36)),
    ("skip_p0", 3, 0, (8, 20, 64), (8, 10, 32)),
    ("skip_p2", 3, 2, (8, 18, 46), (8, 9, 23)),
    ("up_p0", 4, 0, (8, 34, 72), (8, 17, 36)),
    ("up_p1", 4, 1, (8, 36, 66), (8, 18, 33)),
]


@pytest.mark.parametrize("case", PHASE_CASES, ids=[c[0] for c in PHASE_CASES])
def test_upcat_phase_forward(nconv_amd, gpu, case):
    """The phase path (upsampled half at native resolution with summed fp32 weights) against the
    oracle's reference glue (cat + F.interpolate nearest) + NConv2d.forward, same tolerance as the
    dense kernels; nconv_plan must name the phase kernel and the dense path must agree."""
    name, mode, pad, a_shape, b_shape = case
    g = torch.Generator().manual_seed(11)
    xa, ca = rand_pair(g, 3, *a_shape, dtype=torch.float64)
    xb, cb = rand_pair(g, 3, *b_shape, dtype=torch.float64)
    w = rand_weight(g, 8, 16, 3, 3, torch.float64)
    b = torch.rand(8, generator=g, dtype=torch.float64) * 0.1
    ry, rc = oracle_layer(mode, xa, ca, xb, cb, w, b, (1, 1), (pad, pad))
    spec = nconv_amd.LayerSpec(16, 8, (3, 3), (1, 1), (pad, pad), mode=mode)
    t = [_gpu(v, gpu) for v in (xa, ca, xb, cb, w, b)]
    wsum = _wsum(nconv_amd, t[4])
    wph = torch.empty(1024, device=gpu)
    nconv_amd.nconv.phase_weights([t[4]], [8 if mode == 3 else 0], [wph])
    assert nconv_amd.nconv.kernel_plan(spec, *t[:4], t[4], t[5], wsum)[0] == "tiled_fp32"
    L = spec.descriptor(*t[:4], t[4], t[5], wsum, wph)
    import ctypes
    k = ctypes.c_int(-1)
    assert nconv_amd._lib.lib().nconv_plan(ctypes.byref(L), ctypes.byref(k), None, None) == 0
    assert nconv_amd._lib.KERNEL_NAMES[k.value] == "tiled_fp32_phase"
    y, c = nconv_amd.nconv.layer_forward_raw(spec, *t[:4], t[4], t[5], wsum, wphase=wph)
    yd, cd = nconv_amd.nconv.layer_forward_raw(spec, *t[:4], t[4], t[5], wsum)
    torch.cuda.synchronize()
    for got, ref in ((y, ry), (c, rc), (yd, ry), (cd, rc)):
        got = got.double().cpu()
        err = (got - ref).abs()
        bound = 1e-4 * ref.abs() + 1e-5
        assert (err <= bound).all(), f"{name}: max err {err.max():.3e}, worst ratio {(err / bound).max():.3f}"
    print(f"{name}: phase vs dense max rel {((y - yd).abs() / (yd.abs() + 1e-30)).max().item():.2e}")


@pytest.mark.parametrize("case", PHASE_CASES, ids=[c[0] for c in PHASE_CASES])
def test_upcat_phase_backward(nconv_amd, gpu, case):
    """Exact-fp32 backward of exactly-2x UpCat layers: the input gradient of the upsampled half runs
    at native resolution with box-summed weights (dgrad_phase, no staged plane or gather kernel).
    Every gradient against the oracle's autograd of cat + F.interpolate + NConv2d (normwise 1e-3,
    SURVEY 8(c)), with nconv_plan naming the phase kernel; padding 0 / 1 / 2 and both channel orders
    put the low pixels' 4x4 windows at every alignment against the image edge."""
    name, mode, pad, a_shape, b_shape = case
    g = torch.Generator().manual_seed(23)
    xa, ca = rand_pair(g, 2, *a_shape, dtype=torch.float64)
    xb, cb = rand_pair(g, 2, *b_shape, dtype=torch.float64)
    w = rand_weight(g, 8, 16, 3, 3, torch.float64)
    b = torch.rand(8, generator=g, dtype=torch.float64) * 0.1
    leaves = [t.clone().requires_grad_(True) for t in (xa, ca, xb, cb, w, b)]
    ry, rc = oracle_layer(mode, *leaves, (1, 1), (pad, pad))
    gy = torch.randn(ry.shape, generator=g, dtype=torch.float64)
    gc = torch.randn(rc.shape, generator=g, dtype=torch.float64)
    (ry * gy + rc * gc).sum().backward()
    spec = nconv_amd.LayerSpec(16, 8, (3, 3), (1, 1), (pad, pad), mode=mode)
    gl = [_gpu(t, gpu, grad=True) for t in (xa, ca, xb, cb, w, b)]
    wsum = _wsum(nconv_amd, gl[4])
    assert nconv_amd.nconv.kernel_plan(spec, *gl[:4], gl[4], gl[5], wsum)[1:] == ("tiled_fp32_phase", "mfma_fp32")
    y, c = nconv_amd.nconv_layer(spec, *gl[:4], gl[4], gl[5], wsum)
    (y * gy.to(gpu, torch.float32) + c * gc.to(gpu, torch.float32)).sum().backward()
    torch.cuda.synchronize()
    for lab, ref_leaf, got_leaf in zip(("g_xa", "g_ca", "g_xb", "g_cb", "g_w", "g_b"), leaves, gl):
        ref, got = ref_leaf.grad, got_leaf.grad.double().cpu()
        rel = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
        assert rel <= 1e-3, f"{name} {lab}: normwise rel err {rel:.3e}"
