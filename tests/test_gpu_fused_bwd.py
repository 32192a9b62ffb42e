"""GPU: the one-kernel backward of the exact-fp32 8 -> 8 5x5 layers (nconv_bwd_fused.hip: input and
weight gradient from one staging of {gN, gD}) against the two-kernel form (dgrad_tiled + wgrad_mfma,
NCONV_BWD_SEPARATE) and, through DNET, against the fp64 oracle (test_gpu_dnet / test_gpu_golden run
the fused kernel by default).

Autograd of models/step1.py:116-149 with the pooled-output gradient (DNET's nconv2 / down1 / down2 in
training) and the fused nconv1 weight gradient (nconv2). The two forms sum the same products in a
different order (per-row weight-gradient partials, the input gradient split over four waves by output
channel), so they agree to fp32 reassociation: normwise 1e-5 per tensor."""
import sys

import pytest
import torch

from nconv_cases import THRESH, rand_weight

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def _setup(nconv_amd, gpu, B, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    N = nconv_amd.nconv
    S = ((torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.1)).to(gpu)
    w1 = rand_weight(g, 8, 1, 5, 5).to(gpu)
    w2 = rand_weight(g, 8, 8, 5, 5).to(gpu)
    b1, b2 = (torch.rand(8, generator=g) * 0.1).to(gpu), (torch.rand(8, generator=g) * 0.1).to(gpu)
    s1, s2 = torch.empty(8, device=gpu), torch.empty(8, device=gpu)
    nconv_amd.weight_prep([w1, w2], [False, False], [s1, s2])
    sp1 = nconv_amd.LayerSpec(1, 8, (5, 5), (1, 1), (2, 2), mode=THRESH)
    sp2 = nconv_amd.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
    x1, c1 = N.layer_forward_raw(sp1, S, None, None, None, w1, b1, s1)
    y, co, py, pc, arg = N.layer_forward_pooled(sp2, x1, c1, None, None, w2, b2, s2, argmax=True)
    gy, gco = torch.randn(y.shape, generator=g).to(gpu), torch.randn(y.shape, generator=g).to(gpu)
    gpy, gpc = torch.randn(py.shape, generator=g).to(gpu), torch.randn(py.shape, generator=g).to(gpu)
    return dict(S=S, w1=w1, b1=b1, s1=s1, w2=w2, b2=b2, s2=s2, sp1=sp1, sp2=sp2, x1=x1, c1=c1, y=y, co=co,
                gy=gy, gco=gco, pool=(gpy, gpc, arg))


def _run(nconv_amd, t, separate, head, accumulate=False, prefill=None):
    N = nconv_amd.nconv
    gxa = torch.full_like(t["x1"], prefill) if prefill is not None else torch.empty_like(t["x1"])
    gca = torch.full_like(t["c1"], prefill) if prefill is not None else torch.empty_like(t["c1"])
    gw, gb = torch.empty_like(t["w2"]), torch.empty_like(t["b2"])
    hgw, hgb = torch.empty_like(t["w1"]), torch.empty_like(t["b1"])
    kw = dict(pool_grad=t["pool"], separate=separate, accumulate=accumulate)
    if head:
        kw["head"] = (t["sp1"], t["S"], t["w1"], t["b1"], t["s1"], hgw, hgb)
    N.layer_backward(t["sp2"], (t["x1"], t["c1"], None, None, t["w2"], t["b2"], t["s2"]), t["y"], t["co"],
                     t["gy"], t["gco"], (gxa, gca, None, None), gw, gb, **kw)
    torch.cuda.synchronize()
    return dict(gxa=gxa, gca=gca, gw=gw, gb=gb, hgw=hgw, hgb=hgb)


@pytest.mark.parametrize("B,H,W", [(2, 64, 128), (2, 45, 67), (1, 100, 200), (3, 20, 64), (8, 352, 1216)])
@pytest.mark.parametrize("head", [False, True])
def test_fused_bwd_matches_separate(nconv_amd, gpu, B, H, W, head):
    t = _setup(nconv_amd, gpu, B, H, W, seed=B * 1000 + H + W)
    a = _run(nconv_amd, t, separate=True, head=head)
    b = _run(nconv_amd, t, separate=False, head=head)
    keys = ("gxa", "gca", "gw", "gb") + (("hgw", "hgb") if head else ())
    rels = {k: _rel(b[k], a[k]) for k in keys}
    print(B, H, W, head, {k: f"{v:.2e}" for k, v in rels.items()})
    for k in keys:
        assert torch.isfinite(b[k]).all(), k
        assert rels[k] <= 1e-5, (k, rels[k])


def test_fused_bwd_accumulate(nconv_amd, gpu):
    """NCONV_BWD_ACCUMULATE through the one-kernel form (no head): added into pre-filled buffers,
    every element of them (ragged width, the last strip partly outside the image)."""
    t = _setup(nconv_amd, gpu, 2, 37, 90, seed=5)
    base = _run(nconv_amd, t, separate=False, head=False)
    acc = _run(nconv_amd, t, separate=False, head=False, accumulate=True, prefill=1.5)
    for k in ("gxa", "gca"):
        assert _rel(acc[k], base[k] + 1.5) <= 1e-6, k
    over = _run(nconv_amd, t, separate=False, head=False, prefill=float("nan"))
    for k in ("gxa", "gca"):  # overwrite: no NaN of the pre-fill survives
        assert torch.isfinite(over[k]).all() and torch.equal(over[k], base[k]), k


def test_fused_bwd_deterministic(nconv_amd, gpu):
    """Fixed-order sums: two runs bitwise equal."""
    t = _setup(nconv_amd, gpu, 2, 96, 160, seed=9)
    a = _run(nconv_amd, t, separate=False, head=True)
    b = _run(nconv_amd, t, separate=False, head=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("layers", [("nconv2",), ("nconv6",), ("nconv2", "nconv6"),
                                    ("nconv2", "nconv_down1", "nconv_down2", "nconv6")])
def test_dnet_fused_bwd_matches_two_kernel(nconv_amd, gpu, monkeypatch, layers):
    """The DNET training backward with the one-kernel forms (nconv2, the pooled 8 -> 8 5x5 down
    layers, nconv6 + nconv7) against the two-kernel forms: outputs bitwise, every gradient within
    1e-5 normwise (nconv1's, fused into nconv2's backward in both, and nconv7's, fused into
    nconv6's, too)."""
    dnet = sys.modules[nconv_amd.DNET.__module__]
    g = torch.Generator().manual_seed(77)
    B, H, W = 2, 96, 200
    S = ((torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.05)).to(gpu)
    gt = (torch.rand(B, 1, H, W, generator=g) * 80).to(gpu)
    res = {}
    for fused in (frozenset(), frozenset(layers)):
        monkeypatch.setattr(dnet, "FUSED_BWD", fused)
        torch.manual_seed(0)
        net = nconv_amd.SETP1_NCONV(crop="generalized").to(gpu)
        net.train()
        out = net(S)
        nconv_amd.train.calculate_loss(out, gt, True).backward()
        torch.cuda.synchronize()
        res[fused] = (out.detach(), {k: p.grad.detach().clone() for k, p in net.named_parameters() if p.grad is not None})
    (oa, ga), (ob, gb) = res.values()
    assert torch.equal(oa, ob)
    assert set(ga) == set(gb) and len(ga) == 18
    bad = [(k, _rel(gb[k], ga[k])) for k in ga if _rel(gb[k], ga[k]) > 1e-5]
    assert not bad, bad


def _tail_setup(nconv_amd, gpu, B, H, W, seed):
    """nconv6 (16 -> 8 3x3 padding 0 on cat(up2x(x7), x2)) + nconv7 (1x1 padding 2) as DNET's training
    tail builds them, with random inputs and a random gradient of nconv7's output."""
    dnet = sys.modules[nconv_amd.DNET.__module__]
    N = nconv_amd.nconv
    torch.manual_seed(seed)
    net = nconv_amd.SETP1_NCONV(crop="generalized").to(gpu)
    d = net.d_net
    with torch.no_grad():  # trained-like positive weights
        for m in (d.nconv6, d.nconv7):
            m.weight.copy_(torch.nn.functional.softplus(m.weight, beta=10))
    g = torch.Generator().manual_seed(seed)
    x2 = (torch.rand(B, 8, H, W, generator=g) * 5).to(gpu)
    c2 = torch.rand(B, 8, H, W, generator=g).to(gpu)
    x7 = (torch.rand(B, 8, H // 2, W // 2, generator=g) * 5).to(gpu)
    c7 = torch.rand(B, 8, H // 2, W // 2, generator=g).to(gpu)
    l6, l7 = d.nconv6, d.nconv7
    s6, s7 = torch.empty(8, device=gpu), torch.empty(1, device=gpu)
    N.weight_prep([l6.weight.detach(), l7.weight.detach()], [False, False], [s6, s7])
    w6 = d._phase_weights(gpu)[2]
    sp6, sp7 = l6.spec(nconv_amd._lib.UPCAT_UP_FIRST), l7.spec()
    W6 = (l6.weight.detach(), l6.bias.detach(), s6)
    W7 = (l7.weight.detach(), l7.bias.detach(), s7)
    x8, c8, x9, c9 = dnet._tail_train(sp6, sp7, x2, c2, x7, c7, W6, W7, w6)
    g9 = torch.randn(x9.shape, generator=g).to(gpu)
    return dict(sp6=sp6, sp7=sp7, x2=x2, c2=c2, x7=x7, c7=c7, W6=W6, W7=W7, x8=x8, c8=c8, x9=x9, c9=c9, g9=g9)


def _tail_run(nconv_amd, t, separate):
    N = nconv_amd.nconv
    out = dict(gxa=torch.empty_like(t["x2"]), gca=torch.empty_like(t["c2"]), gxb=torch.empty_like(t["x7"]),
               gcb=torch.empty_like(t["c7"]), gw=torch.empty_like(t["W6"][0]), gb=torch.empty_like(t["W6"][1]),
               gw7=torch.empty_like(t["W7"][0]))
    N.layer_backward(t["sp6"], (t["x2"], t["c2"], t["x7"], t["c7"], *t["W6"]), t["x8"], t["c8"], None, None,
                     (out["gxa"], out["gca"], out["gxb"], out["gcb"]), out["gw"], out["gb"],
                     tail=(t["sp7"], *t["W7"], t["x9"], t["c9"], t["g9"], out["gw7"]), separate=separate)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("B,H,W", [(2, 64, 128), (1, 48, 200), (3, 20, 66), (2, 100, 130), (8, 352, 1216)])
def test_fused_tail_bwd_matches_separate(nconv_amd, gpu, B, H, W):
    """nconv6 + nconv7 backward in one kernel against dgrad_phase<T7> + wgrad_mfma<T7>: the skip
    channels' gradient, the upsampled channels' (low-resolution) gradient, nconv6's and nconv7's
    weight gradients and nconv6's bias gradient within 1e-5 normwise (fp32 reassociation)."""
    t = _tail_setup(nconv_amd, gpu, B, H, W, seed=B * 100 + H + W)
    a = _tail_run(nconv_amd, t, separate=True)
    b = _tail_run(nconv_amd, t, separate=False)
    rels = {k: _rel(b[k], a[k]) for k in a}
    print(B, H, W, {k: f"{v:.2e}" for k, v in rels.items()})
    for k in a:
        assert torch.isfinite(b[k]).all(), k
        # nconv7's 8 weights are each one sum over every nconv6 pixel of the batch (3.4 M terms at
        # B=8 352x1216): the two forms' summation orders differ by ~1e-5 of its largest entry there
        assert rels[k] <= (3e-5 if k == "gw7" else 1e-5), (k, rels[k])


def test_fused_tail_bwd_deterministic(nconv_amd, gpu):
    t = _tail_setup(nconv_amd, gpu, 2, 96, 160, seed=3)
    a = _tail_run(nconv_amd, t, separate=False)
    b = _tail_run(nconv_amd, t, separate=False)
    for k in a:
        assert torch.equal(a[k], b[k]), k
