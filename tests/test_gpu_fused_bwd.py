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


@pytest.mark.parametrize("layers", [("nconv2",), ("nconv2", "nconv_down1", "nconv_down2")])
def test_dnet_fused_bwd_matches_two_kernel(nconv_amd, gpu, monkeypatch, layers):
    """The DNET training backward with the one-kernel form on nconv2 (default) or on every pooled
    8 -> 8 5x5 layer against the two-kernel form: outputs bitwise, every gradient within 1e-5
    normwise (nconv1's, fused into nconv2's backward in both, too)."""
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
