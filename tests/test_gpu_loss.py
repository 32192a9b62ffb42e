"""The fused training loss (train.DepthLossFn: nconv_depth_loss_fwd / _bwd) against the reference's
PyTorch op sequence (train._calculate_loss_torch = utils.py:95-151 on the same device tensors).

Loss: relative 2e-6 (fp32 sums in a different order; the block sums are combined in double).
Gradient: elementwise |g - g_ref| <= 1e-5 * max|g_ref| (the Sobel signs are formed with the same
operation order as the reference, so they agree exactly; the rest is fp32 rounding of the scale
factors). Covers both loss modes, cropped (row-strided) views like DNET's output, odd and tiny
planes, all-zero targets in a region (masked_fill), exact zeros of the Sobel response (sign 0),
an upstream gradient other than 1, and capture in a hipGraph."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _planes(gen, H, W, dev, crop=False, density=0.3):
    Hp, Wp = (H + 2, W + 2) if crop else (H, W)
    r = (torch.rand(1, Hp, Wp, generator=gen) * 80).to(dev)
    t = ((torch.rand(1, H, W, generator=gen) * 79 + 1) * (torch.rand(1, H, W, generator=gen) < density)).to(dev)
    if crop:
        r = r[:, 1:1 + H, 1:1 + W]
    return r, t


def _check(nconv_amd, r, t, use_grad, scale=1.0):
    tr = nconv_amd.train
    a = r.detach().clone().requires_grad_(True) if r.is_contiguous() else r.detach()
    if not r.is_contiguous():
        base = r._base.detach().clone().requires_grad_(True)
        a = base[:, 1:1 + t.shape[-2], 1:1 + t.shape[-1]]
    assert tr._fused_loss_ok(a, t)
    b = r.detach().clone().requires_grad_(True)
    L = tr.calculate_loss(a, t, use_grad)
    Lr = tr._calculate_loss_torch(b, t, use_grad)
    assert L.grad_fn is not None and "DepthLossFn" in type(L.grad_fn).__name__
    assert abs(L.item() - Lr.item()) <= 2e-6 * abs(Lr.item()) + 1e-12, (L.item(), Lr.item())
    (L * scale).backward()
    (Lr * scale).backward()
    ga = (base.grad[:, 1:1 + t.shape[-2], 1:1 + t.shape[-1]] if not r.is_contiguous() else a.grad)
    gb = b.grad
    tol = 1e-5 * gb.abs().max().item() + 1e-12
    err = (ga - gb).abs().max().item()
    assert err <= tol, (err, tol)
    assert torch.equal(ga == 0, gb == 0) or use_grad  # masked positions: exactly zero gradient
    assert torch.all(ga[t == 0] == 0)


@pytest.mark.parametrize("use_grad", [True, False])
@pytest.mark.parametrize("H,W,crop", [(352, 1216, True), (64, 96, False), (7, 3, False), (1, 5, False),
                                      (33, 65, True)])
def test_depth_loss_matches_reference_ops(nconv_amd, gpu, use_grad, H, W, crop):
    g = torch.Generator().manual_seed(H * 1000 + W)
    r, t = _planes(g, H, W, gpu, crop=crop)
    _check(nconv_amd, r, t, use_grad)


def test_depth_loss_zero_regions_and_scale(nconv_amd, gpu):
    g = torch.Generator().manual_seed(3)
    r, t = _planes(g, 48, 80, gpu, density=0.9)
    t[:, 10:30, 20:60] = 0  # masked block: diff == 0 there, Sobel response exactly 0 inside
    r[:, 0:5, :] = 7.0       # flat data: exact zeros of the Sobel response where t is dense
    t[:, 0:5, :] = 7.0
    _check(nconv_amd, r, t, True, scale=3.5)


def test_depth_loss_in_hipgraph(nconv_amd, gpu):
    g = torch.Generator().manual_seed(9)
    r, t = _planes(g, 40, 72, gpu)
    x = r.clone().requires_grad_(True)
    tr = nconv_amd.train
    ref = tr._calculate_loss_torch(r, t, True).item()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tr.calculate_loss(x, t, True).backward()  # warm-up
    torch.cuda.current_stream().wait_stream(s)
    x.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        L = tr.calculate_loss(x, t, True)
        L.backward()
    graph.replay()
    torch.cuda.synchronize()
    assert abs(L.item() - ref) <= 2e-6 * abs(ref)
    assert torch.isfinite(x.grad).all() and x.grad.abs().sum().item() > 0
