"""CPU: the training-step glue (utils.py restated in nconv_amd.train) against the oracle, and the
reference checkpoint format round trip (module. prefixes, weights-only load)."""
import os

import torch

from oracle import nconv_ref as R


def test_losses_match_oracle(nconv_amd):
    g = torch.Generator().manual_seed(0)
    for shape in [(1, 20, 30), (1, 33, 47)]:
        gt = torch.rand(shape, generator=g, dtype=torch.float64) * 80
        gt = gt * (torch.rand(shape, generator=g, dtype=torch.float64) < 0.3)
        rec = torch.rand(shape, generator=g, dtype=torch.float64) * 80
        for ug in (True, False):
            a = nconv_amd.train.calculate_loss(rec, gt, ug)
            b = R.calculate_loss(rec, gt, ug)
            torch.testing.assert_close(a, b, rtol=1e-12, atol=1e-12)
    imgs = [torch.rand(2, 1, h, w, generator=g, dtype=torch.float64) for h, w in [(60, 80), (120, 160)]]
    gt = torch.rand(2, 1, 480, 640, generator=g, dtype=torch.float64)
    torch.testing.assert_close(nconv_amd.train.calculate_loss_multi_resolution(imgs, gt, True),
                               R.calculate_loss_multi_resolution(imgs, gt, True), rtol=1e-12, atol=1e-12)


def test_optimizer_factory(nconv_amd):
    net = torch.nn.Linear(2, 2)
    assert isinstance(nconv_amd.train.get_optimizer(net, "adam", 1e-2, 1e-7), torch.optim.AdamW)
    assert isinstance(nconv_amd.train.get_optimizer(net, "sgd", 1e-2, 1e-7), torch.optim.SGD)


def test_checkpoint_roundtrip_with_module_prefix(nconv_amd, tmp_path):
    torch.manual_seed(0)
    net = nconv_amd.dp.DataParallelRCCL(nconv_amd.SETP1_NCONV(), broadcast=False)
    assert all(k.startswith("module.") for k in net.state_dict())
    nconv_amd.train.save_checkpoint(net, 3, str(tmp_path), {"loss": 1.0}, "ck")
    fresh = nconv_amd.SETP1_NCONV()
    nconv_amd.train.load_checkpoint(fresh, os.path.join(tmp_path, "ck.pth.tar"), strict=True)
    for (k, v), (k2, v2) in zip(fresh.state_dict().items(), net.module.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)


def test_crop_backward_is_the_slice_backward(nconv_amd):
    """DNET's training output crop (dnet.CropFn: one zero-pad in the backward) against autograd's
    slice of step1.py:94, for the literal and generalized crops."""
    g = torch.Generator().manual_seed(3)
    for H, W in [(10, 12), (480, 640), (352, 1216)]:
        for crop in ("literal", "generalized"):
            h, w = nconv_amd.dnet.crop_hw(H, W, crop)
            x = torch.randn(1, 1, H + 2, W + 2, generator=g, requires_grad=True)
            y = nconv_amd.dnet.CropFn.apply(x, h, w)
            ref = x[:, :, 1:1 + h, 1:1 + w]
            assert torch.equal(y, ref) and not y._is_view()
            go = torch.randn(ref.shape, generator=g)
            a, = torch.autograd.grad(y, x, go)
            b, = torch.autograd.grad(ref, x, go)
            assert torch.equal(a, b)
    # in-place operations on the output (a script's clamp_ / masked_fill_) are legal under autograd,
    # as they are on the reference's slice
    x = torch.randn(1, 1, 12, 14, generator=g, requires_grad=True)
    y = nconv_amd.dnet.CropFn.apply(x, 10, 12)
    y.clamp_(min=0.0)
    ref = x[:, :, 1:11, 1:13].clone().clamp_(min=0.0)
    go = torch.randn(ref.shape, generator=g)
    a, = torch.autograd.grad(y, x, go)
    b, = torch.autograd.grad(ref, x, go)
    assert torch.equal(a, b)
