"""The hipGraph-replayed training step (train.GraphedTrainStep) against the same iterations run
eagerly: identical kernels in the same order, so parameters after three steps agree to fp32
round-off (tolerance: 1e-5 relative + 1e-7 absolute per element; AdamW's update is normalised, so
any ordering difference would show as O(lr) = 1e-2 changes). Also checks that constructing the
step leaves the model untouched (the warm-up runs on a snapshot)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(nconv_amd, dev, capturable, fused=False):
    torch.manual_seed(0)
    net = nconv_amd.SETP1_NCONV(crop="generalized").to(dev)
    net.train()
    opt = nconv_amd.train.get_optimizer(net, "adam", 1e-2, 1e-7, capturable=capturable, fused=fused)
    return net, opt


def _loss(nconv_amd):
    def fn(model, S, gt):
        return nconv_amd.train.calculate_loss(model(S)[0, :, :, :], gt[0, :, :, :], True)
    return fn


@pytest.mark.parametrize("fused", [False, True])
def test_graphed_train_step_matches_eager(nconv_amd, gpu, fused):
    g = torch.Generator().manual_seed(5)
    S = ((torch.rand(2, 1, 64, 96, generator=g) * 79 + 1) * (torch.rand(2, 1, 64, 96, generator=g) < 0.1)).to(gpu)
    gt = ((torch.rand(2, 1, 64, 96, generator=g) * 79 + 1) * (torch.rand(2, 1, 64, 96, generator=g) < 0.3)).to(gpu)
    fn = _loss(nconv_amd)

    net_e, opt_e = _setup(nconv_amd, gpu, capturable=True, fused=fused)
    net_g, opt_g = _setup(nconv_amd, gpu, capturable=True, fused=fused)
    before = {k: v.clone() for k, v in net_g.state_dict().items()}
    step = nconv_amd.train.GraphedTrainStep(net_g, opt_g, fn, (S, gt))
    for k, v in net_g.state_dict().items():
        assert torch.equal(v, before[k]), f"GraphedTrainStep construction changed {k}"

    losses_e, losses_g = [], []
    for _ in range(3):
        opt_e.zero_grad(set_to_none=True)
        loss = fn(net_e, S, gt)
        loss.backward()
        opt_e.step()
        losses_e.append(loss.item())
        losses_g.append(step().item())
    torch.cuda.synchronize()
    assert losses_g == pytest.approx(losses_e, rel=1e-5)
    sd_e, sd_g = net_e.state_dict(), net_g.state_dict()
    for k in sd_e:
        torch.testing.assert_close(sd_g[k], sd_e[k], rtol=1e-5, atol=1e-7, msg=k)
