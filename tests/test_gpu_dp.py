"""The data-parallel gradient reduction (dp.DataParallelRCCL, replacing nn.DataParallel of
train_step1.py:153 / train_step2.py:135) on the device through RCCL: a one-rank `nccl` process group
on the box's GPU (the multi-rank exchange itself is covered by the gloo world-2 tests on CPU; an
8-GPU run is the driver's). Checks that the training step's bucket really goes through
torch.distributed.all_reduce on the nccl (RCCL) backend, that the reduced gradients and the AdamW
update equal an unwrapped model's bitwise (sum over one rank, / 1), and that the all-reduce can be
captured in the hipGraph of train.GraphedTrainStep (parameters after three replays within 1e-5 of
the eager DP steps)."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_group(gpu):
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=gpu)
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


def _count_allreduce(monkeypatch):
    calls = []
    real = dist.all_reduce

    def wrapped(t, *a, **k):
        calls.append((t.numel(), t.device.type))
        return real(t, *a, **k)
    monkeypatch.setattr(dist, "all_reduce", wrapped)
    return calls


def _data(gpu, B=2, H=64, W=96, seed=5):
    g = torch.Generator().manual_seed(seed)
    S = ((torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.1)).to(gpu)
    gt = ((torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < 0.3)).to(gpu)
    return S, gt


def _step1(nconv_amd, gpu, wrap, capturable=False):
    torch.manual_seed(0)
    net = nconv_amd.SETP1_NCONV(crop="generalized").to(gpu)
    if wrap:
        net = nconv_amd.dp.DataParallelRCCL(net)
    net.train()
    opt = nconv_amd.train.get_optimizer(net, "adam", 1e-2, 1e-7, capturable=capturable, fused=capturable)
    return net, opt


def test_step1_allreduce_eager_matches_single_process(nconv_amd, gpu, rccl_group, monkeypatch):
    calls = _count_allreduce(monkeypatch)
    S, gt = _data(gpu)
    dp, opt_dp = _step1(nconv_amd, gpu, True)
    ref, opt_ref = _step1(nconv_amd, gpu, False)
    assert dp.world_size() == 1
    for _ in range(2):
        for net, opt in ((dp, opt_dp), (ref, opt_ref)):
            opt.zero_grad()
            nconv_amd.train.calculate_loss(net(S), gt, True).backward()
            if net is dp:
                net.allreduce_grads()
            opt.step()
        torch.cuda.synchronize()
        for (n, a), (_, b) in zip(dp.grad_bucket(), ((n, p.grad) for n, p in ref.named_parameters()
                                                      if p.grad is not None)):
            assert torch.equal(a, b), n
    assert len(calls) == 2 and calls[0] == (sum(p.numel() for _, p in dp.grad_bucket()), "cuda")
    assert len(dp.grad_bucket()) == 18  # nine weights + nine biases; the unused bnorm.* have none
    for (n, a), (_, b) in zip(dp.module.named_parameters(), ref.named_parameters()):
        assert torch.equal(a, b), n


def test_step1_allreduce_graph_captured(nconv_amd, gpu, rccl_group, monkeypatch):
    calls = _count_allreduce(monkeypatch)
    S, gt = _data(gpu, seed=6)
    fn = lambda model, S, gt: nconv_amd.train.calculate_loss(model(S), gt, True)
    net_g, opt_g = _step1(nconv_amd, gpu, True, capturable=True)
    net_e, opt_e = _step1(nconv_amd, gpu, True, capturable=True)
    step = nconv_amd.train.GraphedTrainStep(net_g, opt_g, fn, (S, gt))
    n_capture = len(calls)
    assert n_capture >= 2  # warm-up iteration(s) + the captured one
    for _ in range(3):
        step(S, gt)
        opt_e.zero_grad()
        fn(net_e, S, gt).backward()
        net_e.allreduce_grads()
        opt_e.step()
    torch.cuda.synchronize()
    assert len(calls) == n_capture + 3  # replays issue no Python-side call: the collective is in the graph
    for (n, a), (_, b) in zip(net_g.module.named_parameters(), net_e.module.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7, msg=n)


def test_guided_bucket_allreduce(nconv_amd, gpu, rccl_group, monkeypatch):
    """SETP2_BP_TRAIN's bucket (82 tensors: frozen step 1 and unused rgb_encoder4 skipped) through
    RCCL equals the unwrapped model's gradients."""
    from guided_cases import f5_inputs
    calls = _count_allreduce(monkeypatch)
    rgb0, d0, rgb1, d1 = (t.to(gpu) for t in f5_inputs(48, 80))
    g = torch.Generator().manual_seed(2)
    gt = ((torch.rand(1, 1, 480, 640, generator=g) * 80) * (torch.rand(1, 1, 480, 640, generator=g) < 0.3)).to(gpu)
    grads = []
    for wrap in (True, False):
        torch.manual_seed(1)
        model = nconv_amd.SETP2_BP_TRAIN(None, step1_crop="generalized").to(gpu)
        net = nconv_amd.dp.DataParallelRCCL(model) if wrap else model
        net.train()
        est, _ = net(rgb0, d0, rgb1, d1)
        nconv_amd.train.calculate_loss_multi_resolution(est, gt, False).backward()
        if wrap:
            net.allreduce_grads()
            bucket = net.grad_bucket()
            assert len(bucket) == 82 and not any(n.startswith(("step1.", "rgb_encoder4.")) for n, _ in bucket)
        torch.cuda.synchronize()
        grads.append({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    assert len(calls) == 1
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n
