"""CPU, world_size 2 over gloo: DataParallelRCCL on the real models (SETP1_NCONV and
SETP2_BP_TRAIN), the reference's nn.DataParallel wraps (train_step1.py:153, train_step2.py:135).

Which parameters receive a gradient is taken from the oracle (oracle/nconv_ref.py: the
reference's forward restated in torch CPU ops, pinned by golden fixtures) run under autograd on
tiny inputs: DNET's 9 NConv weights + biases, and SETP2's encoder / decoder parameters with the
step-1 network frozen (models/step2.py:37-40) and rgb_encoder4 unused (step2.py:60-77). The test
asserts that the gradient bucket holds exactly those tensors (18 / 40.5 KB and 82 / 3.91 MB,
SURVEY.md 8(a17)/(e)), that bnorm.* and rgb_encoder4.* are skipped, that the all-reduce averages,
and the BatchNorm buffer policy (sync_buffers: rank 0's running statistics everywhere).
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _grad_names_from_oracle(kind):
    """State-dict keys that get a gradient in the reference's training step, by autograd through
    the oracle on CPU (small inputs, generalized crop)."""
    import nconv_pkg
    from oracle import nconv_ref as R
    m = nconv_pkg.load()
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(5)
    if kind == "setp1":
        model = m.SETP1_NCONV(crop="generalized")
        sd = {k: v.detach().double().clone() for k, v in model.state_dict().items()}
        leaves = {k: v.requires_grad_(True) for k, v in sd.items()
                  if (k.endswith(".weight") or k.endswith(".bias")) and ".bnorm." not in k}
        params = R.dnet_params_from_state_dict(sd)
        S = (torch.rand(2, 1, 32, 48, generator=g, dtype=torch.float64) * 79 + 1) * \
            (torch.rand(2, 1, 32, 48, generator=g, dtype=torch.float64) < 0.3)
        out = R.dnet_forward(S, {n: (R.softplus_pos(w), b) for n, (w, b) in params.items()}, "generalized")
        loss = R.calculate_loss(out, torch.rand(out.shape, generator=g, dtype=torch.float64) * 10 + 1, True)
    else:
        model = m.SETP2_BP_TRAIN(None, step1_crop="generalized")
        sd = {k: v.detach().double().clone() for k, v in model.state_dict().items()}
        # step 1 frozen (requires_grad False in the reference): not leaves
        leaves = {k: v.requires_grad_(True) for k, v in sd.items()
                  if not k.startswith("step1.") and (k.endswith(".weight") or k.endswith(".bias"))}
        rgb = lambda: torch.rand(1, 3, 64, 96, generator=g, dtype=torch.float64) * 255
        dep = lambda: (torch.rand(1, 1, 64, 96, generator=g, dtype=torch.float64) * 79 + 1) * \
            (torch.rand(1, 1, 64, 96, generator=g, dtype=torch.float64) < 0.3)
        o0, o1 = R.setp2_forward(sd, rgb(), dep(), rgb(), dep(), crop="generalized", variant="train", training=True)
        gt = torch.rand(1, 1, 480, 640, generator=g, dtype=torch.float64) * 10 + 1
        loss = R.calculate_loss_multi_resolution(o0, gt, False) + R.calculate_loss_multi_resolution(o1, gt, False)
    loss.backward()
    return sorted(k for k, v in leaves.items() if v.grad is not None)


def _worker(rank, world, port, kind, names, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import nconv_pkg
    m = nconv_pkg.load()
    torch.manual_seed(100 + rank)  # different init per rank: the wrap broadcasts rank 0's
    model = m.SETP1_NCONV(crop="generalized") if kind == "setp1" else m.SETP2_BP_TRAIN(None, step1_crop="generalized")
    net = m.dp.DataParallelRCCL(model)
    want = set(names)
    g = torch.Generator().manual_seed(1000 + rank)
    for n, p in net.module.named_parameters():  # what the backward leaves behind on this rank
        p.grad = torch.randn(p.shape, generator=g) if n in want else None
    bucket = [(n, t.numel() * t.element_size()) for n, t in net.grad_bucket()]
    local = {n: p.grad.clone() for n, p in net.module.named_parameters() if p.grad is not None}
    net.allreduce_grads()
    # BN policy: perturb this rank's running stats, then sync_buffers -> rank 0's everywhere
    with torch.no_grad():
        for n, b in net.module.named_buffers():
            if b.is_floating_point():
                b.add_(rank + 1.0)
    net.sync_buffers()
    q.put((rank, bucket, {n: t.numpy() for n, t in local.items()},
           {n: p.grad.numpy().copy() for n, p in net.module.named_parameters() if p.grad is not None},
           {n: b.numpy().copy() for n, b in net.module.named_buffers()}, net.is_primary()))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,count,nbytes", [("setp1", 18, 40_500), ("setp2", 82, 3_910_000)])
def test_dp_bucket_on_real_models(kind, count, nbytes):
    names = _grad_names_from_oracle(kind)
    assert not any(".bnorm." in n or n.startswith("rgb_encoder4.") or n.startswith("step1.") and kind == "setp2"
                   for n in names)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, names, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, bucket0, local0, red0, buf0, prim0), (_, bucket1, local1, red1, buf1, prim1) = res
    # the bucket: exactly the oracle's gradient set, in one flat all-reduce
    assert [n for n, _ in bucket0] == [n for n, _ in bucket1]
    assert sorted(n for n, _ in bucket0) == names
    assert len(bucket0) == count
    total = sum(b for _, b in bucket0)
    assert abs(total - nbytes) <= 0.01 * nbytes, total
    assert not any(".bnorm." in n or n.startswith("rgb_encoder4.") for n, _ in bucket0)
    # averaging: every rank ends with the mean of the two ranks' gradients
    for n in names:
        mean = (torch.from_numpy(local0[n]) + torch.from_numpy(local1[n])) / 2
        torch.testing.assert_close(torch.from_numpy(red0[n]), mean)
        torch.testing.assert_close(torch.from_numpy(red1[n]), mean)
    # BN running statistics after sync_buffers: rank 0's on both ranks
    for n in buf0:
        assert (buf0[n] == buf1[n]).all(), n
    assert prim0 and not prim1
