"""CPU, world_size 2 over gloo: DataParallelRCCL's bucketed all-reduce averages the present
gradients (skipping parameters without one) so every rank ends with the gradient of the mean of
the per-rank losses, and wrap-time broadcast makes replicas identical."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(4, 3)
        self.unused = torch.nn.Linear(3, 3)  # never receives a gradient (like rgb_encoder4)
        self.bn = torch.nn.BatchNorm1d(3)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import nconv_pkg
    m = nconv_pkg.load()
    torch.manual_seed(100 + rank)  # different init per rank: the wrap must broadcast rank 0's
    net = m.dp.DataParallelRCCL(Tiny())
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2 * world, 4, generator=g)
    loss = net.module.a(x[2 * rank:2 * rank + 2]).pow(2).mean()
    loss.backward()
    net.allreduce_grads()
    # numpy arrays travel by value: torch tensors would be passed as shared-memory handles that
    # vanish when this process exits before the parent has received them
    q.put((rank, {k: v.detach().numpy().copy() for k, v in net.module.state_dict().items()},
           net.module.a.weight.grad.numpy().copy(), net.module.unused.weight.grad))
    dist.destroy_process_group()


def test_allreduce_matches_mean_loss_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    res = [(r, {k: torch.from_numpy(v) for k, v in sd.items()}, torch.from_numpy(g), u) for r, sd, g, u in res]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, sd0, g0, u0), (_, sd1, g1, u1) = res
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), f"replicas differ at {k}"
    assert u0 is None and u1 is None
    assert torch.equal(g0, g1)
    # reference: mean over ranks of each rank's loss, on rank 0's (broadcast) weights
    torch.manual_seed(100)
    ref = Tiny()
    ref.load_state_dict(sd0)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2 * world, 4, generator=g)
    losses = [ref.a(x[2 * r:2 * r + 2]).pow(2).mean() for r in range(world)]
    (sum(losses) / world).backward()
    torch.testing.assert_close(g0, ref.a.weight.grad, rtol=1e-6, atol=1e-7)
