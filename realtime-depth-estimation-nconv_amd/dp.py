"""Data-parallel gradient reduction over RCCL — replaces the reference's single-process
nn.DataParallel (train_step1.py:153, train_step2.py:135).

One process per GPU (torchrun), backend "nccl" (= RCCL on ROCm, xGMI between MI355X GPUs). Frames
are independent, so the forward is a pure batch split with no exchange; the one exchange step is
the gradient all-reduce after backward:
  * one flat fp32 bucket holding every gradient that exists (step 1: 40.5 KB, step 2: 3.91 MB);
    parameters that never receive a gradient (the unused bnorm.* of NConv2d, rgb_encoder4 of
    SETP2_BP_TRAIN, frozen step-1 weights) are skipped without DDP's unused-parameter search;
  * all_reduce(SUM) then / world_size, i.e. the gradient of the mean of the per-rank losses;
  * parameters and buffers are broadcast from rank 0 once at wrap time.
EnforcePos mutates weights deterministically on every rank, so replicas stay identical without
further communication.

BatchNorm running statistics (SETP2's encoder / decoder, train mode): each rank updates its own
from its own frames, as each nn.DataParallel replica does; DataParallel then keeps only device 0's
replica as THE module, so its stats are device 0's. Policy here, the same: rank 0's buffers are the
model's. sync_buffers() (every rank calls it, e.g. before evaluation or a checkpoint) broadcasts
them; checkpoints are written by rank 0 (is_primary()), so a checkpoint and an evaluation see the
buffers DataParallel would have.

state_dict() keys carry the `module.` prefix, like nn.DataParallel's, so checkpoints written by
save_checkpoint stay loadable by the reference's loaders (models/step2.py:32-35).
"""
import torch
import torch.distributed as dist
import torch.nn as nn


class DataParallelRCCL(nn.Module):
    def __init__(self, module, process_group=None, broadcast=True):
        super().__init__()
        self.module = module
        self.process_group = process_group
        if broadcast and dist.is_available() and dist.is_initialized() and self.world_size() > 1:
            with torch.no_grad():
                for t in list(module.parameters()) + list(module.buffers()):
                    dist.broadcast(t.data, src=self._src_rank(), group=process_group)

    def world_size(self):
        if not (dist.is_available() and dist.is_initialized()):
            return 1
        return dist.get_world_size(self.process_group)

    def _src_rank(self):
        return dist.get_global_rank(self.process_group, 0) if self.process_group is not None else 0

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def is_primary(self):
        """True on the rank whose buffers (BatchNorm running statistics) are the model's."""
        if not (dist.is_available() and dist.is_initialized()):
            return True
        return dist.get_rank() == self._src_rank()

    @torch.no_grad()
    def sync_buffers(self):
        """Broadcast rank 0's buffers (BatchNorm running statistics) to every rank (collective:
        every rank calls it)."""
        if self.world_size() <= 1:
            return
        for t in self.module.buffers():
            dist.broadcast(t.data, src=self._src_rank(), group=self.process_group)

    def grad_bucket(self):
        """(name, gradient) of every parameter that has a gradient, in registration order: what one
        allreduce_grads call reduces. Parameters without one (the unused bnorm.* of NConv2d, the
        unused rgb_encoder4 and the frozen step 1 of SETP2_BP_TRAIN) are not in it."""
        return [(n, p.grad) for n, p in self.module.named_parameters() if p.grad is not None]

    @torch.no_grad()
    def allreduce_grads(self):
        """Average present gradients across ranks in one bucketed all-reduce. Runs whenever a process
        group is initialised, a one-rank group included (the same RCCL path, so it can be exercised
        and graph-captured on one GPU); without one it is a no-op."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        ws = self.world_size()
        grads = [g for _, g in self.grad_bucket()]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.process_group)
        flat.div_(ws)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n
