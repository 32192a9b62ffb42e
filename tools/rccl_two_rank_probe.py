#!/usr/bin/env python3
"""Two ranks on ONE GPU over the nccl (RCCL) backend (developer probe, GPU): can RCCL run a
world-size-2 all-reduce with both ranks on cuda:0? Launched by torch.distributed.run:
    python3 -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/rccl_two_rank_probe.py
Each rank all-reduces [rank + 1] * 4 and prints the result (expected 3.0 each)."""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}/{world}: all_reduce -> {t.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
