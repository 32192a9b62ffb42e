#!/usr/bin/env python3
"""HBM bandwidth probes with PyTorch ops (developer tool, GPU): write-only fill, copy, and a
2-read/2-write elementwise op at the sizes of nconv2's B=8 352x1216 launch."""
import torch


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    n = 8 * 8 * 352 * 1216
    x, c = torch.rand(n, device=dev), torch.rand(n, device=dev)
    y, z = torch.empty(n, device=dev), torch.empty(n, device=dev)
    mb = n * 4 / 1e6
    us = t(lambda: y.fill_(1.0))
    print(f"fill  {mb:.0f} MB write: {us:.1f} us  {mb / us:.2f} TB/s")
    us = t(lambda: y.copy_(x))
    print(f"copy  {mb:.0f}+{mb:.0f} MB: {us:.1f} us  {2 * mb / us:.2f} TB/s")
    us = t(lambda: torch.mul(x, c, out=y))
    print(f"mul   {2 * mb:.0f}+{mb:.0f} MB: {us:.1f} us  {3 * mb / us:.2f} TB/s")
    us = t(lambda: (torch.add(x, c, out=y), torch.mul(x, c, out=z)))
    print(f"add+mul 2x({2 * mb:.0f}+{mb:.0f}) MB: {us:.1f} us  {6 * mb / us:.2f} TB/s")


if __name__ == "__main__":
    main()
