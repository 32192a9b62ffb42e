#!/usr/bin/env python3
"""Training-step probe (developer tool, GPU): the bench's graphed config-2 training step
(B=8 352x1216) with dnet's module switches set from the command line, e.g.
    python3 tools/train_probe.py WGRAD_STREAM=0 FUSE_HEAD_BWD=0 [--steps 20] [--eager]
prints ms per step (hipGraph-replayed; --eager: the eager step); run under rocprofv3 --kernel-trace
for the per-kernel split."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import nconv_pkg
    m = nconv_pkg.load()
    steps = 20
    args = sys.argv[1:]
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    eager = "--eager" in args
    if eager:
        args.remove("--eager")
    for a in args:
        k, v = a.split("=")
        obj = m.dnet
        if k.startswith("DNET."):  # a DNET class attribute (merged_prologue, crop_in_tail, ...)
            obj, k = m.DNET, k[5:]
        assert hasattr(obj, k), k
        setattr(obj, k, bool(int(v)) if isinstance(getattr(obj, k), bool) else int(v))
    dev = torch.device("cuda:0")
    step = bench.make_train_step(m, dev, 8, 352, 1216, 0, graph=not eager)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    e1.synchronize()
    print(f"train step{' eager' if eager else ''} {' '.join(args) or 'default'}: {e0.elapsed_time(e1) / steps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
