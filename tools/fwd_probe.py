#!/usr/bin/env python3
"""Inference-forward probe (developer tool, GPU): the bench's hipGraph-replayed config-2 forward
(B=8 352x1216, exact fp32, generalized crop) with DNET attributes set from the command line, e.g.
    python3 tools/fwd_probe.py fused_head=0 inference_streams=1 [--steps 200] [--density 0.05]
prints frames/s; run under rocprofv3 --kernel-trace and read the replayed step's kernel timeline
with tools/fwd_timeline.py."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import nconv_pkg
    m = nconv_pkg.load()
    args = sys.argv[1:]
    opts = {"--steps": 200, "--density": 0.05, "--batch": 8}
    for k in list(opts):
        if k in args:
            i = args.index(k)
            opts[k] = type(opts[k])(args[i + 1])
            del args[i:i + 2]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = m.SETP1_NCONV(crop="generalized").to(dev)
    net.train()
    with torch.no_grad():
        net(torch.zeros(1, 1, 32, 32, device=dev))
    net.eval()
    for a in args:
        k, v = a.split("=")
        assert hasattr(net.d_net, k), k
        cur = getattr(net.d_net, k)
        setattr(net.d_net, k, bool(int(v)) if isinstance(cur, bool) else (None if v == "None" else int(v)))
    g = torch.Generator().manual_seed(0)
    B, H, W = opts["--batch"], 352, 1216
    S = ((torch.rand(B, 1, H, W, generator=g) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g) < opts["--density"])).to(dev)
    with torch.no_grad():
        for _ in range(3):
            net(S)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            net(S)
    for _ in range(50):
        graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(opts["--steps"]):
        graph.replay()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / opts["--steps"]
    print(f"forward {' '.join(args) or 'default'}: {ms:.4f} ms per B={B} step, {B / ms * 1e3:.1f} frames/s", flush=True)


if __name__ == "__main__":
    main()
