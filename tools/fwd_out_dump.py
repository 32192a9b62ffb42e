#!/usr/bin/env python3
"""DNET eval forward of a fixed B=8 352x1216 input, saved to a file (A/B bitwise checks between library
variants; developer tool, GPU): python3 tools/fwd_out_dump.py OUT.pt"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import nconv_pkg
    m = nconv_pkg.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = m.SETP1_NCONV(crop="generalized").to(dev)
    net.train()
    with torch.no_grad():
        net(torch.zeros(1, 1, 32, 32, device=dev))
    net.eval()
    S = bench.sparse_depth(torch.Generator().manual_seed(1000), 8, 352, 1216, dev)
    with torch.no_grad():
        out = net(S)
    torch.save(out.cpu(), sys.argv[1])


if __name__ == "__main__":
    main()
