#!/usr/bin/env python3
"""Rounding bias of the dense convolutions' fp32 accumulation (developer tool, GPU): long dot
products of positive terms through nconv_dense_conv_fwd (1x1 and 3x3), torch's fp32 GPU conv and an
fp32 CPU conv, each against float64. Round-to-nearest gives a signed mean error near 0 (|bias| ~
1/sqrt(n) of the mean |error|); truncating accumulation gives a bias near -1."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stats(tag, got, ref):
    e = got.double().cpu() - ref
    print(f"{tag:28s} rel {(e.abs().max() / ref.abs().max()).item():.2e}  mean|e|/mean|ref| "
          f"{(e.abs().mean() / ref.abs().mean()).item():.2e}  bias {(e.mean() / e.abs().mean()).item():+.3f}",
          flush=True)


def main():
    import nconv_pkg
    m = nconv_pkg.load()
    D = m.dense
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    for kind, k, cin in ((D.DENSE_1X1, 1, 512), (D.DENSE_3X3, 3, 128), (D.DENSE_3X3, 3, 64)):
        x = torch.rand(2, cin, 32, 64, generator=g)
        w = torch.rand(32, cin, k, k, generator=g)
        ref = F.conv2d(x.double(), w.double(), None, 1, k // 2)
        wp = D.pack(kind, w.to(dev), cin, 32)
        ours = D.conv(x.to(dev).contiguous(), kind, 1, wp, None, False, 32)
        torch.cuda.synchronize()
        stats(f"libnconv {k}x{k} cin {cin}", ours, ref)
        stats(f"torch gpu {k}x{k} cin {cin}", F.conv2d(x.to(dev), w.to(dev), None, 1, k // 2), ref)
        stats(f"torch cpu {k}x{k} cin {cin}", F.conv2d(x, w, None, 1, k // 2), ref)
    # zero-mean data (the backward's case): the error's bias against the sign of the value
    x = torch.randn(2, 128, 32, 64, generator=g)
    w = torch.randn(32, 128, 3, 3, generator=g)
    ref = F.conv2d(x.double(), w.double(), None, 1, 1)
    ours = D.conv(x.to(dev).contiguous(), D.DENSE_3X3, 1, D.pack(D.DENSE_3X3, w.to(dev), 128, 32), None, False, 32)
    e = ours.double().cpu() - ref
    print("signed data 3x3: rel", (e.abs().max() / ref.abs().max()).item(), "bias vs sign(ref)",
          ((e * ref.sign()).mean() / e.abs().mean()).item(), "sum e / sum |e|", (e.sum() / e.abs().sum()).item())


if __name__ == "__main__":
    main()
