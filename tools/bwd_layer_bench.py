#!/usr/bin/env python3
"""One NConv layer backward at B=8 352x1216, repeated (developer tool for rocprofv3 / counter passes,
GPU): python3 tools/bwd_layer_bench.py [nconv2|down1|nconv6|nconv5] [reps] -> us per backward.
NCONV_BWD_MATH selects the backward arithmetic."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import nconv_pkg
    m = nconv_pkg.load()
    which = sys.argv[1] if len(sys.argv) > 1 else "nconv2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, H, W = 8, 352, 1216
    r = lambda *s: torch.rand(*s, device=dev, generator=g)
    lib = m._lib
    if which in ("nconv2", "down1"):  # down1: 2x2 max-pooled full-resolution source
        spec = m.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2), mode=lib.PLAIN if which == "nconv2" else lib.POOL2)
        xa, ca = r(B, 8, H, W) * 10, r(B, 8, H, W)
        xb = cb = None
        w = r(8, 8, 5, 5) + 0.05
    else:
        f = 1 if which == "nconv6" else 2
        mode = lib.UPCAT_UP_FIRST if which == "nconv6" else lib.UPCAT_SKIP_FIRST
        pad = 0 if which == "nconv6" else 1
        spec = m.LayerSpec(16, 8, (3, 3), (1, 1), (pad, pad), mode=mode)
        xa, ca = r(B, 8, H // f, W // f) * 10, r(B, 8, H // f, W // f)
        xb, cb = r(B, 8, H // (2 * f), W // (2 * f)) * 10, r(B, 8, H // (2 * f), W // (2 * f))
        w = r(8, 16, 3, 3) + 0.05
    b = r(8) * 0.1
    leaves = [t.requires_grad_(True) if t is not None else None for t in (xa, ca, xb, cb)]
    wl, bl = w.requires_grad_(True), b.requires_grad_(True)
    s = torch.empty(8, device=dev)
    m.weight_prep([wl.detach()], [False], [s])
    y, c = m.nconv_layer(spec, *leaves, wl, bl, s)
    gy, gc = torch.randn_like(y), torch.randn_like(c)

    def step():
        torch.autograd.grad((y, c), [t for t in leaves + [wl, bl] if t is not None], (gy, gc), retain_graph=True)
    step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        step()
    e1.record()
    e1.synchronize()
    print(f"{which} bwd [{os.environ.get('NCONV_BWD_MATH', 'fp32')}]: {e0.elapsed_time(e1) / reps * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
