#!/usr/bin/env python3
"""Per-shape throughput of the dense MFMA kernels (developer tool, GPU):
python3 tools/dense_microbench.py  ->  one line per (op, shape): us per launch and TF/s."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=10):
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
    import nconv_pkg
    m = nconv_pkg.load()
    D = m.dense
    dev = torch.device("cuda:0")
    B = 8
    # (name, kind, stride, cin, cout, H, W): layers of the guided model at 352x1216
    shapes = [("fuse3 conv 64->32", 0, 1, 64, 32, 352, 1216), ("fuse3 conv 32->32", 0, 1, 32, 32, 352, 1216),
              ("fuse2 conv 128->64", 0, 1, 128, 64, 176, 608), ("fuse2 conv 64->64", 0, 1, 64, 64, 176, 608),
              ("enc1 3x3 s2 32->64", 0, 2, 32, 64, 352, 1216), ("fuse3 upf TR 33->32", 2, 2, 33, 32, 176, 608),
              ("fuse2 upf TR 65->64", 2, 2, 65, 64, 88, 304), ("dgrad TR: C4 32->33", 3, 2, 32, 33, 352, 1216)]
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None  # name substrings
    fwd_only = os.environ.get("DENSE_FWD_ONLY") == "1"
    ops = os.environ.get("DENSE_OPS", "fwd,wgrad,dgrad").split(",")  # e.g. DENSE_OPS=wgrad
    for name, kind, s, cin, cout, H, W in shapes:
        if only and not any(o in name for o in only):
            continue
        x = torch.randn(B, cin, H, W, device=dev)
        k = 3 if kind == 0 else (4 if kind == 3 else 1)
        w = torch.randn(cin, cout, 4, 4, device=dev) if kind == 2 else torch.randn(cout, cin, k, k, device=dev)
        wp = D.pack(kind, w, cin, cout)
        out = D.conv(x, kind, s, wp, None, False, cout)
        taps = {0: 9, 1: 1, 2: 4, 3: 16}[kind]
        pix = out.shape[0] * out.shape[2] * out.shape[3]
        fl = 2 * cin * cout * taps * pix
        if "fwd" in ops:
            us = timeit(lambda: D.conv(x, kind, s, wp, None, False, cout, out=out))
            print(f"fwd   {name:24s} {us:9.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
        if kind in (0, 2) and not fwd_only:
            g = torch.randn_like(out)
            if "wgrad" in ops:
                us = timeit(lambda: D.wgrad(x, None, g, kind, s, w.shape))
                print(f"wgrad {name:24s} {us:9.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
            if "dgrad" in ops:
                us = timeit(lambda: D.dgrad(g, w, kind, s, x.shape))
                print(f"dgrad {name:24s} {us:9.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
