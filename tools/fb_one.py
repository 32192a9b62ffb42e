#!/usr/bin/env python3
"""One backward form repeated, for counter passes (developer tool, GPU):
    python3 tools/fb_one.py [head|nohead|tail] [fused|separate] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import nconv_pkg
    from test_gpu_fused_bwd import _run, _setup, _tail_run, _tail_setup
    m = nconv_pkg.load()
    which = sys.argv[1] if len(sys.argv) > 1 else "head"
    sep = (sys.argv[2] if len(sys.argv) > 2 else "fused") == "separate"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    if which == "tail":
        t = _tail_setup(m, dev, 8, 352, 1216, seed=1)
        fn = lambda: _tail_run(m, t, sep)
    else:
        t = _setup(m, dev, 8, 352, 1216, seed=1)
        fn = lambda: _run(m, t, separate=sep, head=which == "head")
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("done", which, "separate" if sep else "fused", flush=True)


if __name__ == "__main__":
    main()
