#!/usr/bin/env python3
"""nconv2's training backward at B=8 352x1216 (pooled-output gradient + fused nconv1 weight gradient),
one-kernel form (nconv_bwd_fused.hip) vs the two kernels (NCONV_BWD_SEPARATE; serial on one stream),
and the same for a down1-shaped layer (176x608, no head). Developer tool (GPU):
    python3 tools/fused_bwd_bench.py [reps] -> us per backward, each form"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import nconv_pkg
    from test_gpu_fused_bwd import _setup
    m = nconv_pkg.load()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    N = m.nconv
    for (B, H, W, head) in ((8, 352, 1216, True), (8, 352, 1216, False), (8, 176, 608, False), (8, 88, 304, False)):
        t = _setup(m, dev, B, H, W, seed=1)
        outs = dict(gxa=torch.empty_like(t["x1"]), gca=torch.empty_like(t["c1"]), gw=torch.empty_like(t["w2"]),
                    gb=torch.empty_like(t["b2"]), hgw=torch.empty_like(t["w1"]), hgb=torch.empty_like(t["b1"]))
        res = {}
        for sep in (True, False):
            kw = dict(pool_grad=t["pool"], separate=sep)
            if head:
                kw["head"] = (t["sp1"], t["S"], t["w1"], t["b1"], t["s1"], outs["hgw"], outs["hgb"])
            gin = (None, None, None, None) if head else (outs["gxa"], outs["gca"], None, None)

            def step():
                N.layer_backward(t["sp2"], (t["x1"], t["c1"], None, None, t["w2"], t["b2"], t["s2"]), t["y"],
                                 t["co"], t["gy"], t["gco"], gin, outs["gw"], outs["gb"], **kw)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                step()
            e1.record()
            e1.synchronize()
            res["separate" if sep else "fused"] = e0.elapsed_time(e1) / reps * 1e3
        print(f"B={B} {H}x{W} head={head}: two kernels {res['separate']:.1f} us, one kernel {res['fused']:.1f} us",
              flush=True)
    # nconv6 + nconv7 (the training tail)
    from test_gpu_fused_bwd import _tail_run, _tail_setup
    t = _tail_setup(m, dev, 8, 352, 1216, seed=1)
    res = {}
    for sep in (True, False):
        for _ in range(3):
            _tail_run(m, t, sep)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _tail_run(m, t, sep)
        e1.record()
        e1.synchronize()
        res["separate" if sep else "fused"] = e0.elapsed_time(e1) / reps * 1e3
    print(f"tail B=8 352x1216: two kernels {res['separate']:.1f} us, one kernel {res['fused']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
