#!/usr/bin/env python3
"""One NConv layer forward, repeated (developer tool for rocprofv3 / counter passes, GPU):
python3 tools/fwd_layer_bench.py [nconv1|nconv2|head|tail|down1|down2|down3|nconv4|nconv5] [reps] -> us per launch."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import nconv_pkg
    m = nconv_pkg.load()
    which = sys.argv[1] if len(sys.argv) > 1 else "nconv2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, H, W = 8, 352, 1216
    r = lambda *s: torch.rand(*s, device=dev, generator=g)
    w8 = r(8, 8, 5, 5) + 0.05
    w16 = r(8, 16, 3, 3) + 0.05
    b = r(8) * 0.1
    s8 = w8.sum((1, 2, 3)).contiguous()
    s16 = w16.sum((1, 2, 3)).contiguous()
    N = m.nconv
    if which == "nconv2":
        x, c = r(B, 8, H, W) * 10, r(B, 8, H, W)
        spec = m.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
        fn = lambda: N.layer_forward_pooled(spec, x, c, None, None, w8, b, s8)
    elif which == "nconv1":  # exact-fp32 nconv1 on the thresholded sparse depth
        S = (r(B, 1, H, W) * 79 + 1) * (r(B, 1, H, W) < 0.05)
        w1 = r(8, 1, 5, 5) + 0.05
        s1 = w1.sum((1, 2, 3)).contiguous()
        spec = m.LayerSpec(1, 8, (5, 5), (1, 1), (2, 2), mode=m._lib.THRESH)
        fn = lambda: N.layer_forward_raw(spec, S, None, None, None, w1, b, s1)
    elif which == "head":  # nconv1 inside nconv2 (nconv_fwd_head); NCONV_DENSITY: depth density (0.05)
        S = (r(B, 1, H, W) * 79 + 1) * (r(B, 1, H, W) < float(os.environ.get("NCONV_DENSITY", "0.05")))
        w1 = r(8, 1, 5, 5) + 0.05
        s1 = w1.sum((1, 2, 3)).contiguous()
        sp1 = m.LayerSpec(1, 8, (5, 5), (1, 1), (2, 2), mode=m._lib.THRESH)
        spec = m.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
        w21 = N.head_weights(sp1, spec, S, w1, b, s1, w8, b, s8) if N.FORWARD_MATH == m._lib.MATH_FP32 else None
        fn = lambda: N.layer_forward_head(sp1, spec, S, w1, b, s1, w8, b, s8, w21)
    elif which in ("down1", "down2", "down3"):
        f = {"down1": 2, "down2": 4, "down3": 8}[which]
        x, c = r(B, 8, H // f, W // f) * 10, r(B, 8, H // f, W // f)
        spec = m.LayerSpec(8, 8, (5, 5), (1, 1), (2, 2))
        fn = lambda: N.layer_forward_pooled(spec, x, c, None, None, w8, b, s8)
    elif which in ("nconv5", "nconv4"):
        f = 2 if which == "nconv5" else 4
        xa, ca = r(B, 8, H // f, W // f) * 10, r(B, 8, H // f, W // f)
        xb, cb = r(B, 8, H // (2 * f), W // (2 * f)) * 10, r(B, 8, H // (2 * f), W // (2 * f))
        spec = m.LayerSpec(16, 8, (3, 3), (1, 1), (1, 1), mode=m._lib.UPCAT_SKIP_FIRST)
        wph = None
        if os.environ.get("NCONV_PHASE", "1") == "1":
            wph = torch.empty(1024, device=dev)
            N.phase_weights([w16], [8], [wph])
        fn = lambda: N.layer_forward_raw(spec, xa, ca, xb, cb, w16, b, s16, wphase=wph)
    else:  # nconv6 + nconv7 tail
        net = m.DNET(32, crop="generalized").to(dev).eval()
        xa, ca = r(B, 8, H, W) * 10, r(B, 8, H, W)
        xb, cb = r(B, 8, H // 2, W // 2) * 10, r(B, 8, H // 2, W // 2)
        out = torch.empty(B, 1, H, W, device=dev)
        s6 = net.nconv6.weight.sum((1, 2, 3)).contiguous()
        s7 = net.nconv7.weight.sum((1, 2, 3)).contiguous()
        net.phase_upcat = os.environ.get("NCONV_PHASE", "1") == "1"
        wph = net._phase_weights(dev)
        fn = lambda: net._fused_tail(net.nconv6, net.nconv7, s6, s7, xa, ca, xb, cb, out, None if wph is None else wph[2])
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    print(f"{which}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per launch", flush=True)


if __name__ == "__main__":
    main()
