#!/usr/bin/env python3
"""Why does the traced DNET (the reference's op sequence, export.py) deviate on device? (GPU tool)

    python3 tools/export_probe.py

1. The traced SETP1_NCONV graph of golden f2 (64x96) on cuda, against the reference's f2 output,
   under each convolution backend torch offers on ROCm: MIOpen (torch.backends.cudnn.enabled,
   the default), MIOpen with deterministic algorithms, and torch's native convolution
   (cudnn.enabled = False: im2col + rocBLAS fp32 GEMM).
2. Each DNET convolution shape on NConv-like inputs (sparse confidence, positive weights) under
   the same backends: max |conv_gpu - conv_fp64| / conv_fp64(|x|, |w|), the per-output error in
   units of the sum of the magnitudes of its terms (fp32 accumulation: ~1e-7; bf16 products ~4e-3,
   fp16 ~5e-4; Winograd-type transforms: unbounded relative to that sum when terms cancel).
Prints one line per measurement; run it once with MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 to
see the solver MIOpen picks per shape.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BACKENDS = {
    "miopen": dict(enabled=True, deterministic=False, benchmark=False),
    "miopen_det": dict(enabled=True, deterministic=True, benchmark=False),
    "native": dict(enabled=False, deterministic=False, benchmark=False),
}


def set_backend(name):
    cfg = BACKENDS[name]
    torch.backends.cudnn.enabled = cfg["enabled"]
    torch.backends.cudnn.deterministic = cfg["deterministic"]
    torch.backends.cudnn.benchmark = cfg["benchmark"]


def traced_f2(dev):
    import nconv_pkg
    m = nconv_pkg.load()
    f = np.load(os.path.join(ROOT, "tests", "golden", "f2_dnet.npz"), allow_pickle=False)
    net = m.SETP1_NCONV(crop="literal")
    own = net.state_dict()
    net.load_state_dict({k: torch.from_numpy(np.array(f[k])) for k in own if k in f.files}, strict=False)
    net = net.eval().to(dev)
    S = torch.from_numpy(np.array(f["S_64x96"])).to(dev)
    ref = torch.from_numpy(np.array(f["out_64x96"])).double()
    with torch.no_grad():
        hip = net(S)
        err = (hip.double().cpu() - ref).abs()
        print(f"hip forward vs f2: max abs {err.max():.3e}, max rel {(err / (ref.abs() + 1e-4)).max():.3e}")
        for name in BACKENDS:
            set_backend(name)
            traced = torch.jit.trace(net, (S,), check_trace=False)
            out = traced(S)
            torch.cuda.synchronize()
            err = (out.double().cpu() - ref).abs()
            print(f"traced [{name}] vs f2: max abs {err.max():.3e}, max rel {(err / (ref.abs() + 1e-4)).max():.3e}")


# (name, Cin, Cout, K, pad, H, W): DNET's convolutions at B=2 64x96 (step1.py:38-49)
SHAPES = [("nconv1", 1, 8, 5, 2, 64, 96), ("nconv2", 8, 8, 5, 2, 64, 96), ("down1", 8, 8, 5, 2, 32, 48),
          ("down3", 8, 8, 5, 2, 8, 12), ("nconv4", 16, 8, 3, 1, 16, 24), ("nconv6", 16, 8, 3, 0, 66, 98),
          ("nconv7", 8, 1, 1, 2, 64, 96)]


def conv_accuracy(dev):
    g = torch.Generator().manual_seed(0)
    for name, cin, cout, k, pad, H, W in SHAPES:
        c = (torch.rand(2, cin, H, W, generator=g) < 0.1).double() * torch.rand(2, cin, H, W, generator=g)
        x = torch.rand(2, cin, H, W, generator=g).double() * 80 * c
        w = torch.rand(cout, cin, k, k, generator=g).double() + 0.01
        ref = F.conv2d(x, w, padding=pad)
        mag = F.conv2d(x.abs(), w.abs(), padding=pad).clamp_min(1e-30)
        for bname in BACKENDS:
            set_backend(bname)
            with torch.no_grad():
                got = F.conv2d(x.float().to(dev), w.float().to(dev), padding=pad).double().cpu()
            e = ((got - ref).abs() / mag).max().item()
            print(f"conv {name} ({cin}->{cout} {k}x{k}) [{bname}]: max err / sum|terms| = {e:.3e}")


def main():
    dev = torch.device("cuda:0")
    print(f"torch {torch.__version__}, hip {torch.version.hip}, miopen {torch.backends.cudnn.version()}")
    traced_f2(dev)
    conv_accuracy(dev)
    set_backend("miopen")


if __name__ == "__main__":
    main()
