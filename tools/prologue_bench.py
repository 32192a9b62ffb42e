#!/usr/bin/env python3
"""The training weight prologue (nconv_train_prologue) by role, against the separate launches it
replaces (developer tool, GPU): python3 tools/prologue_bench.py [reps] -> us per launch."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    for _ in range(3):
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
    N = m.nconv
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = m.SETP1_NCONV(crop="generalized").to(dev)
    layers = [getattr(net.d_net, n) for n in m.dnet.LAYERS]
    ws = [l.weight.detach() for l in layers]
    s = [torch.empty(w.shape[0], device=dev) for w in ws]
    w21 = torch.empty(N.HEAD_WEIGHTS_FLOATS, device=dev)
    ph = [torch.empty(1024, device=dev) for _ in range(3)]
    bx = [torch.empty(1024, device=dev) for _ in range(3)]
    nosp = [False] * 9  # (no softplus: repeated calls keep the weights)
    sp = [True] * 9
    cases = {
        "all roles": lambda: N.train_prologue(ws, nosp, s, head=(0, 1, w21, N.sync_counter(dev)), phase=([5, 6, 7], [8, 8, 0], ph, bx)),
        "all roles, softplus": None,
        "prep only (9 layers)": lambda: N.train_prologue(ws, nosp, s),
        "head only": lambda: N.train_prologue(ws[:2], nosp[:2], s[:2], head=(0, 1, w21, N.sync_counter(dev))),
        "phase only": lambda: N.train_prologue(ws[5:8], nosp[:3], s[5:8], phase=([0, 1, 2], [8, 8, 0], ph, bx)),
        "eval weight_prologue": lambda: N.weight_prologue(ws, s, head=(ws[0], ws[1], w21),
                                                          phase=([ws[5], ws[6], ws[7]], [8, 8, 0], ph)),
        "weight_prep (9)": lambda: N.weight_prep(ws, nosp, s),
        "head_weights": lambda: N.head_weights(layers[0].spec(m._lib.THRESH, 0.01), layers[1].spec(),
                                               torch.zeros(1, 1, 32, 32, device=dev), ws[0], layers[0].bias, s[0],
                                               ws[1], layers[1].bias, s[1], out=w21),
        "phase_weights": lambda: N.phase_weights([ws[5], ws[6], ws[7]], [8, 8, 0], ph),
    }
    wcopy = [w.clone() for w in ws]

    def with_sp():  # (softplus on copies reset each call: the copy kernels are timed too)
        for a, b in zip(wcopy, ws):
            a.copy_(b)
        N.train_prologue(wcopy, sp, s, head=(0, 1, w21, N.sync_counter(dev)), phase=([5, 6, 7], [8, 8, 0], ph, bx))
    cases["all roles, softplus"] = with_sp
    cases["(the 9 copies alone)"] = lambda: [a.copy_(b) for a, b in zip(wcopy, ws)]
    for k, fn in cases.items():
        print(f"{k}: {timed(fn, reps):.1f} us", flush=True)


if __name__ == "__main__":
    main()
