#!/usr/bin/env python3
"""CPU emulation (numpy, float64) of bwd_fused_tail's work decomposition (csrc/nconv_bwd_fused.hip):
the strip / segment partition, the ring slots (every read asserts the slot still holds the row it
wants) and the index math of the weight gradient, the skip-channel input gradient and the box-weight
low-resolution gradient, against torch autograd of nconv6 + nconv7 in float64. Developer tool; it
checks the decomposition, not the kernel's concurrency.
    python3 tools/debug/emulate_fused_tail.py"""
import numpy as np
import torch
import torch.nn.functional as F

TW, NSX, NSG = 64, 3, 4


def nconv(x, c, w, b, pad, eps):
    D = F.conv2d(c, w, None, 1, pad)
    N = F.conv2d(x * c, w, None, 1, pad)
    s = w.sum(dim=(1, 2, 3))
    return N / (D + eps) + b.view(1, -1, 1, 1), D / s.view(1, -1, 1, 1)


def grad_nd(gy, gco, y, co, eps, b, s):
    D = co * s
    r = y - b
    return gy / (D + eps), -(gy * r) / (D + eps) + gco / s


def main(B=2, H=12, W=70, seed=0, seg_rows=4):
    g = torch.Generator().manual_seed(seed)
    dt = torch.float64
    x2, c2 = torch.rand(B, 8, H, W, generator=g, dtype=dt) * 5, torch.rand(B, 8, H, W, generator=g, dtype=dt)
    x7, c7 = torch.rand(B, 8, H // 2, W // 2, generator=g, dtype=dt) * 5, torch.rand(B, 8, H // 2, W // 2, generator=g, dtype=dt)
    W6 = torch.rand(8, 16, 3, 3, generator=g, dtype=dt) + 0.05
    b6 = torch.rand(8, generator=g, dtype=dt) * 0.1
    w7 = torch.rand(1, 8, 1, 1, generator=g, dtype=dt) + 0.05
    b7 = torch.rand(1, generator=g, dtype=dt) * 0.1
    e6, e7 = 1e-20, 1e-20
    leaves = [t.clone().requires_grad_(True) for t in (x2, c2, x7, c7, W6, b6, w7)]
    lx2, lc2, lx7, lc7, lW6, lb6, lw7 = leaves
    up = lambda t: F.interpolate(t, scale_factor=2, mode="nearest")
    y8, c8 = nconv(torch.cat((up(lx7), lx2), 1), torch.cat((up(lc7), lc2), 1), lW6, lb6, 0, e6)
    y9, c9 = nconv(y8, c8, lw7, b7, 2, e7)
    g9 = torch.randn(y9.shape, generator=g, dtype=dt)
    (y9 * g9).sum().backward()
    ref = {k: t.grad.numpy() for k, t in zip(("gx2", "gc2", "gx7", "gc7", "gw", "gb", "gw7"), leaves)}
    y8, c8, y9, c9 = (t.detach().numpy() for t in (y8, c8, y9, c9))
    x2, c2, x7, c7, W6, b6, w7, b7, g9 = (t.numpy() for t in (x2, c2, x7, c7, W6, b6, w7, b7, g9))
    s6, s7 = W6.sum((1, 2, 3)), w7.sum()
    Ho, Wo, Hl, Wl = H - 2, W - 2, H // 2, W // 2
    wb = np.zeros((8, 8, 4, 4))
    S = {0: [2], 1: [1, 2], 2: [0, 1], 3: [0]}
    for t in range(4):
        for u in range(4):
            wb[:, :, t, u] = sum(W6[:, :8, kh, kw] for kh in S[t] for kw in S[u])
    out = {k: np.zeros_like(v) for k, v in ref.items()}
    nstrip = (W + TW - 1) // TW
    seg_rows += seg_rows & 1
    nseg = (H + seg_rows - 1) // seg_rows
    for b in range(B):
        for st in range(nstrip):
            for sg in range(nseg):
                c0, r0 = st * TW, sg * seg_rows
                r1 = min(H, r0 + seg_rows)
                X = [None] * NSX
                G = [None] * NSG

                def xrow(ih):
                    xc, cc = np.zeros((16, TW)), np.zeros((16, TW))
                    for j in range(TW):
                        iw = c0 + j
                        if 0 <= ih < H and iw < W:
                            xu, cu = x7[b, :, ih // 2, iw // 2], c7[b, :, ih // 2, iw // 2]
                            xc[:8, j], cc[:8, j] = xu * cu, cu
                            xc[8:, j], cc[8:, j] = x2[b, :, ih, iw] * c2[b, :, ih, iw], c2[b, :, ih, iw]
                    X[ih % NSX] = (ih, xc, cc)

                def grow(oh, count):
                    gn, gd = np.zeros((8, TW + 2)), np.zeros((8, TW + 2))
                    for m in range(TW + 2):
                        ow = c0 - 2 + m
                        if not (0 <= oh < Ho and 0 <= ow < Wo):
                            continue
                        n7, d7 = grad_nd(g9[b, 0, oh + 2, ow + 2], 0.0, y9[b, 0, oh + 2, ow + 2], c9[b, 0, oh + 2, ow + 2],
                                         e7, b7[0], s7)
                        for o in range(8):
                            gxc, gcc = w7[0, o, 0, 0] * n7, w7[0, o, 0, 0] * d7
                            gy, gco = gxc * c8[b, o, oh, ow], gcc + gxc * y8[b, o, oh, ow]
                            gn[o, m], gd[o, m] = grad_nd(gy, gco, y8[b, o, oh, ow], c8[b, o, oh, ow], e6, b6[o], s6[o])
                            if count and m >= 2:
                                out["gb"][o] += gy
                                out["gw"][o] += -(gco * c8[b, o, oh, ow]) / s6[o]  # (finish: -sum gco*cout / s)
                                out["gw7"][0, o, 0, 0] += y8[b, o, oh, ow] * c8[b, o, oh, ow] * n7 + c8[b, o, oh, ow] * d7
                    G[oh % NSG] = (oh, gn, gd)

                def xget(ih):
                    r, xc, cc = X[ih % NSX]
                    assert r == ih, (r, ih)
                    return xc, cc

                def gget(oh):
                    r, gn, gd = G[oh % NSG]
                    assert r == oh, (r, oh)
                    return gn, gd

                for r in range(r0, r0 + 2):
                    xrow(r)
                for r in range(r0 - 2, r0):
                    grow(r, False)
                for s in range(r0, r1):
                    xrow(s + 2)
                    grow(s, True)
                    if s < Ho:  # weight gradient of output row s
                        gn, gd = gget(s)
                        for kh in range(3):
                            xc, cc = xget(s + kh)
                            for kw in range(3):
                                for j in range(TW):
                                    m = j + 2 - kw
                                    out["gw"][:, :, kh, kw] += np.outer(gn[:, m], xc[:, j]) + np.outer(gd[:, m], cc[:, j])
                    Gs = np.zeros((8, 2, TW))  # skip channels' input gradient of row s
                    for kh in range(3):
                        gn, gd = gget(s - kh)
                        for kw in range(3):
                            for j in range(TW):
                                m = j + 2 - kw
                                Gs[:, 0, j] += W6[:, 8:, kh, kw].T @ gn[:, m]
                                Gs[:, 1, j] += W6[:, 8:, kh, kw].T @ gd[:, m]
                    for j in range(TW):
                        iw = c0 + j
                        if iw < W:
                            out["gx2"][b, :, s, iw] = Gs[:, 0, j] * c2[b, :, s, iw]
                            out["gc2"][b, :, s, iw] = Gs[:, 1, j] + Gs[:, 0, j] * x2[b, :, s, iw]
                    if s & 1:  # low row p: g rows s-3 .. s
                        p = (s - 1) // 2
                        for q in range(TW // 2):
                            ql = c0 // 2 + q
                            if ql >= Wl:
                                continue
                            Gl = np.zeros((8, 2))
                            for t in range(4):
                                gn, gd = gget(s - 3 + t)
                                for u in range(4):
                                    m = 2 * q + u
                                    Gl[:, 0] += wb[:, :, t, u].T @ gn[:, m]
                                    Gl[:, 1] += wb[:, :, t, u].T @ gd[:, m]
                            out["gx7"][b, :, p, ql] = Gl[:, 0] * c7[b, :, p, ql]
                            out["gc7"][b, :, p, ql] = Gl[:, 1] + Gl[:, 0] * x7[b, :, p, ql]
    # (the emulation adds the normaliser term -sum gco*cout/s[o] to every weight of output channel o)
    for k, v in ref.items():
        got = out[k]
        err = np.abs(got - v).max() / max(np.abs(v).max(), 1e-30)
        print(f"{k}: normwise {err:.2e}")
        assert err < 1e-9, k


if __name__ == "__main__":
    main()
    main(B=1, H=8, W=130, seed=1, seg_rows=2)
    main(B=1, H=16, W=64, seed=2, seg_rows=6)
    print("ok")
