#!/usr/bin/env python3
"""CPU emulation (numpy, float64) of bwd_fused<GP, HW>'s work decomposition (csrc/nconv_bwd_fused.hip)
for nconv2 with the pooled-output gradient and the fused nconv1 weight gradient: the strip / segment
partition, the ring slots (reads assert the slot still holds the wanted row), the row-lagged input
gradient, the per-row nconv1 weight gradient over the S rows' sample lists, against torch autograd
of nconv1 -> nconv2 (+ 2x2 max-pools) in float64. Developer tool (decomposition, not concurrency).
    python3 tools/debug/emulate_fused_bwd.py"""
import numpy as np
import torch
import torch.nn.functional as F

TW, NSX, NSG, NSS = 64, 5, 5, 6


def nconv(x, c, w, b, pad, eps):
    D = F.conv2d(c, w, None, 1, pad)
    N = F.conv2d(x * c, w, None, 1, pad)
    s = w.sum(dim=(1, 2, 3))
    return N / (D + eps) + b.view(1, -1, 1, 1), D / s.view(1, -1, 1, 1)


def grad_nd(gy, gco, y, co, eps, b, s):
    D = co * s
    return gy / (D + eps), -(gy * (y - b)) / (D + eps) + gco / s


def main(B=2, H=14, W=70, seed=0, seg_rows=5, thresh=0.01):
    g = torch.Generator().manual_seed(seed)
    dt = torch.float64
    S = (torch.rand(B, 1, H, W, generator=g, dtype=dt) * 79 + 1) * (torch.rand(B, 1, H, W, generator=g, dtype=dt) < 0.2)
    W1 = torch.rand(8, 1, 5, 5, generator=g, dtype=dt) + 0.05
    b1 = torch.rand(8, generator=g, dtype=dt) * 0.1
    W2 = torch.rand(8, 8, 5, 5, generator=g, dtype=dt) + 0.05
    b2 = torch.rand(8, generator=g, dtype=dt) * 0.1
    e = 1e-20
    leaves = [t.clone().requires_grad_(True) for t in (W1, b1, W2, b2)]
    lW1, lb1, lW2, lb2 = leaves
    c0 = (S > thresh).double()
    y1, c1 = nconv(S, c0, lW1, lb1, 2, e)
    y2, c2 = nconv(y1, c1, lW2, lb2, 2, e)
    gy = torch.randn(y2.shape, generator=g, dtype=dt)
    gco = torch.randn(y2.shape, generator=g, dtype=dt)
    py, iy = F.max_pool2d(y2, 2, 2, return_indices=True)
    pc, ic = F.max_pool2d(c2, 2, 2, return_indices=True)
    gpy = torch.randn(py.shape, generator=g, dtype=dt)
    gpc = torch.randn(pc.shape, generator=g, dtype=dt)
    (gy * y2 + gco * c2).sum().__add__((gpy * py + gpc * pc).sum()).backward()
    ref = {k: t.grad.numpy() for k, t in zip(("gw1", "gb1", "gw2", "gb2"), leaves)}
    y1, c1, y2, c2 = (t.detach().numpy() for t in (y1, c1, y2, c2))
    S, W1, b1, W2, b2 = (t.numpy() for t in (S, W1, b1, W2, b2))
    gy, gco, gpy, gpc, iy, ic = (t.numpy() for t in (gy, gco, gpy, gpc, iy, ic))
    s1, s2 = W1.sum((1, 2, 3)), W2.sum((1, 2, 3))
    Hp, Wp = H // 2, W // 2
    out = {k: np.zeros_like(v) for k, v in ref.items()}
    nstrip = (W + TW - 1) // TW
    nseg = (H + seg_rows - 1) // seg_rows
    for b in range(B):
        for st in range(nstrip):
            for sg in range(nseg):
                cs, r0 = st * TW, sg * seg_rows
                r1 = min(H, r0 + seg_rows)
                X, G, SL = [None] * NSX, [None] * NSG, [None] * NSS

                def xrow(ih):
                    xc, cc = np.zeros((8, TW)), np.zeros((8, TW))
                    for j in range(TW):
                        if 0 <= ih < H and cs + j < W:
                            xc[:, j] = y1[b, :, ih, cs + j] * c1[b, :, ih, cs + j]
                            cc[:, j] = c1[b, :, ih, cs + j]
                    X[ih % NSX] = (ih, xc, cc)

                def grow(oh, count):
                    gn, gd = np.zeros((8, TW + 4)), np.zeros((8, TW + 4))
                    for m in range(TW + 4):
                        ow = cs - 2 + m
                        if not (0 <= oh < H and 0 <= ow < W):
                            continue
                        for o in range(8):
                            gyv, gcv = gy[b, o, oh, ow], gco[b, o, oh, ow]
                            if oh // 2 < Hp and ow // 2 < Wp:  # pool routing at the window's first maximum
                                flat = oh * W + ow
                                if iy[b, o, oh // 2, ow // 2] == flat:
                                    gyv += gpy[b, o, oh // 2, ow // 2]
                                if ic[b, o, oh // 2, ow // 2] == flat:
                                    gcv += gpc[b, o, oh // 2, ow // 2]
                            gn[o, m], gd[o, m] = grad_nd(gyv, gcv, y2[b, o, oh, ow], c2[b, o, oh, ow], e, b2[o], s2[o])
                            if count and 2 <= m < TW + 2:
                                out["gb2"][o] += gyv
                                out["gw2"][o] += -(gcv * c2[b, o, oh, ow]) / s2[o]
                    G[oh % NSG] = (oh, gn, gd)

                def srow(r):
                    lst = []
                    for m in range(TW + 4):
                        col = cs - 2 + m
                        if 0 <= r < H and 0 <= col < W and S[b, 0, r, col] > thresh:
                            lst.append((m, S[b, 0, r, col]))
                    SL[r % NSS] = (r, lst)

                def get(ring, n, r):
                    v = ring[r % n]
                    assert v[0] == r, (v[0], r)
                    return v[1:]

                for r in range(r0 - 2, r0 + 2):
                    xrow(r)
                for r in range(r0 - 2, r0):
                    grow(r, False)
                    srow(r)
                for s in range(r0, r1 + 2):
                    xrow(s + 2)
                    grow(s, s < r1)
                    srow(s)
                    if s < r1:  # weight gradient of output row s
                        gn, gd = get(G, NSG, s)
                        for kh in range(5):
                            xc, cc = get(X, NSX, s - 2 + kh)
                            for kw in range(5):
                                for j in range(TW):
                                    m = j + 4 - kw
                                    out["gw2"][:, :, kh, kw] += np.outer(gn[:, m], xc[:, j]) + np.outer(gd[:, m], cc[:, j])
                    if s >= r0 + 2:  # input gradient of row ih = s - 2 -> nconv1's weight gradient
                        ih = s - 2
                        Gi = np.zeros((8, 2, TW))
                        for kh in range(5):
                            gn, gd = get(G, NSG, s - kh)
                            for kw in range(5):
                                for j in range(TW):
                                    m = j + 4 - kw
                                    Gi[:, 0, j] += W2[:, :, kh, kw].T @ gn[:, m]
                                    Gi[:, 1, j] += W2[:, :, kh, kw].T @ gd[:, m]
                        hn = np.zeros((8, 2, TW))
                        for j in range(TW):
                            iw = cs + j
                            if iw >= W:
                                continue
                            for i in range(8):
                                x, c = y1[b, i, ih, iw], c1[b, i, ih, iw]
                                g1, gc1 = Gi[i, 0, j] * c, Gi[i, 1, j] + Gi[i, 0, j] * x
                                hn[i, 0, j], hn[i, 1, j] = grad_nd(g1, gc1, x, c, e, b1[i], s1[i])
                                out["gb1"][i] += g1
                                out["gw1"][i] += -(gc1 * c) / s1[i]
                        for o1 in range(8):
                            for kh in range(5):
                                (lst,) = get(SL, NSS, ih + kh - 2)
                                for kw in range(5):
                                    for m, v in lst:
                                        jj = m - kw
                                        if 0 <= jj < TW:
                                            out["gw1"][o1, 0, kh, kw] += hn[o1, 0, jj] * v + hn[o1, 1, jj]
    for k, v in ref.items():
        err = np.abs(out[k] - v).max() / max(np.abs(v).max(), 1e-30)
        print(f"{k}: normwise {err:.2e}")
        assert err < 1e-9, k


if __name__ == "__main__":
    main()
    main(B=1, H=9, W=130, seed=1, seg_rows=3)
    main(B=1, H=20, W=64, seed=2, seg_rows=7)
    print("ok")
