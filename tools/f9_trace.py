#!/usr/bin/env python3
"""Golden f9's training iteration on the GPU with the gradient of every decoder intermediate kept
(upf's convolution output and its BN-ReLU output, UpCat's output, each ConvBlock's output, each
scale's (features, depth)), against the same intermediates of the float64 oracle: where along the
backward chain the fp32 gradient first departs from float64 (developer tool, GPU)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def main():
    import torch.nn.functional as F
    import nconv_pkg
    from oracle import nconv_ref as R
    from guided_cases import f5_models, f9_inputs, trainable_setp2
    m = nconv_pkg.load()
    G, D = m.guided, m.dense
    dev = torch.device("cuda:0")
    ours, ref = {}, {}

    def keep(store, name, t):
        if t.requires_grad:
            t.retain_grad()
        store[name] = t
        return t

    model = f5_models(m).to(dev)
    names = {id(mod): n for n, mod in model.named_modules()}

    def trans_fwd(self, x0, x1=None):
        n = names[id(self)]
        y = keep(ours, n + ".conv", D.conv_fn(x0, self.conv.weight, self.conv.bias, D.DENSE_TRANSPOSED_4X4, 2, x1=x1))
        return keep(ours, n, G._bn_act(y, self.bn, self.relu))

    def basic_fwd(self, x0, x1=None):
        conv, bn, act = self.conv.conv, self.conv.bn, self.conv.relu
        n = names[id(self)]
        y = keep(ours, n + ".conv", D.conv_fn(x0, conv.weight, conv.bias, D.DENSE_3X3, conv.stride[0], relu=False, x1=x1))
        return keep(ours, n, G._bn_act(y, bn, act))

    cb_orig = G.ConvBlock.train_forward

    def cb_fwd(self, x0, x1=None):
        return keep(ours, names[id(self)], cb_orig(self, x0, x1))

    fr_orig, f0_orig = G.FusionResolutionBlock.train_forward, G.FusionResolution0.train_forward

    def fr_fwd(self, *a):
        f, d = fr_orig(self, *a)
        n = names[id(self)]
        return keep(ours, n + ".f", f), keep(ours, n + ".d", d)

    def f0_fwd(self, *a):
        f, d = f0_orig(self, *a)
        n = names[id(self)]
        return keep(ours, n + ".f", f), keep(ours, n + ".d", d)

    def enc_fwd(self, x):
        conv, bn, act, sc = self.encoder[0], self.encoder[1], self.encoder[2], self.downsample[0]
        y = keep(ours, names[id(self)] + ".enc",
                 G._bn_act(D.conv_fn(x, conv.weight, conv.bias, D.DENSE_3X3, conv.stride[0]), bn, act))
        return y + D.conv_fn(x, sc.weight, None, D.DENSE_1X1, sc.stride[0])

    G.RGBEncoder.train_forward = enc_fwd
    G.Basic2dTrans.train_forward = trans_fwd
    G.Basic2d.train_forward = basic_fwd
    G.ConvBlock.train_forward = cb_fwd
    G.FusionResolutionBlock.train_forward = fr_fwd
    G.FusionResolution0.train_forward = f0_fwd

    sd0 = {k: v.detach().double().cpu().clone() for k, v in model.state_dict().items()}
    rgb, depth, gt = f9_inputs()
    model.train()
    est, _ = model(rgb.to(dev), depth.to(dev), rgb.to(dev), depth.to(dev))
    loss = m.train.calculate_loss_multi_resolution(est, gt.to(dev), False)
    loss.backward()
    torch.cuda.synchronize()

    # the float64 oracle with the same intermediates kept
    def o_convblock(x, sd, p):
        return keep(ref, p[:-1], F.relu(F.conv2d(x, sd[p + "conv.weight"], sd[p + "conv.bias"], 1, 1)))

    def o_upcat(y, x, d, sd, p, training, momentum=0.0):
        keep(ref, p + "upf.in", torch.cat([x, d], 1))
        u = keep(ref, p + "upf.conv", F.conv_transpose2d(torch.cat([x, d], 1), sd[p + "upf.conv.weight"], None, 2, 1))
        u = keep(ref, p + "upf", F.relu(R._bn(u, sd, p + "upf.bn.", training, momentum)))
        u = keep(ref, p + "conv.conv", F.conv2d(torch.cat([u, y], 1), sd[p + "conv.conv.conv.weight"], None, 1, 1))
        return keep(ref, p + "conv", F.relu(R._bn(u, sd, p + "conv.conv.bn.", training, momentum)))
    nf_orig = R._new_fusion

    def o_new_fusion(rgb_, depth_, sd, p):
        return keep(ref, p[:-len("fuse.")] + "f", nf_orig(rgb_, depth_, sd, p))
    R._convblock, R._upcat, R._new_fusion = o_convblock, o_upcat, o_new_fusion
    sd = dict(sd0)
    p1 = R.dnet_params_from_state_dict({k: (R.softplus_pos(v) if k.endswith(".weight") and "bnorm" not in k else v)
                                        for k, v in sd.items()}, "step1.d_net.")
    named = dict(model.named_parameters())
    pn = trainable_setp2(None, named.items())
    leaves = {k: sd[k].clone().requires_grad_(True) for k in pn}
    sd.update(leaves)
    o0, _ = R.setp2_forward(sd, rgb.double(), depth.double(), rgb.double(), depth.double(), "literal", "train",
                            training=True, step1_params=p1)
    R.calculate_loss_multi_resolution(o0, gt.double(), False).backward()

    order = ["fuse3.f", "fuse3.fuse.fuse_conv3", "fuse3.fuse.rgb_conv", "fuse3.upcat.conv", "fuse3.upcat.upf",
             "fuse2.f", "fuse2.fuse.fuse_conv3", "fuse2.fuse.fuse_conv2", "fuse2.fuse.fuse_conv1",
             "fuse2.fuse.rgb_conv", "fuse2.fuse.depth_conv", "fuse2.upcat.conv", "fuse2.upcat.conv.conv",
             "fuse2.upcat.upf", "fuse2.upcat.upf.conv",
             "fuse1.f", "fuse1.fuse.fuse_conv3", "fuse1.fuse.fuse_conv2", "fuse1.fuse.fuse_conv1",
             "fuse1.fuse.rgb_conv", "fuse1.fuse.depth_conv", "fuse1.upcat.conv", "fuse1.upcat.conv.conv",
             "fuse1.upcat.upf", "fuse1.upcat.upf.conv", "fuse0.f", "fuse0.fuse.fuse_conv3", "fuse0.fuse.rgb_conv"]
    print(f"{'tensor':34s} {'shape':>22s} {'fwd rel':>9s} {'grad rel':>9s} {'grad L1':>9s} {'max|g64|':>10s}")
    for k in order:
        a, b = ours.get(k), ref.get(k)
        if a is None or b is None:
            print(f"{k:34s} missing ours={a is not None} ref={b is not None}")
            continue
        ga, gb = a.grad, b.grad
        gr = rel(ga, gb) if ga is not None and gb is not None else float("nan")
        l1 = ((ga.double().cpu() - gb).abs().sum() / gb.abs().sum()).item() if ga is not None and gb is not None else float("nan")
        print(f"{k:34s} {str(tuple(a.shape)):>22s} {rel(a, b):9.2e} {gr:9.2e} {l1:9.2e} "
              f"{(gb.abs().max().item() if gb is not None else 0):10.3e}", flush=True)
    # one ConvBlock backward (ReLU mask + input gradient) in float64 from OUR fp32 tensors: the
    # dgrad kernel's own error, and the ReLU mask flips against the oracle's forward
    for lvl in ("fuse0", "fuse1", "fuse2"):
        out = ours[lvl + ".fuse.fuse_conv3"]
        go = out.grad.double().cpu()
        xin = ours[lvl + ".fuse.fuse_conv2"]
        conv = dict(model.named_modules())[lvl + ".fuse.fuse_conv3"].conv
        xi = xin.detach().double().cpu().requires_grad_(True)
        F.conv2d(xi, conv.weight.detach().double().cpu(), None, 1, 1).backward(go * (out.detach().cpu() > 0))
        gk = xin.grad.double().cpu()
        refo = ref[lvl + ".fuse.fuse_conv3"].detach()
        flips = ((out.detach().cpu() > 0) != (refo > 0)).sum().item()
        print(f"{lvl} fuse_conv3 backward: kernel vs fp64-of-our-tensors L1 "
              f"{((gk - xi.grad).abs().sum() / xi.grad.abs().sum()).item():.2e} max "
              f"{((gk - xi.grad).abs().max() / xi.grad.abs().max()).item():.2e}; ReLU flips vs oracle {flips} of "
              f"{out.numel()}; exact zeros ours {(out.detach() == 0).sum().item()} oracle {(refo == 0).sum().item()}")
    # fuse1's ConvTranspose weight gradient recomputed in float64 from OUR fp32 inputs (cat(d0, f0)
    # and dL/dy): kernel error (ours vs this) against input error (this vs the oracle's)
    for lvl, prev in (("fuse1", "fuse0"), ("fuse2", "fuse1"), ("fuse3", "fuse2")):
        x = torch.cat([ours[prev + ".d"], ours[prev + ".f"]], 1).detach().double().cpu()
        gy = ours[lvl + ".upcat.upf.conv"].grad.double().cpu()
        w = named[lvl + ".upcat.upf.conv.weight"].detach().double().cpu().requires_grad_(True)
        F.conv_transpose2d(x, w, None, 2, 1).backward(gy)
        gk = named[lvl + ".upcat.upf.conv.weight"].grad.double().cpu()
        g64 = leaves[lvl + ".upcat.upf.conv.weight"].grad
        s = g64.abs().max()
        print(f"{lvl} upf wgrad: kernel vs fp64-of-our-inputs {((gk - w.grad).abs().max() / s).item():.2e} "
              f"(row 0 {((gk[0] - w.grad[0]).abs().max() / s).item():.2e}); fp64-of-our-inputs vs oracle "
              f"{((w.grad - g64).abs().max() / s).item():.2e} (row 0 {((w.grad[0] - g64[0]).abs().max() / s).item():.2e})")
        # the forward's rounding on the same fp32 inputs: ours, torch CPU fp32, against float64
        u64 = F.conv_transpose2d(x, w.detach(), None, 2, 1)
        u32 = F.conv_transpose2d(x.float(), w.detach().float(), None, 2, 1).double()
        uo = ours[lvl + ".upcat.upf.conv"].detach().double().cpu()
        cen = u64 - u64.mean(dim=(0, 2, 3), keepdim=True)
        sc = cen.abs().amax(dim=(0, 2, 3), keepdim=True)  # per channel, about the batch mean (BN's view)
        print(f"  upf forward error / max|u - mean|: ours {((uo - u64).abs() / sc).max().item():.2e} (mean "
              f"{((uo - u64).abs() / sc).mean().item():.2e}), torch cpu fp32 {((u32 - u64).abs() / sc).max().item():.2e} "
              f"(mean {((u32 - u64).abs() / sc).mean().item():.2e})")
        gyr = ref[lvl + ".upcat.upf.conv"].grad
        xr = ref[lvl + ".upcat.upf.in"].detach()
        for tag, xx, yy in (("our x, oracle dy", x, gyr), ("oracle x, our dy", xr, gy)):
            w2 = w.detach().clone().requires_grad_(True)
            F.conv_transpose2d(xx, w2, None, 2, 1).backward(yy)
            print(f"  fp64 wgrad from {tag}: vs oracle {((w2.grad - g64).abs().max() / s).item():.2e}")
        print(f"  dL/dy channel sums: ours max|sum| {gy.sum(dim=(0, 2, 3)).abs().max().item():.3e}, oracle "
              f"{gyr.sum(dim=(0, 2, 3)).abs().max().item():.3e}; max|dy| {gyr.abs().max().item():.3e}; "
              f"sum|dy - dy64| {(gy - gyr).abs().sum().item():.3e}")
    # the float64 oracle once more with every ReLU taking OUR forward's mask (y * mask instead of
    # relu(y)): what is left of the gradient error once the fp32-unresolvable ReLU decisions match
    def mask(name):
        return (ours[name].detach().cpu() > 0).double()

    def m_convblock(x, sd, p):
        return F.conv2d(x, sd[p + "conv.weight"], sd[p + "conv.bias"], 1, 1) * mask(p[:-1])

    def m_upcat(y, x, d, sd, p, training, momentum=0.0):
        u = F.conv_transpose2d(torch.cat([x, d], 1), sd[p + "upf.conv.weight"], None, 2, 1)
        u = R._bn(u, sd, p + "upf.bn.", training, momentum) * mask(p + "upf")
        u = F.conv2d(torch.cat([u, y], 1), sd[p + "conv.conv.conv.weight"], None, 1, 1)
        return R._bn(u, sd, p + "conv.conv.bn.", training, momentum) * mask(p + "conv")

    def m_rgb_encoder(x, sd, p, stride, training=False, momentum=0.0):
        y = F.conv2d(x, sd[p + "encoder.0.weight"], sd[p + "encoder.0.bias"], stride, 1)
        y = R._bn(y, sd, p + "encoder.1.", training, momentum) * mask(p[:-1] + ".enc")
        return y + F.conv2d(x, sd[p + "downsample.0.weight"], None, stride)
    R._convblock, R._upcat, R._new_fusion, R.rgb_encoder = m_convblock, m_upcat, nf_orig, m_rgb_encoder
    sd = {k: v.clone() for k, v in sd0.items()}
    leaves_m = {k: sd[k].clone().requires_grad_(True) for k in pn}
    sd.update(leaves_m)
    o0, _ = R.setp2_forward(sd, rgb.double(), depth.double(), rgb.double(), depth.double(), "literal", "train",
                            training=True, step1_params=p1)
    R.calculate_loss_multi_resolution(o0, gt.double(), False).backward()
    worst = []
    for k in pn:
        g = named[k].grad.double().cpu()
        s64 = leaves[k].grad.abs().max().clamp_min(1e-30)
        worst.append((((g - leaves[k].grad).abs().max() / s64).item(),
                      ((g - leaves_m[k].grad).abs().max() / leaves_m[k].grad.abs().max().clamp_min(1e-30)).item(), k))
    worst.sort(reverse=True)
    print("gradient vs float64 oracle / vs the mask-matched float64 oracle (worst 15):")
    for a, b, k in worst[:15]:
        print(f"  {k:40s} {a:.2e}  {b:.2e}")
    print("max over tensors, mask-matched:", max(b for _, b, _ in worst))
    for k in ("fuse1.upcat.upf.conv.weight", "fuse1.upcat.upf.bn.bias", "fuse1.upcat.conv.conv.conv.weight"):
        g, g64 = named[k].grad.double().cpu(), leaves[k].grad
        e = (g - g64).abs()
        print(k, "rel", rel(g, g64), "argmax", [int(i) for i in torch.nonzero(e == e.max())[0]],
              "max|g64|", g64.abs().max().item())
        if g.dim() == 4:  # per input-channel row of the weight gradient (dim 0 for a ConvTranspose)
            per = (e.amax(dim=(1, 2, 3)) / g64.abs().max()).tolist()
            print("  per dim-0 row:", " ".join(f"{v:.1e}" for v in per[:8]), "...", f"max {max(per):.2e}")


if __name__ == "__main__":
    main()
