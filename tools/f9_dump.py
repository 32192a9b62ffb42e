#!/usr/bin/env python3
"""Golden f9's training iteration on the GPU, twice -- libnconv's dense kernels, and the plain torch
modules on the device (model.dense_kernels = False: MIOpen convolutions, torch BatchNorm) -- (and with cudnn disabled: torch's native im2col + GEMM convolutions) with
every trainable gradient saved to gpurun_out/f9_grads.pt for an offline comparison against the
reference (f9) and the float64 oracle (developer tool, GPU)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import nconv_pkg
    from guided_cases import f5_models, f9_inputs
    m = nconv_pkg.load()
    dev = torch.device("cuda:0")
    out = {}
    import torch.nn.functional as F
    real_bn = m.dense.bn_relu

    def torch_bn(x, bn, relu):  # torch's own BatchNorm (MIOpen with cudnn enabled, native otherwise)
        y = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, True, bn.momentum, bn.eps)
        return torch.relu(y) if relu else y
    for tag, dense, cudnn, bnf in (("hip", True, True, real_bn), ("torch", False, True, real_bn),
                                   ("torch_native", False, False, real_bn), ("hip_conv_miopen_bn", True, True, torch_bn),
                                   ("hip_conv_native_bn", True, False, torch_bn)):
        torch.backends.cudnn.enabled = cudnn
        m.dense.bn_relu = bnf
        model = f5_models(m).to(dev)
        model.dense_kernels = dense
        for mod in model.modules():
            mod.dense_kernels = dense
        rgb, depth, gt = (t.to(dev) for t in f9_inputs())
        model.train()
        est, _ = model(rgb, depth, rgb, depth)
        loss = m.train.calculate_loss_multi_resolution(est, gt, False)
        loss.backward()
        torch.cuda.synchronize()
        out[tag] = {"loss": loss.item(), "est": [e.detach().cpu() for e in est],
                    "grads": {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None}}
        print(tag, "loss", loss.item(), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    torch.save(out, os.path.join(ROOT, "gpurun_out", "f9_grads.pt"))


if __name__ == "__main__":
    main()
