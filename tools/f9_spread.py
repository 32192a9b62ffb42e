#!/usr/bin/env python3
"""Per-tensor fp32 spread of the reference's guided training gradients (golden f9), for the GPU
gradient bounds of tests/test_gpu_guided.py.

For every trainable SETP2 gradient of f9's iteration (train_step2.py:60-66 as the imported
reference ran it in fp32 on the CPU, stored in tests/golden/f9_guided_train.npz) this computes its
normwise distance from the float64 oracle of the same iteration (guided_cases.grad_rel) and writes
tests/golden/f9_ref_spread.json. The GPU tests then hold each gradient to
max(1e-3, 1.5 x that tensor's reference spread) against float64: the bound is
the reference's own fp32 error on that tensor, not one blanket figure.

    python tools/f9_spread.py        # CPU, ~1 min; test infrastructure (reads oracle/ and tests/golden)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from guided_cases import f5_models, f9_inputs, grad_rel, trainable_setp2  # noqa: E402
from oracle import nconv_ref as R  # noqa: E402


def main():
    import nconv_pkg
    m = nconv_pkg.load()
    f = np.load(os.path.join(ROOT, "tests", "golden", "f9_guided_train.npz"))
    model = f5_models(m)
    sd = {k: v.detach().double().cpu().clone() for k, v in model.state_dict().items()}
    rgb, depth, gt = f9_inputs()
    names = trainable_setp2(None, model.named_parameters())
    p1 = R.dnet_params_from_state_dict({k: (R.softplus_pos(v) if k.endswith(".weight") and "bnorm" not in k else v)
                                        for k, v in sd.items()}, "step1.d_net.")
    leaves = {k: sd[k].clone().requires_grad_(True) for k in names}
    sd.update(leaves)
    o0, _ = R.setp2_forward(sd, rgb.double(), depth.double(), rgb.double(), depth.double(), "literal", "train",
                            training=True, step1_params=p1)
    R.calculate_loss_multi_resolution(o0, gt.double(), False).backward()
    g64 = {k: leaves[k].grad for k in names}
    refs = {k: torch.from_numpy(f["grad_" + k]).double() for k in names}
    spread = {k: grad_rel(refs[k], g64[k], k, g64) for k in names}
    out = {"source": "tests/golden/f9_guided_train.npz gradients (reference, fp32 CPU) vs the float64 oracle "
                     "of the same iteration; normwise, guided_cases.grad_rel; written by tools/f9_spread.py",
           "spread": {k: float(f"{v:.4e}") for k, v in sorted(spread.items())}}
    path = os.path.join(ROOT, "tests", "golden", "f9_ref_spread.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(f"wrote {path}: {len(spread)} tensors, max spread {max(spread.values()):.2e}")


if __name__ == "__main__":
    main()
