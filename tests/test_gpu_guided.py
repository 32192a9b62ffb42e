"""GPU: the RGB-guided model (SETP2_BP_TRAIN / EXPORT) with step 1 on libnconv, against the reference's
golden outputs (480x640, f5) and against the oracle at KITTI-like shapes with the generalized crop.
Tolerance: |gpu - ref| <= 1e-4*|ref| + 1e-3 (fp32 conv stacks of depth ~15 on values up to ~80)."""
import numpy as np
import pytest
import torch

from guided_cases import f5_inputs, f5_models
from oracle import nconv_ref as R

pytestmark = pytest.mark.gpu


def _close(got, ref, what):
    got = got.double().cpu()
    ref = torch.as_tensor(np.asarray(ref)).double() if not torch.is_tensor(ref) else ref.double()
    err = (got - ref).abs()
    bound = 1e-4 * ref.abs() + 1e-3
    assert (err <= bound).all(), f"{what}: max err {err.max():.3e}"


def test_guided_train_model_matches_reference_f5(nconv_amd, gpu):
    import os
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "f5_guided.npz"))
    model = f5_models(nconv_amd).to(gpu).eval()
    ins = [t.to(gpu) for t in f5_inputs()]
    with torch.no_grad():
        o0, o1 = model(*ins)
    for i in range(4):
        for tag, o in (("out0", o0[i]), ("out1", o1[i])):
            full = o[0, 0]
            _close(full if i < 2 else full[::4, ::4], f[f"{tag}_{i}"], f"{tag} scale {i}")
    exp = f5_models(nconv_amd, "export").to(gpu).eval()
    with torch.no_grad():
        e0, e1 = exp(*ins)
    _close(e0[0, 0, ::4, ::4], f["export0"], "export")


@pytest.mark.parametrize("H,W", [(64, 96), (96, 320)])
def test_guided_generalized_crop_vs_oracle(nconv_amd, gpu, H, W):
    torch.manual_seed(2)
    model = nconv_amd.SETP2_BP_TRAIN(None, step1_crop="generalized").to(gpu).eval()
    with torch.no_grad():  # trained-like positive step-1 weights
        for n, p in model.step1.named_parameters():
            if n.endswith("weight") and "bnorm" not in n:
                p.copy_(torch.nn.functional.softplus(p, beta=10))
    rgb0, d0, rgb1, d1 = f5_inputs(H, W)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        g0, g1 = model(rgb0.to(gpu), d0.to(gpu), rgb1.to(gpu), d1.to(gpu))
        r0, r1 = R.setp2_forward(sd, rgb0, d0, rgb1, d1, "generalized", "train")
    for i in range(4):
        _close(g0[i], r0[i], f"pair0 scale {i}")
        _close(g1[i], r1[i], f"pair1 scale {i}")
