"""CPU: drop-in API surface of the modules — constructor signatures, RNG consumption (seeded
initialisation equals the reference's, golden f6), state_dict keys, crop geometry."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_seeded_init_matches_reference_bitwise(nconv_amd):
    f = np.load(os.path.join(GOLD, "f6_init.npz"))
    torch.manual_seed(0)
    net = nconv_amd.SETP1_NCONV()
    sd = net.state_dict()
    keys = sorted(k[len("setp1_"):] for k in f.files if k.startswith("setp1_"))
    assert keys == sorted(k for k, v in sd.items() if v.dtype == torch.float32)
    for k in keys:
        assert np.array_equal(sd[k].numpy(), f["setp1_" + k]), k


def test_state_dict_layout(nconv_amd):
    sd = nconv_amd.SETP1_NCONV().state_dict()
    assert len(sd) == 63  # 9 layers x (weight, bias, 5 bnorm entries)
    assert "d_net.nconv7.bnorm.num_batches_tracked" in sd
    assert tuple(sd["d_net.nconv4.weight"].shape) == (8, 16, 3, 3)
    assert tuple(sd["d_net.nconv7.weight"].shape) == (1, 8, 1, 1)


def test_nconv2d_signature_and_hook(nconv_amd):
    from nconv_amd.nconv import EnforcePos
    m = nconv_amd.NConv2d(4, 6, (3, 3), "softplus", "x", stride=(2, 2), padding=(1, 1))
    assert m.eps == 1e-7 and m.pos_fn == "softplus" and m.init_method == "x"
    assert tuple(m.weight.shape) == (6, 4, 3, 3)
    assert torch.allclose(m.bias, torch.full((6,), 0.01))
    hooks = list(m._forward_pre_hooks.values())
    assert len(hooks) == 1 and isinstance(hooks[0], EnforcePos)
    # the hook applies softplus in training mode only (CPU tensor -> torch op path)
    w0 = m.weight.detach().clone()
    m.eval()
    hooks[0](m, None)
    assert torch.equal(m.weight.detach(), w0)
    m.train()
    hooks[0](m, None)
    assert torch.allclose(m.weight.detach(), torch.nn.functional.softplus(w0, beta=10))


@pytest.mark.parametrize("H,W,crop,expect", [
    (480, 640, "literal", (480, 640)), (352, 1216, "literal", (353, 640)), (1024, 2048, "literal", (480, 640)),
    (64, 96, "literal", (65, 97)), (352, 1216, "generalized", (352, 1216)), (480, 640, "generalized", (480, 640)),
])
def test_crop_geometry(nconv_amd, H, W, crop, expect):
    """the reference's crop [1:481, 1:641] of the (H+2) x (W+2) nconv7 grid."""
    assert nconv_amd.crop_hw(H, W, crop) == expect
