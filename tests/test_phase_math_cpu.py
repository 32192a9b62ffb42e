"""CPU: the identity behind the forward's phase path (realtime-depth-estimation-nconv_amd/csrc/
nconv_fwd_phase.hip), in float64 on the reference's own ops. A 3x3 convolution (any padding) of a
nearest-2x-upsampled plane equals, at every output pixel, a 2x2 convolution of the low-resolution
plane whose weights are sums of the 3x3 taps that land on the same low pixel -- which taps do
depends only on the parity of the window's first input row / column:
    first index even: taps {0,1} -> low pixel m, {2} -> m + 1; odd: {0} -> m, {1,2} -> m + 1.
This restates the phase-weight table of nconv_phase_weights (S(a, d) below) and checks it against
F.conv2d(F.interpolate(nearest)) -- the reference's glue + NConv2d sums (models/step1.py:78-90,
119-122)."""
import pytest
import torch
import torch.nn.functional as F

S = {(0, 0): (0, 1), (0, 1): (2,), (1, 0): (0,), (1, 1): (1, 2)}


def phase_conv(v, w, pad):
    """sum_{dh,dw} Wp[a][b][dh][dw] * v[(ih0>>1)+dh][(iw0>>1)+dw], ih0 = oh - pad (one channel)."""
    H, W = 2 * v.shape[0], 2 * v.shape[1]
    Ho, Wo = H + 2 * pad - 2, W + 2 * pad - 2
    vp = F.pad(v, (2, 2, 2, 2))  # low plane with a zero border: indices -2.. shifted by +2
    out = torch.zeros(Ho, Wo, dtype=v.dtype)
    for oh in range(Ho):
        for ow in range(Wo):
            ih0, iw0 = oh - pad, ow - pad
            a, bt = ih0 & 1, iw0 & 1
            acc = 0.0
            for dh in (0, 1):
                for dw in (0, 1):
                    wp = sum(w[kh, kw] for kh in S[(a, dh)] for kw in S[(bt, dw)])
                    acc += wp * vp[(ih0 >> 1) + dh + 2, (iw0 >> 1) + dw + 2]
            out[oh, ow] = acc
    return out


@pytest.mark.parametrize("pad", [0, 1, 2])
@pytest.mark.parametrize("hw", [(5, 7), (6, 4)])
def test_phase_weights_identity(pad, hw):
    g = torch.Generator().manual_seed(pad * 10 + hw[0])
    v = torch.rand(*hw, generator=g, dtype=torch.float64)
    w = torch.rand(3, 3, generator=g, dtype=torch.float64)
    up = F.interpolate(v[None, None], scale_factor=2, mode="nearest")
    ref = F.conv2d(up, w[None, None], padding=pad)[0, 0]
    torch.testing.assert_close(phase_conv(v, w, pad), ref, rtol=1e-12, atol=1e-12)


def test_phase_weights_host_validation(nconv_amd):
    import ctypes
    lib = nconv_amd._lib.lib()
    P, I = ctypes.c_void_p * 1, ctypes.c_int * 1
    rc = lib.nconv_phase_weights(1, P(0x1000), I(16), I(9), P(0x2000), None)  # channels 9..16 > Cin
    assert rc == -22 and "upsampled channels" in lib.nconv_last_error().decode()
    rc = lib.nconv_phase_weights(1, P(None), I(16), I(8), P(0x2000), None)
    assert rc == -22
