"""Shared input builders and the oracle-side layer (glue + nconv2d) for the parity tests."""
import torch
import torch.nn.functional as F

from oracle import nconv_ref as R

PLAIN, THRESH, POOL2, UPCAT_SKIP_FIRST, UPCAT_UP_FIRST = 0, 1, 2, 3, 4


def oracle_layer(mode, xa, ca, xb, cb, w, b, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups=1, thresh=0.01):
    """The reference's glue op followed by NConv2d.forward, on whatever device/dtype given."""
    if mode == THRESH:
        x, c = xa, (xa > thresh).to(xa.dtype)
    elif mode == PLAIN:
        x, c = xa, ca
    elif mode == POOL2:
        x, c = F.max_pool2d(xa, 2, 2), F.max_pool2d(ca, 2, 2)
    else:
        up = lambda t: F.interpolate(t, xa.shape[2:], mode="nearest")
        if mode == UPCAT_SKIP_FIRST:
            x, c = torch.cat((xa, up(xb)), 1), torch.cat((ca, up(cb)), 1)
        else:
            x, c = torch.cat((up(xb), xa), 1), torch.cat((up(cb), ca), 1)
    return R.nconv2d(x, c, w, b, stride, pad, dil, groups)


def rand_pair(g, B, C, H, W, dtype=torch.float32, density=0.7):
    """data U(0,10); confidence 0 with prob 1-density, else U(0.05, 1)."""
    x = torch.rand(B, C, H, W, generator=g, dtype=dtype) * 10
    keep = torch.rand(B, C, H, W, generator=g, dtype=dtype) < density
    c = (torch.rand(B, C, H, W, generator=g, dtype=dtype) * 0.95 + 0.05) * keep
    return x, c


def rand_weight(g, cout, cin, kh, kw, dtype=torch.float32):
    """Positive weights like a trained (softplus'd) NConv layer."""
    return torch.rand(cout, cin, kh, kw, generator=g, dtype=dtype) + 0.05


# (name, mode, cin, cout, k, pad, stride, dil, groups, a-shape, b-shape) — a/b shapes (C, H, W)
LAYER_CASES = [
    ("nconv1_thresh", THRESH, 1, 8, 5, 2, 1, 1, 1, (1, 37, 70), None),
    ("nconv2_plain", PLAIN, 8, 8, 5, 2, 1, 1, 1, (8, 37, 70), None),
    ("down_pool_odd", POOL2, 8, 8, 5, 2, 1, 1, 1, (8, 37, 71), None),
    ("down_pool_even", POOL2, 8, 8, 5, 2, 1, 1, 1, (8, 48, 130), None),
    ("down_pool_ties", POOL2, 8, 8, 5, 2, 1, 1, 1, (8, 30, 66), None),  # integer data: exact ties
    ("nconv4_upcat_exact", UPCAT_SKIP_FIRST, 16, 8, 3, 1, 1, 1, 1, (8, 24, 70), (8, 12, 35)),
    ("nconv5_upcat_inexact", UPCAT_SKIP_FIRST, 16, 8, 3, 1, 1, 1, 1, (8, 25, 71), (8, 12, 35)),
    ("nconv6_upfirst_p0", UPCAT_UP_FIRST, 16, 8, 3, 0, 1, 1, 1, (8, 37, 70), (8, 18, 35)),
    ("nconv7_1x1_p2", PLAIN, 8, 1, 1, 2, 1, 1, 1, (8, 35, 68), None),
    # widths a multiple of 4: the 16-byte store (and LDS-DMA staging) paths of the MFMA kernels
    ("nconv2_w4", PLAIN, 8, 8, 5, 2, 1, 1, 1, (8, 21, 68), None),
    ("nconv5_upcat_w4", UPCAT_SKIP_FIRST, 16, 8, 3, 1, 1, 1, 1, (8, 26, 72), (8, 13, 36)),
    ("nconv6_upfirst_w4", UPCAT_UP_FIRST, 16, 8, 3, 0, 1, 1, 1, (8, 34, 72), (8, 17, 36)),
    # 1, 2 and 5 output rows: the row-pair weight gradient's single-row / lone-pair segments
    ("nconv2_h1", PLAIN, 8, 8, 5, 2, 1, 1, 1, (8, 1, 70), None),
    ("nconv2_h2", PLAIN, 8, 8, 5, 2, 1, 1, 1, (8, 2, 40), None),
    ("down_pool_h5", POOL2, 8, 8, 5, 2, 1, 1, 1, (8, 10, 33), None),
    ("generic_3x3_plain", PLAIN, 8, 8, 3, 1, 1, 1, 1, (8, 29, 41), None),
    ("generic_stride2", PLAIN, 4, 6, 3, 1, 2, 1, 1, (4, 29, 41), None),
    ("generic_dil2_groups2", PLAIN, 4, 6, 3, 2, 1, 2, 2, (4, 29, 41), None),
    ("generic_pool_c3", POOL2, 3, 5, 5, 2, 1, 1, 1, (3, 21, 30), None),
]
