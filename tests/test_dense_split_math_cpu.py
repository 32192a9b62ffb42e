"""The split-bf16 arithmetic of the guided 3x3 convolutions (dense_conv_bf9, include/nconv.h enum
nconv_dense_math), emulated on the CPU with torch's round-to-nearest-even bf16 conversion, the
conversion the kernel uses ((__bf16)v):
  * three parts v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1) sum to v exactly;
  * every partial product vi * wj is exact in fp32 (two 8-bit significands);
  * NCONV_DENSE_MATH_BF16X6 drops v1*w2 + v2*w1 + v2*w2, at most ~2^-23 of |v w| (the bound the
    header states; fp32's unit round-off is 2^-24).
Values within 2^+-30 (the kernel's operands are activations and weights; far from fp32's underflow,
where the lo*lo terms of two tiny operands would leave the normal range)."""
import pytest
import torch


def _split3(v):
    p0 = v.to(torch.bfloat16).float()
    r1 = v - p0
    p1 = r1.to(torch.bfloat16).float()
    r2 = r1 - p1
    p2 = r2.to(torch.bfloat16).float()
    return p0, p1, p2


def _values(seed, n=200000):
    g = torch.Generator().manual_seed(seed)
    mant = torch.rand(n, generator=g) + 1.0                     # [1, 2)
    expo = torch.randint(-30, 30, (n,), generator=g).float()  # products and their lo terms stay normal
    sign = torch.where(torch.rand(n, generator=g) < 0.5, -1.0, 1.0)
    v = (sign * mant * torch.pow(2.0, expo)).float()
    # adversarial significands: all ones, halfway patterns, powers of two
    special = torch.tensor([1.0, 1.0 + 2 ** -23, 2 - 2 ** -23, 1 + 2 ** -8, 1 + 2 ** -9, 1 + 2 ** -16 + 2 ** -17,
                            1.00390625, 0.99609375, 3.1415927, -2.7182817, 1e-6, 3e6], dtype=torch.float32)
    return torch.cat([v, special])


@pytest.mark.parametrize("seed", [1, 2])
def test_three_part_split_is_exact(seed):
    v = _values(seed)
    p0, p1, p2 = _split3(v)
    assert torch.equal(p2.to(torch.bfloat16).float(), p2)      # the last part is a bf16 value
    assert torch.equal(p0.double() + p1.double() + p2.double(), v.double())


@pytest.mark.parametrize("seed", [3, 4])
def test_partial_products_exact_and_bf16x6_bound(seed):
    v, w = _values(seed), _values(seed + 100)
    n = min(v.numel(), w.numel())
    v, w = v[:n], w[:n]
    pv, pw = _split3(v), _split3(w)
    exact = v.double() * w.double()
    total = torch.zeros_like(exact)
    dropped = torch.zeros_like(exact)
    for i in range(3):
        for j in range(3):
            prod32 = (pv[i] * pw[j]).double()                     # the fp32 product ...
            assert torch.equal(prod32, pv[i].double() * pw[j].double())  # ... is exact
            total += prod32
            if i + j > 2:
                dropped += prod32
    assert torch.equal(total, exact)                            # all nine: v * w exactly
    ratio = (dropped.abs() / exact.abs()).max().item()
    assert ratio <= 2.0 ** -23, ratio
