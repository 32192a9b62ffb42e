"""DNET's inference split (DNET.split_bounds: frames per inference stream, even or by relative
shares) and bench.py's --inference-shares validation. CPU only: bounds arithmetic, no launch."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_even_split(nconv_amd):
    sb = nconv_amd.DNET.split_bounds
    assert sb(8, 2) == [0, 4, 8]
    assert sb(5, 3) == [0, 1, 3, 5]
    assert sb(1, 1) == [0, 1]


def test_shares_split(nconv_amd):
    sb = nconv_amd.DNET.split_bounds
    assert sb(8, 2, (5, 3)) == [0, 5, 8]
    assert sb(8, 2, (1, 1)) == [0, 4, 8]
    b = sb(7, 3, (1.0, 2.0, 4.0))
    assert b[0] == 0 and b[-1] == 7 and all(x <= y for x, y in zip(b, b[1:]))
    # an extreme share still gives monotone bounds inside [0, B]
    b = sb(4, 2, (1e9, 1e-9))
    assert b == [0, 4, 4]


@pytest.mark.parametrize("shares", [(0, 1), (-1, 2), (float("nan"), 1), (float("inf"), 1)])
def test_shares_must_be_positive_finite(nconv_amd, shares):
    with pytest.raises(ValueError):
        nconv_amd.DNET.split_bounds(8, 2, shares)


def test_shares_count_must_match_streams(nconv_amd):
    sb = nconv_amd.DNET.split_bounds
    with pytest.raises(ValueError):
        sb(8, 2, (1, 2, 3))
    with pytest.raises(ValueError):
        sb(8, 2, (1,), configured=2)
    # batch smaller than the configured streams (n clamped to B): shares for the configured count
    # are accepted and the split is even
    assert sb(2, 2, (1, 2, 3), configured=3) == [0, 1, 2]
    with pytest.raises(ValueError):
        sb(2, 2, (1, 2), configured=3)


def test_bench_inference_shares_argparse():
    a = bench.parse(["--inference-shares", "5,3"])
    assert a.inference_shares == [5.0, 3.0]
    a = bench.parse(["--inference-streams", "3", "--inference-shares", "1,1,2"])
    assert a.inference_shares == [1.0, 1.0, 2.0]
    for bad in (["--inference-shares", "0,1"], ["--inference-shares", "a,b"], ["--inference-shares", "1,-2"],
                ["--inference-shares", "1,2,3"], ["--inference-streams", "3", "--inference-shares", "1,2"]):
        with pytest.raises(SystemExit):
            bench.parse(bad)
