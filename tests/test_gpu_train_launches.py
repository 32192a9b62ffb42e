"""GPU: the training step's launch trimming against the launches it replaces.

* nconv_train_prologue (one launch: EnforcePos in place, normalisers, the exact head's weights, the
  phase weights and the backward's box weights of nconv4/5/6) writes bitwise what weight_prep +
  head_weights + phase_weights write, and the box weights are the row-major sums of 1, 2 or 4
  weights (models/step1.py:190-207's softplus hook, then the forward's weight-only inputs);
* a whole DNET training iteration with the merged prologue equals the separate-launch path
  bitwise (weights after the drift, output, every gradient);
* the cropped training output written by the fused tail (step1.py:94, no crop copy, the backward
  reading the loss gradient through the window) equals nconv7's whole grid + CropFn bitwise,
  except nconv7's bias gradient (the same sum over another layout; 1e-6 normwise);
* nconv_wgrad_reduce_ex's plain sums (nconv7's bias gradient) against a float64 sum, ragged
  lengths included, and deterministic (two runs bitwise).
"""
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from test_gpu_dnet import make_net, sparse_depth  # noqa: E402


def _box_ref(w, first_up):
    """Box weights [o][i][t][u] as fp32 sums in row-major tap order (kh ascending, then kw)."""
    S = {0: [2], 1: [1, 2], 2: [0, 1], 3: [0]}
    out = torch.empty(8, 8, 4, 4, dtype=torch.float32)
    wc = w.detach().cpu()
    for o in range(8):
        for i in range(8):
            for t in range(4):
                for u in range(4):
                    s = torch.zeros((), dtype=torch.float32)
                    for kh in S[t]:
                        for kw in S[u]:
                            s = s + wc[o, first_up + i, kh, kw]
                    out[o, i, t, u] = s
    return out.reshape(-1)


def test_train_prologue_bitwise_separate_launches(nconv_amd, gpu):
    N = nconv_amd.nconv
    torch.manual_seed(5)
    net = nconv_amd.SETP1_NCONV(crop="generalized").to(gpu)
    layers = [getattr(net.d_net, n) for n in nconv_amd.dnet.LAYERS]
    # raw (pre-softplus) weights with both branches of the softplus threshold (beta * w > 20)
    with torch.no_grad():
        for m in layers:
            m.weight.mul_(3.0)
            m.weight.view(-1)[:3] = torch.tensor([2.5, -3.0, 2.0000002])
    wa = [m.weight.detach().clone() for m in layers]
    wb = [m.weight.detach().clone() for m in layers]
    sa = [torch.empty(w.shape[0], device=gpu) for w in wa]
    sb = [torch.full((w.shape[0],), float("nan"), device=gpu) for w in wb]
    N.weight_prep(wa, [True] * 9, sa)
    l1, l2 = layers[0], layers[1]
    sp1, sp2 = l1.spec(nconv_amd._lib.THRESH, 0.01), l2.spec()
    S = torch.zeros(1, 1, 32, 32, device=gpu)
    ha = N.head_weights(sp1, sp2, S, wa[0], l1.bias.detach(), sa[0], wa[1], l2.bias.detach(), sa[1])
    pa = [torch.empty(1024, device=gpu) for _ in range(3)]
    N.phase_weights([wa[5], wa[6], wa[7]], [8, 8, 0], pa)
    hb = torch.full((N.HEAD_WEIGHTS_FLOATS,), float("nan"), device=gpu)
    pb = [torch.full((1024,), float("nan"), device=gpu) for _ in range(3)]
    bb = [torch.full((N.BOX_WEIGHT_FLOATS,), float("nan"), device=gpu) for _ in range(3)]
    sp = [True, True, False, True, True, True, False, True, True]  # two layers without the hook
    wa[2].copy_(wb[2])  # (layers 2 and 6 keep their raw weights in the merged call)
    wa[6].copy_(wb[6])
    N.weight_prep([wa[2], wa[6]], [False, False], [sa[2], sa[6]])
    pa[1] = torch.empty(1024, device=gpu)
    N.phase_weights([wa[6]], [8], [pa[1]])
    sync = torch.zeros(1, dtype=torch.int32, device=gpu)
    N.train_prologue(wb, sp, sb, head=(0, 1, hb, sync), phase=([5, 6, 7], [8, 8, 0], pb, bb))
    torch.cuda.synchronize()
    for k, (a, b) in enumerate(zip(wa, wb)):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), k
    for k, (a, b) in enumerate(zip(sa, sb)):
        assert torch.equal(a, b), k
    assert torch.equal(ha.view(torch.int32), hb.view(torch.int32))
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
    for k, (li, up) in enumerate(((5, 8), (6, 8), (7, 0))):
        assert torch.equal(bb[k].cpu(), _box_ref(wb[li], up)), k
    assert sync.item() == 0  # (left at zero for the next call)
    # repeated calls on the same counter (as graph replays run them): same outputs each time
    hc = torch.full_like(hb, float("nan"))
    for _ in range(3):
        N.train_prologue([w.clone() for w in wb], [False] * 9, [torch.empty_like(v) for v in sb],
                         head=(0, 1, hc, sync))
    torch.cuda.synchronize()
    assert sync.item() == 0
    hd = N.head_weights(sp1, sp2, S, wb[0], l1.bias.detach(), sb[0], wb[1], l2.bias.detach(), sb[1])
    assert torch.equal(hc.view(torch.int32), hd.view(torch.int32))


def test_train_prologue_without_head_or_phase(nconv_amd, gpu):
    """Only prep roles (no head, no phase layers): the weight_prep results."""
    N = nconv_amd.nconv
    torch.manual_seed(6)
    ws = [torch.randn(8, 16, 3, 3, device=gpu), torch.randn(1, 8, 1, 1, device=gpu)]
    wa, wb = [w.clone() for w in ws], [w.clone() for w in ws]
    sa = [torch.empty(w.shape[0], device=gpu) for w in ws]
    sb = [torch.empty(w.shape[0], device=gpu) for w in ws]
    N.weight_prep(wa, [True, False], sa)
    N.train_prologue(wb, [True, False], sb)
    torch.cuda.synchronize()
    for a, b in zip(wa + sa, wb + sb):
        assert torch.equal(a, b)


def _train_iteration(nconv_amd, gpu, B, H, W, crop, merged=True, in_tail=True, seed=31, fwd_streams=None):
    if fwd_streams is not None:
        nconv_amd.dnet.TRAIN_FWD_STREAMS = fwd_streams
    g = torch.Generator().manual_seed(seed)
    S = sparse_depth(g, B, H, W).to(gpu)
    net = make_net(nconv_amd, crop, gpu)
    net.d_net.merged_prologue = merged
    net.d_net.crop_in_tail = in_tail
    net.train()
    out = net(S)
    gt = (torch.rand(out.shape, generator=g) * 80).to(gpu)  # (the literal crop keeps H + 1 rows)
    nconv_amd.train.calculate_loss(out, gt, True).backward()
    torch.cuda.synchronize()
    return (out.detach(), {k: v.detach().clone() for k, v in net.named_parameters()},
            {k: v.grad for k, v in net.named_parameters() if v.grad is not None})


@pytest.mark.parametrize("B,H,W", [(2, 64, 96), (2, 48, 200)])
def test_dnet_train_merged_prologue_bitwise(nconv_amd, gpu, B, H, W):
    oa, wa, ga = _train_iteration(nconv_amd, gpu, B, H, W, "generalized", merged=True)
    ob, wb, gb = _train_iteration(nconv_amd, gpu, B, H, W, "generalized", merged=False)
    assert torch.equal(oa, ob)
    for k in wa:
        assert torch.equal(wa[k], wb[k]), k
    assert set(ga) == set(gb) and len(ga) == 18
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k


@pytest.mark.parametrize("crop,B,H,W", [("generalized", 2, 64, 96), ("literal", 2, 64, 96),
                                        ("generalized", 2, 48, 200), ("literal", 1, 480, 640)])
def test_dnet_cropped_tail_matches_uncropped(nconv_amd, gpu, crop, B, H, W):
    """The training output written cropped by the fused tail against the whole grid + CropFn: bitwise."""
    oa, _, ga = _train_iteration(nconv_amd, gpu, B, H, W, crop, in_tail=True)
    ob, _, gb = _train_iteration(nconv_amd, gpu, B, H, W, crop, in_tail=False)
    assert oa.shape == ob.shape and torch.equal(oa, ob)
    assert set(ga) == set(gb) and len(ga) == 18
    for k in ga:
        if k.endswith("nconv7.bias"):  # the same sum over the cropped / the zero-padded plane
            rel = ((ga[k] - gb[k]).abs().max() / gb[k].abs().max()).item()
            assert rel <= 1e-6, (k, rel)
        else:
            assert torch.equal(ga[k], gb[k]), k


def test_dnet_literal_wide_crop_keeps_full_grid(nconv_amd, gpu):
    """At 352x1216 the literal crop (353 x 640) does not cover nconv6's grid: the training pass
    keeps nconv7's whole grid and crops after (CropFn) -- same result as with crop_in_tail off."""
    d = make_net(nconv_amd, "literal", gpu).d_net
    S = torch.zeros(1, 1, 352, 1216, device=gpu)
    assert not d._tail_crop(S, torch.empty(3, 1024, device=gpu))
    S = torch.zeros(1, 1, 64, 96, device=gpu)
    assert d._tail_crop(S, torch.empty(3, 1024, device=gpu))


@pytest.mark.parametrize("n", [1, 255, 1000, 1023, 1024, 4097, 3424256, 3424263])
def test_wgrad_reduce_sum_jobs(nconv_amd, gpu, n):
    g = torch.Generator().manual_seed(n)
    x = (torch.rand(n, generator=g, dtype=torch.float64) - 0.3).float().to(gpu)
    y = torch.rand(7, generator=g).float().to(gpu)
    outs = []
    for _ in range(2):
        red = nconv_amd.nconv.WgradReduce()
        o1, o2 = torch.full((1,), float("nan"), device=gpu), torch.full((1,), float("nan"), device=gpu)
        red.add_sum(x, o1)
        red.add_sum(y, o2)
        red.run(gpu)
        outs.append((o1.clone(), o2.clone()))
    torch.cuda.synchronize()
    ref = x.double().sum().item()
    assert abs(outs[0][0].item() - ref) <= 1e-6 * x.double().abs().sum().item()
    assert abs(outs[0][1].item() - y.double().sum().item()) <= 1e-6
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_wgrad_reduce_sum_empty(nconv_amd, gpu):
    red = nconv_amd.nconv.WgradReduce()
    o = torch.full((1,), float("nan"), device=gpu)
    red.add_sum(torch.empty(0, device=gpu), o)
    red.run(gpu)
    torch.cuda.synchronize()
    assert o.item() == 0.0


@pytest.mark.parametrize("B,H,W,crop", [(2, 64, 96, "generalized"), (3, 48, 200, "literal"),
                                        (8, 352, 1216, "generalized")])
def test_dnet_train_forward_streams_bitwise(nconv_amd, gpu, B, H, W, crop):
    """The training forward in batch slices on two streams (dnet.TRAIN_FWD_STREAMS, each launch
    writing its rows of full-batch tensors) equals the one-stream pass bitwise: output, weights
    after the drift and every gradient (B = 3: uneven slices 1 + 2)."""
    keep = nconv_amd.dnet.TRAIN_FWD_STREAMS
    try:
        oa, wa, ga = _train_iteration(nconv_amd, gpu, B, H, W, crop, fwd_streams=2)
        ob, wb, gb = _train_iteration(nconv_amd, gpu, B, H, W, crop, fwd_streams=1)
    finally:
        nconv_amd.dnet.TRAIN_FWD_STREAMS = keep
    assert torch.equal(oa, ob)
    for k in wa:
        assert torch.equal(wa[k], wb[k]), k
    assert set(ga) == set(gb) and len(ga) == 18
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k


@pytest.mark.parametrize("B,H,W,crop", [(2, 64, 96, "generalized"), (8, 352, 1216, "generalized")])
def test_dnet_train_wgrad_stream_placement_bitwise(nconv_amd, gpu, B, H, W, crop):
    """Where the weight gradients run (dnet.WGRAD_LAST_MAIN: nconv2's on the main stream after its
    input gradient, or with the others on the side stream; dnet.WGRAD_STREAM off: all serial) does
    not change a bit of any gradient: same kernels, same fixed-order reductions."""
    D = nconv_amd.dnet
    keep = (D.WGRAD_LAST_MAIN, D.WGRAD_STREAM)
    runs = []
    try:
        for last_main, stream in ((True, True), (False, True), (True, False)):
            D.WGRAD_LAST_MAIN, D.WGRAD_STREAM = last_main, stream
            runs.append(_train_iteration(nconv_amd, gpu, B, H, W, crop))
    finally:
        D.WGRAD_LAST_MAIN, D.WGRAD_STREAM = keep
    oa, _, ga = runs[0]
    for ob, _, gb in runs[1:]:
        assert torch.equal(oa, ob)
        assert set(ga) == set(gb) and len(ga) == 18
        for k in ga:
            assert torch.equal(ga[k], gb[k]), k
