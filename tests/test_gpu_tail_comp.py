"""GPU: the composed fused tail (nconv_fwd_tail_comp, csrc/nconv_fwd_tail.hip): nconv6's skip-half
confidence mass D6s = W621 (x) c0 on the bf16 matrix cores (the composition of nconv6's, nconv2's and
nconv1's weights applied to the thresholded input, csrc/nconv_tail.h) and the head writing nconv2's
y * cout for it (nconv_fwd_head_xc), against the phase tail over nconv2's y and cout (the reference's
sums, models/step1.py:88-94) and against the float64 oracle.

Tolerances: the composed D6s differs from sum W6 * c2 only by the rounding of the composed weights
(fp64, rounded once) and the sum order (all terms non-negative), so the whole forward stays within the
north star's 1e-4 relative of the oracle (test_gpu_dnet runs the composed path, the default); here
composed vs phase tail |a - b| <= 2e-6 |b| + 1e-6 elementwise; the tail weights bitwise between
their two launches, the composed weights within one fp32 ulp of a float64 recomputation, the re-laid
phase weights bitwise nconv_phase_weights' values.
"""
import numpy as np
import pytest
import torch

from oracle import nconv_ref as R
from test_gpu_dnet import make_net, oracle_params, sparse_depth

pytestmark = pytest.mark.gpu


def _net_weights(net):
    d = net.d_net
    return d.nconv1, d.nconv2, d.nconv6


def _tail_weights(nconv_amd, net, S, prologue):
    """The tail weights from the one-launch eval prologue or from nconv_tail_weights."""
    m, lib = nconv_amd, nconv_amd._lib
    d = net.d_net
    layers = [getattr(d, n) for n in m.dnet.LAYERS]
    if prologue:
        wsum, wph, w21, wt = d._eval_prologue(layers, S)
        assert wt is not None
        return wt
    wsum = d._prologue(layers, S)
    l1, l2, l6 = layers[0], layers[1], layers[7]
    return m.nconv.tail_weights(l1.spec(lib.THRESH, 0.01), l2.spec(), l6.spec(lib.UPCAT_UP_FIRST), S, l1.weight,
                                wsum[0], l2.weight, wsum[1], l6.weight)


def _decode(wt):
    """W621[o][U][V] from the bf16 fragments (hi + mid + lo, nconv_tail.h's layout)."""
    bits = wt[:2048].cpu().numpy().view(np.uint16).astype(np.uint32) << 16
    vals = bits.view(np.float32).astype(np.float64)
    out = np.zeros((8, 11, 11))
    for o in range(8):
        for q in range(16):
            for j in range(8):
                if q <= 10:
                    U, V = q, j
                elif q <= 13:
                    U, V = j, 8 + q - 11
                elif q == 14:
                    U, V = 8 + j // 3, 8 + j % 3
                else:
                    if j:
                        continue
                    U, V = 10, 10
                s = 0.0
                for part in range(3):
                    slot = ((((o >> 2) * 4 + (q >> 2)) * 64 + (q & 3) * 16 + 4 * (o & 3) + part) * 8 + j)
                    s += vals[slot]
                out[o, U, V] = s
    return out


def _composed64(net, s1, s2):
    l1, l2, l6 = _net_weights(net)
    W1 = l1.weight.detach().double().cpu().numpy()[:, 0]    # (8, 5, 5)
    W2 = l2.weight.detach().double().cpu().numpy()          # (8, 8, 5, 5)
    W6 = l6.weight.detach().double().cpu().numpy()[:, 8:]  # (8, 8, 3, 3) skip half
    s1, s2 = s1.double().cpu().numpy(), s2.double().cpu().numpy()
    W21 = np.zeros((8, 9, 9))
    for i in range(8):
        for j in range(8):
            for kh in range(5):
                for kw in range(5):
                    W21[i, kh:kh + 5, kw:kw + 5] += W2[i, j, kh, kw] * W1[j] / s1[j]
    W621 = np.zeros((8, 11, 11))
    for o in range(8):
        for i in range(8):
            for a in range(3):
                for b in range(3):
                    W621[o, a:a + 9, b:b + 9] += W6[o, i, a, b] * W21[i] / s2[i]
    return W621


def test_tail_weights_prologue_bitwise_standalone(nconv_amd, gpu):
    net = make_net(nconv_amd, "generalized", gpu)
    S = torch.zeros(1, 1, 64, 96, device=gpu)
    a = _tail_weights(nconv_amd, net, S, prologue=True)
    b = _tail_weights(nconv_amd, net, S, prologue=False)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_tail_weights_values(nconv_amd, gpu):
    """The composed weights against a float64 recomputation (one fp32 ulp), the padding zero, and the
    re-laid phase weights bitwise nconv_phase_weights' [i][alpha][dh][o][beta][dw] values."""
    net = make_net(nconv_amd, "generalized", gpu)
    d = net.d_net
    S = torch.zeros(1, 1, 64, 96, device=gpu)
    layers = [getattr(d, n) for n in nconv_amd.dnet.LAYERS]
    wsum = d._prologue(layers, S)
    wt = _tail_weights(nconv_amd, net, S, prologue=False)
    got = _decode(wt)
    ref = _composed64(net, wsum[0], wsum[1])
    ref32 = ref.astype(np.float32).astype(np.float64)
    assert (np.abs(got - ref32) <= np.abs(ref32) * 2.0 ** -23).all(), np.abs(got - ref).max()
    assert (got > 0).all()  # positive weights compose to positive taps
    # padding of the fragments: part 3 rows and chunk 15's taps j >= 1 are zero
    bits = wt[:2048].cpu().numpy().view(np.uint16)
    e = np.arange(4096)
    j, l, ks = e & 7, (e >> 3) & 63, (e >> 9) & 3
    q = 4 * ks + (l >> 4)
    pad = ((l & 3) == 3) | ((q == 15) & (j != 0))
    assert (bits[pad] == 0).all()
    wph = d._phase_weights(gpu)[2].cpu()  # nconv6: [i][alpha][dh][o][beta][dw]
    re = wt[2048:].cpu().view(8, 2, 2, 8, 2, 2)  # [i][alpha][dh][o][dw][beta]
    assert torch.equal(re.permute(0, 1, 2, 3, 5, 4).reshape(-1), wph)


@pytest.mark.parametrize("B,H,W", [(2, 64, 96), (1, 96, 160), (2, 352, 1216)])
def test_composed_tail_matches_phase_tail(nconv_amd, gpu, B, H, W):
    """The eval forward with the composed tail against the phase tail (compose_tail False), and
    both against the float64 oracle (edge and interior tiles: 64 x 96 has both kinds)."""
    net = make_net(nconv_amd, "generalized", gpu)
    g = torch.Generator().manual_seed(H + W)
    S = sparse_depth(g, B, H, W).to(gpu)
    d = net.d_net
    assert d._use_tail_comp([getattr(d, n) for n in nconv_amd.dnet.LAYERS], S)
    with torch.no_grad():
        d.compose_tail = True
        a = net(S)
        d.compose_tail = False
        b = net(S)
        d.compose_tail = True
    if H >= 96:
        assert not torch.equal(a, b)  # (the composed path ran: its interior tiles round differently)
    err = (a - b).abs()
    assert (err <= 2e-6 * b.abs() + 1e-6).all(), err.max().item()
    if H * W <= 96 * 160:
        ref = R.dnet_forward(S.double().cpu(), oracle_params(net), "generalized")
        e64 = (a.double().cpu() - ref).abs()
        assert (e64 <= 1e-4 * ref.abs() + 1e-6).all(), e64.max().item()


def test_composed_tail_nan_and_dense_input(nconv_amd, gpu):
    """NaN depth samples (c0 = 0 there, the data sums NaN as the reference's) and 40 % density: the
    composed tail as the phase tail, NaN positions included."""
    net = make_net(nconv_amd, "generalized", gpu)
    g = torch.Generator().manual_seed(5)
    S = sparse_depth(g, 1, 96, 160, density=0.4)
    S[0, 0, 40, 70] = float("nan")
    S = S.to(gpu)
    d = net.d_net
    with torch.no_grad():
        a = net(S)
        d.compose_tail = False
        b = net(S)
        d.compose_tail = True
    assert torch.equal(torch.isnan(a), torch.isnan(b)) and torch.isnan(a).any()
    fin = ~torch.isnan(b)
    assert ((a - b).abs()[fin] <= 2e-6 * b.abs()[fin] + 1e-6).all()


def test_composed_tail_graph_and_split(nconv_amd, gpu):
    """The composed forward replays from a hipGraph and splits over streams bitwise."""
    net = make_net(nconv_amd, "generalized", gpu)
    g = torch.Generator().manual_seed(9)
    S = sparse_depth(g, 4, 96, 160).to(gpu)
    d = net.d_net
    with torch.no_grad():
        a = net(S)
        d.inference_streams = 1
        b = net(S)
        d.inference_streams = None
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            c = net(S)
        graph.replay()
        torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c)
