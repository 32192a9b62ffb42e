"""GPU parity of the guided model's training path: the dense autograd functions (dense.DenseConvFn,
dense.HeadFn — MFMA forward for any Cout, input gradient on re-arranged weights through the
cropped transposed / conv 4x4 s2 kinds, nconv_dense_conv_wgrad) against float64 PyTorch CPU
autograd of the same ops, and one whole SETP2_BP_TRAIN training step against the oracle
(oracle/nconv_ref.setp2_forward, training-mode BatchNorm) in float64.

Tolerances (normwise, max|gpu - ref| / max|ref| per tensor): 2e-5 for outputs and input gradients,
1e-4 for weight / bias gradients (fp32 sums over every pixel of the batch); whole training step:
outputs 1e-4 * |ref| + 1e-3 elementwise, gradients 1e-3 normwise."""
import pytest
import torch
import torch.nn.functional as F

from oracle import nconv_ref as R

pytestmark = pytest.mark.gpu


def _close(got, ref, what, tol):
    got = got.double().cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= tol * scale + 1e-12, f"{what}: max err {err:.3e} (ref max {scale:.3e}, tol {tol})"


# kind (0 3x3, 1 1x1, 2 ConvTranspose 4x4 s2), stride, C0, C1 (second source), Cout, H, W, relu, bias
CASES = [
    (0, 1, 32, 32, 32, 19, 45, True, True),     # ConvBlock fuse_conv1 on cat(rgb_feat, depth_feat)
    (0, 1, 64, 64, 64, 12, 40, False, False),   # UpCat conv 128 -> 64 (BatchNorm follows)
    (0, 1, 1, 0, 32, 13, 33, True, True),       # depth_conv 1 -> 32
    (0, 1, 64, 0, 64, 9, 70, True, True),       # rgb_conv 64 -> 64
    (0, 2, 32, 0, 64, 17, 43, False, True),     # encoder 3x3 s2, odd sizes (cropped transposed dgrad)
    (0, 2, 64, 0, 64, 16, 40, False, True),     # encoder 3x3 s2, even sizes
    (0, 1, 3, 0, 32, 16, 40, False, True),      # encoder0 3 -> 32
    (1, 1, 3, 0, 32, 11, 35, False, False),     # encoder0 shortcut 1x1
    (1, 2, 64, 0, 64, 15, 41, False, False),    # shortcut 1x1 s2, odd sizes
    (2, 2, 1, 64, 64, 7, 20, False, False),     # Basic2dTrans on cat(depth, features): 65 -> 64
    (2, 2, 1, 32, 32, 9, 19, False, True),      # 33 -> 32, with bias
    (0, 1, 32, 0, 1, 14, 37, False, False),     # 3x3 to one channel through the generic tiles
    (0, 1, 1, 32, 32, 11, 37, True, True),      # 33 input channels, the depth channel first (a chunk
                                                #   straddling the sources; two weight-gradient n-groups)
    (0, 2, 33, 0, 64, 13, 29, False, True),     # stride 2, 33 input channels, odd sizes
]


@pytest.mark.parametrize("math", ["bf16x9", "fp32", "bf16x6"])
@pytest.mark.parametrize("kind,stride,c0,c1,cout,H,W,relu,bias", CASES)
def test_dense_conv_fn_forward_backward(nconv_amd, gpu, monkeypatch, math, kind, stride, c0, c1, cout, H, W, relu,
                                        bias):
    """Forward, input and weight gradients under each nconv_dense_math (the split-bf16 weight
    gradient runs the 3x3 cases of >= 4 input channels)."""
    D = nconv_amd.dense
    monkeypatch.setattr(D, "MATH", math)
    g = torch.Generator().manual_seed(kind * 1000 + c0 * 10 + cout + H)
    B, cin = 2, c0 + c1
    x0 = torch.randn(B, c0, H, W, generator=g, dtype=torch.float64)
    x1 = torch.randn(B, c1, H, W, generator=g, dtype=torch.float64) if c1 else None
    if kind == 2:
        w = torch.randn(cin, cout, 4, 4, generator=g, dtype=torch.float64) * 0.1
    else:
        k = 3 if kind == 0 else 1
        w = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64) * 0.1
    b = torch.randn(cout, generator=g, dtype=torch.float64) if bias else None

    q = [t.to(gpu, torch.float32).requires_grad_(True) if t is not None else None for t in (x0, x1, w, b)]
    yg = D.conv_fn(q[0], q[2], q[3], kind, stride, relu=relu, x1=q[1])
    gy = torch.randn(yg.shape, generator=g, dtype=torch.float64)
    yg.backward(gy.to(gpu, torch.float32))
    torch.cuda.synchronize()

    r = [t.clone().requires_grad_(True) if t is not None else None for t in (x0, x1, w, b)]
    x = torch.cat([r[0], r[1]], 1) if c1 else r[0]
    if kind == 2:
        y = F.conv_transpose2d(x, r[2], r[3], 2, 1)
    else:
        y = F.conv2d(x, r[2], r[3], stride, r[2].shape[-1] // 2)
    if relu:  # the ReLU mask the GPU took (elements within rounding of 0 may differ)
        y = y * (yg.detach().double().cpu() > 0)
    y.backward(gy)
    _close(yg.detach(), y.detach(), "forward", 2e-5)
    for name, a, ref, tol in zip(("x0", "x1", "weight", "bias"), q, r, (2e-5, 2e-5, 1e-4, 1e-4)):
        if a is not None:
            _close(a.grad, ref.grad, f"grad {name}", tol)


def test_head_fn_forward_backward(nconv_amd, gpu):
    """depth + Conv3x3(fout) (step2.py:255-257) with its gradients."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(21)
    x, w, res = (torch.randn(2, 64, 21, 70, generator=g, dtype=torch.float64),
                 torch.randn(1, 64, 3, 3, generator=g, dtype=torch.float64) * 0.1,
                 torch.randn(2, 1, 21, 70, generator=g, dtype=torch.float64))
    q = [t.to(gpu, torch.float32).requires_grad_(True) for t in (x, w, res)]
    out = D.head_fn(*q)
    gy = torch.randn(out.shape, generator=g, dtype=torch.float64)
    out.backward(gy.to(gpu, torch.float32))
    r = [t.clone().requires_grad_(True) for t in (x, w, res)]
    ref = F.conv2d(r[0], r[1], padding=1) + r[2]
    ref.backward(gy)
    _close(out.detach(), ref.detach(), "forward", 2e-5)
    for name, a, b, tol in zip(("x", "w", "res"), q, r, (2e-5, 1e-4, 1e-7)):
        _close(a.grad, b.grad, f"grad {name}", tol)


def test_dense_conv_any_cout_and_conv4x4(nconv_amd, gpu):
    """Forward kernel with output-channel tiling (Cout 1, 3, 65, 128) and the Conv 4x4 s2 kind."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(5)
    for kind, cin, cout, H, W in ((0, 16, 3, 11, 30), (0, 32, 65, 10, 33), (0, 8, 128, 9, 40), (3, 32, 65, 13, 35),
                                  (3, 64, 33, 12, 40)):
        x = torch.randn(2, cin, H, W, generator=g, dtype=torch.float64)
        k = 3 if kind == 0 else 4
        w = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64) * 0.1
        bias = torch.randn(cout, generator=g, dtype=torch.float64)
        if kind == 0:
            ref = F.conv2d(x, w, bias, 1, 1)
        else:  # 4x4 s2 p1 with Ho = ceil(H / 2): an extra zero row / column at the far edge
            ref = F.conv2d(F.pad(x, (1, 2, 1, 2)), w, bias, 2)[:, :, :(H + 1) // 2, :(W + 1) // 2]
        f = lambda t: t.to(gpu, torch.float32).contiguous()
        got = D.conv(f(x), kind, 1 if kind == 0 else 2, D.pack(kind, f(w), cin, cout), f(bias), False, cout)
        torch.cuda.synchronize()
        assert got.shape == ref.shape
        _close(got, ref, f"kind {kind} cin {cin} cout {cout}", 2e-5)


def test_transposed_cropped_output(nconv_amd, gpu):
    """ConvTranspose 4x4 s2 p1 written into a (2H-1) x (2W-1) output (odd-size input gradients)."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 64, 9, 21, generator=g, dtype=torch.float64)
    w = torch.randn(64, 32, 4, 4, generator=g, dtype=torch.float64) * 0.1
    ref = F.conv_transpose2d(x, w, None, 2, 1)[:, :, :17, :41]
    f = lambda t: t.to(gpu, torch.float32).contiguous()
    out = torch.full((2, 32, 17, 41), 3.0, device=gpu)
    D.conv(f(x), D.DENSE_TRANSPOSED_4X4, 2, D.pack(D.DENSE_TRANSPOSED_4X4, f(w), 64, 32), None, False, 32, out=out)
    torch.cuda.synchronize()
    _close(out, ref, "cropped transposed", 2e-5)


@pytest.mark.parametrize("H,W", [(64, 96), (48, 80)])
def test_guided_training_step_matches_oracle(nconv_amd, gpu, H, W):
    """SETP2_BP_TRAIN train-mode forward (frozen, EnforcePos-drifted step 1; batch-statistics
    BatchNorm) + calculate_loss_multi_resolution (MSE, train_step2.py:21,64) + backward: every
    trainable gradient against the float64 oracle."""
    from guided_cases import f5_inputs
    torch.manual_seed(3)
    model = nconv_amd.SETP2_BP_TRAIN(None, step1_crop="generalized").to(gpu)
    with torch.no_grad():  # trained-like positive step-1 weights
        for n, p in model.step1.named_parameters():
            if n.endswith("weight") and "bnorm" not in n:
                p.copy_(F.softplus(p, beta=10))
    sd0 = {k: v.detach().double().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    rgb0, d0, rgb1, d1 = f5_inputs(H, W)
    g = torch.Generator().manual_seed(9)
    # calculate_loss_multi_resolution resizes every scale to 480x640 (utils.py:67): NYU-sized gt
    gt = (torch.rand(1, 1, 480, 640, generator=g) * 80) * (torch.rand(1, 1, 480, 640, generator=g) < 0.3)
    est, _ = model(rgb0.to(gpu), d0.to(gpu), rgb1.to(gpu), d1.to(gpu))
    loss = nconv_amd.train.calculate_loss_multi_resolution(est, gt.to(gpu), False)
    loss.backward()
    torch.cuda.synchronize()

    # oracle: step 1 with this forward's EnforcePos applied, step 2 trainable in float64
    sd = dict(sd0)
    for k in sd:
        if k.startswith("step1.") and k.endswith(".weight") and "bnorm" not in k:
            sd[k] = R.softplus_pos(sd[k])
    named = dict(model.named_parameters())
    leaves = {k: sd[k].clone().requires_grad_(True) for k, p in named.items()
              if p.requires_grad and not k.startswith("step1.") and not k.startswith("rgb_encoder4.")}
    sd.update(leaves)
    r0, _ = R.setp2_forward(sd, rgb0.double(), d0.double(), rgb1.double(), d1.double(), "generalized", "train",
                            training=True)
    R.calculate_loss_multi_resolution(r0, gt.double(), False).backward()
    for i in range(4):
        err = (est[i].detach().double().cpu() - r0[i].detach()).abs()
        assert (err <= 1e-4 * r0[i].detach().abs() + 1e-3).all(), f"scale {i}: max err {err.max():.3e}"
    bad = []
    for k, leaf in leaves.items():
        got = named[k].grad
        assert got is not None, f"{k}: no gradient"
        scale = leaf.grad.abs().max()
        if k.endswith("encoder.0.bias"):
            # a bias right before training-mode BatchNorm cancels out: its exact gradient is 0, so
            # measure the round-off against the same convolution's weight gradient instead
            scale = leaves[k[:-4] + "weight"].grad.abs().max()
        rel = ((got.double().cpu() - leaf.grad).abs().max() / scale.clamp_min(1e-30)).item()
        if rel > 1e-3:
            bad.append(f"{k}: {rel:.2e}")
    assert not bad, "\n".join(bad)
    assert named["rgb_encoder4.encoder.0.weight"].grad is None  # unused in forward (step2.py:46)


@pytest.mark.parametrize("B,C,H,W,relu", [(2, 32, 19, 45, True), (3, 64, 8, 10, False), (1, 33, 100, 130, True),
                                          # the bench's guided batch (4 frames per pair) at decoder sizes
                                          (4, 32, 352, 1216, True), (4, 128, 44, 152, False)])
def test_batchnorm_relu_train(nconv_amd, gpu, B, C, H, W, relu):
    """Training-mode BatchNorm2d (+ ReLU) against nn.BatchNorm2d in float64: output, running-stat
    update (momentum 0.1, unbiased variance), num_batches_tracked, and the three gradients."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(B * 100 + C)
    x = torch.randn(B, C, H, W, generator=g, dtype=torch.float64) * 3 + 1.5
    ref_bn = torch.nn.BatchNorm2d(C).double()
    with torch.no_grad():
        ref_bn.weight.uniform_(0.5, 1.5, generator=g)
        ref_bn.bias.uniform_(-0.5, 0.5, generator=g)
        ref_bn.running_mean.uniform_(-1, 1, generator=g)
        ref_bn.running_var.uniform_(0.5, 2, generator=g)
    bn = torch.nn.BatchNorm2d(C).to(gpu)
    bn.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref_bn.state_dict().items()})
    bn.train()
    ref_bn.train()
    xg = x.to(gpu, torch.float32).requires_grad_(True)
    y = D.bn_relu(xg, bn, relu)
    xr = x.clone().requires_grad_(True)
    yr = ref_bn(xr)
    yr = torch.relu(yr) if relu else yr
    if relu:  # the ReLU mask the GPU took
        yr = yr * (y.detach().double().cpu() > 0)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(gy.to(gpu, torch.float32))
    yr.backward(gy)
    torch.cuda.synchronize()
    _close(y.detach(), yr.detach(), "forward", 1e-5)
    _close(bn.running_mean, ref_bn.running_mean, "running_mean", 1e-5)
    _close(bn.running_var, ref_bn.running_var, "running_var", 1e-5)
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1
    _close(xg.grad, xr.grad, "grad x", 1e-4)
    _close(bn.weight.grad, ref_bn.weight.grad, "grad weight", 1e-4)
    _close(bn.bias.grad, ref_bn.bias.grad, "grad bias", 1e-4)


@pytest.mark.parametrize("B,C,H,W,relu", [(2, 32, 19, 45, True), (3, 64, 8, 10, False), (1, 5, 3, 7, True)])
def test_relu_bias_bwd(nconv_amd, gpu, B, C, H, W, relu):
    """nconv_relu_bias_bwd: g * (out > 0) bit-exact, per-channel sum of the masked gradient within
    1e-5 normwise of float64."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(B * 7 + C)
    gy = torch.randn(B, C, H, W, generator=g)
    out = torch.randn(B, C, H, W, generator=g).clamp_min(0)
    gg, og = gy.to(gpu), out.to(gpu)
    gm = torch.empty_like(gg) if relu else None
    gb = torch.empty(C, device=gpu)
    D.relu_bias_bwd(gg, og if relu else None, gm, gb)
    torch.cuda.synchronize()
    ref = gy.masked_fill(out <= 0, 0.0) if relu else gy
    if relu:
        assert torch.equal(gm.cpu(), ref)
    _close(gb, ref.double().sum(dim=(0, 2, 3)), "gbias", 1e-5)


@pytest.mark.parametrize("c0,c1,cout,H,W", [(1, 32, 32, 9, 19), (1, 64, 64, 7, 20), (32, 1, 32, 12, 33),
                                            (64, 1, 64, 5, 17), (2, 32, 32, 20, 41), (1, 32, 32, 44, 152)])
def test_transposed_wgrad_row_split(nconv_amd, gpu, c0, c1, cout, H, W, monkeypatch):
    """ConvTranspose2d weight gradient with the few channels beside whole 32-channel groups on the
    vector ALU (dense_wgrad_tr_rows; UpCat's cat(depth, features)): against float64 autograd (1e-4
    normwise) and against every row on the matrix cores (NCONV_WGD_TR_ROWS=0, 1e-5)."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(c0 * 100 + c1 + H)
    B = 2
    x0 = torch.randn(B, c0, H, W, generator=g, dtype=torch.float64)
    x1 = torch.randn(B, c1, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(c0 + c1, cout, 4, 4, generator=g, dtype=torch.float64) * 0.1
    gy = torch.randn(B, cout, 2 * H, 2 * W, generator=g, dtype=torch.float64)
    r = w.clone().requires_grad_(True)
    F.conv_transpose2d(torch.cat([x0, x1], 1), r, None, 2, 1).backward(gy)
    grads = {}
    for split in ("1", "0"):
        monkeypatch.setenv("NCONV_WGD_TR_ROWS", split)
        q = w.to(gpu, torch.float32).requires_grad_(True)
        y = D.conv_fn(x0.to(gpu, torch.float32), q, None, 2, 2, x1=x1.to(gpu, torch.float32))
        y.backward(gy.to(gpu, torch.float32))
        torch.cuda.synchronize()
        grads[split] = q.grad.detach().double().cpu()
        _close(grads[split], r.grad, f"weight gradient (split={split})", 1e-4)
    _close(grads["1"], grads["0"], "split vs matrix cores", 1e-5)
