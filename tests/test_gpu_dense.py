"""GPU parity of the matrix-core dense convolutions (dense_conv.hip via dense.py) against float64
PyTorch CPU references of the same modules (torch.nn.functional conv2d / conv_transpose2d, eval
BatchNorm): every kind / stride / output width, two-source (concatenated) inputs, channel-offset
outputs, the RGBEncoder shortcut, ragged sizes. Tolerance: max|gpu - ref| <= 2e-5 * max|ref| per
tensor (fp32 products are exact on MFMA; only the summation order differs)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _close(got, ref, what):
    got = got.double().cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 2e-5 * scale + 1e-12, f"{what}: max err {err:.3e} (ref max {scale:.3e})"


def _rand(g, *shape):
    return torch.randn(*shape, generator=g, dtype=torch.float64)


@pytest.mark.parametrize("kind,stride,cout,c0,c1,H,W", [
    (0, 1, 32, 5, 3, 13, 37),     # 3x3 s1, two sources, partial chunk, ragged tile edges
    (0, 1, 64, 64, 64, 20, 70),   # 3x3 s1 128 -> 64 (UpCat conv)
    (0, 1, 32, 1, 0, 9, 33),      # depth_conv (1 input channel)
    (0, 2, 64, 32, 0, 15, 41),    # 3x3 s2 (encoder), odd sizes
    (1, 1, 32, 8, 0, 11, 35),     # 1x1
    (1, 2, 64, 16, 0, 12, 40),    # 1x1 s2
    (2, 2, 32, 32, 1, 7, 19),     # ConvTranspose 4x4 s2 from cat(features, depth)
    (2, 2, 64, 1, 64, 6, 40),     # ConvTranspose with the 1-channel source first
    (3, 2, 33, 32, 0, 12, 40),    # Conv 4x4 s2 (the transposed convolution's input gradient)
    (3, 2, 64, 64, 1, 14, 38),    # ... 64-channel tile, two sources (even sizes: Ho = (H - 1) // 2 + 1 = H / 2)
])
@pytest.mark.parametrize("math", ["fp32", "bf16x9", "bf16x6"])
def test_dense_conv_kinds(nconv_amd, gpu, monkeypatch, math, kind, stride, cout, c0, c1, H, W):
    D = nconv_amd.dense
    monkeypatch.setattr(D, "MATH", math)
    g = torch.Generator().manual_seed(7 + kind * 10 + stride)
    B, cin = 2, c0 + c1
    x0, x1 = _rand(g, B, c0, H, W), (_rand(g, B, c1, H, W) if c1 else None)
    x = torch.cat([x0, x1], 1) if c1 else x0
    if kind == 2:
        w = _rand(g, cin, cout, 4, 4) * 0.1
        ref = F.conv_transpose2d(x, w, stride=2, padding=1)
    elif kind == 3:
        w = _rand(g, cout, cin, 4, 4) * 0.1
        ref = F.conv2d(x, w, stride=2, padding=1)
    else:
        k = 3 if kind == 0 else 1
        w = _rand(g, cout, cin, k, k) * 0.1
        ref = F.conv2d(x, w, stride=stride, padding=k // 2)
    bias = _rand(g, cout)
    scale = torch.rand(cout, generator=g, dtype=torch.float64) + 0.5
    ref = torch.relu(ref * scale.view(1, -1, 1, 1) + bias.view(1, -1, 1, 1))
    f = lambda t: None if t is None else t.to(gpu, torch.float32).contiguous()
    wp = D.pack(kind, f(w), cin, cout, f(scale))
    out_full = torch.full((B, cout + 8, ref.shape[2], ref.shape[3]), 7.0, device=gpu)
    D.conv(f(x0), kind, stride, wp, f(bias), True, cout, x1=f(x1), out=out_full, out_c0=8)
    torch.cuda.synchronize()
    assert torch.equal(out_full[:, :8].cpu(), torch.full((B, 8) + tuple(ref.shape[2:]), 7.0)), "wrote outside its channel range"
    _close(out_full[:, 8:], ref, f"kind {kind} stride {stride} cout {cout}")


@pytest.mark.parametrize("stride,cin,cout", [(1, 3, 32), (2, 32, 64), (2, 64, 64)])
def test_rgb_encoder_dense_matches_module(nconv_amd, gpu, stride, cin, cout):
    """RGBEncoder (step2.py:134-154) in eval mode with non-trivial BatchNorm statistics."""
    torch.manual_seed(stride * 100 + cin)
    enc = nconv_amd.guided.RGBEncoder(cin, cout, stride).double().eval()
    bn = enc.encoder[1]
    with torch.no_grad():
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(2, cin, 17, 45, dtype=torch.float64) * 50
    with torch.no_grad():
        ref = enc(x)
        got = enc.float().to(gpu).dense_forward(x.float().to(gpu))
    torch.cuda.synchronize()
    _close(got, ref, "RGBEncoder")


def test_conv3x3_c1_residual(nconv_amd, gpu):
    g = torch.Generator().manual_seed(3)
    x, w, res = _rand(g, 2, 64, 21, 70), _rand(g, 1, 64, 3, 3) * 0.1, _rand(g, 2, 1, 21, 70)
    ref = F.conv2d(x, w, padding=1) + res
    f = lambda t: t.to(gpu, torch.float32).contiguous()
    got = nconv_amd.dense.conv3x3_c1(f(x), f(w), f(res))
    torch.cuda.synchronize()
    _close(got, ref, "conv3x3_c1")


@pytest.mark.parametrize("H,W", [(64, 96), (96, 320)])
def test_guided_dense_path_matches_torch_modules(nconv_amd, gpu, H, W):
    """The whole SETP2 eval forward: dense kernels vs the PyTorch modules (same weights, BN with
    non-trivial running statistics), fp32 on the GPU both ways. Tolerance 1e-4 relative to the
    largest magnitude per scale (the torch path runs MIOpen's Winograd kernels)."""
    from guided_cases import f5_inputs
    torch.manual_seed(4)
    model = nconv_amd.SETP2_BP_EXPORT(step1_crop="generalized")
    with torch.no_grad():
        for mod in model.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    model = model.to(gpu).eval()
    ins = [t.to(gpu) for t in f5_inputs(H, W)]
    with torch.no_grad():
        got = nconv_amd.guided._guided_forward(model, *ins)
        model.dense_kernels = False
        ref = nconv_amd.guided._guided_forward(model, *ins)
    for i, (a, b) in enumerate(zip(got, ref)):
        err = (a - b).abs().max().item()
        assert err <= 1e-4 * b.abs().max().item() + 1e-5, f"scale {i}: max err {err:.3e}"


@pytest.mark.parametrize("H,W,k", [(352, 1216, 8), (352, 1216, 4), (352, 1216, 2), (352, 1216, 1), (480, 640, 8),
                                   (45, 67, 2), (96, 320, 8), (17, 9, 8)])
def test_bilinear_down_matches_cpu_interpolate(nconv_amd, gpu, H, W, k):
    """dense.bilinear_down (nconv_bilinear_ac) against the reference's own call on the CPU,
    F.interpolate(x, scale_factor=1/k, mode="bilinear", align_corners=True) (models/step2.py:249,277):
    same output size, and values within 2e-5 absolute (two ulps) on 0..80 planes (bitwise at the model's KITTI /
    NYU sizes; the CPU kernel's vectorised and scalar column paths round a few odd sizes' blends
    differently). The KITTI-width case checks the fp32 sampling position of the last column
    (1214.9999, not 1215) by an isolated value there."""
    g = torch.Generator().manual_seed(H * 7 + W + k)
    x = torch.rand(2, 3, H, W, generator=g) * 80
    x[:, :, :, -1] = 0.0  # a border ring next to large interior values, as DNET's output has
    ref = F.interpolate(x, scale_factor=1 / k, mode="bilinear", align_corners=True)
    got = nconv_amd.dense.bilinear_down(x.to(gpu), k).cpu()
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= 2e-5  # two fp32 ulps at 64..80
    if (H, W) in ((352, 1216), (480, 640)):
        assert torch.equal(got, ref)


@pytest.mark.parametrize("math", ["fp32", "bf16x9", "bf16x6"])
@pytest.mark.parametrize("cout,c0,c1,H,W", [
    (32, 16, 0, 13, 37),     # one source, ragged tile edges
    (64, 64, 64, 20, 70),    # 128 -> 64 from two sources (UpCat conv)
    (40, 24, 0, 11, 45),     # Cout padded to the 64-channel tile
    (96, 32, 8, 9, 33),      # three 32-channel tiles
    (32, 1, 0, 9, 33),       # depth_conv (1 input channel)
    (64, 8, 16, 17, 65),     # source boundary on a chunk boundary
])
def test_dense_3x3_split_maths(nconv_amd, gpu, math, monkeypatch, cout, c0, c1, H, W):
    """The 3x3 stride-1 convolution under each nconv_dense_math against float64, element-wise:
    |gpu - ref| <= 1e-6 * (|x| conv |w| + |bias|)  (fp32 accumulation of exact products, and bf16x6's
    dropped terms <= ~2^-23 of each product, both far inside; a wrong or missing term is not).
    The split maths also agree with the fp32-MFMA kernel to the same bound."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(11 + cout + c0)
    B, cin = 2, c0 + c1
    r32 = lambda t: t.float().double()  # the operands the GPU sees
    x0, x1 = r32(_rand(g, B, c0, H, W)), (r32(_rand(g, B, c1, H, W)) if c1 else None)
    x = torch.cat([x0, x1], 1) if c1 else x0
    w = r32(_rand(g, cout, cin, 3, 3) * 0.1)
    bias = r32(_rand(g, cout))
    ref = F.conv2d(x, w, padding=1) + bias.view(1, -1, 1, 1)
    bound = 1e-6 * (F.conv2d(x.abs(), w.abs(), padding=1) + bias.abs().view(1, -1, 1, 1)) + 1e-12
    f = lambda t: None if t is None else t.to(gpu, torch.float32).contiguous()
    outs = {}
    for m in ("fp32", math):
        monkeypatch.setattr(D, "MATH", m)
        wp = D.pack(0, f(w), cin, cout)
        outs[m] = D.conv(f(x0), 0, 1, wp, f(bias), False, cout, x1=f(x1)).double().cpu()
    got = outs[math]
    err = (got - ref).abs()
    assert (err <= bound).all(), f"{math}: worst err/bound {(err / bound).max().item():.3g}"
    assert ((got - outs["fp32"]).abs() <= 2 * bound).all()


@pytest.mark.parametrize("math", ["bf16x9", "bf16x6"])
def test_dense_3x3_split_maths_nan_spread(nconv_amd, gpu, math, monkeypatch):
    """A NaN input pixel makes exactly its 3x3 neighbourhood NaN in every output channel, as in the
    fp32 kernel: the padded tenth tap (zero weights) reads no data (its fragment is zeroed)."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 16, 12, 40, generator=g)
    x[0, 3, 5, 31] = float("nan")
    x[0, 0, 0, 0] = float("nan")
    w = torch.randn(32, 16, 3, 3, generator=g) * 0.1
    nan = {}
    for m in ("fp32", math):
        monkeypatch.setattr(D, "MATH", m)
        out = D.conv(x.to(gpu), 0, 1, D.pack(0, w.to(gpu), 16, 32), None, False, 32)
        nan[m] = torch.isnan(out).cpu()
    assert torch.equal(nan[math], nan["fp32"])
    assert nan[math][0, :, 4:7, 30:33].all() and int(nan[math].sum()) == 32 * (9 + 4)


@pytest.mark.parametrize("math", ["fp32", "bf16x9", "bf16x6"])
@pytest.mark.parametrize("stride,shortcut,cout,cin,H,W", [
    (2, False, 64, 32, 15, 41),   # the encoder's stride-2 3x3 (training path: no fused shortcut)
    (2, True, 64, 32, 15, 41),    # RGBEncoder eval: stride 2 with the fused 1x1 shortcut
    (2, True, 32, 16, 21, 70),    # 32-channel tile, odd sizes
    (1, True, 32, 3, 9, 33),      # rgb_encoder0: 3 input channels, stride 1 with shortcut
    (1, True, 64, 64, 12, 40),
])
def test_dense_3x3_split_maths_stride_shortcut(nconv_amd, gpu, math, monkeypatch, stride, shortcut, cout, cin, H, W):
    """relu(conv3x3_s(x) + b) [+ conv1x1_s(x)] under each nconv_dense_math against float64 of the same
    fp32 operands, element-wise at 1e-6 x (|x| conv |w| + |b| [+ |x| conv |ws|])."""
    D = nconv_amd.dense
    g = torch.Generator().manual_seed(31 + cout + cin + stride)
    r32 = lambda t: t.float().double()
    B = 2
    x = r32(_rand(g, B, cin, H, W))
    w = r32(_rand(g, cout, cin, 3, 3) * 0.1)
    ws = r32(_rand(g, cout, cin, 1, 1) * 0.1) if shortcut else None
    bias = r32(_rand(g, cout))
    ref = torch.relu(F.conv2d(x, w, stride=stride, padding=1) + bias.view(1, -1, 1, 1))
    bound = F.conv2d(x.abs(), w.abs(), stride=stride, padding=1) + bias.abs().view(1, -1, 1, 1)
    if shortcut:
        ref = ref + F.conv2d(x, ws, stride=stride)
        bound = bound + F.conv2d(x.abs(), ws.abs(), stride=stride)
    bound = 1e-6 * bound + 1e-12
    f = lambda t: None if t is None else t.to(gpu, torch.float32).contiguous()
    monkeypatch.setattr(D, "MATH", math)
    wp = D.pack(0, f(w), cin, cout)
    wsp = D.pack(1, f(ws), cin, cout) if shortcut else None
    got = D.conv(f(x), 0, stride, wp, f(bias), True, cout, wshort=wsp).double().cpu()
    assert got.shape == ref.shape
    err = (got - ref).abs()
    assert (err <= bound).all(), f"{math}: worst err/bound {(err / bound).max().item():.3g}"
