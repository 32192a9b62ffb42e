"""CPU: the C-ABI library builds, loads after torch, and exports every entry point include/nconv.h
declares with the declared ABI version; descriptor validation rejects malformed calls before any
launch (no GPU needed: validation happens on the host)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nconv.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(nconv_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points(nconv_amd):
    assert set(header_functions()) == set(nconv_amd._lib.EXPORTED)


def test_library_exports_all_symbols(nconv_amd):
    lib = nconv_amd._lib.lib()
    for name in header_functions():
        assert hasattr(lib, name), f"libnconv.so does not export {name}"
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_abi_version_matches_header(nconv_amd):
    v = int(re.search(r"#define NCONV_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert nconv_amd._lib.lib().nconv_abi_version() == v == nconv_amd._lib.ABI_VERSION


def _layer(nconv_amd, **kw):
    L = nconv_amd._lib.NconvLayer()
    L.B, L.Cin, L.H, L.W, L.Cout, L.Ho, L.Wo = 1, 8, 16, 16, 8, 16, 16
    L.KH = L.KW = 5
    L.SH = L.SW = L.DH = L.DW = L.groups = 1
    L.PH = L.PW = 2
    L.eps = 1e-7
    L.load_mode = nconv_amd._lib.PLAIN
    fake = 0x1000  # never dereferenced: validation fails or passes on the host first
    L.a.x, L.a.c, L.a.C, L.a.H, L.a.W = fake, fake, 8, 16, 16
    L.weight = L.bias = L.wsum = fake
    for k, v in kw.items():
        setattr(L, k, v)
    return L


@pytest.mark.parametrize("bad,msg", [
    (dict(Ho=15), "Ho/Wo inconsistent"),
    (dict(groups=3), "groups"),
    (dict(load_mode=9), "unknown load mode"),
    (dict(Cin=4), "PLAIN"),
    (dict(weight=None), "null weight"),
])
def test_fwd_rejects_bad_descriptors(nconv_amd, bad, msg):
    lib = nconv_amd._lib.lib()
    L = _layer(nconv_amd, **bad)
    rc = lib.nconv_fwd(ctypes.byref(L), ctypes.c_void_p(0x2000), ctypes.c_void_p(0x3000), None)
    assert rc == -22
    assert msg in lib.nconv_last_error().decode()


def test_bwd_workspace_query_is_host_only(nconv_amd):
    lib = nconv_amd._lib.lib()
    L = _layer(nconv_amd)
    assert lib.nconv_bwd_workspace_bytes(ctypes.byref(L)) > 0
    bad = _layer(nconv_amd, Ho=3)
    assert lib.nconv_bwd_workspace_bytes(ctypes.byref(bad)) == 0


def test_product_path_refuses_cpu_tensors(nconv_amd):
    """No CPU fallback: the NConv modules compute only on the ROCm device and say so."""
    import torch
    net = nconv_amd.SETP1_NCONV()
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        net(torch.zeros(1, 1, 16, 16))
    layer = nconv_amd.NConv2d(8, 8, (5, 5))
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        layer(torch.zeros(1, 8, 8, 8), torch.zeros(1, 8, 8, 8))


def _wgrad_desc(nconv_amd, **kw):
    d = nconv_amd._lib.NconvDenseWgrad()
    fake = 0x1000  # never dereferenced
    d.B, d.kind, d.stride = 1, nconv_amd._lib.DENSE_3X3, 1
    d.x0, d.C0, d.x1, d.C1 = fake, 8, None, 0
    d.H = d.W = 16
    d.gy, d.Cout, d.Ho, d.Wo, d.gw = fake, 32, 16, 16, fake
    for k, v in kw.items():
        setattr(d, k, v)
    return d


@pytest.mark.parametrize("bad,msg", [
    (dict(kind=7), "unknown kind"),
    (dict(Ho=15), "Ho/Wo inconsistent"),
    (dict(stride=3), "stride"),
    (dict(kind=1, C0=65), "at most 64 input channels"),
    (dict(Cout=97), "at most 96 output channels"),
    (dict(kind=2, stride=2, Ho=33, Wo=32), "Ho/Wo inconsistent"),
    (dict(kind=2, stride=2, C0=97, Ho=32, Wo=32), "at most 96 input channels"),
    (dict(gw=None), "null pointer"),
])
def test_dense_wgrad_rejects_bad_descriptors(nconv_amd, bad, msg):
    lib = nconv_amd._lib.lib()
    d = _wgrad_desc(nconv_amd, **bad)
    assert lib.nconv_dense_wgrad_workspace_bytes(ctypes.byref(d)) == 0
    rc = lib.nconv_dense_conv_wgrad(ctypes.byref(d), None, 0, None)
    assert rc == -22
    assert msg in lib.nconv_last_error().decode()


def test_dense_wgrad_workspace_query_is_host_only(nconv_amd):
    lib = nconv_amd._lib.lib()
    for kw in (dict(), dict(stride=2, Ho=8, Wo=8), dict(kind=1), dict(kind=2, stride=2, C0=1, C1=64, Ho=31, Wo=32)):
        d = _wgrad_desc(nconv_amd, **kw)
        if kw.get("C1"):
            d.x1 = 0x2000
        assert lib.nconv_dense_wgrad_workspace_bytes(ctypes.byref(d)) > 0, kw


def test_dense_fwd_geometry_validation(nconv_amd):
    """Transposed output 2H or 2H-1 only; conv 4x4 s2 output ceil(H/2); any Cout >= 1."""
    L = nconv_amd._lib
    lib = L.lib()
    d = L.NconvDenseConv()
    d.B, d.x0, d.C0, d.x1, d.C1, d.H, d.W = 1, 0x1000, 8, None, 0, 10, 10
    d.Cout, d.kind, d.stride, d.wpack, d.out, d.out_C, d.out_c0 = 5, L.DENSE_TRANSPOSED_4X4, 2, 0x1000, 0x1000, 5, 0
    d.Ho, d.Wo = 21, 20
    assert lib.nconv_dense_conv_fwd(ctypes.byref(d), None) == -22
    assert "Ho/Wo inconsistent" in lib.nconv_last_error().decode()
    d.kind, d.Ho, d.Wo = L.DENSE_CONV4X4_S2, 6, 5
    assert lib.nconv_dense_conv_fwd(ctypes.byref(d), None) == -22
    d.Cout = 0
    assert lib.nconv_dense_conv_fwd(ctypes.byref(d), None) == -22
    assert "Cout" in lib.nconv_last_error().decode()


def test_depth_loss_validation_is_host_only(nconv_amd):
    """nconv_depth_loss_*: workspace query and argument checks (null planes, strides below W or
    overlapping images, short workspace, non-positive sizes) fail on the host with -22 before any
    launch; the loss on CPU tensors runs the reference's PyTorch ops, not the library."""
    import torch
    L = nconv_amd._lib
    lib = L.lib()
    ws_bytes = lib.nconv_depth_loss_workspace_bytes(1, 352, 1216)
    tiles = lambda B, H, W: B * -(-H // 16) * -(-W // 64)  # one partial triple per 16 x 64 tile
    assert ws_bytes >= (3 * tiles(1, 352, 1216) + 4) * 4
    assert lib.nconv_depth_loss_workspace_bytes(8, 352, 1216) >= (3 * tiles(8, 352, 1216) + 4) * 4
    assert lib.nconv_depth_loss_workspace_bytes(1, 0, 5) == 0
    assert lib.nconv_depth_loss_workspace_bytes(0, 5, 5) == 0
    p = ctypes.c_void_p(0x1000)
    ws2 = lib.nconv_depth_loss_workspace_bytes(2, 4, 8)
    # (r, r_image_stride, r_row_stride, t, t_image_stride, t_row_stride, B, H, W, grad, loss, ws, ws_bytes, stream)
    cases = [
        ((None, 32, 8, p, 32, 8, 1, 4, 8, 1, p, p, ws_bytes, None), "null plane"),
        ((p, 32, 7, p, 32, 8, 1, 4, 8, 1, p, p, ws_bytes, None), "row stride"),
        ((p, 32, 8, p, 32, 8, 1, 0, 8, 1, p, p, ws_bytes, None), "non-positive"),
        ((p, 32, 8, p, 32, 8, 0, 4, 8, 1, p, p, ws_bytes, None), "non-positive"),
        ((p, 31, 8, p, 32, 8, 2, 4, 8, 1, p, p, ws2, None), "image stride"),
        ((p, 32, 8, p, 32, 8, 1, 4, 8, 1, p, p, 4, None), "workspace too small"),
        ((p, 32, 8, p, 32, 8, 2, 4, 8, 1, p, p, ws2 - 4, None), "workspace too small"),
        ((p, 32, 8, p, 32, 8, 1, 4, 8, 1, None, p, ws_bytes, None), "null loss"),
    ]
    for args, msg in cases:
        assert lib.nconv_depth_loss_fwd(*args) == -22, msg
        assert msg in lib.nconv_last_error().decode()
    assert lib.nconv_depth_loss_bwd(p, 32, 8, p, 32, 8, 1, 4, 8, 1, None, p, ws_bytes, None, None) == -22
    assert "null g" in lib.nconv_last_error().decode()
    r = torch.rand(1, 6, 9) * 10
    t = (torch.rand(1, 6, 9) * 10) * (torch.rand(1, 6, 9) < 0.5)
    assert not nconv_amd.train._fused_loss_ok(r, t)
    got = nconv_amd.train.calculate_loss(r, t, True)
    assert torch.equal(got, nconv_amd.train._calculate_loss_torch(r, t, True))


def test_loss_plane_geometry(nconv_amd):
    """The batch geometry the fused loss accepts: (H, W), (1, H, W), (B, 1, H, W) incl. cropped views
    (row / image strides); several channels or a non-unit column stride are not loss planes."""
    import torch
    P = nconv_amd.train._planes
    assert P(torch.empty(5, 7)) == (1, 0, 7)
    assert P(torch.empty(1, 5, 7)) == (1, 0, 7)
    assert P(torch.empty(3, 1, 5, 7)) == (3, 35, 7)
    v = torch.empty(3, 1, 9, 11)[:, :, 1:6, 1:8]
    assert P(v) == (3, 99, 11)
    assert P(torch.empty(3, 2, 5, 7)) is None
    assert P(torch.empty(2, 5, 7)) is None
    assert P(torch.empty(7, 5).t()) is None


def test_fwd_rejects_unknown_math(nconv_amd):
    """nconv_layer.math outside enum nconv_math (e.g. a host struct without the field) is refused."""
    lib = nconv_amd._lib.lib()
    for m in (3, -1, 0x7fff):
        L = _layer(nconv_amd, math=m)
        assert lib.nconv_fwd(ctypes.byref(L), ctypes.c_void_p(0x2000), ctypes.c_void_p(0x3000), None) == -22
        assert "unknown math" in lib.nconv_last_error().decode()


def _plan(nconv_amd, L):
    lib = nconv_amd._lib.lib()
    f, d, w = ctypes.c_int(-1), ctypes.c_int(-1), ctypes.c_int(-1)
    rc = lib.nconv_plan(ctypes.byref(L), ctypes.byref(f), ctypes.byref(d), ctypes.byref(w))
    assert rc == 0, lib.nconv_last_error().decode()
    return tuple(nconv_amd._lib.KERNEL_NAMES[v.value] for v in (f, d, w))


def test_zero_math_is_exact_fp32(nconv_amd):
    """A descriptor whose math / bwd_math are left zero (ctypes zero-initialises, as `= {0}` in C)
    runs the reference's arithmetic: exact fp32 products forward and backward (include/nconv.h
    enum nconv_math; the reference's F.conv2d in fp32, models/step1.py:119-122)."""
    L = _layer(nconv_amd)
    assert (L.math, L.bwd_math) == (0, 0) == (nconv_amd._lib.MATH_FP32,) * 2
    assert _plan(nconv_amd, L) == ("tiled_fp32", "tiled_fp32", "mfma_fp32")


@pytest.mark.parametrize("math,expect", [
    ("fp32", ("tiled_fp32", "tiled_fp32", "mfma_fp32")),
    ("bf16x3", ("mfma_bf16x3", "mfma_bf16x3", "mfma_bf16x3")),
    ("bf16x9", ("mfma_bf16x9", "mfma_bf16x9", "mfma_bf16x9")),
])
def test_plan_follows_requested_math(nconv_amd, math, expect):
    """nconv_plan names the kernels a math selects, so a bf16 request can never silently run
    another arithmetic (tests/test_gpu_layers.py asserts the plan next to each parity check)."""
    m = nconv_amd.nconv._MATH_NAMES[math]
    assert _plan(nconv_amd, _layer(nconv_amd, math=m, bwd_math=m)) == expect
    # nconv1 (1 input channel) and the 1x1 nconv7 stay on the exact VALU / tiled kernels
    L1 = _layer(nconv_amd, Cin=1, load_mode=nconv_amd._lib.THRESH, math=m, bwd_math=m)
    L1.a.C = 1
    assert _plan(nconv_amd, L1) == ("tiled_fp32",) * 3
    L7 = _layer(nconv_amd, Cout=1, KH=1, KW=1, PH=0, PW=0, math=m, bwd_math=m)
    assert _plan(nconv_amd, L7) == ("tiled_fp32",) * 3
    # other geometries: the generic kernels whatever the math
    assert _plan(nconv_amd, _layer(nconv_amd, SH=2, SW=2, Ho=8, Wo=8, math=m, bwd_math=m)) == ("generic",) * 3


def test_weight_prologue_validation_is_host_only(nconv_amd):
    """nconv_weight_prologue rejects malformed arguments on the host with -22 before any launch."""
    lib = nconv_amd._lib.lib()
    P, I = ctypes.c_void_p, ctypes.c_int
    p = P(0x1000)
    w, s = (P * 1)(p), (P * 1)(p)
    cout, fan = (I * 1)(8), (I * 1)(25)
    pw, po = (P * 1)(p), (P * 1)(p)
    cin, up = (I * 1)(16), (I * 1)(8)
    cases = [
        ((-1, w, cout, fan, s, None, None, None, 0, None, None, None, None, None), "negative count"),
        ((1, None, cout, fan, s, None, None, None, 0, None, None, None, None, None), "null argument"),
        ((1, w, (I * 1)(0), fan, s, None, None, None, 0, None, None, None, None, None), "bad layer entry"),
        ((1, w, cout, fan, s, None, p, p, 0, None, None, None, None, None), "head_w1 and head_w2"),
        ((0, None, None, None, None, None, None, None, 1, None, cin, up, po, None), "null phase argument"),
        ((0, None, None, None, None, None, None, None, 1, pw, cin, (I * 1)(9), po, None), "outside [0, Cin)"),
    ]
    for args, msg in cases:
        assert lib.nconv_weight_prologue(*args) == -22, msg
        assert msg in lib.nconv_last_error().decode(), msg


def test_train_prologue_validation_is_host_only(nconv_amd):
    """nconv_train_prologue rejects malformed arguments on the host with -22 before any launch."""
    lib = nconv_amd._lib.lib()
    P, I = ctypes.c_void_p, ctypes.c_int
    p = P(0x1000)
    w2, s2 = (P * 2)(p, p), (P * 2)(p, p)
    cout2, fan2, sp2 = (I * 2)(8, 8), (I * 2)(25, 200), (I * 2)(1, 1)
    w1, s1, cout1, fan1 = (P * 1)(p), (P * 1)(p), (I * 1)(8), (I * 1)(144)
    pl, up, po = (I * 1)(0), (I * 1)(8), (P * 1)(p)
    SYNC = p
    cases = [
        ((-1, w2, cout2, fan2, sp2, s2, 0, 1, None, SYNC, 0, None, None, None, None), "negative count"),
        ((2, None, cout2, fan2, sp2, s2, 0, 1, None, SYNC, 0, None, None, None, None), "null argument"),
        ((2, w2, cout2, fan2, sp2, s2, 0, 0, p, SYNC, 0, None, None, None, None), "two distinct layer indices"),
        ((2, w2, cout2, (I * 2)(25, 144), sp2, s2, 0, 1, p, SYNC, 0, None, None, None, None), "must be nconv1"),
        ((2, w2, cout2, fan2, sp2, s2, 0, 1, p, None, 0, None, None, None, None), "need the sync counter"),
        ((1, w1, cout1, fan1, None, s1, -1, -1, None, SYNC, 1, None, up, po, None), "null phase argument"),
        ((1, w1, cout1, fan1, None, s1, -1, -1, None, SYNC, 1, (I * 1)(3), up, po, None), "bad phase entry"),
        ((1, w1, cout1, (I * 1)(200), None, s1, -1, -1, None, SYNC, 1, pl, up, po, None), "8 x 16 x 3 x 3"),
        ((1, w1, cout1, fan1, None, s1, -1, -1, None, SYNC, 1, pl, (I * 1)(4), po, None), "up_first must be 0 or 8"),
        ((2, (P * 2)(p, p), (I * 2)(8, 8), (I * 2)(144, 144), None, s2, -1, -1, None, SYNC, 2, (I * 2)(1, 1),
          (I * 2)(8, 8), (P * 2)(p, p), None), "listed twice"),
    ]
    for args, msg in cases:
        assert lib.nconv_train_prologue(*args, None) == -22, msg
        assert msg in lib.nconv_last_error().decode(), msg


def test_wgrad_reduce_ex_validation_is_host_only(nconv_amd):
    """nconv_wgrad_reduce_ex (layers + plain sums) rejects malformed arguments on the host."""
    lib = nconv_amd._lib.lib()
    P = ctypes.c_void_p
    p = P(0x1000)
    x, out, n = (P * 1)(p), (P * 1)(p), (ctypes.c_longlong * 1)(100)
    nbytes = lib.nconv_sum_workspace_bytes(1)
    assert nbytes == 1024 * 4 and lib.nconv_sum_workspace_bytes(0) == 0
    cases = [
        ((0, None, None, None, None, None, 0, None, None, None, None, 0), "1..16 layers and sums"),
        ((0, None, None, None, None, None, 17, x, n, out, p, 17 * nbytes), "1..16 layers and sums"),
        ((0, None, None, None, None, None, 1, None, n, out, p, nbytes), "null sum array"),
        ((0, None, None, None, None, None, 1, x, n, out, p, nbytes - 4), "sum workspace too small"),
        ((0, None, None, None, None, None, 1, x, (ctypes.c_longlong * 1)(-1), out, p, nbytes), "bad sum entry"),
        ((0, None, None, None, None, None, 1, (P * 1)(None), n, out, p, nbytes), "bad sum entry"),
    ]
    for args, msg in cases:
        assert lib.nconv_wgrad_reduce_ex(*args, None) == -22, msg
        assert msg in lib.nconv_last_error().decode(), msg
