"""Dense convolutions of the RGB-guided model on libnconv's matrix-core kernels.

Host side of nconv_dense_conv_fwd / nconv_dense_pack / nconv_conv3x3_c1 / nconv_dense_conv_wgrad
(include/nconv.h):
  * inference (guided.py's eval path): weight packing with eval-BatchNorm folding, cached per
    module and rebuilt when a weight / BN tensor changes (torch's in-place version counters);
  * training (guided.py's train path): autograd functions for Conv2d 3x3 / 1x1 and
    ConvTranspose2d 4x4 s2 (+ bias, + fused ReLU, two-source input = the reference's torch.cat)
    and for the 3x3 -> 1 depth heads. Backward: the input gradient is the forward kernel on
    re-arranged weights (_dgrad_plan), the weight gradient nconv_dense_conv_wgrad, the bias
    gradient a reduction; training-mode BatchNorm (batch statistics + ReLU, forward and backward)
    on libnconv's nconv_bn_train_* / nconv_relu_bias_bwd kernels (bn_relu).
"""
import ctypes
import math
import os

import torch

from . import _lib
from ._lib import DENSE_1X1, DENSE_3X3, DENSE_CONV4X4_S2, DENSE_TRANSPOSED_4X4  # noqa: F401  (re-exported)


# Arithmetic of the convolutions other than the 1x1 (include/nconv.h enum nconv_dense_math): "bf16x9"
# (default: exact products on the bf16 matrix cores -- three-part split operands, all nine partial
# products, fp32 accumulation), "fp32" (v_mfma_f32_32x32x2_f32, exact products, an fmaf chain), or
# "bf16x6" (the six largest partial products: each product within ~2^-23 relative; opt-in,
# reported separately). The 1x1 always runs the fp32 MFMA kernel.
MATH = os.environ.get("NCONV_DENSE_MATH", "bf16x9")


def bn_fold(bn, conv_bias=None):
    """Eval BatchNorm after a convolution as (scale, shift): bn(conv(x) + b) = scale*conv(x) + shift."""
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    shift = bn.bias - bn.running_mean * scale
    if conv_bias is not None:
        shift = shift + conv_bias * scale
    return scale.detach().contiguous(), shift.detach().contiguous()


def pack(kind, w, cin, cout, scale=None):
    """Packed weights for nconv_dense_conv_fwd (Conv2d (Cout,Cin,k,k) / ConvTranspose2d (Cin,Cout,4,4))."""
    L = _lib.lib()
    w = w.detach().contiguous()
    out = torch.empty(L.nconv_dense_packed_floats(kind, cin, cout), device=w.device, dtype=torch.float32)
    _lib.check(L.nconv_dense_pack(kind, cin, cout, _lib.ptr(w), _lib.ptr(scale), _lib.ptr(out),
                                  _lib.stream_handle(w.device)), "nconv_dense_pack")
    return out


def cached(mod, name, tensors, build):
    """build() once per (module, name) until one of `tensors` is replaced or modified in place."""
    key = tuple((t.data_ptr(), t._version) for t in tensors)
    cache = mod.__dict__.setdefault("_dense_plans", {})
    ent = cache.get(name)
    if ent is None or ent[0] != key:
        ent = (key, build())
        cache[name] = ent
    return ent[1]


def conv(x0, kind, stride, wpack, bias, relu, cout, x1=None, wshort=None, out=None, out_c0=0):
    """[relu](conv(cat(x0, x1)) + bias) [+ shortcut]; written to out[:, out_c0:out_c0+cout] if out is given."""
    B, C0, H, W = x0.shape
    C1 = 0 if x1 is None else x1.shape[1]
    if out is not None:  # (a transposed convolution may write a cropped 2H-1 x 2W-1 output)
        Ho, Wo = out.shape[2], out.shape[3]
    elif kind == DENSE_TRANSPOSED_4X4:
        Ho, Wo = 2 * H, 2 * W
    else:
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    if out is None:
        out = torch.empty((B, cout, Ho, Wo), device=x0.device, dtype=torch.float32)
    d = _lib.NconvDenseConv()
    d.B, d.x0, d.C0 = B, x0.data_ptr(), C0
    d.x1, d.C1 = (x1.data_ptr() if x1 is not None else None), C1
    d.H, d.W, d.Cout, d.Ho, d.Wo = H, W, cout, Ho, Wo
    d.kind, d.stride = kind, stride
    d.wpack = wpack.data_ptr()
    d.bias = bias.data_ptr() if bias is not None else None
    d.relu = 1 if relu else 0
    d.wshort = wshort.data_ptr() if wshort is not None else None
    d.out, d.out_C, d.out_c0 = out.data_ptr(), out.shape[1], out_c0
    d.math = _lib.DENSE_MATHS[MATH]
    if B == 0:
        return out
    _lib.check(_lib.lib().nconv_dense_conv_fwd(ctypes.byref(d), _lib.stream_handle(x0.device)),
               "nconv_dense_conv_fwd")
    return out


def bilinear_down(x, k):
    """F.interpolate(x, scale_factor=1/k, mode="bilinear", align_corners=True) (models/step2.py:249,
    277) on libnconv's nconv_bilinear_ac, whose sampling arithmetic is the reference CPU kernel's
    (fp32 positions: PyTorch-ROCm's own kernel samples KITTI's last column elsewhere, include/nconv.h).
    Output size floor(H / k) x floor(W / k) as F.interpolate's. A tensor that records autograd (step 1
    frozen in SETP2, so never on the model's path) goes through F.interpolate for its backward."""
    if torch.is_grad_enabled() and x.requires_grad:
        return torch.nn.functional.interpolate(x, scale_factor=1 / k, mode="bilinear", align_corners=True)
    x = x.contiguous()
    B, C, H, W = x.shape
    Ho, Wo = int(math.floor(H * (1.0 / k))), int(math.floor(W * (1.0 / k)))
    out = torch.empty((B, C, Ho, Wo), device=x.device, dtype=torch.float32)
    if out.numel():
        _lib.check(_lib.lib().nconv_bilinear_ac(_lib.ptr(x), B, C, H, W, _lib.ptr(out), Ho, Wo,
                                                _lib.stream_handle(x.device)), "nconv_bilinear_ac")
    return out


def conv3x3_c1(x, w, res=None):
    """conv3x3(x; w (1, Cin, 3, 3), padding 1, no bias) + res."""
    B, C, H, W = x.shape
    out = torch.empty((B, 1, H, W), device=x.device, dtype=torch.float32)
    w = w.detach().contiguous()
    _lib.check(_lib.lib().nconv_conv3x3_c1(_lib.ptr(x), B, C, H, W, _lib.ptr(w), _lib.ptr(res), _lib.ptr(out),
                                           _lib.stream_handle(x.device)), "nconv_conv3x3_c1")
    return out


# ------------------------------------------------------------------------------------------------
# Training: autograd functions
# ------------------------------------------------------------------------------------------------
def _dgrad_plan(weight, kind, stride):
    """The input gradient of conv(x; weight) as another convolution of dL/dy on the same kernels:
    (kind', stride', weight' in kind's layout, Cin', Cout').
      3x3 / 1x1 stride 1: the transposed, flipped kernel (Ci, Co, k, k), same geometry;
      3x3 / 1x1 stride 2: ConvTranspose 4x4 s2 p1 whose (Co, Ci, 4, 4) kernel embeds the 3x3
                          kernel at [0:3, 0:3] (the 1x1 at [1, 1]), output cropped to H x W;
      ConvTranspose 4x4 s2 p1 (Ci, Co, 4, 4): Conv 4x4 s2 p1 with the same tensor read as a
                          (Cout' = Ci, Cin' = Co) Conv2d weight."""
    w = weight.detach()
    if kind == DENSE_TRANSPOSED_4X4:
        return DENSE_CONV4X4_S2, 2, w.contiguous(), w.shape[1], w.shape[0]
    co, ci = w.shape[0], w.shape[1]
    if stride == 1:
        return kind, 1, w.transpose(0, 1).flip(2, 3).contiguous(), co, ci
    w4 = w.new_zeros((co, ci, 4, 4))
    if kind == DENSE_3X3:
        w4[:, :, :3, :3] = w
    else:
        w4[:, :, 1, 1] = w[:, :, 0, 0]
    return DENSE_TRANSPOSED_4X4, 2, w4, co, ci


def dgrad(g, weight, kind, stride, in_shape):
    """dL/dx (B, Cin, H, W) of conv(x; weight) from g = dL/dy (contiguous)."""
    k2, s2, w2, cin2, cout2 = _dgrad_plan(weight, kind, stride)
    B, _, H, W = in_shape
    out = torch.empty((B, cout2, H, W), device=g.device, dtype=torch.float32)
    return conv(g, k2, s2, pack(k2, w2, cin2, cout2), None, False, cout2, out=out)


def wgrad(x0, x1, g, kind, stride, wshape):
    """dL/dW of conv(cat(x0, x1); W) from g = dL/dy (nconv_dense_conv_wgrad; deterministic)."""
    L = _lib.lib()
    d = _lib.NconvDenseWgrad()
    d.B, d.kind, d.stride = x0.shape[0], kind, stride
    d.x0, d.C0 = x0.data_ptr(), x0.shape[1]
    d.x1, d.C1 = (x1.data_ptr(), x1.shape[1]) if x1 is not None else (None, 0)
    d.H, d.W = x0.shape[2], x0.shape[3]
    d.gy, d.Cout, d.Ho, d.Wo = g.data_ptr(), g.shape[1], g.shape[2], g.shape[3]
    gw = torch.empty(wshape, device=x0.device, dtype=torch.float32)
    d.gw = gw.data_ptr()
    d.math = _lib.DENSE_MATHS[MATH]
    nbytes = L.nconv_dense_wgrad_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(max(nbytes, 4) // 4, device=x0.device, dtype=torch.float32)
    _lib.check(L.nconv_dense_conv_wgrad(ctypes.byref(d), _lib.ptr(ws), nbytes, _lib.stream_handle(x0.device)),
               "nconv_dense_conv_wgrad")
    return gw


def relu_bias_bwd(g, out, g_masked, gbias):
    """g_masked = g * (out > 0) (out given), gbias = sum of the (masked) gradient per channel."""
    B, C, H, W = g.shape
    L = _lib.lib()
    nb = L.nconv_relu_bias_bwd_workspace_bytes(B, C, H, W)
    ws = torch.empty(max(nb, 4) // 4, device=g.device, dtype=torch.float32)
    _lib.check(L.nconv_relu_bias_bwd(B, C, H, W, _lib.ptr(g), _lib.ptr(out), _lib.ptr(g_masked), _lib.ptr(gbias),
                                     _lib.ptr(ws), nb, _lib.stream_handle(g.device)), "nconv_relu_bias_bwd")


# The training backward's weight gradient on a side stream, concurrent with the same layer's input
# gradient(s), joined before the node returns (1; 0 = serial). Joining once at the end of the
# backward pass measured slower (43.3 -> 44.0 ms per guided step, profiles/r5_ab_guided_wgrad_join.log)
WGRAD_STREAM = int(os.environ.get("NCONV_DENSE_WGRAD_STREAM", "1"))
_WGRAD_STREAMS = {}


def _wgrad_stream(device):
    if device.index not in _WGRAD_STREAMS:
        _WGRAD_STREAMS[device.index] = torch.cuda.Stream(device=device)
    return _WGRAD_STREAMS[device.index]


class DenseConvFn(torch.autograd.Function):
    """y = [relu](conv(cat(x0, x1); weight) + bias) for Conv2d 3x3 pad 1 / 1x1 (stride 1 | 2) and
    ConvTranspose2d 4x4 s2 p1 — nn.Conv2d / nn.ConvTranspose2d (+ ReLU, + the torch.cat before
    them) of models/step2.py — forward and backward on libnconv's MFMA kernels."""

    @staticmethod
    def forward(ctx, x0, x1, weight, bias, kind, stride, relu):
        x0 = x0.contiguous()
        x1 = x1.contiguous() if x1 is not None else None
        cin = x0.shape[1] + (0 if x1 is None else x1.shape[1])
        cout = weight.shape[1] if kind == DENSE_TRANSPOSED_4X4 else weight.shape[0]
        wp = pack(kind, weight, cin, cout)
        b = bias.detach().contiguous() if bias is not None else None
        out = conv(x0, kind, stride, wp, b, relu, cout, x1=x1)
        ctx.kind, ctx.stride, ctx.relu, ctx.c0 = kind, stride, relu, x0.shape[1]
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x0, x1, weight, out if relu else None)
        return out

    @staticmethod
    def backward(ctx, g):
        x0, x1, weight, out = ctx.saved_tensors
        g = g.contiguous()
        need = ctx.needs_input_grad
        gx0 = gx1 = gw = gb = None
        if ctx.relu or (ctx.has_bias and need[3]):
            # ReLU backward (gradient where the output is positive) and the bias gradient, one pass
            gb = torch.empty(g.shape[1], device=g.device, dtype=torch.float32) if ctx.has_bias and need[3] else None
            gm = torch.empty_like(g) if ctx.relu else None
            relu_bias_bwd(g, out if ctx.relu else None, gm, gb)
            g = gm if ctx.relu else g
        # input gradient per source: the forward weight's input-channel slice of each source, so
        # each gradient is written contiguous (no split / copy of a concatenated gradient)
        co = ctx.c0
        tr = ctx.kind == DENSE_TRANSPOSED_4X4
        w = weight.detach()
        side = None
        if need[2] and WGRAD_STREAM and (need[0] or (x1 is not None and need[1])):
            cur, side = torch.cuda.current_stream(g.device), _wgrad_stream(g.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                gw = wgrad(x0, x1, g, ctx.kind, ctx.stride, weight.shape)
        if need[0]:
            w0 = w if x1 is None else (w[:co] if tr else w[:, :co])
            gx0 = dgrad(g, w0, ctx.kind, ctx.stride, x0.shape)
        if x1 is not None and need[1]:
            gx1 = dgrad(g, w[co:] if tr else w[:, co:], ctx.kind, ctx.stride, x1.shape)
        if side is not None:
            cur.wait_stream(side)
            gw.record_stream(cur)  # (made on the side stream, read on this one)
        elif need[2]:
            gw = wgrad(x0, x1, g, ctx.kind, ctx.stride, weight.shape)
        return gx0, gx1, gw, gb, None, None, None


def conv_fn(x0, weight, bias, kind, stride, relu=False, x1=None):
    """Differentiable [relu](conv(cat(x0, x1)) + bias) (see DenseConvFn)."""
    if not x0.is_cuda:
        raise RuntimeError("nconv_amd dense convolutions compute on ROCm devices only")
    return DenseConvFn.apply(x0, x1, weight, bias, kind, stride, relu)


class HeadFn(torch.autograd.Function):
    """res + conv3x3(x; w (1, Cin, 3, 3), pad 1) — the depth heads `dout = depth + self.conv(fout)`
    (models/step2.py:255-257, 274-276); backward on the dense kernels (dgrad: 3x3 kernel with
    Cout' = Cin; wgrad: M = 1)."""

    @staticmethod
    def forward(ctx, x, w, res):
        x = x.contiguous()
        out = conv3x3_c1(x, w, res.contiguous())
        ctx.save_for_backward(x, w)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous()
        need = ctx.needs_input_grad
        gx = dgrad(g, w, DENSE_3X3, 1, x.shape) if need[0] else None
        gw = wgrad(x, None, g, DENSE_3X3, 1, w.shape) if need[1] else None
        return gx, gw, (g if need[2] else None)


def head_fn(x, w, res):
    return HeadFn.apply(x, w, res)


# ------------------------------------------------------------------------------------------------
# Training-mode BatchNorm2d + ReLU (nconv_bn_train_fwd / _bwd)
# ------------------------------------------------------------------------------------------------
def _bn_desc(x, bn, relu, y=None, mean=None, invstd=None, update=True):
    d = _lib.NconvBnTrain()
    d.B, d.C, d.H, d.W = x.shape
    d.x = x.data_ptr()
    d.gamma = bn.weight.data_ptr() if bn.weight is not None else None
    d.beta = bn.bias.data_ptr() if bn.bias is not None else None
    track = update and bn.track_running_stats and bn.running_mean is not None
    d.running_mean = bn.running_mean.data_ptr() if track else None
    d.running_var = bn.running_var.data_ptr() if track else None
    if bn.momentum is None:  # cumulative moving average (num_batches_tracked already incremented)
        d.momentum = 1.0 / float(bn.num_batches_tracked.item()) if track else 0.0
    else:
        d.momentum = bn.momentum
    d.eps = bn.eps
    d.relu = 1 if relu else 0
    d.y = y.data_ptr() if y is not None else None
    d.mean, d.invstd = mean.data_ptr(), invstd.data_ptr()
    return d


class BatchNormReLUFn(torch.autograd.Function):
    """[relu](BatchNorm2d(x)) with batch statistics (module in training mode): the forward
    updates bn.running_mean / running_var / num_batches_tracked like nn.BatchNorm2d."""

    @staticmethod
    def forward(ctx, x, weight, bias, bn, relu):
        x = x.contiguous()
        C = x.shape[1]
        mean = torch.empty(C, device=x.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        y = torch.empty_like(x)
        if bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
        d = _bn_desc(x, bn, relu, y, mean, invstd)
        L = _lib.lib()
        nb = L.nconv_bn_workspace_bytes(ctypes.byref(d))
        ws = torch.empty(max(nb, 4) // 4, device=x.device, dtype=torch.float32)
        _lib.check(L.nconv_bn_train_fwd(ctypes.byref(d), _lib.ptr(ws), nb, _lib.stream_handle(x.device)),
                   "nconv_bn_train_fwd")
        ctx.bn, ctx.relu = bn, relu
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, bias, mean, invstd = ctx.saved_tensors
        g = g.contiguous()
        need = ctx.needs_input_grad
        gx = torch.empty_like(x) if need[0] else None
        gw = torch.empty_like(weight) if (weight is not None and need[1]) else None
        gb = torch.empty_like(bias) if (bias is not None and need[2]) else None
        d = _bn_desc(x, ctx.bn, ctx.relu, None, mean, invstd, update=False)
        L = _lib.lib()
        nb = L.nconv_bn_workspace_bytes(ctypes.byref(d))
        ws = torch.empty(max(nb, 4) // 4, device=x.device, dtype=torch.float32)
        _lib.check(L.nconv_bn_train_bwd(ctypes.byref(d), _lib.ptr(g), _lib.ptr(gx), _lib.ptr(gw), _lib.ptr(gb),
                                        _lib.ptr(ws), nb, _lib.stream_handle(x.device)), "nconv_bn_train_bwd")
        return gx, gw, gb, None, None


def bn_relu(x, bn, relu):
    """[relu](bn(x)) for an nn.BatchNorm2d: libnconv kernels in training mode (batch statistics),
    the module itself (running statistics) otherwise."""
    if bn.training or not bn.track_running_stats:
        return BatchNormReLUFn.apply(x, bn.weight, bn.bias, bn, relu)
    y = bn(x)
    return torch.relu(y) if relu else y
