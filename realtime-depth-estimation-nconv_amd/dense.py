"""Dense convolutions of the RGB-guided model on libnconv's matrix-core kernels (eval mode).

Host side of nconv_dense_conv_fwd / nconv_dense_pack / nconv_conv3x3_c1 (include/nconv.h): weight
packing with eval-BatchNorm folding, cached per module and rebuilt when a weight / BN tensor
changes (torch's in-place version counters), and the launch wrappers. Used by guided.py's
inference path; training keeps the PyTorch modules (BatchNorm batch statistics, autograd).
"""
import ctypes

import torch

from . import _lib
from ._lib import DENSE_1X1, DENSE_3X3, DENSE_TRANSPOSED_4X4  # noqa: F401  (re-exported)


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
    if kind == DENSE_TRANSPOSED_4X4:
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
    _lib.check(_lib.lib().nconv_dense_conv_fwd(ctypes.byref(d), _lib.stream_handle(x0.device)),
               "nconv_dense_conv_fwd")
    return out


def conv3x3_c1(x, w, res=None):
    """conv3x3(x; w (1, Cin, 3, 3), padding 1, no bias) + res."""
    B, C, H, W = x.shape
    out = torch.empty((B, 1, H, W), device=x.device, dtype=torch.float32)
    w = w.detach().contiguous()
    _lib.check(_lib.lib().nconv_conv3x3_c1(_lib.ptr(x), B, C, H, W, _lib.ptr(w), _lib.ptr(res), _lib.ptr(out),
                                           _lib.stream_handle(x.device)), "nconv_conv3x3_c1")
    return out
