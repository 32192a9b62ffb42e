"""NConv2d / EnforcePos — drop-in for the reference's models/step1.py:97-212, computed by libnconv.

`NConv2d` keeps the reference's constructor signature, parameter names, RNG consumption and
state_dict layout (weight, bias, and the unused-but-saved bnorm.*), and its forward(data, conf)
returns (nconv, cout) like step1.py:116-149. The arithmetic runs in hand-written gfx950 kernels
through the C ABI (include/nconv.h); there is no PyTorch or CPU fallback for it.
"""
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.modules.conv import _ConvNd
from torch.nn.modules.utils import _pair

from . import _lib, export


# Arithmetic of the forward sums N = W*(x*c), D = W*c (include/nconv.h enum nconv_math): "fp32"
# (default: exact fp32 products on the vector ALU, as the reference's F.conv2d), "bf16x9" (exact
# products on the matrix cores: both operands split into three bf16 parts, an exact
# decomposition, all nine partial products accumulated in fp32) or "bf16x3" (split-bf16 products,
# <= ~1.1e-5 relative per product). With either matrix-core math a NaN input may spread one row
# further than in the reference. NCONV_FWD_MATH selects it; tests switch this global.
_MATH_NAMES = {"bf16x3": _lib.MATH_BF16X3, "fp32": _lib.MATH_FP32, "bf16x9": _lib.MATH_BF16X9}
FORWARD_MATH = _MATH_NAMES[os.environ.get("NCONV_FWD_MATH", "fp32")]
# Arithmetic of the backward's products, weight and input gradient of the 3x3 / 5x5 layers with
# several input channels (include/nconv.h nconv_layer.bwd_math): "fp32" (default: exact fp32
# products — fp32 matrix cores for the weight gradient, packed fp32 on the vector ALU for the input
# gradient), "bf16x3" (split-bf16 matrix cores, ~1e-5 relative per product, inside the backward's
# 1e-3 normwise tolerance) or "bf16x9" (exact products on the bf16 matrix cores).
# NCONV_BWD_MATH selects it; tests switch this global.
BACKWARD_MATH = _MATH_NAMES[os.environ.get("NCONV_BWD_MATH", "fp32")]


def _require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(
            f"{what}: nconv_amd computes on ROCm devices only (got a {t.device} tensor); "
            "move the module and inputs to the GPU")
    if t.dtype != torch.float32:
        raise TypeError(f"{what}: expected float32, got {t.dtype} (the reference is fp32-only, step1.py:53)")


@dataclass(frozen=True)
class LayerSpec:
    """Geometry + glue of one fused NConv application (mirrors struct nconv_layer)."""
    cin: int
    cout: int
    kernel: Tuple[int, int]
    stride: Tuple[int, int] = (1, 1)
    padding: Tuple[int, int] = (0, 0)
    dilation: Tuple[int, int] = (1, 1)
    groups: int = 1
    eps: float = 1e-7
    mode: int = _lib.PLAIN
    thresh: float = 0.01

    def in_hw(self, a_shape, b_shape=None):
        H, W = a_shape[2], a_shape[3]
        if self.mode == _lib.POOL2:
            return H // 2, W // 2
        return H, W

    def out_hw(self, H, W):
        kh, kw = self.kernel
        ho = (H + 2 * self.padding[0] - self.dilation[0] * (kh - 1) - 1) // self.stride[0] + 1
        wo = (W + 2 * self.padding[1] - self.dilation[1] * (kw - 1) - 1) // self.stride[1] + 1
        return ho, wo

    def descriptor(self, xa, ca, xb, cb, weight, bias, wsum, waux=None):
        H, W = self.in_hw(xa.shape)
        Ho, Wo = self.out_hw(H, W)
        L = _lib.NconvLayer()
        L.B, L.Cin, L.H, L.W = xa.shape[0], self.cin, H, W
        L.Cout, L.Ho, L.Wo = self.cout, Ho, Wo
        L.KH, L.KW = self.kernel
        L.SH, L.SW = self.stride
        L.PH, L.PW = self.padding
        L.DH, L.DW = self.dilation
        L.groups = self.groups
        L.eps = self.eps
        L.load_mode = self.mode
        L.thresh = self.thresh
        L.a = _lib.src(xa, ca)
        L.b = _lib.src(xb, cb)
        L.weight = weight.data_ptr()
        L.bias = bias.data_ptr() if bias is not None else None
        L.wsum = wsum.data_ptr() if wsum is not None else None
        L.math = FORWARD_MATH
        L.bwd_math = BACKWARD_MATH
        L.waux = waux.data_ptr() if waux is not None else None
        return L


def weight_prep(weights, softplus_flags, wsums):
    """One launch: optional in-place softplus (EnforcePos) + s[o] = sum(W[o]) for each layer."""
    n = len(weights)
    if n == 0:
        return
    dev = weights[0].device
    ptrs = _lib.ctypes.c_void_p * n
    ints = _lib.ctypes.c_int * n
    wp = ptrs(*[w.data_ptr() for w in weights])
    sp = ptrs(*[s.data_ptr() for s in wsums])
    couts = ints(*[w.shape[0] for w in weights])
    fans = ints(*[w[0].numel() for w in weights])
    flags = ints(*[1 if f else 0 for f in softplus_flags])
    rc = _lib.lib().nconv_weight_prep(n, wp, couts, fans, flags, sp, _lib.stream_handle(dev))
    _lib.check(rc, "nconv_weight_prep")


def _outputs(out, n, shapes, device, dtypes=None):
    """The launch's output tensors: fresh (out None), the caller's (a sequence), or from a callable
    out(shapes, dtypes, device) -> tensors (e.g. batch rows of full-batch tensors, dnet's split
    training forward)."""
    dtypes = dtypes or [torch.float32] * n
    if out is None:
        return [torch.empty(sh, device=device, dtype=dt) for sh, dt in zip(shapes, dtypes)]
    if callable(out):
        return list(out(shapes, dtypes, device))
    if len(out) != n or any(tuple(t.shape) != tuple(sh) or not t.is_contiguous() or t.dtype != torch.float32
                            for t, sh in zip(out, shapes)):
        raise ValueError("out= tensors must be contiguous fp32 of the layer's output shapes")
    return list(out)


PHASE_WEIGHT_FLOATS = 1024  # one UpCat layer's phase-weight buffer (nconv_phase_weights_floats)


def phase_weights(weights, up_first, outs):
    """nconv_phase_weights: one launch filling outs[i] (PHASE_WEIGHT_FLOATS floats) with the phase weights of the
    UPCAT layer whose (8, Cin, 3, 3) weight is weights[i] and whose upsampled channels start at
    up_first[i], from the current weights (after weight_prep)."""
    n = len(weights)
    if n == 0:
        return
    for o in outs:
        if o.numel() < PHASE_WEIGHT_FLOATS or not o.is_contiguous() or o.dtype != torch.float32:
            raise ValueError(f"phase-weight buffers need {PHASE_WEIGHT_FLOATS} contiguous fp32 elements")
    P, I = _lib.ctypes.c_void_p * n, _lib.ctypes.c_int * n
    rc = _lib.lib().nconv_phase_weights(n, P(*[w.data_ptr() for w in weights]), I(*[w.shape[1] for w in weights]),
                                        I(*up_first), P(*[o.data_ptr() for o in outs]),
                                        _lib.stream_handle(outs[0].device))
    _lib.check(rc, "nconv_phase_weights")


def weight_prologue(weights, wsums, head=None, phase=None):
    """nconv_weight_prologue: the eval-mode weight prologue in one launch, bitwise what
    weight_prep(weights, [False] * n, wsums) + head_weights + phase_weights write.
    head: (w1, w2, out) -- nconv1 (8, 1, 5, 5), nconv2 (8, 8, 5, 5), HEAD_WEIGHTS_FLOATS out -- or
    None; phase: (weights, up_first, outs) as phase_weights' arguments, or None."""
    n = len(weights)
    w1, w2, w21 = head if head is not None else (None, None, None)
    pw, pup, pout = phase if phase is not None else ([], [], [])
    if w21 is not None and (w21.numel() < HEAD_WEIGHTS_FLOATS or not w21.is_contiguous() or
                            w21.dtype != torch.float32):
        raise ValueError(f"head-weight buffer needs {HEAD_WEIGHTS_FLOATS} contiguous fp32 elements")
    for o in pout:
        if o.numel() < PHASE_WEIGHT_FLOATS or not o.is_contiguous() or o.dtype != torch.float32:
            raise ValueError(f"phase-weight buffers need {PHASE_WEIGHT_FLOATS} contiguous fp32 elements")
    m = len(pw)
    P, I = _lib.ctypes.c_void_p, _lib.ctypes.c_int
    dev = (weights[0] if n else (w1 if w1 is not None else pw[0])).device
    rc = _lib.lib().nconv_weight_prologue(
        n, (P * max(n, 1))(*[w.data_ptr() for w in weights]), (I * max(n, 1))(*[w.shape[0] for w in weights]),
        (I * max(n, 1))(*[w[0].numel() for w in weights]), (P * max(n, 1))(*[s.data_ptr() for s in wsums]),
        _lib.ptr(w1), _lib.ptr(w2), _lib.ptr(w21),
        m, (P * max(m, 1))(*[w.data_ptr() for w in pw]), (I * max(m, 1))(*[w.shape[1] for w in pw]),
        (I * max(m, 1))(*pup), (P * max(m, 1))(*[o.data_ptr() for o in pout]), _lib.stream_handle(dev))
    _lib.check(rc, "nconv_weight_prologue")


def train_prologue(weights, softplus, wsums, head=None, phase=None):
    """nconv_train_prologue: the training pass's weight prologue in one launch -- EnforcePos's
    softplus in place on the layers flagged in `softplus`, every layer's normalisers into wsums, and
    from the transformed weights: head = (i1, i2, w21, sync) the exact head's weights of layers i1
    (nconv1) / i2 (nconv2) and a zero int32 device counter the call leaves at zero (sync_counter), or
    None; phase = (layer indices, up_first, phase outs, box outs or None) as
    phase_weights' outputs plus the backward's box weights (BOX_WEIGHT_FLOATS each). Bitwise what
    weight_prep + head_weights + phase_weights + the backward's box-weight builds write."""
    n = len(weights)
    i1, i2, w21, sync = head if head is not None else (-1, -1, None, None)
    if w21 is not None and (sync is None or sync.dtype != torch.int32 or sync.numel() < 1):
        raise ValueError("the head weights need a zero int32 sync counter (sync_counter)")
    pl, pup, pout, pbox = phase if phase is not None else ([], [], [], None)
    if w21 is not None and (w21.numel() < HEAD_WEIGHTS_FLOATS or not w21.is_contiguous() or
                            w21.dtype != torch.float32):
        raise ValueError(f"head-weight buffer needs {HEAD_WEIGHTS_FLOATS} contiguous fp32 elements")
    for o in list(pout) + list(pbox or []):
        if o.numel() < PHASE_WEIGHT_FLOATS or not o.is_contiguous() or o.dtype != torch.float32:
            raise ValueError(f"phase / box buffers need {PHASE_WEIGHT_FLOATS} contiguous fp32 elements")
    m = len(pl)
    P, I = _lib.ctypes.c_void_p, _lib.ctypes.c_int
    rc = _lib.lib().nconv_train_prologue(
        n, (P * max(n, 1))(*[w.data_ptr() for w in weights]), (I * max(n, 1))(*[w.shape[0] for w in weights]),
        (I * max(n, 1))(*[w[0].numel() for w in weights]), (I * max(n, 1))(*[int(bool(v)) for v in softplus]),
        (P * max(n, 1))(*[s.data_ptr() for s in wsums]), i1, i2, _lib.ptr(w21), _lib.ptr(sync), m,
        (I * max(m, 1))(*pl),
        (I * max(m, 1))(*pup), (P * max(m, 1))(*[o.data_ptr() for o in pout]),
        (P * max(m, 1))(*[o.data_ptr() for o in pbox]) if pbox is not None else None,
        _lib.stream_handle(weights[0].device))
    _lib.check(rc, "nconv_train_prologue")


_SYNC = {}


def sync_counter(device):
    """A zero int32 counter for train_prologue (made once, zero-filled; every call leaves it at
    zero), one per (device, current stream): two prologues running concurrently on different
    streams must not count their last-block arrivals on one counter."""
    device = torch.device(device)
    key = (device.index, torch.cuda.current_stream(device).stream_id)
    if key not in _SYNC:
        _SYNC[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return _SYNC[key]


BOX_WEIGHT_FLOATS = 1024  # (8, 8, 4, 4) box weights of an exactly-2x UPCAT layer (nconv_bwd_io.box_weights)


def layer_forward_raw(spec: LayerSpec, xa, ca, xb, cb, weight, bias, wsum, out=None, wphase=None):
    """Enqueue nconv_fwd; returns (y, cout) (written into `out` if given). No autograd. `wphase`:
    the layer's phase weights (UPCAT layers, phase_weights), or None."""
    L = spec.descriptor(xa, ca, xb, cb, weight, bias, wsum, wphase)
    sh = (L.B, L.Cout, L.Ho, L.Wo)
    y, co = _outputs(out, 2, (sh, sh), xa.device)
    rc = _lib.lib().nconv_fwd(_lib.ctypes.byref(L), _lib.ptr(y), _lib.ptr(co), _lib.stream_handle(xa.device))
    _lib.check(rc, "nconv_fwd")
    return y, co


def layer_forward_pooled(spec: LayerSpec, xa, ca, xb, cb, weight, bias, wsum, out=None, argmax=False):
    """nconv_fwd_pooled: (y, cout, maxpool2x2(y), maxpool2x2(cout)) in one launch (written into
    `out` if given). With argmax=True also the pooling windows' first-maximum codes (int32, one per
    pooled element; the training backward routes the pooled tensors' gradient by them) as a fifth
    result. No autograd."""
    L = spec.descriptor(xa, ca, xb, cb, weight, bias, wsum)
    sh, shp = (L.B, L.Cout, L.Ho, L.Wo), (L.B, L.Cout, L.Ho // 2, L.Wo // 2)
    if callable(out) and argmax:
        y, co, py, pc, arg = _outputs(out, 5, (sh, sh, shp, shp, shp), xa.device, [torch.float32] * 4 + [torch.int32])
    else:
        y, co, py, pc = _outputs(out, 4, (sh, sh, shp, shp), xa.device)
        arg = torch.empty(shp, dtype=torch.int32, device=xa.device) if argmax else None
    rc = _lib.lib().nconv_fwd_pooled(_lib.ctypes.byref(L), _lib.ptr(y), _lib.ptr(co), _lib.ptr(py), _lib.ptr(pc),
                                     _lib.ptr(arg), _lib.stream_handle(xa.device))
    _lib.check(rc, "nconv_fwd_pooled")
    return (y, co, py, pc, arg) if argmax else (y, co, py, pc)


HEAD_WEIGHTS_FLOATS = 3136  # include/nconv.h NCONV_HEAD_WEIGHTS_FLOATS


def head_weights(spec1: LayerSpec, spec2: LayerSpec, S, w1, b1, s1, w2, b2, s2, out=None):
    """nconv_head_weights: the exact fused head's auxiliary weights (HEAD_WEIGHTS_FLOATS = 3136
    floats: the composed confidence weights sum_i W2[o,i] (x) W1[i] / s1[i] as exact three-part bf16
    matrix-core operands, then nconv2's weights transposed) from the current weights and nconv1's
    s[o]; one launch."""
    L1 = spec1.descriptor(S, None, None, None, w1, b1, s1)
    L2 = spec2.descriptor(S, S, None, None, w2, b2, s2)
    if out is None:
        out = torch.empty(HEAD_WEIGHTS_FLOATS, device=S.device, dtype=torch.float32)
    rc = _lib.lib().nconv_head_weights(_lib.ctypes.byref(L1), _lib.ctypes.byref(L2), _lib.ptr(out),
                                       _lib.stream_handle(S.device))
    _lib.check(rc, "nconv_head_weights")
    return out


def layer_forward_head(spec1: LayerSpec, spec2: LayerSpec, S, w1, b1, s1, w2, b2, s2, w21=None, train=False,
                       out=None):
    """nconv_fwd_head: nconv2(nconv1(S)) with nconv1 evaluated inside nconv2's staging (its output
    never reaches HBM); returns nconv2's (y, cout, maxpool2x2(y), maxpool2x2(cout)). No autograd.
    With FORWARD_MATH == exact fp32 the composed weights `w21` (head_weights) are required.
    train=True (exact fp32): also the pooling argmax codes and nconv1's (y, cout), which the
    training backward reads -- returns (y, cout, py, pc, argmax, y1, cout1). out: None (fresh
    tensors) or a callable as _outputs takes."""
    L1 = spec1.descriptor(S, None, None, None, w1, b1, s1)
    L2 = spec2.descriptor(S, S, None, None, w2, b2, s2, w21)  # geometry only: the kernel reads S via L1
    B, H, W = S.shape[0], L1.Ho, L1.Wo
    sh, shp, f32 = (B, 8, H, W), (B, 8, H // 2, W // 2), torch.float32
    if train:
        y, co, py, pc, arg, y1, c1 = _outputs(out, 7, (sh, sh, shp, shp, shp, sh, sh), S.device,
                                              [f32] * 4 + [torch.int32, f32, f32])
    else:
        y, co, py, pc = _outputs(out, 4, (sh, sh, shp, shp), S.device)
        arg = y1 = c1 = None
    rc = _lib.lib().nconv_fwd_head(_lib.ctypes.byref(L1), _lib.ctypes.byref(L2), _lib.ptr(y), _lib.ptr(co),
                                   _lib.ptr(py), _lib.ptr(pc), _lib.ptr(arg), _lib.ptr(y1), _lib.ptr(c1),
                                   _lib.stream_handle(S.device))
    _lib.check(rc, "nconv_fwd_head")
    return (y, co, py, pc, arg, y1, c1) if train else (y, co, py, pc)


class NConvLayerFn(torch.autograd.Function):
    """Autograd node of one fused NConv layer (glue + NConv2d.forward), kernels in libnconv."""

    @staticmethod
    def forward(ctx, spec, xa, ca, xb, cb, weight, bias, wsum, wphase=None):
        y, co = layer_forward_raw(spec, xa, ca, xb, cb, weight, bias, wsum, wphase=wphase)
        ctx.spec = spec
        ctx.save_for_backward(xa, ca, xb, cb, weight, bias, wsum, y, co)
        return y, co

    @staticmethod
    def backward(ctx, gy, gco):
        spec = ctx.spec
        xa, ca, xb, cb, weight, bias, wsum, y, co = ctx.saved_tensors
        need = ctx.needs_input_grad  # (spec, xa, ca, xb, cb, weight, bias, wsum)
        # the kernels overwrite every element of the input gradients (no zero-fill)
        z = lambda t, n: torch.empty_like(t) if (t is not None and n) else None
        gxa, gca, gxb, gcb = z(xa, need[1]), z(ca, need[2]), z(xb, need[3]), z(cb, need[4])
        gw = torch.empty_like(weight) if need[5] else None
        gb = torch.empty_like(bias) if need[6] else None
        layer_backward(spec, (xa, ca, xb, cb, weight, bias, wsum), y, co, gy, gco, (gxa, gca, gxb, gcb), gw, gb)
        return None, gxa, gca, gxb, gcb, gw, gb, None, None


def layer_backward(spec: LayerSpec, inputs, y, co, gy, gco, gin, gw, gb, accumulate=False, defer=None,
                   pool_grad=None, head=None, tail=None, box=None):
    """nconv_bwd of one fused layer: gin = (gxa, gca, gxb, gcb) (None: skip) overwritten, or added
    into with accumulate=True (NCONV_BWD_ACCUMULATE: a tensor consumed by two layers); gw, gb
    overwritten (None: skip). defer: a WgradReduce collecting the layer's weight-gradient partial
    rows (NCONV_BWD_DEFER_REDUCE): gw / gb are then written by its run(). pool_grad: (gy_pool,
    gcout_pool, argmax) -- the gradient of this layer's 2x2-pooled outputs (the next down layer read
    layer_forward_pooled's copies), routed into gy / gco by the argmax codes (nconv_bwd_ex). head:
    (spec, S, weight, bias, wsum, gw, gb) of the producer nconv1, whose weight / bias gradients are
    then computed inside this layer's input gradient (nconv_bwd_ex head; gin's gxa / gca optional).
    tail: (spec, weight, bias, wsum, y9, cout9, gy9, gw9) of the 1x1 consumer nconv7, whose backward
    is fused into this layer's (nconv_bwd_ex tail; gy / gco are then unused and may be None; nconv7's
    bias gradient is the caller's). The input and the weight gradient are separate kernels. tail may
    carry a 9th element, the crop origin of nconv7's planes when they hold a window of its grid
    (DNET's crop: nconv_bwd_io tail_crop0 / tail_h / tail_w). box: an exactly-2x UPCAT layer's box
    weights (train_prologue), else built by this call."""
    xa, ca, xb, cb, weight, bias, wsum = inputs
    gxa, gca, gxb, gcb = gin
    dev = y.device
    if gy is None and tail is None:
        gy = torch.zeros_like(y)
    gy = gy.contiguous() if gy is not None else None
    gco = gco.contiguous() if gco is not None else None
    L = spec.descriptor(xa, ca, xb, cb, weight, bias, wsum)
    lib = _lib.lib()
    ws_bytes = lib.nconv_bwd_workspace_bytes(_lib.ctypes.byref(L))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    flags = (_lib.BWD_ACCUMULATE if accumulate else 0) | (_lib.BWD_DEFER_REDUCE if defer is not None else 0)
    io = _lib.NconvBwdIo()
    gpy, gpc, parg = pool_grad if pool_grad is not None else (None, None, None)
    for name, t in (("y", y), ("cout", co), ("gy", gy), ("gcout", gco), ("gxa", gxa), ("gca", gca), ("gxb", gxb),
                    ("gcb", gcb), ("gw", gw), ("gbias", gb), ("gy_pool", gpy), ("gcout_pool", gpc),
                    ("pool_argmax", parg)):
        setattr(io, name, t.data_ptr() if t is not None else None)
    if head is not None:
        hspec, S, hw, hb, hs, hgw, hgb = head
        HL = hspec.descriptor(S, None, None, None, hw, hb, hs)
        hbytes = lib.nconv_bwd_head_workspace_bytes(_lib.ctypes.byref(L))
        hws = torch.empty(max(hbytes, 1), dtype=torch.uint8, device=dev)
        io.head = _lib.ctypes.pointer(HL)
        io.head_workspace, io.head_workspace_bytes = hws.data_ptr(), hbytes
        io.head_gw, io.head_gbias = _lib.ptr(hgw), _lib.ptr(hgb)
    io.box_weights = _lib.ptr(box)
    if tail is not None:
        tspec, tw, tb, ts, ty, tco, tgy, tgw = tail[:8]
        if len(tail) > 8 and tail[8] is not None:  # the planes hold a window of nconv7's grid
            io.tail_crop0, io.tail_h, io.tail_w = int(tail[8]), ty.shape[2], ty.shape[3]
        TL = tspec.descriptor(y, co, None, None, tw, tb, ts)
        tbytes = lib.nconv_bwd_tail_workspace_bytes(_lib.ctypes.byref(L))
        tws = torch.empty(max(tbytes, 1), dtype=torch.uint8, device=dev)
        io.tail = _lib.ctypes.pointer(TL)
        io.tail_y, io.tail_cout, io.tail_gy = ty.data_ptr(), tco.data_ptr(), tgy.contiguous().data_ptr()
        io.tail_workspace, io.tail_workspace_bytes = tws.data_ptr(), tbytes
        io.tail_gw = _lib.ptr(tgw)
    rc = lib.nconv_bwd_ex(_lib.ctypes.byref(L), _lib.ctypes.byref(io), _lib.ptr(ws), ws_bytes, flags,
                          _lib.stream_handle(dev))
    if defer is not None and rc >= 0:
        defer.add(L, ws, rc, gw, gb)
        if head is not None:
            defer.add(HL, hws, io.head_nparts, hgw, hgb)
        if tail is not None:
            defer.add(TL, tws, io.tail_nparts, tgw, None)
        return
    _lib.check(rc, "nconv_bwd")


class WgradReduce:
    """The deferred weight-gradient reductions of one backward pass (nconv_wgrad_reduce): every
    layer's partial rows reduced in two launches instead of two per layer. Keeps the layers'
    workspaces alive until run()."""

    def __init__(self):
        self.jobs = []
        self.sums = []

    def add(self, L, ws, nparts, gw, gb):
        if nparts > 0 and (gw is not None or gb is not None):  # (input-gradient-only calls add none)
            self.jobs.append((L, ws, nparts, gw, gb, torch.cuda.current_stream(ws.device)))

    def add_sum(self, x, out):
        """out[0] = x.sum() in the same two launches (nconv_wgrad_reduce_ex; fixed order)."""
        self.sums.append((x.contiguous(), out, torch.cuda.current_stream(x.device)))

    def run(self, device):
        cur = torch.cuda.current_stream(device)
        for j in self.jobs:
            # a workspace allocated on another stream (the weight-gradient side stream) is read here
            # by the current one: keep the allocator from reusing it before this reduction ran
            if j[5] != cur:
                j[1].record_stream(cur)
        for j in self.sums:
            if j[2] != cur:
                j[0].record_stream(cur)
        items = [("job", j) for j in self.jobs] + [("sum", j) for j in self.sums]
        lib = _lib.lib()
        for k in range(0, len(items), 16):
            jobs = [j for t, j in items[k:k + 16] if t == "job"]
            sums = [j for t, j in items[k:k + 16] if t == "sum"]
            n, ns = len(jobs), len(sums)
            VP = _lib.ctypes.c_void_p * max(n, 1)
            layers = (_lib.NconvLayer * max(n, 1))(*[j[0] for j in jobs])
            wss = VP(*[j[1].data_ptr() for j in jobs])
            nparts = (_lib.ctypes.c_int * max(n, 1))(*[j[2] for j in jobs])
            gws = VP(*[(j[3].data_ptr() if j[3] is not None else None) for j in jobs])
            gbs = VP(*[(j[4].data_ptr() if j[4] is not None else None) for j in jobs])
            SP = _lib.ctypes.c_void_p * max(ns, 1)
            sws_bytes = lib.nconv_sum_workspace_bytes(ns)
            sws = torch.empty(max(sws_bytes, 4), dtype=torch.uint8, device=device) if ns else None
            rc = lib.nconv_wgrad_reduce_ex(n, layers, wss, nparts, gws, gbs, ns, SP(*[j[0].data_ptr() for j in sums]),
                                           (_lib.ctypes.c_longlong * max(ns, 1))(*[j[0].numel() for j in sums]),
                                           SP(*[j[1].data_ptr() for j in sums]), _lib.ptr(sws), sws_bytes,
                                           _lib.stream_handle(device))
            _lib.check(rc, "nconv_wgrad_reduce")
        self.jobs = []
        self.sums = []


def kernel_plan(spec: LayerSpec, xa, ca, xb, cb, weight, bias, wsum):
    """nconv_plan: the kernel families (forward, input gradient, weight gradient) that nconv_fwd /
    nconv_bwd run for this layer under the current FORWARD_MATH / BACKWARD_MATH, by name
    (_lib.KERNEL_NAMES). Host-only: no device work."""
    L = spec.descriptor(xa, ca, xb, cb, weight, bias, wsum)
    out = [_lib.ctypes.c_int(-1) for _ in range(3)]
    rc = _lib.lib().nconv_plan(_lib.ctypes.byref(L), *[_lib.ctypes.byref(v) for v in out])
    _lib.check(rc, "nconv_plan")
    return tuple(_lib.KERNEL_NAMES[v.value] for v in out)


def nconv_layer(spec: LayerSpec, xa, ca, xb, cb, weight, bias, wsum, wphase=None):
    """Differentiable fused layer. Inputs must be contiguous fp32 device tensors. `wphase`: the
    layer's phase weights (UPCAT layers, phase_weights; no gradient flows through them), or None."""
    return NConvLayerFn.apply(spec, xa, ca, xb, cb, weight, bias, wsum, wphase)


# ------------------------------------------------------------------------------------------------
# EnforcePos (models/step1.py:176-212)
# ------------------------------------------------------------------------------------------------
class EnforcePos(object):
    """Non-negativity enforcement as a forward pre-hook: in training mode, before every forward,
    weight.data <- pos_fn(weight) (step1.py:190-193). Not idempotent: softplus grows the weights
    on every training forward, exactly like the reference."""

    def __init__(self, pos_fn, name):
        self.name = name
        self.pos_fn = pos_fn

    @staticmethod
    def apply(module, name, pos_fn):
        fn = EnforcePos(pos_fn, name)
        module.register_forward_pre_hook(fn)
        return fn

    def __call__(self, module, inputs):
        if module.training:
            weight = getattr(module, self.name)
            if self.pos_fn.lower() == "softplus" and weight.is_cuda and weight.dtype == torch.float32 \
                    and weight.is_contiguous():
                wsum = torch.empty(weight.shape[0], device=weight.device, dtype=torch.float32)
                weight_prep([weight.data], [True], [wsum])
            else:
                weight.data = self._pos(weight).data

    def _pos(self, p):
        pos_fn = self.pos_fn.lower()
        if pos_fn == "softmax":
            p_sz = p.size()
            return F.softmax(p.view(p_sz[0], p_sz[1], -1), -1).view(p_sz)
        if pos_fn == "exp":
            return torch.exp(p)
        if pos_fn == "softplus":
            return F.softplus(p, beta=10)
        if pos_fn == "sigmoid":
            return torch.sigmoid(p)
        print("Undefined positive function!")
        return None


def _poisson_kernel(k):
    """Outer product of the Poisson(k/2) pmf over 0..k-1 (step1.py:159-163), float64."""
    from scipy.stats import poisson
    y = poisson(k / 2).pmf(np.arange(0, k))
    return np.outer(y, y)


class NConv2d(_ConvNd):
    """Normalized convolution layer (reference models/step1.py:97-172).

    forward(data, conf) -> (nconv, cout) with nconv = conv(data*conf, W)/(conv(conf, W)+eps) + b and
    cout = conv(conf, W) / sum(W[o]). The unused bnorm/relu submodules are kept for state_dict
    compatibility (step1.py:110-111).
    """

    def __init__(self, in_channels, out_channels, kernel_size, pos_fn="softplus", init_method="k",
                 stride=(1, 1), padding=(2, 2), dilation=(1, 1), groups=1, bias=True):
        super().__init__(in_channels, out_channels, _pair(kernel_size), _pair(stride), _pair(padding),
                         _pair(dilation), False, output_padding=(0, 0), groups=groups, bias=bias,
                         padding_mode="zeros")
        self.eps = 1e-7
        self.pos_fn = pos_fn
        self.init_method = init_method
        self.init_parameters()
        self.bnorm = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU()
        if self.pos_fn is not None:
            EnforcePos.apply(self, "weight", pos_fn)

    def init_parameters(self):
        # Same RNG consumption as the reference (after _ConvNd.reset_parameters): 'x' xavier,
        # 'k' kaiming, 'p' Poisson outer product + torch.rand; bias replaced by zeros + 0.01.
        if self.init_method == "x":
            torch.nn.init.xavier_uniform_(self.weight)
        elif self.init_method == "k":
            torch.nn.init.kaiming_uniform_(self.weight)
        elif self.init_method == "p":
            w = torch.tensor(_poisson_kernel(self.kernel_size[0]), dtype=torch.float32).type_as(self.weight)
            w = w[None, None].repeat(self.out_channels, 1, 1, 1).repeat(1, self.in_channels, 1, 1)
            self.weight.data = w + torch.rand(w.shape)
        self.bias = torch.nn.Parameter(torch.zeros(self.out_channels) + 0.01)

    def spec(self, mode=_lib.PLAIN, thresh=0.01):
        return LayerSpec(self.in_channels, self.out_channels, tuple(self.kernel_size), tuple(self.stride),
                         tuple(self.padding), tuple(self.dilation), self.groups, self.eps, mode, thresh)

    def weight_sum(self):
        """s[o] = sum(W[o]) computed on device (no autograd; its gradient is folded into gW)."""
        w = self.weight.detach()
        wsum = torch.empty(w.shape[0], device=w.device, dtype=torch.float32)
        weight_prep([w], [False], [wsum])
        return wsum

    def forward(self, data, conf):
        if export.is_exporting():  # the export graph: the reference's own ops (export.py)
            return export.nconv2d(self, data, conf)
        _require_device(data, "NConv2d.forward")
        _require_device(conf, "NConv2d.forward")
        if data.shape != conf.shape:
            raise ValueError(f"data {tuple(data.shape)} and conf {tuple(conf.shape)} differ")
        w = self.weight if self.weight.is_contiguous() else self.weight.contiguous()
        return nconv_layer(self.spec(), data.contiguous(), conf.contiguous(), None, None, w, self.bias,
                           self.weight_sum())
