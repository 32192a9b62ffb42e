"""DNET / SETP1_NCONV — drop-in for the reference's unguided NConv U-Net (models/step1.py:15-94).

The 9-layer graph (step1.py:51-94) runs as one libnconv launch per layer with the glue fused
into each layer's load stage:

    nconv1   THRESH      c0 = (S > 0.01), x0 = S                     step1.py:53-56
    nconv2   PLAIN                                                  step1.py:57
    down1-3  POOL2       independent 2x2 max-pool of x and c         step1.py:62-75
    nconv4/5 UPCAT_SKIP  cat(skip, nearest-up(low))                  step1.py:78-85
    nconv6   UPCAT_UP    cat(nearest-up(low), skip), padding 0       step1.py:88-90
    nconv7   PLAIN       1x1, default padding 2                      step1.py:92
    crop     [1:481, 1:641] (literal, default) or [1:H+1, 1:W+1]     step1.py:94

Without autograd (inference) nconv6 and nconv7 are fused into one launch that writes the cropped
output directly. EnforcePos pre-hooks of all nine layers are applied in one launch in training
mode, before any layer runs (the reference applies each right before its layer; the layers share
no weights, so the results are identical).
"""
import dataclasses
import itertools
import math
import os

import torch
import torch.nn as nn

from . import _lib, dense, export, nconv
from .nconv import (EnforcePos, NConv2d, WgradReduce, _require_device, head_weights, layer_backward,
                    layer_forward_head, layer_forward_pooled, layer_forward_raw, nconv_layer, phase_weights,
                    train_prologue, weight_prep)

LAYERS = ("nconv1", "nconv2", "nconv_down1", "nconv_down2", "nconv_down3", "nconv4", "nconv5",
          "nconv6", "nconv7")


# Training forward in batch slices on this many streams (DNETFn.forward): the exact-fp32 pooled
# graph with the fused head and tail only; 1 = one launch per layer over the whole batch
TRAIN_FWD_STREAMS = int(os.environ.get("NCONV_TRAIN_FWD_STREAMS", "2"))
_TRAIN_FWD_STREAMS = {}


def _train_fwd_streams(device, n):
    key = (device.index, n)
    if key not in _TRAIN_FWD_STREAMS:
        _TRAIN_FWD_STREAMS[key] = [torch.cuda.Stream(device=device) for _ in range(n)]
    return _TRAIN_FWD_STREAMS[key]


def _tail_exact_up(sp, S):
    """nconv6's skip input (nconv2's grid, S's) is exactly twice nconv5's grid (the pooled one)."""
    return S.shape[2] % 2 == 0 and S.shape[3] % 2 == 0


def _train_fwd_chain(sp, W, S, w21, wph, crop, out, pooled=True):
    """DNETFn's forward launches over S's frames; out: None (fresh tensors) or a callable handing
    out each launch's output tensors (nconv._outputs). Returns x1, c1, ..., x9, c9, then the pooled
    copies and argmax codes (pooled graph)."""
    w4, w5, w6 = (None, None, None) if wph is None else tuple(wph)
    if pooled:
        spp = [dataclasses.replace(sp[k], mode=_lib.PLAIN) for k in (2, 3, 4)]
        if FUSE_HEAD_FWD:  # nconv1 inside nconv2's tile, nconv1's outputs written for the backward
            if w21 is None:
                w21 = head_weights(sp[0], sp[1], S, *W[0], *W[1])
            x2, c2, p2x, p2c, a2, x1, c1 = layer_forward_head(sp[0], sp[1], S, *W[0], *W[1], w21, train=True,
                                                              out=out)
        else:
            x1, c1 = layer_forward_raw(sp[0], S, None, None, None, *W[0], out=out)
            x2, c2, p2x, p2c, a2 = layer_forward_pooled(sp[1], x1, c1, None, None, *W[1], out=out, argmax=True)
        x3, c3, p3x, p3c, a3 = layer_forward_pooled(spp[0], p2x, p2c, None, None, *W[2], out=out, argmax=True)
        x4, c4, p4x, p4c, a4 = layer_forward_pooled(spp[1], p3x, p3c, None, None, *W[3], out=out, argmax=True)
        x5, c5 = layer_forward_raw(spp[2], p4x, p4c, None, None, *W[4], out=out)
        pools = (p2x, p2c, a2, p3x, p3c, a3, p4x, p4c, a4)
    else:
        x1, c1 = layer_forward_raw(sp[0], S, None, None, None, *W[0], out=out)
        x2, c2 = layer_forward_raw(sp[1], x1, c1, None, None, *W[1], out=out)
        x3, c3 = layer_forward_raw(sp[2], x2, c2, None, None, *W[2], out=out)
        x4, c4 = layer_forward_raw(sp[3], x3, c3, None, None, *W[3], out=out)
        x5, c5 = layer_forward_raw(sp[4], x4, c4, None, None, *W[4], out=out)
        pools = ()
    x6, c6 = layer_forward_raw(sp[5], x4, c4, x5, c5, *W[5], out=out, wphase=w4)
    x7, c7 = layer_forward_raw(sp[6], x3, c3, x6, c6, *W[6], out=out, wphase=w5)
    if pooled and FUSE_TAIL_FWD and w6 is not None and x2.shape[2:] == tuple(2 * v for v in x7.shape[2:]):
        x8, c8, x9, c9 = _tail_train(sp[7], sp[8], x2, c2, x7, c7, W[7], W[8], w6, crop, out=out)
    elif crop is not None:
        raise RuntimeError("DNETFn: a cropped output needs the fused training tail")
    else:
        x8, c8 = layer_forward_raw(sp[7], x2, c2, x7, c7, *W[7], out=out, wphase=w6)
        x9, c9 = layer_forward_raw(sp[8], x8, c8, None, None, *W[8], out=out)
    return (x1, c1, x2, c2, x3, c3, x4, c4, x5, c5, x6, c6, x7, c7, x8, c8, x9, c9, *pools)


class DNETFn(torch.autograd.Function):
    """Autograd node of the whole 9-layer DNET graph (training path). The backward runs the layer
    backwards in reverse order itself. Inputs: specs, capture (dict or None), S, then (weight, bias,
    s[o]) of each layer in LAYERS order, then the phase weights; outputs: nconv7's (uncropped) y,
    cout.

    crop: None, or DNET's output size (h, w) when the fused training tail writes nconv7's output
    already cropped (DNET._tail_crop): the outputs are then the cropped (y, cout), and the backward
    reads their gradient through the window (nconv_bwd_io tail_crop0), with no crop copy and no
    zero-padded gradient.

    Three tensors are read by two layers each (nconv2's output: down1 through the 2x2 max-pool and
    nconv6; down1's: down2 and nconv5; down2's: down3 and nconv4). With exact-fp32 forward and
    backward (the default) the pool is materialised: nconv2 / down1 / down2 write their pooled
    outputs and the pooling argmax codes in the same launch (nconv_fwd_pooled), the down layers read
    the pooled copies with plain loads, their input gradients stay pooled-sized, and each producer's
    backward adds them to the other consumer's full-resolution gradient at the argmax while forming
    {gN, gD} (nconv_bwd_ex) -- no full-resolution read-modify-write and no argmax recomputation.
    With a bf16 backward the down layers pool while loading and their input gradients are added
    into the full-resolution gradient (NCONV_BWD_ACCUMULATE)."""

    @staticmethod
    def forward(ctx, specs, capture, crop, S, *p):
        """p: (weight, bias, s[o]) of each layer, then the phase weights of nconv4/5/6 (a (3, 1024)
        tensor, DNET._phase_weights) or None, then optionally the exact head's weights (None: built
        here) and the box weights of nconv4/5/6 (a (3, 1024) tensor, None: built by the backward),
        both from DNET._train_prologue."""
        W = [p[3 * i:3 * i + 3] for i in range(9)]
        wph = p[27] if len(p) > 27 and p[27] is not None else None
        w21 = p[28] if len(p) > 28 else None
        ctx.wbox = p[29] if len(p) > 29 else None
        w6 = None if wph is None else wph[2]
        sp = specs
        pooled = _materialise_pool(S)
        ctx.crop = crop
        B = S.shape[0]
        nst = max(1, min(int(TRAIN_FWD_STREAMS), B))
        if (pooled and FUSE_HEAD_FWD and FUSE_TAIL_FWD and w6 is not None and nst > 1 and
                _tail_exact_up(sp, S)):
            # the batch in nst slices, one stream each, every launch writing its rows of full-batch
            # tensors (allocated by the first slice's launches): the slices' kernels overlap as the
            # inference split's do; each frame's arithmetic is unchanged (bitwise the one-stream pass)
            if w21 is None:
                w21 = head_weights(sp[0], sp[1], S, *W[0], *W[1])
            bounds = [B * k // nst for k in range(nst + 1)]
            full = []
            cur = torch.cuda.current_stream(S.device)
            side = _train_fwd_streams(S.device, nst - 1)
            for st in side:
                st.wait_stream(cur)
            res = None
            for k, st in enumerate([cur] + side):
                b0, b1 = bounds[k], bounds[k + 1]

                def rows(shapes, dtypes, device, b0=b0, b1=b1, it=itertools.count()):
                    # the i-th output of this slice's launches = rows b0:b1 of full-batch tensor i
                    out = []
                    for sh, dt in zip(shapes, dtypes):
                        i = next(it)
                        if i == len(full):
                            full.append(torch.empty((B,) + tuple(sh[1:]), device=device, dtype=dt))
                        out.append(full[i][b0:b1])
                    return out
                with torch.cuda.stream(st):
                    r = _train_fwd_chain(sp, W, S[b0:b1], w21, wph, crop, rows)
                res = r if res is None else res
            for st in side:
                cur.wait_stream(st)
            base = {t.data_ptr(): t for t in full}
            (x1, c1, x2, c2, x3, c3, x4, c4, x5, c5, x6, c6, x7, c7, x8, c8, x9, c9, *pools) = [
                base[t.data_ptr()] for t in res]
        else:
            (x1, c1, x2, c2, x3, c3, x4, c4, x5, c5, x6, c6, x7, c7, x8, c8, x9, c9, *pools) = \
                _train_fwd_chain(sp, W, S, w21, wph, crop, None, pooled=pooled)
        if capture is not None:  # the three pooling stages' inputs (DNET.capture)
            capture.update(down1=(x2.detach(), c2.detach()), down2=(x3.detach(), c3.detach()),
                           down3=(x4.detach(), c4.detach()))
        ctx.specs = specs
        ctx.pooled = pooled
        ctx.n_extra = len(p) - 27
        ctx.save_for_backward(S, *p[:27], x1, c1, x2, c2, x3, c3, x4, c4, x5, c5, x6, c6, x7, c7, x8, c8, x9, c9,
                              *pools)
        ctx.mark_non_differentiable(c9)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the never-used c9
        return x9, c9

    @staticmethod
    def backward(ctx, g9, gc9):
        sv = ctx.saved_tensors
        if g9 is None:  # (grads are not materialised)
            g9 = torch.zeros_like(sv[44])
        S, p, acts, pools = sv[0], sv[1:28], sv[28:46], sv[46:]
        wbox = (None, None, None) if ctx.wbox is None else tuple(ctx.wbox)
        W = [p[3 * i:3 * i + 3] for i in range(9)]
        X = [None] + [(acts[2 * i], acts[2 * i + 1]) for i in range(9)]  # X[k] = output of layer k
        need = ctx.needs_input_grad[2:]  # (capture, S, w1, b1, s1, ...)
        gw = [torch.empty_like(W[i][0]) if need[2 + 3 * i] else None for i in range(9)]
        gb = [torch.empty_like(W[i][1]) if need[3 + 3 * i] else None for i in range(9)]
        e = torch.empty_like
        # input gradients: G[k] = (gx, gc) of layer k's output
        G = [None] * 10
        sp = ctx.specs
        red = WgradReduce()  # every layer's weight-gradient reduction in two launches at the end
        cur = torch.cuda.current_stream(S.device)
        side = _wgrad_stream(S.device) if (ctx.pooled and WGRAD_STREAM) else None

        def layer_bwd(spec, inputs, y, co, gy, gco, gin, gw_, gb_, **kw):
            # the weight gradient runs on the side stream, concurrent with this layer's input gradient
            # (and the next layers' input gradients, which do not depend on it): it needs only tensors
            # that are complete when this layer's backward starts
            if side is None or (gw_ is None and gb_ is None):
                layer_backward(spec, inputs, y, co, gy, gco, gin, gw_, gb_, defer=red, **kw)
                return
            st = side
            st.wait_stream(cur)
            tail, head = kw.pop("tail", None), kw.pop("head", None)
            layer_backward(spec, inputs, y, co, gy, gco, gin, None, None, defer=red, head=head,
                           tail=None if tail is None else tail[:7] + (None,) + tail[8:], **kw)  # (no gw7)
            with torch.cuda.stream(st):
                layer_backward(spec, inputs, y, co, gy, gco, (None,) * 4, gw_, gb_, defer=red, tail=tail, **kw)

        def bwd(k, a, b, ga, gb_, acc=False, src_a=None, spec=None, pool_grad=None, box=None):
            xa, ca = src_a if src_a is not None else (X[a] if a else (S, None))
            xb, cb = X[b] if b else (None, None)
            gy, gco = G[k] if G[k] is not None else (g9, None)
            layer_bwd(spec or sp[k - 1], (xa, ca, xb, cb, *W[k - 1]), X[k][0], X[k][1], gy, gco,
                      (*(ga or (None, None)), *(gb_ or (None, None))), gw[k - 1], gb[k - 1], accumulate=acc,
                      pool_grad=pool_grad, box=box)

        def finish():
            if side is not None:
                cur.wait_stream(side)
            red.run(S.device)

        G[2], G[7] = (e(X[2][0]), e(X[2][1])), (e(X[7][0]), e(X[7][1]))
        exact_up = X[2][0].shape[2:] == tuple(2 * v for v in X[7][0].shape[2:])  # nconv6's phase form
        # (c9 is non-differentiable; nconv7's weight gradient is accumulated inside nconv6's weight-
        # gradient pass, so the fused form needs nconv6's gw or gb too)
        if ctx.crop is not None or (FUSE_TAIL_BWD and ctx.pooled and exact_up and gw[8] is not None and
                                    (gw[7] is not None or gb[7] is not None)):
            # nconv7's backward inside nconv6's (nconv_bwd_ex tail): its input gradient never reaches
            # HBM; its bias gradient is the sum of its output gradient (every output pixel, padding ring
            # included, as autograd's conv bias gradient), summed by the batched reduction. With the
            # cropped output nconv7's planes are the crop window from grid row / column 1
            # (step1.py:94); the gradient outside it is 0
            g9c = g9.contiguous()
            layer_bwd(sp[7], (X[2][0], X[2][1], X[7][0], X[7][1], *W[7]), X[8][0], X[8][1], None, None,
                      (*G[2], *G[7]), gw[7], gb[7],
                      tail=(sp[8], *W[8], X[9][0], X[9][1], g9c, gw[8], None if ctx.crop is None else 1),
                      box=wbox[2])
            if gb[8] is not None:
                red.add_sum(g9c, gb[8])
        else:
            G[8] = (e(X[8][0]), e(X[8][1]))
            bwd(9, 8, 0, G[8], None)                        # nconv7
            bwd(8, 2, 7, G[2], G[7])                        # nconv6: nconv2's output (overwrite) + up
        G[3], G[6] = (e(X[3][0]), e(X[3][1])), (e(X[6][0]), e(X[6][1]))
        bwd(7, 3, 6, G[3], G[6], box=wbox[1])           # nconv5: down1's output + up
        G[4], G[5] = (e(X[4][0]), e(X[4][1])), (e(X[5][0]), e(X[5][1]))
        bwd(6, 4, 5, G[4], G[5], box=wbox[0])           # nconv4: down2's output + up
        if ctx.pooled:
            p2x, p2c, a2, p3x, p3c, a3, p4x, p4c, a4 = pools
            plain = [dataclasses.replace(sp[k], mode=_lib.PLAIN) for k in (2, 3, 4)]
            gp4 = (e(p4x), e(p4c))
            bwd(5, 0, 0, gp4, None, src_a=(p4x, p4c), spec=plain[2])     # down3 -> pooled gradient
            gp3 = (e(p3x), e(p3c))
            bwd(4, 0, 0, gp3, None, src_a=(p3x, p3c), spec=plain[1], pool_grad=(*gp4, a4))  # down2
            gp2 = (e(p2x), e(p2c))
            bwd(3, 0, 0, gp2, None, src_a=(p2x, p2c), spec=plain[0], pool_grad=(*gp3, a3))  # down1
            if FUSE_HEAD_BWD and not need[1]:  # nconv2's input gradient feeds nconv1's weight gradient in-tile
                args = (sp[1], (X[1][0], X[1][1], None, None, *W[1]), X[2][0], X[2][1], *G[2],
                        (None, None, None, None), gw[1], gb[1])
                kw = dict(pool_grad=(*gp2, a2), head=(sp[0], S, *W[0], gw[0], gb[0]))
                if WGRAD_LAST_MAIN:  # the last layer's weight gradient after its input gradient, on this stream
                    layer_backward(*args, defer=red, **kw)
                else:
                    layer_bwd(*args, **kw)
                finish()
                out = [None, None, None, None]
                for i in range(9):
                    out += [gw[i], gb[i], None]
                return tuple(out + [None] * ctx.n_extra)
            G[1] = (e(X[1][0]), e(X[1][1]))
            bwd(2, 1, 0, G[1], None, pool_grad=(*gp2, a2))                 # nconv2
        else:
            bwd(5, 4, 0, G[4], None, acc=True)              # down3 adds into down2's output gradient
            bwd(4, 3, 0, G[3], None, acc=True)              # down2 -> down1's
            bwd(3, 2, 0, G[2], None, acc=True)              # down1 -> nconv2's
            G[1] = (e(X[1][0]), e(X[1][1]))
            bwd(2, 1, 0, G[1], None)                        # nconv2
        gS = e(S) if need[1] else None
        layer_bwd(sp[0], (S, None, None, None, *W[0]), X[1][0], X[1][1], G[1][0], G[1][1],
                  (gS, None, None, None), gw[0], gb[0])  # nconv1 (threshold: c0 has no gradient)
        finish()
        out = [None, None, None, gS]
        for i in range(9):
            out += [gw[i], gb[i], None]
        return tuple(out + [None] * ctx.n_extra)


# Exact-fp32 training (DNETFn, pooled graph): the forward's head fused; nconv7's backward inside
# nconv6's and nconv1's weight gradient inside nconv2's input gradient (nconv_bwd_ex tail / head);
# the weight gradients on a second stream, concurrent with the input-gradient chain. Switches for
# tests.
FUSE_TAIL_BWD = True
FUSE_HEAD_BWD = True
FUSE_HEAD_FWD = True  # the training forward's nconv1 + nconv2 as the exact fused head (nconv_fwd_head)
FUSE_TAIL_FWD = True  # ... and nconv6 + nconv7 as the fused tail (nconv_fwd_tail over nconv7's whole grid)


def _tail_train(sp6, sp7, x2, c2, x7, c7, W6, W7, w6, crop=None, out=None):
    """nconv6 + nconv7 in one phase-tail launch writing nconv6's outputs and nconv7's whole
    (uncropped) output grid -- what the training backward reads (nconv_fwd_tail, crop0 = 0) -- or,
    with crop = (h, w), nconv7's output cropped as step1.py:94 (crop0 = 1). out: None or a callable
    as nconv._outputs takes."""
    L = sp6.descriptor(x2, c2, x7, c7, *W6, w6)
    (w7, b7, s7), p7 = W7, sp7.padding[0]
    B, dev = x2.shape[0], x2.device
    (H9, W9), crop0 = ((L.Ho + 2 * p7, L.Wo + 2 * p7), 0) if crop is None else (tuple(crop), 1)
    sh8, sh9 = (B, sp6.cout, L.Ho, L.Wo), (B, 1, H9, W9)
    x8, c8, x9, c9 = nconv._outputs(out, 4, (sh8, sh8, sh9, sh9), dev)
    rc = _lib.lib().nconv_fwd_tail(_lib.ctypes.byref(L), _lib.ptr(w7), _lib.ptr(b7), _lib.ptr(s7), sp7.cin, p7,
                                   sp7.eps, _lib.ptr(x9), _lib.ptr(c9), H9, W9, crop0, _lib.ptr(x8), _lib.ptr(c8),
                                   _lib.stream_handle(dev))
    _lib.check(rc, "nconv_fwd_tail")
    return x8, c8, x9, c9


class CropFn(torch.autograd.Function):
    """xo[:, :, 1:1+h, 1:1+w] (step1.py:94); its backward zero-pads the gradient in one launch
    (autograd's two slice backwards zero-fill and copy twice). The crop is returned as a fresh
    tensor (not a view, as the reference's slice is), so in-place operations on DNET's output
    (clamp_, masked_fill_, ...) stay legal under autograd; the copy is the output's size only."""

    @staticmethod
    def forward(ctx, x, h, w):
        ctx.pad = (1, x.shape[3] - 1 - w, 1, x.shape[2] - 1 - h)
        return x[:, :, 1:1 + h, 1:1 + w].contiguous()

    @staticmethod
    def backward(ctx, g):
        return torch.nn.functional.pad(g, ctx.pad), None, None


# The training backward's weight gradients on one side stream (two round-robin streams measured
# slower: 2.20 -> 2.26 ms per graphed step, profiles/r5_ab_two_wgrad_streams.log), except the last
# layer's (nconv2's, WGRAD_LAST_MAIN): it runs on the main stream after that layer's input
# gradient, which is the main stream's last kernel, instead of queueing behind the side stream's
# backlog while the main stream idles
WGRAD_STREAM = True
WGRAD_LAST_MAIN = True
_WGRAD_STREAMS = {}


def _wgrad_stream(device):
    if device.index not in _WGRAD_STREAMS:
        _WGRAD_STREAMS[device.index] = torch.cuda.Stream(device=device)
    return _WGRAD_STREAMS[device.index]


def _materialise_pool(S):
    """The training graph's pooled form (DNETFn): both arithmetics exact fp32 and every pooled
    level at least 2x2 (nconv_fwd_pooled / the pooled-gradient backward are built for that)."""
    return (nconv.FORWARD_MATH == _lib.MATH_FP32 and nconv.BACKWARD_MATH == _lib.MATH_FP32 and
            min(S.shape[2], S.shape[3]) >= 16)


def crop_hw(H, W, crop):
    """Output size after nconv7 (grid (H+2) x (W+2)) and the crop of step1.py:94."""
    if crop == "literal":
        return max(0, min(481, H + 2) - 1), max(0, min(641, W + 2) - 1)
    if crop == "generalized":
        return H, W
    raise ValueError(f"crop must be 'literal' or 'generalized', got {crop!r}")


class DNET(nn.Module):
    """NConv U-Net (step1.py:30-94). `out_ch` is accepted and ignored like the reference (:19,31,36).

    crop='literal' reproduces xout[:, :, 1:481, 1:641] (e.g. 353x640 at 352x1216 input);
    crop='generalized' returns [1:H+1, 1:W+1], identical to literal at 480x640.
    """

    def __init__(self, out_ch, crop="literal"):
        super().__init__()
        pos_fn = "softplus"
        num_channels = 8
        self.crop = crop
        self.nconv1 = NConv2d(1, num_channels, (5, 5), pos_fn, "p", padding=(2, 2))
        self.nconv2 = NConv2d(num_channels, num_channels, (5, 5), pos_fn, "p", padding=(2, 2))
        self.nconv_down1 = NConv2d(num_channels, num_channels, (5, 5), pos_fn, "p", padding=(2, 2))
        self.nconv_down2 = NConv2d(num_channels, num_channels, (5, 5), pos_fn, "p", padding=(2, 2))
        self.nconv_down3 = NConv2d(num_channels, num_channels, (5, 5), pos_fn, "p", padding=(2, 2))
        self.nconv4 = NConv2d(2 * num_channels, num_channels, (3, 3), pos_fn, "p", padding=(1, 1))
        self.nconv5 = NConv2d(2 * num_channels, num_channels, (3, 3), pos_fn, "p", padding=(1, 1))
        self.nconv6 = NConv2d(2 * num_channels, num_channels, (3, 3), pos_fn, "p", padding=(0, 0))
        self.nconv7 = NConv2d(num_channels, 1, (1, 1), pos_fn, "k")
        # Set to a dict to receive the (x, c) inputs of the three pooling stages on the next
        # forward (diagnostics / tests); None in normal use.
        self.capture = None

    # Training path: one autograd node for the whole graph (DNETFn, gradients of shared tensors
    # accumulated in-kernel); False: one node per layer (NConvLayerFn), for comparison.
    whole_graph_autograd = True

    # -- hooks ----------------------------------------------------------------------------------
    def _prologue(self, layers, S):
        """Run each layer's forward pre-hooks (EnforcePos) and compute s[o] for every layer."""
        batched_sp, weights, wsums = [], [], []
        for m in layers:
            hooks = list(m._forward_pre_hooks.values())
            ours = len(hooks) == 1 and isinstance(hooks[0], EnforcePos) and hooks[0].name == "weight" \
                and hooks[0].pos_fn.lower() == "softplus"
            if not ours:
                for h in hooks:
                    h(m, (S,))
            w = m.weight
            if not (w.is_cuda and w.dtype == torch.float32 and w.is_contiguous()):
                raise RuntimeError(f"{type(m).__name__}.weight must be a contiguous fp32 device tensor")
            weights.append(w.data)
            batched_sp.append(ours and m.training)
        buf = torch.empty(sum(w.shape[0] for w in weights), device=S.device, dtype=torch.float32)
        off = 0
        for w in weights:
            wsums.append(buf[off:off + w.shape[0]])
            off += w.shape[0]
        weight_prep(weights, batched_sp, wsums)
        return wsums

    def _train_prologue(self, layers, S):
        """(wsums, phase weights, head weights, box weights) of the whole-graph training pass from
        one nconv_train_prologue launch (EnforcePos applied in place first, as the hooks would),
        or None where the separate path must run: merged_prologue off, a forward pre-hook other
        than this package's softplus EnforcePos, weights that are not contiguous fp32 device
        tensors, or a matrix-core arithmetic. Phase / box weights are None when phase_upcat is off
        or the UpCat layers do not have the phase form's geometry; head weights None when the
        fused training head is off."""
        if not self.merged_prologue or nconv.FORWARD_MATH != _lib.MATH_FP32 or not _materialise_pool(S):
            return None
        sp = []
        for m in layers:
            hooks = list(m._forward_pre_hooks.values())
            ours = len(hooks) == 1 and isinstance(hooks[0], EnforcePos) and hooks[0].name == "weight" \
                and hooks[0].pos_fn.lower() == "softplus"
            if not (len(hooks) == 0 or ours):
                return None
            w = m.weight
            if not (w.is_cuda and w.dtype == torch.float32 and w.is_contiguous()):
                return None
            sp.append(ours and m.training)
        dev = S.device
        weights = [m.weight.data for m in layers]
        buf = torch.empty(sum(w.shape[0] for w in weights), device=dev, dtype=torch.float32)
        wsums, off = [], 0
        for w in weights:
            wsums.append(buf[off:off + w.shape[0]])
            off += w.shape[0]
        head, w21 = None, None
        if FUSE_HEAD_FWD and self._head_shapes(layers[0], layers[1]):
            w21 = torch.empty(nconv.HEAD_WEIGHTS_FLOATS, device=dev, dtype=torch.float32)
            head = (0, 1, w21, nconv.sync_counter(dev))
        phase, wph, wbox = None, None, None
        ls = (self.nconv4, self.nconv5, self.nconv6)
        if self.phase_upcat and all(m.weight.shape[0] == 8 and m.weight.shape[1] == 16 and
                                    tuple(m.weight.shape[2:]) == (3, 3) for m in ls):
            wph = torch.empty((3, 1024), device=dev, dtype=torch.float32)
            wbox = torch.empty((3, nconv.BOX_WEIGHT_FLOATS), device=dev, dtype=torch.float32)
            phase = ([5, 6, 7], [8, 8, 0], list(wph), list(wbox))
        train_prologue(weights, sp, wsums, head=head, phase=phase)
        return wsums, wph, w21, wbox

    # The whole-graph training pass writes DNET's cropped output from the fused tail where it can
    # (_tail_crop); False: nconv7's whole grid, then CropFn (tests compare the two).
    crop_in_tail = True

    def _tail_crop(self, S, wph):
        """Whether the whole-graph training pass writes DNET's cropped output straight from the
        fused tail (no crop copy, no zero-padded gradient): the pooled graph with the fused
        training tail and its backward, exactly-2x UpCat, a crop window covering every nconv6 pixel
        (crop0 = 1 <= nconv7's padding, the window at least (H - 1) x (W - 1): the generalized crop,
        or the literal one up to 481 x 641), and nconv7's weight gradient only with nconv6's
        (it is accumulated in nconv6's weight-gradient pass)."""
        H, W = S.shape[2], S.shape[3]
        oh, ow = crop_hw(H, W, self.crop)
        l6, l7 = self.nconv6, self.nconv7
        return (self.crop_in_tail and wph is not None and FUSE_TAIL_FWD and FUSE_TAIL_BWD and _materialise_pool(S) and H % 2 == 0
                and W % 2 == 0 and tuple(l7.padding) == (2, 2) and oh >= H - 1 and ow >= W - 1
                and (not l7.weight.requires_grad or l6.weight.requires_grad or l6.bias.requires_grad))

    # The eval-mode forward builds its weight-only prologue -- the normalisers, the exact head's
    # composed weights and nconv4/5/6's phase weights -- in one launch (nconv_weight_prologue,
    # bitwise the three separate launches); False: the separate launches.
    merged_prologue = True

    def _eval_prologue_ok(self, layers):
        """Whether the one-launch eval prologue applies (see _eval_prologue)."""
        if not self.merged_prologue:
            return False
        for m in layers:
            hooks = list(m._forward_pre_hooks.values())
            ours = len(hooks) == 1 and isinstance(hooks[0], EnforcePos) and hooks[0].name == "weight" \
                and hooks[0].pos_fn.lower() == "softplus"
            if m.training or not (len(hooks) == 0 or ours):
                return False
            w = m.weight
            if not (w.is_cuda and w.dtype == torch.float32 and w.is_contiguous()):
                return False
        return True

    def _eval_prologue(self, layers, S):
        """(wsums, phase weights or None, head weights or None) from one nconv_weight_prologue launch, or None where the separate path must run: merged_prologue off,
        a layer in training mode (EnforcePos then rewrites the weights first), a forward pre-hook
        other than this package's EnforcePos, or weights that are not contiguous fp32 device
        tensors."""
        if not self._eval_prologue_ok(layers):
            return None
        dev = S.device
        weights = [m.weight.data for m in layers]
        buf = torch.empty(sum(w.shape[0] for w in weights), device=dev, dtype=torch.float32)
        wsums, off = [], 0
        for w in weights:
            wsums.append(buf[off:off + w.shape[0]])
            off += w.shape[0]
        head = None
        l1, l2 = layers[0], layers[1]
        if nconv.FORWARD_MATH == _lib.MATH_FP32 and self._use_head(l1, l2):
            head = (l1.weight.data, l2.weight.data,
                    torch.empty(nconv.HEAD_WEIGHTS_FLOATS, device=dev, dtype=torch.float32))
        phase, wph = None, None
        ls = (self.nconv4, self.nconv5, self.nconv6)
        if self.phase_upcat and nconv.FORWARD_MATH == _lib.MATH_FP32 and all(
                m.weight.shape[0] == 8 and m.weight.shape[1] == 16 and tuple(m.weight.shape[2:]) == (3, 3)
                and m.weight.is_contiguous() for m in ls):
            wph = torch.empty((3, 1024), device=dev, dtype=torch.float32)
            phase = ([m.weight.data for m in ls], [8, 8, 0], list(wph))
        nconv.weight_prologue(weights, wsums, head=head, phase=phase)
        return wsums, wph, (head[2] if head is not None else None)

    # -- forward ----------------------------------------------------------------------------------
    def forward(self, S):
        if export.is_exporting():  # the export graph: the reference's own ops (export.py)
            return export.dnet(self, S)
        _require_device(S, "DNET.forward")
        if S.dim() != 4 or S.shape[1] != 1:
            raise ValueError(f"DNET expects (B, 1, H, W) sparse depth, got {tuple(S.shape)}")
        S = S.contiguous()
        layers = [getattr(self, n) for n in LAYERS]
        grad = torch.is_grad_enabled() and (S.requires_grad or any(p.requires_grad for p in self.parameters()))
        H, W = S.shape[2], S.shape[3]
        out_h, out_w = crop_hw(H, W, self.crop)
        if not grad and min(H, W) >= 16:
            out = torch.empty((S.shape[0], 1, out_h, out_w), device=S.device, dtype=torch.float32)
            pro = self._eval_prologue(layers, S)
            if pro is None:
                wsum, wph, w21 = self._prologue(layers, S), self._phase_weights(S.device), None
            else:
                wsum, wph, w21 = pro
            self._infer_split(S, layers, wsum, out, wph, w21)
            return out

        (l1, l2, d1, d2, d3, l4, l5, l6, l7) = layers
        if grad and self.whole_graph_autograd and S.shape[0] > 0:
            specs = (l1.spec(_lib.THRESH, 0.01), l2.spec(), d1.spec(_lib.POOL2), d2.spec(_lib.POOL2),
                     d3.spec(_lib.POOL2), l4.spec(_lib.UPCAT_SKIP_FIRST), l5.spec(_lib.UPCAT_SKIP_FIRST),
                     l6.spec(_lib.UPCAT_UP_FIRST), l7.spec())
            pro = self._train_prologue(layers, S)
            if pro is None:
                wsum = self._prologue(layers, S)
                wph = self._phase_weights(S.device)
                extra = (wph,)
            else:
                wsum, wph, w21, wbox = pro
                extra = (wph, w21, wbox)
            params = []
            for m_, s_ in zip(layers, wsum):
                params += [m_.weight, m_.bias, s_]
            crop = (out_h, out_w) if self._tail_crop(S, extra[0]) else None
            xo, _ = DNETFn.apply(specs, self.capture, crop, S, *params, *extra)
            return xo if crop is not None else CropFn.apply(xo, out_h, out_w)

        wsum = self._prologue(layers, S)
        (s1, s2, sd1, sd2, sd3, s4, s5, s6, s7) = wsum
        f = nconv_layer if grad else (lambda spec, *a, wphase=None: layer_forward_raw(spec, *a, wphase=wphase))

        wph = self._phase_weights(S.device)
        w4, w5, w6 = (None, None, None) if wph is None else tuple(wph)

        x1, c1 = f(l1.spec(_lib.THRESH, 0.01), S, None, None, None, l1.weight, l1.bias, s1)
        x1, c1 = f(l2.spec(), x1, c1, None, None, l2.weight, l2.bias, s2)
        x2, c2 = f(d1.spec(_lib.POOL2), x1, c1, None, None, d1.weight, d1.bias, sd1)
        x3, c3 = f(d2.spec(_lib.POOL2), x2, c2, None, None, d2.weight, d2.bias, sd2)
        x4, c4 = f(d3.spec(_lib.POOL2), x3, c3, None, None, d3.weight, d3.bias, sd3)
        if self.capture is not None:
            self.capture.update(down1=(x1.detach(), c1.detach()), down2=(x2.detach(), c2.detach()),
                                down3=(x3.detach(), c3.detach()))
        x34, c34 = f(l4.spec(_lib.UPCAT_SKIP_FIRST), x3, c3, x4, c4, l4.weight, l4.bias, s4, wphase=w4)
        x23, c23 = f(l5.spec(_lib.UPCAT_SKIP_FIRST), x2, c2, x34, c34, l5.weight, l5.bias, s5, wphase=w5)
        xo, co = f(l6.spec(_lib.UPCAT_UP_FIRST), x1, c1, x23, c23, l6.weight, l6.bias, s6, wphase=w6)
        xo, co = f(l7.spec(), xo, co, None, None, l7.weight, l7.bias, s7)
        return xo[:, :, 1:1 + out_h, 1:1 + out_w]

    # -- inference ------------------------------------------------------------------------------
    # Exact-fp32 inference convolves the nearest-2x-upsampled half of nconv4/5/6's inputs at its
    # own resolution with phase weights (include/nconv.h nconv_layer.wphase; the kernel uses them
    # where the upsampling is exactly 2x); False: the 3x3 taps over the upsampled planes.
    phase_upcat = True

    def _phase_weights(self, device):
        """Phase weights of nconv4, nconv5 (cat(skip, up): up channels 8..15) and nconv6
        (cat(up, skip): 0..7) from the current weights, one launch; None when not in use."""
        if not self.phase_upcat or nconv.FORWARD_MATH != _lib.MATH_FP32:
            return None
        ls = (self.nconv4, self.nconv5, self.nconv6)
        if any(m.weight.shape[0] != 8 or m.weight.shape[1] != 16 or tuple(m.weight.shape[2:]) != (3, 3)
               for m in ls):
            return None
        buf = torch.empty((3, 1024), device=device, dtype=torch.float32)
        phase_weights([m.weight for m in ls], [8, 8, 0], list(buf))
        return buf
    # Frames are independent, so the batch can be split over `inference_streams` HIP streams, each
    # running the whole layer chain on its share, so that one stream's kernels fill the partial
    # last round of the other's (and its small quarter / eighth-resolution layers overlap the other
    # share's large ones). None = automatic: 2 for the exact-fp32 kernels (B=8 352x1216: 0.616 vs
    # 0.628 ms), 1 for the matrix-core maths, whose persistent grids are sized to the chip and
    # leave no such gaps (0.507 vs 0.555 ms). A frame's result does not depend on the split.
    inference_streams = None
    # Frames per stream of the inference split, as relative shares (None = even); an uneven split
    # staggers the streams' phases so one stream's small quarter / eighth-resolution layers run
    # beside the other's full-resolution head or tail instead of beside its own small layers.
    inference_shares = None

    def _n_streams(self, B):
        return max(1, min(self._configured_streams(), B))

    def _configured_streams(self):
        n = self.inference_streams
        if n is None:
            n = 2 if nconv.FORWARD_MATH == _lib.MATH_FP32 else 1
        return int(n)

    @staticmethod
    def split_bounds(B, n, shares=None, configured=None):
        """Frame bounds [b0 = 0, b1, ..., bn = B] of an n-way inference split: even, or by the
        relative `shares` (one positive finite number per configured stream). Shares whose count
        differs from the configured stream count, or that are not all positive and finite, raise
        ValueError; when the batch is smaller than the configured count (n clamped to B) the split
        is even."""
        bounds = [B * k // n for k in range(n + 1)]
        if shares is None:
            return bounds
        sh = [float(v) for v in shares]
        want = n if configured is None else configured
        if len(sh) != want:
            raise ValueError(f"inference_shares has {len(sh)} entries for {want} inference streams")
        if not all(math.isfinite(v) and v > 0 for v in sh):
            raise ValueError(f"inference_shares must be positive and finite, got {tuple(shares)}")
        if len(sh) != n:  # batch smaller than the configured streams: even split
            return bounds
        tot, acc = sum(sh), 0.0
        for k in range(1, n):
            acc += sh[k - 1]
            bounds[k] = min(max(int(round(B * acc / tot)), bounds[k - 1]), B)
        return bounds

    def _side_streams(self, device, n):
        key = (device.index, n)
        cache = self.__dict__.setdefault("_stream_cache", {})
        if key not in cache:
            cache[key] = [torch.cuda.Stream(device=device) for _ in range(n)]
        return cache[key]

    def _infer_split(self, S, layers, wsum, out, wph=None, w21=None):
        """The inference chain on batch slices, one stream each (the weight prologue once, on the
        current stream, before the fork: a prologue per stream measured slower, 16.3-16.5 k against
        16.9-17.2 k frames/s, profiles/r5_ab_stream_prologue.log)."""
        B = S.shape[0]
        n = self._n_streams(B)
        bounds = self.split_bounds(B, n, self.inference_shares, self._configured_streams())
        if n == 1:
            self._infer(S, layers, wsum, out, wph, w21=w21)
            return
        cur = torch.cuda.current_stream(S.device)
        side = self._side_streams(S.device, n - 1)
        for st in side:
            st.wait_stream(cur)
        for k, st in enumerate([cur] + side):
            if bounds[k + 1] == bounds[k]:
                continue
            with torch.cuda.stream(st):
                Sk = S[bounds[k]:bounds[k + 1]]
                self._infer(Sk, layers, wsum, out[bounds[k]:bounds[k + 1]], wph, w21=w21)
        for st in side:
            cur.wait_stream(st)

    def _infer(self, S, layers, wsum, out, wph=None, w21=None):
        """The inference chain on the current stream: each producer also writes the pooled input
        of the next down layer, and nconv6+nconv7+crop run as one launch writing `out`. wph: the
        phase weights of nconv4/5/6 (_phase_weights) or None. w21: the exact head's weights when
        the prologue already built them (_eval_prologue), else built here."""
        (l1, l2, d1, d2, d3, l4, l5, l6, l7) = layers
        (s1, s2, sd1, sd2, sd3, s4, s5, s6, s7) = wsum
        w4, w5, w6 = (None, None, None) if wph is None else tuple(wph)
        f, fp = layer_forward_raw, layer_forward_pooled
        if self._use_head(l1, l2):
            # nconv1 inside nconv2's staging: its 8-channel output never reaches HBM
            sp1, sp2 = l1.spec(_lib.THRESH, 0.01), l2.spec()
            if w21 is None and nconv.FORWARD_MATH == _lib.MATH_FP32:  # the exact head's composed weights
                w21 = head_weights(sp1, sp2, S, l1.weight, l1.bias, s1, l2.weight, l2.bias, s2)
            x1, c1, p1, q1 = layer_forward_head(sp1, sp2, S, l1.weight, l1.bias, s1, l2.weight, l2.bias, s2, w21)
        else:
            x1, c1 = f(l1.spec(_lib.THRESH, 0.01), S, None, None, None, l1.weight, l1.bias, s1)
            x1, c1, p1, q1 = fp(l2.spec(), x1, c1, None, None, l2.weight, l2.bias, s2)
        x2, c2, p2, q2 = fp(d1.spec(), p1, q1, None, None, d1.weight, d1.bias, sd1)
        x3, c3, p3, q3 = fp(d2.spec(), p2, q2, None, None, d2.weight, d2.bias, sd2)
        x4, c4 = f(d3.spec(), p3, q3, None, None, d3.weight, d3.bias, sd3)
        x34, c34 = f(l4.spec(_lib.UPCAT_SKIP_FIRST), x3, c3, x4, c4, l4.weight, l4.bias, s4, wphase=w4)
        if self.capture is not None:
            self.capture.update(down1=(x1, c1), down2=(x2, c2), down3=(x3, c3))
        x23, c23 = f(l5.spec(_lib.UPCAT_SKIP_FIRST), x2, c2, x34, c34, l5.weight, l5.bias, s5, wphase=w5)
        self._fused_tail(l6, l7, s6, s7, x1, c1, x23, c23, out, w6)

    # Inference evaluates nconv1 inside nconv2's kernel (nconv_fwd_head) when the layers have
    # DNET's geometry -- in exact fp32 with nconv1 on the nonzero taps only and nconv2's confidence
    # mass from composed weights (include/nconv.h nconv_fwd_head); set False to run them as two
    # launches.
    fused_head = True

    def _use_head(self, l1, l2):
        return self.fused_head and self._head_shapes(l1, l2)

    @staticmethod
    def _head_shapes(l1, l2):
        return (l1.in_channels, l1.out_channels, tuple(l1.kernel_size), tuple(l1.padding), tuple(l1.stride)) == \
            (1, 8, (5, 5), (2, 2), (1, 1)) and \
            (l2.in_channels, l2.out_channels, tuple(l2.kernel_size), tuple(l2.padding), tuple(l2.stride)) == \
            (8, 8, (5, 5), (2, 2), (1, 1)) and tuple(l1.dilation) == (1, 1) and tuple(l2.dilation) == (1, 1) \
            and l1.groups == 1 and l2.groups == 1

    def _fused_tail(self, l6, l7, s6, s7, x1, c1, x23, c23, out, w6=None):
        """nconv6 + nconv7 + crop into `out` (nconv_fwd_tail)."""
        out_h, out_w = out.shape[2], out.shape[3]
        if out_h == 0 or out_w == 0 or out.shape[0] == 0:
            return out
        L = l6.spec(_lib.UPCAT_UP_FIRST).descriptor(x1, c1, x23, c23, l6.weight, l6.bias, s6, w6)
        if tuple(l7.kernel_size) != (1, 1) or l7.padding[0] != l7.padding[1] or tuple(l7.stride) != (1, 1):
            raise RuntimeError("fused tail needs nconv7 = 1x1, stride 1, square padding")
        rc = _lib.lib().nconv_fwd_tail(
            _lib.ctypes.byref(L), _lib.ptr(l7.weight), _lib.ptr(l7.bias), _lib.ptr(s7), l7.in_channels,
            l7.padding[0], l7.eps, _lib.ptr(out), None, out_h, out_w, 1, None, None, _lib.stream_handle(x1.device))
        _lib.check(rc, "nconv_fwd_tail")
        return out


class SETP1_NCONV(nn.Module):
    """Unguided depth network wrapper (step1.py:15-27); state_dict prefix `d_net.`.

    forward(S) -> d_net(S). Also accepts forward(depth0, depth1, ...) and runs DNET on their
    batch concatenation: the call the guided model makes (models/step2.py:62,107), which the
    reference's one-argument forward rejects with a TypeError.
    """

    def __init__(self, crop="literal"):
        super().__init__()
        self.d_net = DNET(32, crop=crop)

    def forward(self, x0_d, *more):
        if more:
            x0_d = torch.cat((x0_d,) + tuple(more), dim=0)
        return self.d_net(x0_d)
