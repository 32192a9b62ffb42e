"""RGB-guided depth refinement — drop-in for the reference's models/step2.py:22-297.

SETP2_BP_TRAIN / SETP2_BP_EXPORT keep the reference's constructors, forward(rgb0, depth0, rgb1,
depth1), submodule names (hence state_dict keys, including the unused rgb_encoder4 of the TRAIN
variant, step2.py:46) and RNG consumption order. Step 1 is this package's SETP1_NCONV (libnconv
kernels); it is called as step1(depth0, depth1), which the reference intends (step2.py:62-63) but
its one-argument SETP1_NCONV.forward rejects.

Inference (eval mode, no autograd): every dense convolution of the RGB encoder and the fusion
decoder runs on libnconv's fp32-MFMA kernels (dense.py, nconv_dense_conv_fwd) with eval
BatchNorm folded into the packed weights, bias + ReLU + the RGBEncoder shortcut fused into the
epilogue, and each torch.cat replaced by two-source loads / channel-offset stores.

Training (or any forward that records autograd) on the device: every convolution is a
dense.DenseConvFn / dense.HeadFn — forward, input gradient and weight gradient on the same MFMA
kernels, ReLU after a bias-only convolution fused, torch.cat replaced by two-source loads — and
training-mode BatchNorm (batch statistics, running-stat updates) + ReLU on libnconv's BN kernels
(dense.bn_relu); the bilinear depth downsampling on nconv_bilinear_ac (the reference CPU kernel's
sampling arithmetic, dense.bilinear_down).
`model.dense_kernels = False` runs the dense layers as the plain torch modules — the fp32
PyTorch reference the GPU tests compare the kernels against (tests/test_gpu_dense.py), not a
product path (step 1 still runs on libnconv and refuses CPU tensors).
"""
import os
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import dense as D
from .dnet import SETP1_NCONV


def _bn_act(y, bn, act):
    """act(bn(y)): BatchNorm (+ ReLU) on libnconv's kernels (dense.bn_relu)."""
    if isinstance(act, nn.ReLU):
        return D.bn_relu(y, bn, True)
    return act(D.bn_relu(y, bn, False))


def Conv1x1(in_planes, out_planes, stride, bias=False, groups=1, dilation=1, padding_mode="zeros"):
    """1x1 projection shortcut (step2.py:130-132)."""
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=bias)


def Conv3x3(in_planes, stride=1, groups=1, dilation=1, padding_mode="zeros", bias=False):
    """3x3 residual head producing one depth channel (step2.py:156-158)."""
    return nn.Conv2d(in_planes, 1, kernel_size=3, stride=stride, padding=dilation, padding_mode=padding_mode,
                     groups=groups, bias=bias, dilation=dilation)


class RGBEncoder(nn.Module):
    """ReLU(BN(conv3x3_s(x))) + conv1x1_s(x) (step2.py:134-154)."""

    def __init__(self, in_channel, out_channel, stride):
        super().__init__()
        self.stride = stride
        self.encoder = nn.Sequential(
            nn.Conv2d(in_channels=in_channel, out_channels=out_channel, kernel_size=3, stride=stride, padding=1),
            nn.BatchNorm2d(out_channel),
            nn.ReLU(inplace=True))
        self.downsample = nn.Sequential(Conv1x1(in_channel, out_channel, stride))

    def forward(self, x):
        return self.encoder(x) + self.downsample(x)

    def dense_plans(self):
        """(packed 3x3 weights with eval BN folded, shift, packed shortcut), cached (dense.cached)."""
        conv, bn, sc = self.encoder[0], self.encoder[1], self.downsample[0]

        def build():
            scale, shift = D.bn_fold(bn, conv.bias)
            return (D.pack(D.DENSE_3X3, conv.weight, conv.in_channels, conv.out_channels, scale), shift,
                    D.pack(D.DENSE_1X1, sc.weight, sc.in_channels, sc.out_channels))
        return D.cached(self, "enc", [conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean,
                                      bn.running_var, sc.weight], build)

    def dense_forward(self, x):
        conv = self.encoder[0]
        wp, bias, ws = self.dense_plans()
        return D.conv(x, D.DENSE_3X3, conv.stride[0], wp, bias, True, conv.out_channels, wshort=ws)

    def train_forward(self, x):
        conv, bn, act, sc = self.encoder[0], self.encoder[1], self.encoder[2], self.downsample[0]
        y = _bn_act(D.conv_fn(x, conv.weight, conv.bias, D.DENSE_3X3, conv.stride[0]), bn, act)
        return y + D.conv_fn(x, sc.weight, None, D.DENSE_1X1, sc.stride[0])


class Basic2d(nn.Module):
    """conv (+BN when norm_layer, then no conv bias) + activation (step2.py:178-195)."""

    def __init__(self, in_channels, out_channels, norm_layer=None, kernel_size=3, padding=1, padding_mode="zeros",
                 act=nn.ReLU, stride=1):
        super().__init__()
        conv = nn.Conv2d(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=padding, bias=not norm_layer, padding_mode=padding_mode)
        self.conv = nn.Sequential(OrderedDict([("conv", conv)]))
        if norm_layer:
            self.conv.add_module("bn", norm_layer(out_channels))
        self.conv.add_module("relu", act())

    def forward(self, x):
        return self.conv(x)

    def dense_plans(self):
        conv = self.conv.conv
        bn = getattr(self.conv, "bn", None)
        if conv.kernel_size != (3, 3) or conv.padding != (1, 1) or not isinstance(self.conv.relu, nn.ReLU):
            raise NotImplementedError("dense path: 3x3 / padding 1 / ReLU Basic2d only")

        def build():
            if bn is not None:
                scale, shift = D.bn_fold(bn, conv.bias)
            else:
                scale, shift = None, conv.bias.detach().contiguous()
            return D.pack(D.DENSE_3X3, conv.weight, conv.in_channels, conv.out_channels, scale), shift
        ts = [conv.weight] + ([conv.bias] if conv.bias is not None else []) + \
            ([bn.weight, bn.bias, bn.running_mean, bn.running_var] if bn is not None else [])
        return D.cached(self, "conv", ts, build)

    def dense_forward(self, x0, x1=None, out=None, out_c0=0):
        conv = self.conv.conv
        wp, bias = self.dense_plans()
        return D.conv(x0, D.DENSE_3X3, conv.stride[0], wp, bias, True, conv.out_channels, x1=x1, out=out,
                      out_c0=out_c0)

    def train_forward(self, x0, x1=None):
        conv, bn, act = self.conv.conv, getattr(self.conv, "bn", None), self.conv.relu
        if conv.kernel_size != (3, 3) or conv.padding != (1, 1):
            raise NotImplementedError("dense path: 3x3 / padding 1 Basic2d only")
        fuse = bn is None and isinstance(act, nn.ReLU)  # conv + bias + ReLU in one kernel
        y = D.conv_fn(x0, conv.weight, conv.bias, D.DENSE_3X3, conv.stride[0], relu=fuse, x1=x1)
        return y if fuse else (_bn_act(y, bn, act) if bn is not None else act(y))


class Basic2dTrans(nn.Module):
    """ConvTranspose 4x4 / stride 2 / padding 1 + BN + activation (step2.py:197-214)."""

    def __init__(self, in_channels, out_channels, norm_layer=None, act=nn.ReLU):
        super().__init__()
        bias = norm_layer is None
        self.conv = nn.ConvTranspose2d(in_channels=in_channels, out_channels=out_channels, kernel_size=4, stride=2,
                                       padding=1, bias=bias)
        self.bn = (norm_layer or nn.Identity)(out_channels)
        self.relu = act()

    def forward(self, x):
        return self.relu(self.bn(self.conv(x.contiguous())))

    def dense_plans(self):
        conv, bn = self.conv, self.bn

        def build():
            if isinstance(bn, nn.BatchNorm2d):
                scale, shift = D.bn_fold(bn, conv.bias)
            else:
                scale = None
                shift = conv.bias.detach().contiguous() if conv.bias is not None else None
            return D.pack(D.DENSE_TRANSPOSED_4X4, conv.weight, conv.in_channels, conv.out_channels, scale), shift
        ts = [conv.weight] + ([conv.bias] if conv.bias is not None else []) + \
            ([bn.weight, bn.bias, bn.running_mean, bn.running_var] if isinstance(bn, nn.BatchNorm2d) else [])
        return D.cached(self, "convT", ts, build)

    def dense_forward(self, x0, x1=None):
        wp, bias = self.dense_plans()
        return D.conv(x0, D.DENSE_TRANSPOSED_4X4, 2, wp, bias, isinstance(self.relu, nn.ReLU),
                      self.conv.out_channels, x1=x1)

    def train_forward(self, x0, x1=None):
        y = D.conv_fn(x0, self.conv.weight, self.conv.bias, D.DENSE_TRANSPOSED_4X4, 2, x1=x1)
        return _bn_act(y, self.bn, self.relu) if isinstance(self.bn, nn.BatchNorm2d) else self.relu(self.bn(y))


class UpCat(nn.Module):
    """Upsample cat(x, d) by the transposed conv, then fuse with the skip y (step2.py:160-176)."""

    def __init__(self, in_channels, out_channels, norm_layer=nn.BatchNorm2d, kernel_size=3, padding=1,
                 padding_mode="zeros", act=nn.ReLU):
        super().__init__()
        self.upf = Basic2dTrans(in_channels + 1, out_channels, norm_layer=norm_layer, act=act)
        self.conv = Basic2d(out_channels * 2, out_channels, norm_layer=norm_layer, kernel_size=kernel_size,
                            padding=padding, padding_mode=padding_mode, act=act)

    def forward(self, y, x, d):
        up = self.upf(torch.cat([x, d], dim=1))
        return self.conv(torch.cat([up, y], dim=1))

    def dense_forward(self, y, x, d):
        up = self.upf.dense_forward(x, d)
        return self.conv.dense_forward(up, y)

    def train_forward(self, y, x, d):
        return self.conv.train_forward(self.upf.train_forward(x, d), y)


class ConvBlock(nn.Module):
    """3x3 conv (bias) + ReLU (step2.py:290-297)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding)
        self.relu = nn.ReLU()

    def forward(self, x):
        return self.relu(self.conv(x))

    def dense_plans(self):
        conv = self.conv

        def build():
            return D.pack(D.DENSE_3X3, conv.weight, conv.in_channels, conv.out_channels), conv.bias.detach().contiguous()
        return D.cached(self, "conv", [conv.weight, conv.bias], build)

    def dense_forward(self, x, out=None, out_c0=0):
        conv = self.conv
        wp, bias = self.dense_plans()
        return D.conv(x, D.DENSE_3X3, conv.stride[0], wp, bias, True, conv.out_channels, out=out, out_c0=out_c0)

    def train_forward(self, x0, x1=None):
        conv = self.conv
        return D.conv_fn(x0, conv.weight, conv.bias, D.DENSE_3X3, conv.stride[0], relu=True, x1=x1)


class NewFusionBlock(nn.Module):
    """rgb / depth branches, concat, three fusing convs (step2.py:216-236)."""

    def __init__(self, rgb_channels, out_channels):
        super().__init__()
        self.rgb_conv = ConvBlock(rgb_channels, rgb_channels)
        self.depth_conv = ConvBlock(1, rgb_channels)
        self.fuse_conv1 = ConvBlock(rgb_channels * 2, rgb_channels)
        self.fuse_conv2 = ConvBlock(rgb_channels, out_channels)
        self.fuse_conv3 = ConvBlock(out_channels, out_channels)

    def forward(self, rgb, depth):
        fused = torch.cat((self.rgb_conv(rgb), self.depth_conv(depth)), 1)
        return self.fuse_conv3(self.fuse_conv2(self.fuse_conv1(fused)))

    def dense_forward(self, rgb, depth):
        C = self.rgb_conv.conv.out_channels
        B, _, H, W = rgb.shape
        fused = torch.empty((B, 2 * C, H, W), device=rgb.device, dtype=torch.float32)
        self.rgb_conv.dense_forward(rgb, out=fused, out_c0=0)      # the cat, written in place
        self.depth_conv.dense_forward(depth, out=fused, out_c0=C)
        return self.fuse_conv3.dense_forward(self.fuse_conv2.dense_forward(self.fuse_conv1.dense_forward(fused)))

    def train_forward(self, rgb, depth):
        # the torch.cat of step2.py:232 becomes fuse_conv1's two-source input
        f = self.fuse_conv1.train_forward(self.rgb_conv.train_forward(rgb), self.depth_conv.train_forward(depth))
        return self.fuse_conv3.train_forward(self.fuse_conv2.train_forward(f))


class FusionResolutionBlock(nn.Module):
    """One decoder scale: UpCat, bilinear depth downsample (align_corners=True), fusion, residual
    depth head (step2.py:238-259)."""

    def __init__(self, in_channel, out_channel, downsample_factor):
        super().__init__()
        self.upcat = UpCat(in_channel, in_channel)
        self.fuse = NewFusionBlock(in_channel, out_channel)
        self.conv = Conv3x3(out_channel, 1)
        self.downsample_factor = downsample_factor

    def forward(self, rgb, depth, depth_last_step, fusion_festure):
        fout = self.upcat(rgb, fusion_festure, depth_last_step)
        depth = F.interpolate(depth, scale_factor=1 / self.downsample_factor, mode="bilinear", align_corners=True)
        fout = self.fuse(fout, depth)
        return fout, depth + self.conv(fout)

    def dense_forward(self, rgb, depth, depth_last_step, fusion_festure):
        fout = self.upcat.dense_forward(rgb, fusion_festure, depth_last_step)
        depth = D.bilinear_down(depth, self.downsample_factor)
        fout = self.fuse.dense_forward(fout, depth)
        return fout, D.conv3x3_c1(fout, self.conv.weight, depth)

    def train_forward(self, rgb, depth, depth_last_step, fusion_festure):
        fout = self.upcat.train_forward(rgb, fusion_festure, depth_last_step)
        depth = D.bilinear_down(depth, self.downsample_factor)
        fout = self.fuse.train_forward(fout, depth)
        return fout, D.head_fn(fout, self.conv.weight, depth)


class FusionResolution0(nn.Module):
    """Coarsest decoder scale (step2.py:262-278)."""

    def __init__(self, in_channel, downsample_factor):
        super().__init__()
        self.fuse = NewFusionBlock(in_channel, in_channel)
        self.conv = Conv3x3(in_channel, 1)
        self.downsample_factor = downsample_factor

    def forward(self, rgb, depth):
        depth = F.interpolate(depth, scale_factor=1 / self.downsample_factor, mode="bilinear", align_corners=True)
        fout = self.fuse(rgb, depth)
        return fout, depth + self.conv(fout)

    def dense_forward(self, rgb, depth):
        depth = D.bilinear_down(depth, self.downsample_factor)
        fout = self.fuse.dense_forward(rgb, depth)
        return fout, D.conv3x3_c1(fout, self.conv.weight, depth)

    def train_forward(self, rgb, depth):
        depth = D.bilinear_down(depth, self.downsample_factor)
        fout = self.fuse.train_forward(rgb, depth)
        return fout, D.head_fn(fout, self.conv.weight, depth)


def _encoders_and_decoder(m, first_set):
    """Submodule construction in the reference's order (RNG consumption parity)."""
    if first_set:  # SETP2_BP_TRAIN builds a first encoder set and overwrites 0-3 (step2.py:42-51)
        m.rgb_encoder0 = RGBEncoder(3, 32, 1)
        m.rgb_encoder1 = RGBEncoder(32, 32, 2)
        m.rgb_encoder2 = RGBEncoder(32, 64, 2)
        m.rgb_encoder3 = RGBEncoder(64, 64, 2)
        m.rgb_encoder4 = RGBEncoder(64, 64, 2)  # never used in forward; kept for state_dict keys
    m.rgb_encoder0 = RGBEncoder(3, 32, 1)
    m.rgb_encoder1 = RGBEncoder(32, 64, 2)
    m.rgb_encoder2 = RGBEncoder(64, 64, 2)
    m.rgb_encoder3 = RGBEncoder(64, 64, 2)
    m.fuse0 = FusionResolution0(64, 8)
    m.fuse1 = FusionResolutionBlock(64, 64, 4)
    m.fuse2 = FusionResolutionBlock(64, 32, 2)
    m.fuse3 = FusionResolutionBlock(32, 32, 1)


def _use_dense(m, x):
    """libnconv's MFMA kernels for the dense convolutions: eval mode, device tensors, no autograd."""
    if m.training or not x.is_cuda or not getattr(m, "dense_kernels", True):
        return False
    return not (torch.is_grad_enabled() and any(p.requires_grad for p in m.parameters()))


# The eval (dense) forward's encoders and decoder in this many batch slices, one stream each (every
# frame's arithmetic is per frame: bitwise the one-stream pass); 1 = one launch per layer
GUIDED_STREAMS = int(os.environ.get("NCONV_GUIDED_STREAMS", "2"))
_GUIDED_STREAMS = {}


def _dense_chain(m, rgb, sparse):
    e0 = m.rgb_encoder0.dense_forward(rgb)
    e1 = m.rgb_encoder1.dense_forward(e0)
    e2 = m.rgb_encoder2.dense_forward(e1)
    e3 = m.rgb_encoder3.dense_forward(e2)
    f0, d0 = m.fuse0.dense_forward(e3, sparse)
    f1, d1 = m.fuse1.dense_forward(e2, sparse, f0, d0)
    f2, d2 = m.fuse2.dense_forward(e1, sparse, f1, d1)
    f3, d3 = m.fuse3.dense_forward(e0, sparse, f2, d2)
    return d0, d1, d2, d3


_DENSE_CHAIN = ("rgb_encoder0", "rgb_encoder1", "rgb_encoder2", "rgb_encoder3", "fuse0", "fuse1", "fuse2", "fuse3")


def prepare_dense_plans(m):
    """Build (or validate) every packed-weight plan the eval chain reads, on the current stream.
    The batch-sliced forward calls this before forking: a plan built lazily inside one slice's
    chain would be launched on that slice's stream, and the other slices -- which find it cached --
    would read it with no ordering after the pack launch (a cold cache, or any weight / BatchNorm
    change bumping a version counter)."""
    for name in _DENSE_CHAIN:
        for mod in getattr(m, name).modules():
            plans = getattr(mod, "dense_plans", None)
            if plans is not None:
                plans()


def _guided_forward_dense(m, rgb0, depth0, rgb1, depth1):
    sparse = m.step1(depth0, depth1).contiguous()
    rgb = torch.cat((rgb0, rgb1), dim=0).contiguous()
    B = rgb.shape[0]
    n = max(1, min(int(GUIDED_STREAMS), B))
    if n == 1:
        return _dense_chain(m, rgb, sparse)
    dev = rgb.device
    prepare_dense_plans(m)  # on cur, before the side streams' wait_stream(cur)
    if (dev.index, n) not in _GUIDED_STREAMS:
        _GUIDED_STREAMS[(dev.index, n)] = [torch.cuda.Stream(device=dev) for _ in range(n - 1)]
    side = _GUIDED_STREAMS[(dev.index, n)]
    cur = torch.cuda.current_stream(dev)
    for st in side:
        st.wait_stream(cur)
    bounds = [B * k // n for k in range(n + 1)]
    parts = []
    for k, st in enumerate([cur] + side):
        with torch.cuda.stream(st):
            parts.append(_dense_chain(m, rgb[bounds[k]:bounds[k + 1]], sparse[bounds[k]:bounds[k + 1]]))
    for st in side:
        cur.wait_stream(st)
    for part in parts[1:]:  # the side streams' outputs are read on cur (under capture the
        for t in part:      # allocator holds such blocks until the capture ends)
            t.record_stream(cur)
    return tuple(torch.cat([part[i] for part in parts], dim=0) for i in range(4))


def _guided_forward_train(m, rgb0, depth0, rgb1, depth1):
    """Autograd-recording forward with every convolution on the MFMA kernels (dense.conv_fn)."""
    sparse = m.step1(depth0, depth1)
    rgb = torch.cat((rgb0, rgb1), dim=0)
    e0 = m.rgb_encoder0.train_forward(rgb)
    e1 = m.rgb_encoder1.train_forward(e0)
    e2 = m.rgb_encoder2.train_forward(e1)
    e3 = m.rgb_encoder3.train_forward(e2)
    f0, d0 = m.fuse0.train_forward(e3, sparse)
    f1, d1 = m.fuse1.train_forward(e2, sparse, f0, d0)
    f2, d2 = m.fuse2.train_forward(e1, sparse, f1, d1)
    f3, d3 = m.fuse3.train_forward(e0, sparse, f2, d2)
    return d0, d1, d2, d3


def _guided_forward(m, rgb0, depth0, rgb1, depth1):
    if _use_dense(m, rgb0):
        return _guided_forward_dense(m, rgb0, depth0, rgb1, depth1)
    if rgb0.is_cuda and getattr(m, "dense_kernels", True):
        return _guided_forward_train(m, rgb0, depth0, rgb1, depth1)
    sparse = m.step1(depth0, depth1)
    rgb = torch.cat((rgb0, rgb1), dim=0)
    e0 = m.rgb_encoder0(rgb)
    e1 = m.rgb_encoder1(e0)
    e2 = m.rgb_encoder2(e1)
    e3 = m.rgb_encoder3(e2)
    # the reference passes (features, depth) into the (depth_last_step, fusion_festure) slots
    # (step2.py:72-74 vs :248), so UpCat concatenates [depth, features]; kept as is
    f0, d0 = m.fuse0(e3, sparse)
    f1, d1 = m.fuse1(e2, sparse, f0, d0)
    f2, d2 = m.fuse2(e1, sparse, f1, d1)
    f3, d3 = m.fuse3(e0, sparse, f2, d2)
    return d0, d1, d2, d3


class SETP2_BP_TRAIN(nn.Module):
    """Guided training model (step2.py:22-77). Loads ./checkpoints/<name>.pth.tar into step 1
    (weights-only load, `module.` prefix stripped, strict=False) and freezes it. forward returns the
    four scales of frame pair 0 and of frame pair 1 (batch slices [0:1] and [1:2])."""

    def __init__(self, step1_checkpoint_name, step1_crop="literal", checkpoint_dir="./checkpoints"):
        super().__init__()
        self.step1 = SETP1_NCONV(crop=step1_crop)
        if step1_checkpoint_name is not None:
            from .train import load_checkpoint
            load_checkpoint(self.step1, f"{checkpoint_dir}/{step1_checkpoint_name}.pth.tar", strict=False)
        for p in self.step1.parameters():
            p.requires_grad = False
        _encoders_and_decoder(self, first_set=True)

    def forward(self, rgb0, depth0, rgb1, depth1):
        d = _guided_forward(self, rgb0, depth0, rgb1, depth1)
        return [x[0:1] for x in d], [x[1:2] for x in d]


class SETP2_BP_EXPORT(nn.Module):
    """Guided export model (step2.py:80-126): finest scale only, with 45 rows top and bottom and
    20 columns on the left zeroed; returns (frame 0, frame 1)."""

    def __init__(self, step1_crop="literal"):
        super().__init__()
        self.step1 = SETP1_NCONV(crop=step1_crop)
        _encoders_and_decoder(self, first_set=False)

    def forward(self, rgb0, depth0, rgb1, depth1):
        d3 = _guided_forward(self, rgb0, depth0, rgb1, depth1)[3]
        d3[:, :, :45, :] = 0
        d3[:, :, -45:, :] = 0
        d3[:, :, :, :20] = 0
        return d3[0:1], d3[1:2]
