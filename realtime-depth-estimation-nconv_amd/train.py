"""Training-step glue of the reference (utils.py), on device: losses, optimizer factory, checkpoints.

Cheap elementwise/reduction glue around the NConv path (PyTorch-ROCm ops), except the loss itself.
  calculate_loss                    utils.py:138-151   masked RMSE*0.8 + Sobel-gradient*0.2 (or MSE);
                                    on device planes / batches the fused libnconv kernels (DepthLossFn)
  gradient_loss / gradient_x / _y   utils.py:95-136
  calculate_loss_multi_resolution   utils.py:63-71     each scale bilinear-resized to 480x640, [0] only
  get_optimizer                     utils.py:53-61     AdamW / SGD / RMSprop
  save_checkpoint / load_state_dict_compat  utils.py:42-51, models/step2.py:29-36
  GraphedTrainStep                  one training iteration (train_step1.py:59-65) captured in a
                                    hipGraph and replayed: removes the per-kernel host launch cost
"""
import os

import torch
import torch.nn.functional as F
import torch.optim as optimizer


def _padded(img):
    if img.dim() == 3:
        img = img.unsqueeze(0)
    return F.pad(img, (1, 1, 1, 1)), img.shape[-2], img.shape[-1]


def gradient_x(img):
    """F.conv2d(img, [[1,0,-1],[2,0,-2],[1,0,-1]], padding=1) (utils.py:95-106) as shifted
    differences: a 1-channel 3x3 correlation is a poor fit for a library conv (MIOpen picks a naive
    fp64-accumulating kernel for this shape)."""
    p, H, W = _padded(img)
    d = p[..., :, 0:W] - p[..., :, 2:W + 2]
    return (d[..., 0:H, :] + 2 * d[..., 1:H + 1, :] + d[..., 2:H + 2, :]).squeeze(0)


def gradient_y(img):
    """F.conv2d(img, [[1,2,1],[0,0,0],[-1,-2,-1]], padding=1) (utils.py:109-122)."""
    p, H, W = _padded(img)
    d = p[..., 0:H, :] - p[..., 2:H + 2, :]
    return (d[..., :, 0:W] + 2 * d[..., :, 1:W + 1] + d[..., :, 2:W + 2]).squeeze(0)


def gradient_loss(input_img, predicted_img):
    diff = input_img - predicted_img
    return torch.abs(gradient_x(diff)).mean() + torch.abs(gradient_y(diff)).mean()


def _calculate_loss_torch(reconstructed_img, target_img, use_gradient_loss):
    rec = reconstructed_img.masked_fill(target_img == 0, 0)
    if use_gradient_loss:
        return torch.sqrt(F.mse_loss(rec, target_img)) * 0.8 + gradient_loss(target_img, rec) * 0.2
    return F.mse_loss(rec, target_img)


def _planes(x):
    """(B, H, W) view geometry of a loss operand: (H, W), (1, H, W) or (B, 1, H, W) -> (B, image
    stride, row stride); None if it is not such a set of unit-stride rows."""
    if x.dim() == 2:
        B, bs = 1, 0
    elif x.dim() == 3 and x.shape[0] == 1:
        B, bs = 1, 0
    elif x.dim() == 4 and x.shape[1] == 1:
        B, bs = x.shape[0], x.stride(0)
    else:
        return None
    H, W = x.shape[-2], x.shape[-1]
    if x.stride(-1) != 1 or x.stride(-2) < W or (B > 1 and bs < H * x.stride(-2)):
        return None
    return B, bs, x.stride(-2)


class DepthLossFn(torch.autograd.Function):
    """calculate_loss (utils.py:138-151) on a (H, W) / (1, H, W) plane or a (B, 1, H, W) batch as
    libnconv kernels (nconv_depth_loss_fwd / _bwd: 2 launches forward, 1 backward, instead of ~45
    PyTorch ops). The batch form is the training loop's call (train_step1.py:63): means over all
    B*H*W elements, each image's Sobel response padded on its own, like F.conv2d on the batch."""

    @staticmethod
    def forward(ctx, r, t, use_gradient_loss):
        from . import _lib
        H, W = r.shape[-2], r.shape[-1]
        B, rbs, rs = _planes(r)
        _, tbs, ts = _planes(t)
        lib = _lib.lib()
        nbytes = lib.nconv_depth_loss_workspace_bytes(B, H, W)
        ws = torch.empty(max(nbytes, 4), dtype=torch.uint8, device=r.device)
        loss = torch.empty((), dtype=torch.float32, device=r.device)
        rc = lib.nconv_depth_loss_fwd(_lib.ptr(r), rbs, rs, _lib.ptr(t), tbs, ts, B, H, W,
                                      int(bool(use_gradient_loss)), _lib.ptr(loss), _lib.ptr(ws), nbytes,
                                      _lib.stream_handle(r.device))
        _lib.check(rc, "nconv_depth_loss_fwd")
        ctx.use_gradient_loss = bool(use_gradient_loss)
        ctx.save_for_backward(r, t, ws)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        from . import _lib
        r, t, ws = ctx.saved_tensors
        H, W = r.shape[-2], r.shape[-1]
        B, rbs, rs = _planes(r)
        _, tbs, ts = _planes(t)
        g = torch.empty(r.shape, dtype=torch.float32, device=r.device)
        gloss = gloss.contiguous()
        rc = _lib.lib().nconv_depth_loss_bwd(_lib.ptr(r), rbs, rs, _lib.ptr(t), tbs, ts, B, H, W,
                                             int(ctx.use_gradient_loss), _lib.ptr(gloss), _lib.ptr(ws),
                                             ws.numel(), _lib.ptr(g), _lib.stream_handle(r.device))
        _lib.check(rc, "nconv_depth_loss_bwd")
        return g, None, None


def _fused_loss_ok(r, t):
    def ok(x):
        return x.is_cuda and x.dtype == torch.float32 and _planes(x) is not None
    return ok(r) and ok(t) and r.shape == t.shape and not t.requires_grad and r.device == t.device


def calculate_loss(reconstructed_img, target_img, use_gradient_loss):
    """utils.py:138-151. Device planes / (B, 1, H, W) batches run the fused libnconv loss
    (DepthLossFn); anything else (CPU tensors, several channels) the PyTorch ops of the reference."""
    if _fused_loss_ok(reconstructed_img, target_img):
        return DepthLossFn.apply(reconstructed_img, target_img, use_gradient_loss)
    return _calculate_loss_torch(reconstructed_img, target_img, use_gradient_loss)


def calculate_loss_multi_resolution(reconstructed_img, target_img, use_gradient_loss):
    total = 0.0
    for img in reconstructed_img:
        r = F.interpolate(img, size=(480, 640), mode="bilinear", align_corners=False)
        total += calculate_loss(r[0, :, :, :], target_img[0, :, :, :], use_gradient_loss)
    return total / len(reconstructed_img)


def get_optimizer(net, optim_type, lr, weight_decay, capturable=False, fused=False):
    """utils.py:53-61; capturable=True keeps AdamW's step count on the device (GraphedTrainStep);
    fused=True runs AdamW's whole update as one multi-tensor kernel (same update rule; one launch
    instead of ~45 small per-parameter ones for DNET)."""
    if optim_type == "adam":
        if fused:
            return optimizer.AdamW(net.parameters(), lr=lr, weight_decay=weight_decay, capturable=capturable,
                                   fused=True)
        return optimizer.AdamW(net.parameters(), lr=lr, weight_decay=weight_decay, capturable=capturable)
    if optim_type == "sgd":
        return optimizer.SGD(net.parameters(), lr=lr, weight_decay=weight_decay, momentum=0.9)
    if optim_type == "rmsprop":
        return optimizer.RMSprop(net.parameters(), lr=lr, weight_decay=weight_decay, momentum=0.9)
    raise ValueError("Unsupported optimizer type. Choose 'adam', 'sgd', or 'rmsprop'.")


def save_checkpoint(model, epoch, checkpoint_dir, stats, name):
    """{"epoch", "state_dict", "stats"} at <dir>/<name>.pth.tar (utils.py:42-51)."""
    state = {"epoch": epoch, "state_dict": model.state_dict(), "stats": stats}
    torch.save(state, os.path.join(checkpoint_dir, f"{name}.pth.tar"))


def strip_module_prefix(state_dict):
    """Drop the `module.` prefix DataParallel / DDP add (models/step2.py:32-35)."""
    return {(k[7:] if k.startswith("module.") else k): v for k, v in state_dict.items()}


def load_checkpoint(model, path, strict=False, map_location="cpu"):
    """Load a reference-format checkpoint (weights only: torch.load(weights_only=True))."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    sd = ck["state_dict"] if isinstance(ck, dict) and "state_dict" in ck else ck
    return model.load_state_dict(strip_module_prefix(sd), strict=strict)


class GraphedTrainStep:
    """One training iteration — zero_grad, forward (EnforcePos drift included), loss, backward,
    the data-parallel gradient all-reduce (DataParallelRCCL.allreduce_grads, if the model has it)
    and the optimizer step — captured once in a hipGraph and replayed per call.

    loss_fn(model, *inputs) -> scalar loss tensor. The optimizer must keep its state on the device
    and update it without host synchronisation (torch AdamW / Adam with capturable=True). Inputs
    are copied into static buffers on every call (pass the same tensors to skip the copy). The
    warm-up iterations needed before capture run on a snapshot: parameters, buffers and optimizer
    state are restored in place afterwards, so constructing the step does not train the model.
    """

    def __init__(self, model, optimizer, loss_fn, example_inputs, warmup=3):
        self.model, self.optimizer, self.loss_fn = model, optimizer, loss_fn
        self.static_inputs = [x.detach().clone() for x in example_inputs]
        tensors = [t for t in list(model.parameters()) + list(model.buffers())]
        tensors += [v for st in optimizer.state.values() for v in st.values() if torch.is_tensor(v)]
        snap = [t.detach().clone() for t in tensors]
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self._body()
        cur.wait_stream(side)
        # optimizer state created during warm-up (first step) is part of the captured graph too
        new_state = [v for st in optimizer.state.values() for v in st.values() if torch.is_tensor(v)]
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.static_loss = self._body(zero=False)
        with torch.no_grad():
            for t, v in zip(tensors, snap):
                t.copy_(v)
            known = {id(t) for t in tensors}
            for v in new_state:  # state that did not exist before the warm-up starts from zero
                if id(v) not in known:
                    v.zero_()
        torch.cuda.synchronize()

    def _body(self, zero=True):
        if zero:
            self.optimizer.zero_grad(set_to_none=True)
        loss = self.loss_fn(self.model, *self.static_inputs)
        # d loss / d loss from a persistent tensor made during the warm-up (outside the capture):
        # loss.backward() would fill a fresh one with a launch of its own every replay
        if getattr(self, "_seed", None) is None or self._seed.shape != loss.shape:
            self._seed = torch.ones_like(loss)
        loss.backward(self._seed)
        if hasattr(self.model, "allreduce_grads"):
            self.model.allreduce_grads()
        self.optimizer.step()
        return loss

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst and src.data_ptr() != dst.data_ptr():
                dst.copy_(src)
        self.graph.replay()
        return self.static_loss
