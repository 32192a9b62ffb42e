"""Training-step glue of the reference (utils.py), on device: losses, optimizer factory, checkpoints.

These are cheap elementwise/reduction ops around the NConv path; they run as PyTorch-ROCm ops.
  calculate_loss                    utils.py:138-151   masked RMSE*0.8 + Sobel-gradient*0.2 (or MSE)
  gradient_loss / gradient_x / _y   utils.py:95-136
  calculate_loss_multi_resolution   utils.py:63-71     each scale bilinear-resized to 480x640, [0] only
  get_optimizer                     utils.py:53-61     AdamW / SGD / RMSprop
  save_checkpoint / load_state_dict_compat  utils.py:42-51, models/step2.py:29-36
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


def calculate_loss(reconstructed_img, target_img, use_gradient_loss):
    rec = reconstructed_img.masked_fill(target_img == 0, 0)
    if use_gradient_loss:
        return torch.sqrt(F.mse_loss(rec, target_img)) * 0.8 + gradient_loss(target_img, rec) * 0.2
    return F.mse_loss(rec, target_img)


def calculate_loss_multi_resolution(reconstructed_img, target_img, use_gradient_loss):
    total = 0.0
    for img in reconstructed_img:
        r = F.interpolate(img, size=(480, 640), mode="bilinear", align_corners=False)
        total += calculate_loss(r[0, :, :, :], target_img[0, :, :, :], use_gradient_loss)
    return total / len(reconstructed_img)


def get_optimizer(net, optim_type, lr, weight_decay):
    if optim_type == "adam":
        return optimizer.AdamW(net.parameters(), lr=lr, weight_decay=weight_decay)
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
