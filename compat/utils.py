"""Drop-in for the reference's utils.py (`from utils import *` in train_step1.py / train_step2.py):
the training glue of nconv_amd.train (fused loss kernels on device tensors, the reference's
optimizer factory and checkpoint format) and the validation loops, plus the KITTI loader names
that utils.py re-exports (utils.py:1).

save_depth writes the min-max normalised depth as an 8-bit PNG (the reference colours it with
OpenCV's INFERNO map, utils.py:12-16; OpenCV is not available, so the image is grayscale).
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F  # noqa: F401  (the reference's namespace)
from torch import nn  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nconv_pkg  # noqa: E402

_m = nconv_pkg.load()
from dataset.kittiloader import *  # noqa: E402,F401,F403

calculate_loss = _m.train.calculate_loss
calculate_loss_multi_resolution = _m.train.calculate_loss_multi_resolution
gradient_loss = _m.train.gradient_loss
gradient_x = _m.train.gradient_x
gradient_y = _m.train.gradient_y
get_optimizer = _m.train.get_optimizer
save_checkpoint = _m.train.save_checkpoint


def save_depth(depth_data, path):
    d = np.asarray(depth_data, dtype=np.float64)
    lo, hi = float(d.min()), float(d.max())
    img = np.zeros(d.shape, np.uint8) if hi <= lo else ((d - lo) / (hi - lo) * 255.0 + 0.5).astype(np.uint8)
    from PIL import Image
    Image.fromarray(img).save(path)


def get_performance(model, val_loader, device_str, use_gradient_loss):
    """Mean validation loss of a step-1 model on element [0] of each batch (utils.py:18-40)."""
    device = torch.device(device_str if device_str == "cuda" and torch.cuda.is_available() else "cpu")
    model.to(device)
    model.eval()
    with torch.no_grad():
        losses = []
        for data in val_loader:
            depth, gt = data["depth"].to(device), data["gt"].to(device)
            est = model(depth)
            losses.append(calculate_loss(est[0, :, :, :], gt[0, :, :, :], use_gradient_loss).item())
    return sum(losses) / len(losses)


def get_performance_multi_resolution(model, val_loader, device_str, use_gradient_loss):
    """Mean multi-resolution validation loss of a guided model (utils.py:74-93)."""
    device = torch.device(device_str if device_str == "cuda" and torch.cuda.is_available() else "cpu")
    model.to(device)
    losses = []
    for data in val_loader:
        rgb, depth, gt = data["rgb"].to(device), data["depth"].to(device), data["gt"].to(device)
        est, _ = model(rgb, depth, rgb, depth)
        losses.append(calculate_loss_multi_resolution(est, gt, use_gradient_loss).item())
    return sum(losses) / len(losses)
