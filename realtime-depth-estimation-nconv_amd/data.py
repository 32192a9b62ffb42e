"""Input pipeline — drop-in for the reference's dataset/kittiloader.py and dataset/nyuloader.py, plus
a device-side prefetcher that overlaps the host-to-HBM copies of the next batch with the step.

The Dataset classes keep the reference's constructors, directory layouts, sample dicts
({'rgb', 'depth', 'gt', 'k'}), crops and intrinsics adjustments. The reference decodes images with
OpenCV (absent here); this module decodes with Pillow and reproduces cv2.imread's results:
  * cv2.imread(path) -> uint8 BGR (H, W, 3): the RGB decode with the channel order reversed;
  * cv2.imread(path, cv2.IMREAD_GRAYSCALE) of a 16-bit PNG (KITTI depth) -> 8-bit: OpenCV's PNG
    reader strips the low byte (png_set_strip_16: v >> 8), so the reference's `/ 256.0` yields
    (v >> 8) / 256, not metres (SURVEY.md 8(f4) notes this latent bug). depth_decode="reference"
    (default) keeps that behaviour bit for bit; depth_decode="kitti16" reads the 16-bit value
    (v / 256 metres, the KITTI devkit's convention). 8-bit grayscale PNGs decode as stored; colour
    PNGs read as grayscale use OpenCV's BT.601 integer weights.
NYU (dataset/nyuloader.py) reads .npy arrays (np.load, allow_pickle=False) and, as the reference
does, derives the sparse input from the ground truth with a random mask file
(preprocess_depth(self.depths[index], ...), nyuloader.py:55), resized with PIL NEAREST when it is
not 480 x 640. Parity with cv2 itself is unpinned in this image (OpenCV is not installed); the
decode semantics are restated and tested against hand-built PNGs (tests/test_data_cpu.py).
"""
import glob
import os
import random

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset


# ---- decoding (cv2.imread semantics) ---------------------------------------------------------------
def imread_bgr(path):
    """cv2.imread(path): uint8 (H, W, 3) in BGR order."""
    with Image.open(path) as im:
        a = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(a[:, :, ::-1])


def imread_gray(path, depth_decode="reference"):
    """cv2.imread(path, cv2.IMREAD_GRAYSCALE) as the reference uses it (see module docstring)."""
    with Image.open(path) as im:
        mode = im.mode
        if mode in ("I;16", "I;16B", "I;16L", "I"):
            v = np.asarray(im).astype(np.uint32)
            if depth_decode == "kitti16":
                return v.astype(np.float32)
            if depth_decode != "reference":
                raise ValueError(f"depth_decode must be 'reference' or 'kitti16', got {depth_decode!r}")
            return (v >> 8).astype(np.uint8)
        if mode == "L":
            return np.asarray(im).copy()
        rgb = np.asarray(im.convert("RGB")).astype(np.int32)
    # OpenCV's RGB -> gray: (R*4899 + G*9617 + B*1868 + 8192) >> 14 (BT.601, 14-bit fixed point)
    return ((rgb[..., 0] * 4899 + rgb[..., 1] * 9617 + rgb[..., 2] * 1868 + 8192) >> 14).astype(np.uint8)


def read_calib_file(filepath):
    """Read a KITTI calibration file into a dict of float arrays (kittiloader.py:9-23)."""
    data = {}
    with open(filepath, "r") as f:
        for line in f.readlines():
            key, value = line.split(":", 1)
            try:
                data[key] = np.array([float(x) for x in value.split()])
            except ValueError:
                pass
    return data


# ---- KITTI (dataset/kittiloader.py) ----------------------------------------------------------------
class _KittiBase(Dataset):
    depth_decode = "reference"

    def __len__(self):
        return len(self.depths)

    def __getitem__(self, idx):
        return self.get_item(idx)

    def get_rgb(self, rgb_path):
        return torch.FloatTensor(imread_bgr(rgb_path)).permute(2, 0, 1)

    def get_depth(self, depth_path):
        d = imread_gray(depth_path, self.depth_decode).astype(np.float32) / 256.0
        return torch.FloatTensor(np.expand_dims(d, axis=0))

    get_gt = get_depth

    def _crop(self, rgb, k, *planes):
        """Bottom rows and centred columns (kittiloader.py:53-60), K shifted by the crop."""
        tp = rgb.shape[1] - self.height
        lp = (rgb.shape[2] - self.width) // 2
        out = [t[:, tp:tp + self.height, lp:lp + self.width] for t in (rgb,) + planes]
        if k is not None:
            k[0, 2] -= lp
            k[1, 2] -= tp
        return out, k


class DataLoader_KITTI(_KittiBase):
    """KITTI depth completion train / val split (kittiloader.py:25-97)."""

    def __init__(self, data_dir, mode, height=256, width=1216, tp_min=50, depth_decode="reference"):
        self.depth_path = os.path.join(data_dir, "data_depth_annotated", mode)
        self.lidar_path = os.path.join(data_dir, "data_depth_velodyne", mode)
        self.depths = list(sorted(glob.iglob(self.depth_path + "/**/*.png", recursive=True)))
        self.lidars = list(sorted(glob.iglob(self.lidar_path + "/**/*.png", recursive=True)))
        self.height, self.width, self.tp_min = height, width, tp_min
        self.depth_decode = depth_decode

    def _rgb_path(self, index):
        f = self.depths[index].split("/")
        return os.path.join(*f[:-7], "raw", f[-5].split("_drive")[0], f[-5], f[-2], "data", f[-1])

    def get_item(self, index):
        rgb = self.get_rgb(("/" if self.depths[index].startswith("/") else "") + self._rgb_path(index))
        depth = self.get_depth(self.lidars[index])
        gt = self.get_gt(self.depths[index])
        (rgb, depth, gt), k = self._crop(rgb, self.get_k(index), depth, gt)
        return {"rgb": rgb, "depth": depth, "gt": gt, "k": k}

    def get_k(self, index):
        f = self.depths[index].split("/")
        calib = os.path.join(*f[:-7], "raw", f[-5].split("_drive")[0], "calib_cam_to_cam.txt")
        data = read_calib_file(("/" if self.depths[index].startswith("/") else "") + calib)
        if f[-2] == "image_02":
            K = np.reshape(data["P_rect_02"], (3, 4))[0:3, 0:3]
        elif f[-2] == "image_03":
            K = np.reshape(data["P_rect_03"], (3, 4))[0:3, 0:3]
        else:
            raise ValueError("Unknown mode: {}".format(f[-2]))
        return torch.FloatTensor(np.array(K).astype(np.float32).reshape(3, 3))


class DataLoader_KITTI_seltest(_KittiBase):
    """KITTI val_selection_cropped (kittiloader.py:100-154)."""

    def __init__(self, data_dir, height=256, width=1216, tp_min=50, depth_decode="reference"):
        base = os.path.join(data_dir, "val_selection_cropped")
        self.depths = list(sorted(glob.iglob(os.path.join(base, "groundtruth_depth") + "/*.png")))
        self.lidars = list(sorted(glob.iglob(os.path.join(base, "velodyne_raw") + "/*.png")))
        self.images = list(sorted(glob.iglob(os.path.join(base, "image") + "/*.png")))
        self.height, self.width, self.tp_min = height, width, tp_min
        self.depth_decode = depth_decode

    def get_item(self, index):
        rgb = self.get_rgb(self.images[index])
        depth = self.get_depth(self.lidars[index])
        gt = self.get_gt(self.depths[index])
        (rgb, depth, gt), k = self._crop(rgb, self.get_k(index), depth, gt)
        return {"rgb": rgb, "depth": depth, "gt": gt, "k": k}

    def get_k(self, index):
        fns = self.images[index].split("/")
        path = os.path.join(*fns[:-2], "intrinsics", fns[-1][:-3] + "txt")
        with open(("/" if self.images[index].startswith("/") else "") + path) as f:
            K = f.read().split()
        return torch.FloatTensor(np.array(K).astype(np.float32).reshape(3, 3))


class DataLoader_KITTI_test(DataLoader_KITTI_seltest):
    """KITTI test_depth_completion_anonymous (kittiloader.py:157-210): no ground truth."""

    def __init__(self, data_dir, height=352, width=1216, tp_min=50, depth_decode="reference"):
        base = os.path.join(data_dir, "test_depth_completion_anonymous")
        self.lidars = list(sorted(glob.iglob(os.path.join(base, "velodyne_raw") + "/*.png")))
        self.images = list(sorted(glob.iglob(os.path.join(base, "image") + "/*.png")))
        self.depths = self.lidars
        self.height, self.width, self.tp_min = height, width, tp_min
        self.depth_decode = depth_decode

    def get_item(self, index):
        rgb = self.get_rgb(self.images[index])
        depth = self.get_depth(self.lidars[index])
        (rgb, depth), k = self._crop(rgb, self.get_k(index), depth)
        return {"rgb": rgb, "depth": depth, "k": k}


# ---- NYU (dataset/nyuloader.py) --------------------------------------------------------------------
class DataLoader_NYU(Dataset):
    """NYU-v2 .npy split (nyuloader.py:10-119). The sparse input is the ground truth times a random
    mask (use_mask) or with as many random points zeroed as the mask has zeros, optionally with
    +-10 % noise on 10 % of the points (add_noise), exactly as the reference."""

    def __init__(self, data_dir, mode, use_mask, add_noise, height=480, width=640, tp_min=50):
        self.depth_path = os.path.join(data_dir, mode, "gt")
        self.lidar_path = os.path.join(data_dir, mode, "depth")
        self.rgb_path = os.path.join(data_dir, mode, "img")
        self.mask_path = os.path.join(data_dir, "mask")
        self.depths = list(sorted(glob.iglob(self.depth_path + "/*.npy")))
        self.lidars = list(sorted(glob.iglob(self.lidar_path + "/*.npy")))
        self.rgbs = list(sorted(glob.iglob(self.rgb_path + "/*.png")))
        self.masks = list(sorted(glob.iglob(self.mask_path + "/*.npy")))
        self.height, self.width, self.tp_min = height, width, tp_min
        self.use_mask, self.add_noise = use_mask, add_noise
        self.k = np.array([[582.62448, 0.0, 313.04476], [0.0, 582.69103, 238.44390], [0.0, 0.0, 1.0]])

    def __len__(self):
        return len(self.depths)

    def __getitem__(self, idx):
        return self.get_item(idx)

    def get_item(self, index):
        rgb = self.get_rgb(self.rgbs[index])
        depth = self.get_depth(self.lidars[index])
        gt = self.get_gt(self.depths[index])
        k = torch.FloatTensor(self.k)
        tp = rgb.shape[1] - self.height
        lp = (rgb.shape[2] - self.width) // 2
        rgb = rgb[:, tp:tp + self.height, lp:lp + self.width]
        depth = depth[:, tp:tp + self.height, lp:lp + self.width]
        gt = gt[:, tp:tp + self.height, lp:lp + self.width]
        k[0, 2] -= lp
        k[1, 2] -= tp
        depth = self.preprocess_depth(self.depths[index], self.use_mask, self.add_noise)
        return {"rgb": rgb, "depth": depth, "gt": gt, "k": k}

    def get_rgb(self, rgb_path):
        return torch.FloatTensor(imread_bgr(rgb_path)).permute(2, 0, 1)

    def get_depth(self, depth_path):
        d = np.load(depth_path, allow_pickle=False).reshape(480, 640)
        return torch.FloatTensor(np.expand_dims(d, axis=0))

    get_gt = get_depth

    def preprocess_depth(self, depth_path, apply_mask, apply_noise):
        raw_depth = self.get_depth(depth_path)
        mask_raw = np.load(random.choice(self.masks), allow_pickle=False)
        if mask_raw.shape != (480, 640):
            mask = np.array(Image.fromarray(mask_raw).resize((640, 480), Image.NEAREST))
        else:
            mask = mask_raw
        if apply_noise:
            n = raw_depth.numel()
            nn_ = int(n * 0.1)
            idx = torch.randperm(n)[:nn_]
            noise = torch.FloatTensor(nn_).uniform_(-0.1, 0.1)
            flat = raw_depth.reshape(-1)
            flat[idx] += flat[idx] * noise
            depth = flat.view_as(raw_depth)
        else:
            depth = raw_depth
        if apply_mask:
            depth = depth * torch.FloatTensor(mask)
        else:
            zeros = np.count_nonzero(mask == 0)
            n = depth.numel()
            idx = torch.randperm(n)[:min(zeros, n)]
            flat = depth.reshape(-1)
            flat[idx] = 0
            depth = flat.view_as(depth)
        return depth


class DataLoader_NYU_test(Dataset):
    """NYU test split without ground truth (nyuloader.py:121-169); no crop."""

    def __init__(self, data_dir, mode, height=640, width=480, tp_min=50):
        self.lidar_path = os.path.join(data_dir, mode, "depth")
        self.rgb_path = os.path.join(data_dir, mode, "img")
        self.lidars = list(sorted(glob.iglob(self.lidar_path + "/*.npy")))
        self.rgbs = list(sorted(glob.iglob(self.rgb_path + "/*.png")))
        self.height, self.width, self.tp_min = height, width, tp_min
        self.k = np.array([[329.64, 0.0, 318.0], [0.0, 328.62, 236.0], [0.0, 0.0, 1.0]])

    def __len__(self):
        return len(self.lidars)

    def __getitem__(self, idx):
        return {"rgb": torch.FloatTensor(imread_bgr(self.rgbs[idx])).permute(2, 0, 1),
                "depth": torch.FloatTensor(np.load(self.lidars[idx], allow_pickle=False).reshape(1, 480, 640)),
                "k": torch.FloatTensor(self.k)}


# ---- device prefetch ---------------------------------------------------------------------------------
class DevicePrefetcher:
    """Iterate a DataLoader's batches already resident in HBM: each batch is copied host -> device
    from pinned memory on a side HIP stream while the previous batch's step runs, and the compute
    stream waits on that copy only when the batch is taken (train_step1.py:55-57 moves every batch
    with .to(device, non_blocking=True) from pageable memory, which serialises the copy)."""

    def __init__(self, loader, device, keys=("rgb", "depth", "gt", "k")):
        self.loader, self.device, self.keys = loader, torch.device(device), keys
        self.stream = torch.cuda.Stream(device=self.device)

    def _load(self, it):
        try:
            batch = next(it)
        except StopIteration:
            return None
        out = {}
        with torch.cuda.stream(self.stream):
            for k, v in batch.items():
                if k in self.keys and torch.is_tensor(v):
                    out[k] = (v if v.is_pinned() else v.pin_memory()).to(self.device, non_blocking=True)
                else:
                    out[k] = v
        return out

    def __iter__(self):
        it = iter(self.loader)
        nxt = self._load(it)
        while nxt is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.stream)
            for v in nxt.values():
                if torch.is_tensor(v) and v.device == self.device:
                    v.record_stream(cur)
            batch, nxt = nxt, self._load(it)
            yield batch

    def __len__(self):
        return len(self.loader)
