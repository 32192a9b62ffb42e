"""CPU: the input pipeline (nconv_amd.data; the reference's dataset/kittiloader.py and
dataset/nyuloader.py) on hand-built KITTI / NYU directory trees.

The expected values restate the reference's code: cv2.imread -> BGR uint8; cv2.imread(...,
IMREAD_GRAYSCALE) of a 16-bit PNG -> its high byte (v >> 8), then / 256 (kittiloader.py:69-79);
the bottom-centre crop and the intrinsics shift (kittiloader.py:53-60); NYU's input = ground truth
x random mask, the mask NEAREST-resized to 640 x 480 (nyuloader.py:79-119). OpenCV itself is not
installed, so cv2's decoding is restated, not run (parity unpinned against cv2 binaries).
"""
import os
import random
import subprocess
import sys

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kitti_tree(tmp, H=300, W=1300):
    rng = np.random.default_rng(0)
    drive, date, f = "2011_09_26_drive_0001_sync", "2011_09_26", "0000000005.png"
    gt_dir = os.path.join(tmp, "data_depth_annotated", "train", drive, "proj_depth", "groundtruth", "image_02")
    li_dir = os.path.join(tmp, "data_depth_velodyne", "train", drive, "proj_depth", "velodyne_raw", "image_02")
    rgb_dir = os.path.join(tmp, "raw", date, drive, "image_02", "data")
    for d in (gt_dir, li_dir, rgb_dir):
        os.makedirs(d)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    gt = (rng.integers(0, 30000, (H, W)) * (rng.random((H, W)) < 0.3)).astype(np.uint16)
    li = (rng.integers(0, 30000, (H, W)) * (rng.random((H, W)) < 0.05)).astype(np.uint16)
    Image.fromarray(rgb).save(os.path.join(rgb_dir, f))
    Image.fromarray(gt).save(os.path.join(gt_dir, f))
    Image.fromarray(li).save(os.path.join(li_dir, f))
    P2 = np.arange(12, dtype=np.float64) + 1.5
    with open(os.path.join(tmp, "raw", date, "calib_cam_to_cam.txt"), "w") as fh:
        fh.write("calib_time: 09-Jan-2012 13:57:47\n")
        fh.write("P_rect_02: " + " ".join(str(v) for v in P2) + "\n")
        fh.write("P_rect_03: " + " ".join(str(v) for v in P2 + 100) + "\n")
    return rgb, gt, li, P2.reshape(3, 4)[:, :3]


def test_kitti_loader_matches_reference_semantics(tmp_path, nconv_amd):
    rgb, gt, li, K = _kitti_tree(str(tmp_path))
    for decode in ("reference", "kitti16"):
        ds = nconv_amd.data.DataLoader_KITTI(str(tmp_path), "train", depth_decode=decode)
        assert len(ds) == 1
        s = ds[0]
        H, W = rgb.shape[:2]
        tp, lp = H - 256, (W - 1216) // 2
        exp_rgb = torch.from_numpy(rgb[:, :, ::-1].astype(np.float32).copy()).permute(2, 0, 1)[:, tp:tp + 256, lp:lp + 1216]
        assert torch.equal(s["rgb"], exp_rgb)
        conv = (lambda v: (v >> 8).astype(np.float32) / 256.0) if decode == "reference" else \
            (lambda v: v.astype(np.float32) / 256.0)
        assert torch.equal(s["depth"][0], torch.from_numpy(conv(li)[tp:tp + 256, lp:lp + 1216]))
        assert torch.equal(s["gt"][0], torch.from_numpy(conv(gt)[tp:tp + 256, lp:lp + 1216]))
        k = torch.tensor(K, dtype=torch.float32)
        k[0, 2] -= lp
        k[1, 2] -= tp
        assert torch.equal(s["k"], k)


def test_gray_decode_of_colour_and_8bit_pngs(tmp_path, nconv_amd):
    rng = np.random.default_rng(1)
    c = rng.integers(0, 256, (5, 7, 3), dtype=np.uint8)
    Image.fromarray(c).save(tmp_path / "c.png")
    g = rng.integers(0, 256, (5, 7), dtype=np.uint8)
    Image.fromarray(g).save(tmp_path / "g.png")
    ci = c.astype(np.int64)
    exp = (ci[..., 0] * 4899 + ci[..., 1] * 9617 + ci[..., 2] * 1868 + 8192) >> 14  # cv2 BT.601 fixed point
    assert (nconv_amd.data.imread_gray(str(tmp_path / "c.png")) == exp).all()
    assert (nconv_amd.data.imread_gray(str(tmp_path / "g.png")) == g).all()


def test_nyu_loader_masks_the_ground_truth(tmp_path, nconv_amd):
    rng = np.random.default_rng(2)
    for d in ("train/gt", "train/depth", "train/img", "mask"):
        os.makedirs(tmp_path / d)
    gt = rng.random((480, 640)).astype(np.float32) * 10
    np.save(tmp_path / "train/gt/000.npy", gt)
    np.save(tmp_path / "train/depth/000.npy", rng.random((480, 640)).astype(np.float32))
    Image.fromarray(rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)).save(tmp_path / "train/img/000.png")
    mask = (rng.random((240, 320)) < 0.1).astype(np.uint8)
    np.save(tmp_path / "mask/m0.npy", mask)
    ds = nconv_amd.data.DataLoader_NYU(str(tmp_path), "train", use_mask=True, add_noise=False)
    random.seed(0)
    s = ds[0]
    big = np.array(Image.fromarray(mask).resize((640, 480), Image.NEAREST))
    assert torch.equal(s["depth"][0], torch.from_numpy(gt) * torch.from_numpy(big).float())
    assert torch.equal(s["gt"][0], torch.from_numpy(gt))
    assert s["rgb"].shape == (3, 480, 640) and s["k"].shape == (3, 3)
    # use_mask False: as many points zeroed as the mask has zeros
    ds2 = nconv_amd.data.DataLoader_NYU(str(tmp_path), "train", use_mask=False, add_noise=False)
    d2 = ds2[0]["depth"]
    assert int((d2 == 0).sum()) >= int((big == 0).sum())


def test_reference_import_lines_for_data_and_utils(tmp_path):
    _kitti_tree(str(tmp_path))
    code = ("from dataset.kittiloader import DataLoader_KITTI\n"
            "from dataset.nyuloader import DataLoader_NYU\n"
            "from utils import *\n"
            f"ds = DataLoader_KITTI({str(tmp_path)!r}, 'train')\n"
            "from torch.utils.data import DataLoader\n"
            "b = next(iter(DataLoader(ds, batch_size=1)))\n"
            "print(tuple(b['depth'].shape), callable(calculate_loss), callable(get_optimizer))\n")
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "compat"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split("\n")[0] == "(1, 1, 256, 1216) True True"
