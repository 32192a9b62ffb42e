"""Drop-in for the reference's dataset/kittiloader.py: same names, backed by nconv_amd.data.

    from dataset.kittiloader import DataLoader_KITTI, DataLoader_KITTI_seltest, DataLoader_KITTI_test
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import nconv_pkg  # noqa: E402

_d = nconv_pkg.load().data
read_calib_file = _d.read_calib_file
DataLoader_KITTI = _d.DataLoader_KITTI
DataLoader_KITTI_seltest = _d.DataLoader_KITTI_seltest
DataLoader_KITTI_test = _d.DataLoader_KITTI_test
