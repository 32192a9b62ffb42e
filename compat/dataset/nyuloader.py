"""Drop-in for the reference's dataset/nyuloader.py: same names, backed by nconv_amd.data.

    from dataset.nyuloader import DataLoader_NYU, DataLoader_NYU_test
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import nconv_pkg  # noqa: E402

_d = nconv_pkg.load().data
DataLoader_NYU = _d.DataLoader_NYU
DataLoader_NYU_test = _d.DataLoader_NYU_test
