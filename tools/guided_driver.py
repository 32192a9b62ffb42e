#!/usr/bin/env python3
"""Config-3 guided forward driver for rocprofv3 (developer tool): python3 tools/guided_driver.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(reps):
    import bench
    import nconv_pkg
    m = nconv_pkg.load()
    dev = torch.device("cuda:0")
    bench.guided_forward(m, dev, 8, 352, 1216, reps, 2, 0)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
