#!/usr/bin/env python3
"""Config-4 guided training-step driver for rocprofv3 (developer tool):
python3 tools/guided_train_driver.py [steps] [torch]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps, kernels):
    import bench
    import nconv_pkg
    m = nconv_pkg.load()
    dev = torch.device("cuda:0")
    step = bench.make_guided_train_step(m, dev, 8, 352, 1216, 0, kernels=kernels)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4, len(sys.argv) < 3 or sys.argv[2] != "torch")
