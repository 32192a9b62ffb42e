#!/usr/bin/env python3
"""Config-4 guided training-step driver for rocprofv3 (developer tool):
python3 tools/guided_train_driver.py [steps]  (prints the wall time per step)"""
import time
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(steps):
    import bench
    import nconv_pkg
    m = nconv_pkg.load()
    dev = torch.device("cuda:0")
    step = bench.make_guided_train_step(m, dev, 8, 352, 1216, 0, graph=False)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"guided training step: {(time.perf_counter() - t0) / steps * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
