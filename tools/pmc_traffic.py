#!/usr/bin/env python3
"""Measured HBM traffic per forward kernel (rocprofv3 PMC), for bench.py's roofline.traffic.

Two steps (MI355X_MICROARCH.md, HBM section: FETCH_SIZE and WRITE_SIZE do not fit one pass, and
on gfx950 FETCH_SIZE reports half of a wide coalesced read, so it is doubled):

  1. on the GPU box, one rocprofv3 pass per counter over the same driver:
       rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \\
           python3 tools/pmc_traffic.py run
       rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \\
           python3 tools/pmc_traffic.py run
  2. anywhere: python3 tools/pmc_traffic.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write
     -> profiles/pmc_traffic.json  {config: [B,H,W], kernels: {name: {hbm_bytes_per_launch, ...}}}

FETCH_SIZE / WRITE_SIZE are in KiB. hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B, H, W = 8, 352, 1216
REPS = 10


def run():
    import torch
    import bench
    import nconv_pkg
    m = nconv_pkg.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = m.SETP1_NCONV(crop="generalized").to(dev)
    net.train()
    with torch.no_grad():
        net(torch.zeros(1, 1, 32, 32, device=dev))
    net.eval()
    net.d_net.inference_streams = 1  # full-batch launches, as bench.time_layers times them
    S = bench.sparse_depth(torch.Generator().manual_seed(1000), B, H, W, dev)
    with torch.no_grad():
        for _ in range(REPS):
            net(S)
    torch.cuda.synchronize()


ORDER = ["nconv1+nconv2_head", "nconv_down1", "nconv_down2", "nconv_down3", "nconv4", "nconv5", "nconv6+7_tail"]
# (without the fused head: "nconv1", "nconv2", ... as separate launches)
ORDER_UNFUSED = ["nconv1", "nconv2"] + ORDER[1:]


def _read(dirpath, counter):
    """Per layer mean of `counter` over the timed inference forwards. Dispatches are taken in
    order: an inference forward is weight_prep followed by the 7 layer launches of ORDER (8 without
    the fused head; the warm-up training forward has 9 and is skipped)."""
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {dirpath}")
    rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    groups, cur = [], None
    for r in rows:
        if "weight_prep" in r["Kernel_Name"]:
            cur = []
            groups.append(cur)
        elif cur is not None and ("nconv::" in r["Kernel_Name"]):
            cur.append(r)
    per = defaultdict(list)
    for g in groups:
        order = {len(ORDER): ORDER, len(ORDER_UNFUSED): ORDER_UNFUSED}.get(len(g))
        if order is None:
            continue
        for name, r in zip(order, g):
            per[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def parse(fetch_dir, write_dir):
    fetch, nf = _read(fetch_dir, "FETCH_SIZE")
    write, nw = _read(write_dir, "WRITE_SIZE")
    out = {"config": [B, H, W],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "tools/pmc_traffic.py run; hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                     "(FETCH_SIZE doubled: gfx950 reports half of a wide coalesced read)",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        out["kernels"][k] = {"fetch_kib": round(fetch[k], 1), "write_kib": round(write[k], 1),
                             "hbm_bytes_per_launch": int((2 * fetch[k] + write[k]) * 1024),
                             "dispatches": [nf[k], nw[k]]}
    dst = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3])
