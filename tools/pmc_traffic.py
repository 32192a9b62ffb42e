#!/usr/bin/env python3
"""Measured HBM traffic per forward kernel (rocprofv3 PMC), for bench.py's roofline.traffic.

Two steps (MI355X_MICROARCH.md, HBM section: FETCH_SIZE and WRITE_SIZE do not fit one pass, and
on gfx950 FETCH_SIZE reports half of a wide coalesced read, so it is doubled):

  1. on the GPU box, one rocprofv3 pass per counter over the same driver:
       rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \\
           python3 tools/pmc_traffic.py run
       rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \\
           python3 tools/pmc_traffic.py run
  2. anywhere: python3 tools/pmc_traffic.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write [MATH] [REV]
     -> profiles/pmc_traffic.json  {config: [B,H,W], kernels: {MATH: {name: {hbm_bytes_per_launch, ...}}}}

FETCH_SIZE / WRITE_SIZE are in KiB. The guide's factor 2 on FETCH_SIZE is calibrated for 16-byte
per-lane reads; the NConv kernels stage with 4-byte buffer loads, so the run also times a
calibration launch of known bytes in the same access pattern (a 1x1 8 -> 1 NConv layer over B=8
352x1216 fresh planes: reads 64 B and writes 8 B per pixel, no reuse) and the parse scales every
kernel's counters by that launch's measured/algorithmic ratios (reported beside the raw counts).
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
        # calibration: known bytes, the forward kernels' staging loads (4 B per lane) and stores
        spec = m.LayerSpec(8, 1, (1, 1))
        w = torch.rand(1, 8, 1, 1, device=dev) + 0.1
        bias = torch.zeros(1, device=dev)
        wsum = w.sum((1, 2, 3)).contiguous()
        for _ in range(REPS):
            x, c = torch.rand(B, 8, H, W, device=dev), torch.rand(B, 8, H, W, device=dev)
            m.nconv.layer_forward_raw(spec, x, c, None, None, w, bias, wsum)
    torch.cuda.synchronize()


CALIB_READ, CALIB_WRITE = B * H * W * 16 * 4, B * H * W * 2 * 4  # bytes per calibration launch


ORDER = ["nconv1+nconv2_head", "nconv_down1", "nconv_down2", "nconv_down3", "nconv4", "nconv5", "nconv6+7_tail"]
# (without the fused head: "nconv1", "nconv2", ... as separate launches)
ORDER_UNFUSED = ["nconv1", "nconv2"] + ORDER[1:]


def _read(dirpath, counter):
    """Per layer mean of `counter` over the timed inference forwards. Dispatches are taken in
    order: an inference forward is its weight prologue (weight_prologue; weight_prep before round
    4's one-launch prologue) followed by the 7 layer launches of ORDER (8 without
    the fused head; the warm-up training forward has 9 and is skipped)."""
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {dirpath}")
    rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    groups, cur, calib = [], None, []
    for r in rows:
        name = r["Kernel_Name"]
        if "fwd_tiled<8, 1, 1," in name and int(r["Grid_Size"]) >= 1 << 20:
            calib.append(float(r["Counter_Value"]))
            cur = None
        elif "weight_prep" in name or "weight_prologue" in name:  # a forward's first launch
            cur = []
            groups.append(cur)
        elif cur is not None and "nconv::" in name and "phase_weights" not in name and "head_weights" not in name:
            cur.append(r)
    per = defaultdict(list)
    for g in groups:
        order = {len(ORDER): ORDER, len(ORDER_UNFUSED): ORDER_UNFUSED}.get(len(g))
        if order is None:
            continue
        for name, r in zip(order, g):
            per[name].append(float(r["Counter_Value"]))
    if calib:
        per["_calibration"] = calib
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def parse(fetch_dir, write_dir, math="fp32", revision="unknown"):
    fetch, nf = _read(fetch_dir, "FETCH_SIZE")
    write, nw = _read(write_dir, "WRITE_SIZE")
    fr = fw = None
    if "_calibration" in fetch and "_calibration" in write:
        fr = CALIB_READ / (fetch.pop("_calibration") * 1024)
        fw = CALIB_WRITE / (write.pop("_calibration") * 1024)
    out = {"config": [B, H, W],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "tools/pmc_traffic.py run (inference forwards, then a calibration launch of known "
                     "bytes in the kernels' own access pattern: 4-byte staging loads, 8-byte stores); "
                     "hbm_bytes = FETCH_SIZE*1024*read_scale + WRITE_SIZE*1024*write_scale with the "
                     "scales measured on the calibration launch (without one: 2 and 1, the guide's "
                     "16-byte-read correction)",
           "calibration": {"read_scale": fr and round(fr, 4), "write_scale": fw and round(fw, 4),
                           "read_bytes": CALIB_READ, "write_bytes": CALIB_WRITE},
           "revision": revision, "math": math, "kernels": {math: {}}}
    rs, ws = (fr, fw) if fr else (2.0, 1.0)
    for k in sorted(set(fetch) & set(write)):
        out["kernels"][math][k] = {"fetch_kib": round(fetch[k], 1), "write_kib": round(write[k], 1),
                             "hbm_bytes_per_launch": int((rs * fetch[k] + ws * write[k]) * 1024),
                             "dispatches": [nf[k], nw[k]]}
    dst = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3], *sys.argv[4:6])
