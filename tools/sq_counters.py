#!/usr/bin/env python3
"""Summarise rocprofv3 SQ counter passes per forward kernel (developer tool).

usage: python tools/sq_counters.py gpurun_out/pmcA gpurun_out/pmcB [min_grid]
Prints per (kernel, grid) the per-wave averages and the parked / issue-stall / active split.
"""
import collections
import csv
import glob
import sys


def main(dirs, min_grid):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if int(r["Grid_Size"]) < min_grid:
                    continue
                key = (r["Kernel_Name"].split("(")[0].replace("void nconv::", ""), int(r["Grid_Size"]))
                agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (k, g), v in sorted(agg.items(), key=lambda kv: -kv[0][1]):
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m.get("SQ_WAVES", 0) or 1
        tot = sum(m.get(c, 0) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")) or 1
        line = f"{k:42s} grid {g:8d} waves {int(w):6d}"
        if "SQ_WAIT_ANY" in m:
            line += (f" parked {m['SQ_WAIT_ANY']/tot:.2f} issue-stall {m['SQ_WAIT_INST_ANY']/tot:.2f}"
                     f" active {m['SQ_ACTIVE_INST_ANY']/tot:.2f}")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
            if c in m:
                line += f" {c[3:].lower()}/w {m[c]/w:.0f}"
        for c, val in sorted(m.items()):  # any other counter: mean per dispatch
            if not c.startswith("SQ_"):
                line += f" {c}={val:.4g}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1:3], int(sys.argv[3]) if len(sys.argv) > 3 else 100000)
