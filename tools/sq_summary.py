#!/usr/bin/env python3
"""Per-wave SQ counter summary of the libnconv kernels in gpu_probe.sh's pmcA_/pmcB_ passes
(developer tool): python3 tools/sq_summary.py gpurun_out head down1 ..."""
import collections
import csv
import glob
import sys

PER_CHIP = ("SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def main(root, layers):
    for L in layers:
        agg = collections.defaultdict(list)
        for d in (f"{root}/pmcA_{L}", f"{root}/pmcB_{L}"):
            for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
                for r in csv.DictReader(open(f)):
                    if "nconv::" not in r["Kernel_Name"]:
                        continue
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        m = {k: sum(v) / len(v) for k, v in agg.items()}
        w = m.get("SQ_WAVES", 1) or 1
        out = {k: round(v if k in PER_CHIP else v / w) for k, v in sorted(m.items()) if k != "SQ_WAVES"}
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc:
            out["mfma_busy_frac"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / cyc, 3)
        print(L, f"waves={int(w)}", out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
