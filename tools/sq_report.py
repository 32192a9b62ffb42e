#!/usr/bin/env python3
"""Per-kernel SQ counter report from r4_sq.sh's passes (gpurun_out/sq/{pmcA,pmcB,pmcC}_<layer>,
bpmc*_<layer> for the backward), written as JSON for profiles/ and read by bench.py for the
executed-rate figures (developer tool):

    python3 tools/sq_report.py gpurun_out/sq profiles/r4_sq_counters.json

Per kernel (the dominant dispatches of each layer run, grouped by kernel name): dispatches seen,
waves per dispatch, per-wave instruction counts (VALU, FMA-class VALU, MFMA, LDS, SALU, SMEM), the
wave-cycle split (active / issue-stall / parked on a counter), LDS bank conflicts, and the chip's
busy cycles per dispatch. Counts are as rocprofv3 reports them (SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_* in quad-cycles, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import json
import os
import sys

PER_CHIP = ("SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def collect(root):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*pmc?_*"))):
        name = os.path.basename(d)
        kind = "bwd" if name.startswith("b") else "fwd"
        layer = name.split("_", 1)[1]
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "nconv::" not in k:
                    continue
                kn = k.split("(")[0].replace("void nconv::", "").replace("(anonymous namespace)::", "")
                e = out.setdefault((kind, layer, kn), collections.defaultdict(list))
                e[r["Counter_Name"]].append(float(r["Counter_Value"]))
                e["_grid"].append(float(r.get("Grid_Size", 0) or 0))
    return out


def summarise(out):
    rep = {}
    for (kind, layer, kn), e in out.items():
        m = {c: sum(v) / len(v) for c, v in e.items() if v}
        waves = m.get("SQ_WAVES", 0)
        if not waves:
            continue
        per_w = lambda c: round(m[c] / waves, 1) if c in m else None
        r = {"kernel": kn, "dispatches": len(e.get("SQ_WAVES", [])), "waves_per_dispatch": round(waves),
             "grid": round(m["_grid"])}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_F32",
                  "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT",
                  "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            v = per_w(c)
            if v is not None:
                r[c.lower() + "_per_wave"] = v
        tot = sum(m.get(c, 0) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
        if tot:
            r["cycles_split"] = {"parked_on_counter": round(m["SQ_WAIT_ANY"] / tot, 3),
                                 "issue_stall": round(m["SQ_WAIT_INST_ANY"] / tot, 3),
                                 "active": round(m["SQ_ACTIVE_INST_ANY"] / tot, 3)}
        for c in PER_CHIP:
            if c in m:
                r[c.lower() + "_per_dispatch"] = round(m[c])
        rep.setdefault(kind, {}).setdefault(layer, []).append(r)
    for kind in rep.values():
        for layer in kind:
            kind[layer].sort(key=lambda r: -r["waves_per_dispatch"])
    return rep


if __name__ == "__main__":
    rep = summarise(collect(sys.argv[1]))
    txt = json.dumps(rep, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)
