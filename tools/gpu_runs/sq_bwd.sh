#!/bin/bash
# SQ counter passes over one layer backward (tools/bwd_layer_bench.py LAYER 5): usage
#   gpurun -- bash tools/gpu_runs/sq_bwd.sh LAYER...  -> gpurun_out/sqbw{A,B,C}_LAYER/, summary on stdout
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC"
for L in "$@"; do
  timeout -k 10 120 python3 tools/bwd_layer_bench.py $L 5 || exit $?
  for p in A B C; do
    rm -rf gpurun_out/sqbw${p}_$L
    eval "CS=\$$p"
    timeout -s KILL 90 rocprofv3 --pmc $CS --output-format csv -d gpurun_out/sqbw${p}_$L -o run -- python3 tools/bwd_layer_bench.py $L 5 > gpurun_out/sqbw${p}_$L.log 2>&1 || exit $?
  done
  python3 - gpurun_out/sqbwA_$L gpurun_out/sqbwB_$L gpurun_out/sqbwC_$L <<'P'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "grad" not in r["Kernel_Name"]:
                continue
            agg[r["Kernel_Name"].split("(")[0].replace("void nconv::", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    m = {c: sum(x) / len(x) for c, x in v.items()}
    w = m.get("SQ_WAVES", 1) or 1
    out = {c[3:] if c.startswith("SQ_") else c: round(val / w if c.startswith(("SQ_INSTS", "SQ_WAIT", "SQ_ACTIVE", "SQ_WAVE_CYCLES", "SQ_LDS")) else val)
           for c, val in sorted(m.items())}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        out["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc, 3)
    print(k, out)
P
done
