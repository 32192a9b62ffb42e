#!/bin/bash
# Round 6: SQ counter passes of the dense 3x3 kernels (fp32 MFMA vs bf16x9) on one microbench shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/db9sq
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
SHAPE=${SHAPE:-conv 128->64}
for arm in "$@"; do
  for P in A B C; do
    env $arm DENSE_OPS=${OPS:-fwd} timeout -k 10 90 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/db9sq/${arm//[= \/]/_}_$P -o run -- \
        python3 tools/dense_microbench.py "$SHAPE" > gpurun_out/db9sq/log_$P.txt 2>&1
    rc=$?; if fatal $rc; then echo "pass $P rc=$rc"; exit $rc; fi
  done
  echo "== $arm"
  python3 - gpurun_out/db9sq/${arm//[= \/]/_}_ <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for P in "ABC":
    for f in glob.glob(f"{sys.argv[1]}{P}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dense_" not in r["Kernel_Name"] or "reduce" in r["Kernel_Name"] or "pack" in r["Kernel_Name"]:
                continue
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:28s} {sum(x)/len(x):14.4g}")
PY
done | tee gpurun_out/db9sq/summary.txt
