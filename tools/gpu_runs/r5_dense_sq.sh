#!/bin/bash
# SQ counter passes over the dense weight gradient of one shape (tools/dense_microbench.py,
# DENSE_OPS=wgrad), one rocprofv3 --pmc run per pass under its own time limit, then sq_report.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dsq5
export DENSE_OPS=wgrad
SH=${MB_SHAPES:-fuse3 conv 32->32}
python3 tools/dense_microbench.py "$SH" 2>/dev/null | tail -2
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for P in A B C; do
  rm -rf gpurun_out/dsq5/pmc${P}_wgrad
  timeout -k 10 -s KILL 90 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/dsq5/pmc${P}_wgrad -o run -- \
      python3 tools/dense_microbench.py "$SH" > gpurun_out/dsq5/$P.log 2>&1
  rc=$?; echo "$P rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
python3 tools/sq_report.py gpurun_out/dsq5 gpurun_out/dsq5/report.json > /dev/null && echo report ok
