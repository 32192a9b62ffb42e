#!/bin/bash
# SQ counter passes over the one-kernel backward forms and the two-kernel forms they replace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sqfb
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for W in head tail; do
  for F in fused separate; do
    for P in A B C; do
      timeout -k 10 90 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sqfb/bpmc${P}_${W}${F} -o run -- \
          python3 tools/fb_one.py $W $F 3 > gpurun_out/sqfb/${W}_${F}_$P.log 2>&1
      rc=$?; echo "$W $F $P rc=$rc"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
