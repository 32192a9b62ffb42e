#!/bin/bash
# SQ counter passes over the dense weight gradient (tools/dense_microbench.py, DENSE_OPS=wgrad) for
# the shapes in MB_SHAPES; one rocprofv3 --pmc run per pass, each under its own time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dsq
export DENSE_OPS=wgrad
SH=${MB_SHAPES:-fuse3 conv 32->32}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for who in base cur; do
  dir=.; [ $who = base ] && dir=variants/base_pkg
  for P in A B C; do
    rm -rf $GRAFT_REPO_ROOT/gpurun_out/dsq/${who}_$P
    (cd $dir && timeout -k 10 -s KILL 90 rocprofv3 --pmc ${!P} --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dsq/${who}_$P -o run -- python3 tools/dense_microbench.py "$SH" > $GRAFT_REPO_ROOT/gpurun_out/dsq/${who}_$P.log 2>&1)
    rc=$?; echo "$who $P rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
