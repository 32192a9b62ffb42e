#!/bin/bash
# SQ counter passes of nconv2's and nconv6's backward kernels only (r4_sq.sh without the forward
# layers), for the weight gradient's LDS bank-conflict counts after the bank re-layout.
cd "$GRAFT_REPO_ROOT" || exit 1
FWD_LAYERS=" " BWD_LAYERS="nconv2 nconv6" bash tools/gpu_runs/r4_sq.sh
