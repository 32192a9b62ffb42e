#!/bin/bash
# Round-4 final measurement: round_measure.sh (GPU tests, smoke, bench line, kernel trace/stats,
# PMC traffic passes), then the SQ counter passes of the kernels the review names (head and tail
# forward, nconv2 / nconv6 backward) and down1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_runs/round_measure.sh || exit $?
FWD_LAYERS="head tail down1" BWD_LAYERS="nconv2 nconv6" bash tools/gpu_runs/r4_sq.sh || exit $?
