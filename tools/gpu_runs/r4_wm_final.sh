#!/bin/bash
# Weight-gradient A/B (r4_wm_ab.sh), then the round measurement (round_measure.sh: GPU suite, smoke, bench, kernel trace, PMC traffic).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_runs/r4_wm_ab.sh || exit $?
bash tools/gpu_runs/round_measure.sh
