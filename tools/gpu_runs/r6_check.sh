#!/bin/bash
# Round 6: full GPU suite + smoke (pytest_gpu.sh), the guided gradient reports (-s), then the bench
# (stdout JSON line to gpurun_out/bench_<TAG>.json).  gpurun --timeout 1100 -- bash tools/gpu_runs/r6_check.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-r6}
bash tools/gpu_runs/pytest_gpu.sh $tag tests || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_guided.py -m gpu -s -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "f9 or config4_full" > gpurun_out/guided_grads_$tag.log 2>&1 || exit $?
echo "guided grads ok"
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
tail -c 600 gpurun_out/bench_$tag.json
