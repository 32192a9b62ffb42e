#!/bin/bash
# Training-kernel A/B through gpurun: GPU tests of the training graph and layer backwards, then the
# training-step probe for the in-tree library and each variant library given (NCONV_LIB), then a
# kernel trace of the in-tree library's step (gpurun_out/tab_prof).
#   gpurun -- bash tools/gpu_runs/train_ab.sh "pytest selection" variants/x/libnconv.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
sel=$1; shift
if [ -n "$sel" ]; then
  timeout -k 10 500 python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/tab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/tab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 || exit $?
  for v in "$@"; do
    echo -n "[$v] "; NCONV_LIB=$v timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 || exit $?
  done
done
rm -rf gpurun_out/tab_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tab_prof -o run -- \
    python3 tools/train_probe.py --steps 30 > gpurun_out/tab_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
