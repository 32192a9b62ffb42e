cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_dnet.py > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; exit $rc
