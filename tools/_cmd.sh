cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_dnet.py > gpurun_out/pt.log 2>&1; rc=$?; tail -15 gpurun_out/pt.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash tools/ab_layers.sh "head" variants/nc1valu
