cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_r2c.log 2>&1
echo "pytest rc=$?"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r2c.log 2>&1 || exit 1
PROBE_TESTS=0 PROBE_LAYERS="nconv2 tail down1 nconv5" bash tools/gpu_probe.sh
