set -e
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_dnet.py > gpurun_out/pytest_mfma.log 2>&1 || { tail -30 gpurun_out/pytest_mfma.log; exit 1; }
tail -1 gpurun_out/pytest_mfma.log
NCONV_MFMA_DMA=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_dnet.py > gpurun_out/pytest_mfma_dma.log 2>&1 || { tail -30 gpurun_out/pytest_mfma_dma.log; exit 1; }
tail -1 gpurun_out/pytest_mfma_dma.log
