#!/bin/bash
# nconv2's input-gradient kernel (dgrad_tiled<8,8,5,0,GP,HW>): occupancy A/B. Variants under
# variants/: hwh (the fused head weight-gradient epilogue in channel halves: 22 KB of LDS instead
# of 38 KB), oa1 (+ the pooled stager one plane ahead: 85 instead of 105 VGPRs), oa2 (one plane
# ahead in every dgrad_tiled), oa1w6 (oa1 with a 6-waves hint). Parity tests on oa1, then the
# graphed training step alternated, then the kernel's time under rocprof for base and oa1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dg
for V in oa1 oa2; do
  NCONV_LIB=$PWD/variants/$V/libnconv.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 \
      --timeout-method thread -m gpu tests/test_gpu_dnet.py -k "train or tail" tests/test_gpu_golden.py \
      tests/test_gpu_train_launches.py > gpurun_out/dg/pytest_$V.log 2>&1
  rc=$?; echo "$V: $(tail -1 gpurun_out/dg/pytest_$V.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for V in base hwh oa1 oa2 oa1w6; do
    lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
    echo -n "$V "; NCONV_LIB=$lib timeout -k 10 120 python3 tools/train_probe.py --steps 60 2>/dev/null || exit 1
  done
done
for V in base oa1; do
  lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
  rm -rf gpurun_out/dg/prof_$V
  NCONV_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dg/prof_$V -o run -- \
      python3 tools/train_probe.py --steps 20 > gpurun_out/dg/prof_$V.log 2>&1 || exit 1
  echo "== $V"; grep -E "dgrad_tiled|wgrad_mfma" gpurun_out/dg/prof_$V/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
