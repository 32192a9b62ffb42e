#!/bin/bash
# Round-5 fused backward: its GPU tests, the layer timing, and the training step both ways.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-fb}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_bwd.py -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -rf -s > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$tag.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python3 -u tools/fused_bwd_bench.py 20 > gpurun_out/fbench_$tag.log 2>&1
brc=$?; echo "fbench rc=$brc"; cat gpurun_out/fbench_$tag.log | tail -6
case $brc in 0) ;; *) exit $brc;; esac
for F in "" nconv2 "nconv2,nconv_down1,nconv_down2"; do
  NCONV_FUSED_BWD="$F" timeout -k 10 200 python3 -u bench.py --no-config5 --no-guided --no-guided-train \
      --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/btrain_${tag}_${F//,/_}.json 2> gpurun_out/btrain_${tag}_${F//,/_}.err
  r=$?; echo "bench[$F] rc=$r"; [ $r -ne 0 ] && exit $r
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['train_fwd_bwd_adamw']; print(sys.argv[2], t['ms_per_step'], t['eager'])" gpurun_out/btrain_${tag}_${F//,/_}.json "[$F]"
done
exit $rc
