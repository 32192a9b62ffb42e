#!/bin/bash
# Round-5 fused backward + graphed guided step: their GPU tests, the layer timing, and the training
# step with each fused-layer set; then the guided training leg (graphed and eager).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-fb}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused_bwd.py \
    tests/test_gpu_guided.py::test_guided_graphed_train_step_matches_eager -v --timeout 250 \
    --timeout-method thread -p no:cacheprovider -rf -s > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_$tag.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python3 -u tools/fused_bwd_bench.py 20 > gpurun_out/fbench_$tag.log 2>&1
brc=$?; echo "fbench rc=$brc"; tail -6 gpurun_out/fbench_$tag.log
case $brc in 0) ;; *) exit $brc;; esac
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof_$tag -o run -- \
    python3 tools/fused_bwd_bench.py 5 > gpurun_out/fprof_$tag.log 2>&1
prc=$?; echo "fprof rc=$prc"
case $prc in 0) ;; *) exit $prc;; esac
f=$(ls gpurun_out/fprof_$tag/*/run_kernel_stats.csv gpurun_out/fprof_$tag/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if any(k in n for k in ('bwd_fused','dgrad','wgrad_mfma','wgrad_reduce','box_weights')):
        print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>4}  {n[:90]}\")
" "$f"
for F in "" nconv2 nconv6 "nconv2,nconv6" "nconv2,nconv_down1,nconv_down2,nconv6"; do
  NCONV_FUSED_BWD="$F" timeout -k 10 200 python3 -u bench.py --no-config5 --no-guided --no-guided-train \
      --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/btrain_${tag}_${F//,/_}.json 2> gpurun_out/btrain_${tag}_${F//,/_}.err
  r=$?; echo "bench[$F] rc=$r"; [ $r -ne 0 ] && exit $r
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d['train_fwd_bwd_adamw']; print(sys.argv[2], t['ms_per_step'], t['eager'])" gpurun_out/btrain_${tag}_${F//,/_}.json "[$F]"
done
timeout -k 10 300 python3 -u bench.py --no-train --no-config5 --no-guided --no-cpu-baseline --alt-math "" \
    --head-density 0 > gpurun_out/bguided_$tag.json 2> gpurun_out/bguided_$tag.err
r=$?; echo "bench guided rc=$r"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps(d['guided_train_fwd_bwd_adamw']))" gpurun_out/bguided_$tag.json
exit $rc
