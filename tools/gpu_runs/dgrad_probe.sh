#!/bin/bash
# Per-kernel times of one layer's backward (tools/bwd_layer_bench.py) for the in-tree library and
# each variant library given: gpurun -- bash tools/gpu_runs/dgrad_probe.sh "nconv2 down1" variants/x/libnconv.so ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
layers=$1; shift
for lib in "" "$@"; do
  for L in $layers; do
    rm -rf gpurun_out/dgp
    NCONV_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dgp -o run -- python3 tools/bwd_layer_bench.py $L 20 > /dev/null 2>&1 || exit $?
    python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/dgp/run_kernel_stats.csv')):
    if 'dgrad' in r['Name'] or 'wgrad_mfma' in r['Name']: print('[$lib] $L', r['Name'][:60], r['AverageNs'])
"
  done
done
