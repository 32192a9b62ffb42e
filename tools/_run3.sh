set -e
B="python -u bench.py --no-guided --no-guided-train --no-cpu-baseline --no-train"
for fh in 1 0; do for st in 1 2; do
  timeout -k 10 120 $B --fused-head $fh --streams $st > gpurun_out/b.json 2> gpurun_out/b.err
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print('head', $fh, 'streams', $st, d['value'], d['ms_per_step'])"
done; done
