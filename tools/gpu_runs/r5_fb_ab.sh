#!/bin/bash
# A/B of one-kernel backward variants: kernel times by rocprofv3 (fb_one.py), in-tree library vs
# variants/*/libnconv.so, and the grid-rounds knob.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fbab
run() {  # run NAME [env...]
  local name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fbab/$name -o run -- \
      python3 tools/fb_one.py head fused 5 > gpurun_out/fbab/$name.log 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fbab/${name}_tail -o run -- \
      python3 tools/fb_one.py tail fused 5 > gpurun_out/fbab/${name}_tail.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "$name tail rc=$rc"; exit $rc; }
  python3 - gpurun_out/fbab/$name gpurun_out/fbab/${name}_tail "$name" <<'PY'
import csv, glob, sys
for d in sys.argv[1:3]:
    f = (glob.glob(d + "/**/run_kernel_stats.csv", recursive=True) + glob.glob(d + "/run_kernel_stats.csv"))[0]
    for r in csv.DictReader(open(f)):
        if "bwd_fused" in r["Name"]:
            print(f"{sys.argv[3]:12s} {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:60]}")
PY
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_bwd.py -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/fbab/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fbab/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
run base
run ldsw NCONV_LIB=$PWD/variants/ldsw/libnconv.so
run rounds2 NCONV_FB_ROUNDS=2
run rounds4 NCONV_FB_ROUNDS=4
run rounds6 NCONV_FB_ROUNDS=6
