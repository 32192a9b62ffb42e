#!/bin/bash
# The deferred-join A/B (r5_dws2_ab.sh), then the round's final measurement (r5_final.sh) with the
# faster of NCONV_DENSE_WGRAD_STREAM 2 / 1 (2 if it wins every pair by > 0.5 %; the default is then
# switched to it in the source).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_runs/r5_dws2_ab.sh | tee gpurun_out/dws2_ab.txt || exit 1
win=$(python3 - <<'PY'
import re
v={}
for l in open('gpurun_out/dws2_ab.txt'):
    m=re.match(r'dense wgrad stream (\d) \S+ (\S+)', l)
    if m: v.setdefault(m.group(1), []).append(float(m.group(2)))
ok=len(v.get('2',[]))==len(v.get('1',[]))>0 and all(a < 0.995*b for a,b in zip(v['2'], v['1']))
print(2 if ok else 1)
PY
)
echo "final with NCONV_DENSE_WGRAD_STREAM=$win"
export NCONV_DENSE_WGRAD_STREAM=$win
bash tools/gpu_runs/r5_final.sh ${1:-r5f5}
