#!/bin/bash
# Register / LDS / spill summary of the fwd (or given) kernels: tools/kstats.sh [file.hip] [filter]
f=${1:-nconv_fwd.hip}; filt=${2:-_tiled}
cd "$(dirname "$0")/../realtime-depth-estimation-nconv_amd/csrc" || exit 1
hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o /tmp/kstats.s "$f" 2>&1 | grep -v hip-link
python3 - "$filt" <<'PY'
import re, sys
txt = open('/tmp/kstats.s').read()
for b in txt.split('- .agpr_count')[1:]:
    name = re.search(r'\.name:\s+(\S+)', b).group(1)
    if sys.argv[1] not in name: continue
    g = lambda k: re.search(r'\.' + k + r':\s+(\d+)', b).group(1)
    print(f"{name[:64]:64s} sgpr {g('sgpr_count'):>3} vgpr {g('vgpr_count'):>3} lds {g('group_segment_fixed_size'):>6} "
          f"spill v{g('vgpr_spill_count')} s{g('sgpr_spill_count')}")
PY
