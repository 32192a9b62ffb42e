#!/bin/bash
# Build libnconv.so of another git revision (same-box A/Bs): tools/build_rev.sh REV OUTDIR
# (load it with NCONV_LIB=OUTDIR/libnconv.so)
set -e
rev=$1; out=$2
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$root" archive "$rev" include realtime-depth-estimation-nconv_amd/csrc | tar -x -C "$tmp"
mkdir -p "$out"
objs=()
for f in "$tmp"/realtime-depth-estimation-nconv_amd/csrc/*.hip; do
  o="$out/$(basename "$f").o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$tmp/include" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/libnconv.so" "${objs[@]}"
rm -f "$out"/*.o; rm -rf "$tmp"
echo "built $out/libnconv.so ($rev)"
