#!/bin/bash
# Build an experimental variant of libnconv.so: tools/build_variant.sh OUTDIR -DMACRO=VAL ...
# (load it with NCONV_LIB=OUTDIR/libnconv.so)
set -e
out=$1; shift
root="$(cd "$(dirname "$0")/.." && pwd)"
src="$root/realtime-depth-estimation-nconv_amd/csrc"
mkdir -p "$out"
objs=()
for f in "$src"/*.hip; do
  o="$out/$(basename "$f").o"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$root/include" "$@" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/libnconv.so" "${objs[@]}"
echo "built $out/libnconv.so"
