#!/bin/bash
# Build libtasx with one kernel source taken from a git revision, for A/B
# timing against the working tree in the same GPU call:
#   tools/ab_lib.sh REV txseg_kernels   ->  tools/bin/ab_REV/libtasx.so
#   TASX_LIB=tools/bin/ab_REV/libtasx.so python tools/txseg_probe.py ...
set -euo pipefail
rev=$1; src=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/bin/ab_$rev
mkdir -p "$out"
rm -f "$out"/*.h
git -C "$root" show "$rev:tas_amd/csrc/$src.hip" > "$out/$src.hip"
objs=()
for o in "$root"/tas_amd/_lib/*.o; do
  case "$(basename "$o")" in ab_*.o) continue;; esac
  b=$(basename "$o" .o)
  if [ "$b" = "$src" ]; then objs+=("$out/$src.o"); else objs+=("$o"); fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Werror -Wno-unused-function \
  -I "$root/include" -I "$root/tas_amd/csrc" -c "$out/$src.hip" -o "$out/$src.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libtasx.so" "${objs[@]}" \
  -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -Wl,-soname,libtasx.so
echo "$out/libtasx.so"
