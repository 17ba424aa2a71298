#!/bin/bash
# Like tools/ab_build.sh, but recompiles only nw_pair.hip with the extra flags
# and links it with the in-tree objects of the other kernels (obj/, from make):
#   [GEN="--exp-no-bcast ..."] bash tools/ab_build_pair.sh NAME [hipcc flags]
# GEN regenerates the pair block (tools/gen_pair_asm.py) with those options
# into the variant's private copy of csrc/.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OBJ=$ROOT/needleman-wunsch_amd/obj
W=$(mktemp -d)
cp -r "$ROOT/needleman-wunsch_amd/csrc" "$W/csrc"
if [ -n "${GEN:-}" ]; then
  python3 "$ROOT/tools/gen_pair_asm.py" --out "$W/csrc/nw_pair_chunk.inc" $GEN > /dev/null
fi
mkdir -p "$ROOT/lib_ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I"$ROOT/include" "$@" \
    -c -o "$W/nw_pair.o" "$W/csrc/nw_pair.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/lib_ab/libnwfill_$NAME.so" \
    "$OBJ/nw_fill.o" "$OBJ/nw_skew.o" "$W/nw_pair.o" "$OBJ/nw_panel.o" "$OBJ/nw_walk.o" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$W"
echo "built lib_ab/libnwfill_$NAME.so"
