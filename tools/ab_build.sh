#!/bin/bash
# Build A/B variants of libnwfill.so into lib_ab/ from the current sources:
#   bash tools/ab_build.sh NAME [gen_chunk_asm.py options...]
# The chunk blocks are regenerated with the given options into a private copy
# of csrc/, so the tree's own nw_chunk.inc is untouched.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
W=$(mktemp -d)
cp -r "$ROOT/needleman-wunsch_amd/csrc" "$W/csrc"
python3 "$ROOT/tools/gen_chunk_asm.py" --out "$W/csrc/nw_chunk.inc" "$@" > /dev/null
mkdir -p "$ROOT/lib_ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I"$ROOT/include" ${NW_AB_FLAGS:-} -shared \
    -o "$ROOT/lib_ab/libnwfill_$NAME.so" "$W/csrc/nw_fill.hip" "$W/csrc/nw_panel.hip" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$W"
echo "built lib_ab/libnwfill_$NAME.so"
