#!/bin/bash
# Build an A/B variant of libnwfill.so whose pair block is regenerated with
# extra generator flags (tools/gen_pair_asm.py), into lib_ab/:
#   bash tools/ab_build_gen.sh NAME [gen_pair_asm.py flags, e.g. --align 0]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
W=$(mktemp -d)
cp -r "$ROOT/needleman-wunsch_amd/csrc" "$W/csrc"
python3 "$ROOT/tools/gen_pair_asm.py" --out "$W/csrc/nw_pair_chunk.inc" "$@" > /dev/null
mkdir -p "$ROOT/lib_ab"
OBJS=()
for f in nw_fill nw_skew nw_pair nw_panel nw_walk; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I"$ROOT/include" \
      -c -o "$W/$f.o" "$W/csrc/$f.hip" &
  OBJS+=("$W/$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/lib_ab/libnwfill_$NAME.so" "${OBJS[@]}" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$W"
echo "built lib_ab/libnwfill_$NAME.so"
