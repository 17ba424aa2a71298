#!/bin/bash
# Build an A/B variant of libnwfill.so into lib_ab/ from the current sources:
#   [GEN="gen_pair_asm.py flags"] [GEN_SCAN="gen_chunk_asm.py flags"] [PAIR_ONLY=1] bash tools/ab_build.sh NAME [hipcc flags, e.g. -DNW_TRACE_EXT=1]
# GEN regenerates the pair kernel's block (tools/gen_pair_asm.py, e.g.
# "--exp-no-bcast", "--align 0") into the variant's private copy of csrc/.
# PAIR_ONLY=1 recompiles only nw_pair.hip and links the in-tree objects of the
# other kernels (needleman-wunsch_amd/obj/, from make).
# tools/ab_run.py --libs 'lib_ab/*.so' then times every variant.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OBJ=$ROOT/needleman-wunsch_amd/obj
W=$(mktemp -d)
cp -r "$ROOT/needleman-wunsch_amd/csrc" "$W/csrc"
if [ -n "${GEN:-}" ]; then
  python3 "$ROOT/tools/gen_pair_asm.py" --out "$W/csrc/nw_pair_chunk.inc" $GEN > /dev/null
fi
if [ -n "${GEN_QUAD:-}" ]; then   # the quad kernel's block (tools/gen_quad_asm.py)
  python3 "$ROOT/tools/gen_quad_asm.py" --out "$W/csrc/nw_quad_chunk.inc" $GEN_QUAD > /dev/null
fi
if [ -n "${GEN_SCAN:-}" ]; then   # the one-row scan kernel's block (tools/gen_chunk_asm.py)
  python3 "$ROOT/tools/gen_chunk_asm.py" --out "$W/csrc/nw_chunk.inc" $GEN_SCAN > /dev/null
fi
mkdir -p "$ROOT/lib_ab"
HIPFLAGS=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops -I"$ROOT/include")
OBJS=()
for f in nw_fill nw_skew nw_pair nw_quad nw_panel nw_walk; do
  if [ -n "${ONLY:-}" ] && [ "$f" != "$ONLY" ]; then
    OBJS+=("$OBJ/$f.o")
    continue
  fi
  if [ -n "${PAIR_ONLY:-}" ] && [ "$f" != nw_pair ]; then
    OBJS+=("$OBJ/$f.o")
    continue
  fi
  /opt/rocm/bin/hipcc "${HIPFLAGS[@]}" "$@" -c -o "$W/$f.o" "$W/csrc/$f.hip" 2> >(grep -v "packed-fp32-ops" >&2) &
  OBJS+=("$W/$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/lib_ab/libnwfill_$NAME.so" "${OBJS[@]}" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$W"
echo "built lib_ab/libnwfill_$NAME.so"
