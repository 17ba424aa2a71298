#!/bin/bash
# one workgroup, W compute waves (L2 = 64 W): per-stripe time vs waves per SIMD
for W in 1 2 4 6 8 12 15; do
  for o in sd _; do
    oo=$o; [ "$o" = "_" ] && oo=""
    echo "== W=$W outputs='$oo'"
    NW_WAVES=$W timeout -k 10 60 python tools/trace_fill.py 100000 $((64 * W)) "$oo" | grep -E "kernel_ms"
  done
done
