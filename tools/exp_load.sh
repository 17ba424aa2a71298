#!/bin/bash
# per-stripe duration vs load (in-kernel timeline)
for o in sd ""; do
for cfg in "512 8" "512 1" "4096 8" "25600 8" "51200 8" "100000 8" "100000 4"; do
  set -- $cfg
  echo "== L2=$1 W=$2 outputs='$o'"
  NW_WAVES=$2 timeout -k 10 120 python tools/trace_fill.py 100000 $1 "$o" | grep -E "kernel_ms|duration"
done; done
