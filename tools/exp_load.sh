#!/bin/bash
# per-stripe duration, shader clock and start lag vs load and outputs (in-kernel timeline)
for cfg in "64 1 sd" "512 8 sd" "4096 8 sd" "51200 8 sd" "100000 8 sd" "100000 8 s" "100000 8 d" "100000 8 _" "512 8 _"; do
  set -- $cfg
  o=$3; [ "$o" = "_" ] && o=""
  echo "== L2=$1 W=$2 outputs='$o'"
  NW_WAVES=$2 timeout -k 10 120 python tools/trace_fill.py 100000 $1 "$o" | grep -E "kernel_ms|duration|clock|end of"
done
