#!/bin/bash
# Timeline of the skew kernel at a few shapes (run via gpurun from the repo root).
set -euo pipefail
mkdir -p gpurun_out
{
for shape in "100000 64" "100000 448" "100000 100000"; do
  timeout -k 10 120 python tools/trace_fill.py $shape sd
done
NW_KERNEL=scan timeout -k 10 120 python tools/trace_fill.py 100000 64 sd
} > gpurun_out/skew_trace.txt 2>&1
