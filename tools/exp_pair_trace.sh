#!/bin/bash
# Timeline of the pair kernel (run via gpurun from the repo root).
set -euo pipefail
mkdir -p gpurun_out
{
for shape in "100000 128" "100000 512" "100000 100000"; do
  NW_KERNEL=pair timeout -k 10 120 python tools/trace_fill.py $shape sd
done
NW_KERNEL=pair timeout -k 10 120 python tools/trace_fill.py 100000 100000 ""
} > gpurun_out/pair_trace.txt 2>&1
