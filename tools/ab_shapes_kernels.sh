#!/bin/bash
# Skew vs scan kernel over table shapes and output modes (run via gpurun).
#   bash tools/ab_shapes_kernels.sh "L1 L2 MODE" ...   MODE: sd | none (score-only)
set -euo pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_shapes_kernels.txt
: > $out
for spec in "$@"; do
  set -- $spec
  outs=$3; [ "$outs" = none ] && outs=""
  for K in skew scan pair; do
    NW_KERNEL=$K timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --L1 $1 --L2 $2 --outputs "$outs" > gpurun_out/abk.log 2>&1
    python3 - "$K" "$1x$2" "$3" >> $out <<'PY'
import json, sys
j = json.loads(open('gpurun_out/abk.log').read().strip().splitlines()[-1])
print(*sys.argv[1:], j['roofline']['kernel_ms'], 'ms', j['roofline']['kernel_gcups'], 'GCUPS W', j['config']['waves_per_wg'])
PY
  done
done
