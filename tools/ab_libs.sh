#!/bin/bash
# A/B alternate builds of libnwfill.so (lib_ab/*.so) on the bench workload (run via gpurun).
#   bash tools/ab_libs.sh [bench.py args...]
set -euo pipefail
for rep in 1 2; do
  for L in lib_ab/*.so; do
    NW_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/abl.log 2>&1
    python3 -c "import json; j=json.loads(open('gpurun_out/abl.log').read().strip().splitlines()[-1]); print('$L', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS')"
  done
done
