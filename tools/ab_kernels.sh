#!/bin/bash
# A/B the two fill kernels on the bench workload (run via gpurun from the repo root):
#   bash tools/ab_kernels.sh [extra bench.py args]
set -euo pipefail
mkdir -p gpurun_out
for K in skew scan pair; do
  NW_KERNEL=$K timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > gpurun_out/ab_$K.log 2>&1
  echo "$K: $(python3 -c "import json,sys; j=json.loads(open('gpurun_out/ab_$K.log').read().strip().splitlines()[-1]); print(j['value'], 'GCUPS', j['roofline']['kernel_ms'], 'ms kernel, frac', j['roofline']['frac'])")"
done
