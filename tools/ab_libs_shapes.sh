#!/bin/bash
# A/B every lib_ab/*.so over a few fill shapes (run via gpurun):
#   bash tools/ab_libs_shapes.sh ["L1xL2 ..."]
set -euo pipefail
SHAPES=${1:-"10000x10000 100000x12500 100000x50000 100000x100000"}
for rep in 1 2; do
  for s in $SHAPES; do
    for L in lib_ab/*.so; do
      NW_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-c2 --L1 ${s%x*} --L2 ${s#*x} \
          --steps 10 --warmup 2 > gpurun_out/abs.log 2>&1
      python3 -c "import json; j=json.loads(open('gpurun_out/abs.log').read().strip().splitlines()[-1]); print('$s', '$L', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS', j.get('parity', {}).get('ok'))"
    done
  done
done
