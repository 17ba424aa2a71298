#!/bin/bash
# Compute waves per workgroup ($NW_WAVES) on a bench workload (run via gpurun):
#   bash tools/ab_waves.sh "4 5 6 8" [bench.py args...]
set -euo pipefail
WS=$1; shift
for w in $WS; do
  NW_WAVES=$w timeout -k 10 200 python bench.py --no-cpu-baseline --no-c2 "$@" > gpurun_out/wv.log 2>&1
  python3 -c "import json; j=json.loads(open('gpurun_out/wv.log').read().strip().splitlines()[-1]); print('W=$w', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS', j.get('parity', {}).get('ok'))"
done
